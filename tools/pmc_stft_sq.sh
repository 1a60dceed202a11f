#!/bin/bash
# SQ counter passes over the isolated STFT kernels (tools/stft_probe.py, product library), one
# rocprofv3 run per pass (a pass holds at most 8 SQ counters):  bash tools/pmc_stft_sq.sh <tag>
set -o pipefail
tag=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcsq_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"
P2="SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
P3="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_IFETCH SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex k_stft_slide --output-format csv -d $O/p$i -o p -- python3 $R/tools/stft_probe.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $R/tools/pmc_sum.py $O/p1/p_counter_collection.csv $O/p2/p_counter_collection.csv $O/p3/p_counter_collection.csv > $O/summary.txt
cat $O/summary.txt
