#!/bin/bash
# SQ counter passes (3 × 8 counters, one rocprofv3 run each) over the pipeline kernels matching a
# regex, in a one-step bench run:  bash tools/pmc_sq.sh <tag> <kernel-regex> [tracks]
set -o pipefail
tag=$1; rx=$2; n=${3:-64}
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
  SDSP_SERIAL_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$rx" --output-format csv -d $O/p$i -o p -- python3 $R/bench.py --tracks $n --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $R/tools/pmc_sum.py $O/p1/p_counter_collection.csv $O/p2/p_counter_collection.csv $O/p3/p_counter_collection.csv > $O/summary.txt
cat $O/summary.txt
