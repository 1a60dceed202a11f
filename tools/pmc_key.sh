#!/bin/bash
# HBM bytes of the key-path and feature kernels (k_mask_r, k_hpcp, k_features) and the chip's HBM
# ceiling (tools/micro/hbm_ceiling), from the repo root on the GPU box:  bash tools/pmc_key.sh <tag>
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmckey_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/micro/hbm_ceiling > $O/hbm_ceiling.txt 2>&1 || { echo "ceiling failed"; cat $O/hbm_ceiling.txt; exit 1; }
cat $O/hbm_ceiling.txt
RX="k_mask_r|k_hpcp|k_features"  # k_mask_rp, k_hpcp_band included
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/fetch -o f -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/write -o w -- python3 $R/bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 || { echo "write pass failed"; tail -5 $O/write.log; exit 1; }
python3 $R/tools/pmc_kernels.py $O/fetch/f_counter_collection.csv $O/write/w_counter_collection.csv > $O/pmc_kernels.json && cat $O/pmc_kernels.json
