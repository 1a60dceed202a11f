#!/usr/bin/env python3
"""Sums rocprofv3 counter-collection CSVs per (kernel, counter) and prints one table per kernel
with per-dispatch means (tools/pmc_stft_sq.sh)."""
import collections
import csv
import sys

tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
kernels = sorted({k for k, _ in tot})
for k in kernels:
    print(k)
    for (kk, c), v in sorted(tot.items()):
        if kk == k:
            n = len(disp[(kk, c)])
            print(f"  {c:32s} {v / n:18.1f}  ({n} dispatches)")
