#!/usr/bin/env python3
"""Tabulates tools/kernel_ab.sh output (one line per library and kernel) as kernel x library:
    python3 tools/ab_table.py gpurun_out/<file>.txt [lib ...]"""
import collections
import re
import sys

d = collections.defaultdict(list)
libs = []
for line in open(sys.argv[1]):
    m = re.match(r"(\S+)\s+(.*?)\s+calls\s+\d+\s+avg\s+([\d.]+)", line)
    if not m:
        continue
    lib, kern, us = m.group(1), re.sub(r"^(void )?sdsp::", "", m.group(2))[:40], float(m.group(3))
    d[(kern, lib)].append(us)
    if lib not in libs:
        libs.append(lib)
libs = sys.argv[2:] or libs
for k in sorted({k for k, _ in d}):
    cells = ["/".join(f"{x:.0f}" for x in d[(k, lib)]) if (k, lib) in d else "-" for lib in libs]
    print(f"{k:40s} " + "  ".join(f"{lib}: {c:>13s}" for lib, c in zip(libs, cells)))
