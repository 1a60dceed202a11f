#!/usr/bin/env python3
"""Which main-stream kernels run beside each key-stream kernel in a two-stream kernel trace:
    python3 tools/overlap.py <kernel_trace.csv> [key-kernel-regex]
Per key-stream kernel (queue of the 8192-point STFT), the time-weighted overlap with every
kernel of the other queues, summed over its launches, in ms."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rx = sys.argv[2] if len(sys.argv) > 2 else "k_stft_slide8"
iv = []
for r in rows:
    name = re.sub(r"^(void )?sdsp::", "", r["Kernel_Name"]).split("(")[0]
    iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id") or r.get("Stream_Id")))
keyq = {q for s, e, n, q in iv if re.search(rx, n)}
key = [x for x in iv if re.search(rx, x[2])]
other = [x for x in iv if x[3] not in keyq]
ov = collections.Counter()
tot = 0
for s, e, n, q in key:
    tot += e - s
    for s2, e2, n2, q2 in other:
        o = min(e, e2) - max(s, s2)
        if o > 0:
            ov[n2] += o
qs = collections.Counter((r["Queue_Id"], r.get("Stream_Id")) for r in rows)
print("queue/stream launches:", dict(qs))
print(f"{rx}: {len(key)} launches, {tot / 1e6:.1f} ms; overlapped by (ms):")
for n, o in ov.most_common(14):
    print(f"  {n[:50]:50s} {o / 1e6:9.1f}")
