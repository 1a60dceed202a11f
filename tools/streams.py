"""Per-queue busy time of a rocprofv3 kernel trace over a time window: which stream is the
critical path of the two-stream pipeline.
usage: tools/streams.py run_kernel_trace.csv [from_ms]  (from_ms: skip kernels starting earlier)"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
t00 = min(int(r["Start_Timestamp"]) for r in rows)
frm = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 0.0
rows = [r for r in rows if int(r["Start_Timestamp"]) - t00 >= frm]
t0 = min(int(r["Start_Timestamp"]) for r in rows)
t1 = max(int(r["End_Timestamp"]) for r in rows)
by = collections.defaultdict(list)
for r in rows:
    by[r.get("Queue_Id", r.get("Stream_Id", "?"))].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
print(f"span {(t1 - t0) / 1e6:.1f} ms")
for q, iv in sorted(by.items()):
    iv.sort()
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e, _ in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    tot = collections.Counter()
    for s, e, n in iv:
        tot[n.split("(")[0].replace("void ", "")[:38]] += e - s
    top = ", ".join(f"{k} {v / 1e6:.0f}" for k, v in tot.most_common(6))
    print(f"queue {q}: {len(iv)} kernels, busy {busy / 1e6:.1f} ms ({100 * busy / (t1 - t0):.0f}%): {top}")
