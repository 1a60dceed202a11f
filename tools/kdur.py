"""Per-kernel launch durations of a rocprofv3 kernel trace, split by queue: count, mean and max
per launch (concurrent-pipeline durations include the wait for free CU slots).
usage: tools/kdur.py run_kernel_trace.csv [from_ms]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
t00 = min(int(r["Start_Timestamp"]) for r in rows)
frm = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 0.0
d = collections.defaultdict(list)
for r in rows:
    if int(r["Start_Timestamp"]) - t00 < frm:
        continue
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    d[(q, name)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for (q, name), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"q{q:>3} {name:40s} n {len(v):4d} total {sum(v):8.2f} ms mean {sum(v) / len(v):8.3f} max {max(v):8.3f}")
