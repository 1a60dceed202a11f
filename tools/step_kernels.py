"""Per-step kernel time of a serial-stream rocprofv3 kernel trace of bench.py (one call = one step;
each call's sub-batches start with k_peak_abs): the kernels of the last complete call, summed by
name, busy time and span.  usage: tools/step_kernels.py run_kernel_trace.csv [subbatches_per_call]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 3
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sdsp::", "")
starts = [i for i, r in enumerate(rows) if name(r).startswith("k_peak_abs")]
calls = [starts[i] for i in range(0, len(starts), per)]
a, b = calls[-2], calls[-1]  # the last complete call (the probe launches follow the last one)
seg = rows[a:b]
tot = collections.Counter()
cnt = collections.Counter()
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot[name(r)] += d
    cnt[name(r)] += 1
busy = sum(tot.values())
span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
print(f"step: busy {busy:.1f} ms, span {span:.1f} ms")
for k, v in tot.most_common():
    print(f"{k[:44]:44s} n {cnt[k]:3d} {v:8.2f} ms {100 * v / busy:5.1f} %")
