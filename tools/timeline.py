"""GPU busy fraction and largest idle gaps from a rocprofv3 kernel trace (csv).
usage: tools_timeline.py run_kernel_trace.csv [from_ms]   (from_ms: skip kernels starting earlier)"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:40]) for r in rows)
t00 = iv[0][0]
if len(sys.argv) > 2:
    skip = [x for x in iv if x[0] - t00 >= float(sys.argv[2]) * 1e6]
    iv = skip if skip else iv
t0 = iv[0][0]; t1 = max(e for _, e, _ in iv)
busy = 0; cur_s, cur_e = iv[0][0], iv[0][1]; gaps = []
for s, e, n in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s; gaps.append((s - cur_e, cur_e - t00, n)); cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"span {(t1-t0)/1e6:.1f} ms busy {busy/1e6:.1f} ms ({100*busy/(t1-t0):.1f}%)")
gaps.sort(reverse=True)
print("largest gaps (ms, at ms, next kernel):")
for g, at, n in gaps[:15]: print(f"  {g/1e6:8.2f} {at/1e6:9.1f} {n}")
print("total gap", sum(g for g,_,_ in gaps)/1e6, "ms in", len(gaps), "gaps")
