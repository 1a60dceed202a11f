"""Derives profiles/pmc_stft<N>.json (HBM bytes / algorithmic bytes of the N-point sliding STFT
kernel) from two rocprofv3 PMC passes of one `bench.py ... --steps 1 --warmup 0
--no-cpu-baseline` command:

  tools/pmc_stft.py N FETCH.csv WRITE.csv BENCH.log > profiles/pmc_stft<N>.json

FETCH_SIZE / WRITE_SIZE are in KB (1024 B); FETCH_SIZE is doubled (gfx950 reports half the
bytes of wide streaming reads, MI355X_MICROARCH.md HBM section).  The algorithmic bytes come from
the bench line that run printed: roofline.bytes_per_launch x roofline.launches, the pipeline's
launches of the kernel in its one timed step.  Those are the kernel's first `launches` dispatches
(bench.py's isolated probe launches come after them and are excluded).
"""
import csv
import json
import sys

N = int(sys.argv[1])
KERNEL = "k_stft_slide8w3<" if N == 8192 else "k_stft_slide2s<"  # the pipeline's sliding-strip kernels


def dispatches(path, name):
    # the product kernel (k_stft_slide; k_stft_mag is its out-of-line fix-up pass)
    rows = [r for r in csv.DictReader(open(path))
            if r["Counter_Name"] == name and KERNEL in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"{path}: no {KERNEL} dispatch")
    by = {}
    for r in rows:
        by[int(r["Dispatch_Id"])] = by.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"]) * 1024.0
    return [by[k] for k in sorted(by)]


line = [ln for ln in open(sys.argv[4]) if ln.startswith("{")][-1]
rf = json.loads(line)["roofline"]
nl = int(rf.get("launches", 1))
alg = rf["bytes_per_launch"] * nl
fetch = 2.0 * sum(dispatches(sys.argv[2], "FETCH_SIZE")[:nl])
write = sum(dispatches(sys.argv[3], "WRITE_SIZE")[:nl])
print(json.dumps({
    "kernel": "k_stft_slide8w3" if N == 8192 else "k_stft_slide2s",
    "workload": f"bench.py one step, {nl} pipeline launch(es): {json.loads(line)['config']['workload']}",
    "source": f"{sys.argv[2]} (FETCH_SIZE pass), {sys.argv[3]} (WRITE_SIZE pass); "
              "separate rocprofv3 --pmc runs; tools/pmc_stft.py",
    "correction": "FETCH_SIZE x2 (gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md HBM section); KB = 1024 B",
    "launches": nl,
    "algorithmic_bytes": alg,
    "hbm_read_bytes": fetch,
    "hbm_write_bytes": write,
    "hbm_bytes": fetch + write,
    "hbm_over_algorithmic": round((fetch + write) / alg, 5),
}, indent=1))
