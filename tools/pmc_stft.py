"""Derives profiles/pmc_stft8192.json (HBM bytes / algorithmic bytes of k_stft_mag<8192>) from
two rocprofv3 PMC passes of `bench.py --tracks 64 --steps 1 --warmup 0 --no-cpu-baseline`:

  tools/pmc_stft.py FETCH.csv WRITE.csv BENCH.log > profiles/pmc_stft8192.json

FETCH_SIZE / WRITE_SIZE are in KB (1024 B); FETCH_SIZE is doubled (gfx950 reports half the
bytes of wide streaming reads, MI355X_MICROARCH.md HBM section).  The algorithmic bytes of the
launch come from the bench line that run printed (roofline.bytes_per_launch: one launch).
"""
import csv
import json
import sys

KERNEL = "k_stft_slide<8192"


def counter(path, name):
    # the 8192-point product kernel (k_stft_slide; k_stft_mag is its out-of-line fix-up pass);
    # the first dispatch is the bench launch, later ones are bench.py's isolated probe
    rows = [r for r in csv.DictReader(open(path))
            if r["Counter_Name"] == name and KERNEL in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"{path}: no {KERNEL} dispatch")
    first = min(int(r["Dispatch_Id"]) for r in rows)
    return sum(float(r["Counter_Value"]) for r in rows if int(r["Dispatch_Id"]) == first) * 1024.0


fetch = 2.0 * counter(sys.argv[1], "FETCH_SIZE")
write = counter(sys.argv[2], "WRITE_SIZE")
line = [ln for ln in open(sys.argv[3]) if ln.startswith("{")][-1]
alg = json.loads(line)["roofline"]["bytes_per_launch"]
print(json.dumps({
    "kernel": "k_stft_slide<8192,1,false>",
    "workload": "bench.py --tracks 64 --steps 1 --warmup 0 (one launch = 64 synthetic 3-min tracks)",
    "source": f"{sys.argv[1]} (FETCH_SIZE pass), {sys.argv[2]} (WRITE_SIZE pass); "
              "separate rocprofv3 --pmc runs; tools/pmc_stft.py",
    "correction": "FETCH_SIZE x2 (gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md HBM section); KB = 1024 B",
    "algorithmic_bytes_per_launch": alg,
    "hbm_read_bytes_per_launch": fetch,
    "hbm_write_bytes_per_launch": write,
    "hbm_bytes_per_launch": fetch + write,
    "hbm_over_algorithmic": round((fetch + write) / alg, 5),
}, indent=1))
