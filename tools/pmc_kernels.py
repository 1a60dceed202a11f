"""HBM bytes per kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of one bench run,
against each kernel's algorithmic bytes:

  tools/pmc_kernels.py FETCH.csv WRITE.csv > profiles/pmc_<tag>_kernels.json

FETCH_SIZE / WRITE_SIZE are in KB (1024 B); FETCH_SIZE is doubled (gfx950 reports half the bytes
of wide streaming reads, MI355X_MICROARCH.md HBM section).  Algorithmic bytes per dispatch from its
grid: k_mask_r reads and writes every (frame, bin) of the 8192-point spectrogram (grid = tracks x 65
workgroups x 64 lanes; F8 = 15,488 frames of a 3-min track, 4,097 bins); k_hpcp reads every bin of
its frames (one thread per frame); k_features reads bins 0..1024 of its frames (252 frames per
256-thread workgroup).  Frame counts from grids are upper bounds (the last tile of a track is
partial), so the ratios are lower bounds of the true over-fetch.
"""
import csv
import json
import re
import sys

F8, B8, B2 = 15488, 4097, 1025
BAND, NBLK = 912, 65  # default key path at 44.1 kHz: HPCP's peak band [18, 929] and 65 64-bin block sums
KERNELS = {
    "k_mask_r": lambda grid: grid / (65 * 64) * F8 * B8 * 4 * 2,
    "k_hpcp": lambda grid: grid * B8 * 4,
    # band path: the mask reads every bin, writes the band and the block sums;
    # HPCP reads the band and the block sums
    "k_mask_rp": lambda grid: grid / (65 * 64) * F8 * (B8 + BAND + NBLK) * 4,
    "k_hpcp_band": lambda grid: grid * (BAND + NBLK) * 4,
    "k_features": lambda grid: grid / 256 * 252 * B2 * 4,
}


def load(path, counter):
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        k = next((k for k in KERNELS if re.search(r"\b" + k + r"\b|" + k + "<|" + k + r"\(", name)), None)
        if k is None:
            continue
        d = per.setdefault(k, {})
        e = d.setdefault(int(r["Dispatch_Id"]), {"bytes": 0.0, "grid": int(r.get("Grid_Size", 0) or 0)})
        e["bytes"] += float(r["Counter_Value"]) * 1024.0
    return per


fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
out = {"source": f"{sys.argv[1]} (FETCH_SIZE pass), {sys.argv[2]} (WRITE_SIZE pass); tools/pmc_kernels.py",
       "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KB = 1024 B", "kernels": {}}
for k in KERNELS:
    f, w = fetch.get(k, {}), write.get(k, {})
    if not f or not w:
        continue
    rd = 2.0 * sum(e["bytes"] for e in f.values())
    wr = sum(e["bytes"] for e in w.values())
    alg = sum(KERNELS[k](e["grid"]) for e in f.values())
    out["kernels"][k] = {"dispatches": len(f), "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                         "algorithmic_bytes": alg, "hbm_over_algorithmic": round((rd + wr) / alg, 4) if alg else None}
print(json.dumps(out, indent=1))
