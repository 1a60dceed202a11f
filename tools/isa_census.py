#!/usr/bin/env python3
"""Instruction census of a kernel's frame loop, from the gfx950 ISA hipcc emits.

    python tools/isa_census.py [--src csrc/k_stft.hip] [--kernel REGEX ...] [--flags "..."] [--out FILE]

Compiles one source of stratum-dsp_amd with the Makefile's flags to device assembly, finds each
matching kernel's outermost loop with the most instructions (the frame loop of the STFT kernels) and
counts its instructions per wave and iteration by class (the per-frame VALU figure divides by the
frames one iteration runs):
  valu (split into f32 add/sub, mul, fma, transcendental, move, select, integer), lds (ds_*), vmem
  (buffer_/global_ loads and stores), scratch (spill traffic), smem, salu, waitcnt, barrier.
It also reports the kernel's VGPR / LDS / spill figures (-Rpass-analysis=kernel-resource-usage).
bench.py reads the committed output (profiles/isa_census_stft.json) to state the STFT kernels'
VALU-issue fraction beside their HBM fraction.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "stratum-dsp_amd")
FLAGS = ("--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math "
         "-fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize")
TRANS = ("v_rsq_", "v_sqrt_", "v_rcp_", "v_exp_", "v_log_", "v_sin_", "v_cos_")

# kernel (mangled-name regex) -> (waves per frame, frames per loop iteration); the census is per frame
DEFAULT_KERNELS = {
    r"k_stft_slide8w3ILi1E": (4, 2),     # 256 threads per frame; the loop body runs two frames (hop 512)
    r"k_stft_slide2sILi4ELb1E": (1, 1),  # one wave per frame per iteration (4 strips per workgroup)
    r"k_stft_slide2sILi4ELb0E": (1, 1),
}


def classify(op):
    if op.startswith("v_"):
        if op.startswith(TRANS):
            return "valu_trans"
        if op.startswith("v_mov") or op.startswith("v_accvgpr"):
            return "valu_mov"
        if op.startswith("v_cndmask"):
            return "valu_select"
        if re.match(r"v_(add|sub|subrev)_f32", op):
            return "valu_addsub"
        if re.match(r"v_mul_f32", op):
            return "valu_mul"
        if re.match(r"v_(fma|fmac|fmaak|fmamk)_f32", op):
            return "valu_fma"
        if re.match(r"v_pk_", op):
            return "valu_packed"
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem_store" if "store" in op or "atomic" in op else "vmem_load"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def functions(asm):
    """{mangled name: list of (label or None, instruction or None, comment)} per kernel body."""
    out, cur, name = {}, None, None
    for ln in asm.splitlines():
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            name, cur = m.group(1), []
            out[name] = cur
            continue
        if cur is None:
            continue
        if ln.strip().startswith("s_endpgm"):
            cur.append((None, "s_endpgm", ""))
            cur = None
            continue
        m = re.match(r"^(\.LBB\w+):\s*(;.*)?$", ln)
        if m:
            cur.append((m.group(1), None, m.group(2) or ""))
            continue
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur.append((None, s.split()[0], ""))
    return out


def main_loop(body):
    """Instructions of the loop (header + every block "in Loop: Header=" it) with the most instructions."""
    headers = [lab for lab, _, c in body if lab and "Loop Header" in c]
    best = []
    for h in headers:
        key = h.replace(".L", "")
        ins, inside = [], False
        for lab, op, c in body:
            if lab:
                inside = lab == h or f"Header={key}" in c or (inside and "in Loop" in c and "Depth" in c and
                                                               f"Header={key}" in c)
                continue
            if inside and op:
                ins.append(op)
        if len(ins) > len(best):
            best = ins
    return best


def resources(src, flags):
    r = subprocess.run(["/opt/rocm/bin/hipcc"] + flags.split() + ["-I" + os.path.join(PKG, "csrc"), "--cuda-device-only",
                        "-c", "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage", src],
                       capture_output=True, text=True)
    res, fn = {}, None
    for ln in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            fn = m.group(1)
            res[fn] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|"
                      r"LDS Size \[bytes/block\]|TotalSGPRs): (\d+)", ln)
        if m and fn:
            res[fn][m.group(1)] = int(m.group(2))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(PKG, "csrc", "k_stft.hip"))
    ap.add_argument("--kernel", action="append", help="mangled-name regex (default: the STFT frame loops)")
    ap.add_argument("--waves-per-frame", type=int, default=1)
    ap.add_argument("--frames-per-iteration", type=int, default=1)
    ap.add_argument("--flags", default=FLAGS)
    ap.add_argument("--extra", default="", help="extra hipcc flags (variants)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    kernels = {k: (a.waves_per_frame, a.frames_per_iteration) for k in a.kernel} if a.kernel else DEFAULT_KERNELS
    flags = a.flags + " " + a.extra
    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "k.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc"] + flags.split() + ["-I" + os.path.join(PKG, "csrc"),
                               "--cuda-device-only", "-S", "-o", s, a.src])
        asm = open(s).read()
    fns = functions(asm)
    res = resources(a.src, flags)
    out = {"source": os.path.relpath(a.src, ROOT), "flags": flags.strip(), "kernels": {}}
    for pat, (wpf, fpi) in kernels.items():
        for name, body in fns.items():
            if not re.search(pat, name):
                continue
            loop = main_loop(body)
            cnt = {}
            for op in loop:
                c = classify(op)
                cnt[c] = cnt.get(c, 0) + 1
            valu = sum(v for k, v in cnt.items() if k.startswith("valu"))
            out["kernels"][name] = {
                "waves_per_frame": wpf, "frames_per_iteration": fpi, "loop_instructions_per_wave": len(loop),
                "valu_per_wave": valu, "valu_per_frame": valu * wpf / fpi, "classes_per_wave": dict(sorted(cnt.items())),
                "resources": res.get(name, {}),
            }
    js = json.dumps(out, indent=1)
    print(js)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    sys.exit(main())
