"""The drop-in boundary (include/stratum_hip.h, libstratum_hip.so) without a GPU (CPU only).

* the library loads and exports every function the header declares;
* the Python binding's ctypes mirrors (sdsp_abi) have exactly the C layout (offset of every
  field checked against a compiled probe of the header);
* sdsp_config_default() == AnalysisConfig::default() (reference src/config.rs:594-744) as the
  CPU restatement states it, field by field;
* with no GPU the product path fails loudly (no CPU fallback).
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
import sdsp
import sdsp_abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "stratum_hip.h")


DEBUG_HEADER = os.path.join(ROOT, "include", "stratum_hip_debug.h")


def _declared_functions(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sdsp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_functions():
    lib = sdsp.lib()
    names = _declared_functions()
    assert "sdsp_analyze_audio" in names and "sdsp_analyze_batch" in names and len(names) >= 14
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_every_export_is_declared():
    """Every exported sdsp_* function is declared in include/stratum_hip.h (the boundary) or in
    include/stratum_hip_debug.h (test and probe entry points)."""
    lib_path = sdsp.lib()._name
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib_path]).decode()
    exported = sorted({ln.split()[-1] for ln in out.splitlines() if " T sdsp_" in ln})
    declared = set(_declared_functions()) | set(_declared_functions(DEBUG_HEADER))
    assert "sdsp_debug_set_test_hooks" in declared
    assert not [n for n in exported if n not in declared]
    assert not [n for n in declared if n not in exported]


def test_no_test_switch_read_from_environment():
    """The shipping library reads no test hook from the environment (they are set only through
    sdsp_debug_set_test_hooks), so a user's environment cannot fail or re-route real work."""
    data = open(sdsp.lib()._name, "rb").read()
    for name in (b"SDSP_TEST_FAIL_CHUNK", b"SDSP_DEVICE_LIST", b"SDSP_STFT_FRAME_PARALLEL", b"SDSP_SERIAL_STREAMS",
                 b"SDSP_NO_KEY_DEFER", b"SDSP_NO_ROW_REUSE", b"SDSP_HOST_TRACE", b"SDSP_BATCH_CHUNK_TRACKS",
                 b"SDSP_HBM_BUDGET_GB"):
        assert name not in data, name


def test_shipping_library_refuses_failure_injection():
    """Failure injection and the device override are compiled only into the test build
    (libstratum_hip_testhooks.so, -DSDSP_TEST_HOOKS): the shipping library refuses both (Not
    implemented) and keeps the frame-parallel STFT switch, which changes no result; the test build
    accepts all three.  No device is touched."""
    f = sdsp.lib().sdsp_debug_set_test_hooks
    dev = (C.c_int32 * 2)(0, 0)
    assert f(0, None, 0, 0) == 4
    assert f(-1, dev, 2, 0) == 4
    assert f(-1, None, 0, 1) == 0 and f(-1, None, 0, 0) == 0
    th = sdsp._load(sdsp.TESTHOOKS_LIB_PATH)
    assert th.sdsp_debug_set_test_hooks(0, dev, 2, 1) == 0
    assert th.sdsp_debug_set_test_hooks(-1, None, 0, 0) == 0
    data = open(sdsp.lib()._name, "rb").read()
    assert b"injected chunk failure" not in data and b"injected chunk failure" in open(th._name, "rb").read()


def test_key_energy_blocked_query():
    """sdsp_debug_key_energy_blocked names the configurations whose key_confidence / key_clarity
    are block-folded: the default path yes; tuning, log-frequency chroma, whitening,
    bass blend, key HPSS, another mask margin or power, no mask: no."""
    assert sdsp.key_energy_blocked() and sdsp.key_energy_blocked(sample_rate=22050)
    for k, v in (("enable_key_tuning_compensation", 1), ("enable_key_log_frequency", 1),
                 ("enable_key_hpss_harmonic", 1), ("enable_key_harmonic_mask", 0), ("key_spectrogram_smooth_margin", 8),
                 ("key_harmonic_mask_power", 1.0), ("enable_key_hpcp_bass_blend", 1), ("enable_key_hpcp", 0)):
        c = sdsp.default_config()
        setattr(c, k, v)
        assert not sdsp.key_energy_blocked(c), k


def test_library_reads_no_environment():
    """The schedule switches reach the library only through sdsp_debug_set_schedule (the Python
    layer maps the SDSP_* variables onto it): no source of the shipping library calls getenv."""
    src = os.path.join(ROOT, "stratum-dsp_amd", "csrc")
    for f in sorted(os.listdir(src)):
        if f.endswith((".hip", ".hpp", ".h", ".cpp")):
            assert "getenv" not in open(os.path.join(src, f)).read(), f


def test_version():
    v = sdsp.version()
    assert v.startswith("stratum-hip ") and v.endswith("gfx950")


STRUCTS = {"sdsp_config": sdsp_abi.SdspConfig, "sdsp_result": sdsp_abi.SdspResult,
           "sdsp_tempo_candidate": sdsp_abi.SdspTempoCandidate, "sdsp_stage_times": sdsp_abi.SdspStageTimes,
           "sdsp_confidence": sdsp_abi.SdspConfidence}


def test_struct_layout_matches_header(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in STRUCTS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-std=c11", "-o", str(exe), str(src)])
    out = subprocess.check_output([str(exe)]).decode().split("\n")
    c = {}
    for ln in out:
        if ln:
            k, v = ln.rsplit(" ", 1)
            c[k] = int(v)
    for cname, py in STRUCTS.items():
        assert c[f"{cname} size"] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert c[f"{cname}.{f}"] == getattr(py, f).offset, f"{cname}.{f}"


def _fields(cfg):
    out = {}
    for f, t in sdsp_abi.SdspConfig._fields_:
        v = getattr(cfg, f)
        if isinstance(v, C.Array):
            v = list(v)
        elif f.endswith("_ptr") or isinstance(v, (C._Pointer,)):
            continue
        out[f] = v
    return out


def test_config_default_matches_reference_defaults():
    got, want = _fields(sdsp.default_config()), _fields(oracle.default_config())
    diff = {k: (got[k], want[k]) for k in want if not (got[k] == want[k] or (got[k] != got[k] and want[k] != want[k]))}
    assert not diff, diff


def test_no_gpu_fails_loudly():
    if sdsp.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(sdsp.AnalysisError) as e:
        sdsp.analyze_audio(np.ones(44100, np.float32), 44100)
    assert "no HIP device" in str(e.value)
    with pytest.raises(sdsp.AnalysisError) as e:
        sdsp.analyze_batch([np.ones(44100, np.float32)], 44100)
    assert "no HIP device" in str(e.value)
