"""The Rust shim (rust/src/{ffi,lib}.rs) against the C ABI it binds (include/stratum_hip.h).  CPU
only: the image has no Rust toolchain, so the shim is checked as source.

- `ffi::sdsp_config` / `ffi::sdsp_result` / `ffi::sdsp_tempo_candidate` declare the header's fields
  in the header's order with the matching Rust types (#[repr(C)] layout equality);
- `to_c` assigns every `sdsp_config` field exactly once, from the AnalysisConfig field of the same
  name (Option -> has_x + x, Vec -> pointer + length);
- when the reference is present (this container), every `pub` field of AnalysisConfig
  (/root/reference/src/config.rs:8-592) is read by `to_c`;
- `error_from_c` maps all five AnalysisError variants (src/error.rs:7-22) and `from_c` fills every
  AnalysisResult / AnalysisMetadata / BeatGrid field (src/analysis/result.rs:144-263).
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = open(os.path.join(ROOT, "include", "stratum_hip.h")).read()
FFI = open(os.path.join(ROOT, "rust", "src", "ffi.rs")).read()
LIB = open(os.path.join(ROOT, "rust", "src", "lib.rs")).read()
REF_CONFIG = "/root/reference/src/config.rs"

CTYPES = {"float": "f32", "int32_t": "i32", "uint8_t": "u8", "uint32_t": "u32", "uint64_t": "u64", "int8_t": "i8",
          "char": "c_char"}


def c_fields(struct):
    body = HDR[HDR.index(f"typedef struct {struct} {{"):HDR.index(f"}} {struct};")]
    out = []
    for line in body.splitlines()[1:]:
        line = line.split("/*")[0].strip()
        if not line:
            continue
        m = re.match(r"(const )?(\w+)\s*(\*\*|\*)?\s*(\w+)(\[(\d+)\])?;", line)
        assert m, line
        _, ty, ptr, name, _, n = m.groups()
        t = CTYPES.get(ty, ty)
        if ptr == "*":
            t = ("*const " if line.startswith("const") else "*mut ") + t
        elif ptr == "**":
            t = "*mut *mut " + t
        if n:
            t = f"[{t}; {n}]"
        out.append((name, t))
    return out


def rust_fields(struct):
    body = FFI[FFI.index(f"pub struct {struct} {{"):]
    body = body[:body.index("\n}")]
    return [(m.group(1), m.group(2).strip()) for m in re.finditer(r"pub (\w+): ([^,]+),", body)]


@pytest.mark.parametrize("struct", ["sdsp_config", "sdsp_result", "sdsp_tempo_candidate"])
def test_ffi_struct_layout(struct):
    want = c_fields(struct)
    got = rust_fields(struct)
    assert [n for n, _ in got] == [n for n, _ in want]
    for (n, tr), (_, tc) in zip(got, want):
        tc = tc.replace("sdsp_tempo_candidate", "sdsp_tempo_candidate")
        assert tr == tc, (n, tr, tc)


def _to_c_body():
    s = LIB[LIB.index("fn to_c("):]
    s = s[s.index("ffi::sdsp_config {"):]
    return s[:s.index("\n    };")]


def test_to_c_assigns_every_field_once():
    body = _to_c_body()
    assigned = re.findall(r"^\s+(\w+): ", body, re.M)
    names = [n for n, _ in c_fields("sdsp_config")]
    assert sorted(assigned) == sorted(names)
    assert len(assigned) == len(set(assigned))
    for line in body.splitlines()[1:]:
        m = re.match(r"\s+(\w+): (.+),$", line)
        if not m:
            continue
        field, expr = m.groups()
        src = field[4:] if field.startswith("has_") else field[:-4] if field.endswith("_len") else field
        if field == "key_multi_scale_lengths":
            assert "keep.multi_scale_lengths" in expr
        elif field == "enable_ml_refinement":
            assert expr == "ml_refinement(c)"
        else:
            assert f"c.{src}" in expr, (field, expr)


@pytest.mark.skipif(not os.path.exists(REF_CONFIG), reason="reference source not present")
def test_to_c_reads_every_reference_field():
    pub = re.findall(r"^\s+pub (\w+): ", open(REF_CONFIG).read(), re.M)
    assert len(pub) == 125
    body = _to_c_body()
    for f in pub:
        if f == "enable_ml_refinement":
            assert "c.enable_ml_refinement" in LIB
        else:
            assert f"c.{f}" in body, f


def test_error_mapping_and_result_fields():
    s = LIB[LIB.index("fn error_from_c"):]
    s = s[:s.index("\n}\n")]
    for variant, prefix in [("InvalidInput", "Invalid input: "), ("DecodingError", "Decoding error: "),
                            ("ProcessingError", "Processing error: "), ("NotImplemented", "Not implemented: "),
                            ("NumericalError", "Numerical error: ")]:
        assert f'AnalysisError::{variant}(strip("{prefix}"))' in s, variant
    f = LIB[LIB.index("unsafe fn from_c"):]
    f = f[:f.index("\n}\n")]
    for field in ["bpm", "bpm_confidence", "key", "key_confidence", "key_clarity", "beat_grid", "grid_stability",
                  "downbeats", "beats", "bars", "duration_seconds", "sample_rate", "processing_time_ms",
                  "algorithm_version", "onset_method_consensus", "methods_used", "flags", "confidence_warnings",
                  "tempogram_candidates", "tempogram_multi_res_triggered", "tempogram_multi_res_used",
                  "tempogram_percussive_triggered", "tempogram_percussive_used"]:
        assert re.search(rf"\b{field}[:,]", f), field
