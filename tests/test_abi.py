"""C ABI of libscm.so (include/scm.h) on the CPU: the library loads, exports
every declared entry point, and its host-only functions (options, proto2
args decoding, per-pair seeds, struct layout) behave as documented.  No
compute calls: there is no GPU here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from scanner_colmap_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "scm.h")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(scm_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree():
    assert _declared() == sorted(_abi.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = _abi.load_library()
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\b(scm_[a-z0-9_]+)\b", out))
    assert set(_declared()) <= exported


def test_abi_version_matches_header():
    ver = int(re.search(r"#define SCM_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert _abi.load_library().scm_abi_version() == ver


def test_struct_layout_matches_c(tmp_path):
    """ctypes mirror of scm_matching_options / scm_element / scm_blob has the
    C compiler's size and field offsets."""
    fields = [f for f, _ in _abi.MatchingOptions._fields_]
    src = ['#include "scm.h"', "#include <stdio.h>", "#include <stddef.h>", "int main(void){",
           'printf("%zu %zu %zu\\n", sizeof(scm_matching_options), sizeof(scm_element), '
           "sizeof(scm_blob));"]
    for f in fields:
        src.append(f'printf("%zu\\n", offsetof(scm_matching_options, {f}));')
    src.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)],
                   check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    sizes = [int(x) for x in lines[:3]]
    assert sizes == [ctypes.sizeof(_abi.MatchingOptions), ctypes.sizeof(_abi.Element),
                     ctypes.sizeof(_abi.Blob)]
    offs = [int(x) for x in lines[3:]]
    assert offs == [getattr(_abi.MatchingOptions, f).offset for f in fields]


PROTO_DEFAULTS = dict(  # colmap.proto:6-65 (proto2 defaults) + COLMAP defaults
    use_gpu=0, gpu_index=-1, max_ratio=0.8, max_distance=0.7, cross_check=1,
    max_num_matches=32768, max_error=4.0, confidence=0.999, min_num_trials=30,
    max_num_trials=10000, min_inlier_ratio=0.25, min_num_inliers=15, multiple_models=0,
    guided_matching=0, loop_detection=0, overlap=10, quadratic_overlap=0,
    min_E_F_inlier_ratio=0.95, max_H_inlier_ratio=0.8, watermark_min_inlier_ratio=0.7,
    watermark_border_size=0.1, detect_watermark=1, dyn_num_trials_multiplier=3.0,
    ransac_seed=0)


def test_default_options():
    o = _abi.default_options()
    for k, v in PROTO_DEFAULTS.items():
        assert getattr(o, k) == pytest.approx(v), k


def test_default_options_match_oracle():
    from oracle import oracle
    a, b = _abi.default_options(), oracle.default_options()
    for f, _ in _abi.MatchingOptions._fields_:
        assert getattr(a, f) == getattr(b, f), f


# --- proto2 wire encoding (written out by hand from colmap.proto) ---------
def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wt):
    return _varint((field << 3) | wt)


def _sift_args(**kw):
    b = b""
    if "use_gpu" in kw:
        b += _key(1, 0) + _varint(int(kw["use_gpu"]))
    if "gpu_index" in kw:
        s = kw["gpu_index"].encode()
        b += _key(2, 2) + _varint(len(s)) + s
    for name, field in (("max_ratio", 3), ("max_distance", 4), ("confidence", 8),
                        ("min_inlier_ratio", 11)):
        if name in kw:
            b += _key(field, 1) + np.float64(kw[name]).tobytes()
    for name, field in (("cross_check", 5), ("max_num_matches", 6), ("min_num_trials", 9),
                        ("max_num_trials", 10), ("min_num_inliers", 12),
                        ("multiple_models", 13), ("guided_matching", 14)):
        if name in kw:
            b += _key(field, 0) + _varint(int(kw[name]))
    if "max_error" in kw:
        b += _key(7, 5) + np.float32(kw["max_error"]).tobytes()
    return b


def _seq_args(sift=None, **kw):
    b = b""
    if "loop_detection" in kw:
        b += _key(1, 0) + _varint(int(kw["loop_detection"]))
    if "overlap" in kw:
        b += _key(2, 0) + _varint(kw["overlap"])
    if "quadratic_overlap" in kw:
        b += _key(3, 0) + _varint(int(kw["quadratic_overlap"]))
    if sift is not None:
        b += _key(4, 2) + _varint(len(sift)) + sift
    return b


def test_parse_empty_args_gives_defaults():
    o = _abi.parse_args(b"")
    for k, v in PROTO_DEFAULTS.items():
        assert getattr(o, k) == pytest.approx(v), k


def test_parse_args_overrides():
    sift = _sift_args(use_gpu=True, gpu_index="3", max_ratio=0.75, max_distance=0.6,
                      cross_check=False, max_num_matches=1000, max_error=2.5,
                      confidence=0.99, min_num_trials=40, max_num_trials=500,
                      min_inlier_ratio=0.3, min_num_inliers=20, guided_matching=True)
    o = _abi.parse_args(_seq_args(sift, overlap=25, quadratic_overlap=True))
    assert (o.use_gpu, o.gpu_index, o.cross_check, o.max_num_matches) == (1, 3, 0, 1000)
    assert (o.max_ratio, o.max_distance, o.confidence) == (0.75, 0.6, 0.99)
    assert o.max_error == np.float32(2.5)
    assert (o.min_num_trials, o.max_num_trials, o.min_num_inliers) == (40, 500, 20)
    assert o.min_inlier_ratio == 0.3 and o.guided_matching == 1
    assert (o.overlap, o.quadratic_overlap, o.loop_detection) == (25, 1, 0)
    # untouched fields keep their defaults
    assert o.max_H_inlier_ratio == 0.8 and o.detect_watermark == 1


def test_parse_args_skips_unknown_fields():
    unknown = _key(99, 0) + _varint(7) + _key(98, 2) + _varint(3) + b"abc"
    o = _abi.parse_args(_seq_args(_sift_args(max_ratio=0.5) + unknown, overlap=4) + unknown)
    assert o.max_ratio == 0.5 and o.overlap == 4


@pytest.mark.parametrize("bad", [b"\x10", b"\x22\x05ab", b"\x19\x00\x00", b"\xff" * 11])
def test_parse_args_rejects_malformed(bad):
    with pytest.raises(_abi.ScmError) as e:
        _abi.parse_args(bad)
    assert e.value.code == _abi.SCM_E_INVALID


def _seed_py(base, id1, id2):
    m = 0xFFFFFFFF
    h = base ^ 0x9E3779B9
    h ^= (id1 + 0x7F4A7C15 + ((h << 6) & m) + (h >> 2)) & m
    h ^= (id2 + 0x85EBCA77 + ((h << 6) & m) + (h >> 2)) & m
    return h & m


def test_pair_seed():
    from oracle import oracle
    rng = np.random.default_rng(0)
    for base, a, b in rng.integers(0, 2**32, size=(200, 3), dtype=np.uint64):
        base, a, b = int(base), int(a), int(b)
        s = _abi.pair_seed(base, a, b)
        assert s == _seed_py(base, a, b) == oracle.pair_seed(base, a, b)
    assert _abi.pair_seed(0, 1, 2) != _abi.pair_seed(0, 2, 1)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_context_without_gpu_fails_loudly():
    """No CPU fallback: creating a context without a gfx950 device errors."""
    with pytest.raises(_abi.ScmError) as e:
        _abi.Context(0)
    assert e.value.code == _abi.SCM_E_DEVICE


def test_null_arguments_are_rejected_without_a_gpu():
    """Entry points validate their arguments before touching the device:
    a null context or callback is SCM_E_INVALID (no crash, no GPU needed)."""
    lib = _abi.load_library()
    cb = _abi.PASS_FN(lambda *a: None)
    assert lib.scm_table_run_passes(None, 3, 0, 1, 1, cb, None) == _abi.SCM_E_INVALID
    a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    assert lib.scm_stencil_spec_stats(None, ctypes.byref(a), ctypes.byref(b),
                                      ctypes.byref(c)) == _abi.SCM_E_INVALID
    t = (ctypes.c_double * 12)()
    assert lib.scm_table_timings(None, t, 12) == _abi.SCM_E_INVALID
