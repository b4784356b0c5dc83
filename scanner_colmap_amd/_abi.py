"""ctypes binding of the product C ABI (include/scm.h, lib/libscm.so).

This is the Python-side FFI a Scanner job script (reference
integration/feature_matching.py:39-54) would use in place of
``db.load_op(libsequential_matching.so)``.  There is no CPU fallback: if
the HIP library cannot be loaded, or no gfx950 device is visible,
``Context`` raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, byref, c_char_p, c_double, c_float,
                    c_int, c_int32, c_int64, c_size_t, c_uint8, c_uint32,
                    c_void_p)

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SCM_LIB (diagnostics only): load another build of the library, e.g. a probes/build variant.
LIB_PATH = os.environ.get("SCM_LIB") or os.path.join(_HERE, "lib", "libscm.so")

SCM_OK = 0
SCM_E_INVALID = -1
SCM_E_DEVICE = -2
SCM_E_NOMEM = -3
SCM_E_CAPACITY = -4
SCM_E_STATE = -5

# Every function include/scm.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "scm_abi_version", "scm_last_error", "scm_default_options",
    "scm_parse_args", "scm_pair_seed", "scm_blob_free",
    "scm_context_create", "scm_context_destroy", "scm_match_pair",
    "scm_verify_pair", "scm_execute_stencil", "scm_execute_batch", "scm_stencil_stats",
    "scm_stencil_spec_stats", "scm_stencil_cache_clear",
    "scm_table_load",
    "scm_table_run", "scm_table_run_packed", "scm_table_run_passes", "scm_table_run_chunks",
    "scm_set_keep_matches",
    "scm_set_keep_matches_range", "scm_add_keep_matches_range",
    "scm_table_matches", "scm_table_timings", "scm_set_serial", "scm_extract_frames",
)


class MatchingOptions(Structure):
    """scm_matching_options (include/scm.h) = colmap.proto:6-65 + COLMAP
    TwoViewGeometry / RANSAC defaults."""
    _fields_ = [
        ("use_gpu", c_int32), ("gpu_index", c_int32),
        ("max_ratio", c_double), ("max_distance", c_double),
        ("cross_check", c_int32), ("max_num_matches", c_int32),
        ("max_error", c_float), ("confidence", c_double),
        ("min_num_trials", c_int32), ("max_num_trials", c_int32),
        ("min_inlier_ratio", c_double), ("min_num_inliers", c_int32),
        ("multiple_models", c_int32), ("guided_matching", c_int32),
        ("loop_detection", c_int32), ("overlap", c_int32),
        ("quadratic_overlap", c_int32),
        ("min_E_F_inlier_ratio", c_double), ("max_H_inlier_ratio", c_double),
        ("watermark_min_inlier_ratio", c_double),
        ("watermark_border_size", c_double), ("detect_watermark", c_int32),
        ("dyn_num_trials_multiplier", c_double), ("ransac_seed", c_uint32),
    ]


class Element(Structure):
    _fields_ = [("buffer", POINTER(c_uint8)), ("size", c_size_t)]


class Frame(Structure):
    """scm_frame: a Scanner Frame's buffer (height x width x channels bytes)."""
    _fields_ = [("data", POINTER(c_uint8)), ("width", c_int32), ("height", c_int32),
                ("channels", c_int32)]


class Blob(Structure):
    _fields_ = [("data", POINTER(c_uint8)), ("size", c_size_t)]


class ScmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"scm error {code}: {msg}")
        self.code = code


_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libscm.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built: run `make -C scanner_colmap_amd/csrc` "
                      "or __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    lib.scm_abi_version.restype = c_int32
    lib.scm_last_error.restype = c_char_p
    lib.scm_default_options.argtypes = [POINTER(MatchingOptions)]
    lib.scm_parse_args.argtypes = [c_void_p, c_size_t, POINTER(MatchingOptions)]
    lib.scm_pair_seed.argtypes = [c_uint32, c_uint32, c_uint32]
    lib.scm_pair_seed.restype = c_uint32
    lib.scm_blob_free.argtypes = [POINTER(Blob)]
    lib.scm_context_create.argtypes = [c_int32, POINTER(MatchingOptions), POINTER(c_void_p)]
    lib.scm_context_destroy.argtypes = [c_void_p]
    lib.scm_match_pair.argtypes = [c_void_p, c_void_p, c_int64, c_void_p, c_int64,
                                   c_void_p, c_int64, POINTER(c_int64)]
    lib.scm_verify_pair.argtypes = [c_void_p, c_void_p, c_int64, c_void_p, c_int64,
                                    c_void_p, c_int64, c_uint32, c_uint32, POINTER(Blob)]
    lib.scm_execute_stencil.argtypes = [c_void_p, c_int64, POINTER(Element),
                                        POINTER(Element), POINTER(Element),
                                        POINTER(Blob), POINTER(Blob)]
    lib.scm_execute_batch.argtypes = [c_void_p, c_int64, c_int64, POINTER(Element),
                                      POINTER(Element), POINTER(Element),
                                      POINTER(Blob), POINTER(Blob)]
    lib.scm_stencil_stats.argtypes = [c_void_p, POINTER(c_int64), POINTER(c_int64)]
    lib.scm_stencil_spec_stats.argtypes = [c_void_p, POINTER(c_int64), POINTER(c_int64),
                                           POINTER(c_int64)]
    lib.scm_stencil_cache_clear.argtypes = [c_void_p]
    lib.scm_table_load.argtypes = [c_void_p, c_int64, POINTER(Element),
                                   POINTER(Element), POINTER(Element)]
    lib.scm_table_run.argtypes = [c_void_p, c_int64, c_int64, c_int64,
                                  POINTER(Blob), POINTER(Blob)]
    lib.scm_table_run_packed.argtypes = [c_void_p, c_int64, c_int64, c_int64,
                                         POINTER(Blob), c_void_p]
    lib.scm_table_run_passes.argtypes = [c_void_p, c_int64, c_int64, c_int64, c_int64, PASS_FN,
                                         c_void_p]
    lib.scm_table_run_chunks.argtypes = [c_void_p, c_int64, c_int64, c_int64, CHUNK_FN, c_void_p]
    lib.scm_set_keep_matches.argtypes = [c_void_p, c_int32]
    lib.scm_set_keep_matches_range.argtypes = [c_void_p, c_int64, c_int64]
    lib.scm_add_keep_matches_range.argtypes = [c_void_p, c_int64, c_int64]
    lib.scm_table_matches.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_int64,
                                      POINTER(c_int64)]
    lib.scm_table_timings.argtypes = [c_void_p, POINTER(c_double), c_int32]
    lib.scm_set_serial.argtypes = [c_void_p, c_int32]
    lib.scm_extract_frames.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p]
    for name in EXPORTS:
        if name not in ("scm_abi_version", "scm_last_error", "scm_default_options",
                        "scm_pair_seed", "scm_blob_free", "scm_context_destroy"):
            getattr(lib, name).restype = c_int
    lib.scm_default_options.restype = None
    lib.scm_blob_free.restype = None
    lib.scm_context_destroy.restype = None
    _lib = lib
    return lib


def default_options() -> MatchingOptions:
    o = MatchingOptions()
    load_library().scm_default_options(byref(o))
    return o


def parse_args(data: bytes) -> MatchingOptions:
    o = MatchingOptions()
    buf = ctypes.create_string_buffer(data, len(data)) if data else None
    _check(load_library().scm_parse_args(buf, len(data), byref(o)))
    return o


def pair_seed(base: int, id1: int, id2: int) -> int:
    return int(load_library().scm_pair_seed(base, id1, id2))


def _check(rc: int) -> None:
    if rc != SCM_OK:
        msg = load_library().scm_last_error()
        raise ScmError(rc, msg.decode() if msg else "")


def _blob_bytes(b: Blob) -> bytes:
    out = ctypes.string_at(b.data, b.size) if b.size else b""
    load_library().scm_blob_free(byref(b))
    return out


_U8P = POINTER(c_uint8)
# Offset of a bytes object's data from its id() (CPython's PyBytesObject
# layout), measured once: bytes elements -- what Scanner hands over -- are
# passed by address with no per-element ctypes objects.
_probe = b"scm"
_BYTES_OFF = ctypes.cast(c_char_p(_probe), ctypes.c_void_p).value - id(_probe)


def _elements(chunks) -> tuple:
    """An scm_element array over a list of bytes / bytearray / numpy buffers,
    zero-copy (the buffers are kept alive by the returned tuple): a (pointer,
    size) uint64 table filled from the bytes objects' own data addresses."""
    n = len(chunks)
    tab = np.zeros((max(1, n), 2), dtype=np.uint64)
    keep = [tab]
    if n and set(map(type, chunks)) == {bytes}:
        # the common case (Scanner's elements), filled without a per-element
        # numpy store: ~15K elements per 256-stencil call
        tab[:n, 0] = np.fromiter(map(id, chunks), dtype=np.uint64, count=n) + np.uint64(_BYTES_OFF)
        tab[:n, 1] = np.fromiter(map(len, chunks), dtype=np.uint64, count=n)
        keep.append(chunks)
        return tab.ctypes.data_as(POINTER(Element)), keep
    for i, c in enumerate(chunks):
        if type(c) is bytes:
            tab[i, 0] = id(c) + _BYTES_OFF
            tab[i, 1] = len(c)
            continue
        a = np.frombuffer(c, dtype=np.uint8) if isinstance(c, (bytes, bytearray)) else c
        a = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        keep.append(a)
        tab[i, 0] = a.ctypes.data
        tab[i, 1] = a.nbytes
    keep.append(chunks)
    return tab.ctypes.data_as(POINTER(Element)), keep


# scm_pass_fn (include/scm.h): (user, pass, rows, rows_size, row_offsets)
PASS_FN = ctypes.CFUNCTYPE(None, c_void_p, c_int64, c_void_p, c_size_t, POINTER(c_int64))
CHUNK_FN = ctypes.CFUNCTYPE(None, c_void_p, c_int64, c_int64, c_void_p, c_size_t, POINTER(c_int64))


class _BlobOwner:
    """Frees a library-owned buffer (scm_blob_free) when the last numpy view
    of it dies: PackedRows.data and every slice of it keep this alive."""

    def __init__(self, blob: Blob):
        self.blob = blob

    def __del__(self):
        try:
            if self.blob is not None and self.blob.data:
                load_library().scm_blob_free(byref(self.blob))
                self.blob = None
        except Exception:
            pass


class PackedRows:
    """Output of scm_table_run_packed: one library-owned buffer plus the
    element offsets.  Element 2r is row r's pair_image_ids, element 2r+1 its
    two_view_geometries.  The buffer is freed (returned to the library's pool)
    only when this object and every view of `data` are gone, so views handed
    to a background gather stay valid however long it keeps them."""

    def __init__(self, blob: Blob, offsets: np.ndarray):
        self.offsets = offsets
        n = int(blob.size)
        if n:
            owner = _BlobOwner(blob)
            buf = (ctypes.c_uint8 * n).from_address(ctypes.addressof(blob.data.contents))
            buf._owner = owner  # the array's base chain ends here
            self.data = np.frombuffer(buf, dtype=np.uint8)
        else:
            _BlobOwner(blob)  # frees a zero-sized allocation at once
            self.data = np.zeros(0, dtype=np.uint8)

    def __len__(self) -> int:
        return (len(self.offsets) - 1) // 2

    def element(self, k: int) -> bytes:
        return self.data[self.offsets[k]:self.offsets[k + 1]].tobytes()

    def rows(self) -> tuple[list[bytes], list[bytes]]:
        n = len(self)
        return ([self.element(2 * r) for r in range(n)],
                [self.element(2 * r + 1) for r in range(n)])


class Context:
    """One kernel instance on one HIP device (SequentialMatchingCPUKernel
    constructor, sequential_matching.cc:30-33)."""

    def __init__(self, device: int = 0, options: MatchingOptions | None = None):
        self._lib = load_library()
        self._ptr = c_void_p()
        opts = options if options is not None else default_options()
        self.options = opts
        _check(self._lib.scm_context_create(device, byref(opts), byref(self._ptr)))

    def close(self) -> None:
        if self._ptr:
            self._lib.scm_context_destroy(self._ptr)
            self._ptr = c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- pair granularity -------------------------------------------------
    def match_pair(self, desc1: np.ndarray, desc2: np.ndarray) -> np.ndarray:
        d1 = np.ascontiguousarray(desc1, dtype=np.uint8).reshape(-1, 128)
        d2 = np.ascontiguousarray(desc2, dtype=np.uint8).reshape(-1, 128)
        cap = max(1, len(d1))  # one match per row at most (n1 without the cross-check)
        out = np.zeros((cap, 2), dtype=np.uint32)
        n = c_int64()
        _check(self._lib.scm_match_pair(self._ptr, d1.ctypes.data, len(d1), d2.ctypes.data,
                                        len(d2), out.ctypes.data, cap, byref(n)))
        return out[: n.value].copy()

    def verify_pair(self, kp1: np.ndarray, kp2: np.ndarray, matches: np.ndarray,
                    id1: int, id2: int) -> bytes:
        k1 = np.ascontiguousarray(kp1, dtype=np.float32).reshape(-1, 6)
        k2 = np.ascontiguousarray(kp2, dtype=np.float32).reshape(-1, 6)
        m = np.ascontiguousarray(matches, dtype=np.uint32).reshape(-1, 2)
        b = Blob()
        _check(self._lib.scm_verify_pair(self._ptr, k1.ctypes.data, len(k1), k2.ctypes.data,
                                         len(k2), m.ctypes.data, len(m), id1, id2, byref(b)))
        return _blob_bytes(b)

    # --- op granularity ---------------------------------------------------
    def execute_stencil(self, ids, kps, descs) -> tuple[bytes, bytes]:
        e_ids, k1 = _elements(ids)
        e_kps, k2 = _elements(kps)
        e_desc, k3 = _elements(descs)
        a, b = Blob(), Blob()
        _check(self._lib.scm_execute_stencil(self._ptr, len(ids), e_ids, e_kps, e_desc,
                                             byref(a), byref(b)))
        return _blob_bytes(a), _blob_bytes(b)

    def execute_batch(self, stencils) -> tuple[list[bytes], list[bytes]]:
        """scm_execute_batch over a list of stencils, each (ids, kps, descs)
        lists of equal length K: one (pair_image_ids, tvgs) element per
        stencil."""
        B = len(stencils)
        if B == 0:
            return [], []
        K = len(stencils[0][0])
        if any(len(st[0]) != K or len(st[1]) != K or len(st[2]) != K for st in stencils):
            raise ValueError("every stencil of a batch has the same size")
        e_ids, k1 = _elements([x for st in stencils for x in st[0]])
        e_kps, k2 = _elements([x for st in stencils for x in st[1]])
        e_desc, k3 = _elements([x for st in stencils for x in st[2]])
        a = (Blob * B)()
        b = (Blob * B)()
        _check(self._lib.scm_execute_batch(self._ptr, B, K, e_ids, e_kps, e_desc, a, b))
        return [_blob_bytes(a[i]) for i in range(B)], [_blob_bytes(b[i]) for i in range(B)]

    def stencil_stats(self) -> tuple[int, int]:
        """(images reused from HBM, images uploaded) by execute calls so far."""
        r, u = c_int64(), c_int64()
        _check(self._lib.scm_stencil_stats(self._ptr, byref(r), byref(u)))
        return r.value, u.value

    def stencil_spec_stats(self) -> tuple[int, int, int]:
        """(elements speculated, speculations refused by the sampled words,
        calls run again because a speculated key did not hold) so far."""
        a, b, c = c_int64(), c_int64(), c_int64()
        _check(self._lib.scm_stencil_spec_stats(self._ptr, byref(a), byref(b), byref(c)))
        return a.value, b.value, c.value

    def stencil_cache_clear(self) -> None:
        """Drop the execute() HBM image cache (Scanner Kernel::reset())."""
        _check(self._lib.scm_stencil_cache_clear(self._ptr))

    # --- table granularity ------------------------------------------------
    def table_load(self, ids, kps, descs) -> None:
        e_ids, k1 = _elements(ids)
        e_kps, k2 = _elements(kps)
        e_desc, k3 = _elements(descs)
        _check(self._lib.scm_table_load(self._ptr, len(ids), e_ids, e_kps, e_desc))

    def table_run(self, overlap: int, row_begin: int, row_end: int):
        n = row_end - row_begin
        a = (Blob * max(1, n))()
        b = (Blob * max(1, n))()
        _check(self._lib.scm_table_run(self._ptr, overlap, row_begin, row_end, a, b))
        return [_blob_bytes(a[i]) for i in range(n)], [_blob_bytes(b[i]) for i in range(n)]

    def table_run_packed(self, overlap: int, row_begin: int, row_end: int) -> PackedRows:
        n = row_end - row_begin
        offs = np.zeros(2 * n + 1, dtype=np.int64)
        b = Blob()
        _check(self._lib.scm_table_run_packed(self._ptr, overlap, row_begin, row_end, byref(b),
                                              offs.ctypes.data))
        return PackedRows(b, offs)

    def table_run_passes(self, overlap: int, row_begin: int, row_end: int, passes: int,
                         on_pass) -> None:
        """scm_table_run_passes: `passes` runs of the row range as one batch
        stream (no drain between passes); on_pass(k, PackedRows) receives pass
        k's rows as soon as they are serialised, in order."""
        n = row_end - row_begin
        err = []

        def cb(user, k, data, size, offs):
            try:
                b = Blob()
                b.data = ctypes.cast(data, POINTER(c_uint8))
                b.size = size
                o = np.ctypeslib.as_array(offs, shape=(2 * n + 1,)).copy()
                on_pass(int(k), PackedRows(b, o))
            except BaseException as e:  # noqa: BLE001 -- re-raised after the call
                err.append(e)

        fn = PASS_FN(cb)
        _check(self._lib.scm_table_run_passes(self._ptr, overlap, row_begin, row_end, passes, fn,
                                              None))
        if err:
            raise err[0]

    def table_run_chunks(self, overlap: int, row_begin: int, row_end: int, on_chunk) -> None:
        """scm_table_run_chunks: the rows of [row_begin, row_end) handed over
        batch by batch, in row order -- on_chunk(first_row, PackedRows) as
        soon as each batch is serialised (the multi-GPU gather starts on them
        while the next batches compute)."""
        err = []

        def cb(user, first, nrows, data, size, offs):
            try:
                b = Blob()
                b.data = ctypes.cast(data, POINTER(c_uint8))
                b.size = size
                o = np.ctypeslib.as_array(offs, shape=(2 * nrows + 1,)).copy()
                on_chunk(int(first), PackedRows(b, o))
            except BaseException as e:  # noqa: BLE001 -- re-raised after the call
                err.append(e)

        fn = CHUNK_FN(cb)
        _check(self._lib.scm_table_run_chunks(self._ptr, overlap, row_begin, row_end, fn, None))
        if err:
            raise err[0]

    def extract_frames(self, frames, image_ids=None) -> list:
        """SiftExtractionKernel::execute on each frame (H x W x C uint8 arrays;
        extraction_op.cc:70-121): a list of (keypoints, descriptors, camera)
        io.cc element bytes."""
        n = len(frames)
        ids = np.asarray(image_ids if image_ids is not None else range(n), dtype=np.uint64)
        keep = []
        arr = (Frame * max(1, n))()
        for i, f in enumerate(frames):
            a = np.ascontiguousarray(f, dtype=np.uint8)
            if a.ndim == 2:
                a = a[:, :, None]
            keep.append(a)
            arr[i].data = a.ctypes.data_as(POINTER(c_uint8))
            arr[i].height, arr[i].width, arr[i].channels = a.shape
        outs = [(Blob * max(1, n))() for _ in range(3)]
        _check(self._lib.scm_extract_frames(self._ptr, n, ids.ctypes.data, arr, outs[0], outs[1],
                                            outs[2]))
        return [tuple(_blob_bytes(o[i]) for o in outs) for i in range(n)]

    def set_serial(self, serial: bool = True) -> None:
        """Measurement only: stages one after the other (isolated kernel times)."""
        _check(self._lib.scm_set_serial(self._ptr, 1 if serial else 0))

    def set_keep_matches(self, keep: bool = True) -> None:
        _check(self._lib.scm_set_keep_matches(self._ptr, 1 if keep else 0))

    def set_keep_matches_range(self, row_begin: int, row_end: int) -> None:
        _check(self._lib.scm_set_keep_matches_range(self._ptr, row_begin, row_end))

    def add_keep_matches_range(self, row_begin: int, row_end: int) -> None:
        _check(self._lib.scm_add_keep_matches_range(self._ptr, row_begin, row_end))

    def table_matches(self, row: int, offset: int, cap: int = 1 << 16) -> np.ndarray:
        out = np.zeros((max(1, cap), 2), dtype=np.uint32)
        n = c_int64()
        _check(self._lib.scm_table_matches(self._ptr, row, offset, out.ctypes.data, cap,
                                           byref(n)))
        return out[: n.value].copy()

    def table_timings(self) -> dict:
        t = (c_double * 16)()
        _check(self._lib.scm_table_timings(self._ptr, t, 16))
        return {"match_ms": t[0], "finalize_ms": t[1], "verify_ms": t[2], "wall_ms": t[3],
                "match_launches": int(t[4]), "score_ms": t[5], "evals_f": int(t[6]),
                "evals_h": int(t[7]), "hash_ms": t[8], "stage_ms": t[9], "run_ms": t[10],
                "out_ms": t[11], "spec_taken": int(t[12]), "spec_equal": int(t[13]),
                "spec_differ": int(t[14]), "spec_void": int(t[15])}
