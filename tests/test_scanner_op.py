"""The Scanner op `SequentialMatchingGPU` (scanner_colmap_amd/scanner_op/
sequential_matching_gpu.cc), the drop-in for the reference's
`SequentialMatchingCPU` (integration/op_cpp/sequential_matching.cc:27-205):
compiled against a test stub of the Scanner API subset it uses
(tests/scanner_stub) and driven the way a Scanner worker drives a kernel —
instantiate by op name with a KernelConfig, execute() on one stencil of
io.cc elements, read the two output elements."""
import os
import subprocess

import numpy as np
import pytest

from scanner_colmap_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "scanner_stub")
OP_SRC = os.path.join(ROOT, "scanner_colmap_amd", "scanner_op", "sequential_matching_gpu.cc")
LIB_DIR = os.path.dirname(_abi.LIB_PATH)


def _build_driver(tmp_path):
    exe = tmp_path / "drive_op"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", STUB, "-I",
                    os.path.join(ROOT, "include"), os.path.join(STUB, "drive_op.cc"), OP_SRC,
                    "-L", LIB_DIR, "-lscm", f"-Wl,-rpath,{LIB_DIR}", "-o", str(exe)], check=True)
    return exe


def _write_stencil(d, ids, kps, descs, args=b""):
    for c, col in enumerate((ids, kps, descs)):
        for s, el in enumerate(col):
            (d / f"in_{c}_{s}").write_bytes(el)
    if args:
        (d / "args").write_bytes(args)


def test_op_compiles_against_scanner_api_and_links(tmp_path):
    _build_driver(tmp_path)


def _placements(exe, op):
    r = subprocess.run([str(exe), "--placements", op], capture_output=True, text=True, check=True)
    return [tuple(line.split()) for line in r.stdout.splitlines()]


def test_op_declares_cpu_placed_columns(tmp_path):
    """A GPU kernel whose columns are host bytes must say so
    (KernelBuilder::input_device / output_device): otherwise a Scanner
    worker would move the inputs to the GPU before execute() and treat the
    outputs as device buffers.  Every column of SequentialMatchingGPU is
    CPU-placed; the kernel itself holds a GPU."""
    exe = _build_driver(tmp_path)
    assert _placements(exe, "SequentialMatchingGPU") == [
        ("kernel", "GPU"),
        ("input", "image_ids", "CPU"), ("input", "keypoints", "CPU"),
        ("input", "descriptors", "CPU"),
        ("output", "pair_image_ids", "CPU"), ("output", "two_view_geometries", "CPU")]


def test_driver_refuses_gpu_placed_columns(tmp_path):
    """The stub driver refuses a GPU kernel that leaves a column on the GPU
    (it would receive host pointers where Scanner hands device pointers)."""
    src = tmp_path / "bad_op.cc"
    src.write_text("""
#include "scanner/api/kernel.h"
#include "scanner/api/op.h"
class BadKernel : public scanner::StenciledBatchedKernel {
 public:
  explicit BadKernel(const scanner::KernelConfig& c) : scanner::StenciledBatchedKernel(c) {}
  void execute(const scanner::StenciledBatchedElements&, scanner::BatchedElements&) override {}
};
REGISTER_OP(BadOp).stencil().input("image_ids").output("out");
REGISTER_KERNEL(BadOp, BadKernel).device(scanner::DeviceType::GPU)
    .output_device("out", scanner::DeviceType::CPU);
""")
    exe = tmp_path / "drive_bad"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", STUB,
                    os.path.join(STUB, "drive_op.cc"), str(src), "-o", str(exe)], check=True)
    d = tmp_path / "io"
    d.mkdir()
    (d / "in_0_0").write_bytes(b"\0" * 8)
    r = subprocess.run([str(exe), "BadOp", str(d), "1"], capture_output=True, text=True)
    assert r.returncode == 3 and "input image_ids is not placed on the CPU device" in r.stderr


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_op_aborts_without_gpu(tmp_path):
    """No CPU fallback: the kernel constructor aborts the worker (the
    reference's glog CHECK behaviour) when no gfx950 device exists."""
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    exe = _build_driver(tmp_path)
    ids, kps, descs = table_rows(Corridor(2, 64, 2, seed=3).images())
    d = tmp_path / "io"
    d.mkdir()
    _write_stencil(d, ids, kps, descs)
    r = subprocess.run([str(exe), "SequentialMatchingGPU", str(d), "2"], capture_output=True,
                       text=True)
    assert r.returncode != 0
    assert "scm_context_create failed" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("k,kpts,seed", [(5, 700, 41), (3, 300, 42), (1, 200, 43)])
def test_op_execute_matches_oracle(tmp_path, k, kpts, seed):
    from oracle import oracle
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    exe = _build_driver(tmp_path)
    ids, kps, descs = table_rows(Corridor(k, kpts, max(k, 2), seed=seed).images())
    d = tmp_path / "io"
    d.mkdir()
    _write_stencil(d, ids, kps, descs)
    r = subprocess.run([str(exe), "SequentialMatchingGPU", str(d), str(k)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ref_ids, ref_tvgs = oracle.execute_stencil(ids, kps, descs)
    assert (d / "out_0").read_bytes() == ref_ids
    assert (d / "out_1").read_bytes() == ref_tvgs


@pytest.mark.gpu
def test_op_parses_scanner_args(tmp_path):
    """Serialised SequentialMatchingArgs reach the kernel (here: a tighter
    max_ratio and min_num_inliers), compared with the oracle under the same
    options."""
    from oracle import oracle
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    # siftargs (field 4) { max_ratio (3, double) = 0.6, min_num_inliers (12, varint) = 40 }
    sift = bytes([0x19]) + np.float64(0.6).tobytes() + bytes([0x60, 40])
    args = bytes([0x22, len(sift)]) + sift
    exe = _build_driver(tmp_path)
    ids, kps, descs = table_rows(Corridor(4, 500, 4, seed=44).images())
    d = tmp_path / "io"
    d.mkdir()
    _write_stencil(d, ids, kps, descs, args)
    r = subprocess.run([str(exe), "SequentialMatchingGPU", str(d), "4"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    opts = oracle.default_options()
    opts.max_ratio = 0.6
    opts.min_num_inliers = 40
    ref_ids, ref_tvgs = oracle.execute_stencil(ids, kps, descs, opts)
    assert (d / "out_0").read_bytes() == ref_ids
    assert (d / "out_1").read_bytes() == ref_tvgs


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 5])
def test_op_batched_rows_match_table_oracle(tmp_path, batch):
    """A Scanner job over a 12-row table (stencil range(0, 4)) through the op:
    consecutive execute() calls of `batch` stencils each (the reference's
    default batch of 1, and a 5-stencil `.batch()` call with a short last
    call), stencils clamped at the table end as Scanner does; every output
    row equals the oracle's, and the HBM image cache is exercised across
    calls."""
    from oracle import oracle
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    exe = _build_driver(tmp_path)
    n, K = 12, 4
    ids, kps, descs = table_rows(Corridor(n, 600, K, seed=45).images())
    d = tmp_path / "io"
    d.mkdir()
    _write_stencil(d, ids, kps, descs)
    r = subprocess.run([str(exe), "SequentialMatchingGPU", str(d), str(K), "0", str(n), str(batch)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ref_ids, ref_tvgs = oracle.table_run(ids, kps, descs, K, 0, n)
    for row in range(n):
        assert (d / f"out_0_{row}").read_bytes() == ref_ids[row], row
        assert (d / f"out_1_{row}").read_bytes() == ref_tvgs[row], row


# ---------------------------------------------------------------------------
# SiftExtractionGPU (scanner_colmap_amd/scanner_op/sift_extraction_gpu.cc), the
# drop-in for the reference's SiftExtraction op (extraction_op.cc:22-130).
# ---------------------------------------------------------------------------
SIFT_OP_SRC = os.path.join(ROOT, "scanner_colmap_amd", "scanner_op", "sift_extraction_gpu.cc")


def _build_frame_driver(tmp_path):
    exe = tmp_path / "drive_frame_op"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", STUB, "-I",
                    os.path.join(ROOT, "include"), os.path.join(STUB, "drive_frame_op.cc"),
                    SIFT_OP_SRC, "-L", LIB_DIR, "-lscm", f"-Wl,-rpath,{LIB_DIR}", "-o", str(exe)],
                   check=True)
    return exe


def _write_frames(d, frames, ids):
    import struct
    for r, (f, i) in enumerate(zip(frames, ids)):
        a = np.ascontiguousarray(f, dtype=np.uint8)
        if a.ndim == 2:
            a = a[:, :, None]
        (d / f"in_0_{r}").write_bytes(struct.pack("<Q", i))
        (d / f"frame_{r}").write_bytes(a.tobytes())
        (d / f"shape_{r}").write_text(f"{a.shape[1]} {a.shape[0]} {a.shape[2]}")


def test_sift_op_compiles_against_scanner_api_and_links(tmp_path):
    _build_frame_driver(tmp_path)


def test_sift_op_declares_cpu_placed_columns(tmp_path):
    """SiftExtractionGPU reads the frame as host bytes (check_frame with
    CPU_DEVICE) and writes host outputs: every column is CPU-placed."""
    exe = _build_frame_driver(tmp_path)
    assert _placements(exe, "SiftExtractionGPU") == [
        ("kernel", "GPU"), ("input", "image_ids", "CPU"), ("input", "frames", "CPU"),
        ("output", "keypoints", "CPU"), ("output", "descriptors", "CPU"),
        ("output", "cameras", "CPU")]


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_sift_op_aborts_without_gpu(tmp_path):
    from scanner_colmap_amd.synthetic import synthetic_frame
    exe = _build_frame_driver(tmp_path)
    d = tmp_path / "io"
    d.mkdir()
    _write_frames(d, [synthetic_frame(32, 40, 1)], [3])
    r = subprocess.run([str(exe), "SiftExtractionGPU", str(d), "1"], capture_output=True, text=True)
    assert r.returncode != 0
    assert "scm_context_create failed" in r.stderr


@pytest.mark.gpu
def test_sift_op_execute_matches_oracle(tmp_path):
    """execute() per row, as a Scanner worker runs the op over a frame table:
    the three output elements equal the oracle's SiftExtractionKernel."""
    from oracle import oracle
    from scanner_colmap_amd.synthetic import synthetic_frame
    exe = _build_frame_driver(tmp_path)
    d = tmp_path / "io"
    d.mkdir()
    frames = [synthetic_frame(120, 160, 1), synthetic_frame(90, 70, 2, channels=1),
              synthetic_frame(64, 200, 3, channels=4)]
    ids = [11, 12, 13]
    _write_frames(d, frames, ids)
    subprocess.run([str(exe), "SiftExtractionGPU", str(d), str(len(frames))], check=True,
                   timeout=120)
    for r, (f, i) in enumerate(zip(frames, ids)):
        ref = oracle.sift_extract(f, i)
        got = tuple((d / f"out_{c}_{r}").read_bytes() for c in range(3))
        assert got == ref, f"row {r}"
