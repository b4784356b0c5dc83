#!/usr/bin/env python3
"""Headline benchmark: sequential SIFT feature matching (descriptor matching +
two-view geometry + io.cc output rows) on synthetic 8192-keypoint images.

Metric (BASELINE.json): image-pairs/s (+ Gdesc-dist/s) on 8192x8192-keypoint
pairs at 1/2/4/8 GPUs.  One process per GPU; for N > 1 launch with
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
... bench.py --gpus N`.  A "step" is one full pass of the op over the rank's
shard of the `extraction` table (already resident in HBM): every pair of the
stencil range(0, overlap) is matched on MFMA, verified on the GPU and written
as io.cc rows; for N > 1 the rows are gathered to rank 0 over RCCL.
Scaling is weak: every rank owns `images` pivot rows of one long sequence.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "image-pairs/s + Gdesc-dist/s, 8192×8192-kpt pairs, 1/2/4/8 GPU"
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (spec)
I8_DENSE_PEAK_TOPS = 5000.0      # MI355X_MICROARCH.md matrix cores: i8 32x32x32 = 2x the bf16 rate
FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector, packed)
HBM_PEAK_GBPS = 8000.0           # MI355X_MICROARCH.md: HBM3E ~8 TB/s
# Reference residual arithmetic (upstream COLMAP estimators): ComputeSquaredSampsonError
# (F x1, F^T x2, x2^T F x1, e^2 / (4 squares)) and HomographyMatrixEstimator::Residuals
# (H s, one division, two differences, two squares).
SAMPSON_FLOPS = 33
TRANSFER_FLOPS = 20

# BASELINE.json configs (synthetic stand-ins; no dataset is present).
WORKLOADS = {
    "gerrard-hall-synth": dict(images=100, kpts=8192, overlap=10, seed=20251,
                               desc="Gerrard Hall stand-in: 100 imgs x 8192 kpts, overlap 10"),
    "synth-1000x8192-k20": dict(images=1000, kpts=8192, overlap=20, seed=20252,
                                desc="Synthetic 1000 imgs x 8192 SIFT kpts, overlap 20"),
    "south-building-synth": dict(images=128, kpts=8192, overlap=128, seed=20253,
                                 desc="South-Building stand-in: 128 imgs x 8192, exhaustive"),
    "synth-10000x4096-k50": dict(images=10000, kpts=4096, overlap=50, seed=20254,
                                 desc="Synthetic 10000 imgs x 4096 kpts, overlap 50"),
}


def parse():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", default="synth-1000x8192-k20", choices=sorted(WORKLOADS))
    p.add_argument("--images", type=int, default=None,
                   help="override the workload's image count (per rank for weak scaling)")
    p.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                   help="weak: every rank owns the workload's images (default); strong: the "
                        "workload's images in total, pivot rows split over the ranks "
                        "(BASELINE configs 4 and 5)")
    p.add_argument("--kpts", type=int, default=None, help="override keypoints per image")
    p.add_argument("--gen-workers", type=int, default=16)
    p.add_argument("--cpu-baseline-pairs", type=int, default=64)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--stencil-rows", type=int, default=1024,
                   help="rows of the Scanner drop-in path (scm_execute_batch) timed after the "
                        "table run, rank 0 at N = 1 (0 = skip): the most any --stencil-batches "
                        "leg takes; its images come from a corridor of their own (rows + overlap "
                        "images)")
    p.add_argument("--stream", action="store_true",
                   help="run the K steps as one streamed run (scm_table_run_passes: no pipeline "
                        "drain between steps) instead of one scm_table_run_packed call per step; "
                        "measured equal or slower (DESIGN.md section 4)")
    p.add_argument("--no-isolated", dest="isolated", action="store_false",
                   help="skip the extra serialised step that measures isolated kernel rates")
    p.add_argument("--gather", choices=("chunked", "step"), default=None,
                   help="N > 1: gather each batch's rows inside the step as soon as they are "
                        "serialised (scm_table_run_chunks), or each step's rows on a background "
                        "thread while the next step computes.  Default: step on nccl (the form "
                        "whose collectives have the simplest RCCL pattern; the chunked form's "
                        "per-peer receive threads have run on gloo only), chunked on gloo")
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="nccl = RCCL over xGMI, one GPU per rank (the measured path); gloo = a "
                        "rehearsal of the N > 1 sharding and gather with ranks sharing GPUs")
    p.add_argument("--extract-frames", type=int, default=32,
                   help="frames of the SIFT extraction leg (§8f rank 4; 0 = skip), rank 0 at N = 1")
    p.add_argument("--extract-height", type=int, default=1080)
    p.add_argument("--extract-width", type=int, default=1920)
    p.add_argument("--stencil-batches", default="1:128,16:256,64:128,256:1024,512:1024",
                   help="Scanner batch sizes (stencils per execute() call) to time, each as "
                        "batch[:rows] (rows default --stencil-rows)")
    return p.parse_args()


def cpu_threads() -> tuple[int, int, float | None]:
    """(threads to use, CPUs in this process's affinity mask, cgroup CPU
    quota).  On the GPU box the affinity mask shows the whole machine while
    the job's cgroup quota is its real CPU share."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, aff, quota


def sample_pairs(n_per_img: list, overlap: int, npairs: int) -> list:
    """The first `npairs` pairs of the stencil order (row 0's pairs, then row
    1's, ...) — the pairs the CPU baseline times and the parity check reads."""
    out = []
    T = len(n_per_img)
    for r in range(T):
        for j in range(r + 1, min(r + overlap, T)):
            out.append((r, j))
            if len(out) == npairs:
                return out
    return out


def late_pairs(n_per_img: list, overlap: int, row: int = 500, first: int = 12,
               tail_rows: int = 4) -> list:
    """Parity pairs past the first batch boundary (8,192 pairs = 431 rows of the
    default workload): the first `first` pairs of pivot row `row`, and every
    pair of the last `tail_rows` pivot rows that have pairs (the stencil
    clamped at the table's end, the short last batch)."""
    T = len(n_per_img)
    out = []
    if row < T - 1:
        out += [(row, j) for j in range(row + 1, min(row + overlap, T))][:first]
    for r in range(max(row + 1, T - 1 - tail_rows), T - 1):
        out += [(r, j) for j in range(r + 1, min(r + overlap, T))]
    return out


def oracle_fast(imgs: dict, pairs: list) -> dict:
    """The oracle's outputs for `pairs` with its BLAS-dot matcher
    (oracle.match_pair_fast, pinned to the scalar matcher by
    tests/test_oracle_match.py) and its LO-RANSAC; a thread per pair."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle

    def one(pr):
        i, j = pr
        m = oracle.match_pair_fast(imgs[i][2], imgs[j][2])
        return pr, (m, oracle.verify_pair(imgs[i][1], imgs[j][1], m, imgs[i][0], imgs[j][0]))

    with ThreadPoolExecutor(max_workers=max(1, cpu_threads()[0])) as ex:
        return dict(ex.map(one, pairs))


def cpu_baseline(imgs: dict, pairs: list) -> tuple[dict, dict]:
    """The CPU oracle (faithful restatement of the reference op's matcher +
    TwoViewGeometry, SURVEY.md §8d: scalar ColMajor-strided integer dot
    matrix, two one-way scans, sequential LO-RANSAC F + H + watermark) timed
    on this host, one worker thread per CPU of the job's share, each taking
    whole pairs (a Scanner pipeline instance per core).  Reported, not
    optimised.  Returns the baseline and the oracle's per-pair outputs (raw
    matches, TVG bytes) for the parity check of the timed GPU run."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle

    if not pairs:
        return None, {}
    oracle.lib()
    threads, aff, quota = cpu_threads()
    lat = {}
    res = {}

    def work(pr):
        i, j = pr
        t = time.perf_counter()
        m = oracle.match_pair(imgs[i][2], imgs[j][2])
        tvg = oracle.verify_pair(imgs[i][1], imgs[j][1], m, imgs[i][0], imgs[j][0])
        lat[pr] = time.perf_counter() - t
        res[pr] = (m, tvg)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(work, pairs))
    dt = time.perf_counter() - t0
    n1 = imgs[pairs[0][0]][2].shape[0]
    base = {"value": len(pairs) / dt, "unit": "image-pairs/s", "cores": min(threads, len(pairs)),
            "kind": "port", "cpu_model": cpu_model(), "nproc_affinity": aff,
            "cgroup_cpu_quota": quota,
            "pair_latency_s": round(sum(lat.values()) / len(lat), 2),
            "sample": f"the first {len(pairs)} pairs of the stencil order (rows "
                      f"{pairs[0][0]}..{pairs[-1][0]}) of {n1}x{n1} kpts, "
                      f"{min(threads, len(pairs))} worker threads, {dt:.1f} s wall "
                      "(oracle/oracle.cc, -O3 scalar restatement)"}
    return base, res


def parity_check(ctx, packed, row_lo: int, oracle_out: dict, pairs: list) -> dict:
    """Compare the timed run's GPU outputs for `pairs` with the oracle's:
    raw cross-checked matches bit-exact, io.cc TVG bytes equal."""
    from scanner_colmap_amd.codecs import split_tvg_list

    rows = {}
    ok_m = ok_t = True
    bad = []
    for (i, j) in pairs:
        if i not in rows:
            rows[i] = split_tvg_list(packed.element(2 * (i - row_lo) + 1))
        m_ref, tvg_ref = oracle_out[(i, j)]
        m_gpu = ctx.table_matches(i, j - i, cap=max(1, len(m_ref) + 1))
        same_m = m_gpu.shape == m_ref.shape and bool((m_gpu == m_ref).all())
        same_t = rows[i][j - i - 1] == tvg_ref
        ok_m &= same_m
        ok_t &= same_t
        if not (same_m and same_t):
            bad.append([i, j])
    return {"pairs": len(pairs), "matches_bit_exact": ok_m, "tvg_bytes_equal": ok_t,
            "mismatched_pairs": bad[:8],
            "checked_against": "oracle/oracle.cc (CPU restatement), same inputs and seeds",
            "source": "GPU outputs of the last timed step (raw matches kept for these rows)"}


def stencil_bench(ctx, src, overlap: int, legs: list) -> dict:
    """The Scanner drop-in path (scm_execute_batch, what the op's execute()
    calls; sequential_matching.cc:103-185): per leg (b, rows), output rows
    0..rows-1 of a sequence in consecutive calls of `b` stencils each (the
    job's `batch`; feature_matching.py:50-54), inputs as host io.cc elements
    (so every new image crosses PCIe inside the timed region), the HBM image
    cache carried across calls.  One untimed call warms each leg up."""
    ids, kps, descs = src
    n = len(ids)

    def stencils(r0, r1):
        out = []
        for r in range(r0, r1):
            sel = [min(r + s, n - 1) for s in range(overlap)]
            out.append(([ids[i] for i in sel], [kps[i] for i in sel], [descs[i] for i in sel]))
        return out

    res = {"stencil": overlap, "inputs": "host io.cc elements (PCIe inside the timed region)",
           "source": f"a corridor of {n} images (8192 kpts) of its own"}
    for b, rows in legs:
        rows = min(rows, n)
        calls = [stencils(r0, min(rows, r0 + b)) for r0 in range(0, rows, b)]
        ctx.execute_batch(calls[0])  # warm-up (buffers, cache)
        r0_, u0_ = ctx.stencil_stats()
        s0_ = ctx.stencil_spec_stats()
        t0 = time.perf_counter()
        npairs = 0
        for c in calls:
            a, _ = ctx.execute_batch(c)
            npairs += sum(int(np.frombuffer(x[:8], np.uint64)[0]) for x in a)
        dt = time.perf_counter() - t0
        r1_, u1_ = ctx.stencil_stats()
        s1_ = ctx.stencil_spec_stats()
        res[f"batch{b}"] = {"pairs_per_s": round(npairs / dt, 1), "ms_per_call": round(dt / len(calls) * 1e3, 2),
                            "rows": rows, "calls": len(calls), "pairs": npairs,
                            "images_uploaded": u1_ - u0_, "images_reused": r1_ - r0_,
                            "keys_speculated": s1_[0] - s0_[0], "speculation_refused": s1_[1] - s0_[1],
                            "calls_rerun": s1_[2] - s0_[2]}
    return res


def extraction_bench(ctx, frames: int, height: int, width: int, check: bool, cpu: bool) -> dict:
    """§8f rank 4, the producer of the table: scm_extract_frames (GPU SIFT,
    SiftExtractionKernel::execute, extraction_op.cc:70-121) on `frames`
    synthetic frames (4 distinct textures, host buffers in: PCIe inside the
    timed region), its parity on one frame against the oracle, and the
    oracle's frames/s on the job's CPU share (one frame per thread)."""
    from concurrent.futures import ThreadPoolExecutor
    from scanner_colmap_amd.codecs import decode_keypoints
    from scanner_colmap_amd.synthetic import synthetic_frame

    uniq = [synthetic_frame(height, width, 300 + i) for i in range(4)]
    batch = [uniq[i % 4] for i in range(frames)]
    ctx.extract_frames(batch[:4])  # warm-up (slots, workspaces)
    t0 = time.perf_counter()
    out = ctx.extract_frames(batch, list(range(frames)))
    dt = time.perf_counter() - t0
    res = {"frames": frames, "size": f"{width}x{height}x3", "frames_per_s": round(frames / dt, 2),
           "ms_per_frame": round(dt / frames * 1e3, 3),
           "features_per_frame": round(sum(len(decode_keypoints(o[0])) for o in out) / frames, 1),
           "inputs": "host frame buffers (PCIe inside the timed region)",
           "dominant_kernel": "descriptor_kernel (profiles/r03_sift_kernel_stats.csv)"}
    if check or cpu:
        from oracle import oracle
    if check:
        ref = oracle.sift_extract(batch[1], 1)
        res["parity"] = {"frames": 1, "elements_byte_equal": out[1] == ref,
                         "checked_against": "oracle/sift_oracle.cc"}
    if cpu:
        threads, aff, quota = cpu_threads()
        n = min(threads, 16)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(lambda i: oracle.sift_extract(uniq[i % 4], i), range(n)))
        cdt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n / cdt, 3), "unit": "frames/s", "cores": n,
                               "kind": "port", "sample": f"{n} frames of {width}x{height}, one per "
                               f"thread, {cdt:.1f} s wall (oracle/sift_oracle.cc, scalar VLFeat "
                               "restatement)"}
    return res


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def lib_sha16() -> str:
    """sha256[:16] of the libscm.so this process loads (PMC summaries record
    the hash of the library they profiled; a summary of another build is
    reported as stale, never as this run's figures)."""
    import hashlib
    from scanner_colmap_amd._abi import LIB_PATH
    return hashlib.sha256(open(LIB_PATH, "rb").read()).hexdigest()[:16]


def pmc_summary_file(pattern: str):
    """The committed PMC summary to use: the one recorded for the library this
    process loads (lib_sha16), else the last by name (then reported stale)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        return None
    sha = lib_sha16()
    for f in reversed(files):
        try:
            if json.load(open(f)).get("lib_sha16") == sha:
                return f
        except (OSError, ValueError):
            continue
    return files[-1]


def pmc_traffic(workload: str, kpts: int, images: int, kernel: str):
    """HBM bytes per matcher launch from the committed rocprofv3 PMC summary
    of this workload (profiles/rNN_pmc_match.json, profiles/pmc_summary.py),
    or None when no summary matches the configuration being run."""
    f = pmc_summary_file("r*_pmc_match.json")
    if f is None:
        return None
    d = json.load(open(f))
    wl = WORKLOADS.get(workload, {})
    if (d.get("workload") != workload or kpts != wl.get("kpts") or images != wl.get("images")
            or d.get("kernel") != kernel):
        return None
    return d, os.path.relpath(f, ROOT)


def pmc_sq(kernels: tuple):
    """MFMA / VALU utilisation of the given kernels from the committed
    rocprofv3 SQ summary (profiles/rNN_pmc_sq.json, profiles/pmc_sq_summary.py:
    SQ_INSTS_VALU / SQ_INSTS_MFMA, SQ_VALU_MFMA_BUSY_CYCLES and
    SQ_ACTIVE_INST_VALU over the chip's SIMD cycles), or None."""
    f = pmc_summary_file("r*_pmc_sq.json")
    if f is None:
        return None
    d = json.load(open(f))
    out = {k: d[k] for k in kernels if k in d}
    if out:
        out["lib_sha16"] = d.get("lib_sha16")
    return (out, os.path.relpath(f, ROOT)) if out else None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    wl = dict(WORKLOADS[args.workload])
    kpts = args.kpts or wl["kpts"]
    overlap = wl["overlap"]
    from scanner_colmap_amd import distributed as sd
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor

    plan = sd.ShardPlan(args.images or wl["images"], overlap, world, rank, args.scaling)
    total_images = plan.total_images
    row_b, row_e = plan.row_begin, plan.row_end
    tab_b, tab_e = plan.table_begin, plan.table_end
    # Scene overlap = the stencil's (K = 50 and exhaustive runs included): every pair of a
    # stencil shares scene points, so every pair is matched and verified.
    corridor = Corridor(total_images, kpts, min(overlap, total_images), seed=wl["seed"])
    # Data generation happens before any GPU runtime call (forked workers).
    t0 = time.perf_counter()
    imgs = corridor.images(tab_b, tab_e, workers=args.gen_workers)
    gen_s = time.perf_counter() - t0
    ids, kps, descs = table_rows(imgs)
    n_per_img = [im[2].shape[0] for im in imgs]
    # The drop-in legs' stencils: images of a corridor of their own, so a leg
    # may take more rows than the table holds (generated here, before the GPU
    # runtime starts: forked workers).
    srows = args.stencil_rows if world == 1 else 0
    stencil_src = None
    if srows:
        s_imgs = Corridor(srows + overlap, kpts, overlap, seed=wl["seed"] + 7).images(
            0, srows + overlap, workers=args.gen_workers)
        stencil_src = table_rows(s_imgs)
        del s_imgs
    # Pairs the CPU baseline times and the parity check compares (rank 0, N = 1).
    check_pairs = (sample_pairs(n_per_img, overlap, args.cpu_baseline_pairs)
                   if world == 1 and args.cpu_baseline_pairs > 0 else [])
    # ... and pairs past the first batch boundary and at the table's end (parity only).
    tail_pairs = late_pairs(n_per_img, overlap) if check_pairs else []
    keep_rows = sorted({i for p in check_pairs + tail_pairs for i in p})
    sample_imgs = {i: imgs[i] for i in keep_rows}
    keep_hi = max([i for i, _ in check_pairs], default=-1) + 1
    del imgs

    import torch
    import torch.distributed as dist
    from scanner_colmap_amd import Context

    device = None
    gpu = local_rank if world > 1 else 0
    if world > 1 and args.dist_backend == "nccl":
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
        dist.init_process_group("nccl", device_id=device)
    elif world > 1:  # rehearsal of the N > 1 path on fewer GPUs: gloo gather, ranks share GPUs
        gpu = local_rank % max(1, torch.cuda.device_count())
        dist.init_process_group("gloo")
    ctx = Context(gpu)
    t_load = time.perf_counter()
    ctx.table_load(ids, kps, descs)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    table_load_ms = (time.perf_counter() - t_load) * 1e3
    del ids, kps, descs
    lr_b, lr_e = plan.local_rows

    # Pair count and algorithmic work of this rank's shard.
    npairs = 0
    gdesc = 0.0
    T = len(n_per_img)
    for r in range(lr_b, lr_e):
        for j in range(r + 1, min(r + overlap, T)):
            npairs += 1
            gdesc += float(n_per_img[r]) * n_per_img[j]

    if keep_hi > 0:  # raw matches of the parity rows are kept in every step (bounded copy)
        ctx.set_keep_matches_range(0, keep_hi)
        for r in sorted({i for i, _ in tail_pairs}):
            ctx.add_keep_matches_range(r, r + 1)
    last = {}

    if args.gather is None:
        args.gather = "step" if args.dist_backend == "nccl" else "chunked"
    chunked = world > 1 and args.gather == "chunked"

    def step():
        if chunked:
            # N > 1: each batch's io.cc rows travel to rank 0 as soon as they are
            # serialised, while the next batches compute; the step ends when
            # rank 0 holds every rank's rows
            plan.step_chunked(ctx, device=device)
            return ctx.table_timings()
        # N > 1 (--gather step): the step's io.cc rows travel to rank 0 on the
        # plan's gather thread while the next step computes (drained before the
        # clock stops)
        packed, _ = plan.step(ctx, device=device, background=world > 1, keep=False)
        last["packed"] = packed
        return ctx.table_timings()

    def streamed(k):
        # k steps as one batch stream (scm_table_run_passes): no pipeline drain
        # between steps; every step's rows are produced (and gathered for N > 1)
        last["packed"] = plan.run_passes(ctx, k, device=device, keep=False)
        return ctx.table_timings()

    if args.stream:
        if args.warmup > 0:
            streamed(args.warmup)
    else:
        for _ in range(args.warmup):
            step()
    plan.drain()
    if world > 1:
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    match_ms = 0.0
    verify_ms = 0.0
    final_ms = 0.0
    score_ms = 0.0
    evals_f = evals_h = 0
    launches = 0
    for tm in ([streamed(args.steps)] if args.stream else (step() for _ in range(args.steps))):
        match_ms += tm["match_ms"]
        verify_ms += tm["verify_ms"]
        final_ms += tm["finalize_ms"]
        score_ms += tm["score_ms"]
        evals_f += tm["evals_f"]
        evals_h += tm["evals_h"]
        launches += tm["match_launches"]
    t_tail = time.perf_counter()
    plan.drain()  # the last steps' gathers: the exposed tail of the overlapped gather
    gather_tail_ms = (time.perf_counter() - t_tail) * 1e3
    if chunked:  # per step: the rows still travelling once the compute is done
        gather_tail_ms = float(np.mean(plan.tail_ms[-args.steps:])) if plan.tail_ms else 0.0
    if world > 1:
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, float(npairs), gdesc], dtype=torch.float64,
                         device=device if device is not None else "cpu")
        mx = t.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        tot = t.clone()
        dist.all_reduce(tot[1:], op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        total_pairs = float(tot[1])
        total_gdesc = float(tot[2])
    else:
        total_pairs = float(npairs)
        total_gdesc = gdesc

    if rank == 0:
        steps = args.steps
        value = total_pairs * steps / elapsed
        flops_rank = 2.0 * 128.0 * gdesc * steps
        achieved_tf = flops_rank / (match_ms * 1e-3) / 1e12 if match_ms > 0 else None
        launches = max(1, launches)  # matcher launches the library reported
        avg_n = float(np.mean(n_per_img)) if n_per_img else 0.0
        bf16 = os.environ.get("SCM_MATCH_BF16", "0") == "1"  # else the default i8 matcher
        kernel = "match_tiles_kernel" if bf16 else "match_g8_kernel"
        peak = BF16_DENSE_PEAK_TFLOPS if bf16 else I8_DENSE_PEAK_TOPS
        # descriptors of both images, bf16 (2 B) or offset i8 (1 B) per element
        alg_bytes_launch = npairs * steps / launches * 2 * avg_n * 128 * (2 if bf16 else 1)
        pmc = (pmc_traffic(args.workload, kpts, total_images, kernel)
               if world == 1 and not args.images else None)
        sq = pmc_sq((kernel, "rs_score_kernel<1>", "rs_score_kernel<0>"))
        launch_s = match_ms * 1e-3 / launches  # average matcher launch (HIP events)
        hbm = {}
        util = {}
        stale = {}
        loaded_sha = lib_sha16()
        if pmc:
            gbps = pmc[0]["traffic_bytes_per_launch"] / launch_s / 1e9
            hbm = {"hbm_gbps": round(gbps, 1), "hbm_frac": round(gbps / HBM_PEAK_GBPS, 4)}
            if pmc[0].get("lib_sha16") != loaded_sha:
                stale["traffic"] = round(pmc[0]["traffic_bytes_per_launch"])
                stale["traffic_source"] = pmc[1]
                stale.update(hbm)
                stale["traffic_lib_sha16"] = pmc[0].get("lib_sha16")
                hbm = {}
                pmc = None
        if sq and kernel in sq[0]:
            k = sq[0][kernel]
            util = {"mfma_busy": round(k["mfma_busy"], 4), "valu_per_mfma": round(k["valu_per_mfma"], 2),
                    "util_source": f"{sq[1]} (SQ PMC, separate rocprofv3 passes of one bench step)"}
            if sq[0].get("lib_sha16") != loaded_sha:
                stale.update(util)
                stale["util_lib_sha16"] = sq[0].get("lib_sha16")
                util = {}
                sq = None
        if stale:
            stale["loaded_lib_sha16"] = loaded_sha
            stale["note"] = ("committed PMC summaries of another libscm.so build: not this run's "
                             "kernels, kept only for reference")
        cpu = parity = None
        if check_pairs:
            if args.no_cpu_baseline:  # parity only, with the oracle's BLAS-dot matcher
                from oracle import oracle
                ref = {}
                for (i, j) in check_pairs:
                    m = oracle.match_pair_fast(sample_imgs[i][2], sample_imgs[j][2])
                    ref[(i, j)] = (m, oracle.verify_pair(sample_imgs[i][1], sample_imgs[j][1], m,
                                                         sample_imgs[i][0], sample_imgs[j][0]))
            else:
                cpu, ref = cpu_baseline(sample_imgs, check_pairs)
            ref.update(oracle_fast(sample_imgs, tail_pairs))
            parity = parity_check(ctx, last["packed"], lr_b, ref, check_pairs + tail_pairs)
            parity["rows"] = sorted({i for i, _ in check_pairs + tail_pairs})
        # Isolated kernel rates: one extra untimed step with matching and verification
        # serialised (scm_set_serial; same bytes), so no stage shares the CUs.
        iso = None
        if world == 1 and args.isolated:
            ctx.set_serial(True)
            ti = step()
            ctx.set_serial(False)
            ops1 = 2.0 * 128.0 * gdesc
            sf1 = (SAMPSON_FLOPS + 1) * ti["evals_f"] + (TRANSFER_FLOPS + 1) * ti["evals_h"]
            iso = {"match_tops": round(ops1 / (ti["match_ms"] * 1e-3) / 1e12, 2),
                   "match_frac": round(ops1 / (ti["match_ms"] * 1e-3) / 1e12 / peak, 4),
                   "score_tflops": (round(sf1 / (ti["score_ms"] * 1e-3) / 1e12, 2)
                                    if ti["score_ms"] > 0 else None),
                   "score_frac": (round(sf1 / (ti["score_ms"] * 1e-3) / 1e12 / FP32_VECTOR_PEAK_TFLOPS, 4)
                                  if ti["score_ms"] > 0 else None),
                   "ms": {"match": round(ti["match_ms"], 3), "finalize": round(ti["finalize_ms"], 3),
                          "verify": round(ti["verify_ms"], 3), "score": round(ti["score_ms"], 3),
                          "wall": round(ti["wall_ms"], 3)},
                   "how": ("one extra untimed step after the timed region with matching and "
                           "verification serialised (scm_set_serial, output bytes identical): "
                           "each kernel alone on the GPU, HIP events")}
        extraction = (extraction_bench(ctx, args.extract_frames, args.extract_height,
                                       args.extract_width, check=bool(check_pairs),
                                       cpu=not args.no_cpu_baseline)
                      if world == 1 and args.extract_frames > 0 else None)
        legs = []
        for x in args.stencil_batches.split(","):
            if x:
                b, _, r = x.partition(":")
                legs.append((int(b), min(srows, int(r) if r else srows)))
        drop_in = stencil_bench(ctx, stencil_src, overlap, legs) if srows else None
        score_flops = (SAMPSON_FLOPS + 1) * evals_f + (TRANSFER_FLOPS + 1) * evals_h
        # SURVEY.md §8d headline fraction: kernel-1 work over the whole step's wall time.
        wall_tops = flops_rank / elapsed / 1e12
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "image-pairs/s",
            "gdesc_dist_per_s": round(total_gdesc * steps / elapsed / 1e9, 2),
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": ("bf16 MFMA" if bf16 else "i8 MFMA on offset u8 descriptors, int32 accumulate")
                     + " (exact u8 dot products) + f64 geometry",
            "data": "synthetic (seeded corridor scene, RootSIFT u8 descriptors; no dataset)",
            "config": {"workload": args.workload, "description": wl["desc"],
                       "images": total_images, "kpts": kpts, "overlap": overlap,
                       "pairs_per_step": int(total_pairs), "parallelism": f"pairs sharded x{world}",
                       "steps_as": ("one streamed run (scm_table_run_passes: the batches of step k+1 "
                                    "enter the GPU pipeline while step k's last batches verify)"
                                    if args.stream else "one scm_table_run_packed call per step"),
                       "dist_backend": (args.dist_backend if world > 1 else None)},
            "roofline": {
                "bound": "mfma",
                "kernel": kernel,
                "achieved": round(achieved_tf, 2) if achieved_tf else None,
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": round(achieved_tf / peak, 4) if achieved_tf else None,
                "frac_of_bf16_peak": (round(achieved_tf / BF16_DENSE_PEAK_TFLOPS, 4)
                                      if achieved_tf else None),
                "traffic": round(pmc[0]["traffic_bytes_per_launch"]) if pmc else None,
                "traffic_source": (f"{pmc[1]}: FETCH_SIZE x2 + WRITE_SIZE per launch, "
                                   f"separate rocprofv3 --pmc passes") if pmc else None,
                "algorithmic_bytes_per_launch": round(alg_bytes_launch),
                **hbm,
                **util,
                **({"stale_profile": stale} if stale else {}),
                "launches_per_step": round(launches / steps, 2),
                "wall_achieved": round(wall_tops, 2),
                "wall_frac": round(wall_tops / peak, 4),
                "wall_frac_of_bf16_peak": round(wall_tops / BF16_DENSE_PEAK_TFLOPS, 4),
                "algorithmic": ("2*N1*N2*128 ops per pair (one multiply-add = 2 ops, i8 or bf16); "
                                "per-launch time from HIP events; peak = dense MFMA peak of the "
                                "kernel's dtype (i8 5.0 POP/s, bf16 2.5 PFLOP/s); wall_* = the "
                                "same ops over the whole step's wall time (SURVEY.md §8d)"),
            },
            "roofline_verify": {
                "bound": "valu",
                "kernel": "rs_score_kernel<F> + rs_score_kernel<H>",
                "achieved": round(score_flops / (score_ms * 1e-3) / 1e12, 2) if score_ms > 0 else None,
                "peak": FP32_VECTOR_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": (round(score_flops / (score_ms * 1e-3) / 1e12 / FP32_VECTOR_PEAK_TFLOPS, 4)
                         if score_ms > 0 else None),
                "evals_per_step": {"F": evals_f // steps, "H": evals_h // steps},
                "valu_active": ({"H": round(sq[0]["rs_score_kernel<1>"]["valu_active_frac_of_simd_cycles"], 4),
                                 "F": round(sq[0]["rs_score_kernel<0>"]["valu_active_frac_of_simd_cycles"], 4),
                                 "source": sq[1]}
                                if sq and "rs_score_kernel<1>" in sq[0] and "rs_score_kernel<0>" in sq[0]
                                else None),
                "score_ms_per_step": round(score_ms / steps, 3),
                "algorithmic": ("reference residual arithmetic per (model, point): Sampson error "
                                f"{SAMPSON_FLOPS} flops (F), transfer error {TRANSFER_FLOPS} flops (H), "
                                "each + 1 compare, counted over the trials the sequential "
                                "LO-RANSAC scores up to its stop; time = HIP events around "
                                "each window's scoring kernels; peak = FP32 vector (packed) "
                                "157.3 TF (MI355X_MICROARCH.md): the kernels evaluate packed "
                                "fp32 filters with fp64 exact tests for undecided points"),
            },
            "isolated": iso,
            "stage_ms_per_step": {"match": round(match_ms / steps, 3),
                                  "finalize": round(final_ms / steps, 3),
                                  "verify": round(verify_ms / steps, 3)},
            "gather": ({"how": (("each batch's packed io.cc rows (a header + offsets + bytes, P2P "
                                 "messages per chunk) sent to rank 0 from a background thread as soon "
                                 "as the library serialises them (scm_table_run_chunks), inside the "
                                 "step; tail_ms_rank0 = mean per step of the gather left after rank "
                                 "0's compute") if chunked else
                                ("each step's packed io.cc rows (offsets + bytes, two P2P messages per "
                                 "rank) gathered to rank 0 on a background thread while the next step "
                                 "computes; the last ones drained inside the timed region")),
                        "backend": args.dist_backend,
                        "avg_gather_ms": (round(float(np.mean(plan.gatherer.ms)), 2)
                                          if plan.gatherer and plan.gatherer.ms else None),
                        "tail_ms_rank0": round(gather_tail_ms, 2)} if world > 1 else None),
            "cpu_baseline": cpu,
            "parity": parity,
            "drop_in": drop_in,
            "extraction": extraction,
            "table_load_ms": round(table_load_ms, 1),
            "pcie_inclusive_pairs_per_s": round(total_pairs / (elapsed / steps + table_load_ms * 1e-3), 2),
            "gen_s": round(gen_s, 1),
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
