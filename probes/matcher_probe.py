"""Diagnostics (not product, not tests): time the matcher + finalize kernels
of a libscm.so build on a synthetic table in serial mode (SCM_SERIAL=1, the
stages one after the other, HIP-event times from scm_table_timings), and
check the table's raw matches of row 0 against the oracle's BLAS-dot matcher.
usage: python probes/matcher_probe.py [LIB.so] ; env IMAGES (40), KPTS (8192),
OVERLAP (20), REPS (3)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ.setdefault("SCM_SERIAL", "1")
    images = int(os.environ.get("IMAGES", "40"))
    kpts = int(os.environ.get("KPTS", "8192"))
    overlap = int(os.environ.get("OVERLAP", "20"))
    reps = int(os.environ.get("REPS", "3"))
    from scanner_colmap_amd import _abi
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    imgs = Corridor(1000, kpts, overlap, seed=20252).images(0, images, workers=8)
    ids, kps, descs = table_rows(imgs)
    lib = sys.argv[1] if len(sys.argv) > 1 else _abi.LIB_PATH
    _abi.load_library(lib)
    ctx = _abi.Context(0)
    ctx.table_load(ids, kps, descs)
    ctx.set_keep_matches_range(0, 1)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.table_run_packed(overlap, 0, images)
        wall = time.perf_counter() - t0
        t = ctx.table_timings()
        t["wall"] = wall
        best = t if best is None or t["match_ms"] < best["match_ms"] else best
    npairs = sum(min(overlap - 1, images - 1 - i) for i in range(images))
    tops = 2 * 128 * kpts * kpts * npairs / (best["match_ms"] * 1e-3) / 1e12
    from oracle import oracle
    def same(a, b):
        return a.shape == b.shape and bool((a == b).all())
    ok = all(same(ctx.table_matches(0, j), oracle.match_pair_fast(imgs[0][2], imgs[j][2]))
             for j in (1, overlap - 1))
    print(f"{os.path.basename(lib)} {os.environ.get('TAG', '')}: pairs {npairs} match "
          f"{best['match_ms']:.2f} ms ({tops:.0f} TOP/s) finalize {best['finalize_ms']:.2f} ms "
          f"verify {best['verify_ms']:.2f} ms launches {best['match_launches']} row0_ok {ok}",
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
