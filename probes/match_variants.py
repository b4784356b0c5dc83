"""Diagnostics (not product, not tests): time the matcher kernels of one or
more builds of libscm.so on the same synthetic table, serial mode.
usage: python probes/match_variants.py LIB.so [LIB2.so ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_one(lib, images, kpts, overlap, reps):
    os.environ["SCM_SERIAL"] = "1"
    from scanner_colmap_amd import _abi
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    imgs = Corridor(images, kpts, overlap, seed=5).images(0, images, workers=16)
    ids, kps, descs = table_rows(imgs)
    _abi.load_library(lib)
    ctx = _abi.Context(0)
    ctx.table_load(ids, kps, descs)
    best = None
    for _ in range(reps):
        ctx.table_run_packed(overlap, 0, images)
        t = ctx.table_timings()
        best = t if best is None or t["match_ms"] < best["match_ms"] else best
    npairs = sum(min(overlap - 1, images - 1 - i) for i in range(images))
    tf = 2 * 128 * kpts * kpts * npairs / (best["match_ms"] * 1e-3) / 1e12
    print(f"{os.path.basename(lib)}: pairs {npairs} match {best['match_ms']:.2f} ms "
          f"({tf:.0f} TF/s) finalize {best['finalize_ms']:.2f} verify {best['verify_ms']:.2f}",
          flush=True)
    ctx.close()


if __name__ == "__main__":
    if len(sys.argv) > 2 or (len(sys.argv) == 2 and not sys.argv[1].startswith("--one=")):
        for lib in sys.argv[1:]:
            r = subprocess.run([sys.executable, __file__, "--one=" + lib], timeout=600)
            if r.returncode != 0:
                sys.exit(r.returncode)
    else:
        run_one(sys.argv[1][6:], int(os.environ.get("IMAGES", "80")), 8192, 20, 3)
