"""Diagnostics (not product, not tests): table-path steps (scm_table_run_packed
over the bench workload's 1000 x 8192 table) timed from the host, with the
process's HIP runtime chosen by import order: PRE=torch initialises torch
first, so the library binds torch's bundled libamdhip64; otherwise the
system ROCm runtime the library was linked against.
usage: python probes/table_probe.py ; env PRE (none), STEPS (4), IMAGES (1000)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    if os.environ.get("PRE", "") == "torch":
        import torch
        torch.zeros(1, device="cuda")
    steps = int(os.environ.get("STEPS", "4"))
    n = int(os.environ.get("IMAGES", "1000"))
    from scanner_colmap_amd import Context
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    imgs = Corridor(n, 8192, 20, seed=20252).images(0, n, workers=16)
    ids, kps, descs = table_rows(imgs)
    hip = [l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l]
    ctx = Context(0)
    ctx.table_load(ids, kps, descs)
    hip = sorted(set(l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l))
    print("runtime", hip, flush=True)
    ws = []
    for s in range(steps + 1):
        t0 = time.perf_counter()
        ctx.table_run_packed(20, 0, n)
        w = (time.perf_counter() - t0) * 1e3
        if s:
            ws.append(w)
        print(f"step {s} {w:.1f} ms", flush=True)
    ws.sort()
    print(f"median step {ws[len(ws) // 2]:.1f} ms", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
