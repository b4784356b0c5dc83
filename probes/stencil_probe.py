"""Diagnostics (not product, not tests): per-call latency of the Scanner
drop-in path (scm_execute_batch with batch B) on the bench workload's first
rows.  Prints per-call wall and the HIP-event stage times of the call.
usage: python probes/stencil_probe.py ; env ROWS (40), B (1), KPTS (8192), K (20)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rows = int(os.environ.get("ROWS", "40"))
    B = int(os.environ.get("B", "1"))
    kpts = int(os.environ.get("KPTS", "8192"))
    K = int(os.environ.get("K", "20"))
    pre = os.environ.get("PRE", "")
    if pre == "torch":  # torch's HIP initialisation first (as in bench.py)
        import torch
        torch.zeros(1, device="cuda")
    elif pre in ("spin", "yield", "block"):  # the device's host-wait mode
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        flag = {"spin": 1, "yield": 2, "block": 4}[pre]
        print("hipSetDeviceFlags", pre, hip.hipSetDeviceFlags(flag), flush=True)
    from scanner_colmap_amd import Context
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    imgs = Corridor(1000, kpts, K, seed=20252).images(0, rows + K, workers=8)
    ids, kps, descs = table_rows(imgs)
    n = len(ids)
    ctx = Context(0)
    walls = []
    for r0 in range(0, rows, B):
        st = []
        for r in range(r0, min(rows, r0 + B)):
            sel = [min(r + s, n - 1) for s in range(K)]
            st.append(([ids[i] for i in sel], [kps[i] for i in sel], [descs[i] for i in sel]))
        t0 = time.perf_counter()
        ctx.execute_batch(st)
        w = (time.perf_counter() - t0) * 1e3
        t = ctx.table_timings()
        walls.append(w)
        py = w - t['hash_ms'] - t['stage_ms'] - t['run_ms'] - t['out_ms']
        print(f"call {r0 // B:3d} wall {w:7.2f} ms match {t['match_ms']:6.2f} finalize "
              f"{t['finalize_ms']:5.2f} verify {t['verify_ms']:6.2f} hash {t['hash_ms']:5.2f} "
              f"stage {t['stage_ms']:5.2f} run {t['run_ms']:5.2f} out {t['out_ms']:5.2f} "
              f"rest {py:5.2f}", flush=True)
    walls = sorted(walls[1:])
    print(f"median wall {walls[len(walls) // 2]:.2f} ms per call of {B} stencils", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
