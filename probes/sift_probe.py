"""Diagnostics (GPU box): time scm_extract_frames on synthetic frames.
usage: python probes/sift_probe.py [H W NFRAMES]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scanner_colmap_amd import Context  # noqa: E402
from scanner_colmap_amd.codecs import decode_keypoints  # noqa: E402
from scanner_colmap_amd.synthetic import synthetic_frame  # noqa: E402

h, w, n = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1080, 1920, 16)))
t = time.time()
uniq = [synthetic_frame(h, w, 100 + i) for i in range(4)]
frames = [uniq[i % 4] for i in range(n)]
print(f"gen {time.time() - t:.1f} s", flush=True)
with Context(0) as ctx:
    ctx.extract_frames(frames[:4])
    for rep in range(3):
        t = time.perf_counter()
        out = ctx.extract_frames(frames)
        dt = time.perf_counter() - t
        nk = sum(len(decode_keypoints(o[0])) for o in out)
        print(f"{h}x{w}: {n} frames {dt * 1e3:.1f} ms = {n / dt:.1f} frames/s, "
              f"{nk / n:.0f} features/frame", flush=True)
