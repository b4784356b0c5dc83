"""Diagnostics (not product, not tests): randomized soak of the small-batch
path -- Scanner batches of two-image stencils from mixed geometry scenes
(random kinds, sizes, outlier fractions, seeds), every row compared with the
oracle's, speculative watermark decisions recomputed (SCM_DIAG_SPEC_CHECK=1).
usage: python probes/soak_small.py ; env SEEDS (20)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SCM_DIAG_SPEC_CHECK"] = "1"


def main():
    from oracle import oracle
    from scanner_colmap_amd import Context
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import descriptors_for_matches, geometry_scene
    kinds = ["general", "two_translations", "plane_and_depth", "planar", "translation", "random",
             "two_motions"]
    seeds = int(os.environ.get("SEEDS", "20"))
    bad = 0
    tot = {"pairs": 0, "spec_taken": 0, "spec_equal": 0, "spec_differ": 0, "spec_void": 0}
    with Context(0) as ctx:
        for seed in range(seeds):
            rng = np.random.default_rng(9000 + seed)
            n = int(rng.integers(3, 12))
            stencils, refs = [], []
            for i in range(n):
                kind = kinds[int(rng.integers(len(kinds)))]
                m = int(rng.integers(60, 1500))
                out = float(rng.uniform(0.0, 0.7))
                s = 100000 + 1000 * seed + i
                kp1, kp2, mt = geometry_scene(kind, m, s, outlier_frac=out)
                d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), s)
                ids, kps, descs = table_rows([(2 * s, kp1, d1), (2 * s + 1, kp2, d2)])
                stencils.append((ids, kps, descs))
                refs.append((kind, m, round(out, 2), oracle.execute_stencil(ids, kps, descs)))
            got_ids, got_tvgs = ctx.execute_batch(stencils)
            t = ctx.table_timings()
            for k in tot:
                if k != "pairs":
                    tot[k] += t[k]
            tot["pairs"] += n
            for j, (a, b) in enumerate(zip(got_ids, got_tvgs)):
                if (a, b) != refs[j][3]:
                    bad += 1
                    print(f"MISMATCH seed {seed} stencil {j} {refs[j][:3]}", flush=True)
            print(f"seed {seed}: {n} pairs, spec {t['spec_taken']}/{t['spec_equal']}/"
                  f"{t['spec_differ']}/{t['spec_void']}", flush=True)
    print(f"soak: {tot}, mismatched rows {bad}", flush=True)
    sys.exit(1 if bad or tot["spec_differ"] else 0)


if __name__ == "__main__":
    main()
