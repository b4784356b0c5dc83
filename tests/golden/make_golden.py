"""Regenerate the golden vectors in this directory (run from the repo root:
`python tests/golden/make_golden.py`).

Inputs are seeded synthetic cases; expected outputs come from the CPU oracle
(oracle/oracle.cc), whose own correctness is pinned by the known-answer tests
(tests/test_oracle_*.py) — the reference ships no fixtures for this path and
cannot be built or imported here, so parity at the COLMAP
boundary stays "unpinned" beyond those known answers.  The fixtures freeze
the oracle's outputs so that both the oracle (CPU suite) and the HIP path
(GPU suite) are checked against the same bytes on every run."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle  # noqa: E402
from scanner_colmap_amd.codecs import table_rows  # noqa: E402
from scanner_colmap_amd.synthetic import (Corridor, geometry_scene, random_descriptors,  # noqa: E402
                                          tie_stress_pair)

# Two-view-geometry outcome scenes (name, kind, matches, seed): one per branch of
# EstimateUncalibrated / DetectWatermark / the op's post-filter.
OUTCOME_CASES = (("general", "general", 300, 0), ("planar", "planar", 300, 1),
                 ("watermark", "translation", 300, 2), ("degenerate", "random", 40, 3),
                 ("few_inliers", "random", 300, 4), ("planar_big", "planar", 2000, 5),
                 ("watermark_big", "translation", 2000, 6))


def _blob_array(blobs):
    offs = np.cumsum([0] + [len(b) for b in blobs]).astype(np.int64)
    data = np.frombuffer(b"".join(blobs), np.uint8) if blobs else np.zeros(0, np.uint8)
    return offs, data.copy()


def main():
    out = {}
    # --- matcher cases ----------------------------------------------------------
    rng = np.random.default_rng(7)
    d1 = random_descriptors(333, 1)
    d2 = random_descriptors(517, 2)
    pick = rng.permutation(333)[:200]
    d2[rng.permutation(517)[:200]] = np.clip(
        d1[pick].astype(np.int64) + rng.integers(-4, 5, (200, 128)), 0, 255).astype(np.uint8)
    cases = [("random_ragged", d1, d2), ("tie_stress", *tie_stress_pair(400, 380, 3))]
    imgs = Corridor(6, 600, 4, seed=101).images()
    cases.append(("corridor", imgs[0][2], imgs[1][2]))
    for name, d1, d2 in cases:
        out[f"match_{name}_d1"] = d1
        out[f"match_{name}_d2"] = d2
        out[f"match_{name}_matches"] = oracle.match_pair(d1, d2)
    # --- geometry cases ---------------------------------------------------------
    for a, b in ((0, 1), (0, 3), (2, 3)):
        m = oracle.match_pair(imgs[a][2], imgs[b][2])
        out[f"verify_{a}{b}_kp1"] = imgs[a][1]
        out[f"verify_{a}{b}_kp2"] = imgs[b][1]
        out[f"verify_{a}{b}_matches"] = m
        out[f"verify_{a}{b}_ids"] = np.array([imgs[a][0], imgs[b][0]], np.uint32)
        out[f"verify_{a}{b}_tvg"] = np.frombuffer(
            oracle.verify_pair(imgs[a][1], imgs[b][1], m, imgs[a][0], imgs[b][0]), np.uint8)
    # --- whole table (io.cc rows) -------------------------------------------------
    ids, kps, descs = table_rows(imgs)
    out["table_ids"] = np.array([im[0] for im in imgs], np.uint32)
    for k, (lst) in (("kps", kps), ("descs", descs)):
        o, d = _blob_array(lst)
        out[f"table_{k}_offs"], out[f"table_{k}_data"] = o, d
    pa, pb = oracle.table_run(ids, kps, descs, 4, 0, len(imgs))
    out["table_overlap"] = np.array([4])
    out["table_pairs_offs"], out["table_pairs_data"] = _blob_array(pa)
    out["table_tvgs_offs"], out["table_tvgs_data"] = _blob_array(pb)
    # --- scalar known answers -----------------------------------------------------
    out["acosf_threshold"] = np.array([200499])
    out["num_trials_F_cap"] = np.array([oracle.num_trials(25000, 100000, 0.999, 3.0, 7)])
    np.savez_compressed(os.path.join(HERE, "golden_v1.npz"), **out)
    print("wrote", os.path.join(HERE, "golden_v1.npz"))
    outcomes()


def outcomes():
    """golden_outcomes.npz: per scene the keypoints, matches, image ids, the
    oracle's configuration before the post-filter, its F-inlier count and the
    io.cc TVG bytes after it."""
    out = {}
    for name, kind, m, seed in OUTCOME_CASES:
        kp1, kp2, mt = geometry_scene(kind, m, seed)
        ids = np.array([100 + seed, 200 + seed], np.uint32)
        cfg, ninl = oracle.verify_pair_config(kp1, kp2, mt, int(ids[0]), int(ids[1]))
        out[f"{name}_kp1"], out[f"{name}_kp2"], out[f"{name}_matches"] = kp1, kp2, mt
        out[f"{name}_ids"] = ids
        out[f"{name}_raw"] = np.array([cfg, ninl], np.int64)
        out[f"{name}_tvg"] = np.frombuffer(
            oracle.verify_pair(kp1, kp2, mt, int(ids[0]), int(ids[1])), np.uint8)
    np.savez_compressed(os.path.join(HERE, "golden_outcomes.npz"), **out)
    print("wrote", os.path.join(HERE, "golden_outcomes.npz"))


if __name__ == "__main__":
    main()
