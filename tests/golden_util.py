"""Loader of the committed golden vectors (tests/golden/golden_v1.npz, made
by tests/golden/make_golden.py).  Plain arrays only: allow_pickle=False."""
import os

import numpy as np

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_v1.npz")
MATCH_CASES = ("random_ragged", "tie_stress", "corridor")
VERIFY_CASES = ("01", "03", "23")


def load():
    with np.load(PATH, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def blobs(g, name):
    offs, data = g[f"{name}_offs"], g[f"{name}_data"]
    return [data[offs[i]:offs[i + 1]].tobytes() for i in range(len(offs) - 1)]


def table(g):
    from scanner_colmap_amd.codecs import encode_image_id
    ids = [encode_image_id(int(i)) for i in g["table_ids"]]
    return ids, blobs(g, "table_kps"), blobs(g, "table_descs")


OUTCOMES_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             "golden_outcomes.npz")
# name -> (configuration before the post-filter, configuration in the output row)
OUTCOMES = {"general": (3, 3), "planar": (6, 6), "watermark": (7, 7), "degenerate": (1, 0),
            "few_inliers": (3, 3), "planar_big": (6, 6), "watermark_big": (7, 7)}


def load_outcomes():
    with np.load(OUTCOMES_PATH, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
