"""Diagnostics: spectra of the LO normal equations (A^T A) on synthetic pairs,
and how fast shifted inverse iteration converges on them.
usage: python probes/ata_spectra.py [kpts] [pairs]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402
from scanner_colmap_amd.synthetic import Corridor  # noqa: E402

oracle.LIB = os.path.join(ROOT, "probes", "build", "libata_dump.so")
L = oracle.lib()
L.ata_dump_count.restype = ctypes.c_long

kpts = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
npairs = int(sys.argv[2]) if len(sys.argv) > 2 else 6
c = Corridor(20, kpts, 20, seed=20253)
imgs = c.images(0, 20)
atas = []
for j in range(1, 1 + npairs):
    j2 = [1, 3, 6, 10, 15, 19][(j - 1) % 6]
    m = oracle.match_pair(imgs[0][2], imgs[j2][2])
    oracle.verify_pair(imgs[0][1], imgs[j2][1], m, imgs[0][0], imgs[j2][0])
    n = L.ata_dump_count()
    buf = np.zeros(45 * n)
    L.ata_dump_get(buf.ctypes.data_as(ctypes.c_void_p))
    atas.append(buf.reshape(n, 45))
    print(f"pair (0,{j2}): {len(m)} matches, {n} LO solves", flush=True)
atas = np.concatenate(atas)
np.save(os.path.join(ROOT, "probes", "build", "atas.npy"), atas)
iu = np.triu_indices(9)
ratios = []
for a45 in atas:
    A = np.zeros((9, 9))
    A[iu] = a45
    A = A + np.triu(A, 1).T
    w = np.linalg.eigvalsh(A)
    ratios.append(w[0] / w[1])
ratios = np.array(ratios)
print("lambda1/lambda2 quantiles:", np.quantile(ratios, [0, 0.5, 0.9, 0.99, 1.0]))
