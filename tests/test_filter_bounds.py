"""The margins of the packed-fp32 inlier filters of the scoring kernels
(verify_kernels.hip) against the reference's fp64 residuals,
on host restatements of the filters' fp32 FMA sequences:
  * homography (h_filter_consts / h_filter_pair) vs the transfer error of
    HomographyMatrixEstimator::Residuals (tests/hfilter_check.c): random
    homographies of arbitrary scale, destinations within 1e-7 and 1e-3
    (relative) of the threshold and uniformly around it;
  * Sampson (f_filter_consts / f_filter_pair) vs ComputeSquaredSampsonError
    (tests/ffilter_check.c): random F = [t]x M of arbitrary scale, second
    points placed along the epipolar line's normal at the same distances.
Every point a filter decides must agree with the fp64 test; the undecided
share on uniform residuals must stay small (it only costs exact tests)."""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checkers(tmp_path_factory):
    d = tmp_path_factory.mktemp("filters")
    out = {}
    for kind in ("h", "f"):
        exe = str(d / f"{kind}fc")
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                        os.path.join(HERE, f"{kind}filter_check.c"), "-lm"], check=True)
        out[kind] = exe
    return out


@pytest.mark.parametrize("kind", ["h", "f"])
@pytest.mark.parametrize("maxr", ["16", "9", "2.5", "1"])
@pytest.mark.parametrize("uniform", [False, True])
def test_filter_margin_never_misdecides(checkers, kind, maxr, uniform):
    args = [checkers[kind], maxr] + (["u"] if uniform else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"undecided=(\d+) \(([\d.]+)%.*wrong=(\d+)", r.stdout)
    assert m and int(m.group(3)) == 0, r.stdout
    if uniform:
        assert float(m.group(2)) < 0.5, r.stdout
