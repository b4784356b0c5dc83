"""The margin of the packed-fp32 homography inlier filter (verify_kernels.hip
h_filter_consts / h_filter_pair) against the reference's fp64
transfer residual (HomographyMatrixEstimator::Residuals), on a host
restatement of the filter's fp32 FMA sequence (tests/hfilter_check.c):
random homographies of arbitrary scale, destinations placed within 1e-7 and
1e-3 (relative) of the threshold and uniformly around it.  Every point the
filter decides must agree with the fp64 test; the undecided share on uniform
radii must stay small (it only costs exact tests)."""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hfc(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("hfc") / "hfc")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(HERE, "hfilter_check.c"), "-lm"], check=True)
    return exe


@pytest.mark.parametrize("maxr", ["16", "9", "2.5", "1"])
@pytest.mark.parametrize("uniform", [False, True])
def test_h_filter_margin_never_misdecides(hfc, maxr, uniform):
    args = [hfc, maxr] + (["u"] if uniform else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"undecided=(\d+) \(([\d.]+)%.*wrong=(\d+)", r.stdout)
    assert m and int(m.group(3)) == 0, r.stdout
    if uniform:
        assert float(m.group(2)) < 0.5, r.stdout
