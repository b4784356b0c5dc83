"""ComputeNumTrials exhaustively: the libm-free geom::num_trials that the GPU
replay kernel and the oracle evaluate (scanner_colmap_amd/csrc/geom_solvers.h)
against COLMAP's std::pow / std::log / std::ceil formula [upstream
optim/ransac.h ComputeNumTrials] on the host libm, for EVERY
(num_inliers <= num_samples <= 16384) at the four kMinNumSamples on this path
(7-pt F: 7, LO 8-pt: 8, H: 4, watermark translation: 1), at the default
confidence / multiplier and two other confidences and multipliers
(SequentialMatchingArgs confidence, dyn_num_trials_multiplier: colmap.proto;
sequential_matching.cc:154-159 builds the options).  One ulp across a ceil
boundary would change the trial count and with it the whole TwoViewGeometry.
Host restatement: tests/num_trials_check.cc (threads over num_samples)."""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("ntc") / "ntc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-o", exe,
                    os.path.join(HERE, "num_trials_check.cc")], check=True)
    return exe


@pytest.mark.parametrize("confidence,multiplier", [
    ("0.999", "3.0"),   # proto2 defaults (colmap.proto)
    ("0.99", "3.0"), ("0.9999", "3.0"),
    ("0.999", "1.0"), ("0.999", "2.5"),
])
@pytest.mark.parametrize("kmin", [1, 4, 7, 8])
def test_num_trials_exhaustive(checker, kmin, confidence, multiplier):
    r = subprocess.run([checker, str(kmin), confidence, multiplier, "16384"],
                       capture_output=True, text=True, timeout=300)
    m = re.search(r"evals=(\d+) mismatches=(\d+)", r.stdout)
    assert m, r.stdout + r.stderr
    assert int(m.group(1)) == 16384 * 16385 // 2 + 16384
    assert int(m.group(2)) == 0 and r.returncode == 0, r.stdout
