"""Host model of the windowed LO-RANSAC's trial bookkeeping (verify_kernels.hip
run_windows / rs_draw_body / rs_replay_body): windows drawn only up to
trials_left -- the last trial the sequential loop can still reach,
max(dyn_max, min_num_trials), with the dyn_max of the last replay (one window
old on the speculative small-batch schedule) -- process exactly the trials the
sequential loop processes, never leave a running pair without trials, and
stop at the same trial.  The window sizes are the product's: table path
1, 2, 4, ... 32 rounds; small batches 4 then 128 rounds (64 trials a round)."""
import math

import numpy as np
import pytest


def num_trials(best_n, n, confidence=0.999, mult=3.0, kmin=4):
    # ComputeNumTrials (COLMAP optim/ransac.h): monotone non-increasing in best_n
    if best_n <= 0:
        return 2 ** 31 - 1
    ratio = best_n / n
    denom = 1.0 - ratio ** kmin
    if denom <= 0.0:
        return 1
    return int(min(2 ** 31 - 1, math.ceil(math.log(1.0 - confidence) / math.log(denom) * mult)))


def sequential(counts, n, max_trials, min_trials):
    """Trials processed and the stop trial of the reference's loop."""
    best, dyn = 0, max_trials
    for tt in range(max_trials):
        if counts[tt] > best:
            best = counts[tt]
            dyn = num_trials(best, n)
        if tt >= dyn and tt >= min_trials:
            return tt
    return max_trials - 1


def trials_left(max_trials, dyn_max, min_trials, drawn):
    cap = max_trials
    last = max(dyn_max, min_trials)
    if last < cap:
        cap = last + 1
    return cap - drawn


def windowed(counts, n, max_trials, min_trials, sizes, lag):
    """The windows' draws with the cap; lag = 1: the dyn_max the draws see is one
    window old (speculative schedule).  Returns the stop trial and trials drawn."""
    best, dyn, drawn, tt = 0, max_trials, 0, 0
    dyn_seen = [max_trials]  # dyn_max after each window's replay
    for r in range(10 ** 6):
        W = sizes[min(r, len(sizes) - 1)] * 64
        known = dyn_seen[max(0, len(dyn_seen) - 1 - lag)]
        B = max(0, min(W, trials_left(max_trials, known, min_trials, drawn)))
        assert B > 0, "a running pair got a window with no trials"
        lo, drawn = drawn, drawn + B
        for tt in range(lo, drawn):  # the replay of this window, in order
            if counts[tt] > best:
                best = counts[tt]
                dyn = num_trials(best, n)
            if tt >= dyn and tt >= min_trials:
                return tt, drawn
        if drawn >= max_trials:
            return max_trials - 1, drawn
        dyn_seen.append(dyn)
    raise AssertionError("no stop")


@pytest.mark.parametrize("sizes", [[1, 2, 4, 8, 16, 32], [4, 128]])
@pytest.mark.parametrize("lag", [0, 1])
def test_capped_windows_stop_where_the_sequential_loop_stops(sizes, lag):
    rng = np.random.default_rng(5 + lag + len(sizes))
    for case in range(300):
        n = int(rng.integers(20, 4000))
        max_trials = int(rng.choice([5295, 10000, 300]))
        min_trials = int(rng.choice([0, 30, 100]))
        ratio = rng.uniform(0.01, 0.95)
        # per-trial counts: mostly low, occasional good models
        counts = rng.binomial(n, ratio * rng.uniform(0.0, 1.0, max_trials) ** 3)
        stop = sequential(counts, n, max_trials, min_trials)
        got, drawn = windowed(counts, n, max_trials, min_trials, sizes, lag)
        assert got == stop, (case, got, stop)
        assert drawn >= stop + 1
        if lag == 0 and drawn > stop + 1:
            # past the stop only within the window the stop fell in
            assert drawn - (stop + 1) < max(sizes) * 64
