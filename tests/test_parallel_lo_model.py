"""Host model of a restructured replay (design for the next round):
the sequential LO-RANSAC replay of a window equals

  1. its record trials -- counts reaching the running maximum of the counts
     before them (the best count after trial s is at least every count up to s,
     so no other trial can be a candidate);
  2. each record's local-optimisation chain computed on its own (a chain starts
     from the candidate as the new best, and its steps compare only against
     counts and sums of its own models, so its outcome depends on the candidate
     alone) -- in parallel;
  3. a sequential resolution over the trials with those outcomes (accept /
     tie-break / dynamic trial bound / abort).

The model abstracts the geometry: a trial is (count, residual sum), a chain is a
deterministic function of its start; the reference semantics are those of
rs_replay_body (verify_kernels.hip) / LORANSAC::Estimate."""
import math

import numpy as np


def num_trials(best_n, n, confidence=0.999, mult=3.0, kmin=7):
    if best_n <= 0:
        return 2 ** 31 - 1
    denom = 1.0 - (best_n / n) ** kmin
    if denom <= 0.0:
        return 1
    if denom >= 1.0:
        return 2 ** 31 - 1
    return int(min(2 ** 31 - 1, math.ceil(math.log(1.0 - confidence) / math.log(denom) * mult)))


def lo_chain(start, n, seed):
    """Recursive LO from a model accepted as the best: up to 10 steps while the
    count grows, or stays equal with a smaller residual sum.  Returns the final
    (count, sum) and the number of steps -- a function of the start only."""
    rng = np.random.default_rng(seed)
    cnt, sm = start
    steps = 0
    for _ in range(10):
        steps += 1
        prev = cnt
        c2 = int(min(n, cnt + rng.integers(-3, 6)))
        s2 = float(sm * rng.uniform(0.9, 1.1) + (c2 - cnt))
        if c2 > cnt or (c2 == cnt and s2 < sm):  # lbetter: the LO model becomes the best
            cnt, sm = c2, s2
        if cnt <= prev:  # `if (s.best_n <= prev) break;`
            break
    return (cnt, sm), steps


def sequential(trials, n, min_trials):
    best = (0, float("inf"))
    dyn, chains = 2 ** 31 - 1, 0
    accepted = []
    for t, (c, sm, seed) in enumerate(trials):
        if c >= best[0]:
            better = c > best[0] or sm < best[1]
            if better:
                best, steps = lo_chain((c, sm), n, seed)
                chains += steps
                accepted.append(t)
                dyn = num_trials(best[0], n)
        if t >= dyn and t >= min_trials:
            return best, t, accepted, chains
    return best, len(trials) - 1, accepted, chains


def restructured(trials, n, min_trials):
    # 1. records: counts reaching the running maximum of the counts before them
    records, run = [], -1
    for t, (c, _, _) in enumerate(trials):
        if c >= run:
            records.append(t)
        run = max(run, c)
    # 2. every record's chain on its own (the parallel step)
    outcome = {t: lo_chain((trials[t][0], trials[t][1]), n, trials[t][2]) for t in records}
    # 3. sequential resolution
    best = (0, float("inf"))
    dyn = 2 ** 31 - 1
    accepted, rec = [], set(records)
    for t, (c, sm, _) in enumerate(trials):
        if c >= best[0]:
            assert t in rec, "a candidate that is not a record"
            if c > best[0] or sm < best[1]:
                best = outcome[t][0]
                accepted.append(t)
                dyn = num_trials(best[0], n)
        if t >= dyn and t >= min_trials:
            return best, t, accepted, len(records)
    return best, len(trials) - 1, accepted, len(records)


def test_records_and_independent_chains_reproduce_the_sequential_replay():
    rng = np.random.default_rng(3)
    total_records = total_trials = 0
    for case in range(400):
        n = int(rng.integers(50, 3000))
        T = int(rng.choice([64, 256, 2048, 5295]))
        ratio = rng.uniform(0.02, 0.9)
        counts = rng.binomial(n, ratio * rng.uniform(0, 1, T) ** 4)
        if case % 5 == 0:  # many equal counts: ties decided by the sums
            counts = np.minimum(counts, int(np.percentile(counts, 90)))
        sums = rng.uniform(1.0, 5.0, T) * np.maximum(counts, 1)
        seeds = rng.integers(0, 2 ** 31, T)
        trials = list(zip(counts.tolist(), sums.tolist(), seeds.tolist()))
        min_trials = int(rng.choice([0, 30]))
        b1, stop1, acc1, _ = sequential(trials, n, min_trials)
        b2, stop2, acc2, nrec = restructured(trials, n, min_trials)
        assert (b1, stop1, acc1) == (b2, stop2, acc2), case
        total_records += nrec
        total_trials += T
    # records are few (about ln T per window): the parallel step is small
    assert total_records < 0.05 * total_trials
