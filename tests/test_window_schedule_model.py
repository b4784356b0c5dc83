"""Host model of the small-batch window schedule's stream and event order
(run_windows / launch_verify, verify_kernels.hip): decoupled draws on their own
stream, replays (and the first windows' parallel LO chains) on the replay
stream, the early final passes on the final stream, window buffers in 2 or 3
parities, rotating active lists.

Every launch is listed with the per-kind buffers it reads and writes (window
buffers by parity, list contents and counts, PRNG states, sample-index
vectors, the speculative watermark fields).  The reference semantics are the
plain sequential order (begin; per window: draws, prune, solves, scores, LO
chains, replay; then the final passes); the check is that every pair of
conflicting accesses (one a write) is ordered the same way by the streams and
events -- i.e. every read sees the writer the sequential order gives it, and no
write overtakes a read.  Reads that the design makes order-free on purpose
(RansacState: the draws' trials_left and the scores' best, lagging values only
bound higher; the final passes' per-pair done flags; per-pair scratch of done
pairs) are outside the model and argued in DESIGN.md §3.3."""
import itertools

import pytest

KMAX = 64  # kMaxVerifyWindows


class Sched:
    def __init__(self):
        self.ops = []  # (stream, kind, name, reads, writes) in launch order
        self.seq = []  # kernel op ids in sequential-semantics order

    def kernel(self, stream, name, reads=(), writes=()):
        self.ops.append((stream, "k", name, frozenset(reads), frozenset(writes)))
        return len(self.ops) - 1

    def record(self, stream, ev):
        self.ops.append((stream, "rec", ev, None, None))

    def wait(self, stream, ev):
        self.ops.append((stream, "wait", ev, None, None))


def windows(max_f, max_h, smallf=4, second_f=80, maxw=128, tb=64):
    """Per window (f, h) flags, as run_windows' loop covers each kind."""
    out, cf, ch, r, wf, wh = [], 0, 0, 0, smallf, smallf
    while cf < max_f or ch < max_h:
        out.append((cf < max_f, ch < max_h))
        cf += wf * tb
        ch += wh * tb
        wf = min(second_f, maxw) if r == 0 else maxw
        wh = maxw
        r += 1
    return out


def build(max_f, max_h, np_, lo_windows=1, spec_wm=True, beside=True):
    """The launch sequence of launch_verify for a small batch with decoupled
    draws (dsplit), np_ parities."""
    S, R, D, FS = "stream", "rstream", "dstream", "fstream"
    s = Sched()
    kinds = ("F", "H")

    def par(buf, k, p):
        return f"{buf}{k}[{p}]"

    seq = []
    seq.append(s.kernel(S, "memset", writes={f"cnt{k}L{l}" for k in kinds for l in range(3)}))
    # begin: list 0, states, dtrial, the first parity's start states (pstate)
    seq.append(s.kernel(S, "begin", writes={f"list{k}L0" for k in kinds} | {f"cnt{k}L0" for k in kinds}
                         | {f"state{k}" for k in kinds} | {f"dtrial{k}" for k in kinds}
                         | {par("wstate", k, np_ - 1) for k in kinds} | {f"spec" }))
    s.record(S, "begin")
    wins = windows(max_f, max_h)
    last_h = max(r for r, (_, h) in enumerate(wins) if h)
    for r, (f, h) in enumerate(wins):
        p, pp = r % np_, (r - 1) % np_
        lin, lout = r % 3, (r + 1) % 3
        lw = (r - 1) % 3 if r > 0 else lin
        ks = [k for k, on in zip(kinds, (f, h)) if on]
        if r >= 2:
            s.wait(S, ("win", r - 2, 1))
        # draws on the draw stream
        if np_ == 3:
            if r >= 3:
                s.wait(D, ("win", r - 3, 1))
            if r >= 2:
                s.wait(D, ("draw", r - 2, 1))
            if r == 0:
                s.wait(D, "begin")
            ld = 0 if r < 2 else (r - 2) % 3
        else:
            if r >= 2:
                s.wait(D, ("win", r - 2, 1))
            s.wait(D, "begin" if r == 0 else ("draw", r - 1, 1))
            ld = lw
        rd = set()
        wr = set()
        for k in ks:
            rd |= {f"list{k}L{ld}", f"cnt{k}L{ld}", f"dtrial{k}", par("wstate", k, pp)}
            wr |= {par(b, k, p) for b in ("samp", "wsnap", "wstate", "wB", "cnts", "ucnt")}
            wr |= {f"dtrial{k}", f"sidx{k}"}
            rd |= {f"sidx{k}"}
        seq.append(s.kernel(D, f"draw{r}", rd, wr))
        s.record(D, ("draw", r, 0))
        s.wait(S, ("draw", r, 0))
        # prune: clears the list this window's replay fills (both kinds); the
        # certain-stop skip from window r > 0
        rd, wr = set(), {f"cnt{k}L{lout}" for k in kinds}
        if r > 0:
            for k in ks:
                rd |= {f"list{k}L{lw}", f"cnt{k}L{lw}", par("wB", k, p), par("cnts", k, pp),
                       par("wB", k, pp), par("wsnap", k, p)}
                wr |= {par("wB", k, p)}
        seq.append(s.kernel(S, f"prune{r}", rd, wr))
        s.record(S, ("draw", r, 1))
        for k in ks:
            seq.append(s.kernel(S, f"solve{k}{r}",
                                {f"list{k}L{lw}", f"cnt{k}L{lw}", par("wB", k, p), par("samp", k, p)},
                                {par("nmod", k, p), par("mods", k, p), par("fcon", k, p)}))
        for k in ks:
            seq.append(s.kernel(S, f"score{k}{r}",
                                {f"list{k}L{lw}", f"cnt{k}L{lw}", par("wB", k, p), par("nmod", k, p),
                                 par("mods", k, p), par("fcon", k, p), par("cnts", k, p),
                                 par("ucnt", k, p)},
                                {par("cnts", k, p), par("ucnt", k, p)}))
        s.record(S, ("win", r, 0))
        s.wait(R, ("win", r, 0))
        lo = r < lo_windows and np_ >= 2
        if lo:
            rd, wr = set(), set()
            for k in ks:
                rd |= {f"list{k}L{lin}", f"cnt{k}L{lin}", par("cnts", k, p), par("nmod", k, p),
                       par("mods", k, p), par("wB", k, p), f"state{k}"}
                wr |= {par("lo", k, p)}
            seq.append(s.kernel(R, f"lo{r}", rd, wr))
        rd, wr = set(), set()
        for k in ks:
            rd |= {f"list{k}L{lin}", f"cnt{k}L{lin}", par("cnts", k, p), par("nmod", k, p),
                   par("mods", k, p), par("wB", k, p), par("wsnap", k, p), par("wstate", k, p),
                   f"state{k}", f"cnt{k}L{lout}"}
            if lo:
                rd |= {par("lo", k, p)}
            wr |= {f"state{k}", f"list{k}L{lout}", f"cnt{k}L{lout}"}
        seq.append(s.kernel(R, f"replay{r}", rd, wr))
        s.record(R, ("win", r, 1))
    nw = len(wins)
    s.wait(S, ("win", nw - 1, 1))
    # final passes: the watermark RANSAC continues H's stream (stateH) with
    # its index vector in H's scratch (sidxH); phase 3 from H's last window's
    # draw state
    if spec_wm and last_h >= 1:
        s.wait(FS, ("draw", last_h, 0))
        s.wait(FS, ("win", last_h - 1, 1))
        # (its stateH reads are of pairs whose H was done before H's last
        # window: that window's replay writes only the states of the pairs it
        # runs -- per pair, outside the model)
        seq.append(s.kernel(FS, "final3", {par("wstate", "H", last_h % np_), "sidxH"},
                            {"sidxH", "spec"}))
    # phases 1 and 2 claim disjoint pairs (atomically, beside each other):
    # per-pair resources of the pairs each claims (1 / 2); phase 3 may touch
    # either
    both = {"sidxH1", "sidxH2", "spec1", "spec2"}
    if spec_wm and last_h >= 1:
        s.ops[seq[-1]] = s.ops[seq[-1]][:3] + (s.ops[seq[-1]][3] | both, s.ops[seq[-1]][4] | both)
    if beside:
        s.record(FS, "spec")
    s.wait(FS, ("win", last_h, 1))
    seq.append(s.kernel(FS, "final1", {"stateH", "sidxH1", "spec1"}, {"sidxH1", "spec1", "out1"}))
    s.record(FS, "fin")
    s.wait(S, "spec" if beside else "fin")
    seq.append(s.kernel(S, "final2", {"stateH", "sidxH2", "spec2"}, {"sidxH2", "spec2", "out2"}))
    if beside:
        s.wait(S, "fin")
    seq.append(s.kernel(S, "compact", {"out1", "out2"}, {"rows"}))
    s.seq = seq
    return s, wins


def happens_before(s):
    """Reachability over stream order + record -> wait edges (an op waits for
    the latest record of its event launched before it)."""
    n = len(s.ops)
    preds = [set() for _ in range(n)]
    last_on = {}
    last_rec = {}
    for i, (st, kind, name, _, _) in enumerate(s.ops):
        if st in last_on:
            preds[i].add(last_on[st])
        last_on[st] = i
        if kind == "rec":
            last_rec[name] = i
        elif kind == "wait":
            assert name in last_rec, f"wait on {name} before any record"
            preds[i].add(last_rec[name])
    anc = [set() for _ in range(n)]
    for i in range(n):
        for p in preds[i]:
            anc[i] |= anc[p] | {p}
    return anc


def conflicts(s):
    anc = happens_before(s)
    bad = []
    order = {op: i for i, op in enumerate(s.seq)}
    for a, b in itertools.combinations(s.seq, 2):
        if order[a] > order[b]:
            a, b = b, a
        _, _, na, ra, wa = s.ops[a]
        _, _, nb, rb, wb = s.ops[b]
        clash = (wa & (rb | wb)) | (ra & wb)
        if clash and a not in anc[b]:
            bad.append((na, nb, sorted(clash)))
    return bad


@pytest.mark.parametrize("np_", [2, 3])
@pytest.mark.parametrize("trials", [(10000, 10000), (10000, 5295), (300, 10000), (20000, 8000)])
@pytest.mark.parametrize("lo_windows", [1, 2])
def test_schedule_orders_every_conflict(np_, trials, lo_windows):
    s, wins = build(*trials, np_=np_, lo_windows=lo_windows)
    assert len(wins) >= 2
    assert conflicts(s) == []


def drop(s, pred):
    """The schedule without the ops pred selects (waits only)."""
    keep = [i for i, op in enumerate(s.ops) if not pred(op)]
    remap = {i: j for j, i in enumerate(keep)}
    s2 = Sched()
    s2.ops = [s.ops[i] for i in keep]
    s2.seq = [remap[i] for i in s.seq]
    return s2


def test_model_sees_a_missing_wait():
    """Teeth: three parities whose draws wait for no replay -- window r's
    draws then overwrite the buffers window r - 3's replay reads."""
    s, wins = build(20000, 20000, np_=3)
    assert len(wins) >= 4
    s2 = drop(s, lambda op: op[0] == "dstream" and op[1] == "wait" and op[2][0] == "win")
    bad = conflicts(s2)
    assert any(a.startswith("replay") and b.startswith("draw") for a, b, _ in bad)


def test_three_parities_need_the_prune_wait():
    """Window r's draws zero the counts window r - 2's prune reads as the
    previous window's (three parities): dropping that wait is reported."""
    s, wins = build(20000, 8000, np_=3)
    assert len(wins) >= 4
    s2 = drop(s, lambda op: op[0] == "dstream" and op[1] == "wait" and op[2] != "begin"
              and op[2][0] == "draw")
    bad = conflicts(s2)
    assert any(a.startswith("prune") and b.startswith("draw") for a, b, _ in bad)


def test_two_parities_need_the_prune_wait():
    """With two parities the draws of window r zero the counts window r - 1's
    prune reads as the previous window's: dropping that wait is reported."""
    s, _ = build(10000, 10000, np_=2)
    s2 = drop(s, lambda op: op[0] == "dstream" and op[1] == "wait" and op[2] != "begin"
              and op[2][0] == "draw")
    bad = conflicts(s2)
    assert any(a.startswith("prune") and b.startswith("draw") for a, b, _ in bad)


def test_speculative_watermark_needs_the_last_h_draws():
    """Phase 3 reads the state H's last window's draws leave: without its wait
    on those draws the model reports the race."""
    s, _ = build(10000, 10000, np_=3)
    s2 = drop(s, lambda op: op[0] == "fstream" and op[1] == "wait" and op[2][0] == "draw")
    bad = conflicts(s2)
    assert any(a.startswith("draw") and b == "final3" for a, b, _ in bad)


def test_last_final_pass_needs_the_speculative_pass():
    """The last final pass runs beside the early one but after phase 3 (both
    may run a pair's watermark RANSAC); and the batch's compaction after both."""
    s, _ = build(10000, 10000, np_=3)
    s2 = drop(s, lambda op: op[0] == "stream" and op[1] == "wait" and op[2] == "spec")
    assert any(a == "final3" and b == "final2" for a, b, _ in conflicts(s2))
    s3 = drop(s, lambda op: op[0] == "stream" and op[1] == "wait" and op[2] == "fin")
    assert any(a == "final1" and b == "compact" for a, b, _ in conflicts(s3))
