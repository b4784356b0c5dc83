"""The Scanner drop-in path on the GPU: scm_execute_batch /
scm_execute_stencil (SequentialMatchingCPUKernel::execute replacement,
reference integration/op_cpp/sequential_matching.cc:103-185) over
consecutive stencils, with the HBM image cache carried across calls.  Every
output row must be byte-identical to the CPU oracle's table run over the
same rows (the stencil range(0, K) of feature_matching.py:43)."""
import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd import Context, ScmError
from scanner_colmap_amd.codecs import decode_tvg_list, table_rows
from scanner_colmap_amd.synthetic import Corridor, descriptors_for_matches, geometry_scene

pytestmark = pytest.mark.gpu


def _stencils(ids, kps, descs, K, r0, r1):
    n = len(ids)
    out = []
    for r in range(r0, r1):
        rows = [min(r + s, n - 1) for s in range(K)]
        out.append(([ids[i] for i in rows], [kps[i] for i in rows], [descs[i] for i in rows]))
    return out


@pytest.mark.parametrize("batch", [1, 3, 16])
def test_execute_batches_equal_table_oracle(batch):
    n, K = 16, 5
    ids, kps, descs = table_rows(Corridor(n, 900, K, seed=61).images())
    ref_ids, ref_tvgs = oracle.table_run(ids, kps, descs, K, 0, n)
    got_ids, got_tvgs = [], []
    with Context(0) as ctx:
        for r0 in range(0, n, batch):
            a, b = ctx.execute_batch(_stencils(ids, kps, descs, K, r0, min(n, r0 + batch)))
            got_ids += a
            got_tvgs += b
        reused, uploaded = ctx.stencil_stats()
    assert got_ids == ref_ids
    assert got_tvgs == ref_tvgs
    # every image crosses PCIe once; the rest come from the HBM cache
    assert uploaded == n
    calls = (n + batch - 1) // batch
    assert reused + uploaded == sum(len({min(r + s, n - 1) for r in range(r0, min(n, r0 + batch))
                                         for s in range(K)}) for r0 in range(0, n, batch))
    assert calls >= 1


def test_execute_batch_split_into_batches_equal_table_oracle():
    """Op calls of more than two small batches' pairs run as 2 or 3 pipelined
    batches (run_rows kOpCallBatches): 110 stencils of 19 pairs (2,090: two
    batches), then 70 (1,330: one), and a call of 170 (3,230: three) in a
    second context.  Every row equals the oracle's table run."""
    n, K = 180, 20
    ids, kps, descs = table_rows(Corridor(n, 160, K, seed=64).images())
    ref_ids, ref_tvgs = oracle.table_run(ids, kps, descs, K, 0, n)
    with Context(0) as ctx:
        got_ids, got_tvgs = [], []
        for r0, r1 in ((0, 110), (110, n)):
            a, b = ctx.execute_batch(_stencils(ids, kps, descs, K, r0, r1))
            got_ids += a
            got_tvgs += b
    assert got_ids == ref_ids
    assert got_tvgs == ref_tvgs
    with Context(0) as ctx:
        a, b = ctx.execute_batch(_stencils(ids, kps, descs, K, 0, 170))
    assert a == ref_ids[:170]
    assert b == ref_tvgs[:170]


def test_execute_stencil_repeated_ids_and_table_interleave():
    """Repeated ids inside a stencil (the :141-144 dedup), a table run between
    two execute calls (separate HBM tables), and an id whose features change
    (uploaded again, not served stale from the cache)."""
    n, K = 8, 4
    imgs = Corridor(n, 700, K, seed=62).images()
    ids, kps, descs = table_rows(imgs)
    with Context(0) as ctx:
        st = ([ids[0], ids[1], ids[1], ids[0]], [kps[0], kps[1], kps[1], kps[0]],
              [descs[0], descs[1], descs[1], descs[0]])
        a, b = ctx.execute_stencil(*st)
        ra, rb = oracle.execute_stencil(*st)
        assert (a, b) == (ra, rb)
        ctx.table_load(ids, kps, descs)
        ta, tb = ctx.table_run(K, 0, n)
        assert (ta, tb) == oracle.table_run(ids, kps, descs, K, 0, n)
        a, b = ctx.execute_stencil(ids[2:6], kps[2:6], descs[2:6])
        assert (a, b) == oracle.execute_stencil(ids[2:6], kps[2:6], descs[2:6])
        # image 3 again under the same id with fewer features: re-uploaded
        other = table_rows(Corridor(n, 500, K, seed=63).images())
        st2 = ([ids[2], ids[3]], [kps[2], other[1][3]], [descs[2], other[2][3]])
        a, b = ctx.execute_stencil(*st2)
        assert (a, b) == oracle.execute_stencil(*st2)


def _variant(kp, desc, seed, what):
    """Same id, same counts, other bytes: descriptors or keypoints changed."""
    rng = np.random.default_rng(seed)
    d = np.frombuffer(desc, np.uint8).copy()
    k = np.frombuffer(kp, np.uint8).copy()
    if what == "desc":
        body = d[16:].reshape(-1, 128)
        rows = rng.choice(len(body), size=max(1, len(body) // 3), replace=False)
        body[rows] = body[rng.permutation(rows)][:, rng.permutation(128)]
    else:
        xy = k[8:].view(np.float32).reshape(-1, 6)
        xy[:, :2] += rng.normal(0, 3.0, size=(len(xy), 2)).astype(np.float32)
    return k.tobytes(), d.tobytes()


@pytest.mark.parametrize("what", ["desc", "kp"])
def test_execute_batch_id_collisions_per_element(what):
    """PrepareImage ids are per-instance counters (prepare_image.cc:11-20), so
    one id can name two images.  The reference matches every stencil element
    with its own bytes (sequential_matching.cc:115-122) and dedups ids only
    inside one stencil (:139-146): within a batch and across consecutive calls
    (the HBM image cache) an id reused for other bytes -- equal or unequal
    feature counts -- must give exactly the oracle's per-stencil rows."""
    n, K = 6, 4
    ids, kps, descs = table_rows(Corridor(n, 700, K, seed=66).images())
    other = table_rows(Corridor(n, 520, K, seed=67).images())
    kv, dv = _variant(kps[2], descs[2], 68, what)      # id 2, equal counts, other bytes
    ku, du = other[1][3], other[2][3]                  # id 3, other counts
    stencils = [
        ([ids[0], ids[1], ids[2], ids[3]], [kps[0], kps[1], kps[2], kps[3]],
         [descs[0], descs[1], descs[2], descs[3]]),
        ([ids[1], ids[2], ids[3], ids[4]], [kps[1], kv, ku, kps[4]],
         [descs[1], dv, du, descs[4]]),
        # in-stencil duplicate id with other bytes: the first occurrence wins
        ([ids[2], ids[3], ids[3], ids[5]], [kps[2], ku, kps[3], kps[5]],
         [descs[2], du, descs[3], descs[5]]),
        ([ids[2], ids[0], ids[3], ids[4]], [kv, kps[0], kps[3], kps[4]],
         [dv, descs[0], descs[3], descs[4]]),
    ]
    ref = [oracle.execute_stencil(*st) for st in stencils]
    with Context(0) as ctx:
        # one batch holding every variant
        a, b = ctx.execute_batch(stencils)
        assert list(zip(a, b)) == ref
        # consecutive single-stencil calls: the cache must never serve stale bytes
        for st, r in zip(stencils + stencils[::-1], ref + ref[::-1]):
            assert ctx.execute_stencil(*st) == r
        # batches of two, then a cache reset, then the batch again
        for j in range(0, len(stencils), 2):
            a, b = ctx.execute_batch(stencils[j:j + 2])
            assert list(zip(a, b)) == ref[j:j + 2]
        ctx.stencil_cache_clear()
        a, b = ctx.execute_batch(stencils)
        assert list(zip(a, b)) == ref
    # the variant really changes the outputs of the rows that use it
    assert ref[1] != oracle.execute_stencil(*([x[:1] + [y] + x[2:] for x, y in
                                               zip(stencils[1], (ids[2], kps[2], descs[2]))]))


def _sampled(n):
    """Bytes of an n-byte buffer that the speculation fingerprint reads
    (scm_runtime.cpp sample_words): 64 8-byte words at i * stride, stride =
    ((n - 8) // 64) rounded down to a multiple of 8, and the last 8 bytes."""
    m = np.zeros(n, bool)
    if n < 520:
        m[:] = True
        return m
    stride = ((n - 8) // 64) & ~7
    for i in range(64):
        m[i * stride:i * stride + 8] = True
    m[n - 8:] = True
    return m


def _unsampled_variant(kp, desc, seed, what):
    """Same id and counts, other bytes, every sampled word unchanged."""
    rng = np.random.default_rng(seed)
    d = np.frombuffer(desc, np.uint8).copy()
    k = np.frombuffer(kp, np.uint8).copy()
    if what == "desc":
        body = d[16:]
        free = np.flatnonzero(~_sampled(len(body)))
        pick = free[rng.random(len(free)) < 0.5]
        body[pick] = body[rng.permutation(pick)]
    else:
        body = k[8:]
        m = _sampled(len(body)).reshape(-1, 24)[:, :8].any(axis=1)  # x, y of keypoint q
        xy = body.view(np.float32).reshape(-1, 6)
        rows = np.flatnonzero(~m)
        xy[rows, :2] += rng.normal(0, 3.0, size=(len(rows), 2)).astype(np.float32)
    assert (np.frombuffer(desc, np.uint8)[16:][_sampled(len(d) - 16)] == d[16:][_sampled(len(d) - 16)]).all()
    assert (np.frombuffer(kp, np.uint8)[8:][_sampled(len(k) - 8)] == k[8:][_sampled(len(k) - 8)]).all()
    return k.tobytes(), d.tobytes()


@pytest.mark.parametrize("what", ["desc", "kp"])
@pytest.mark.parametrize("sampled", [True, False])
def test_execute_stencil_buffers_rewritten_in_place(what, sampled):
    """Scanner hands consecutive calls the same element buffers, and a caller
    (or a recycling allocator) may put another image into a buffer between
    calls (same address, same size, other bytes).  A buffer seen in the
    previous call takes its content key speculatively while the GPU runs only
    if a sample of its words is unchanged; a rewrite that changes sampled
    words is hashed before the run (no rerun, one upload), and one that leaves
    them alone is caught by the full hash after the run: the run is discarded
    and the call runs again, keeping the image cache (again one upload).
    Either way the rows are exactly the oracle's for the new bytes."""
    n, K = 6, 4
    ids, kps, descs = table_rows(Corridor(n, 700, K, seed=71).images())
    kb = [bytearray(x) for x in kps]
    db = [bytearray(x) for x in descs]
    st = (ids[:K], kb[:K], db[:K])
    with Context(0) as ctx:
        assert ctx.execute_stencil(*st) == oracle.execute_stencil(ids[:K], kps[:K], descs[:K])
        # unchanged buffers: every image served from HBM, every key speculated
        assert ctx.execute_stencil(*st) == oracle.execute_stencil(ids[:K], kps[:K], descs[:K])
        r0, u0 = ctx.stencil_stats()
        assert u0 == K and r0 == K
        s0 = ctx.stencil_spec_stats()
        assert s0 == (K, 0, 0)
        kv, dv = (_variant if sampled else _unsampled_variant)(kps[2], descs[2], 72, what)
        kb[2][:] = kv
        db[2][:] = dv
        want = oracle.execute_stencil(ids[:K], [bytes(x) for x in kb[:K]],
                                      [bytes(x) for x in db[:K]])
        assert want != oracle.execute_stencil(ids[:K], kps[:K], descs[:K])
        assert ctx.execute_stencil(*st) == want
        r1, u1 = ctx.stencil_stats()
        s1 = ctx.stencil_spec_stats()
        # the changed image is the only upload; the cache survives a rerun
        assert u1 - u0 == 1 and r1 - r0 == K - 1
        if sampled:
            assert s1 == (s0[0] + K - 1, 1, 0)
        else:
            assert s1 == (s0[0] + K, 0, 1)
        assert ctx.execute_stencil(*st) == want
        assert ctx.stencil_stats() == (r1 + K, u1)


def test_execute_stencil_recycled_buffers():
    """A recycling allocator: the buffer of the image that leaves the stencil
    receives the image that enters it (same address, same size, other bytes)
    on every call.  The sampled words refuse the stale key before the run, so
    no call runs twice, each call uploads only its new image, and every row is
    the oracle's."""
    n, K = 12, 4
    ids, kps, descs = table_rows(Corridor(n, 600, K, seed=74).images())
    assert len({len(x) for x in kps}) == 1 and len({len(x) for x in descs}) == 1
    kb = [bytearray(kps[i]) for i in range(K)]
    db = [bytearray(descs[i]) for i in range(K)]
    slot = list(range(K))  # slot[s] = buffer holding stencil entry s
    with Context(0) as ctx:
        for r in range(n - K + 1):
            if r > 0:  # image r - 1 leaves, image r + K - 1 enters its buffer
                b = slot.pop(0)
                kb[b][:] = kps[r + K - 1]
                db[b][:] = descs[r + K - 1]
                slot.append(b)
            st = (ids[r:r + K], [kb[b] for b in slot], [db[b] for b in slot])
            assert ctx.execute_stencil(*st) == oracle.execute_stencil(ids[r:r + K], kps[r:r + K],
                                                                      descs[r:r + K]), r
        spec, refused, rerun = ctx.stencil_spec_stats()
        reused, uploaded = ctx.stencil_stats()
    assert rerun == 0
    assert refused == n - K  # one recycled buffer per call after the first
    assert uploaded == K + (n - K) and reused == (n - K) * (K - 1)


def test_watermark_index_vector_apart_from_speculative_f_draws(monkeypatch):
    """The early final pass of a small batch (configuration + watermark of the
    pairs whose F and H are done when H's last window is replayed) runs beside
    the later windows, whose F draws are speculative: window r + 1 draws for
    the pairs that were running one window back, so a pair whose F stopped in
    window r has its F index vector shuffled once more while its watermark
    RANSAC may be running.  The watermark's own index vector therefore lives in
    the pair's H area (verify_kernels.hip verify_final_kernel).

    No stream order can force the collision (draws that end before the pass
    starts are harmless: the watermark RANSAC starts from the identity), so
    the adversary is deterministic instead: SCM_DIAG_SCRIBBLE_F_SIDX=1 makes
    the final kernel itself zero the F area's index vector before every
    watermark draw, the worst those draws could do at any moment.  On this
    scene the watermark decision depends on the samples (the first inlier is
    in the 24 % set), so a watermark RANSAC that read the F area's vector
    would end at 24 % and drop WATERMARK.  Reference: Estimate, then
    DetectWatermark, sequential per pair (sequential_matching.cc:98-99, 159)."""
    kp1, kp2, mt = geometry_scene("two_translations", 600, 31, outlier_frac=0.1)
    d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), 31)
    extra = Corridor(3, 700, 3, seed=32).images()
    imgs = [(40, kp1, d1), (41, kp2, d2)] + [(42 + i, k, d) for i, (_, k, d) in enumerate(extra)]
    ids, kps, descs = table_rows(imgs)
    ref_st = oracle.execute_stencil(ids[:4], kps[:4], descs[:4])
    ref_tab = oracle.table_run(ids, kps, descs, 3, 0, len(imgs))
    assert decode_tvg_list(ref_st[1])[0].config == 7  # (40, 41): WATERMARK
    monkeypatch.setenv("SCM_DIAG_SCRIBBLE_F_SIDX", "1")
    with Context(0) as ctx:
        for _ in range(3):  # small batch: early pass beside the speculative windows
            assert ctx.execute_stencil(ids[:4], kps[:4], descs[:4]) == ref_st
        ctx.table_load(ids, kps, descs)  # table path (one final pass after all windows)
        assert ctx.table_run(3, 0, len(imgs)) == ref_tab


def test_speculative_watermark_decisions_equal_recomputed(monkeypatch):
    """A small batch takes a pair's watermark decision early (verify_final_kernel
    phase 3), beside H's last window: from H's final PRNG state when H is done,
    else from the state after H's last window's draws, which that window's
    replay leaves as H's final state unless it aborts H.  The decision is used
    only when it was taken from H's final state, or H did not abort; otherwise
    it is void and recomputed.  With SCM_DIAG_SPEC_CHECK=1 every decision the
    pass would use is recomputed from H's final state and compared
    (scm_table_timings entries 12-15).

    Scenes: two_translations (WATERMARK decided by the watermark RANSAC's
    samples, H running its whole trial cap: a draw-state decision that holds),
    plane_and_depth (F stops at once, H's dynamic bound ends it inside its
    last window: a void decision), translation (H done early: a final-state
    decision).  Every row equals the oracle's, no decision differs, and each
    kind of decision occurs.  Reference: Estimate, then DetectWatermark, per
    pair (sequential_matching.cc:98-99, 159)."""
    scenes = [("two_translations", 600, 31, 0.1), ("plane_and_depth", 600, 33, 0.1),
              ("translation", 500, 35, 0.4)]
    extra = Corridor(3, 700, 3, seed=36).images()
    monkeypatch.setenv("SCM_DIAG_SPEC_CHECK", "1")
    seen = {"spec_equal": 0, "spec_void": 0, "spec_differ": 0}
    with Context(0) as ctx:
        for i, (kind, m, seed, out) in enumerate(scenes):
            kp1, kp2, mt = geometry_scene(kind, m, seed, outlier_frac=out)
            d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), seed)
            base = 100 * (i + 1)
            imgs = [(base, kp1, d1), (base + 1, kp2, d2)] + [
                (base + 2 + j, k, d) for j, (_, k, d) in enumerate(extra)]
            ids, kps, descs = table_rows(imgs)
            ref = oracle.execute_stencil(ids[:4], kps[:4], descs[:4])
            for _ in range(2):
                assert ctx.execute_stencil(ids[:4], kps[:4], descs[:4]) == ref, kind
                t = ctx.table_timings()
                for k in seen:
                    seen[k] += t[k]
    assert seen["spec_differ"] == 0, seen
    assert seen["spec_equal"] > 0 and seen["spec_void"] > 0, seen
    monkeypatch.delenv("SCM_DIAG_SPEC_CHECK")
    with Context(0) as ctx:  # without the check the decisions are taken as they are
        kp1, kp2, mt = geometry_scene("two_translations", 600, 31, outlier_frac=0.1)
        d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), 31)
        imgs = [(100, kp1, d1), (101, kp2, d2)] + [(102 + j, k, d) for j, (_, k, d) in enumerate(extra)]
        ids, kps, descs = table_rows(imgs)
        assert ctx.execute_stencil(ids[:4], kps[:4], descs[:4]) == oracle.execute_stencil(
            ids[:4], kps[:4], descs[:4])
        t = ctx.table_timings()
        assert t["spec_taken"] > 0 and t["spec_equal"] == 0, t


@pytest.mark.parametrize("seed", [0, 1])
def test_mixed_scene_small_batches_equal_oracle(monkeypatch, seed):
    """Small batches mixing pairs whose F and H end in different windows:
    F early with H running its whole cap (general, two_translations), H
    ended by its dynamic bound inside a later window (plane_and_depth,
    planar with outliers), both early (translation), degenerate (random) --
    so the speculative schedule's paths (draws two windows ahead of the
    replays, the early and speculative final passes, the last pass beside the
    early one) meet in one batch.  Each Scanner batch holds several two-image
    stencils of different scenes; every row equals the oracle's, and with
    SCM_DIAG_SPEC_CHECK=1 no speculative watermark decision differs from its
    recomputation.  Reference: sequential_matching.cc:103-185."""
    kinds = [("general", 0.2), ("two_translations", 0.1), ("plane_and_depth", 0.1),
             ("planar", 0.55), ("translation", 0.4), ("random", 0.0), ("general", 0.6),
             ("plane_and_depth", 0.3)]
    rng = np.random.default_rng(700 + seed)
    stencils, refs = [], []
    for i, (kind, out) in enumerate(kinds):
        m = int(rng.integers(300, 900))
        s = 7000 + 100 * seed + i
        kp1, kp2, mt = geometry_scene(kind, m, s, outlier_frac=out)
        d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), s)
        ids, kps, descs = table_rows([(2 * s, kp1, d1), (2 * s + 1, kp2, d2)])
        stencils.append((ids, kps, descs))
        refs.append(oracle.execute_stencil(ids, kps, descs))
    monkeypatch.setenv("SCM_DIAG_SPEC_CHECK", "1")
    differ = 0
    with Context(0) as ctx:
        for B in (3, 5, len(stencils)):
            order = list(rng.permutation(len(stencils)))
            for b0 in range(0, len(order), B):
                sel = order[b0:b0 + B]
                got_ids, got_tvgs = ctx.execute_batch([stencils[j] for j in sel])
                for j, a, t in zip(sel, got_ids, got_tvgs):
                    assert (a, t) == refs[j], kinds[j]
                differ += ctx.table_timings()["spec_differ"]
    assert differ == 0


@pytest.mark.parametrize("batch", [1, 4])
def test_speculative_watermark_pass_before_last_replay(monkeypatch, batch):
    """The speculative watermark pass (verify_final_kernel phase 3) reads the
    pairs' F and H states while H's last window's replay may be setting them
    on another stream; nothing orders the two.  SCM_DIAG_HOLD_LAST_REPLAY=1
    forces one extreme: the pass is enqueued before that replay and the replay
    waits for it, so every pair whose F or H ends in that window is still
    running when the pass reads its state (the corridor stencil's middle
    pairs, whose F stops within its 256-5,376th trials, i.e. in H's last
    window; the watermark scenes, whose H runs to its cap there).  Rows equal
    the oracle's, with SCM_DIAG_SPEC_CHECK=1 no speculative decision differs
    from its recomputation (held, draw-state decisions occur, and void ones),
    and without the check decisions are taken and rows still equal.  The other extreme (the
    pass after the replay) is the normal form's fallback order, covered by the
    tests above.  Reference: Estimate, then DetectWatermark, per pair
    (sequential_matching.cc:98-99, 159)."""
    scenes = [("two_translations", 600, 31, 0.1), ("plane_and_depth", 600, 33, 0.1),
              ("translation", 500, 35, 0.4), ("general", 700, 37, 0.3)]
    stencils = []
    for i, (kind, m, seed, out) in enumerate(scenes):
        kp1, kp2, mt = geometry_scene(kind, m, seed, outlier_frac=out)
        d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), seed)
        stencils.append(table_rows([(500 + 2 * i, kp1, d1), (501 + 2 * i, kp2, d2)]))
    ids, kps, descs = table_rows(Corridor(40, 900, 20, seed=38).images(0, 20))
    stencils.append((ids, kps, descs))
    refs = [oracle.execute_stencil(*s) for s in stencils]
    monkeypatch.setenv("SCM_DIAG_HOLD_LAST_REPLAY", "1")
    monkeypatch.setenv("SCM_DIAG_SPEC_CHECK", "1")
    seen = {"spec_taken": 0, "spec_equal": 0, "spec_void": 0, "spec_differ": 0}
    with Context(0) as ctx:
        for rep in range(2):
            for b0 in range(0, len(stencils), batch):
                sel = list(range(b0, min(len(stencils), b0 + batch)))
                got_ids, got_tvgs = ctx.execute_batch([stencils[j] for j in sel])
                for j, a, t in zip(sel, got_ids, got_tvgs):
                    assert (a, t) == refs[j], (j, rep)
                tt = ctx.table_timings()
                for k in seen:
                    seen[k] += tt[k]
    # (with the check every decision the pass would use is recomputed and
    # counted as equal / different; void ones are recomputed anyway)
    assert seen["spec_differ"] == 0, seen
    assert seen["spec_equal"] > 0 and seen["spec_void"] > 0, seen
    monkeypatch.delenv("SCM_DIAG_SPEC_CHECK")
    taken = 0
    with Context(0) as ctx:  # the held order without the check: decisions taken as they are
        for j, st in enumerate(stencils):
            assert ctx.execute_stencil(*st) == refs[j], j
            taken += ctx.table_timings()["spec_taken"]
    assert taken > 0


@pytest.mark.parametrize("parallel_lo", ["1", "0"])
def test_parallel_lo_more_records_than_slots(monkeypatch, parallel_lo):
    """A small batch runs the LO chains of the first window's record models
    (counts reaching the running maximum) in parallel, one slot per record up
    to kLoSlots = 8 (rs_lo_chain2_kernel); records past the slots run inline in
    the replay, in the same window.  A noise-free planar scene with 40 %
    outliers gives every all-inlier 4-point sample the same H inlier count
    (ties reach the maximum: ~33 records in 256 trials), and min_num_trials =
    256 keeps the whole first window in play, so slot outcomes and inline
    chains mix in one window, with residual-sum ties between them.  Rows
    equal the oracle's with the parallel chains (SCM_PARALLEL_LO=1, the
    default) and with every chain inline (=0).  Reference: LORANSAC's loop
    (sequential_matching.cc:98-99 -> TwoViewGeometry::Estimate)."""
    from scanner_colmap_amd import default_options
    monkeypatch.setenv("SCM_PARALLEL_LO", parallel_lo)
    o_gpu, o_ref = default_options(), oracle.default_options()
    for o in (o_gpu, o_ref):
        o.min_num_trials = 256
    stencils = []
    for i, (kind, m, seed, out) in enumerate([("planar", 800, 41, 0.4), ("planar", 600, 42, 0.3),
                                             ("general", 700, 43, 0.3)]):
        kp1, kp2, mt = geometry_scene(kind, m, seed, outlier_frac=out, noise_px=0.0)
        d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), seed)
        stencils.append(table_rows([(600 + 2 * i, kp1, d1), (601 + 2 * i, kp2, d2)]))
    refs = [oracle.execute_stencil(*s, opts=o_ref) for s in stencils]
    assert decode_tvg_list(refs[0][1])[0].config == 6  # PLANAR_OR_PANORAMIC
    with Context(0, o_gpu) as ctx:
        for s, ref in zip(stencils, refs):
            assert ctx.execute_stencil(*s) == ref
        got_ids, got_tvgs = ctx.execute_batch(stencils)
        assert list(zip(got_ids, got_tvgs)) == refs


def test_concurrent_contexts_on_threads():
    """Scanner runs one kernel object per pipeline instance, and instances
    share a worker process (the per-instance constructor,
    sequential_matching.cc:30-33; registration :202-205; SURVEY.md §8b
    Threading).  Two threads, each with its own Context on device 0, run
    interleaved batch-1 stencil streams of two different scenes at the same
    time (ctypes releases the GIL in every library call); every row equals
    the oracle's, and the second pass over the same streams (HBM image
    caches warm, speculated content keys) too."""
    import threading

    K = 6
    srcs = [table_rows(Corridor(14, 700, K, seed=900 + s).images()) for s in range(2)]
    streams = []
    for ids, kps, descs in srcs:
        calls = [(ids[r:r + K], kps[r:r + K], descs[r:r + K]) for r in range(len(ids) - K + 1)]
        streams.append((calls, [oracle.execute_stencil(*c) for c in calls]))
    errors = []
    start = threading.Barrier(2)

    def run(i):
        calls, refs = streams[i]
        try:
            with Context(0) as ctx:
                start.wait()
                for rep in range(2):
                    for j, (c, ref) in enumerate(zip(calls, refs)):
                        got = ctx.execute_stencil(*c)
                        if got != ref:
                            errors.append((i, rep, j))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((i, repr(e)))

    threads = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads)
    assert errors == []
