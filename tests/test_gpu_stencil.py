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
from scanner_colmap_amd.codecs import table_rows
from scanner_colmap_amd.synthetic import Corridor

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


def test_execute_batch_rejects_conflicting_images():
    ids, kps, descs = table_rows(Corridor(3, 300, 3, seed=64).images())
    other = table_rows(Corridor(3, 200, 3, seed=65).images())
    with Context(0) as ctx:
        bad = [([ids[0], ids[1]], [kps[0], kps[1]], [descs[0], descs[1]]),
               ([ids[1], ids[2]], [other[1][1], kps[2]], [other[2][1], descs[2]])]
        with pytest.raises(ScmError):
            ctx.execute_batch(bad)
        # the context stays usable
        a, b = ctx.execute_stencil(ids, kps, descs)
        assert (a, b) == oracle.execute_stencil(ids, kps, descs)
