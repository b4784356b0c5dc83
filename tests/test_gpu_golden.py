"""The HIP path (through the C ABI) reproduces the committed golden vectors
byte for byte."""
import pytest

from golden_util import MATCH_CASES, VERIFY_CASES, blobs, load, table

pytestmark = pytest.mark.gpu
G = load()


@pytest.mark.parametrize("case", MATCH_CASES)
def test_gpu_golden_matches(gpu_ctx, case):
    got = gpu_ctx.match_pair(G[f"match_{case}_d1"], G[f"match_{case}_d2"])
    ref = G[f"match_{case}_matches"]
    assert got.shape == ref.shape and (got == ref).all()


@pytest.mark.parametrize("case", VERIFY_CASES)
def test_gpu_golden_verify(gpu_ctx, case):
    ids = G[f"verify_{case}_ids"]
    got = gpu_ctx.verify_pair(G[f"verify_{case}_kp1"], G[f"verify_{case}_kp2"],
                              G[f"verify_{case}_matches"], int(ids[0]), int(ids[1]))
    assert got == G[f"verify_{case}_tvg"].tobytes()


def test_gpu_golden_table_rows(gpu_ctx):
    ids, kps, descs = table(G)
    k = int(G["table_overlap"][0])
    gpu_ctx.table_load(ids, kps, descs)
    pa, pb = gpu_ctx.table_run(k, 0, len(ids))
    assert pa == blobs(G, "table_pairs")
    assert pb == blobs(G, "table_tvgs")
    packed = gpu_ctx.table_run_packed(k, 0, len(ids)).rows()
    assert packed == (pa, pb)
