"""GPU parity of the split GEMM's 2-wave tile for small launch batches (csrc/k_gemm_s3.hip, knob s3_narrow):
when the 8-wave, 128-row blocks would leave CUs idle, each tower layer runs 32-row x 208-column blocks
(model/encoder/HigherOrderEncoder.scala:34-59: Linear + ReLU per layer).

The tile changes only which block computes a row: every output element is the same split products in the
same K order, so the forward is BITWISE the 8-wave tile's, and both meet the north-star bar (1e-5) against
the fp64 oracle.  The whole-tower kernel and the row-owner head / tail are switched off so every layer runs
on the engine.  Batches: ragged (37, 1,000) and SURVEY.md §8d's small batch 4,096."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x4A77, 0x7AB1E, 0x3A75
FC = (400, 400, 400)
KNOBS = ("s3_small", "s3_head", "s3_tail", "s3_fused", "s3_narrow")


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    for k in KNOBS[:5]:
        rmx.set_tuning(k, 0)
    yield
    for k in KNOBS:
        rmx.set_tuning(k, None)


@pytest.mark.parametrize("kind", ["deepfm", "dnn"])
@pytest.mark.parametrize("B", [37, 1000, 4096])
def test_narrow_tile_bitwise_and_oracle(ctx, kind, B):
    V = 50000
    m = rmx.DeepFM(V, F, K, list(FC)) if kind == "deepfm" else rmx.DNN(V, F, K, list(FC))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = {}
    for knob in (0, 1):
        rmx.set_tuning("s3_narrow", knob)
        m.set_timing(True)
        m.forward_ids(table, B, ids_dev, out)
        ctx.sync()
        stages, _ = m.get_timing()
        m.set_timing(False)
        assert "tower_layer2" in stages and "tower_small" not in stages, stages
        res[knob] = out.numpy().copy()
    assert np.array_equal(res[0], res[1])
    om = oc.make_model(oc.DEEPFM if kind == "deepfm" else oc.DNN, F, K, fc=FC)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    n = min(B, 256)
    r0 = B - n
    ids = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats, 1)
    err = float(np.abs(res[1][r0:] - ref).max())
    print("%s B=%d narrow vs fp64 %.3g" % (kind, B, err))
    assert err <= TOL
