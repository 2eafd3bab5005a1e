"""GPU parity of the CIN's smaller split-GEMM tiles for small batches (csrc/k_gemm_s3.hip launch_cin_s3, knob
cin_narrow): when 256-row blocks would leave CUs idle (B * k < 256 CUs x 256 rows), each CIN layer runs
128-, 64- or 32-row blocks (xdeepfm/CINEncoder.scala:135-176).  The tile changes only which block computes
a row, not the products or their K order, so the forward is BITWISE the 256-row tile's; both meet the
north-star bar (1e-5) against the fp64 oracle.  Batches: 1, 37 (ragged), 512 / 1,000 / 2,048 (32-, 64-,
128-row blocks)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0xC17A, 0x7AB1E, 0x3A75
CIN, FC = (200, 200, 200), (400, 400, 400)


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    rmx.set_tuning("cin_narrow", None)


@pytest.mark.parametrize("B", [1, 37, 512, 1000, 2048])
def test_cin_narrow_tiles_bitwise_and_oracle(ctx, B):
    V = 20_011
    m = rmx.XDeepFM(V, F, K, list(FC), list(CIN))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = {}
    for knob in (0, 1):
        rmx.set_tuning("cin_narrow", knob)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        res[knob] = out.numpy().copy()
    assert np.array_equal(res[0], res[1])
    om = oc.make_model(oc.XDEEPFM, F, K, fc=FC, cin=CIN)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    n = min(B, 48)
    r0 = B - n
    h = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, h)
    ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats, 1, 16)
    err = float(np.abs(res[1][r0:] - ref).max())
    print("xDeepFM B=%d narrow CIN vs fp64 %.3g" % (B, err))
    assert err <= TOL
