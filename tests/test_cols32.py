"""GPU parity of DeepFM's column-split small-batch path (round 6, knob s3_cols = the largest B that takes it):
the encoder writes the gathered rows x with the first order + FM, then each tower layer runs on 128-row x
32-column split-GEMM blocks (k_gemm_s3.hip p.cols32) and the output layer's 13 partial logits are summed in
order by out_finish_kernel with the head (HigherOrderEncoder.scala:34-59, Scatter.scala:17-36,
SecondOrderEncoder.scala:19-34, DeepFM.scala:54-80).

Each case runs the same inputs through the path and through the whole-tower kernel it replaces (s3_cols 0):
both meet 1e-5 against the fp64 oracle and agree within 5e-6 (the products and K order per output are the
engine's; only the output dot's summation order differs); two launches are bitwise equal, also with every
CU's LDS poisoned with NaN first (the 32-column tile reads only LDS it wrote)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0xC0132, 0x7AB1E, 0x3A75
FC = (400, 400, 400)


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    rmx.set_tuning("s3_cols", None)
    rmx.set_tuning("s3_cols_wm", None)


def _forward(ctx, B, V, knob, poison=False, wm=4):
    rmx.set_tuning("s3_cols_wm", wm)
    rmx.set_tuning("s3_cols", knob)  # (before the model's workspace exists: it sizes x for the path)
    m = rmx.DeepFM(V, F, K, list(FC))
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = []
    for rep in range(2):
        if poison and rep == 1:
            rmx.debug_fill_lds(ctx, 0x7FC00000)
        m.set_timing(True)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        stages, _ = m.get_timing()
        m.set_timing(False)
        res.append(out.numpy().copy())
    return res, stages, ids.numpy()


@pytest.mark.parametrize("B", [1, 37, 128, 1000, 1024, 4096, 8192])
def test_cols32_matches_small_kernel_and_oracle(ctx, B):
    V = 50000
    (a, a2), st, h_ids = _forward(ctx, B, V, 1 << 20, poison=True)
    assert "encoder_fm_x" in st and "tower_small" not in st, st
    assert np.array_equal(a, a2)
    for wm in (8, 2):  # the other block heights: the same products in the same order per output
        (w, _), _, _ = _forward(ctx, B, V, 1 << 20, wm=wm)
        assert np.array_equal(a, w), wm
    (b, _), st0, _ = _forward(ctx, B, V, 0)
    assert "encoder_fm_x" not in st0
    assert float(np.abs(a - b).max()) <= 5e-6
    om = oc.make_model(oc.DEEPFM, F, K, fc=FC)
    mats = rmx.DeepFM(V, F, K, list(FC)).initMats(SEED_MATS)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    n = min(B, 512)
    ids = h_ids[:n * F].astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats, 1)
    assert float(np.abs(a[:n] - ref).max()) <= TOL
