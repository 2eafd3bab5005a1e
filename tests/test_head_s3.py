"""GPU parity of DeepFM's row-owner tower layer 1 (csrc/k_head_s3.hip): the gathered Linear(624 -> 400) +
ReLU with the first order and the FM second order fused (model/encoder/HigherOrderEncoder.scala:34-59,
bnn/Scatter.scala:17-36, SecondOrderEncoder.scala:19-34), one persistent launch.

Each case runs DeepFM with the kernel forced on (knob s3_head 2) and off (0: the column-sliced split-GEMM
layer 1) on the same inputs.  The products and K order are the engine's, so the two agree far inside the
north-star bar; both are held to the fp64 oracle at 1e-5 on head / tail slices.  The first order + FM
(y1 + y2, encoder_k16_kernel<1>'s arithmetic) is checked BITWISE: with the output Linear's weights zeroed
the probability is sigmoid(y1 + y2 + b_out + beta) on both paths."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
HEAD_VS_ENGINE = 5e-6
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x4EAD, 0x7AB1E, 0x3A75
FC = (400, 400, 400)
WO_OFF = 624 * 400 + 400 + 2 * (400 * 400 + 400)  # the output Linear(400 -> 1) weights in mats


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    rmx.set_tuning("s3_small", 0)  # (small batches would run the whole-tower kernel, k_small_s3.hip)
    rmx.set_tuning("s3_fused", 0)  # (and batches that fill the GPU the fused tower, k_fused_s3.hip)
    yield
    for k in ("s3_head", "s3_tail", "table_lines", "s3_small", "half_blocks", "s3_fused"):
        rmx.set_tuning(k, None)


def _run(ctx, B, V, mats, heads=(0, 2), tails=(2,), lines=0):
    m = rmx.DeepFM(V, F, K, list(FC))
    m.setMats(mats)
    m.setBias(0.01)
    rmx.set_tuning("table_lines", lines)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = {}
    for h in heads:
        for t in tails:
            rmx.set_tuning("s3_head", h)
            rmx.set_tuning("s3_tail", t)
            m.forward_ids(table, B, ids, out)
            ctx.sync()
            res[(h, t)] = out.numpy().copy()
    return res


@pytest.mark.parametrize("B", [37, 1000, 19217, 65536])
def test_fp32_head_matches_engine_and_oracle(ctx, B):
    V = 50000
    mats = rmx.DeepFM(V, F, K, list(FC)).initMats(SEED_MATS)
    res = _run(ctx, B, V, mats, tails=(0, 2))
    d = max(float(np.abs(res[(2, t)] - res[(0, t)]).max()) for t in (0, 2))
    om = oc.make_model(oc.DEEPFM, F, K, fc=FC)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    errs = []
    for r0 in sorted({0, max(0, B - 256)}):
        n = min(256, B - r0)
        h = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, h)
        ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats, 1)
        errs.append(max(float(np.abs(res[k][r0:r0 + n] - ref).max()) for k in res))
    print("B=%d |head - engine| %.3g, vs fp64 %s" % (B, d, errs))
    assert d <= HEAD_VS_ENGINE
    assert max(errs) <= TOL


@pytest.mark.parametrize("B", [1000, 65536])
def test_fp32_head_first_order_and_fm_bitwise(ctx, B):
    V = 50000
    mats = rmx.DeepFM(V, F, K, list(FC)).initMats(SEED_MATS)
    assert len(mats) == WO_OFF + 400 + 1
    mats = np.array(mats, np.float32)
    mats[WO_OFF:WO_OFF + 400] = 0.0  # p = sigmoid(y1 + y2 + b_out + beta) on every path
    res = _run(ctx, B, V, mats, tails=(0, 2))
    assert np.array_equal(res[(2, 2)], res[(0, 2)])
    assert np.array_equal(res[(2, 0)], res[(0, 0)])


def test_fp32_head_reads_line_tables_bitwise(ctx):
    """With table_lines 1 (the [V][32] [emb | w | pad] line copy: row stride 32, weight stride 32) the
    kernel reads the same rows and weights: identical bits."""
    B, V = 40000, 50000
    mats = rmx.DeepFM(V, F, K, list(FC)).initMats(SEED_MATS)
    a = _run(ctx, B, V, mats, heads=(2,), lines=0)[(2, 2)]
    b = _run(ctx, B, V, mats, heads=(2,), lines=1)[(2, 2)]
    assert np.array_equal(a, b)


@pytest.mark.parametrize("B", [16384, 40000, 49152])
def test_fp32_head_half_blocks_bitwise(ctx, B):
    """Half row blocks (k_rowown.hpp QRows, knob half_blocks) in the head: bitwise the full-block launch."""
    V = 50000
    mats = rmx.DeepFM(V, F, K, list(FC)).initMats(SEED_MATS)
    res = {}
    try:
        for hb in (0, 1):  # (knob 1 forces half blocks on)
            rmx.set_tuning("half_blocks", hb)
            res[hb] = _run(ctx, B, V, mats, heads=(2,), tails=(2,))[(2, 2)]
    finally:
        rmx.set_tuning("half_blocks", None)
    assert np.array_equal(res[0], res[1])
