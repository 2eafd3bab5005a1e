"""GPU parity of DeepFM's whole-tower kernel for small launch batches (csrc/k_small_s3.hip): one block per
16 or 32 samples (knob s3_small_rt 1 / 2: row tiles per block) runs the gather, the first order + FM, the three Linear + ReLU layers and the head
(HigherOrderEncoder.scala:34-59, Scatter.scala:17-36, SecondOrderEncoder.scala:19-34, DeepFM.scala:54-80).

Each case runs DeepFM with the kernel forced on (knob s3_small 2) and off (0: the per-layer split GEMM) on
the same inputs: the two agree far inside the north-star bar and both meet it (1e-5) against the fp64
oracle; the first order + FM is BITWISE the encoder's (checked with the output Linear zeroed: p =
sigmoid(y1 + y2 + b_out + beta) on both paths).  Batches: 1, 15, 17 (ragged 16-sample blocks), 1,000,
4,096 (the small batch of SURVEY.md §8d) and 16,384."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
SMALL_VS_ENGINE = 5e-6
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x5A11, 0x7AB1E, 0x3A75
FC = (400, 400, 400)
WO_OFF = 624 * 400 + 400 + 2 * (400 * 400 + 400)


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    rmx.set_tuning("s3_small", None)
    rmx.set_tuning("s3_small_rt", None)


def _run(ctx, B, V, mats, rt=0):
    rmx.set_tuning("s3_small_rt", rt)
    m = rmx.DeepFM(V, F, K, list(FC))
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = {}
    for knob in (0, 2):
        rmx.set_tuning("s3_small", knob)
        m.set_timing(True)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        stages, _ = m.get_timing()
        m.set_timing(False)
        assert ("tower_small" in stages) == (knob == 2), stages
        res[knob] = out.numpy().copy()
    return res


@pytest.mark.parametrize("rt", [1, 2])
@pytest.mark.parametrize("B", [1, 15, 17, 33, 1000, 4096, 8191, 16384])
def test_small_tower_matches_engine_and_oracle(ctx, B, rt):
    V = 50000
    mats = rmx.DeepFM(V, F, K, list(FC)).initMats(SEED_MATS)
    res = _run(ctx, B, V, mats, rt)
    d = float(np.abs(res[2] - res[0]).max())
    om = oc.make_model(oc.DEEPFM, F, K, fc=FC)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    errs = []
    for r0 in sorted({0, max(0, B - 256)}):
        n = min(256, B - r0)
        h = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, h)
        ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats, 1)
        errs.append(tuple(float(np.abs(res[k][r0:r0 + n] - ref).max()) for k in (2, 0)))
    print("B=%d RT=%d |small - engine| %.3g, vs fp64 (small, engine) %s" % (B, rt, d, errs))
    assert d <= SMALL_VS_ENGINE
    assert max(max(e) for e in errs) <= TOL


@pytest.mark.parametrize("rt", [1, 2])
@pytest.mark.parametrize("B", [17, 4096])
def test_small_tower_first_order_and_fm_bitwise(ctx, B, rt):
    V = 50000
    mats = np.array(rmx.DeepFM(V, F, K, list(FC)).initMats(SEED_MATS), np.float32)
    assert len(mats) == WO_OFF + 400 + 1
    mats[WO_OFF:WO_OFF + 400] = 0.0
    res = _run(ctx, B, V, mats, rt)
    assert np.array_equal(res[2], res[0])


@pytest.mark.parametrize("B", [4096, 8192])
def test_small_tower_auto_selection(ctx, B):
    """knob s3_small 1 (auto) takes the whole-tower kernel while one round of its 16- / 32-sample blocks
    covers the batch: at B = 4,096 and 8,192 the forward is the one launch."""
    rmx.set_tuning("s3_small", 1)
    V = 50000
    m = rmx.DeepFM(V, F, K, list(FC))
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.set_timing(True)
    m.forward_ids(table, B, ids, out)
    ctx.sync()
    stages, _ = m.get_timing()
    assert list(stages) == ["tower_small"], stages


@pytest.mark.parametrize("rt", [1, 2])
@pytest.mark.parametrize("pattern", [0x7FC00000, 0x7F800000, 0x3F800000])
def test_small_tower_ignores_lds_leftovers(ctx, rt, pattern):
    """The K padding of the 400-wide layers (columns 400 .. 415, not computed) is read as zeros: with every
    CU's LDS filled with a NaN, an infinity or 1.0 right before the launch, the output is bitwise the one
    after a clean fill (0).  (Before the fix a leftover NaN there made 0 x NaN = NaN, and ReLU turned it
    into a wrong 0: one row of some blocks was off by up to 5e-3.)"""
    B, V = 8192, 50000
    m = rmx.DeepFM(V, F, K, list(FC))
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    rmx.set_tuning("s3_small", 2)
    rmx.set_tuning("s3_small_rt", rt)
    res = []
    for pat in (0, pattern):
        rmx.debug_fill_lds(ctx, pat)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        res.append(out.numpy().copy())
    assert np.isfinite(res[1]).all()
    assert np.array_equal(res[0], res[1])



@pytest.mark.parametrize("rt", [1, 2])
@pytest.mark.parametrize("Fn", [1, 2, 7, 40])
def test_small_tower_field_counts(ctx, Fn, rt):
    """Field counts other than 39 through the whole-tower kernel (F = 1 / 2: one K step of layer 1; 7: odd;
    40: the maximum): within 5e-6 of the engine path and 1e-5 of the fp64 oracle."""
    V, B = 50000, 1000
    m = rmx.DeepFM(V, Fn, K, list(FC))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * Fn, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, Fn, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    rmx.set_tuning("s3_small_rt", rt)
    res = {}
    for knob in (0, 2):
        rmx.set_tuning("s3_small", knob)
        m.set_timing(True)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        stages, _ = m.get_timing()
        m.set_timing(False)
        assert ("tower_small" in stages) == (knob == 2), stages
        res[knob] = out.numpy().copy()
    assert float(np.abs(res[2] - res[0]).max()) <= SMALL_VS_ENGINE
    om = oc.make_model(oc.DEEPFM, Fn, K, fc=FC)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    n = 256
    h = oc.gen_ids(SEED_IDS, 0, n, Fn, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, h)
    ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), Fn), np.array([0.01], np.float32), w, e, mats, 1)
    assert float(np.abs(res[2][:n] - ref).max()) <= TOL
