"""GPU parity of DeepFM's grid tower for small launch batches (csrc/k_grid_s3.hip): row groups x column groups
in one cooperative launch, layer outputs and partial logits handed between the blocks of a row group through
global memory inside the launch (sc1 payload, counter, one agent-scope acquire per hand-off).

Each layer's products, K order and epilogue are the fused tower's, so h1 / h2 are the same fp32 values; only the
logit's summation order differs (per column group, then the groups in order).  The grid tower is held to 5e-6
against the fused tower (k_fused_s3.hip, forced on) and to 1e-5 against the fp64 AND fp32 oracles on a strided
sample of rows, with W_out = 0 to bitwise equality (the first order + FM path), launch after launch (stale
counters or a missed hand-off would show as NaN outputs, the timeout path, or differing bits), for every
column-group width (knob s3_grid_nt: 1, 2, 4, 7 column tiles per block) whose grid fits the CUs
(model/encoder/HigherOrderEncoder.scala:34-59, SecondOrderEncoder.scala:19-34, DeepFM.scala:54-80)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
GRID_VS_FUSED = 5e-6
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x6A1D, 0x7AB1E, 0x3A75
FC = (400, 400, 400)
KNOBS = ("s3_grid", "s3_grid_nt", "s3_grid_min", "s3_fused", "s3_small", "s3_head", "s3_tail")


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    for k in KNOBS:
        rmx.set_tuning(k, None)


def _ncu():
    return 256  # MI355X; a smaller part only drops the cases whose grid does not fit (the launch refuses them)


def _setup(ctx, B, V, mats=None):
    m = rmx.DeepFM(V, F, K, list(FC))
    mats = m.initMats(SEED_MATS) if mats is None else mats
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    return m, mats, table, ids, out


def _fwd(ctx, m, table, B, ids, out, grid, nt=0):
    if grid:
        rmx.set_tuning("s3_grid", 2)
        rmx.set_tuning("s3_grid_nt", nt)
    else:
        rmx.set_tuning("s3_grid", 0)
        rmx.set_tuning("s3_small", 0)
        rmx.set_tuning("s3_fused", 2)
    m.set_timing(True)
    m.forward_ids(table, B, ids, out)
    ctx.sync()
    stages, _ = m.get_timing()
    m.set_timing(False)
    assert ("tower_grid" in stages) == grid, stages
    return out.numpy().copy()


def _fits(B, nt):
    R = (B + 127) // 128
    return R * ((25 + nt - 1) // nt) <= _ncu()


def _oracle_rows(V, mats, B, rows):
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = oc.make_model(oc.DEEPFM, F, K, fc=FC)
    ids = oc.gen_ids(SEED_IDS, 0, B, F, V).reshape(B, F)[rows].astype(np.int64).ravel()
    w, e = oc.gather(wt, et, 1, ids)
    n = rows.size
    idx = np.repeat(np.arange(n, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    return oc.forward(om, n, idx, bias, w, e, mats, 1), oc.forward(om, n, idx, bias, w, e, mats, 0)


@pytest.mark.parametrize("B", [1, 37, 128, 1000, 1024, 3001, 4096, 8192])
def test_grid_tower_matches_fused_and_oracle(ctx, B):
    V = 100_003
    m, mats, table, ids, out = _setup(ctx, B, V)
    ref = _fwd(ctx, m, table, B, ids, out, False)
    rows = np.union1d(np.arange(0, B, max(1, B // 256)), [B - 1])
    r64, r32 = _oracle_rows(V, mats, B, rows)
    ran = 0
    for nt in (1, 2, 4, 7):
        if not _fits(B, nt):
            continue
        got = _fwd(ctx, m, table, B, ids, out, True, nt)
        assert np.isfinite(got).all(), "nt=%d: NaN outputs (a hand-off timed out)" % nt
        d = float(np.abs(got - ref).max())
        e64, e32 = float(np.abs(got[rows] - r64).max()), float(np.abs(got[rows] - r32).max())
        print("B=%d nt=%d: |grid - fused| %.3g, vs fp64 %.3g, vs fp32 %.3g" % (B, nt, d, e64, e32))
        assert d <= GRID_VS_FUSED
        assert e64 <= TOL and e32 <= TOL
        ran += 1
    assert ran > 0


@pytest.mark.parametrize("B", [1024, 4096, 8192])
def test_grid_tower_first_order_and_fm_bitwise(ctx, B):
    """W_out = 0: p = sigmoid(y1 + y2 + b_out + beta) -- every partial logit is 0, so the grid tower's first order
    + FM (column group 0, from the layer-1 fragments) must give the fused tower's bits."""
    V = 50000
    m = rmx.DeepFM(V, F, K, list(FC))
    mats = np.array(m.initMats(SEED_MATS), np.float32)
    wo = len(mats) - 401
    mats[wo:wo + 400] = 0.0
    m, mats, table, ids, out = _setup(ctx, B, V, mats=mats)
    ref = _fwd(ctx, m, table, B, ids, out, False)
    got = _fwd(ctx, m, table, B, ids, out, True)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("B", [1024, 4096, 8192])
def test_grid_tower_repeated_launches_bitwise(ctx, B):
    """Launch after launch on the same workspace (the hand-off words are re-zeroed per call): the same bits
    every time, and on other batches in between."""
    V = 50000
    m, mats, table, ids, out = _setup(ctx, B, V)
    first = _fwd(ctx, m, table, B, ids, out, True)
    other = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS + 1, 0, B, F, V, other)
    rmx.set_tuning("s3_grid", 2)
    for i in range(20):
        m.forward_ids(table, B, other if i % 3 == 1 else ids, out)
        if i % 3 != 1:
            ctx.sync()
            assert np.array_equal(out.numpy(), first), i
    ctx.sync()


def test_grid_tower_is_the_default_at_small_batches(ctx):
    """B = 1,024 .. 8,192 run the grid tower by default (knob s3_grid 1); B = 512 the whole-tower kernel."""
    V = 50000
    for B, want in ((512, "tower_small"), (1024, "tower_grid"), (4096, "tower_grid"), (8192, "tower_grid")):
        m, mats, table, ids, out = _setup(ctx, B, V)
        m.set_timing(True)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        stages, _ = m.get_timing()
        assert list(stages) == [want], (B, stages)
