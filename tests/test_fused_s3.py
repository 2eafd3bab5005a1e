"""GPU parity of DeepFM's fused fp32 tower (csrc/k_fused_s3.hip): layer 1 over the gathered rows (+ first order
and FM), layers 2 and 3, the output dot and the head in ONE persistent row-owner launch, h1 and h2 kept in
the waves' registers (model/encoder/HigherOrderEncoder.scala:34-59, SecondOrderEncoder.scala:19-34,
bnn/Scatter.scala:17-36, DeepFM.scala:54-80).

Every layer's products, K order and epilogue arithmetic are those of the head + tail pair (k_head_s3.hip,
k_tail_s3.hip), which stores h1 to HBM between them: the fused kernel must give the SAME BITS (knob s3_fused
2 vs 0 with the head and tail forced on), and both meet the north-star bar against the fp64 oracle.
Batches: ragged (37, 1,000), fewer row blocks than CUs (19,217), one full + a half round (40,000, 49,152),
the bench batch (65,536: two row blocks per CU), one row past it and two rounds (131,072); the line table
(table_lines 1), half blocks on / off, and every row block of the bench batch on a strided sample."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0xF05E, 0x7AB1E, 0x3A75
FC = (400, 400, 400)


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    rmx.set_tuning("s3_small", 0)  # (small batches would run the whole-tower kernel, k_small_s3.hip)
    yield
    for k in ("s3_fused", "s3_head", "s3_tail", "s3_small", "table_lines", "half_blocks"):
        rmx.set_tuning(k, None)


def _setup(ctx, B, V, lines=0, mats=None):
    m = rmx.DeepFM(V, F, K, list(FC))
    mats = m.initMats(SEED_MATS) if mats is None else mats
    m.setMats(mats)
    m.setBias(0.01)
    rmx.set_tuning("table_lines", lines)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    return m, mats, table, ids, out


def _fwd(ctx, m, table, B, ids, out, fused):
    rmx.set_tuning("s3_fused", 2 if fused else 0)
    rmx.set_tuning("s3_head", 2)
    rmx.set_tuning("s3_tail", 2)
    m.set_timing(True)
    m.forward_ids(table, B, ids, out)
    ctx.sync()
    stages, _ = m.get_timing()
    m.set_timing(False)
    assert ("tower_fused" in stages) == fused, stages
    return out.numpy().copy()


def _oracle_rows(V, mats, rows):
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = oc.make_model(oc.DEEPFM, F, K, fc=FC)
    B = int(rows.max()) + 1
    ids = oc.gen_ids(SEED_IDS, 0, B, F, V).reshape(B, F)[rows].astype(np.int64).ravel()
    w, e = oc.gather(wt, et, 1, ids)
    n = rows.size
    idx = np.repeat(np.arange(n, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    return oc.forward(om, n, idx, bias, w, e, mats, 1), oc.forward(om, n, idx, bias, w, e, mats, 0)


@pytest.mark.parametrize("B", [37, 1000, 19217, 40000, 49152, 65536, 65537, 131072])
def test_fused_tower_bitwise_head_tail_and_oracle(ctx, B):
    V = 100_003
    m, mats, table, ids, out = _setup(ctx, B, V)
    got = _fwd(ctx, m, table, B, ids, out, True)
    ref = _fwd(ctx, m, table, B, ids, out, False)
    assert np.isfinite(got).all()
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, "%d rows differ from head + tail (first %s, max |d| %.3g)" % (
        bad.size, bad[:8].tolist(), float(np.abs(got - ref).max()))
    rows = np.union1d(np.arange(0, B, max(1, B // 512)), [B - 1])
    r64, r32 = _oracle_rows(V, mats, rows)
    e64, e32 = float(np.abs(got[rows] - r64).max()), float(np.abs(got[rows] - r32).max())
    print("B=%d: fused == head + tail; %d rows vs fp64 %.3g, vs fp32 %.3g" % (B, rows.size, e64, e32))
    assert e64 <= TOL and e32 <= TOL
    # deterministic
    assert np.array_equal(_fwd(ctx, m, table, B, ids, out, True), got)


def test_fused_tower_reads_line_tables_bitwise(ctx):
    """table_lines 1 (the [V][32] [emb | w | pad] line copy: row and weight strides 32): the same bits."""
    B, V = 40000, 50000
    m, mats, table, ids, out = _setup(ctx, B, V, lines=0)
    a = _fwd(ctx, m, table, B, ids, out, True)
    m, mats, table, ids, out = _setup(ctx, B, V, lines=1, mats=mats)
    b = _fwd(ctx, m, table, B, ids, out, True)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("B", [16384, 40000, 49152])
def test_fused_tower_half_blocks_bitwise(ctx, B):
    """Half row blocks (k_rowown.hpp QRows: waves 4 .. 7 keep the ring and the barriers without MFMAs, across all
    three layers) compute every row with the same instructions: bitwise the full-block launch."""
    V = 50000
    m, mats, table, ids, out = _setup(ctx, B, V)
    res = {}
    for hb in (0, 1):
        rmx.set_tuning("half_blocks", hb)
        res[hb] = _fwd(ctx, m, table, B, ids, out, True)
    assert np.array_equal(res[0], res[1])


def test_fused_tower_first_order_and_fm_bitwise(ctx):
    """W_out = 0: p = sigmoid(y1 + y2 + b_out + beta), so the fused kernel's first order + FM (computed from
    the layer-1 fragments) must equal the head + tail path's bit for bit, and the unfused encoder's."""
    B, V = 65536, 50000
    m = rmx.DeepFM(V, F, K, list(FC))
    mats = np.array(m.initMats(SEED_MATS), np.float32)
    wo = len(mats) - 401
    mats[wo:wo + 400] = 0.0
    m, mats, table, ids, out = _setup(ctx, B, V, mats=mats)
    a = _fwd(ctx, m, table, B, ids, out, True)
    b = _fwd(ctx, m, table, B, ids, out, False)
    assert np.array_equal(a, b)


def test_fused_tower_is_the_default_at_the_bench_batch(ctx):
    """configs[1] (DeepFM, B = 65,536) runs the fused tower by default (knob s3_fused 1: row blocks >= CUs)."""
    B, V = 65536, 100000
    m, mats, table, ids, out = _setup(ctx, B, V)
    for k in ("s3_fused", "s3_head", "s3_tail", "s3_small"):
        rmx.set_tuning(k, None)
    m.set_timing(True)
    m.forward_ids(table, B, ids, out)
    ctx.sync()
    stages, _ = m.get_timing()
    assert list(stages) == ["tower_fused"], stages


@pytest.mark.parametrize("B,want", [(8192, ["tower_small"]), (9216, ["tower_fused"]), (16384, ["tower_fused"]),
                                    (32768, ["tower_fused"]), (49152, ["tower_fused"])])
def test_fused_tower_default_batch_rule(ctx, B, want):
    """knob s3_fused 1 (default) takes the fused tower at every batch the small-batch kernels leave to it (they
    take B <= 8,192 on 256 CUs): since round 6 it beats head + tail from B = 9,216 up (107 vs 90 M there)."""
    V = 50000
    m, mats, table, ids, out = _setup(ctx, B, V)
    for k in ("s3_fused", "s3_head", "s3_tail", "s3_small"):
        rmx.set_tuning(k, None)
    m.set_timing(True)
    m.forward_ids(table, B, ids, out)
    ctx.sync()
    stages, _ = m.get_timing()
    assert list(stages) == want, stages


@pytest.mark.parametrize("B", [40000, 65536])
@pytest.mark.parametrize("knob", ["fused_prio", "fused_dma_split"])
def test_fused_tower_schedule_knobs_bitwise(ctx, B, knob):
    """The schedule knobs move work, not arithmetic -- fused_prio (the second half of the waves at priority 1),
    fused_dma_split (0: every wave's DMAs at the early tiles, 1: the second half's late, 2: every wave's late):
    the same bits either way."""
    V = 50000
    m, mats, table, ids, out = _setup(ctx, B, V)
    vals = (0, 1, 2) if knob == "fused_dma_split" else (0, 1)
    res = {}
    try:
        for v in vals:
            rmx.set_tuning(knob, v)
            res[v] = _fwd(ctx, m, table, B, ids, out, True)
    finally:
        rmx.set_tuning(knob, None)
    for v in vals[1:]:
        assert np.array_equal(res[vals[0]], res[v]), v


@pytest.mark.parametrize("Fn", [1, 2, 7, 40])
def test_fused_tower_field_counts(ctx, Fn):
    """Field counts other than the bench's 39 (F = 1 / 2: one K step; 7: odd, a half-empty last step; 40: the
    maximum, 20 full steps): the fused tower gives head + tail's bits and meets the fp64 oracle."""
    B, V = 40000, 50000
    m = rmx.DeepFM(V, Fn, K, list(FC))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * Fn, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, Fn, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    got = _fwd(ctx, m, table, B, ids, out, True)
    ref = _fwd(ctx, m, table, B, ids, out, False)
    assert np.isfinite(got).all()
    assert np.array_equal(got, ref)
    rows = np.union1d(np.arange(0, B, 997), [B - 1])
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = oc.make_model(oc.DEEPFM, Fn, K, fc=FC)
    h = oc.gen_ids(SEED_IDS, 0, B, Fn, V).reshape(B, Fn)[rows].astype(np.int64).ravel()
    w, e = oc.gather(wt, et, 1, h)
    n = rows.size
    r64 = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), Fn), np.array([0.01], np.float32), w, e, mats, 1)
    assert float(np.abs(got[rows] - r64).max()) <= TOL
