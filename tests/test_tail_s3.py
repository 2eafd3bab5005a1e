"""GPU parity of the fp32 tower tail (csrc/k_tail_s3.hip): the last hidden Linear(400 -> 400) + ReLU and
the output Linear(400 -> 1) + head of an fp32 tower in one persistent split-GEMM launch, h2 kept in
registers (model/encoder/HigherOrderEncoder.scala:34-59; heads DeepFM.scala:54-80 and the others).

Each case runs the same model on the same inputs with the tail forced on (knob s3_tail 2) and off (0,
the two split-GEMM launches).  h2 is the same fp32 sums in the same K order, so only the output dot's
summation order differs: the two agree to 5e-6, and both meet the north-star bar (1e-5) against the
fp64 oracle on head / tail slices.  Batch sizes: ragged (37, 1,000, 19,217 -- a partial last row block
and fewer row blocks than CUs) and the bench batch 65,536 (two row blocks per CU)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
TAIL_VS_UNFUSED = 5e-6
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x7A11, 0x7AB1E, 0x3A75
FC = (400, 400, 400)

KINDS = {
    "deepfm": (oc.DEEPFM, dict(fc=FC)),
    "dnn": (oc.DNN, dict(fc=FC)),
    "xdeepfm": (oc.XDEEPFM, dict(fc=FC, cin=(200, 200))),
    "dcn": (oc.DCN, dict(fc=FC, cross_depth=3)),
    "pnn": (oc.PNN, dict(fc=FC)),
}


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    rmx.set_tuning("s3_small", 0)  # (small batches would run the whole-tower kernel, k_small_s3.hip)
    rmx.set_tuning("s3_fused", 0)  # (and DeepFM batches that fill the GPU the fused tower, k_fused_s3.hip)
    yield
    rmx.set_tuning("s3_tail", None)
    rmx.set_tuning("s3_small", None)
    rmx.set_tuning("s3_fused", None)


def _model(kind, V):
    t, kw = KINDS[kind]
    fc = list(kw["fc"])
    if t == oc.DEEPFM:
        return rmx.DeepFM(V, F, K, fc)
    if t == oc.DNN:
        return rmx.DNN(V, F, K, fc)
    if t == oc.XDEEPFM:
        return rmx.XDeepFM(V, F, K, fc, list(kw["cin"]))
    if t == oc.DCN:
        return rmx.DCN(V, F, K, kw["cross_depth"], fc)
    return rmx.PNN(V, F, K, fc)


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("B", [37, 1000, 19217, 65536])
def test_fp32_tail_matches_unfused_and_oracle(ctx, kind, B):
    V = 50000
    m = _model(kind, V)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = {}
    for knob in (0, 2):
        rmx.set_tuning("s3_tail", knob)
        m.set_timing(True)
        m.forward_ids(table, B, ids_dev, out)
        ctx.sync()
        res[knob] = out.numpy().copy()
        stages, _ = m.get_timing()
        m.set_timing(False)
        assert ("tower_tail" in stages) == (knob == 2), stages
    d = float(np.abs(res[2] - res[0]).max())
    t, kw = KINDS[kind]
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = oc.make_model(t, F, K, **kw)
    n = 64 if kind == "xdeepfm" else 256
    errs = []
    for r0 in sorted({0, max(0, B - n)}):
        nn = min(n, B - r0)
        ids = oc.gen_ids(SEED_IDS, r0, nn, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, ids)
        index = np.repeat(np.arange(nn, dtype=np.int64), F)
        ref = oc.forward(om, nn, index, np.array([0.01], np.float32), w, e, mats, 1)
        errs.append((float(np.abs(res[2][r0:r0 + nn] - ref).max()), float(np.abs(res[0][r0:r0 + nn] - ref).max())))
    print("%s B=%d: |tail - unfused| %.3g; vs fp64 (tail, unfused) %s" % (kind, B, d, errs))
    assert d <= TAIL_VS_UNFUSED
    for e_tail, e_unf in errs:
        assert e_tail <= TOL and e_unf <= TOL
    # deterministic: a second launch of the tail gives identical bits
    rmx.set_tuning("s3_tail", 2)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    assert np.array_equal(out.numpy(), res[2])


def test_fp32_tail_is_the_default_at_the_bench_batch(ctx):
    """configs[1] (DeepFM, B = 65,536) without the fused tower (s3_fused 0) runs the tail by default (knob
    s3_tail 1: row blocks >= CUs)."""
    B, V = 65536, 100000
    m = rmx.DeepFM(V, F, K, list(FC))
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.set_timing(True)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    stages, _ = m.get_timing()
    assert "tower_tail" in stages and "tower_layer2" not in stages, stages


@pytest.mark.parametrize("B", [16384, 40000, 49152])
def test_fp32_tail_half_blocks_bitwise(ctx, B):
    """The last round of row blocks as 64-row half blocks (k_rowown.hpp QRows, knob half_blocks: waves 4 .. 7
    keep the ring without MFMAs) computes every row with the same instructions: bitwise the full-block
    launch, at B = 16,384 (all half), 40,000 (one full round + a partial half round) and 49,152 (one full
    round + a full half round)."""
    V = 50000
    m = rmx.DeepFM(V, F, K, list(FC))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = {}
    try:
        rmx.set_tuning("s3_tail", 2)
        for hb in (0, 1):  # (knob 1 forces half blocks on)
            rmx.set_tuning("half_blocks", hb)
            m.forward_ids(table, B, ids_dev, out)
            ctx.sync()
            res[hb] = out.numpy().copy()
    finally:
        rmx.set_tuning("half_blocks", None)
    assert np.array_equal(res[0], res[1])
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = oc.make_model(oc.DEEPFM, F, K, fc=FC)
    r0, n = B - 100, 100
    ids = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats, 1)
    assert np.abs(res[1][r0:] - ref).max() <= TOL
