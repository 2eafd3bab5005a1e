"""bf16 configuration (BASELINE.json configs[4]: DCN + PNN with a bf16 table and bf16 weights).

The device stores the table, the GEMM weights and the activations kept between GEMM layers in
bf16 (round to nearest even) and accumulates in fp32 on v_mfma_f32_16x16x32_bf16.  The oracle runs
on the SAME bf16-rounded parameters and emulates the same storage points (oracle precision 2:
fp64 accumulation, stored activations and PNN inner products rounded to bf16).  Build-defined
tolerance |p_gpu - p_oracle_bf16| <= 2e-4: the fp32-vs-fp64 accumulation order can flip the bf16
rounding of an activation (one bf16 ulp, 2^-8 relative), which moves p by O(1e-5).  The gathers of
a bf16 table are bit-exact.
"""
import numpy as np
import pytest

import oracle_ctypes as oc

pytestmark = pytest.mark.gpu

F, K = 39, 16
TOL_BF16 = 2e-4
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75


def _model(kind, V):
    import rmx
    return {
        "dcn": lambda: (rmx.DCN(V, F, K, 3, [400, 400, 400]), oc.make_model(oc.DCN, F, K, fc=(400, 400, 400),
                                                                          cross_depth=3)),
        "pnn": lambda: (rmx.PNN(V, F, K, [400, 400, 400]), oc.make_model(oc.PNN, F, K, fc=(400, 400, 400))),
        "pnn1": lambda: (rmx.PNN(V, F, K, [64]), oc.make_model(oc.PNN, F, K, fc=(64,))),
        "dnn": lambda: (rmx.DNN(V, F, K, [128, 64]), oc.make_model(oc.DNN, F, K, fc=(128, 64))),
        "dnn32": lambda: (rmx.DNN(V, F, K, [32, 400, 400]), oc.make_model(oc.DNN, F, K, fc=(32, 400, 400))),
        "deepfm": lambda: (rmx.DeepFM(V, F, K, [400, 400, 400]), oc.make_model(oc.DEEPFM, F, K, fc=(400, 400, 400))),
        "lr": lambda: (rmx.LR(V, F), oc.make_model(oc.LR)),
    }[kind]()


def _rounded_table(V):
    wt, et = oc.gen_table(SEED_TAB, V, K)
    return oc.round_bf16(wt), oc.round_bf16(et)


def test_bf16_table_fill_and_gather_bit_exact():
    import rmx
    ctx = rmx.default_context()
    V, n = 50_003, 4096
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    ids = np.random.default_rng(0).integers(0, V, n).astype(np.int32)
    ids_d = rmx.DeviceArray.from_numpy(ctx, ids)
    w = rmx.DeviceArray(ctx, n, np.float32)
    e = rmx.DeviceArray(ctx, n * K, np.float32)
    t.gather(ids_d, n, w, e)
    ctx.sync()
    wt, et = _rounded_table(V)
    assert np.array_equal(w.numpy(), wt[ids]) and np.array_equal(e.numpy().reshape(n, K), et[ids])
    # upload (k-major PS layout) rounds the same way
    wt32, et32 = oc.gen_table(SEED_TAB, V, K)
    t2 = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t2.upload(wt32, np.ascontiguousarray(et32.T), layout=rmx.LAYOUT_K_MAJOR)
    t2.gather(ids_d, n, w, e)
    ctx.sync()
    assert np.array_equal(w.numpy(), wt[ids]) and np.array_equal(e.numpy().reshape(n, K), et[ids])


@pytest.mark.parametrize("kind", ["dcn", "pnn", "pnn1", "dnn", "deepfm", "lr"])
def test_bf16_forward_ids_matches_bf16_oracle(kind):
    import rmx
    ctx = rmx.default_context()
    V, B = 50_003, 517
    m, om = _model(kind, V)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    mats = oc.round_bf16(m.initMats(SEED_MATS)) if kind != "lr" else None
    m.setPrecision(rmx.DTYPE_BF16)
    if mats is not None:
        m.setMats(mats)
    m.setBias(0.01)
    ids = oc.gen_ids(SEED_IDS, 5, B, F, V).astype(np.int64)
    ids_d = rmx.DeviceArray.from_numpy(ctx, ids.astype(np.int32))
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(t, B, ids_d, out)
    ctx.sync()
    got = out.numpy()
    wt, et = _rounded_table(V)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    emb = e if kind != "lr" else None
    ref_bf16 = oc.forward(om, B, index, bias, w, emb, mats, 2)
    ref_f64 = oc.forward(om, B, index, bias, w, emb, mats, 1)
    err = float(np.abs(got - ref_bf16).max())
    print("%s bf16: max|p - p_oracle_bf16| = %.3g, max|p - p_oracle_fp64(no act. rounding)| = %.3g"
          % (kind, err, float(np.abs(got - ref_f64).max())))
    assert err <= TOL_BF16


def test_bf16_host_array_forward_rounds_inputs():
    """L-A (RecModel.forward host arrays) on a bf16 model: the fp32 arrays are read as bf16."""
    import rmx
    V, B = 5000, 300
    m, om = _model("pnn", V)
    mats = oc.round_bf16(m.initMats(SEED_MATS))
    m.setPrecision(rmx.DTYPE_BF16)
    ids = oc.gen_ids(SEED_IDS, 0, B, F, V).astype(np.int64)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    w, e = oc.gather(wt, et, 1, ids)  # unrounded fp32 arrays from the caller
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    got = m.forward(B, (index, ids), bias, w, e, K, mats, m.getMatsSize())
    ref = oc.forward(om, B, index, bias, oc.round_bf16(w), oc.round_bf16(e), mats, 2)
    assert np.abs(got - ref).max() <= TOL_BF16


def test_bf16_rejects_mismatched_table_and_xdeepfm():
    import rmx
    ctx = rmx.default_context()
    m, _ = _model("dcn", 1000)
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(oc.round_bf16(m.initMats(1)))
    m.setBias(0.0)
    t = rmx.EmbeddingTable(ctx, 1000, K)  # fp32 table
    ids = rmx.DeviceArray.from_numpy(ctx, np.zeros(F, np.int32))
    out = rmx.DeviceArray(ctx, 1, np.float32)
    with pytest.raises(rmx.RmxError):
        m.forward_ids(t, 1, ids, out)
    x = rmx.XDeepFM(1000, F, K, [8], [8])
    with pytest.raises(rmx.RmxError):
        x.setPrecision(rmx.DTYPE_BF16)


@pytest.mark.parametrize("kind", ["dcn", "pnn"])
def test_bf16_bench_batch_matches_bf16_oracle(kind):
    """B = 65,536 (the bench batch): the large-batch tower variants (8/16-wave LDS-DMA rings, the
    long-K PNN layer 1) against the bf16 oracle on a head and a tail slice of the batch."""
    import rmx
    ctx = rmx.default_context()
    V, B = 50_003, 65536
    m, om = _model(kind, V)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    mats = oc.round_bf16(m.initMats(SEED_MATS))
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(mats)
    m.setBias(0.01)
    ids_d = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_d)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(t, B, ids_d, out)
    ctx.sync()
    got = out.numpy()
    wt, et = _rounded_table(V)
    for r0, n in ((0, 512), (B - 300, 300)):
        ids = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, ids)
        index = np.repeat(np.arange(n, dtype=np.int64), F)
        ref = oc.forward(om, n, index, np.array([0.01], np.float32), w, e, mats, 2)
        assert np.abs(got[r0:r0 + n] - ref).max() <= TOL_BF16



@pytest.mark.parametrize("kind", ["dcn", "pnn", "dnn32"])
def test_bf16_fast_ring_variant_bitwise(kind):
    """tower_variant 6 (the branch-free 3-deep ring tile with two 208-column slices, k_gemm.hpp
    launch_tower_nt; PNN layer 1's default) accumulates each output in the same K-step order as the
    2-deep ring (variant 4, DCN's default) and the 16-wave 3-deep ring (variant 3): bitwise-equal
    predictions at B = 65,536.  dnn32 has a 400-wide layer with K = 32, one K step: fewer steps than the
    ring's two stages of lead, which the prologue must still fill (the loop's counted wait assumes them)."""
    import rmx
    ctx = rmx.default_context()
    V, B = 50_003, 65536
    m, om = _model(kind, V)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    mats = oc.round_bf16(m.initMats(SEED_MATS))
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(mats)
    m.setBias(0.01)
    ids_d = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_d)
    out = rmx.DeviceArray(ctx, B, np.float32)
    got = {}
    try:
        rmx.set_tuning("bf16_tail", 0)  # the engine's layers 2 / 3 (the tail kernel has its own test)
        for var in (None, 3, 4, 6):
            rmx.set_tuning("tower_variant", var)
            m.forward_ids(t, B, ids_d, out)
            ctx.sync()
            got[var] = out.numpy().copy()
    finally:
        rmx.set_tuning("tower_variant", None)
        rmx.set_tuning("bf16_tail", None)
    for var in (None, 3, 4):
        assert np.array_equal(got[6], got[var]), var
    wt, et = _rounded_table(V)
    n = 256
    ids = oc.gen_ids(SEED_IDS, B - n, n, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(n, dtype=np.int64), F)
    ref = oc.forward(om, n, index, np.array([0.01], np.float32), w, e, mats, 2)
    assert np.abs(got[6][B - n:] - ref).max() <= TOL_BF16


@pytest.mark.parametrize("kind,B", [("dcn", 65536), ("pnn", 65536), ("dcn", 37), ("pnn", 1000),
                                    ("dcn", 300 * 64 + 17), ("dnn32", 4099)])
def test_bf16_tower_tail_matches_unfused(kind, B):
    """The bf16 tower tail (csrc/k_tail.hip: the last hidden layer + the output layer in one persistent
    launch, h2 kept in LDS) against the same model with the tail off (two engine launches, h2 through
    HBM) and against the bf16 oracle.  B covers one partial row block (37), a ragged last block
    (1000), more row blocks than CUs (several per block: 19,217 and 65,536).  dnn32 has no tail
    (its 400-wide layer has K = 32): the fallback must be taken, bitwise."""
    import rmx
    ctx = rmx.default_context()
    V = 50_003
    m, om = _model(kind, V)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    mats = oc.round_bf16(m.initMats(SEED_MATS))
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(mats)
    m.setBias(0.01)
    ids_d = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_d)
    out = rmx.DeviceArray(ctx, B, np.float32)
    got = {}
    try:
        for tail in (0, 1):
            rmx.set_tuning("bf16_tail", tail)
            m.set_timing(True)
            m.forward_ids(t, B, ids_d, out)
            ctx.sync()
            stages, _ = m.get_timing()
            m.set_timing(False)
            got[tail] = out.numpy().copy()
            assert ("tower_tail" in stages) == (tail == 1 and kind != "dnn32"), stages
    finally:
        rmx.set_tuning("bf16_tail", None)
    diff = float(np.abs(got[1] - got[0]).max())
    print("%s B=%d: max|p_tail - p_unfused| = %.3g" % (kind, B, diff))
    if kind == "dnn32":
        assert np.array_equal(got[1], got[0])
    else:
        # h2 is the same bf16 of the same fp32 sums; only the logit's summation order differs
        assert diff <= 5e-5
    wt, et = _rounded_table(V)
    for r0, n in ((0, min(B, 256)), (max(0, B - 100), min(B, 100))):
        ids = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, ids)
        index = np.repeat(np.arange(n, dtype=np.int64), F)
        ref = oc.forward(om, n, index, np.array([0.01], np.float32), w, e, mats, 2)
        assert np.abs(got[1][r0:r0 + n] - ref).max() <= TOL_BF16


@pytest.mark.parametrize("kind,B", [("pnn", 1000), ("pnn", 65536), ("dcn", 1000), ("dcn", 65536)])
def test_bf16_tail_first_order_bitwise(kind, B):
    """PNN bf16, and DCN bf16 when layer 1 does not sum the first order from its weight ring (tower variant 3
    here): the tower tail's head sums the first order itself (tail_fo, default on: field order from 0,
    encoder_k16_kernel<0>'s arithmetic) -- bitwise the predictions of the first-order kernel path."""
    import rmx
    ctx = rmx.default_context()
    V = 50_003
    m, _ = _model(kind, V)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(oc.round_bf16(m.initMats(SEED_MATS)))
    m.setBias(0.01)
    ids_d = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_d)
    out = rmx.DeviceArray(ctx, B, np.float32)
    got = {}
    try:
        if kind == "dcn":
            rmx.set_tuning("tower_variant", 3)
        for fo in (0, 1):
            rmx.set_tuning("tail_fo", fo)
            m.set_timing(True)
            m.forward_ids(t, B, ids_d, out)
            ctx.sync()
            stages, _ = m.get_timing()
            m.set_timing(False)
            got[fo] = out.numpy().copy()
            assert ("first_order" in stages) == (fo == 0), stages
    finally:
        rmx.set_tuning("tail_fo", None)
        rmx.set_tuning("tower_variant", None)
    assert np.array_equal(got[0], got[1])
