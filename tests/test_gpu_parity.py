"""GPU parity: librmx.so (HIP, gfx950) against the oracle on identical inputs.

Tolerances: gathers, ids, table fills, first order and FM are bit-exact (integer / copy /
same-order fp32 work); model outputs are sigmoid probabilities compared with
|p_gpu - p_oracle_fp32| <= 1e-5 (BASELINE.json north_star), and also against the fp64
oracle with the same bound.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


def _kinds():
    return {
        "lr": (oc.LR, {}),
        "deepfm": (oc.DEEPFM, dict(fc=(400, 400, 400))),
        "dnn": (oc.DNN, dict(fc=(64, 48))),
        "xdeepfm1": (oc.XDEEPFM, dict(fc=(64, 32), cin=(200,))),
        "xdeepfm3": (oc.XDEEPFM, dict(fc=(64, 32), cin=(24, 40, 16))),
        "dcn": (oc.DCN, dict(fc=(64, 32), cross_depth=3)),
        "pnn": (oc.PNN, dict(fc=(48, 32))),
    }


def _rmx_model(kind, F=F, k=K, V=1000):
    t, kw = _kinds()[kind]
    fc = list(kw.get("fc", ()))
    if t == oc.LR:
        return rmx.LR(V, F)
    if t == oc.DEEPFM:
        return rmx.DeepFM(V, F, k, fc)
    if t == oc.DNN:
        return rmx.DNN(V, F, k, fc)
    if t == oc.XDEEPFM:
        return rmx.XDeepFM(V, F, k, fc, list(kw["cin"]))
    if t == oc.DCN:
        return rmx.DCN(V, F, k, kw["cross_depth"], fc)
    return rmx.PNN(V, F, k, fc)


def _oracle_model(kind, F=F, k=K):
    t, kw = _kinds()[kind]
    return oc.make_model(t, F, k, **kw)


def _inputs(B, V, F=F, k=K, row0=0):
    ids = oc.gen_ids(SEED_IDS, row0, B, F, V).astype(np.int64)
    wt, et = oc.gen_table(SEED_TAB, V, k)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    return ids, wt, et, w, e, index


# ------------------------------------------------------------ bit-exact ----
def test_synthetic_generators_bit_exact(ctx):
    V, B = 100003, 257
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 77, B, F, V, ids_dev)
    ctx.sync()
    assert np.array_equal(ids_dev.numpy(), oc.gen_ids(SEED_IDS, 77, B, F, V))
    # gather every id of the batch back: bit-exact copies of the oracle table rows
    n = B * F
    w_out = rmx.DeviceArray(ctx, n, np.float32)
    e_out = rmx.DeviceArray(ctx, n * K, np.float32)
    table.gather(ids_dev, n, w_out, e_out)
    ctx.sync()
    w_ref, e_ref = oc.gather(wt, et, 1, ids_dev.numpy().astype(np.int64))
    assert np.array_equal(w_out.numpy(), w_ref)
    assert np.array_equal(e_out.numpy(), e_ref)


def test_table_upload_kmajor_layout_bit_exact(ctx):
    """Reference PS layout: k rows x V columns (ParRecModel.scala:95-101, :300-306)."""
    V = 5003
    wt, et = oc.gen_table(11, V, K)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.upload(wt, np.ascontiguousarray(et.T), layout=rmx.LAYOUT_K_MAJOR)
    ids = np.random.default_rng(0).integers(0, V, 4096).astype(np.int32)
    ids_dev = rmx.DeviceArray.from_numpy(ctx, ids)
    w_out = rmx.DeviceArray(ctx, len(ids), np.float32)
    e_out = rmx.DeviceArray(ctx, len(ids) * K, np.float32)
    table.gather(ids_dev, len(ids), w_out, e_out)
    ctx.sync()
    w_ref, e_ref = oc.gather(wt, np.ascontiguousarray(et.T), 0, ids.astype(np.int64))
    assert np.array_equal(w_out.numpy(), w_ref)
    assert np.array_equal(e_out.numpy(), e_ref)


@pytest.mark.parametrize("B", [1, 63, 1000])
def test_encoder_first_order_fm_bit_exact(ctx, B):
    V = 20000
    ids, wt, et, w, e, index = _inputs(B, V)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.upload(wt, et)
    model = rmx.DeepFM(V, F, K, [32])
    ids_dev = rmx.DeviceArray.from_numpy(ctx, ids.astype(np.int32))
    y = rmx.DeviceArray(ctx, B, np.float32)
    model.encoder_ids(table, B, ids_dev, y)
    ctx.sync()
    ref = oc.first_order(B, index, w) + oc.fm(B, F, K, e)
    assert np.array_equal(y.numpy(), ref)


# ---------------------------------------------------------- L-A drop-in ----
@pytest.mark.parametrize("kind", list(_kinds().keys()))
@pytest.mark.parametrize("B", [1, 37, 300])
def test_forward_host_arrays_matches_oracle(kind, B):
    """RecModel.forward(batchSize, batch, bias, weights, embeddings, k, mats, matSizes)."""
    V = 5000
    ids, wt, et, w, e, index = _inputs(B, V)
    m = _rmx_model(kind)
    om = _oracle_model(kind)
    mats = m.initMats(SEED_MATS)
    bias = np.array([0.01], np.float32)
    coo = rmx.CooLongFloatMatrix(index, ids)
    if kind == "lr":
        got = m.forward(B, coo, bias, w)
        ref32 = oc.forward(om, B, index, bias, w, None, None, 0)
        ref64 = oc.forward(om, B, index, bias, w, None, None, 1)
    else:
        got = m.forward(B, coo, bias, w, e, K, mats, m.getMatsSize())
        ref32 = oc.forward(om, B, index, bias, w, e, mats, 0)
        ref64 = oc.forward(om, B, index, bias, w, e, mats, 1)
    assert got.shape == (B,)
    assert np.abs(got - ref32).max() <= TOL, (kind, np.abs(got - ref32).max())
    assert np.abs(got - ref64).max() <= TOL


def test_lr_ragged_unsorted_index():
    """LR rows carry any number of nonzeros (LIBSVM); Scatter sums in ascending n per row."""
    rng = np.random.default_rng(5)
    B = 97
    lens = rng.integers(0, 60, B)
    index = np.concatenate([np.full(l, b) for b, l in enumerate(lens)]).astype(np.int64)
    perm = rng.permutation(len(index))
    index = index[perm]
    w = rng.uniform(-1, 1, len(index)).astype(np.float32)
    m = rmx.LR(1000)
    bias = np.array([-0.2], np.float32)
    got = m.forward(B, (index, np.zeros_like(index)), bias, w)
    ref = oc.forward(oc.make_model(oc.LR), B, index, bias, w, None, None, 0)
    assert np.array_equal(got, ref) or np.abs(got - ref).max() <= 1e-7


def test_deepfm_irregular_index_first_order():
    """nnz == B*F but rows not in order: embeddings reshape by position, first order by index."""
    B, V = 50, 3000
    ids, wt, et, w, e, index = _inputs(B, V)
    rng = np.random.default_rng(1)
    index = rng.permutation(index)
    m = _rmx_model("deepfm")
    om = _oracle_model("deepfm")
    mats = m.initMats(SEED_MATS)
    bias = np.array([0.01], np.float32)
    got = m.forward(B, (index, ids), bias, w, e, K, mats, m.getMatsSize())
    ref = oc.forward(om, B, index, bias, w, e, mats, 0)
    assert np.abs(got - ref).max() <= TOL


def test_error_modes():
    B, V = 8, 500
    ids, wt, et, w, e, index = _inputs(B, V)
    m = _rmx_model("deepfm")
    mats = m.initMats(1)
    bias = np.array([0.0], np.float32)
    bad = index.copy()
    bad[3] = B  # Scatter require(index < batchSize)
    with pytest.raises(rmx.IllegalArgumentError):
        m.forward(B, (bad, ids), bias, w, e, K, mats, m.getMatsSize())
    with pytest.raises(rmx.ShapeError):  # Reshape(B, F, k) with nnz != B*F
        m.forward(B + 1, (index, ids), bias, w, e, K, mats, m.getMatsSize())
    with pytest.raises(rmx.MatsError):
        m.forward(B, (index, ids), bias, w, e, K, mats, m.getMatsSize()[:-2])
    with pytest.raises(rmx.IllegalArgumentError):  # missing key
        m.forward(B, (index, ids), None, w, e, K, mats, m.getMatsSize())


# ------------------------------------------------------ L-B device path ----
@pytest.mark.parametrize("kind", list(_kinds().keys()))
def test_forward_ids_matches_oracle(ctx, kind):
    B, V = 517, 50000
    ids, wt, et, w, e, index = _inputs(B, V)
    m = _rmx_model(kind, V=V)
    om = _oracle_model(kind)
    mats = m.initMats(SEED_MATS)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.upload(wt, et)
    m.setMats(mats)
    m.setBias(0.01)
    ids_dev = rmx.DeviceArray.from_numpy(ctx, ids.astype(np.int32))
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    bias = np.array([0.01], np.float32)
    ref = oc.forward(om, B, index, bias, w, e if kind != "lr" else None, mats if kind != "lr" else None, 0)
    assert np.abs(out.numpy() - ref).max() <= TOL


def test_deepfm_headline_config(ctx):
    """configs[1]: DeepFM fp32, 39 fields / 1M vocab / k=16, fcDims 400,400,400, B = 16384."""
    B, V = 16384, 1_000_000
    m = rmx.DeepFM(V, F, K, [400, 400, 400])
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    got = out.numpy()
    assert np.isfinite(got).all()
    # oracle on a bounded slice of the same batch (rows 0..2047 and the tail)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = _oracle_model("deepfm")
    for r0, n in ((0, 2048), (B - 333, 333)):
        ids = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, ids)
        index = np.repeat(np.arange(n, dtype=np.int64), F)
        ref = oc.forward(om, n, index, np.array([0.01], np.float32), w, e, mats, 0)
        assert np.abs(got[r0:r0 + n] - ref).max() <= TOL
    # determinism: a second launch gives identical bits
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    assert np.array_equal(out.numpy(), got)


def test_xdeepfm_cin3x200_config(ctx):
    """configs[2]: xDeepFM CIN 200,200,200 (build semantics for L > 1, Appendix A)."""
    B, V = 48, 1_000_000
    m = rmx.XDeepFM(V, F, K, [400, 400, 400], [200, 200, 200])
    om = oc.make_model(oc.XDEEPFM, F, K, fc=(400, 400, 400), cin=(200, 200, 200))
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    wt, et = oc.gen_table(SEED_TAB, V, K)
    ids = oc.gen_ids(SEED_IDS, 0, B, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    ref = oc.forward(om, B, index, np.array([0.01], np.float32), w, e, mats, 1)
    assert np.abs(out.numpy() - ref).max() <= TOL


# ------------------------------------------------- line-row tables (rmx_table::line) ----
@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "dnn", "lr", "xdeepfm", "dcn", "pnn"])
@pytest.mark.parametrize("B", [1, 300, 65536])
@pytest.mark.parametrize("bf16", [False, True])
def test_line_table_forward_bitwise_equals_row_table(kind, B, bf16):
    """With knob table_lines 1, k = 16 tables keep a [V][32] [emb | w | pad] line copy (fp32: one 128-B line
    per id; bf16: one 64-B half line, round 5) that DeepFM / DNN / LR and DCN (cross fused into layer 1)
    forwards read; the gathers are copies, so every model's output is BITWISE the one read from the plain
    emb / w arrays (table_lines 0), through forward_ids and the predict loop."""
    import rmx
    ctx = rmx.default_context()
    V, F, K = 100_003, 39, 16
    fc = [400, 400, 400] if B == 65536 else [64, 32]
    m = {"deepfm": lambda: rmx.DeepFM(V, F, K, fc), "dnn": lambda: rmx.DNN(V, F, K, fc), "lr": lambda: rmx.LR(V, F),
         "xdeepfm": lambda: rmx.XDeepFM(V, F, K, fc, [48, 32]), "dcn": lambda: rmx.DCN(V, F, K, 3, fc),
         "pnn": lambda: rmx.PNN(V, F, K, fc)}[kind]()
    if bf16 and kind == "xdeepfm":
        pytest.skip("xDeepFM runs fp32 (its CIN has no bf16 path)")
    if bf16 and kind != "lr":
        m.setPrecision(rmx.DTYPE_BF16)
    if kind != "lr":
        m.setMats(m.initMats(0x3A75))
    m.setBias(0.01)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, 0x5EED2026, 17, B, F, V, ids)
    outs = []
    for lines in (1, 0):
        rmx.set_tuning("table_lines", lines)
        try:
            t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16 if bf16 else rmx.DTYPE_F32)
            t.fill_synthetic(0x7AB1E)
        finally:
            rmx.set_tuning("table_lines", None)
        o = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(t, B, ids, o)
        p = rmx.DeviceArray(ctx, B, np.float32)
        m.predict_ids(t, B, ids, p, batch=max(1, B // 3))
        ctx.sync()
        outs.append((o.numpy(), p.numpy()))
        t.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    # forward (one launch of B) against the predict loop (launches of B / 3): a batch's size picks its tower
    # kernels (row-owner head / tail from the batch that fills every CU, the whole-tower kernel below it),
    # whose output dots sum in different orders -- equal to fp32 rounding, not bitwise (test_metric.py
    # holds the loop bitwise to forwards of the same batches)
    # (bf16 towers: bf16-stored activations, so the kernels' rounding points differ too: 2e-4, the bf16 bar)
    assert float(np.abs(outs[0][0] - outs[0][1]).max()) <= (2e-4 if bf16 else 2e-6)

