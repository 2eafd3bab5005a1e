"""Backward + BCE (RecModel.backward).

CPU: the oracle backward (oracle/rmx_oracle_train.c, f64) against central finite differences of
the independent numpy forward (tests/ref_numpy.py, f64) for every model type -- this pins the oracle
(the reference ships no gradients to compare with: parity unpinned against BigDL itself).
GPU: librmx's backward (rmx_backward_ids / rmx_backward) against the oracle.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import ref_numpy

EPS = 1e-12
KINDS = {"lr": oc.LR, "deepfm": oc.DEEPFM, "dnn": oc.DNN, "dcn": oc.DCN, "pnn": oc.PNN, "xdeepfm": oc.XDEEPFM}


def _bce(p, t):
    t = (np.asarray(t) > 0).astype(np.float64)
    return float(-np.mean(t * np.log(p + EPS) + (1 - t) * np.log(1 - p + EPS)))


def _case(kind, B=5, F=3, k=4, seed=0):
    rng = np.random.default_rng(seed)
    fc = (5, 3)
    cin = (3, 2) if kind == "xdeepfm" else ()
    cd = 2 if kind == "dcn" else 0
    m = oc.make_model(KINDS[kind], F, k, fc=fc if kind != "lr" else (), cin=cin, cross_depth=cd)
    nnz = B * F
    index = np.repeat(np.arange(B), F).astype(np.int64)
    w = rng.uniform(-0.5, 0.5, nnz).astype(np.float32)
    e = rng.uniform(-0.5, 0.5, nnz * k).astype(np.float32)
    ml = oc.mats_len(m) if kind != "lr" else 0
    mats = rng.uniform(-0.6, 0.6, ml).astype(np.float32)
    bias = np.array([0.1], np.float32)
    t = (rng.random(B) > 0.5).astype(np.float32)
    return m, dict(B=B, F=F, k=k, fc=fc, cin=cin, cd=cd, index=index, w=w, e=e, mats=mats, bias=bias, t=t)


def _loss64(kind, c, w=None, e=None, mats=None, bias=None):
    w = c["w"] if w is None else w
    e = c["e"] if e is None else e
    mats = c["mats"] if mats is None else mats
    bias = c["bias"] if bias is None else bias
    p = ref_numpy.forward(kind, c["B"], c["F"], c["k"], c["index"], bias, w, e, mats, fc=c["fc"], cin=c["cin"],
                          cross_depth=c["cd"])
    return _bce(p, c["t"])


def _fd(kind, c, name, idx, h=1e-5):
    base = {"w": c["w"], "e": c["e"], "mats": c["mats"], "bias": c["bias"]}[name].astype(np.float64)
    a, b = base.copy(), base.copy()
    a[idx] += h
    b[idx] -= h
    return (_loss64(kind, c, **{name: a}) - _loss64(kind, c, **{name: b})) / (2 * h)


@pytest.mark.parametrize("kind", list(KINDS))
def test_oracle_backward_matches_finite_differences(kind):
    m, c = _case(kind)
    g = oc.backward(m, c["B"], c["index"], c["bias"], c["w"] if kind != "dnn" else None,
                    c["e"] if kind != "lr" else None, c["mats"] if kind != "lr" else None, c["t"])
    assert abs(g["loss"] - _loss64(kind, c)) < 1e-9
    rng = np.random.default_rng(1)
    checks = [("bias", np.array([0]))]
    if kind != "dnn":
        checks.append(("w", rng.choice(len(c["w"]), 6, replace=False)))
    if kind != "lr":
        checks.append(("e", rng.choice(len(c["e"]), 12, replace=False)))
        checks.append(("mats", rng.choice(len(c["mats"]), min(40, len(c["mats"])), replace=False)))
    key = {"bias": "bias", "w": "weights", "e": "embedding", "mats": "mats"}
    for name, idxs in checks:
        for i in idxs:
            num = _fd(kind, c, name, i)
            ana = float(g[key[name]][i])
            assert abs(num - ana) <= 2e-6 + 1e-4 * abs(num), (kind, name, int(i), num, ana)


def test_oracle_backward_irregular_lr_index():
    """Scatter backward (bnn/Scatter.scala:38-59): grad of w[n] is the grad of row index[n]."""
    m = oc.make_model(oc.LR, 3, 4)
    index = np.array([2, 0, 0, 1, 2, 2], np.int64)
    w = np.linspace(-0.3, 0.4, 6).astype(np.float32)
    t = np.array([1, 0, 1], np.float32)
    g = oc.backward(m, 3, index, np.array([0.05], np.float32), w, None, None, t)
    y1 = np.zeros(3)
    np.add.at(y1, index, w.astype(np.float64))
    p = 1 / (1 + np.exp(-(y1 + 0.05)))
    gz = (p - (t > 0)) / 3  # BCE + Sigmoid for eps -> 0
    assert np.allclose(g["weights"], gz[index], rtol=1e-6, atol=1e-9)
    assert np.isclose(g["bias"][0], gz.sum(), rtol=1e-6, atol=1e-9)
    assert np.isclose(g["loss"], _bce(p, t), rtol=1e-9)


# ------------------------------------------------------------------ GPU ----
GPU_KINDS = ["lr", "deepfm", "dnn", "dcn", "pnn", "xdeepfm"]
CIN_FOR = {(400, 400, 400): (64, 32), (24, 8): (8, 4), (16,): (16,), (32, 16): (8, 4)}
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75
CROSS = 3


def _gpu_model(rmx, kind, V, F, K, fc):
    return {"lr": lambda: rmx.LR(V, F), "deepfm": lambda: rmx.DeepFM(V, F, K, list(fc)),
            "dnn": lambda: rmx.DNN(V, F, K, list(fc)), "dcn": lambda: rmx.DCN(V, F, K, CROSS, list(fc)),
            "pnn": lambda: rmx.PNN(V, F, K, list(fc)),
            "xdeepfm": lambda: rmx.XDeepFM(V, F, K, list(fc), list(CIN_FOR[tuple(fc)]))}[kind]()


def _orc_model(kind, F, K, fc):
    return oc.make_model(KINDS[kind], F, K, fc=fc if kind != "lr" else (), cross_depth=CROSS if kind == "dcn" else 0,
                         cin=CIN_FOR[tuple(fc)] if kind == "xdeepfm" else ())



def _close(got, ref, rel=2e-5, rtol=1e-3, floor=1e-3):
    """fp32 device vs f64 oracle, two bars:
    max |got - ref| <= rel * max |ref|  (the whole array), and element by element
    |got - ref| <= rtol * max(|ref|, floor * max |ref|)  -- so small entries are held to 1e-6 of the
    largest one (20x the array-wide bar) and entries above the floor to 0.1 % of themselves."""
    ref = np.asarray(ref, np.float64)
    got = np.asarray(got, np.float64)
    mx = max(float(np.abs(ref).max()), 1e-6)
    err = float(np.abs(got - ref).max()) / mx
    bound = rtol * np.maximum(np.abs(ref), floor * mx)
    bad = int((np.abs(got - ref) > bound).sum())
    if err > rel or bad:
        print("relative-to-max error %.3g (bar %.3g); %d entries over the element-wise bar" % (err, rel, bad))
    return err <= rel and bad == 0


def _hidden_pre(kind, E, mats, fc):
    """f64 pre-activations of every ReLU layer (rows = samples) of a tower-bearing model."""
    B, F, k = E.shape
    D = F * k
    mats = np.asarray(mats, np.float64)
    x = E.reshape(B, D)
    pres, off = [], 0
    if kind == "dcn":
        off = CROSS * D + CROSS
    if kind == "pnn":
        rows = [i for i in range(F) for j in range(i + 1, F)]
        cols = [j for i in range(F) for j in range(i + 1, F)]
        ip = (E[:, rows] * E[:, cols]).sum(2)
        P, D1 = len(rows), fc[0]
        pre = x @ mats[:D * D1].reshape(D1, D).T + ip @ mats[D * D1:(D + P) * D1].reshape(D1, P).T + mats[(D + P) * D1]
        pres.append(pre)
        x, off, fc = np.maximum(pre, 0), (D + P) * D1 + 1, fc[1:]
    for d in fc:
        K_ = x.shape[1]
        pre = x @ mats[off:off + K_ * d].reshape(d, K_).T + mats[off + K_ * d:off + K_ * d + d]
        pres.append(pre)
        x, off = np.maximum(pre, 0), off + K_ * d + d
    if kind == "xdeepfm":  # CIN maps, rows (b, j) regrouped per sample
        x0 = E.transpose(0, 2, 1).reshape(B * k, F)
        u, hp = x0, F
        for h in CIN_FOR[tuple(fc)]:
            Z = (x0[:, :, None] * u[:, None, :]).reshape(B * k, F * hp)
            pre = Z @ mats[off:off + F * hp * h].reshape(h, F * hp).T + mats[off + F * hp * h:off + F * hp * h + h]
            pres.append(pre.reshape(B, k * h))
            u, off, hp = np.maximum(pre, 0), off + F * hp * h + h, h
    return pres


def _tie_free(kind, E, mats, fc, rel=1e-5):
    """Rows whose ReLU inputs all stay clear of zero: a pre-activation within fp32 rounding of 0 makes
    the ReLU mask ill-conditioned, and fp32 (device) and f64 (oracle) may then legitimately take
    different branches (observed: one row of 512 with pre = -1e-8, |pre| / mean 6e-7)."""
    ok = np.ones(E.shape[0], bool)
    for pre in _hidden_pre(kind, E, mats, fc):
        ok &= (np.abs(pre) > rel * np.abs(pre).mean()).all(axis=1)
    return np.where(ok)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", GPU_KINDS)
@pytest.mark.parametrize("B,fc", [(512, (400, 400, 400)), (37, (24, 8)), (64, (16,))])
def test_backward_ids_matches_oracle(kind, B, fc):
    _backward_ids_check(kind, B, fc)


@pytest.mark.gpu
def test_backward_cin_more_than_256_fields():
    """the fused dL/dz contraction (cin_back_fused_kernel, 256 threads per row) reduces
    the x0 gradient of EVERY field; F = 260 with CIN (8, 4) takes the fused path on layer 2."""
    _backward_ids_check("xdeepfm", 16, (24, 8), F=260, V=30_000)


def _backward_ids_check(kind, B, fc, F=39, V=20_000):
    import rmx
    ctx = rmx.default_context()
    K = 16
    m = _gpu_model(rmx, kind, V, F, K, fc)
    mats = m.initMats(SEED_MATS) if kind != "lr" else np.zeros(0, np.float32)
    if kind != "lr":
        m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    cand = oc.gen_ids(SEED_IDS, 3, 2 * B, F, V).reshape(2 * B, F)
    if kind != "lr":
        _, et0 = oc.gen_table(SEED_TAB, V, K)
        keep = _tie_free(kind, et0[cand.astype(np.int64)].astype(np.float64), mats, fc)
        assert len(keep) >= B
        cand = cand[keep[:B]]
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(np.ascontiguousarray(cand[:B]).reshape(-1))
    tg = (np.random.default_rng(5).random(B) > 0.7).astype(np.float32)
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload(tg)
    ml = len(mats)
    g_b = rmx.DeviceArray(ctx, 1, np.float32)
    g_w = rmx.DeviceArray(ctx, B * F, np.float32)
    g_e = rmx.DeviceArray(ctx, B * F * K, np.float32)
    g_m = rmx.DeviceArray(ctx, max(ml, 1), np.float32)
    loss = rmx.DeviceArray(ctx, 1, np.float32)
    m.backward_ids(t, B, ids, targets, g_b, g_w, g_e, g_m if ml else None, loss)
    ctx.sync()
    wt, et = oc.gen_table(SEED_TAB, V, K)
    h_ids = ids.numpy().astype(np.int64)
    w, e = oc.gather(wt, et, 1, h_ids)
    om = _orc_model(kind, F, K, fc)
    index = np.repeat(np.arange(B), F).astype(np.int64)
    ref = oc.backward(om, B, index, np.array([0.01], np.float32), w if kind != "dnn" else None,
                      e if kind != "lr" else None, mats if kind != "lr" else None, tg)
    assert abs(loss.numpy()[0] - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    assert _close(g_b.numpy(), ref["bias"])
    if kind != "dnn":
        assert _close(g_w.numpy(), ref["weights"])
    if kind != "lr":
        assert _close(g_e.numpy(), ref["embedding"])
        assert _close(g_m.numpy()[:ml], ref["mats"])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,B", [("deepfm", 65536), ("dnn", 40000)])
def test_backward_slice_reduce4_bitwise(kind, B):
    """slice_reduce4: the dW's slice reduction on float4s sums every output's slices in the scalar kernel's
    order -- bitwise the same gradients (the 208 x 208 dW path, rows >= 32,768)."""
    import rmx
    ctx = rmx.default_context()
    V, F, K = 20_000, 39, 16
    m = _gpu_model(rmx, kind, V, F, K, (400, 400, 400))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(11).random(B) > 0.7).astype(np.float32))
    res = {}
    try:
        for v in (0, 1):
            rmx.set_tuning("slice_reduce4", v)
            out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, len(mats), 1)]
            m.backward_ids(t, B, ids, targets, *out)
            ctx.sync()
            res[v] = [o.numpy().copy() for o in out]
    finally:
        rmx.set_tuning("slice_reduce4", None)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [512, 4099])
def test_backward_head_x_matches_oracle(B):
    """train_head_s3: DeepFM's encoder + tower layer 1 as the row-owner head that also stores x and the FM
    sums (k_head_s3.hip, XS) -- every gradient and the loss against the oracle at the usual bar.  B = 512 runs
    it as half row blocks on part of the chip (s3_head 2 forces it), 4,099 one row past the default rule's
    threshold (16 rows per CU); the stage list shows the head ran."""
    import rmx
    rmx.set_tuning("s3_head", 2)
    try:
        _backward_ids_check("deepfm", B, (400, 400, 400))
        ctx = rmx.default_context()
        V, F, K = 20_000, 39, 16
        m = _gpu_model(rmx, "deepfm", V, F, K, (400, 400, 400))
        m.setMats(m.initMats(SEED_MATS))
        m.setBias(0.01)
        t = rmx.EmbeddingTable(ctx, V, K)
        t.fill_synthetic(SEED_TAB)
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        ids.upload(oc.gen_ids(SEED_IDS, 9, B, F, V).astype(np.int32))
        targets = rmx.DeviceArray(ctx, B, np.float32)
        targets.upload(np.zeros(B, np.float32))
        out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, m.matsLength(), 1)]
        m.set_timing(True)
        m.backward_ids(t, B, ids, targets, *out)
        ctx.sync()
        stages, _ = m.get_timing()
        m.set_timing(False)
        assert "head_x" in stages and "encoder_fm_x" not in stages and "tower_layer1" not in stages, stages
    finally:
        rmx.set_tuning("s3_head", None)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "dnn", "dcn", "pnn"])
def test_backward_row_owner_layers_match_oracle(kind):
    """train_layer_s3: the 400 x 400 hidden layers' forward (ReLU(h W^T + b), stored) and their dX (dPre W
    masked by the ReLU of the layer below) on the row-owner kernel (k_layer_s3.hip), which needs a full round of
    row blocks: B = 20,000 (half blocks, a ragged last block).  Every gradient and the loss against the oracle
    at the usual bar, and against the engine's kernels (knob 0) within fp32 summation-order noise."""
    import rmx
    _backward_ids_check(kind, 20_000, (400, 400, 400))
    ctx = rmx.default_context()
    V, F, K, B = 20_000, 39, 16, 20_000
    m = _gpu_model(rmx, kind, V, F, K, (400, 400, 400))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 13, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(7).random(B) > 0.7).astype(np.float32))
    res = {}
    try:
        for v in (0, 1):
            rmx.set_tuning("train_layer_s3", v)
            out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, len(mats), 1)]
            m.backward_ids(t, B, ids, targets, *out)
            ctx.sync()
            res[v] = [o.numpy().copy() for o in out]
    finally:
        rmx.set_tuning("train_layer_s3", None)
    for a, b in zip(res[0], res[1]):
        scale = max(float(np.abs(a).max()), 1e-30)
        assert float(np.abs(a - b).max()) <= 1e-4 * scale


@pytest.mark.gpu
@pytest.mark.parametrize("variant,gz", [(0, 128), (1, 128), (1, 64), (2, 128)])
@pytest.mark.parametrize("kind", ["deepfm", "xdeepfm", "dcn"])
def test_backward_weight_grad_variants(kind, variant, gz):
    """dW on the f32 MFMA kernel (0) and the split GEMM with 64 x 64 (1) / 128 x 128 (2) tiles, the
    CIN's generated-operand dW on 128 x 128 (wgrad_gz 128, the default) or 64 x 64 tiles: all within
    the same oracle bar (tower, CIN and cross weight gradients)."""
    import rmx
    rmx.set_tuning("wgrad_s3", variant)
    rmx.set_tuning("wgrad_gz", gz)
    try:
        test_backward_ids_matches_oracle(kind, 512, (400, 400, 400))
    finally:
        rmx.set_tuning("wgrad_s3", None)
        rmx.set_tuning("wgrad_gz", None)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,gz", [("deepfm", 128), ("xdeepfm", 128), ("xdeepfm", 64), ("dcn", 128), ("pnn", 128)])
@pytest.mark.parametrize("B", [512, 4099])
def test_backward_wgrad_single_buffer_bitwise(kind, gz, B):
    """dW on the single-buffered split kernel (wgrad_sb 1: 128 x 128 tiles, two blocks per CU; 2: the
    64 x 64 tiles too) stages the same chunks and issues the same MFMA sequence per output as the
    double-buffered one (wgrad_sb 0): every gradient is bitwise equal, tower / CIN / cross / product
    dW alike (PNN: K = 624 + 741 columns)."""
    import rmx
    ctx = rmx.default_context()
    V, F, K, fc = 20_000, 39, 16, (400, 400, 400)
    m = _gpu_model(rmx, kind, V, F, K, fc)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 11, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(7).random(B) > 0.7).astype(np.float32))
    ml = len(mats)

    def grads():
        out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, ml, 1)]
        m.backward_ids(t, B, ids, targets, *out)
        ctx.sync()
        return [o.numpy().copy() for o in out]

    rmx.set_tuning("wgrad_gz", gz)
    rmx.set_tuning("wgrad_nk", 0)
    try:
        res = {}
        for sb in (0, 1, 2):
            rmx.set_tuning("wgrad_sb", sb)
            res[sb] = grads()
        # the 208 x 128 tile (every dW, then the default: the CIN's only): same bar as the others
        rmx.set_tuning("wgrad_sb", None)
        for nk in (2, 1):
            rmx.set_tuning("wgrad_nk", nk)
            g_nk = grads()
            for a, b in zip(res[0], g_nk):
                assert np.abs(a - b).max() <= 2e-5 * max(np.abs(a).max(), 1e-30)
    finally:
        rmx.set_tuning("wgrad_sb", None)
        rmx.set_tuning("wgrad_gz", None)
        rmx.set_tuning("wgrad_nk", None)
    for sb in (1, 2):
        for a, b in zip(res[0], res[sb]):
            assert np.array_equal(a, b)
    assert np.isfinite(res[1][3]).all() and np.abs(res[1][3]).max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "xdeepfm", "dcn"])
def test_backward_fused_x_bitwise(kind):
    """train_fuse_x: the encoder kernel storing the gathered rows as the tower input x (1: DeepFM, the
    default; 2: the first-order models too) gives bitwise the gradients and loss of encoder + gather_x (0):
    x is a copy either way and the first order / FM arithmetic is unchanged."""
    import rmx
    ctx = rmx.default_context()
    V, F, K, B = 20_000, 39, 16, 777
    m = _gpu_model(rmx, kind, V, F, K, (32, 16))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 21, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(2).random(B) > 0.7).astype(np.float32))
    res = {}
    try:
        for v in (0, 1, 2):
            rmx.set_tuning("train_fuse_x", v)
            out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, len(mats), 1)]
            m.backward_ids(t, B, ids, targets, *out)
            ctx.sync()
            res[v] = [o.numpy().copy() for o in out]
    finally:
        rmx.set_tuning("train_fuse_x", None)
    for v in (1, 2):
        for a, b in zip(res[0], res[v]):
            assert np.array_equal(a, b), v


@pytest.mark.gpu
@pytest.mark.parametrize("kind,fx,B", [("deepfm", 1, 777), ("deepfm", 1, 65536), ("xdeepfm", 2, 777), ("dcn", 2, 4099)])
def test_backward_encoder_v2_x_bitwise(kind, fx, B):
    """enc_v2_x: the training forward's encoder (x, the FM sums, y1 + y2 / y1) on the batched-request kernel
    (encoder_k16v2_kernel with XO) against the round-4 kernel (0): every gradient and the loss bit for bit --
    x and the FM sums are copies / sums in the same field order either way.  B = 777 / 4,099: a ragged last
    wave; 65,536: the bench batch."""
    import rmx
    ctx = rmx.default_context()
    V, F, K = 20_000, 39, 16
    m = _gpu_model(rmx, kind, V, F, K, (32, 16))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 5, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(3).random(B) > 0.7).astype(np.float32))
    res = {}
    try:
        rmx.set_tuning("train_fuse_x", fx)
        for v in (0, 1):
            rmx.set_tuning("enc_v2_x", v)
            out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, len(mats), 1)]
            m.backward_ids(t, B, ids, targets, *out)
            ctx.sync()
            res[v] = [o.numpy().copy() for o in out]
    finally:
        rmx.set_tuning("train_fuse_x", None)
        rmx.set_tuning("enc_v2_x", None)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)
    assert np.abs(res[1][2]).max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("fc,B", [((32, 16), 777), ((400, 400, 400), 4099)])
def test_backward_fused_head_and_emb_grad(fc, B):
    """train_emb_fused: DeepFM's layer-1 dX epilogue writes the embedding gradient itself (dX + the FM
    term with emb_grad_kernel's arithmetic, the forward's FM sums) -- bitwise the two-kernel result.
    train_head_fused: logit + BCE + the output layer's backward in one kernel -- p, dz and everything fed
    by them bitwise (g_w, g_emb); the batch sums (loss, bias gradient, dW_out) only change summation
    order: 1e-6 relative."""
    import rmx
    ctx = rmx.default_context()
    V, F, K = 20_000, 39, 16
    m = _gpu_model(rmx, "deepfm", V, F, K, fc)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 33, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(3).random(B) > 0.7).astype(np.float32))
    res = {}
    try:
        for eg, hd in ((0, 0), (1, 0), (1, 1)):
            rmx.set_tuning("train_emb_fused", eg)
            rmx.set_tuning("train_head_fused", hd)
            out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, len(mats), 1)]
            m.backward_ids(t, B, ids, targets, *out)
            ctx.sync()
            res[(eg, hd)] = [o.numpy().copy() for o in out]
    finally:
        rmx.set_tuning("train_emb_fused", None)
        rmx.set_tuning("train_head_fused", None)
    for a, b in zip(res[(0, 0)], res[(1, 0)]):
        assert np.array_equal(a, b)
    loss0, gw0, ge0, gm0, gb0 = res[(1, 0)]
    loss1, gw1, ge1, gm1, gb1 = res[(1, 1)]
    assert np.array_equal(gw0, gw1) and np.array_equal(ge0, ge1)
    for a, b in ((loss0, loss1), (gb0, gb1), (gm0, gm1)):
        assert np.allclose(a, b, rtol=1e-6, atol=1e-9 * max(1.0, float(np.abs(a).max())))


@pytest.mark.gpu
def test_backward_wgrad_sq_tile_cin():
    """The CIN's generated-operand dW on the 208 x 208 tile (wgrad_sq_gz 1) against the 208 x 128 one
    (the default): rows = B k = 65,584 (a ragged chunk), within 2e-5 relative per mats block."""
    import rmx
    ctx = rmx.default_context()
    V, F, K, B = 20_000, 39, 16, 4099
    m = _gpu_model(rmx, "xdeepfm", V, F, K, (400, 400, 400))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 9, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(3).random(B) > 0.7).astype(np.float32))
    res = {}
    try:
        for v in (0, 1):
            rmx.set_tuning("wgrad_sq_gz", v)
            out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, len(mats), 1)]
            m.backward_ids(t, B, ids, targets, *out)
            ctx.sync()
            res[v] = [o.numpy().copy() for o in out]
    finally:
        rmx.set_tuning("wgrad_sq_gz", None)
    sizes = list(m.getMatsSize())
    off = 0
    for i in range(0, len(sizes), 2):
        n = sizes[i] * sizes[i + 1]
        a, b = res[0][3][off:off + n], res[1][3][off:off + n]
        assert np.abs(a - b).max() <= 2e-5 * max(np.abs(a).max(), 1e-30), (i // 2, sizes[i], sizes[i + 1])
        off += n
    for a, b in zip(res[0][:3], res[1][:3]):
        assert np.array_equal(a, b)  # the dW does not feed the other gradients


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "dcn", "pnn"])
def test_backward_wgrad_sq_tile(kind):
    """The 208 x 208 dW tile (wgrad_sq 1, default at >= 32,768 rows), with and without the bias
    gradient fused into it (wgrad_bias), against the 128 x 128 tiles + colsum_kernel (wgrad_sq 0, the
    kernels the oracle tests pin at small B): the same per-output chunk / MFMA order over a different
    row-slice split, so within 2e-5 relative of it.  B = 32,768 + 7 (a ragged last chunk); PNN's
    layer 1 has two Linear blocks (K = 624 and 741)."""
    import rmx
    ctx = rmx.default_context()
    V, F, K, fc, B = 20_000, 39, 16, (400, 400, 400), 32775
    m = _gpu_model(rmx, kind, V, F, K, fc)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 3, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(5).random(B) > 0.7).astype(np.float32))
    ml = len(mats)

    def grads():
        out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, ml, 1)]
        m.backward_ids(t, B, ids, targets, *out)
        ctx.sync()
        return [o.numpy().copy() for o in out]

    res = {}
    try:
        for sq, bias in ((0, 1), (1, 1), (1, 0)):  # wgrad_bias 1: the bias gradient fused into the dW
            rmx.set_tuning("wgrad_sq", sq)
            rmx.set_tuning("wgrad_bias", bias)
            res[sq, bias] = grads()
    finally:
        rmx.set_tuning("wgrad_sq", None)
        rmx.set_tuning("wgrad_bias", None)
    for key in ((1, 1), (1, 0)):
        for a, b in zip(res[0, 1], res[key]):
            assert np.abs(a - b).max() <= 2e-5 * max(np.abs(a).max(), 1e-30), key
    # every getMatsSize block on its own scale (the biases: fused column sums vs colsum_kernel)
    sizes = list(m.getMatsSize())
    off = 0
    for i in range(0, len(sizes), 2):
        n = sizes[i] * sizes[i + 1]
        a, b = res[0, 1][3][off:off + n], res[1, 1][3][off:off + n]
        assert np.abs(a - b).max() <= 2e-5 * max(np.abs(a).max(), 1e-30), (i // 2, sizes[i], sizes[i + 1])
        off += n
    assert np.isfinite(res[1, 1][3]).all() and np.abs(res[1, 1][3]).max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "dcn", "pnn"])
@pytest.mark.parametrize("B", [32775, 65536])
def test_backward_wgrad_sq16_bitwise(kind, B):
    """The 16-wave 208 x 208 dW (wgrad_sq16 1, the default: waves 0 .. 12 take n tiles 0 .. 9 of their k
    tile, waves 13 .. 15 n tiles 10 .. 12 of every k tile) against the 13-wave kernel (0): every output sees
    the same chunks, the same six products in the same order and the same row slices, so every gradient
    is bit-identical, bias fused or not."""
    import rmx
    ctx = rmx.default_context()
    V, F, K, fc = 20_000, 39, 16, (400, 400, 400)
    m = _gpu_model(rmx, kind, V, F, K, fc)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(oc.gen_ids(SEED_IDS, 5, B, F, V).astype(np.int32))
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload((np.random.default_rng(7).random(B) > 0.7).astype(np.float32))
    ml = len(mats)

    def grads():
        out = [rmx.DeviceArray(ctx, n, np.float32) for n in (1, B * F, B * F * K, ml, 1)]
        m.backward_ids(t, B, ids, targets, *out)
        ctx.sync()
        return [o.numpy().copy() for o in out]

    res = {}
    try:
        for bias in (1, 0):
            rmx.set_tuning("wgrad_bias", bias)
            for v in (0, 1):
                rmx.set_tuning("wgrad_sq16", v)
                res[bias, v] = grads()
    finally:
        rmx.set_tuning("wgrad_sq16", None)
        rmx.set_tuning("wgrad_bias", None)
    for bias in (1, 0):
        for a, b in zip(res[bias, 0], res[bias, 1]):
            assert np.array_equal(a, b), bias
    assert np.isfinite(res[1, 1][3]).all() and np.abs(res[1, 1][3]).max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", GPU_KINDS)
def test_backward_host_arrays_in_place(kind):
    """L-A RecModel.backward: the caller's arrays come back holding the gradients."""
    import rmx
    B, F, K, fc = 64, 6, 8, (32, 16)
    if kind == "xdeepfm":
        K = 16  # the CIN kernel's embedding dim
    rng = np.random.default_rng(11)
    m = _gpu_model(rmx, kind, 1000, F, K, fc)
    nnz = B * F
    index = np.repeat(np.arange(B), F).astype(np.int64)
    if kind == "lr":  # irregular, unsorted COO rows (Scatter semantics)
        index = rng.integers(0, B, nnz).astype(np.int64)
    feats = rng.integers(0, 1000, nnz).astype(np.int64)
    w = rng.uniform(-0.1, 0.1, nnz).astype(np.float32)
    e = rng.uniform(-0.1, 0.1, nnz * K).astype(np.float32)
    mats = m.initMats(7) if kind != "lr" else None
    bias = np.array([0.02], np.float32)
    tg = (rng.random(B) > 0.5).astype(np.float32)
    om = _orc_model(kind, F, K, fc)
    ref = oc.backward(om, B, index, bias, w if kind != "dnn" else None, e if kind != "lr" else None, mats, tg)
    args = [B, (index, feats), bias, w if kind != "dnn" else None]
    if kind != "lr":
        args += [e, K, mats, m.getMatsSize()]
    loss = m.backward(*args, tg)
    assert abs(loss - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    assert _close(bias, ref["bias"])
    if kind != "dnn":
        assert _close(w, ref["weights"])
    if kind != "lr":
        assert _close(e, ref["embedding"]) and _close(mats, ref["mats"])


@pytest.mark.gpu
def test_backward_unsupported_raises():
    """bf16 models and DCN stacks deeper than the closed form's 8 layers are rejected loudly."""
    import rmx
    m = rmx.DeepFM(1000, 4, 16, [8])
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(m.initMats(1))
    m.setBias(0.0)
    args = (2, (np.repeat(np.arange(2), 4), np.arange(8)), np.zeros(1, np.float32), np.zeros(8, np.float32),
            np.zeros(8 * 16, np.float32), 16, m.initMats(1), m.getMatsSize(), np.ones(2, np.float32))
    with pytest.raises(rmx.RmxError):
        m.backward(*args)
    d = rmx.DCN(1000, 4, 16, 9, [8])
    d.setMats(d.initMats(1))
    d.setBias(0.0)
    with pytest.raises(rmx.RmxError):
        d.backward(2, (np.repeat(np.arange(2), 4), np.arange(8)), np.zeros(1, np.float32), np.zeros(8, np.float32),
                   np.zeros(8 * 16, np.float32), 16, d.initMats(1), d.getMatsSize(), np.ones(2, np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "dcn", "pnn", "xdeepfm"])
def test_backward_unfiltered_batch_only_ties_differ(kind):
    """The full batch, no row filtering: every row whose embedding gradient misses the element-wise
    bar must be a ReLU-tie row (a pre-activation within 1e-4 of the layer's mean magnitude, where fp32
    and fp64 may take different ReLU branches); the weight gradients meet the array-wide bar."""
    import rmx
    ctx = rmx.default_context()
    B, V, F, K, fc = 512, 20_000, 39, 16, (400, 400, 400)
    m = _gpu_model(rmx, kind, V, F, K, fc)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 777, B, F, V, ids)
    tg = (np.random.default_rng(9).random(B) > 0.7).astype(np.float32)
    targets = rmx.DeviceArray(ctx, B, np.float32)
    targets.upload(tg)
    ml = len(mats)
    g_b = rmx.DeviceArray(ctx, 1, np.float32)
    g_w = rmx.DeviceArray(ctx, B * F, np.float32)
    g_e = rmx.DeviceArray(ctx, B * F * K, np.float32)
    g_m = rmx.DeviceArray(ctx, ml, np.float32)
    loss = rmx.DeviceArray(ctx, 1, np.float32)
    m.backward_ids(t, B, ids, targets, g_b, g_w, g_e, g_m, loss)
    ctx.sync()
    wt, et = oc.gen_table(SEED_TAB, V, K)
    h_ids = ids.numpy().astype(np.int64)
    w, e = oc.gather(wt, et, 1, h_ids)
    index = np.repeat(np.arange(B), F).astype(np.int64)
    ref = oc.backward(_orc_model(kind, F, K, fc), B, index, np.array([0.01], np.float32), w, e, mats, tg)
    assert abs(loss.numpy()[0] - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    assert _close(g_b.numpy(), ref["bias"]) and _close(g_m.numpy(), ref["mats"])
    ge, re_ = g_e.numpy().reshape(B, F * K).astype(np.float64), ref["embedding"].reshape(B, F * K)
    mx = np.abs(re_).max()
    bad_rows = np.where((np.abs(ge - re_) > 1e-3 * np.maximum(np.abs(re_), 1e-3 * mx)).any(axis=1))[0]
    ties = set(range(B)) - set(_tie_free(kind, et[h_ids.reshape(B, F)].astype(np.float64), mats, fc, rel=1e-4))
    print("%s: %d rows off the element-wise bar, %d ReLU-tie rows" % (kind, len(bad_rows), len(ties)))
    assert set(bad_rows.tolist()) <= ties
