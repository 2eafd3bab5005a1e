"""GPU parity of the split fp32 GEMM (csrc/k_gemm_s3.hip, k_gemm.hpp kPrecS3).

fp32 tower and CIN layers whose width pads to a multiple of 208 run on the bf16 matrix cores
through the exact 3-way bf16 split (6 products).  Each case runs the same model on the same
inputs with rmx_set_tuning("f32_split", 1) and ("f32_split", 0) (the f32 MFMA engine) and checks
both against the fp64 oracle at the north-star bar |p_gpu - p_oracle| <= 1e-5, plus that the
split path is no less accurate than the f32 MFMA path (its error stays within 2x + 1e-7 of it).
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75

KINDS = {
    "deepfm": (oc.DEEPFM, dict(fc=(400, 400, 400))),
    "dnn": (oc.DNN, dict(fc=(400, 400))),
    "xdeepfm": (oc.XDEEPFM, dict(fc=(400, 400), cin=(200, 200))),
    "dcn": (oc.DCN, dict(fc=(400, 400), cross_depth=3)),
    "pnn": (oc.PNN, dict(fc=(400, 400))),
}


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    for k, v in {"f32_split": 1, "s3_tower": 1, "s3_dense": 5, "s3_cin": None, "fm_fuse": 1, "fo_fuse": 2, "fm_y1": 2, "tower_variant": None,
                 "cin_map": 1}.items():
        rmx.set_tuning(k, v)


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


def _case(ctx, kind, B, V=50000, row0=0):
    m = _model(kind, V)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, row0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)

    def run():
        m.forward_ids(table, B, ids_dev, out)
        ctx.sync()
        return out.numpy().copy()

    t, kw = KINDS[kind]
    wt, et = oc.gen_table(SEED_TAB, V, K)
    ids = oc.gen_ids(SEED_IDS, row0, B, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    ref64 = oc.forward(oc.make_model(t, F, K, **kw), B, index, np.array([0.01], np.float32), w, e, mats, 1)
    return run, ref64


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("B", [1, 129, 517])
def test_split_matches_oracle_and_f32_engine(ctx, kind, B):
    run, ref64 = _case(ctx, kind, B)
    rmx.set_tuning("f32_split", 0)
    p_f32 = run()
    rmx.set_tuning("f32_split", 1)
    p_s3 = run()
    e_f32 = float(np.abs(p_f32 - ref64).max())
    e_s3 = float(np.abs(p_s3 - ref64).max())
    print("%s B=%d max|p - p_fp64|: f32 MFMA %.3g, split %.3g" % (kind, B, e_f32, e_s3))
    assert e_f32 <= TOL
    assert e_s3 <= TOL
    assert e_s3 <= 2 * e_f32 + 1e-7
    # deterministic: a second launch gives identical bits
    assert np.array_equal(run(), p_s3)


@pytest.mark.parametrize("knob,values", [("s3_tower", [0, 1, 2, 3, 4]), ("s3_cin", [0, 1, 2, 3, 4])])
def test_split_variants(ctx, knob, values):
    kind = "xdeepfm" if knob == "s3_cin" else "dnn"
    run, ref64 = _case(ctx, kind, 300, row0=999)
    for v in values:
        rmx.set_tuning(knob, v)
        err = float(np.abs(run() - ref64).max())
        print("%s=%d: max|p - p_fp64| = %.3g" % (knob, v, err))
        assert err <= TOL


def test_dense_variants_bitwise(ctx):
    """The dense-layer tiles (s3_dense 5: 16 waves of 16 rows; 4: 4-wave blocks of 32-row waves, two
    per CU, single-buffered; 1: the staggered 8-wave tile) accumulate each output element in the same
    K order: identical bits, at a batch large enough (M >= 32,513) for these tiles; head rows against
    the fp64 oracle."""
    B, V = 40000, 50000
    m = _model("dnn", V)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = []
    for v in (1, 4, 5):
        rmx.set_tuning("s3_dense", v)
        m.forward_ids(table, B, ids_dev, out)
        ctx.sync()
        res.append(out.numpy().copy())
    assert np.array_equal(res[0], res[1])
    assert np.array_equal(res[0], res[2])
    wt, et = oc.gen_table(SEED_TAB, V, K)
    n = 512
    ids = oc.gen_ids(SEED_IDS, 0, n, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(n, dtype=np.int64), F)
    ref = oc.forward(oc.make_model(oc.DNN, F, K, fc=(400, 400)), n, index, np.array([0.01], np.float32), w, e, mats, 1)
    assert np.abs(res[1][:n] - ref).max() <= TOL


def test_split_headline_deepfm_full_batch(ctx):
    """configs[1] at B = 65,536 (the bench batch), split on: oracle on slices + determinism."""
    B, V = 65536, 1_000_000
    m = rmx.DeepFM(V, F, K, [400, 400, 400])
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    got = out.numpy().copy()
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = oc.make_model(oc.DEEPFM, F, K, fc=(400, 400, 400))
    for r0, n in ((0, 1024), (B - 1024, 1024)):
        ids = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, ids)
        index = np.repeat(np.arange(n, dtype=np.int64), F)
        ref = oc.forward(om, n, index, np.array([0.01], np.float32), w, e, mats, 1)
        assert np.abs(got[r0:r0 + n] - ref).max() <= TOL
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    assert np.array_equal(out.numpy(), got)


def test_split_headline_xdeepfm_full_batch(ctx):
    """configs[2] at its bench batch (CIN 200,200,200 + fcDims 400^3, B = 16,384, V = 1M), split on:
    the fp64 oracle on head and tail slices (CINEncoder.scala:36-58, XDeepFM.scala:62-86) and
    bitwise determinism across launches."""
    B, V = 16384, 1_000_000
    m = rmx.XDeepFM(V, F, K, [400, 400, 400], [200, 200, 200])
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    got = out.numpy().copy()
    wt, et = oc.gen_table(SEED_TAB, V, K)
    om = oc.make_model(oc.XDEEPFM, F, K, fc=(400, 400, 400), cin=(200, 200, 200))
    for r0, n in ((0, 96), (B // 2 - 17, 64), (B - 96, 96)):
        ids = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, ids)
        index = np.repeat(np.arange(n, dtype=np.int64), F)
        ref = oc.forward(om, n, index, np.array([0.01], np.float32), w, e, mats, 1, 16)
        err = float(np.abs(got[r0:r0 + n] - ref).max())
        print("xDeepFM B=%d rows [%d, %d): max|p - p_fp64| = %.3g" % (B, r0, r0 + n, err))
        assert err <= TOL
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    assert np.array_equal(out.numpy(), got)


@pytest.mark.parametrize("Fm,cin", [(39, (200, 196, 208)), (24, (200, 200)), (17, (208,)), (40, (200,)),
                                    (39, (150, 200)), (13, (200, 200))])
@pytest.mark.parametrize("B", [1, 300])
def test_cin_chunk_map_matches_oracle_and_plain_order(ctx, Fm, cin, B):
    """The split CIN's K order (k_gemm.hip cin_chunk_map, knob cin_map, packed at setMats): layer 1 on
    the h <= f half of its symmetric z = x0 (x) x0 with folded weights C[f,h] + C[h,f], and an h-chunk
    with <= 8 live maps (H_prev = 200, 196; F = 24, 40, 39 in layer 1) carrying two fields.  Same
    bilinear forms (CINEncoder.scala:152-155), different fp32 rounding: both orders against the fp64
    oracle at the north-star bar, and against each other."""
    V = 50000
    wt, et = oc.gen_table(SEED_TAB, V, K)
    ids = oc.gen_ids(SEED_IDS, 7, B, Fm, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), Fm)
    res = {}
    for on in (1, 0):
        rmx.set_tuning("cin_map", on)
        m = rmx.XDeepFM(V, Fm, K, [400, 400], list(cin))
        mats = m.initMats(SEED_MATS)
        m.setMats(mats)
        m.setBias(0.01)
        table = rmx.EmbeddingTable(ctx, V, K)
        table.fill_synthetic(SEED_TAB)
        ids_dev = rmx.DeviceArray(ctx, B * Fm, np.int32)
        rmx.gen_ids(ctx, SEED_IDS, 7, B, Fm, V, ids_dev)
        out = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(table, B, ids_dev, out)
        ctx.sync()
        res[on] = out.numpy().copy()
    ref = oc.forward(oc.make_model(oc.XDEEPFM, Fm, K, fc=(400, 400), cin=cin), B, index, np.array([0.01], np.float32),
                     w, e, mats, 1)
    e_map, e_plain = float(np.abs(res[1] - ref).max()), float(np.abs(res[0] - ref).max())
    print("F=%d cin=%s B=%d max|p - p_fp64|: map %.3g, plain %.3g" % (Fm, cin, B, e_map, e_plain))
    assert e_map <= TOL and e_plain <= TOL
    assert e_map <= 2 * e_plain + 1e-7


def test_split_host_arrays_path(ctx):
    """L-A (RecModel.forward host arrays, implicit ids) runs the split GEMM too."""
    B, V = 200, 5000
    m = _model("deepfm", V)
    mats = m.initMats(SEED_MATS)
    ids = oc.gen_ids(SEED_IDS, 3, B, F, V).astype(np.int64)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    got = m.forward(B, rmx.CooLongFloatMatrix(index, ids), bias, w, e, K, mats, m.getMatsSize())
    ref = oc.forward(oc.make_model(oc.DEEPFM, F, K, fc=(400, 400, 400)), B, index, bias, w, e, mats, 1)
    assert np.abs(np.asarray(got) - ref).max() <= TOL


@pytest.mark.parametrize("y1_in_gemm", [0, 1, 2])
@pytest.mark.parametrize("B", [1, 300, 4099, 40000])  # 40000: BM = 256 tiles (id ring), ragged tail
def test_fused_fm_bitwise_equals_encoder(ctx, B, y1_in_gemm):
    """DeepFM's FM (and, with fm_y1 = 1, the first order) computed inside tower layer 1 (fm_fuse, the
    default) gives the same bits as the standalone encoder kernel (itself bit-exact to the oracle)."""
    run, ref64 = _case(ctx, "deepfm", B)
    rmx.set_tuning("fm_y1", y1_in_gemm)
    rmx.set_tuning("fm_fuse", 0)
    p_enc = run()
    rmx.set_tuning("fm_fuse", 1)
    p_fused = run()
    assert np.array_equal(p_fused, p_enc)
    assert np.abs(p_fused - ref64).max() <= TOL


@pytest.mark.parametrize("kind,bf16", [("xdeepfm", False), ("dcn", False), ("dcn", True)])
@pytest.mark.parametrize("B", [300, 16384, 65536, 65537])
@pytest.mark.parametrize("ring", [True, False])
def test_fused_first_order_bitwise(ctx, kind, bf16, B, ring):
    """xDeepFM / DCN: the first order (Scatter) computed in tower layer 1 gives the same bits as the
    standalone first-order kernel, fp32 and bf16 tables -- summed from the ring's weight DMAs
    (ring=True: the default tiles) or gathered in the epilogue (ring=False: register-staged tiles)."""
    V = 50000
    m = _model(kind, V)
    if bf16:
        m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16 if bf16 else rmx.DTYPE_F32)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    if not ring:
        rmx.set_tuning("tower_variant" if bf16 else "s3_tower", 0 if bf16 else 2)
    res = []
    for fuse in (0, 1):
        rmx.set_tuning("fo_fuse", fuse)
        m.forward_ids(table, B, ids_dev, out)
        ctx.sync()
        res.append(out.numpy().copy())
    assert np.array_equal(res[0], res[1])
