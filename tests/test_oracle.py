"""CPU checks of the oracle (oracle/rmx_oracle.c): it is the checker of every GPU parity test, so
it is pinned here first.

The reference (Scala/BigDL/Angel) cannot run in this container and ships no
tests or golden vectors, so parity at the BigDL boundary is UNPINNED.  The oracle is
pinned instead by
  1. an independent, structurally different numpy (fp64) re-expression of the BigDL module graphs
     (tests/ref_numpy.py) on every model kind;
  2. known-answer identities of each encoder (FM pair identity, one-hot CIN, DCN closed form,
     PNN pair order, Scatter ascending-n order);
  3. the committed fixtures under tests/golden/ (see test_golden.py).
Paths are relative to /root/reference/src/main/scala/io/yaochi/recommendation/.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import ref_numpy as rn

SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75

KINDS = {
    "lr": (oc.LR, {}),
    "deepfm": (oc.DEEPFM, dict(fc=(32, 24))),
    "dnn": (oc.DNN, dict(fc=(20,))),
    "xdeepfm1": (oc.XDEEPFM, dict(fc=(16, 8), cin=(12,))),
    "xdeepfm3": (oc.XDEEPFM, dict(fc=(16, 8), cin=(6, 10, 4))),
    "dcn": (oc.DCN, dict(fc=(16, 8), cross_depth=3)),
    "pnn": (oc.PNN, dict(fc=(12, 8))),
}


def _inputs(B, F, k, V, seed=SEED_IDS):
    ids = oc.gen_ids(seed, 0, B, F, V).astype(np.int64)
    wt, et = oc.gen_table(SEED_TAB, V, k)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    return ids, w, e, index


@pytest.mark.parametrize("kind", list(KINDS))
@pytest.mark.parametrize("F,k", [(3, 4), (7, 16), (39, 16)])
def test_oracle_matches_numpy_restatement(kind, F, k):
    t, kw = KINDS[kind]
    B, V = 13, 40 * F
    m = oc.make_model(t, F, k, **kw)
    ids, w, e, index = _inputs(B, F, k, V)
    mats = oc.init_mats(m, SEED_MATS) if t != oc.LR else None
    bias = np.array([0.03], np.float32)
    ref_kind = "xdeepfm" if kind.startswith("xdeepfm") else kind
    ref = rn.forward(ref_kind, B, F, k, index, bias, w, e if t != oc.LR else None, mats,
                     fc=kw.get("fc", ()), cin=kw.get("cin", ()), cross_depth=kw.get("cross_depth", 0))
    got64 = oc.forward(m, B, index, bias, w, e if t != oc.LR else None, mats, precision=1)
    got32 = oc.forward(m, B, index, bias, w, e if t != oc.LR else None, mats, precision=0)
    assert np.abs(got64 - ref).max() <= 1e-7, np.abs(got64 - ref).max()
    assert np.abs(got32 - ref).max() <= 1e-5, np.abs(got32 - ref).max()


def test_fm_pair_identity():
    """0.5 * (1/k) sum_j[(sum_f e)^2 - sum_f e^2] == (1/k) sum_j sum_{f<g} e_f e_g
    (model/encoder/SecondOrderEncoder.scala:19-34: note the Mean over k, not a Sum)."""
    rng = np.random.default_rng(0)
    B, F, k = 9, 11, 8
    e = rng.uniform(-1, 1, (B, F, k)).astype(np.float32)
    got = oc.fm(B, F, k, e)
    E = e.astype(np.float64)
    ref = np.zeros(B)
    for f in range(F):
        for g in range(f + 1, F):
            ref += (E[:, f, :] * E[:, g, :]).sum(axis=1)
    ref /= k
    assert np.abs(got - ref).max() <= 1e-5


def test_first_order_scatter_order_and_require():
    """bnn/Scatter.scala:17-36: out[index[i]] += w[i] in ascending i; require(index < batchSize)."""
    index = np.array([2, 0, 2, 1, 2], np.int64)
    w = np.array([1e8, 1.0, -1e8, 2.0, 1.0], np.float32)
    y = oc.first_order(3, index, w)
    # ascending order: ((0 + 1e8) + -1e8) + 1 == 1 in fp32; any other order gives 0 or 1
    assert y.tolist() == [1.0, 2.0, 1.0]
    with pytest.raises(IndexError):
        oc.first_order(2, index, w)


def test_cin_one_hot_known_answer():
    """A 1-layer CIN whose C_1 selects one (f, h) product equals that x0[f]*x0[h] summed over k
    (model/xdeepfm/CINEncoder.scala:150-165); DNN and first order zeroed out."""
    F, k, H, B = 4, 3, 2, 5
    m = oc.make_model(oc.XDEEPFM, F, k, fc=(2,), cin=(H,))
    sizes = oc.mats_sizes(m)
    mats = np.zeros(oc.mats_len(m), np.float32)
    # layout: DNN W(2 x 12), b(2), C_1 (H x F*F), c_1 (H), W_out (H + 2)
    off = 2 * F * k + 2
    C = np.zeros((H, F * F), np.float32)
    C[0, 1 * F + 2] = 1.0  # z[f=1, h=2]
    C[1, 3 * F + 3] = 1.0  # z[f=3, h=3]
    mats[off:off + H * F * F] = C.ravel()
    off += H * F * F + H
    mats[off:off + H] = [1.0, 10.0]
    assert off + H + 2 == len(mats) and sizes[-2:].tolist() == [H + 2, 1]
    rng = np.random.default_rng(3)
    e = rng.uniform(0, 1, (B, F, k)).astype(np.float32)  # positive: ReLU is the identity
    w = np.zeros(B * F, np.float32)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    p = oc.forward(m, B, index, np.zeros(1, np.float32), w, e, mats, precision=1)
    E = e.astype(np.float64)
    y = (E[:, 1, :] * E[:, 2, :]).sum(1) + 10 * (E[:, 3, :] ** 2).sum(1)
    assert np.abs(p - 1 / (1 + np.exp(-y))).max() <= 1e-6


def test_dcn_closed_form():
    """One cross layer with w = 0: x_1 = x0 + beta (model/dcn/CrossEncoder.scala:44-49); two layers
    with w = e_0: x_{l+1} = x0 * x_l[0] + x_l + beta."""
    F, k, B = 3, 2, 4
    D = F * k
    m = oc.make_model(oc.DCN, F, k, fc=(2,), cross_depth=2)
    mats = np.zeros(oc.mats_len(m), np.float32)
    mats[0] = 1.0            # w_1 = e_0
    mats[D + 0] = 1.0        # w_2 = e_0
    mats[2 * D:2 * D + 2] = [0.5, -0.25]  # beta_1, beta_2
    wo_off = 2 * D + 2 + D * 2 + 2
    mats[wo_off:wo_off + D] = 1.0  # y = sum(x_L) (DNN slice of W_out left 0)
    rng = np.random.default_rng(4)
    e = rng.uniform(-1, 1, (B, D)).astype(np.float32)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    p = oc.forward(m, B, index, np.zeros(1, np.float32), np.zeros(B * F, np.float32), e, mats, 1)
    x0 = e.astype(np.float64)
    x1 = x0 * x0[:, :1] + x0 + 0.5
    x2 = x0 * x1[:, :1] + x1 - 0.25
    y = x2.sum(1)
    assert np.abs(p - 1 / (1 + np.exp(-y))).max() <= 1e-6


def test_pnn_pair_order():
    """Pairs (i < j) in lexicographic order (model/pnn/ProductEncoder.scala:110-120): put weight 1 on
    pair p only and check which product comes out."""
    F, k, B, D1 = 4, 2, 3, 1
    P = F * (F - 1) // 2
    m = oc.make_model(oc.PNN, F, k, fc=(D1,))
    rng = np.random.default_rng(5)
    e = rng.uniform(0.1, 1, (B, F, k)).astype(np.float32)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    pairs = [(i, j) for i in range(F) for j in range(i + 1, F)]
    for p, (i, j) in enumerate(pairs):
        mats = np.zeros(oc.mats_len(m), np.float32)
        off = D1 * F * k
        mats[off + p] = 1.0                     # Wp[0, p]
        tail = off + P * D1 + 1                 # output Linear(D1 -> 1): W, b
        mats[tail] = 1.0
        prob = oc.forward(m, B, index, np.zeros(1, np.float32), np.zeros(B * F, np.float32), e, mats, 1)
        E = e.astype(np.float64)
        y = (E[:, i, :] * E[:, j, :]).sum(1)
        assert np.abs(prob - 1 / (1 + np.exp(-y))).max() <= 1e-6, (p, i, j)


def test_mats_sizes_match_reference_formulas():
    """getMatsSize of each model (DeepFM.scala:15-20, XDeepFM.scala:15-28, DCN.scala:15-32,
    PNN.scala:15-25, LR.scala:15) at the BASELINE configs."""
    F, k = 39, 16
    D = F * k
    m = oc.make_model(oc.DEEPFM, F, k, fc=(400, 400, 400))
    assert oc.mats_sizes(m).tolist() == [D, 400, 400, 1, 400, 400, 400, 1, 400, 400, 400, 1, 400, 1, 1, 1]
    assert oc.mats_len(m) == 571_201
    m = oc.make_model(oc.XDEEPFM, F, k, fc=(400, 400, 400), cin=(200, 200, 200))
    assert oc.mats_len(m) == 3_996_600
    m = oc.make_model(oc.XDEEPFM, F, k, fc=(400, 400, 400), cin=(200,))
    assert oc.mats_len(m) == 875_800
    m = oc.make_model(oc.DCN, F, k, fc=(400, 400, 400), cross_depth=3)
    assert oc.mats_len(m) == 573_699
    m = oc.make_model(oc.PNN, F, k, fc=(400, 400, 400))
    assert oc.mats_len(m) == 867_202
    assert oc.mats_len(oc.make_model(oc.LR)) == 0


def test_gather_layouts_bit_exact():
    """makeEmbeddings reads Emb_j[id] from a k x V PS layout (ParRecModel.scala:300-306)."""
    V, k = 101, 5
    wt, et = oc.gen_table(9, V, k)
    feats = np.array([0, 100, 7, 7, 55], np.int64)
    w1, e1 = oc.gather(wt, et, 1, feats)
    w0, e0 = oc.gather(wt, np.ascontiguousarray(et.T), 0, feats)
    assert np.array_equal(w0, w1) and np.array_equal(e0, e1)
    assert np.array_equal(e1.reshape(-1, k), et[feats])
    with pytest.raises(IndexError):
        oc.gather(wt, et, 1, np.array([V], np.int64))


def test_oracle_error_modes():
    m = oc.make_model(oc.DEEPFM, 3, 4, fc=(4,))
    mats = oc.init_mats(m, 1)
    index = np.repeat(np.arange(2, dtype=np.int64), 3)
    w = np.zeros(6, np.float32)
    e = np.zeros(24, np.float32)
    with pytest.raises(ValueError):  # Reshape(B, F, k) mismatch
        oc.forward(m, 3, index, np.zeros(1, np.float32), w, e, mats)
    bad = index.copy()
    bad[0] = 5
    with pytest.raises(ValueError):  # Scatter require
        oc.forward(m, 2, bad, np.zeros(1, np.float32), w, e, mats)


def test_generators_are_counter_based():
    """ids / table rows depend only on (seed, position): any slice regenerates identically."""
    a = oc.gen_ids(SEED_IDS, 0, 50, 39, 1_000_000)
    b = oc.gen_ids(SEED_IDS, 20, 10, 39, 1_000_000)
    assert np.array_equal(a[20 * 39:30 * 39], b)
    per = 1_000_000 // 39
    f = np.tile(np.arange(39), 50)
    assert ((a >= f * per) & (a < (f + 1) * per)).all()
    w, e = oc.gen_table(SEED_TAB, 1000, 16)
    w2, e2 = oc.gen_table(SEED_TAB, 1000, 16, id0=400, nrows=17)
    assert np.array_equal(w[400:417], w2) and np.array_equal(e[400:417], e2)
    assert np.abs(e).max() <= 0.05 and np.abs(w).max() <= 0.05
