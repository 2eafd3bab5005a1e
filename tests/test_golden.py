"""Golden fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py).

Each fixture holds the reference's RecModel.forward inputs (RecModel.scala:37-63: COO row index,
gathered weights / embeddings, bias, mats, matSizes) and the expected outputs: first order y1
(Scatter), FM y2, fp32 / fp64 oracle probabilities.  They were cross-checked against the numpy
re-expression when written.  The CPU tests pin the oracle to them; the GPU tests hold librmx to
them (|p - p_fp32| <= 1e-5 and |p - p_fp64| <= 1e-5, BASELINE.json north_star tolerance).
Parity at the BigDL boundary stays "unpinned": no reference vector exists.
"""
import glob
import os

import numpy as np
import pytest

import oracle_ctypes as oc

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MODEL_FILES = sorted(f for f in glob.glob(os.path.join(HERE, "*.npz")) if "gather" not in f)
TOL = 1e-5


def load(path):
    return dict(np.load(path, allow_pickle=False))


def oracle_model(g):
    t, F, k, depth = (int(x) for x in g["model"])
    return oc.make_model(t, F, k, fc=tuple(int(x) for x in g["fc"]), cin=tuple(int(x) for x in g["cin"]),
                         cross_depth=depth)


def test_fixture_set_complete():
    names = {os.path.basename(f)[:-4] for f in MODEL_FILES}
    for kind in ("lr", "deepfm", "dnn", "xdeepfm1", "xdeepfm3", "dcn", "pnn"):
        assert any(n.startswith(kind) for n in names), kind


@pytest.mark.parametrize("path", MODEL_FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden(path):
    g = load(path)
    m = oracle_model(g)
    B = int(g["batch_size"])
    is_lr = int(g["model"][0]) == oc.LR
    assert np.array_equal(oc.first_order(B, g["index"], g["weights"]), g["y1"])
    if not is_lr:
        F, k = int(g["model"][1]), int(g["model"][2])
        assert np.array_equal(oc.fm(B, F, k, g["embedding"]), g["y2"])
        assert np.array_equal(oc.mats_sizes(m), g["mat_sizes"])
    emb = None if is_lr else g["embedding"]
    mats = None if is_lr else g["mats"]
    p32 = oc.forward(m, B, g["index"], g["bias"], g["weights"], emb, mats, 0)
    p64 = oc.forward(m, B, g["index"], g["bias"], g["weights"], emb, mats, 1)
    assert np.abs(p32 - g["p32"]).max() <= 1e-7
    assert np.abs(p64 - g["p64"]).max() <= 1e-7
    assert np.abs(g["p32"] - g["p64"]).max() <= TOL


def test_oracle_gather_golden():
    g = load(os.path.join(HERE, "gather_kmajor.npz"))
    w, e = oc.gather(g["w_table"], g["emb_table_kmajor"], 0, g["feats"])
    assert np.array_equal(w, g["w"]) and np.array_equal(e, g["e"])


# ------------------------------------------------------------------ GPU ----
def _rmx_model(g):
    import rmx
    t, F, k, depth = (int(x) for x in g["model"])
    fc = [int(x) for x in g["fc"]]
    V = int(g["num_rows"])
    if t == oc.LR:
        return rmx.LR(V, F)
    if t == oc.DEEPFM:
        return rmx.DeepFM(V, F, k, fc)
    if t == oc.DNN:
        return rmx.DNN(V, F, k, fc)
    if t == oc.XDEEPFM:
        return rmx.XDeepFM(V, F, k, fc, [int(x) for x in g["cin"]])
    if t == oc.DCN:
        return rmx.DCN(V, F, k, depth, fc)
    return rmx.PNN(V, F, k, fc)


@pytest.mark.gpu
@pytest.mark.parametrize("path", MODEL_FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_librmx_reproduces_golden(path):
    """RecModel.forward drop-in (L-A, host arrays) through librmx.so on the GPU."""
    g = load(path)
    m = _rmx_model(g)
    B = int(g["batch_size"])
    if int(g["model"][0]) == oc.LR:
        got = m.forward(B, (g["index"], g["ids"]), g["bias"], g["weights"])
    else:
        got = m.forward(B, (g["index"], g["ids"]), g["bias"], g["weights"], g["embedding"], int(g["model"][2]),
                        g["mats"], g["mat_sizes"])
    assert np.abs(got - g["p32"]).max() <= TOL
    assert np.abs(got - g["p64"]).max() <= TOL


@pytest.mark.gpu
def test_librmx_gather_golden_kmajor():
    """makeWeights / makeEmbeddings from the reference PS layout: bit-exact on the device."""
    import rmx
    g = load(os.path.join(HERE, "gather_kmajor.npz"))
    ctx = rmx.default_context()
    k, V = g["emb_table_kmajor"].shape
    t = rmx.EmbeddingTable(ctx, V, k)
    t.upload(g["w_table"], g["emb_table_kmajor"], layout=rmx.LAYOUT_K_MAJOR)
    ids = rmx.DeviceArray.from_numpy(ctx, g["feats"].astype(np.int32))
    n = len(g["feats"])
    w = rmx.DeviceArray(ctx, n, np.float32)
    e = rmx.DeviceArray(ctx, n * k, np.float32)
    t.gather(ids, n, w, e)
    ctx.sync()
    assert np.array_equal(w.numpy(), g["w"]) and np.array_equal(e.numpy(), g["e"])
