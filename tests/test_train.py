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
