"""Device predict loop + AUC (rmx_predict_ids / rmx_auc).

The AUC reference is the Mann-Whitney statistic with ties counted 1/2 (the published definition of
the metric the examples print, example/DeepFMLocalExample.scala:44-52 -> Angel metric.AUC, which is
not in the reference tree: parity against Angel itself unpinned), in numpy below and cross-checked
with scikit-learn's roc_auc_score where it is importable.
"""
import numpy as np
import pytest

import oracle_ctypes as oc


def auc_ref(labels, scores):
    y = np.asarray(labels) > 0
    s = np.asarray(scores, np.float64)
    order = np.argsort(s, kind="stable")
    s_sorted = s[order]
    ranks = np.empty(len(s))
    i = 0
    while i < len(s):  # average ranks over ties (1-based)
        j = i
        while j + 1 < len(s) and s_sorted[j + 1] == s_sorted[i]:
            j += 1
        ranks[order[i:j + 1]] = (i + j) / 2.0 + 1.0
        i = j + 1
    P, N = int(y.sum()), int((~y).sum())
    if P == 0 or N == 0:
        return float("nan")
    return (ranks[y].sum() - P * (P + 1) / 2.0) / (P * N)


def test_auc_reference_known_answers():
    assert auc_ref([0, 0, 1, 1], [0.1, 0.2, 0.3, 0.4]) == 1.0
    assert auc_ref([1, 1, 0, 0], [0.1, 0.2, 0.3, 0.4]) == 0.0
    assert auc_ref([0, 1, 0, 1], [0.5, 0.5, 0.5, 0.5]) == 0.5
    assert auc_ref([0, 1, 1], [0.2, 0.2, 0.9]) == 0.75
    try:
        from sklearn.metrics import roc_auc_score
    except ImportError:
        return
    rng = np.random.default_rng(0)
    y = rng.random(500) < 0.3
    s = np.round(rng.random(500), 2)  # many ties
    assert abs(auc_ref(y, s) - roc_auc_score(y, s)) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("n,ties", [(1, False), (7, False), (1000, True), (1_000_000, False), (300_000, True)])
def test_device_auc(n, ties):
    import rmx
    ctx = rmx.default_context()
    rng = np.random.default_rng(n)
    y = (rng.random(n) < 0.25).astype(np.float32)
    s = rng.random(n).astype(np.float32)
    if ties:
        s = np.round(s * 50).astype(np.float32) / 50
    s = np.where(y > 0, s + 0.1, s).astype(np.float32)  # some signal
    dl, ds = rmx.DeviceArray(ctx, n, np.float32), rmx.DeviceArray(ctx, n, np.float32)
    dl.upload(y)
    ds.upload(s)
    got = rmx.auc(ctx, dl, ds)
    ref = auc_ref(y, s)
    if np.isnan(ref):
        assert np.isnan(got)
    else:
        assert abs(got - ref) < 1e-12 * max(1.0, n / 1000), (got, ref)


@pytest.mark.gpu
def test_predict_loop_matches_forward():
    import rmx
    ctx = rmx.default_context()
    V, F, K, n, B = 50_000, 39, 16, 10_000, 4096
    m = rmx.DeepFM(V, F, K, [64, 32])
    m.setMats(m.initMats(3))
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K)
    t.fill_synthetic(7)
    ids = rmx.DeviceArray(ctx, n * F, np.int32)
    rmx.gen_ids(ctx, 0x5EED2026, 0, n, F, V, ids)
    scores = rmx.DeviceArray(ctx, n, np.float32)
    m.predict_ids(t, n, ids, scores, batch=B)
    ref = rmx.DeviceArray(ctx, n, np.float32)
    for r0 in range(0, n, B):
        b = min(B, n - r0)
        m.forward_ids(t, b, ids.view(r0 * F, b * F), ref.view(r0, b))
    ctx.sync()
    assert np.array_equal(scores.numpy(), ref.numpy())
    # and against the oracle on the gathered rows
    wt, et = oc.gen_table(7, V, K)
    w, e = oc.gather(wt, et, 1, ids.numpy().astype(np.int64))
    om = oc.make_model(oc.DEEPFM, F, K, fc=(64, 32))
    p = oc.forward(om, n, np.repeat(np.arange(n), F), np.array([0.01], np.float32), w, e, m.initMats(3), 1)
    assert np.abs(scores.numpy() - p).max() < 1e-5
