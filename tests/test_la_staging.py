"""L-A host arrays through the pinned staging buffer (round 6, csrc/models.hip h2d_staged): rmx_forward and
rmx_backward with arrays >= 4 MiB copy them into a pinned buffer on several host threads, chunk by chunk beside
the chunks' DMAs (knob la_pin_threads; 0 = the runtime's pageable copy).  The device sees the same bytes, so the
results are bitwise those of the plain path, and the oracle bar holds (RecModel.scala:37-48, :65-115)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

F, K, V = 39, 16, 50_000


@pytest.fixture(autouse=True)
def _restore():
    yield
    rmx.set_tuning("la_pin_threads", None)


def _batch(B, seed=3):
    ids = oc.gen_ids(seed, 0, B, F, V).astype(np.int64)
    wt, et = oc.gen_table(5, V, K)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    return index, ids, np.ascontiguousarray(w, np.float32), np.ascontiguousarray(e, np.float32)


@pytest.mark.parametrize("B", [1000, 4096, 17_000])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_la_forward_pinned_staging_bitwise(B, threads):
    m = rmx.DeepFM(V, F, K, [400, 400, 400])
    mats = m.initMats(11)
    index, ids, w, e = _batch(B)
    args = (B, (index, ids), np.array([0.01], np.float32), w, e, K, mats, m.getMatsSize())
    rmx.set_tuning("la_pin_threads", 0)
    ref = m.forward(*args)
    rmx.set_tuning("la_pin_threads", threads)
    got = m.forward(*args)
    got2 = m.forward(*args)  # (the buffer reused by the next call)
    assert np.array_equal(got, ref) and np.array_equal(got2, ref)
    om = oc.make_model(oc.DEEPFM, F, K, fc=(400, 400, 400))
    n = min(B, 256)
    p64 = oc.forward(om, n, index[:n * F], np.array([0.01], np.float32), w[:n * F], e[:n * F], mats, 1)
    assert float(np.abs(got[:n] - p64).max()) <= 1e-5


def test_la_backward_pinned_staging_bitwise():
    B = 4096
    m = rmx.DeepFM(V, F, K, [64, 32])
    mats0 = m.initMats(13)
    index, ids, w0, e0 = _batch(B, seed=9)
    tg = (np.arange(B) % 4 == 0).astype(np.float32)
    res = []
    for thr in (0, 8):
        rmx.set_tuning("la_pin_threads", thr)
        b, w, e, mats = np.array([0.02], np.float32), w0.copy(), e0.copy(), mats0.copy()
        loss = m.backward(B, (index, ids), b, w, e, K, mats, m.getMatsSize(), tg)
        res.append((loss, b, w, e, mats))
    for a, c in zip(res[0], res[1]):
        assert np.array_equal(np.asarray(a), np.asarray(c))
