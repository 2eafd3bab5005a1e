"""Reentrant entry points (SURVEY.md §8b "Threading"; include/rmx.h rmx::ModelUse).

The reference builds fresh BigDL modules on every call (e.g. yr/model/deepfm/DeepFM.scala:63-76),
so Spark local[N] tasks may call RecModel.forward / backward concurrently in one JVM.  librmx's
models own one workspace; every entry point takes the model's lock and, when the caller's stream
differs from the last call's, orders the two on the device.  These tests hit ONE model from several
threads -- each with its own stream (L-B) or through the synchronous host-array API (L-A) -- and
require every result to equal the serial one bit for bit.
"""
import threading

import numpy as np
import pytest

F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75


def _threads(n, fn):
    errs, res = [], [None] * n

    def run(i):
        try:
            res[i] = fn(i)
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs.append((i, e))

    ts = [threading.Thread(target=run, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert not any(t.is_alive() for t in ts), "a thread hung"
    if errs:
        raise AssertionError("thread %d failed: %r" % errs[0])
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "xdeepfm", "pnn"])
def test_forward_ids_many_streams_one_model(kind):
    import rmx
    V, B, T, reps = 200_003, 3000, 4, 6
    ctx0 = rmx.default_context()
    table = rmx.EmbeddingTable(ctx0, V, K)
    table.fill_synthetic(SEED_TAB)
    m = {"deepfm": lambda: rmx.DeepFM(V, F, K, [400, 400, 400], ctx=ctx0),
         "xdeepfm": lambda: rmx.XDeepFM(V, F, K, [64, 32], [48, 32], ctx=ctx0),
         "pnn": lambda: rmx.PNN(V, F, K, [400, 64], ctx=ctx0)}[kind]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    # serial reference, one batch per (thread, rep)
    ids = rmx.DeviceArray(ctx0, T * reps * B * F, np.int32)
    rmx.gen_ids(ctx0, SEED_IDS, 0, T * reps * B, F, V, ids)
    ref = rmx.DeviceArray(ctx0, T * reps * B, np.float32)
    for j in range(T * reps):
        m.forward_ids(table, B, ids.view(j * B * F, B * F), ref.view(j * B, B))
    ctx0.sync()
    ref_h = ref.numpy()

    def worker(t):
        ctx = rmx.Context(0)  # its own stream
        out = rmx.DeviceArray(ctx, reps * B, np.float32)
        for r in range(reps):
            j = t * reps + r
            m.forward_ids(table, B, ids.view(j * B * F, B * F), out.view(r * B, B), ctx.stream)
        ctx.sync()
        return out.numpy()

    got = _threads(T, worker)
    for t in range(T):
        assert np.array_equal(got[t], ref_h[t * reps * B:(t + 1) * reps * B]), t


@pytest.mark.gpu
def test_host_array_forward_and_backward_concurrent():
    """Spark local[N] analogue: N threads call RecModel.forward / backward (host arrays) on one
    model with different batches; each result equals the serial call's."""
    import rmx
    rng = np.random.default_rng(5)
    m = rmx.DeepFM(10_000, F, K, [64, 32])
    mats = m.initMats(SEED_MATS)
    sizes = m.getMatsSize()
    T, B = 4, 257
    batches = []
    for t in range(T):
        index = np.repeat(np.arange(B, dtype=np.int64), F)
        feats = rng.integers(0, 10_000, B * F).astype(np.int64)
        w = rng.uniform(-0.05, 0.05, B * F).astype(np.float32)
        e = rng.uniform(-0.05, 0.05, B * F * K).astype(np.float32)
        y = (rng.random(B) < 0.3).astype(np.float32)
        batches.append((index, feats, w, e, y))

    def fwd(t):
        index, feats, w, e, _ = batches[t]
        return m.forward(B, (index, feats), np.array([0.01], np.float32), w, e, K, mats, sizes)

    def bwd(t):
        index, feats, w, e, y = batches[t]
        b, w2, e2, m2 = np.array([0.01], np.float32), w.copy(), e.copy(), mats.copy()
        loss = m.backward(B, (index, feats), b, w2, e2, K, m2, sizes, y)
        return loss, b, w2, e2, m2

    ref_f = [fwd(t) for t in range(T)]
    ref_b = [bwd(t) for t in range(T)]
    for _ in range(2):
        got_f = _threads(T, fwd)
        got_b = _threads(T, bwd)
        for t in range(T):
            assert np.array_equal(got_f[t], ref_f[t])
            assert got_b[t][0] == ref_b[t][0]
            for a, b in zip(got_b[t][1:], ref_b[t][1:]):
                assert np.array_equal(a, b)


@pytest.mark.gpu
def test_predict_and_forward_interleaved_streams():
    """predict_ids on one stream while another thread runs forward_ids on a second stream."""
    import rmx
    V, B = 100_003, 2048
    ctx0 = rmx.default_context()
    table = rmx.EmbeddingTable(ctx0, V, K)
    table.fill_synthetic(SEED_TAB)
    m = rmx.DCN(V, F, K, 3, [400, 400, 400], ctx=ctx0)
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    n = 8 * B
    ids = rmx.DeviceArray(ctx0, n * F, np.int32)
    rmx.gen_ids(ctx0, SEED_IDS, 0, n, F, V, ids)
    ref = rmx.DeviceArray(ctx0, n, np.float32)
    m.predict_ids(table, n, ids, ref, batch=B)
    ctx0.sync()
    ref_h = ref.numpy()

    def worker(t):
        ctx = rmx.Context(0)
        out = rmx.DeviceArray(ctx, n, np.float32)
        for _ in range(3):
            if t == 0:
                m.predict_ids(table, n, ids, out, batch=B, stream=ctx.stream)
            else:
                for j in range(n // B):
                    m.forward_ids(table, B, ids.view(j * B * F, B * F), out.view(j * B, B), ctx.stream)
        ctx.sync()
        return out.numpy()

    for got in _threads(3, worker):
        assert np.array_equal(got, ref_h)
