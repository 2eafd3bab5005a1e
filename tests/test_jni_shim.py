"""The JNI shim (recommendation-models_amd/jni/rmx_jni.c) driven as Scala would drive it.

There is no JDK here or on the GPU box, so the shim cannot be built against a JVM.  tests/jni_harness
compiles it against a declaration subset of <jni.h> (same type / function names) and links
fake_jni.c, an in-process stand-in for the JVM's array and exception functions.  Calling the
natives through it checks the shim's own logic: argument plumbing, device staging of int[] ids,
in-place gradient write-back (release mode 0) vs read-only inputs (JNI_ABORT), and the
exception types of the reference's failure modes -- against librmx's C ABI called directly.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "jni_harness")
LIB = os.path.join(HARNESS, "libfakejni.so")
F, K = 39, 16
SEED_TAB, SEED_MATS, SEED_IDS = 0x7AB1E, 0x3A75, 0x5EED2026
JNI_ABORT = 2
NATIVES = ["createContext", "destroyContext", "createModel", "destroyModel", "getMatsSize", "forward0", "backward0",
           "setMats", "setBias", "setPrecision", "createTable", "destroyTable", "uploadTable", "fillTableSynthetic",
           "forwardIds", "predictIds", "backwardIds", "auc", "commUniqueId", "createShard", "destroyShard",
           "fillShardSynthetic", "setShardOwnerHash", "forwardIdsSharded"]
PFX = "Java_io_yaochi_recommendation_model_gpu_GpuRecModel_"
INT, LONG, FLOAT, BYTE = 1, 2, 3, 4


def _lib():
    srcs = [os.path.join(HARNESS, "fake_jni.c"), os.path.join(HARNESS, "include", "jni.h"),
            os.path.join(ROOT, "recommendation-models_amd", "jni", "rmx_jni.c")]
    if not os.path.exists(LIB) or max(os.path.getmtime(s) for s in srcs) > os.path.getmtime(LIB):
        subprocess.check_call(["make", "-s", "-C", HARNESS])
    L = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    L.fj_env.restype = vp
    L.fj_new_array.restype = vp
    L.fj_new_array.argtypes = [ctypes.c_int, ctypes.c_int32, vp]
    L.fj_data.restype = vp
    L.fj_data.argtypes = [vp]
    L.fj_len.argtypes = [vp]
    L.fj_release_mode.argtypes = [vp]
    L.fj_free.argtypes = [vp]
    L.fj_exception.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    return L


class Jvm:
    """Calls the natives like the Scala object GpuRecModel."""

    def __init__(self):
        self.L = _lib()
        self.env = self.L.fj_env()

    def arr(self, kind, a):
        if a is None:
            return None
        dt = {INT: np.int32, LONG: np.int64, FLOAT: np.float32, BYTE: np.int8}[kind]
        a = np.ascontiguousarray(a, dt)
        return self.L.fj_new_array(kind, a.size, a.ctypes.data)

    def np(self, h, dtype):
        n = self.L.fj_len(h)
        return np.ctypeslib.as_array(ctypes.cast(self.L.fj_data(h), ctypes.POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                     (n,)).copy() if n > 0 else np.zeros(0, dtype)

    def call(self, name, restype, *args):
        f = getattr(self.L, PFX + name)
        f.restype = restype
        conv = []
        for a in args:
            if isinstance(a, float):
                conv.append(ctypes.c_float(a))
            elif isinstance(a, (int, np.integer)):
                conv.append(ctypes.c_int64(int(a)))
            else:
                conv.append(a)
        self.L.fj_clear()
        return f(ctypes.c_void_p(self.env), None, *conv)

    def exception(self):
        c, m = ctypes.create_string_buffer(96), ctypes.create_string_buffer(512)
        if not self.L.fj_exception(c, 96, m, 512):
            return None
        return c.value.decode(), m.value.decode()


def test_shim_builds_and_exports_every_native():
    L = _lib()
    for n in NATIVES:
        assert hasattr(L, PFX + n), n


def _i32(v):
    return ctypes.c_int32(v)


def test_jni_lb_natives_check_array_lengths():
    """every L-B native checks its Java arrays against batch * nFields (* k), the targets
    against batch and the gradients against the model's sizes BEFORE staging anything -- a short or
    null array throws IllegalArgumentException (the reference's require) instead of reaching the
    device.  The checks run on the host, so a metadata-only model (context 0) exercises them here."""
    j = Jvm()
    V, B = 1000, 8
    jm = j.call("createModel", ctypes.c_int64, ctypes.c_int64(0), _i32(1), ctypes.c_int64(V), _i32(F), _i32(K),
                j.arr(INT, [16]), None, _i32(0))
    assert j.exception() is None and jm
    ml = F * K * 16 + 16 + 16 + 1
    ok_ids = np.zeros(B * F, np.int32)
    short = ok_ids[:-1]
    z = lambda n: j.arr(FLOAT, np.zeros(n, np.float32))  # noqa: E731

    def raises(name, restype, *args, what):
        j.call(name, restype, ctypes.c_int64(jm), *args)
        exc = j.exception()
        assert exc and exc[0] == "java/lang/IllegalArgumentException", (name, exc)
        assert what in exc[1], (name, exc)

    T = ctypes.c_int64(0)
    for ids in (None, j.arr(INT, short)):
        raises("forwardIds", ctypes.c_void_p, T, _i32(B), ids, what="batch * nFields")
        raises("forwardIdsSharded", ctypes.c_void_p, T, _i32(B), ids, what="batch * nFields")
        raises("backwardIds", ctypes.c_float, T, _i32(B), ids, z(B), None, None, None, None, what="batch * nFields")
    raises("predictIds", ctypes.c_void_p, T, ctypes.c_int64(B), j.arr(INT, short), _i32(4), what="nRows * nFields")
    raises("predictIds", ctypes.c_void_p, T, ctypes.c_int64(B), j.arr(INT, ok_ids), _i32(0), what="batch > 0")
    ids = j.arr(INT, ok_ids)
    raises("backwardIds", ctypes.c_float, T, _i32(B), ids, None, None, None, None, None, what="targets")
    raises("backwardIds", ctypes.c_float, T, _i32(B), ids, z(B - 1), None, None, None, None, what="targets")
    raises("backwardIds", ctypes.c_float, T, _i32(B), ids, z(B), z(0), None, None, None, what="gBias")
    raises("backwardIds", ctypes.c_float, T, _i32(B), ids, z(B), None, z(B * F - 1), None, None, what="gWeights")
    raises("backwardIds", ctypes.c_float, T, _i32(B), ids, z(B), None, None, z(B * F * K + 1), None,
           what="gEmbedding")
    raises("backwardIds", ctypes.c_float, T, _i32(B), ids, z(B), None, None, None, z(ml - 1), what="gMats")
    raises("auc", ctypes.c_double, z(B), z(B - 1), what="same length")
    raises("auc", ctypes.c_double, None, z(B), what="same length")
    j.call("destroyModel", None, ctypes.c_int64(jm))


@pytest.mark.gpu
def test_jni_host_array_forward_backward_match_c_abi():
    import rmx
    j = Jvm()
    V, B = 10_000, 300
    fc = [64, 32]
    ctx = j.call("createContext", ctypes.c_int64, _i32(0))
    m = j.call("createModel", ctypes.c_int64, ctypes.c_int64(ctx), _i32(1), ctypes.c_int64(V), _i32(F), _i32(K),
               j.arr(INT, fc), None, _i32(0))
    assert j.exception() is None and m
    ref = rmx.DeepFM(V, F, K, fc)
    sizes = j.np(j.call("getMatsSize", ctypes.c_void_p, ctypes.c_int64(m)), np.int32)
    assert sizes.tolist() == ref.getMatsSize()
    rng = np.random.default_rng(1)
    mats = ref.initMats(SEED_MATS)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    feats = rng.integers(0, V, B * F)
    w = rng.uniform(-0.05, 0.05, B * F).astype(np.float32)
    e = rng.uniform(-0.05, 0.05, B * F * K).astype(np.float32)
    bias = np.array([0.01], np.float32)
    y = (rng.random(B) < 0.3).astype(np.float32)
    args = [j.arr(LONG, index), j.arr(LONG, feats), j.arr(FLOAT, bias), j.arr(FLOAT, w), j.arr(FLOAT, e), _i32(K),
            j.arr(FLOAT, mats), j.arr(INT, sizes), None]
    out = j.call("forward0", ctypes.c_void_p, ctypes.c_int64(m), _i32(B), *args)
    assert j.exception() is None
    got = j.np(out, np.float32)
    assert np.array_equal(got, ref.forward(B, (index, feats), bias, w, e, K, mats, sizes))
    # backward0: gradients written back into bias / weights / embeddings / mats (release mode 0),
    # the COO arrays and targets released read-only (JNI_ABORT)
    tg = j.arr(FLOAT, y)
    loss = j.call("backward0", ctypes.c_float, ctypes.c_int64(m), _i32(B), *args, tg)
    assert j.exception() is None
    b2, w2, e2, m2 = bias.copy(), w.copy(), e.copy(), mats.copy()
    ref_loss = ref.backward(B, (index, feats), b2, w2, e2, K, m2, sizes, y)
    assert loss == ref_loss
    for h, r in zip([args[2], args[3], args[4], args[6]], [b2, w2, e2, m2]):
        assert np.array_equal(j.np(h, np.float32), r)
        assert j.L.fj_release_mode(h) == 0
    for h in (args[0], args[1], args[7], tg):
        assert j.L.fj_release_mode(h) == JNI_ABORT
    # the reference's failure mode: Scatter's require(index < batchSize) -> IllegalArgumentException
    bad = index.copy()
    bad[5] = B
    j.call("forward0", ctypes.c_void_p, ctypes.c_int64(m), _i32(B), j.arr(LONG, bad), *args[1:])
    exc = j.exception()
    assert exc and exc[0] == "java/lang/IllegalArgumentException" and "index should smaller than" in exc[1]
    j.call("destroyModel", None, ctypes.c_int64(m))
    j.call("destroyContext", None, ctypes.c_int64(ctx))


@pytest.mark.gpu
def test_jni_device_table_path_matches_c_abi():
    """createTable / fillTableSynthetic / setMats / setBias / forwardIds / predictIds / backwardIds /
    auc through the shim == the same calls through librmx's C ABI."""
    import rmx
    j = Jvm()
    V, B = 100_003, 1024
    fc = [400, 400, 400]
    jctx = j.call("createContext", ctypes.c_int64, _i32(0))
    jt = j.call("createTable", ctypes.c_int64, ctypes.c_int64(jctx), ctypes.c_int64(V), _i32(K), _i32(0))
    j.call("fillTableSynthetic", None, ctypes.c_int64(jt), ctypes.c_int64(SEED_TAB))
    jm = j.call("createModel", ctypes.c_int64, ctypes.c_int64(jctx), _i32(2), ctypes.c_int64(V), _i32(F), _i32(K),
                j.arr(INT, [64, 32]), j.arr(INT, [48, 32]), _i32(0))
    assert j.exception() is None
    ctx = rmx.default_context()
    ref = rmx.XDeepFM(V, F, K, [64, 32], [48, 32])
    mats = ref.initMats(SEED_MATS)
    ref.setMats(mats)
    ref.setBias(0.01)
    j.call("setMats", None, ctypes.c_int64(jm), j.arr(FLOAT, mats))
    j.call("setBias", None, ctypes.c_int64(jm), 0.01)
    assert j.exception() is None
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, 4 * B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, 4 * B, F, V, ids)
    h_ids = ids.numpy()
    out = rmx.DeviceArray(ctx, 4 * B, np.float32)
    ref.forward_ids(table, B, ids, out)
    ctx.sync()
    got = j.np(j.call("forwardIds", ctypes.c_void_p, ctypes.c_int64(jm), ctypes.c_int64(jt), _i32(B),
                      j.arr(INT, h_ids[:B * F])), np.float32)
    assert j.exception() is None
    assert np.array_equal(got, out.numpy()[:B])
    ref.predict_ids(table, 4 * B, ids, out, batch=B)
    ctx.sync()
    scores = out.numpy()
    jp = j.call("predictIds", ctypes.c_void_p, ctypes.c_int64(jm), ctypes.c_int64(jt), ctypes.c_int64(4 * B),
                j.arr(INT, h_ids), _i32(B))
    assert np.array_equal(j.np(jp, np.float32), scores)
    labels = (np.random.default_rng(3).random(4 * B) < 0.25).astype(np.float32)
    dl = rmx.DeviceArray.from_numpy(ctx, labels)
    a_ref = rmx.auc(ctx, dl, out)
    a = j.call("auc", ctypes.c_double, ctypes.c_int64(jm), j.arr(FLOAT, labels), jp)
    assert a == a_ref
    # backwardIds vs backward_ids
    y = labels[:B]
    ml = ref.matsLength()
    gb, gw, ge, gm = (j.arr(FLOAT, np.zeros(n, np.float32)) for n in (1, B * F, B * F * K, ml))
    loss = j.call("backwardIds", ctypes.c_float, ctypes.c_int64(jm), ctypes.c_int64(jt), _i32(B),
                  j.arr(INT, h_ids[:B * F]), j.arr(FLOAT, y), gb, gw, ge, gm)
    assert j.exception() is None
    d = {n: rmx.DeviceArray(ctx, c, np.float32) for n, c in (("b", 1), ("w", B * F), ("e", B * F * K), ("m", ml),
                                                               ("l", 1))}
    tgt = rmx.DeviceArray.from_numpy(ctx, y)
    ref.backward_ids(table, B, ids.view(0, B * F), tgt, d["b"], d["w"], d["e"], d["m"], d["l"])
    ctx.sync()
    assert np.float32(loss) == d["l"].numpy()[0]
    for h, n in ((gb, "b"), (gw, "w"), (ge, "e"), (gm, "m")):
        assert np.array_equal(j.np(h, np.float32), d[n].numpy()), n
    # a model created without a context answers metadata but refuses device calls
    jm0 = j.call("createModel", ctypes.c_int64, ctypes.c_int64(0), _i32(1), ctypes.c_int64(V), _i32(F), _i32(K),
                 j.arr(INT, fc), None, _i32(0))
    j.call("forwardIds", ctypes.c_void_p, ctypes.c_int64(jm0), ctypes.c_int64(jt), _i32(B), j.arr(INT, h_ids[:B * F]))
    assert j.exception()[0] == "java/lang/IllegalArgumentException"
    for name, h in (("destroyModel", jm0), ("destroyModel", jm), ("destroyTable", jt), ("destroyContext", jctx)):
        j.call(name, None, ctypes.c_int64(h))


@pytest.mark.gpu
def test_jni_sharded_single_rank():
    """commUniqueId / createShard / fillShardSynthetic / forwardIdsSharded on a one-rank communicator."""
    import rmx
    j = Jvm()
    V, B = 100_003, 512
    jctx = j.call("createContext", ctypes.c_int64, _i32(0))
    uid = j.call("commUniqueId", ctypes.c_void_p)
    assert j.exception() is None
    jsh = j.call("createShard", ctypes.c_int64, ctypes.c_int64(jctx), ctypes.c_int64(V), _i32(K), _i32(1), _i32(0),
                 ctypes.c_void_p(uid))
    j.call("fillShardSynthetic", None, ctypes.c_int64(jsh), ctypes.c_int64(SEED_TAB))
    jm = j.call("createModel", ctypes.c_int64, ctypes.c_int64(jctx), _i32(1), ctypes.c_int64(V), _i32(F), _i32(K),
                j.arr(INT, [400, 400, 400]), None, _i32(0))
    ref = rmx.DeepFM(V, F, K, [400, 400, 400])
    mats = ref.initMats(SEED_MATS)
    ref.setMats(mats)
    ref.setBias(0.01)
    j.call("setMats", None, ctypes.c_int64(jm), j.arr(FLOAT, mats))
    j.call("setBias", None, ctypes.c_int64(jm), 0.01)
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 9, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    ref.forward_ids(table, B, ids, out)
    ctx.sync()
    got = j.call("forwardIdsSharded", ctypes.c_void_p, ctypes.c_int64(jm), ctypes.c_int64(jsh), _i32(B),
                 j.arr(INT, ids.numpy()))
    assert j.exception() is None
    assert np.array_equal(j.np(got, np.float32), out.numpy())
    for name, h in (("destroyModel", jm), ("destroyShard", jsh), ("destroyContext", jctx)):
        j.call(name, None, ctypes.c_int64(h))
