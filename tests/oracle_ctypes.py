"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / CPU baseline.  The product (librmx.so and the
``rmx`` package) never loads the oracle.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

LR, DEEPFM, XDEEPFM, DCN, PNN, DNN = range(6)
MAX_LAYERS = 8


class OrcModel(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int32),
        ("n_fields", ctypes.c_int32),
        ("embedding_dim", ctypes.c_int32),
        ("n_fc", ctypes.c_int32),
        ("fc", ctypes.c_int32 * MAX_LAYERS),
        ("n_cin", ctypes.c_int32),
        ("cin", ctypes.c_int32 * MAX_LAYERS),
        ("cross_depth", ctypes.c_int32),
    ]


def make_model(mtype, F=39, k=16, fc=(), cin=(), cross_depth=0):
    m = OrcModel()
    m.type = mtype
    m.n_fields = F
    m.embedding_dim = k
    m.n_fc = len(fc)
    for i, v in enumerate(fc):
        m.fc[i] = v
    m.n_cin = len(cin)
    for i, v in enumerate(cin):
        m.cin[i] = v
    m.cross_depth = cross_depth
    return m


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    srcs = [os.path.join(ORACLE_DIR, f) for f in os.listdir(ORACLE_DIR) if f.endswith((".c", ".h"))]
    if not os.path.exists(LIB_PATH) or max(os.path.getmtime(f) for f in srcs) > os.path.getmtime(LIB_PATH):
        subprocess.check_call(["make", "-s", "-B", "-C", ORACLE_DIR])
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    f32p, i64p, i32p = P(ctypes.c_float), P(ctypes.c_int64), P(ctypes.c_int32)
    L.orc_mats_sizes.argtypes = [P(OrcModel), i32p, ctypes.c_int32]
    L.orc_mats_sizes.restype = ctypes.c_int32
    L.orc_mats_len.argtypes = [P(OrcModel)]
    L.orc_mats_len.restype = ctypes.c_int64
    L.orc_splitmix64.argtypes = [ctypes.c_uint64]
    L.orc_splitmix64.restype = ctypes.c_uint64
    L.orc_gen_ids.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                              ctypes.c_int64, i32p]
    L.orc_gen_table.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                ctypes.c_int64, f32p, f32p]
    L.orc_init_mats.argtypes = [P(OrcModel), ctypes.c_uint64, f32p]
    L.orc_gather.argtypes = [ctypes.c_int64, ctypes.c_int32, f32p, f32p, ctypes.c_int32,
                             ctypes.c_int64, i64p, f32p, f32p]
    L.orc_gather.restype = ctypes.c_int32
    L.orc_forward.argtypes = [P(OrcModel), ctypes.c_int32, ctypes.c_int64, i64p, f32p, f32p, f32p,
                              f32p, ctypes.c_int32, ctypes.c_int32, f32p]
    L.orc_forward.restype = ctypes.c_int32
    L.orc_first_order.argtypes = [ctypes.c_int32, ctypes.c_int64, i64p, f32p, f32p]
    L.orc_first_order.restype = ctypes.c_int32
    L.orc_fm.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, f32p, f32p]
    L.orc_fm.restype = ctypes.c_int32
    L.orc_round_bf16.argtypes = [ctypes.c_int64, f32p, f32p]
    L.orc_backward.argtypes = [P(OrcModel), ctypes.c_int32, ctypes.c_int64, i64p, f32p, f32p, f32p, f32p, f32p,
                               f32p, f32p, f32p, f32p, P(ctypes.c_double)]
    L.orc_backward.restype = ctypes.c_int32
    _lib = L
    return L


def _p(a, ct):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ct))


def mats_sizes(m):
    buf = np.zeros(256, np.int32)
    n = lib().orc_mats_sizes(ctypes.byref(m), _p(buf, ctypes.c_int32), 256)
    return buf[:n].copy()


def mats_len(m):
    return int(lib().orc_mats_len(ctypes.byref(m)))


def splitmix64(x):
    return int(lib().orc_splitmix64(x))


def gen_ids(seed, row0, B, F, V):
    ids = np.zeros(B * F, np.int32)
    lib().orc_gen_ids(seed, row0, B, F, V, _p(ids, ctypes.c_int32))
    return ids


def gen_table(seed, V, k, id0=0, nrows=None):
    nrows = V if nrows is None else nrows
    w = np.zeros(nrows, np.float32)
    emb = np.zeros(nrows * k, np.float32)
    lib().orc_gen_table(seed, V, k, id0, nrows, _p(w, ctypes.c_float), _p(emb, ctypes.c_float))
    return w, emb.reshape(nrows, k)


def gen_rows(seed, V, k, ids):
    """Gathered rows (w[n], E[n*k:(n+1)*k]) of the generated table for arbitrary ids, generating
    only those rows (a V = 100M table need not exist on the host)."""
    ids = np.asarray(ids, np.int64)
    w = np.zeros(len(ids), np.float32)
    e = np.zeros((len(ids), k), np.float32)
    for i, idv in enumerate(ids):
        wi, ei = gen_table(seed, V, k, int(idv), 1)
        w[i] = wi[0]
        e[i] = ei[0]
    return w, e.ravel()


def init_mats(m, seed):
    mats = np.zeros(mats_len(m), np.float32)
    lib().orc_init_mats(ctypes.byref(m), seed, _p(mats, ctypes.c_float))
    return mats


def gather(w_table, emb_table, layout, feats):
    """layout 0: emb_table is k x V (reference PS layout); 1: V x k."""
    feats = np.ascontiguousarray(feats, np.int64)
    if layout == 0:
        k, V = emb_table.shape
    else:
        V, k = emb_table.shape
    w_out = np.zeros(len(feats), np.float32)
    e_out = np.zeros(len(feats) * k, np.float32)
    st = lib().orc_gather(V, k, _p(np.ascontiguousarray(w_table, np.float32), ctypes.c_float),
                          _p(np.ascontiguousarray(emb_table, np.float32), ctypes.c_float), layout,
                          len(feats), _p(feats, ctypes.c_int64), _p(w_out, ctypes.c_float),
                          _p(e_out, ctypes.c_float))
    if st != 0:
        raise IndexError("oracle gather status %d" % st)
    return w_out, e_out


def forward(m, B, index, bias, weights, embedding, mats, precision=0, nthreads=0):
    index = np.ascontiguousarray(index, np.int64)
    bias = np.ascontiguousarray(bias, np.float32).reshape(-1)
    weights = None if weights is None else np.ascontiguousarray(weights, np.float32)
    embedding = None if embedding is None else np.ascontiguousarray(embedding, np.float32).reshape(-1)
    mats = None if mats is None else np.ascontiguousarray(mats, np.float32)
    out = np.zeros(B, np.float32)
    st = lib().orc_forward(ctypes.byref(m), B, len(index), _p(index, ctypes.c_int64),
                           _p(bias, ctypes.c_float), _p(weights, ctypes.c_float),
                           _p(embedding, ctypes.c_float), _p(mats, ctypes.c_float), precision,
                           nthreads, _p(out, ctypes.c_float))
    if st != 0:
        raise ValueError("oracle forward status %d" % st)
    return out


def first_order(B, index, weights):
    index = np.ascontiguousarray(index, np.int64)
    weights = np.ascontiguousarray(weights, np.float32)
    y1 = np.zeros(B, np.float32)
    st = lib().orc_first_order(B, len(index), _p(index, ctypes.c_int64), _p(weights, ctypes.c_float),
                               _p(y1, ctypes.c_float))
    if st != 0:
        raise IndexError("oracle first_order status %d" % st)
    return y1


def fm(B, F, k, embedding):
    e = np.ascontiguousarray(embedding, np.float32).reshape(-1)
    y2 = np.zeros(B, np.float32)
    lib().orc_fm(B, F, k, _p(e, ctypes.c_float), _p(y2, ctypes.c_float))
    return y2


def round_bf16(x):
    """bf16 round-to-nearest-even of an fp32 array (values stay fp32)."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    lib().orc_round_bf16(x.size, _p(x, ctypes.c_float), _p(y, ctypes.c_float))
    return y


def backward(m, B, index, bias, weights, embedding, mats, targets):
    """RecModel.backward restated (f64): returns dict(loss, bias, weights, embedding, mats) of the
    gradients the reference writes back into the caller's arrays."""
    index = np.ascontiguousarray(index, np.int64)
    bias = np.ascontiguousarray(bias, np.float32).reshape(-1)
    weights = None if weights is None else np.ascontiguousarray(weights, np.float32)
    embedding = None if embedding is None else np.ascontiguousarray(embedding, np.float32).reshape(-1)
    mats = None if mats is None else np.ascontiguousarray(mats, np.float32)
    targets = np.ascontiguousarray(targets, np.float32)
    nnz = len(index)
    gb = np.zeros(1, np.float32)
    gw = np.zeros(nnz, np.float32) if weights is not None else None
    ge = np.zeros(embedding.size, np.float32) if embedding is not None else None
    gm = np.zeros(mats.size, np.float32) if mats is not None else None
    loss = ctypes.c_double()
    st = lib().orc_backward(ctypes.byref(m), B, nnz, _p(index, ctypes.c_int64), _p(bias, ctypes.c_float),
                            _p(weights, ctypes.c_float), _p(embedding, ctypes.c_float), _p(mats, ctypes.c_float),
                            _p(targets, ctypes.c_float), _p(gb, ctypes.c_float), _p(gw, ctypes.c_float),
                            _p(ge, ctypes.c_float), _p(gm, ctypes.c_float), ctypes.byref(loss))
    if st != 0:
        raise ValueError("oracle backward status %d" % st)
    return {"loss": loss.value, "bias": gb, "weights": gw, "embedding": ge, "mats": gm}
