"""rmx -- MI355X-native CTR forward path behind the reference's RecModel plugin API.

Host-side mirror of yaochitc/recommendation-models' model boundary
(src/main/scala/io/yaochi/recommendation/model/RecModel.scala:6-155 and the model classes in
model/{lr,deepfm,xdeepfm,dcn,pnn,dnn}/), over the C ABI of librmx.so (include/rmx.h).

    from rmx import DeepFM, CooLongFloatMatrix
    model = DeepFM(inputDim, nFields, embeddingDim, fcDims)
    model.getMatsSize()                      # same sizes as DeepFM.getMatsSize
    probs = model.forward(batchSize, batch, bias, weights, embeddings, embeddingDim, mats, matSizes)

Arguments, their meaning and the failure modes follow the reference (see each docstring).
The math runs in HIP kernels on the GPU; there is no CPU fallback.
"""
import numpy as np

from . import _lib
from ._lib import (IllegalArgumentError, MatsError, RmxError, ShapeError, LAYOUT_K_MAJOR,  # noqa: F401
                   LAYOUT_ROW_MAJOR, DTYPE_F32, DTYPE_BF16, FORMAT_LIBSVM, FORMAT_LIBFFM, check, ptr)

import atexit
import ctypes
import threading
import weakref

__all__ = ["RecModelType", "CooLongFloatMatrix", "RecModel", "LR", "DeepFM", "XDeepFM", "DCN", "PNN", "DNN",
           "Context", "DeviceArray", "EmbeddingTable", "ShardedTable", "ExchangeGroup", "comm_unique_id", "SampleParser", "RmxError", "IllegalArgumentError",
           "ShapeError", "MatsError", "default_context", "set_device", "shutdown"]

MODEL_LR, MODEL_DEEPFM, MODEL_XDEEPFM, MODEL_DCN, MODEL_PNN, MODEL_DNN = range(6)


class RecModelType:
    """yr/model/RecModelType.scala:5-8"""
    BIAS_WEIGHT = "BIAS_WEIGHT"
    BIAS_WEIGHT_EMBEDDING = "BIAS_WEIGHT_EMBEDDING"
    BIAS_WEIGHT_EMBEDDING_MATS = "BIAS_WEIGHT_EMBEDDING_MATS"
    BIAS_WEIGHT_EMBEDDING_MATS_FIELD = "BIAS_WEIGHT_EMBEDDING_MATS_FIELD"


class CooLongFloatMatrix:
    """The COO batch the reference passes around (Angel CooLongFloatMatrix):
    getRowIndices / getColIndices / getValues (RecModel.scala:130-155 reads the first two)."""

    def __init__(self, rows, cols, values=None):
        self.rows = np.ascontiguousarray(rows, dtype=np.int64)
        self.cols = np.ascontiguousarray(cols, dtype=np.int64)
        self.values = (np.ones(len(self.rows), np.float32) if values is None
                       else np.ascontiguousarray(values, dtype=np.float32))
        if not (len(self.rows) == len(self.cols) == len(self.values)):
            raise ValueError("rows / cols / values lengths differ")

    def getRowIndices(self):
        return self.rows

    def getColIndices(self):
        return self.cols

    def getValues(self):
        return self.values


def set_tuning(key, value):
    """Process-wide kernel variant knob (rmx_set_tuning), for A/B timing in one process;
    value None restores the built-in default."""
    check(_lib.lib.rmx_set_tuning(key.encode(), -(2 ** 31) if value is None else int(value)))


def get_tuning(key, default=0):
    return int(_lib.lib.rmx_get_tuning(key.encode(), int(default)))


# ------------------------------------------------------------- teardown ----
# Every handle-owning object registers here.  shutdown() (an atexit hook) destroys the live ones in
# dependency order -- sharded / plain tables, models, device buffers, exchange groups, then contexts --
# while the interpreter, librmx and the HIP runtime are all still up.  Left to __del__, they would be
# freed during interpreter teardown, possibly after the HIP runtime's (or a profiler's) own exit
# handlers (an exit-time SIGSEGV under rocprofv3).
_LIVE_ORDER = ("shard", "table", "model", "array", "group", "ctx")
_live = {k: weakref.WeakSet() for k in _LIVE_ORDER}
_shut = False


def _track(kind, obj):
    _live[kind].add(obj)


def shutdown():
    """Synchronise every live Context, then destroy every live librmx object (idempotent; runs at
    interpreter exit).  Objects destroyed here are closed: using them afterwards raises."""
    global _shut, _default_ctx
    if _shut:
        return
    _shut = True
    for c in list(_live["ctx"]):
        try:
            if c.handle:
                c.sync()
        except Exception:
            pass
    for kind in _LIVE_ORDER:
        for o in list(_live[kind]):
            try:
                o.close()
            except Exception:
                pass
    _default_ctx = None


atexit.register(shutdown)


# ----------------------------------------------------------------- device ----
class Context:
    """One GPU + one HIP stream (rmx_ctx)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(_lib.lib.rmx_ctx_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = int(device)
        _track("ctx", self)

    @property
    def stream(self):
        return _lib.lib.rmx_ctx_stream(self.handle)

    def sync(self, stream=None):
        check(_lib.lib.rmx_stream_sync(stream if stream is not None else self.stream))

    def close(self):
        if self.handle:
            _lib.lib.rmx_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = None
_default_device = 0


def set_device(device):
    global _default_device
    _default_device = int(device)


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(_default_device)
    return _default_ctx


class DeviceArray:
    """A device (HBM) buffer of a numpy dtype, owned by a Context."""

    def __init__(self, ctx, n, dtype, _ptr=None, _owner=None):
        self.ctx = ctx
        self.n = int(n)
        self.dtype = np.dtype(dtype)
        self._owner = _owner  # views keep their parent alive and never free
        if _ptr is not None:
            self.ptr = _ptr
            return
        p = ctypes.c_void_p()
        check(_lib.lib.rmx_malloc(ctx.handle, self.nbytes, ctypes.byref(p)))
        self.ptr = p
        _track("array", self)

    def view(self, offset, n):
        """Non-owning view of elements [offset, offset + n)."""
        if offset < 0 or offset + n > self.n:
            raise IndexError("view out of range")
        return DeviceArray(self.ctx, n, self.dtype, ctypes.c_void_p(self.ptr.value + offset * self.dtype.itemsize),
                           self)

    @property
    def nbytes(self):
        return self.n * self.dtype.itemsize

    @classmethod
    def from_numpy(cls, ctx, a):
        a = np.ascontiguousarray(a)
        d = cls(ctx, a.size, a.dtype)
        d.upload(a)
        return d

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        if a.size != self.n:
            raise ValueError("size mismatch")
        check(_lib.lib.rmx_memcpy_htod(self.ctx.handle, self.ptr, a.ctypes.data, self.nbytes))

    def numpy(self):
        out = np.empty(self.n, self.dtype)
        check(_lib.lib.rmx_memcpy_dtoh(self.ctx.handle, out.ctypes.data, self.ptr, self.nbytes))
        return out

    def free(self):
        if self._owner is not None:
            self.ptr = None
            return
        if self.ptr:
            if self.ctx.handle:  # (a context destroyed first has freed its buffers' stream already)
                _lib.lib.rmx_free(self.ctx.handle, self.ptr)
            self.ptr = None

    close = free

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class EmbeddingTable:
    """HBM-resident first-order weights [V] + embeddings [V][k]: replaces the Angel PS matrices
    "weights" and "embedding" (ParRecModel.scala:74-105) and their pull + make* gather
    (ParRecModel.scala:165-199, 279-306)."""

    def __init__(self, ctx, num_rows, embedding_dim, dtype=DTYPE_F32):
        """dtype DTYPE_BF16: bf16 storage (fp32 uploads / the synthetic fill are rounded to nearest even)."""
        h = ctypes.c_void_p()
        check(_lib.lib.rmx_table_create_ex(ctx.handle, int(num_rows), int(embedding_dim), int(dtype),
                                           ctypes.byref(h)))
        self.handle = h
        self._lock = threading.Lock()
        self.ctx = ctx
        self.rows = int(num_rows)
        self.k = int(embedding_dim)
        self.dtype = int(dtype)
        _track("table", self)

    def upload(self, weights=None, embedding=None, layout=LAYOUT_ROW_MAJOR):
        """layout LAYOUT_K_MAJOR: embedding is the reference PS layout, k x V."""
        w = None if weights is None else np.ascontiguousarray(weights, np.float32)
        e = None if embedding is None else np.ascontiguousarray(embedding, np.float32)
        if w is not None and w.size != self.rows:
            raise ValueError("weights must have num_rows entries")
        if e is not None and e.size != self.rows * self.k:
            raise ValueError("embedding must have num_rows * k entries")
        check(_lib.lib.rmx_table_upload(self.handle, ptr(w, ctypes.c_float), ptr(e, ctypes.c_float), layout))

    def fill_synthetic(self, seed):
        check(_lib.lib.rmx_table_fill_synthetic(self.handle, int(seed)))

    def refresh_lines(self):
        """Rebuild (or, with knob table_lines 0, drop) the [rows][32] line copy of an fp32 k = 16 table."""
        check(_lib.lib.rmx_table_refresh_lines(self.handle))

    def gather(self, ids_dev, n, w_out=None, emb_out=None, stream=None):
        """Debug gather (makeWeights / makeEmbeddings): bit-exact copies into device buffers."""
        check(_lib.lib.rmx_gather(self.handle, int(n), ids_dev.ptr, w_out.ptr if w_out else None,
                                  emb_out.ptr if emb_out else None, stream))

    def close(self):
        if self.handle:
            _lib.lib.rmx_table_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    """RCCL unique id (bytes) for rmx.ShardedTable; rank 0 creates it, the caller broadcasts it."""
    buf = ctypes.create_string_buffer(_lib.UNIQUE_ID_BYTES)
    check(_lib.lib.rmx_comm_unique_id(buf, _lib.UNIQUE_ID_BYTES))
    return buf.raw


class ExchangeGroup:
    """In-process exchange group of nranks virtual ranks (rmx_group): ShardedTable(..., group=g) per
    rank, each driven from its own thread with its own Context, runs the RCCL exchange schedule with
    device copies as the transport (the N > 1 exchange on one GPU)."""

    def __init__(self, nranks):
        h = ctypes.c_void_p()
        check(_lib.lib.rmx_group_create(int(nranks), ctypes.byref(h)))
        self.handle = h
        self.nranks = int(nranks)
        _track("group", self)

    def close(self):
        if self.handle:
            _lib.lib.rmx_group_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedTable:
    """Hash-sharded table (owner = p(id) mod nranks, p a keyed permutation of the ids: OWNER_HASH_DEFAULT
    unless set_owner_hash picks another key, 0 = id mod nranks) over nranks processes, one GPU each,
    exchanging ids and rows over RCCL (replaces the PS partitions + sparse pulls, ParRecModel.scala:74-105, :165-199).
    unique_id=None makes a loopback shard: all partitions in this process (single-GPU testing)."""

    def __init__(self, ctx, num_rows, embedding_dim, nranks, rank=0, unique_id=None, group=None):
        h = ctypes.c_void_p()
        uid = None
        self.group = group  # keeps the ExchangeGroup alive as long as this shard
        if group is not None:
            if unique_id is not None or group.nranks != int(nranks):
                raise ValueError("a group shard takes no unique_id and the group's nranks")
            check(_lib.lib.rmx_shard_create_group(ctx.handle, int(num_rows), int(embedding_dim), group.handle,
                                                  int(rank), ctypes.byref(h)))
        elif unique_id is not None:
            if len(unique_id) != _lib.UNIQUE_ID_BYTES:
                raise ValueError("unique_id must have %d bytes" % _lib.UNIQUE_ID_BYTES)
            uid = ctypes.create_string_buffer(bytes(unique_id), _lib.UNIQUE_ID_BYTES)
        if group is None:
            check(_lib.lib.rmx_shard_create(ctx.handle, int(num_rows), int(embedding_dim), int(nranks), int(rank),
                                            uid, ctypes.byref(h)))
        self.handle = h
        self._lock = threading.Lock()
        self.ctx = ctx
        self.rows = int(num_rows)
        self.k = int(embedding_dim)
        self.nranks = int(nranks)
        self.rank = int(rank)
        _track("shard", self)

    def fill_synthetic(self, seed):
        check(_lib.lib.rmx_shard_fill_synthetic(self.handle, int(seed)))

    def local_rows(self):
        return int(_lib.lib.rmx_shard_local_rows(self.handle))

    def set_owner_hash(self, key):
        """Owner = keyed permutation of the id mod nranks (before fill_synthetic; default
        OWNER_HASH_DEFAULT; 0 = id mod nranks)."""
        check(_lib.lib.rmx_shard_set_owner_hash(self.handle, int(key)))

    def owner_of(self, gid):
        return int(_lib.lib.rmx_shard_owner_of(self.handle, int(gid)))

    def set_dedupe(self, on):
        """Send each distinct id of a batch once (ParRecModel.distinctIntIndices): True, False or
        "auto" (the default: off at one rank, else on, then off for 63 batches when it removed < 10 %
        of the ids)."""
        if on == "auto":
            mode = 2
        elif on is True or on is False:
            mode = int(on)
        else:
            raise ValueError('set_dedupe takes True, False or "auto", got %r' % (on,))
        check(_lib.lib.rmx_shard_set_dedupe(self.handle, mode))

    def set_batch_hint(self, nnz):
        """Seed the first exchange's bucket capacity from the ids per batch (every rank the same nnz, before
        the first exchange; rmx_shard_set_batch_hint), so it does not take the counted overflow round."""
        check(_lib.lib.rmx_shard_set_batch_hint(self.handle, int(nnz)))

    def last_sent(self):
        """Ids this rank sent to owners in its last exchange."""
        return int(_lib.lib.rmx_shard_last_sent(self.handle))

    def overflow_rounds(self):
        """Overflow rounds of the fixed-capacity exchange run so far (nranks > 1)."""
        return int(_lib.lib.rmx_shard_overflow_rounds(self.handle))

    def pull(self, ids_dev, n, slot, stream=None):
        """Collective: exchange n ids into pull slot 0 / 1 (ParRecModel.pull*); a model's
        forward_pulled consumes the slot, possibly on another stream."""
        check(_lib.lib.rmx_shard_pull(self.handle, int(n), ids_dev.ptr, int(slot), stream))

    def gather(self, ids_dev, n, w_out, emb_out, stream=None):
        """Collective: rows of ids_dev from their owners (bit-exact copies)."""
        check(_lib.lib.rmx_shard_gather(self.handle, int(n), ids_dev.ptr, w_out.ptr, emb_out.ptr, stream))

    def abort(self):
        """Tear down the RCCL communicator from any thread (a watchdog over a stuck exchange):
        later exchanges raise; only close() may follow (rmx_shard_abort).  Serialised with close() by
        a lock: once close() has taken the handle, abort() is a no-op (the C side also orders the
        two by a compare-exchange on the communicator's state)."""
        with self._lock:
            if self.handle:
                check(_lib.lib.rmx_shard_abort(self.handle))

    def close(self):
        with self._lock:  # the handle is cleared before the destroy: a later abort() sees None
            h, self.handle = self.handle, None
        if h:
            _lib.lib.rmx_shard_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


OWNER_HASH_DEFAULT = 0x5EED5A4D0C7A11ED  # include/rmx.h RMX_OWNER_HASH_DEFAULT


def owner_hash(key, num_rows, nranks, gid):
    """(owner rank, local row) of id gid under the keyed owner permutation (host only, rmx_owner_hash)."""
    loc = ctypes.c_int64()
    o = int(_lib.lib.rmx_owner_hash(int(key), int(num_rows), int(nranks), int(gid), ctypes.byref(loc)))
    if o < 0:
        raise ValueError("owner_hash: id %d outside [0, %d) or bad arguments" % (gid, num_rows))
    return o, int(loc.value)


def auc(ctx, labels_dev, scores_dev, n=None, stream=None):
    """Device AUC of (label > 0, score) pairs (rmx_auc; ties count 1/2)."""
    n = labels_dev.n if n is None else int(n)
    out = ctypes.c_double()
    check(_lib.lib.rmx_auc(ctx.handle, n, labels_dev.ptr, scores_dev.ptr, ctypes.byref(out), stream))
    return out.value


def gen_ids(ctx, seed, row0, batch, n_fields, num_rows, ids_dev, stream=None, zipf=0.0):
    """Synthetic field-partitioned ids straight into HBM (SURVEY.md §8d generator): uniform within
    the field (bit-identical to oracle orc_gen_ids), or Zipf-like with exponent `zipf` > 0."""
    if zipf:
        check(_lib.lib.rmx_gen_ids_zipf(ctx.handle, int(seed), int(row0), int(batch), int(n_fields),
                                        int(num_rows), float(zipf), ids_dev.ptr, stream))
        return
    check(_lib.lib.rmx_gen_ids(ctx.handle, int(seed), int(row0), int(batch), int(n_fields), int(num_rows),
                               ids_dev.ptr, stream))


def debug_fill_lds(ctx, pattern=0x7FC00000, stream=None):
    """Test hook: fill every CU's LDS with a 32-bit pattern (default a NaN) on the stream."""
    check(_lib.lib.rmx_debug_fill_lds(ctx.handle, int(pattern) & 0xFFFFFFFF, stream))


# ------------------------------------------------------------------ models ---
class RecModel:
    """abstract class RecModel(type) -- yr/model/RecModel.scala:6-127."""

    _kind = None
    _type = None

    def __init__(self, inputDim, nFields=0, embeddingDim=0, fcDims=(), cinDims=(), crossDepth=0, ctx=None):
        self._args = (int(inputDim), int(nFields), int(embeddingDim), tuple(int(d) for d in fcDims),
                      tuple(int(d) for d in cinDims), int(crossDepth))
        self._meta = self._create(None)  # host-only handle: metadata without a GPU
        self._ctx = ctx
        self._dev = None
        self._dev_mats_loaded = False
        _track("model", self)

    def _create(self, ctx):
        inputDim, nFields, k, fc, cin, depth = self._args
        fc_a = (ctypes.c_int32 * max(len(fc), 1))(*fc)
        cin_a = (ctypes.c_int32 * max(len(cin), 1))(*cin)
        h = ctypes.c_void_p()
        check(_lib.lib.rmx_model_create(ctx.handle if ctx else None, self._kind, inputDim, nFields, k, fc_a,
                                        len(fc), cin_a, len(cin), depth, ctypes.byref(h)))
        return h

    def _device(self):
        if self._meta is None:
            raise RmxError(_lib.RMX_E_INVALID, "model is closed")
        if self._dev is None:
            if self._ctx is None:
                self._ctx = default_context()
            self._dev = self._create(self._ctx)
        return self._dev

    @property
    def context(self):
        self._device()
        return self._ctx

    def close(self):
        """Destroy the device and metadata handles (rmx_model_destroy); the model is unusable after."""
        d, self._dev = self._dev, None
        m, self._meta = self._meta, None
        if d:
            _lib.lib.rmx_model_destroy(d)
        if m:
            _lib.lib.rmx_model_destroy(m)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- metadata (RecModel.scala:7, :121-125)
    def getType(self):
        return self._type

    def getMatsSize(self):
        n = ctypes.c_int()
        check(_lib.lib.rmx_model_get_mats_size(self._meta, None, 0, ctypes.byref(n)))
        buf = (ctypes.c_int32 * max(n.value, 1))()
        check(_lib.lib.rmx_model_get_mats_size(self._meta, buf, n.value, ctypes.byref(n)))
        return [int(buf[i]) for i in range(n.value)]

    def matsLength(self):
        """sum over pairs of getMatsSize (ParRecModel.initMats, ParRecModel.scala:107-113)."""
        return int(_lib.lib.rmx_model_mats_len(self._meta))

    def getInputDim(self):
        return int(_lib.lib.rmx_model_get_input_dim(self._meta))

    def getEmbeddingDim(self):
        return int(_lib.lib.rmx_model_get_embedding_dim(self._meta))

    def initMats(self, seed):
        """Deterministic synthetic mats (Xavier-uniform weights, U(-0.01, 0.01) biases)."""
        mats = np.zeros(self.matsLength(), np.float32)
        check(_lib.lib.rmx_model_init_mats(self._meta, int(seed), ptr(mats, ctypes.c_float)))
        return mats

    # -- forward (RecModel.scala:9-63)
    def forward(self, batchSize, batch, bias=None, weights=None, embeddings=None, embeddingDim=None, mats=None,
                matSizes=None, fields=None):
        """RecModel.forward overloads.  batch is a CooLongFloatMatrix (or (rows, cols[, values])); the
        other arrays are the already-gathered flat host arrays of the reference contract.  Returns
        batchSize sigmoid probabilities (np.float32)."""
        if not isinstance(batch, CooLongFloatMatrix):
            batch = CooLongFloatMatrix(*batch)
        index = batch.getRowIndices()
        feats = batch.getColIndices()
        f32 = lambda a: None if a is None else np.ascontiguousarray(a, np.float32).reshape(-1)
        bias, weights, embeddings, mats = f32(bias), f32(weights), f32(embeddings), f32(mats)
        sizes = None if matSizes is None else np.ascontiguousarray(matSizes, np.int32)
        fl = None if fields is None else np.ascontiguousarray(fields, np.int64)
        if embeddingDim is None:
            embeddingDim = self.getEmbeddingDim()
        out = np.zeros(int(batchSize), np.float32)
        h = self._device()
        check(_lib.lib.rmx_forward(
            h, int(batchSize), len(index), ptr(index, ctypes.c_int64), ptr(feats, ctypes.c_int64),
            ptr(bias, ctypes.c_float), ptr(weights, ctypes.c_float), ptr(embeddings, ctypes.c_float),
            int(embeddingDim), ptr(mats, ctypes.c_float), ptr(sizes, ctypes.c_int32),
            0 if sizes is None else len(sizes), ptr(fl, ctypes.c_int64), ptr(out, ctypes.c_float)))
        return out

    def backward(self, batchSize, batch, bias, weights, *rest):
        """RecModel.backward overloads (RecModel.scala:65-115), targets last:
        backward(B, batch, bias, weights, targets)
        backward(B, batch, bias, weights, embeddings, embeddingDim, targets)
        backward(B, batch, bias, weights, embeddings, embeddingDim, mats, matSizes[, fields], targets)
        As in the reference, bias / weights / embeddings / mats are overwritten IN PLACE with their
        gradients (pass contiguous np.float32 arrays); returns the mean BCE loss."""
        if not rest:
            raise TypeError("backward: targets missing")
        targets = np.ascontiguousarray(rest[-1], np.float32)
        rest = rest[:-1]
        embeddings = rest[0] if len(rest) > 0 else None
        embeddingDim = rest[1] if len(rest) > 1 else None
        mats = rest[2] if len(rest) > 2 else None
        matSizes = rest[3] if len(rest) > 3 else None
        fields = rest[4] if len(rest) > 4 else None
        if not isinstance(batch, CooLongFloatMatrix):
            batch = CooLongFloatMatrix(*batch)
        index = batch.getRowIndices()
        feats = batch.getColIndices()
        for name, a in (("bias", bias), ("weights", weights), ("embeddings", embeddings), ("mats", mats)):
            if a is not None and not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
                raise TypeError("backward writes gradients into %s in place: pass a contiguous np.float32 array"
                                % name)
        sizes = None if matSizes is None else np.ascontiguousarray(matSizes, np.int32)
        fl = None if fields is None else np.ascontiguousarray(fields, np.int64)
        if embeddingDim is None:
            embeddingDim = self.getEmbeddingDim()
        loss = ctypes.c_float()
        check(_lib.lib.rmx_backward(
            self._device(), int(batchSize), len(index), ptr(index, ctypes.c_int64), ptr(feats, ctypes.c_int64),
            ptr(bias, ctypes.c_float), ptr(weights, ctypes.c_float), ptr(embeddings, ctypes.c_float),
            int(embeddingDim), ptr(mats, ctypes.c_float), ptr(sizes, ctypes.c_int32),
            0 if sizes is None else len(sizes), ptr(fl, ctypes.c_int64), ptr(targets, ctypes.c_float),
            ctypes.byref(loss)))
        return loss.value

    def backward_ids(self, table, batch, ids_dev, targets_dev, g_bias=None, g_weights=None, g_embedding=None,
                     g_mats=None, loss=None, stream=None):
        """L-B backward: DeviceArrays for ids [batch*F] int32, targets [batch] and the gradient outputs
        (g_bias [1], g_weights [batch*F], g_embedding [batch*F*k], g_mats [mats_len], loss [1])."""
        p = lambda a: None if a is None else a.ptr
        check(_lib.lib.rmx_backward_ids(self._device(), table.handle, int(batch), ids_dev.ptr, targets_dev.ptr,
                                        p(g_bias), p(g_weights), p(g_embedding), p(g_mats), p(loss), stream))

    # -- device-resident path (replaces ParRecModel.pull* + make*)
    def setMats(self, mats):
        mats = np.ascontiguousarray(mats, np.float32)
        check(_lib.lib.rmx_model_set_mats(self._device(), ptr(mats, ctypes.c_float), len(mats)))

    def setPrecision(self, dtype):
        """DTYPE_BF16: bf16 weights / activations on bf16 MFMA with fp32 accumulation (before setMats)."""
        check(_lib.lib.rmx_model_set_precision(self._device(), int(dtype)))

    def setBias(self, bias):
        check(_lib.lib.rmx_model_set_bias(self._device(), float(np.asarray(bias).reshape(-1)[0])))

    def forward_ids(self, table, batch, ids_dev, out_dev, stream=None):
        """L-B forward: ids [batch * nFields] int32 and out [batch] float32 are DeviceArrays."""
        check(_lib.lib.rmx_forward_ids(self._device(), table.handle, int(batch), ids_dev.ptr, out_dev.ptr, stream))

    def predict_ids(self, table, n_rows, ids_dev, scores_dev, batch=65536, stream=None):
        """ParRecModel.predict over a device-resident row set: scores for n_rows rows of ids."""
        check(_lib.lib.rmx_predict_ids(self._device(), table.handle, int(n_rows), ids_dev.ptr, int(batch),
                                       scores_dev.ptr, stream))

    def forward_ids_sharded(self, shard, batch, ids_dev, out_dev, stream=None):
        """Collective L-B forward over a ShardedTable (every rank calls it with its own batch)."""
        check(_lib.lib.rmx_forward_ids_sharded(self._device(), shard.handle, int(batch), ids_dev.ptr, out_dev.ptr,
                                               stream))

    def forward_pulled(self, shard, batch, slot, out_dev, stream=None):
        """Forward over the rows ShardedTable.pull put in `slot` (waits for that pull on the device)."""
        check(_lib.lib.rmx_forward_pulled(self._device(), shard.handle, int(batch), int(slot), out_dev.ptr, stream))

    def encoder_ids(self, table, batch, ids_dev, y_dev, stream=None):
        check(_lib.lib.rmx_encoder_ids(self._device(), table.handle, int(batch), ids_dev.ptr, y_dev.ptr, stream))

    def set_timing(self, enable=True):
        check(_lib.lib.rmx_model_set_timing(self._device(), 1 if enable else 0))

    def get_timing(self):
        """{stage name: total ms} and the number of timed forward calls."""
        cap, stride = 32, 64
        names = ctypes.create_string_buffer(cap * stride)
        ms = (ctypes.c_float * cap)()
        n, calls = ctypes.c_int(), ctypes.c_int()
        check(_lib.lib.rmx_model_get_timing(self._device(), names, stride, ms, cap, ctypes.byref(n),
                                            ctypes.byref(calls)))
        res = {}
        for i in range(min(n.value, cap)):
            res[names.raw[i * stride:(i + 1) * stride].split(b"\0", 1)[0].decode()] = float(ms[i])
        return res, calls.value


class LR(RecModel):
    """class LR(inputDim) -- yr/model/lr/LR.scala:10-40.  nFields is only needed by forward_ids."""
    _kind = MODEL_LR
    _type = RecModelType.BIAS_WEIGHT

    def __init__(self, inputDim, nFields=0, ctx=None):
        super().__init__(inputDim, nFields, 0, ctx=ctx)


class DeepFM(RecModel):
    """class DeepFM(inputDim, nFields, embeddingDim, fcDims) -- yr/model/deepfm/DeepFM.scala:10-49."""
    _kind = MODEL_DEEPFM
    _type = RecModelType.BIAS_WEIGHT_EMBEDDING_MATS

    def __init__(self, inputDim, nFields, embeddingDim, fcDims, ctx=None):
        super().__init__(inputDim, nFields, embeddingDim, fcDims, ctx=ctx)


class DNN(RecModel):
    """class DNN(inputDim, nFields, embeddingDim, fcDims) -- yr/model/dnn/DNN.scala:10-49."""
    _kind = MODEL_DNN
    _type = RecModelType.BIAS_WEIGHT_EMBEDDING_MATS

    def __init__(self, inputDim, nFields, embeddingDim, fcDims, ctx=None):
        super().__init__(inputDim, nFields, embeddingDim, fcDims, ctx=ctx)


class XDeepFM(RecModel):
    """class XDeepFM(inputDim, nFields, embeddingDim, fcDims, cinDims) -- yr/model/xdeepfm/XDeepFM.scala:10-56.
    cinDims with more than one layer follow SURVEY.md Appendix A (the reference only runs one)."""
    _kind = MODEL_XDEEPFM
    _type = RecModelType.BIAS_WEIGHT_EMBEDDING_MATS

    def __init__(self, inputDim, nFields, embeddingDim, fcDims, cinDims, ctx=None):
        super().__init__(inputDim, nFields, embeddingDim, fcDims, cinDims, ctx=ctx)


class DCN(RecModel):
    """class DCN(inputDim, nFields, embeddingDim, crossDepth, fcDims) -- yr/model/dcn/DCN.scala:10-60."""
    _kind = MODEL_DCN
    _type = RecModelType.BIAS_WEIGHT_EMBEDDING_MATS

    def __init__(self, inputDim, nFields, embeddingDim, crossDepth, fcDims, ctx=None):
        super().__init__(inputDim, nFields, embeddingDim, fcDims, (), crossDepth, ctx=ctx)


class PNN(RecModel):
    """class PNN(inputDim, nFields, embeddingDim, fcDims) -- yr/model/pnn/PNN.scala:10-54 (inner product)."""
    _kind = MODEL_PNN
    _type = RecModelType.BIAS_WEIGHT_EMBEDDING_MATS

    def __init__(self, inputDim, nFields, embeddingDim, fcDims, ctx=None):
        super().__init__(inputDim, nFields, embeddingDim, fcDims, ctx=ctx)


# ------------------------------------------------------------------ parser ---
class Samples:
    """Parsed LIBSVM / LIBFFM text (native parser, csrc/parse.cpp): numpy copies of the COO arrays."""

    def __init__(self, text, fmt=_lib.FORMAT_LIBSVM, nthreads=0):
        if isinstance(text, str):
            text = text.encode()
        buf = ctypes.c_char_p(text)  # points into the bytes object: no copy
        h = ctypes.c_void_p()
        check(_lib.lib.rmx_samples_parse(buf, len(text), int(fmt), int(nthreads), ctypes.byref(h)))
        try:
            L = _lib.lib.rmx_samples_lines(h)
            n = _lib.lib.rmx_samples_nnz(h)

            def arr(fn, ct, dt, cnt):
                p = fn(h)
                if not cnt or not p:
                    return np.zeros(0, dt)
                return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ct)), shape=(cnt,)).copy()
            self.rows = arr(_lib.lib.rmx_samples_rows, ctypes.c_int64, np.int64, n)
            self.cols = arr(_lib.lib.rmx_samples_cols, ctypes.c_int64, np.int64, n)
            self.values = arr(_lib.lib.rmx_samples_values, ctypes.c_float, np.float32, n)
            self.targets = arr(_lib.lib.rmx_samples_targets, ctypes.c_float, np.float32, L)
            self.fields = (arr(_lib.lib.rmx_samples_fields, ctypes.c_int64, np.int64, n)
                           if fmt == _lib.FORMAT_LIBFFM else None)
            self._h = h
        except Exception:
            _lib.lib.rmx_samples_free(h)
            raise

    def ids(self, n_fields):
        """int32 ids [lines * n_fields] of a regular batch (rmx_samples_ids)."""
        out = np.zeros(len(self.targets) * int(n_fields), np.int32)
        check(_lib.lib.rmx_samples_ids(self._h, int(n_fields), out.ctypes.data_as(ctypes.c_void_p), out.size))
        return out

    def coo(self):
        return CooLongFloatMatrix(self.rows, self.cols, self.values)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None:
            try:
                _lib.lib.rmx_samples_free(h)
            except Exception:
                pass
            self._h = None


class SampleParser:
    """yr/data/SampleParser.scala:14-85 (LIBSVM / LIBFFM text -> COO, 1-based ids -> id - 1), on the
    native multi-threaded parser (csrc/parse.cpp).  lines: a list of strings (one sample each) or
    one bytes / str blob of '\n'-terminated lines."""

    @staticmethod
    def _text(lines):
        if isinstance(lines, (bytes, str)):
            return lines
        return "\n".join(lines)

    @staticmethod
    def parse(lines, type_):
        if type_ == RecModelType.BIAS_WEIGHT_EMBEDDING_MATS_FIELD:
            return SampleParser.parseLIBFFM(lines)
        coo, targets = SampleParser.parseLIBSVM(lines)
        return coo, None, targets

    @staticmethod
    def parseLIBSVM(lines, nthreads=0):
        s = Samples(SampleParser._text(lines), _lib.FORMAT_LIBSVM, nthreads)
        return s.coo(), s.targets

    @staticmethod
    def parseLIBFFM(lines, nthreads=0):
        s = Samples(SampleParser._text(lines), _lib.FORMAT_LIBFFM, nthreads)
        return s.coo(), s.fields, s.targets
