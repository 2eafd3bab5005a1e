"""ctypes binding of librmx.so (include/rmx.h).

The product path: every call below runs HIP kernels in librmx.so.  There is no CPU
fallback; if the shared library is missing the import fails loudly.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RMX_LIB", os.path.join(os.path.dirname(_HERE), "csrc", "librmx.so"))

RMX_OK = 0
RMX_E_INVALID = -1
RMX_E_INDEX = -2
RMX_E_SHAPE = -3
RMX_E_TYPE = -4
RMX_E_HIP = -5
RMX_E_NOMEM = -6
RMX_E_MATS = -7
RMX_E_COMM = -8
FORMAT_LIBSVM, FORMAT_LIBFFM = 0, 1
UNIQUE_ID_BYTES = 128

DTYPE_F32 = 0
DTYPE_BF16 = 1
LAYOUT_K_MAJOR = 0
LAYOUT_ROW_MAJOR = 1

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "librmx.so not found at %s -- build it first (python -c 'import __graft_entry__ as g; g.build()' "
        "or make -C recommendation-models_amd/csrc)" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

c_int, c_i32, c_i64, c_u64, c_f32 = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
c_vp, c_sz = ctypes.c_void_p, ctypes.c_size_t
P = ctypes.POINTER

# (name, restype, argtypes) -- every symbol declared in include/rmx.h
SIGNATURES = [
    ("rmx_last_error", ctypes.c_char_p, []),
    ("rmx_abi_version", c_int, []),
    ("rmx_set_tuning", c_int, [ctypes.c_char_p, c_int]),
    ("rmx_get_tuning", c_int, [ctypes.c_char_p, c_int]),
    ("rmx_ctx_create", c_int, [c_int, P(c_vp)]),
    ("rmx_ctx_destroy", c_int, [c_vp]),
    ("rmx_ctx_stream", c_vp, [c_vp]),
    ("rmx_stream_sync", c_int, [c_vp]),
    ("rmx_malloc", c_int, [c_vp, c_sz, P(c_vp)]),
    ("rmx_free", c_int, [c_vp, c_vp]),
    ("rmx_memcpy_htod", c_int, [c_vp, c_vp, c_vp, c_sz]),
    ("rmx_memcpy_dtoh", c_int, [c_vp, c_vp, c_vp, c_sz]),
    ("rmx_event_create", c_int, [P(c_vp)]),
    ("rmx_event_destroy", c_int, [c_vp]),
    ("rmx_event_record", c_int, [c_vp, c_vp]),
    ("rmx_event_elapsed_ms", c_int, [c_vp, c_vp, P(c_f32)]),
    ("rmx_model_create", c_int, [c_vp, c_int, c_i64, c_int, c_int, P(c_i32), c_int, P(c_i32), c_int, c_int,
                                 P(c_vp)]),
    ("rmx_model_destroy", c_int, [c_vp]),
    ("rmx_model_get_type", c_int, [c_vp]),
    ("rmx_model_get_mats_size", c_int, [c_vp, P(c_i32), c_int, P(c_int)]),
    ("rmx_model_mats_len", c_i64, [c_vp]),
    ("rmx_model_get_input_dim", c_i64, [c_vp]),
    ("rmx_model_get_embedding_dim", c_int, [c_vp]),
    ("rmx_model_init_mats", c_int, [c_vp, c_u64, P(c_f32)]),
    ("rmx_forward", c_int, [c_vp, c_i32, c_i64, P(c_i64), P(c_i64), P(c_f32), P(c_f32), P(c_f32), c_i32,
                            P(c_f32), P(c_i32), c_i32, P(c_i64), P(c_f32)]),
    ("rmx_model_set_mats", c_int, [c_vp, P(c_f32), c_i64]),
    ("rmx_model_set_bias", c_int, [c_vp, c_f32]),
    ("rmx_table_create", c_int, [c_vp, c_i64, c_int, P(c_vp)]),
    ("rmx_table_create_ex", c_int, [c_vp, c_i64, c_int, c_int, P(c_vp)]),
    ("rmx_table_dtype", c_int, [c_vp]),
    ("rmx_model_set_precision", c_int, [c_vp, c_int]),
    ("rmx_table_destroy", c_int, [c_vp]),
    ("rmx_table_upload", c_int, [c_vp, P(c_f32), P(c_f32), c_int]),
    ("rmx_table_fill_synthetic", c_int, [c_vp, c_u64]),
    ("rmx_table_rows", c_i64, [c_vp]),
    ("rmx_table_embedding_dim", c_int, [c_vp]),
    ("rmx_table_refresh_lines", c_int, [c_vp]),
    ("rmx_table_device_ptrs", c_int, [c_vp, P(c_vp), P(c_vp)]),
    ("rmx_backward", c_int, [c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp,
                             c_vp, c_vp]),
    ("rmx_backward_ids", c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    ("rmx_gen_ids", c_int, [c_vp, c_u64, c_i64, c_i32, c_i32, c_i64, c_vp, c_vp]),
    ("rmx_gen_ids_zipf", c_int, [c_vp, c_u64, c_i64, c_i32, c_i32, c_i64, ctypes.c_double, c_vp, c_vp]),
    ("rmx_debug_fill_lds", c_int, [c_vp, ctypes.c_uint32, c_vp]),
    ("rmx_gather", c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    ("rmx_forward_ids", c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp]),
    ("rmx_model_set_timing", c_int, [c_vp, c_int]),
    ("rmx_model_get_timing", c_int, [c_vp, ctypes.c_char_p, c_int, P(c_f32), c_int, P(c_int), P(c_int)]),
    ("rmx_encoder_ids", c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp]),
    ("rmx_comm_unique_id", c_int, [c_vp, c_sz]),
    ("rmx_shard_create", c_int, [c_vp, c_i64, c_int, c_int, c_int, c_vp, P(c_vp)]),
    ("rmx_shard_destroy", c_int, [c_vp]),
    ("rmx_shard_abort", c_int, [c_vp]),
    ("rmx_group_create", c_int, [c_int, P(c_vp)]),
    ("rmx_group_destroy", c_int, [c_vp]),
    ("rmx_shard_create_group", c_int, [c_vp, c_i64, c_int, c_vp, c_int, P(c_vp)]),
    ("rmx_shard_fill_synthetic", c_int, [c_vp, c_u64]),
    ("rmx_shard_local_rows", c_i64, [c_vp]),
    ("rmx_shard_set_owner_hash", c_int, [c_vp, c_u64]),
    ("rmx_shard_owner_of", c_i64, [c_vp, c_i64]),
    ("rmx_owner_hash", c_i64, [c_u64, c_i64, c_int, c_i64, c_vp]),
    ("rmx_shard_set_dedupe", c_int, [c_vp, c_int]),
    ("rmx_shard_set_batch_hint", c_int, [c_vp, ctypes.c_int64]),
    ("rmx_debug_wgrad_slices", c_int, [ctypes.c_int64, c_int, c_int, c_int]),
    ("rmx_shard_last_sent", c_i64, [c_vp]),
    ("rmx_shard_overflow_rounds", c_i64, [c_vp]),
    ("rmx_predict_ids", c_int, [c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_vp]),
    ("rmx_auc", c_int, [c_vp, c_i64, c_vp, c_vp, ctypes.POINTER(ctypes.c_double), c_vp]),
    ("rmx_samples_parse", c_int, [c_vp, c_sz, c_int, c_int, c_vp]),
    ("rmx_samples_free", c_int, [c_vp]),
    ("rmx_samples_lines", c_i64, [c_vp]),
    ("rmx_samples_nnz", c_i64, [c_vp]),
    ("rmx_samples_rows", c_vp, [c_vp]),
    ("rmx_samples_cols", c_vp, [c_vp]),
    ("rmx_samples_values", c_vp, [c_vp]),
    ("rmx_samples_targets", c_vp, [c_vp]),
    ("rmx_samples_fields", c_vp, [c_vp]),
    ("rmx_samples_ids", c_int, [c_vp, c_i32, c_vp, c_i64]),
    ("rmx_shard_gather", c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    ("rmx_forward_ids_sharded", c_int, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp]),
    ("rmx_shard_pull", c_int, [c_vp, c_i64, c_vp, c_int, c_vp]),
    ("rmx_forward_pulled", c_int, [c_vp, c_vp, c_i32, c_int, c_vp, c_vp]),
]

for _name, _res, _args in SIGNATURES:
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


class RmxError(RuntimeError):
    """Error raised by librmx (status code in .code)."""

    def __init__(self, code, msg):
        super().__init__("%s (rmx status %d)" % (msg, code))
        self.code = code


class IllegalArgumentError(RmxError, ValueError):
    """Scatter's require(index < batchSize) (bnn/Scatter.scala:29-30) and bad arguments."""


class ShapeError(RmxError, ValueError):
    """BigDL Reshape size mismatch (nnz != batchSize * nFields)."""


class MatsError(RmxError, ValueError):
    """mats length / matSizes do not match getMatsSize."""


def check(status):
    if status == RMX_OK:
        return
    msg = (lib.rmx_last_error() or b"").decode("utf-8", "replace")
    if status == RMX_E_INDEX or status == RMX_E_INVALID:
        raise IllegalArgumentError(status, msg)
    if status == RMX_E_SHAPE:
        raise ShapeError(status, msg)
    if status == RMX_E_MATS:
        raise MatsError(status, msg)
    raise RmxError(status, msg)


def ptr(a, ct):
    """numpy array -> ctypes pointer (None stays None)."""
    if a is None:
        return None
    return a.ctypes.data_as(P(ct))
