"""Barrier timeline of the bf16 tower tail (csrc/k_tail.hip, RMX_TAIL_DIAG & 16 build: tools/diag_tail.sh 16).
Runs the DCN bf16 forward at B = 65,536 and prints block 0's s_memtime stamps per wave (cycles since
the first stamp).  Usage: RMX_LIB=tools/diag_lib/tail16/librmx.so python tools/diag_tail_stamps.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rmx  # noqa: E402
from rmx import _lib  # noqa: E402

F, K, V, B = 39, 16, 1_000_000, 65536
ctx = rmx.default_context()
kind = os.environ.get("WL", "dcn")
m = rmx.DCN(V, F, K, 3, [400, 400, 400]) if kind == "dcn" else rmx.PNN(V, F, K, [400, 400, 400])
t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
t.fill_synthetic(7)
m.setPrecision(rmx.DTYPE_BF16)
m.setMats(m.initMats(11))
m.setBias(0.01)
ids = rmx.DeviceArray(ctx, B * F, np.int32)
rmx.gen_ids(ctx, 5, 0, B, F, V, ids)
out = rmx.DeviceArray(ctx, B, np.float32)
for _ in range(30):
    m.forward_ids(t, B, ids, out)
ctx.sync()
fn = _lib.lib.rmx_diag_tail
buf = (ctypes.c_ulonglong * 160)()
assert fn(buf) == 0
a = np.array(buf, dtype=np.int64).reshape(4, 40)
t0 = min(a[s, 0] for s in range(4) if a[s, 0] > 0)
names = ["start", "B0", "<BM2", "BM2>", "<B1", "B1>", "B2>", "<BM3", "BM3>", "<B3", "B3>"]
for s, wn in enumerate(["wave0 (2 tiles)", "wave2 (2 tiles)", "wave12 (1 tile)", "loader0"]):
    row = a[s]
    print(wn)
    for it in range(2):
        ks = [0] if it == 0 else []
        ks += [1 + 10 * it + j for j in range(10)]
        print("  it%d " % it + " ".join("%s=%d" % (names[k - 10 * it if k else 0], row[k] - t0) for k in ks if row[k] > 0))
