#!/usr/bin/env python3
"""Per-phase cycles of one wave of the split GEMM (diagnostic build: tools/diag_build.sh 8, then
RMX_LIB=build/diag8/librmx.so python tools/diag_phases.py --workload xdeepfm|deepfm).  Runs one
forward, then after each stage reads g_rmx_diag_t (block 0, wave 0 of that launch)."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import rmx  # noqa: E402

NAMES = ["dma_wait", "barrier", "dma_issue", "a_frag", "split", "mfma_section", "mfma_tail+prologue"]
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="xdeepfm")
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--warm-s", type=float, default=2.5)
ap.add_argument("--stag", action="store_true", help="name the staggered loop's phases")
ap.add_argument("--set", default="", help="knobs k=v,k=v")
a = ap.parse_args()
if a.stag:
    NAMES = ["wait_before_bar0", "bar0", "prep", "phase1_tiles", "bar1", "phase2_tiles", "tail+prologue"]
F, K, V = 39, 16, 1_000_000
for kv in filter(None, a.set.split(",")):
    k_, v_ = kv.split("=")
    rmx.set_tuning(k_, int(v_))
ctx = rmx.default_context()
if a.workload == "xdeepfm":
    m, B = rmx.XDeepFM(V, F, K, [400, 400, 400], [200, 200, 200]), a.batch or 16384
elif a.workload == "dcn_bf16":
    m, B = rmx.DCN(V, F, K, 3, [400, 400, 400]), a.batch or 65536
    m.setPrecision(rmx.DTYPE_BF16)
else:
    m, B = rmx.DeepFM(V, F, K, [400, 400, 400]), a.batch or 65536
m.setMats(m.initMats(0x3A75))
m.setBias(0.01)
t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16 if a.workload.endswith("bf16") else rmx.DTYPE_F32)
t.fill_synthetic(0x7AB1E)
ids = rmx.DeviceArray(ctx, B * F, np.int32)
rmx.gen_ids(ctx, 0x5EED2026, 0, B, F, V, ids)
out = rmx.DeviceArray(ctx, B, np.float32)
import time
t_end = time.time() + a.warm_s  # >= 2 s of back-to-back launches first (MI355X_MICROARCH.md DVFS item 6)
while True:
    m.forward_ids(t, B, ids, out)
    ctx.sync()
    if time.time() >= t_end:
        break
buf = (ctypes.c_ulonglong * 18)()
fn = rmx._lib.lib.rmx_diag_phases_bf16 if a.workload.endswith("bf16") else rmx._lib.lib.rmx_diag_phases
assert fn(buf) == 0
for w in (0, 1):
    v = list(buf)[8 * w:8 * w + 8]
    steps = v[7]
    tot = sum(v[:7])
    print("last recorded split-GEMM launch (%s): %d K steps, block 0 wave %s" % (a.workload, steps, "0" if w == 0 else "NW/2"))
    for n, x in zip(NAMES, v[:7]):
        print("  %-20s %12d cycles  %6.0f /step  %5.1f %%" % (n, x, x / max(steps, 1), 100.0 * x / max(tot, 1)))
v = list(buf)
if v[17]:
    print("wave 0 of block 0: %d cycles in %.1f us -> in-kernel clock %.2f GHz" % (v[16], v[17] / 100.0, v[16] / v[17] * 0.1))
