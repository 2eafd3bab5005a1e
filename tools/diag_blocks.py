#!/usr/bin/env python3
"""Per-block timeline of one split-GEMM launch (diagnostic build with RMX_GEMM_DIAG & 256, e.g.
tools/diag_build.sh 392 (layer 1, gathered A) or 328 (dense layers; the last one recorded is layer 3)):

    RMX_LIB=build/diag392/librmx.so python tools/diag_blocks.py --workload deepfm --nblocks 512

Every block's wave 0 stamps s_memrealtime (100 MHz) at entry and exit plus its __smid(); this prints
the launch span, block durations, start-time histogram (the dispatch rounds) and per-CU idle time."""
import argparse
import collections
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import rmx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="deepfm")
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--nblocks", type=int, required=True)
ap.add_argument("--warm-s", type=float, default=2.5)
ap.add_argument("--set", default="", help="knobs k=v,k=v")
a = ap.parse_args()
F, K, V = 39, 16, 1_000_000
for kv in filter(None, a.set.split(",")):
    k_, v_ = kv.split("=")
    rmx.set_tuning(k_, int(v_))
ctx = rmx.default_context()
if a.workload == "xdeepfm":
    m, B = rmx.XDeepFM(V, F, K, [400, 400, 400], [200, 200, 200]), a.batch or 16384
else:
    m, B = rmx.DeepFM(V, F, K, [400, 400, 400]), a.batch or 65536
m.setMats(m.initMats(0x3A75))
m.setBias(0.01)
t = rmx.EmbeddingTable(ctx, V, K)
t.fill_synthetic(0x7AB1E)
ids = rmx.DeviceArray(ctx, B * F, np.int32)
rmx.gen_ids(ctx, 0x5EED2026, 0, B, F, V, ids)
out = rmx.DeviceArray(ctx, B, np.float32)
t_end = time.time() + a.warm_s
while True:
    m.forward_ids(t, B, ids, out)
    ctx.sync()
    if time.time() >= t_end:
        break
n = a.nblocks
buf = (ctypes.c_ulonglong * (3 * n))()
assert rmx._lib.lib.rmx_diag_blocks(buf, n) == 0
v = np.array(buf, dtype=np.int64).reshape(n, 3)
t0 = v[:, 0].min()
st, en, cu = (v[:, 0] - t0) / 100.0, (v[:, 1] - t0) / 100.0, v[:, 2]  # us
dur = en - st
span = en.max()
print("%s B=%d: %d blocks, span %.1f us; block duration min %.1f / median %.1f / max %.1f us" %
      (a.workload, B, n, span, dur.min(), np.median(dur), dur.max()))
print("start-time histogram (5 us bins):")
h = collections.Counter((st // 5).astype(int))
for b in sorted(h):
    print("  [%5.0f, %5.0f) us: %d" % (5 * b, 5 * b + 5, h[b]))
print("end-time histogram (5 us bins):")
h = collections.Counter((en // 5).astype(int))
for b in sorted(h):
    print("  [%5.0f, %5.0f) us: %d" % (5 * b, 5 * b + 5, h[b]))
per = collections.defaultdict(list)
for s_, e_, c_ in zip(st, en, cu):
    per[int(c_)].append((s_, e_))
busy = []
for c_, iv in per.items():
    iv.sort()
    cov, cur_s, cur_e = 0.0, None, None
    for s_, e_ in iv:
        if cur_e is None or s_ > cur_e:
            if cur_e is not None:
                cov += cur_e - cur_s
            cur_s, cur_e = s_, e_
        else:
            cur_e = max(cur_e, e_)
    cov += cur_e - cur_s
    busy.append(cov)
busy = np.array(busy)
print("%d distinct __smid values; blocks per id: %s" % (len(per), dict(collections.Counter(len(x) for x in per.values()))))
print("per-id busy (union of its blocks) / span: min %.2f median %.2f max %.2f" %
      (busy.min() / span, np.median(busy) / span, busy.max() / span))
