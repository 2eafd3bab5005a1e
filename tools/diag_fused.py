#!/usr/bin/env python3
"""Per-layer cycles of the fused DeepFM tower (tower_fused_s3_kernel) from s_memtime stamps of block 0's
waves (diagnostic build: bash tools/vbuild.sh fdiag "-DRMX_FUSED_DIAG=1" k_fused_s3.hip, then
RMX_LIB=vbuild/fdiag/librmx.so python tools/diag_fused.py).  Runs ~2.5 s of back-to-back forwards first
(DVFS settles), then one forward, and prints per row block and wave: layer 1 (+ first order + FM), the FM
epilogue + h1 bias / ReLU, layer 2, layer 3 half 0, layer 3 half 1, the head, with the MFMA floor of
each layer (16 cycles per v_mfma_f32_16x16x32_bf16, two waves per SIMD) and the clock measured in the
kernel (s_memtime / s_memrealtime at 100 MHz)."""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import rmx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--warm-s", type=float, default=2.5)
ap.add_argument("--set", default="")
a = ap.parse_args()
for kv in filter(None, a.set.split(",")):
    k_, v_ = kv.split("=")
    rmx.set_tuning(k_, int(v_))
F, K, V, B = 39, 16, 1_000_000, a.batch
ctx = rmx.default_context()
m = rmx.DeepFM(V, F, K, [400, 400, 400])
m.setMats(m.initMats(0x3A75))
m.setBias(0.01)
t = rmx.EmbeddingTable(ctx, V, K)
t.fill_synthetic(0x7AB1E)
ids = rmx.DeviceArray(ctx, B * F, np.int32)
rmx.gen_ids(ctx, 0x5EED2026, 0, B, F, V, ids)
out = rmx.DeviceArray(ctx, B, np.float32)
t_end = time.time() + a.warm_s
n = 0
while time.time() < t_end:
    for _ in range(8):
        m.forward_ids(t, B, ids, out)
        n += 1
    ctx.sync()
m.forward_ids(t, B, ids, out)
ctx.sync()
NW, NIT, NPH = 8, 4, 6
NU1 = 80
buf = (ctypes.c_ulonglong * (NW * NIT * NPH + NW * 4 + NW * NU1))()
fn = rmx._lib.lib.rmx_diag_fused
fn.argtypes = [ctypes.c_void_p]
assert fn(buf) == 0
st = np.array(buf[:NW * NIT * NPH], dtype=np.int64).reshape(NW, NIT, NPH)
clk = np.array(buf[NW * NIT * NPH:NW * NIT * NPH + NW * 4], dtype=np.int64).reshape(NW, 4)
ghz = (clk[:, 2] - clk[:, 0]) / ((clk[:, 3] - clk[:, 1]) / 100e6) / 1e9
span = clk[:, 2] - clk[:, 0]
print("%d warm forwards; block 0: kernel span %.0f cycles (wave 0), clock %.3f GHz (waves %.3f-%.3f)"
      % (n, span[0], ghz[0], ghz.min(), ghz.max()))
KS = (F + 1) // 2
floor = {"layer1": KS * 25 * 6 * 2 * 16, "layer2": 13 * 25 * 6 * 2 * 16, "l3h0": 13 * 13 * 6 * 2 * 16,
         "l3h1": 13 * 12 * 6 * 2 * 16}
names = ["layer1", "fm_epi+h1", "layer2", "l3h0", "l3h1"]
for it in range(NIT):
    if not st[0, it, 0]:
        continue
    print("row block %d (cycles; MFMA floor per SIMD in brackets)" % it)
    rows = []
    for w in range(NW):
        v = st[w, it]
        d = [v[1] - v[0], v[2] - v[1], v[3] - v[2], v[4] - v[3], v[5] - v[4]]
        if it + 1 < NIT and st[w, it + 1, 0]:
            d.append(st[w, it + 1, 0] - v[5])
        rows.append(d)
    for j, nm in enumerate(names + ["head+next"]):
        col = [r[j] for r in rows if len(r) > j]
        if not col:
            continue
        fl = floor.get(nm)
        print("  %-10s mean %8.0f  min %8.0f  max %8.0f %s" % (
            nm, np.mean(col), np.min(col), np.max(col), ("[%d, eff %.2f]" % (fl, fl / np.mean(col))) if fl else ""))
tot = [st[w, 1, 0] - st[w, 0, 0] for w in range(NW) if st[w, 1, 0]]
if tot:
    fl = sum(floor.values())
    print("row block 0 -> 1, whole: mean %.0f cycles, MFMA floor %d (eff %.3f)" % (np.mean(tot), fl, fl / np.mean(tot)))

u = np.array(buf[NW * NIT * NPH + NW * 4:], dtype=np.int64).reshape(NW, NU1)
nu = 2 * KS
ends = np.concatenate([u[:, 1:nu], st[:, 1, 1:2]], axis=1)  # unit k ends at unit k + 1's entry (last: layer 1 end)
d = ends - u[:, :nu]
print("row block 1, layer-1 units (cycles, mean over waves; MFMA floor per unit %d / %d for half 0 / 1):"
      % (13 * 6 * 2 * 16, 12 * 6 * 2 * 16))
h0, h1 = d[:, 0::2].mean(axis=0), d[:, 1::2].mean(axis=0)
print("  half 0: " + " ".join("%d" % x for x in h0))
print("  half 1: " + " ".join("%d" % x for x in h1))
print("  mean half 0 %.0f, half 1 %.0f" % (h0.mean(), h1.mean()))
