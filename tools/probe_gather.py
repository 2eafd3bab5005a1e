#!/usr/bin/env python3
"""Timing probe: DeepFM forward at B = 65,536 with the bench's random ids vs ids whose rows are
consecutive within each field (the layer-1 gather becomes a stream), vs all ids = one row per field
(every gather an L2 hit).  The difference isolates what the random gather costs tower layer 1."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import rmx  # noqa: E402

F, K, V, B = 39, 16, 1_000_000, 65536
ctx = rmx.default_context()
m = rmx.DeepFM(V, F, K, [400, 400, 400])
m.setMats(m.initMats(0x3A75))
m.setBias(0.01)
t = rmx.EmbeddingTable(ctx, V, K)
t.fill_synthetic(0x7AB1E)
out = rmx.DeviceArray(ctx, B, np.float32)
ids = rmx.DeviceArray(ctx, B * F, np.int32)
per = V // F
off = (np.arange(F) * per).astype(np.int64)
cases = {}
rng = np.random.default_rng(1)
cases["random"] = (off[None, :] + rng.integers(0, per, size=(B, F))).astype(np.int32)
cases["field-sequential"] = (off[None, :] + (np.arange(B) % per)[:, None]).astype(np.int32)
cases["one-row-per-field"] = np.broadcast_to(off[None, :], (B, F)).astype(np.int32)
for rnd in range(2):
    for name, a in cases.items():
        ids.upload(a.reshape(-1))
        t_end = time.time() + 1.0
        while time.time() < t_end:
            m.forward_ids(t, B, ids, out)
        ctx.sync()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            m.forward_ids(t, B, ids, out)
        ctx.sync()
        ms = (time.perf_counter() - t0) / n * 1e3
        print("%-18s %.4f ms / forward  (%.1f M examples/s)" % (name, ms, B / ms / 1e3), flush=True)
