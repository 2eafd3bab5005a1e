#!/usr/bin/env python3
"""Throughput of the native LIBSVM parser (csrc/parse.cpp) on Criteo-shaped synthetic text:
N lines x 39 'id:1' pairs (ids from the bench generator, 1-based).  Prints lines/s per thread count.

    python tools/parse_bench.py [--lines 1000000] [--threads 1,2,8]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import rmx  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lines", type=int, default=1_000_000)
ap.add_argument("--threads", default="1,2,8")
a = ap.parse_args()
F, V = 39, 1_000_000
rng = np.random.default_rng(0)
ids = (np.arange(F)[None, :] * (V // F) + rng.integers(0, V // F, (a.lines, F)) + 1).astype(np.int64)
labels = (rng.random(a.lines) < 0.25).astype(np.int64)
t0 = time.perf_counter()
body = np.char.add(ids.astype(str), ":1")
text = "\n".join(str(l) + " " + " ".join(r) for l, r in zip(labels, body)).encode() + b"\n"
print("generated %.1f MB of text in %.1f s" % (len(text) / 1e6, time.perf_counter() - t0), flush=True)
for t in [int(x) for x in a.threads.split(",")]:
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        s = rmx.Samples(text, rmx.FORMAT_LIBSVM, t)
        best = min(best, time.perf_counter() - t0)
    assert len(s.targets) == a.lines and np.array_equal(s.ids(F).reshape(-1), (ids - 1).reshape(-1))
    print("threads %2d: %.3f s  %.2f M lines/s  %.2f GB/s" % (t, best, a.lines / best / 1e6, len(text) / best / 1e9),
          flush=True)
