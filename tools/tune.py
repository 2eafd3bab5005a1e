#!/usr/bin/env python3
"""A/B a kernel-variant knob in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

    python tools/tune.py --knob tower_variant --values 0,1,2 [--workload deepfm|xdeepfm] [--batch B]

Prints, per variant, the median and min per-stage time (HIP events on the launch stream) and the
end-to-end forward time over --iters forwards, and checks that every variant gives the same
probabilities as variant values[0] within 1e-5.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import rmx  # noqa: E402

F, K, V = 39, 16, 1_000_000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--workload", default="deepfm")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bf16", action="store_true", help="bf16 tables and tower (not xdeepfm)")
    ap.add_argument("--set", default="", help="extra knobs applied before building the models, k=v,k=v")
    a = ap.parse_args()
    vals = [int(v) for v in a.values.split(",")]
    ctx = rmx.default_context()
    for kv in filter(None, a.set.split(",")):
        k_, v_ = kv.split("=")
        rmx.set_tuning(k_, int(v_))

    def build():
        if a.workload == "deepfm":
            return rmx.DeepFM(V, F, K, [400, 400, 400], ctx=ctx), a.batch or 65536
        if a.workload == "xdeepfm":
            return rmx.XDeepFM(V, F, K, [400, 400, 400], [200, 200, 200], ctx=ctx), a.batch or 4096
        if a.workload == "dcn":
            return rmx.DCN(V, F, K, 3, [400, 400, 400], ctx=ctx), a.batch or 65536
        return rmx.PNN(V, F, K, [400, 400, 400], ctx=ctx), a.batch or 65536

    models = {}
    for v in vals:  # a model per variant: knobs read at model build (packing) apply too
        rmx.set_tuning(a.knob, v)
        m, B = build()
        if a.bf16:
            m.setPrecision(rmx.DTYPE_BF16)
        m.setMats(m.initMats(0x3A75))
        m.setBias(0.01)
        models[v] = m
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16 if a.bf16 else rmx.DTYPE_F32)
    t.fill_synthetic(0x7AB1E)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, 0x5EED2026, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    ref = None
    res = {v: {"e2e": [], "stages": {}} for v in vals}
    for r in range(a.rounds):
        for v in vals:
            rmx.set_tuning(a.knob, v)
            m = models[v]
            m.forward_ids(t, B, ids, out)
            ctx.sync()
            p = out.numpy()
            if ref is None:
                ref = p
            err = float(np.abs(p - ref).max())
            if err > 1e-5:
                print("variant %d differs from variant %d by %g" % (v, vals[0], err))
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                m.forward_ids(t, B, ids, out)
            ctx.sync()
            res[v]["e2e"].append((time.perf_counter() - t0) / a.iters * 1e3)
            m.set_timing(True)
            for _ in range(a.iters):
                m.forward_ids(t, B, ids, out)
            st, calls = m.get_timing()
            m.set_timing(False)
            for k, ms in st.items():
                res[v]["stages"].setdefault(k, []).append(ms / calls)
    for v in vals:
        e = np.array(res[v]["e2e"])
        print("%s=%d  e2e median %.4f ms min %.4f ms  (%.1f M ex/s)" % (a.knob, v, np.median(e), e.min(),
                                                                       B / np.median(e) / 1e3))
        for k, xs in res[v]["stages"].items():
            xs = np.array(xs)
            print("    %-14s median %.4f  min %.4f ms" % (k, np.median(xs), xs.min()))


if __name__ == "__main__":
    main()
