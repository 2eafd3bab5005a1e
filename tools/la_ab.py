#!/usr/bin/env python3
"""A/B of the L-A staging knobs (la_pin_threads, la_pin_flags): bench.run_la at B = 4,096 and 65,536, rounds
alternating.  python tools/la_ab.py "0:0" "8:0" "8:1" ...  (threads:flags)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv, specs = sys.argv[:1], sys.argv[1:]
import bench  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import rmx  # noqa: E402

ctx = rmx.default_context()
for rnd in range(2):
    for spec in specs:
        th, fl = (int(x) for x in spec.split(":"))
        rmx.set_tuning("la_pin_threads", th)
        rmx.set_tuning("la_pin_flags", fl)
        for B, calls in ((4096, 50), (65536, 10)):
            r = bench.run_la(None, rmx, ctx, B, calls)
            print("round %d threads %d flags %d B %d: %.4f ms/call, la_h2d %.4f ms, ok %s bitwise_vs_lb %s" % (
                rnd, th, fl, B, r["wall_ms_per_call"], r["stages_ms"].get("la_h2d", 0), r["parity_check"]["ok"],
                r["bitwise_vs_lb"]), flush=True)
