#!/usr/bin/env python3
"""One line per bench log of an A/B (tools/gpu_check.sh abw:/ab:): file, examples/s, per-stage avg ms.
Usage: python tools/abw_summary.py gpurun_out/<tag>/abw_*.log > profiles/r0N/ab_<name>.txt"""
import json
import sys

for f in sys.argv[1:]:
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        print("%s: no JSON line" % f)
        continue
    d = json.loads(lines[-1])
    if "encoder" in d and "stages" not in d:
        e = d["encoder"]
        print("%s  encoder V=%d B=%d  row table %.4f ms (%.1f GB/s)  line table %.4f ms (%.1f GB/s)  bitwise %s" % (
            f.split("/")[-1], e["vocab"], e["batch"], e["row_table"]["avg_ms"], e["row_table"]["achieved_gbs"],
            e["line_table"]["avg_ms"], e["line_table"]["achieved_gbs"], e["parity_check"]["bitwise_equal"]))
        continue
    st = "  ".join("%s %.4f" % (k, v["avg_ms"]) for k, v in d.get("stages", {}).items())
    print("%s  %.1f M examples/s  %s" % (f.split("/")[-1], d["value"] / 1e6, st))
