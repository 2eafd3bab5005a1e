#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into per-kernel averages (one line per kernel).

    python tools/pmc_summary.py gpurun_out/r01d [--json profiles/r01/traffic.json]

Reads every ``*counter_collection.csv`` below the directory (one --pmc pass each) and the
``*kernel_stats.csv`` of a --kernel-trace --stats pass when present.  HBM traffic per launch
follows /opt/skills/guides/MI355X_MICROARCH.md §HBM and cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a wide
coalesced read, so hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (an upper estimate for
narrower access widths, which the guide leaves uncalibrated; Infinity-Cache hits are counted).
The effective clock is GRBM_GUI_ACTIVE / 8 XCDs / kernel time (the guide's DVFS recipe).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("rmx::", "")


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] in ("GRBM_GUI_ACTIVE",):
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    stats = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    return vals, dur, stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    a = ap.parse_args()
    vals, dur, stats = load(a.dir)
    out = {}
    for k in sorted(set(vals) | set(stats)):
        v = {c: sum(x) / len(x) for c, x in vals[k].items()}
        e = {"counters": v}
        if k in stats:
            e.update(stats[k])
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            e["hbm_bytes"] = 2 * v["FETCH_SIZE"] * 1024 + v["WRITE_SIZE"] * 1024
            e["fetch_bytes_x2"] = 2 * v["FETCH_SIZE"] * 1024
            e["write_bytes"] = v["WRITE_SIZE"] * 1024
        if "GRBM_GUI_ACTIVE" in v and dur.get(k):
            t = sum(dur[k]) / len(dur[k])
            e["clock_ghz"] = v["GRBM_GUI_ACTIVE"] / 8 / t
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "SQ_BUSY_CYCLES" in v and v["SQ_BUSY_CYCLES"] > 0:
            e["mfma_busy_per_sq_busy"] = v["SQ_VALU_MFMA_BUSY_CYCLES"] / v["SQ_BUSY_CYCLES"]
        out[k] = e
    for k, e in out.items():
        parts = [k[:70]]
        if "avg_ns" in e:
            parts.append("avg %.1f us x%d" % (e["avg_ns"] / 1e3, e["calls"]))
        if "hbm_bytes" in e:
            parts.append("hbm %.1f MB (fetch*2 %.1f, write %.1f)" % (e["hbm_bytes"] / 1e6, e["fetch_bytes_x2"] / 1e6,
                                                                    e["write_bytes"] / 1e6))
        if "clock_ghz" in e:
            parts.append("clk %.2f GHz" % e["clock_ghz"])
        c = e["counters"]
        if "SQ_WAVE_CYCLES" in c:
            w = c["SQ_WAVE_CYCLES"]
            parts.append("wait %.2f inst_wait %.2f active %.2f" % (c.get("SQ_WAIT_ANY", 0) / w,
                                                                   c.get("SQ_WAIT_INST_ANY", 0) / w,
                                                                   c.get("SQ_ACTIVE_INST_ANY", 0) / w))
        if "SQ_LDS_BANK_CONFLICT" in c:
            parts.append("lds_conf %.3g" % c["SQ_LDS_BANK_CONFLICT"])
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            parts.append("mfma_busy %.3g" % c["SQ_VALU_MFMA_BUSY_CYCLES"])
        print(" | ".join(parts))
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        json.dump(out, open(a.json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
