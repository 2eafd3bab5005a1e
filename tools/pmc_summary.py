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
    if name.startswith("_ZN3rmx"):
        # c++filt here does not know the bf16 mangling (DF16b): keep the identifier and the first
        # integer template argument, e.g. _ZN3rmx18encoder_k16_kernelILi0EDF16b... -> encoder_k16_kernel<0, bf16>
        m = re.match(r"_ZN3rmx(\d+)", name)
        n = int(m.group(1))
        ident = name[m.end():m.end() + n]
        rest = name[m.end() + n:]
        t = re.match(r"ILi(\d+)E", rest)
        bf = "bf16" if "DF16b" in rest else "float"
        return "%s<%s%s>" % (ident, (t.group(1) + ", ") if t else "", bf)
    name = re.sub(r"\((int|long|unsigned|float|rmx::|void)[^()]*\)$", "", name)
    return name.replace("void ", "").replace("rmx::", "").replace("__bf16", "bf16")


def load(d, cin_layers=0):
    """cin_layers L > 0: the CIN instantiation's dispatches are told apart by their order in each pass (one
    forward runs L CIN layers back to back), so each CIN layer gets its own entry, '<kernel>#L<i>'."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        order = {}
        if cin_layers:
            cin = sorted({int(r["Dispatch_Id"]) for r in rows
                          if re.search(r"gemm_kernel<Tile<[^>]*>, 3, ", short(r["Kernel_Name"]))})
            order = {dsp: i % cin_layers for i, dsp in enumerate(cin)}
        for r in rows:
            k = short(r["Kernel_Name"])
            if int(r["Dispatch_Id"]) in order:
                k = "%s#L%d" % (k, order[int(r["Dispatch_Id"])])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))  # (once per counter row)
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur[k + "#grbm"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    stats = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    return vals, dur, stats


def stage_of(kernel, workload=""):
    """bench.py stage name of a kernel (template signature -> stage).  PNN's layer 1
    reads the materialised [x | ip] rows (dense A, K = 1,365: the 16-wave 3-deep-ring tile), so it is
    told from its dense layer 2 by the tile."""
    m = re.search(r"gemm_kernel<Tile<([^>]*)>, (\d+), (\d+), (true|false|\d+)>", kernel)
    if m:
        tile, amode, epi = m.group(1), int(m.group(2)), int(m.group(3))
        if amode == 3:
            lm = re.search(r"#L(\d+)$", kernel)
            if lm:
                return ("cin_layer1", "cin_layer2", "cin_layer3+")[min(int(lm.group(1)), 2)]
            return "cin_layer"
        if amode in (1, 2):
            return "tower_layer1"
        if workload.startswith("pnn") and epi == 0:
            # (PNN's layers 2 and 3 run in the bf16 tail: its one stored dense-A GEMM is layer 1 over [x | ip])
            return "tower_layer1"
        return "tower_layer3" if epi == 1 else "tower_layer2"
    kernel = re.sub(r"^\(anonymous namespace\)::", "", kernel)
    for pat, st in (("encoder_k16v2_kernel", "encoder"), ("encoder_k16_kernel<1", "encoder_fm"), ("encoder_k16_kernel<0", "first_order"),
                    ("encoder_k16_kernel<2", "first_order_sigmoid"), ("product16_kernel", "product"),
                    ("product_kernel", "product"), ("cross16_kernel", "cross"), ("cross_kernel", "cross"),
                    ("owner_gather", "shard_exchange"), ("own_rows_kernel", "shard_exchange"),
                    ("own_gather", "shard_exchange"), ("tower_tail_bf16_kernel", "tower_tail"),
                    ("tower_tail_s3_kernel", "tower_tail"), ("tower_head_s3_kernel", "tower_layer1"),
                    ("tower_small_s3_kernel", "tower_small"), ("tower_fused_s3_kernel", "tower_fused"),):
        if kernel.startswith(pat):
            return st
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--stages", nargs=2, metavar=("TRAFFIC_JSON", "WORKLOAD"),
                    help="merge per-stage HBM bytes per launch into TRAFFIC_JSON under WORKLOAD")
    ap.add_argument("--batch", type=int, default=0, help="rows per launch of the profiled run")
    ap.add_argument("--source", default="", help="the committed summary file these counters are in (profiles/...)")
    ap.add_argument("--cin-layers", type=int, default=0, help="CIN layers per forward (per-layer CIN entries)")
    a = ap.parse_args()
    vals, dur, stats = load(a.dir, a.cin_layers)
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
        if dur.get(k):  # dispatch durations under the PMC passes (profiled: clocks run lower than live)
            e["pmc_avg_ns"] = sum(dur[k]) / len(dur[k])
        if "GRBM_GUI_ACTIVE" in v and dur.get(k + "#grbm"):
            t = sum(dur[k + "#grbm"]) / len(dur[k + "#grbm"])
            e["clock_ghz"] = v["GRBM_GUI_ACTIVE"] / 8 / t
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "SQ_BUSY_CYCLES" in v and v["SQ_BUSY_CYCLES"] > 0:
            e["mfma_busy_per_sq_busy"] = v["SQ_VALU_MFMA_BUSY_CYCLES"] / v["SQ_BUSY_CYCLES"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE", 0) > 0:
            # MfmaUtil (rocprofv3 -L): MFMA-busy cycles summed over the 1,024 SIMDs / (per-XCD GPU-active
            # cycles x 1,024); GRBM_GUI_ACTIVE sums the 8 XCDs (MI355X_MICROARCH.md DVFS recipe)
            e["mfma_util"] = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] / 8 * 1024)
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
        if "mfma_util" in e:
            parts.append("MFMA util %.1f %%" % (100 * e["mfma_util"]))
        if c.get("SQ_INSTS_MFMA"):
            parts.append("valu/mfma %.2f" % (c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"]))
        if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
            parts.append("L2 hit %.1f %%" % (100 * c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))
        if "pmc_avg_ns" in e:
            parts.append("pmc avg %.1f us" % (e["pmc_avg_ns"] / 1e3))
        print(" | ".join(parts))
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        json.dump(out, open(a.json, "w"), indent=1, sort_keys=True)
    if a.stages:
        path, wl = a.stages
        db = json.load(open(path)) if os.path.exists(path) else {}
        st = {}
        for k, e in out.items():
            name = stage_of(k, wl)
            if name and "hbm_bytes" in e:
                st[name] = {"hbm_bytes": round(e["hbm_bytes"]), "fetch_bytes_x2": round(e["fetch_bytes_x2"]),
                            "write_bytes": round(e["write_bytes"]), "kernel": k, "batch": a.batch}
                if "mfma_util" in e:
                    st[name]["mfma_util"] = round(e["mfma_util"], 4)
                if "pmc_avg_ns" in e:
                    st[name]["avg_ns"] = round(e["pmc_avg_ns"], 1)
                if "clock_ghz" in e:
                    st[name]["clock_ghz"] = round(e["clock_ghz"], 3)
                st[name]["counters"] = {c: round(x, 1) for c, x in sorted(e["counters"].items())}
                if a.source:
                    st[name]["source"] = a.source
        db[wl] = st
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        json.dump(db, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
