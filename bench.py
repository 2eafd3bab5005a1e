#!/usr/bin/env python3
"""CTR-forward examples/sec on a Criteo-shaped synthetic batch (BASELINE.json metric).

Workload (default, configs[1]): DeepFM fp32, 39 fields / 1M vocab / k = 16, fcDims 400,400,400,
over a 1M-row synthetic set whose ids and table live in HBM before timing starts.  One step =
one forward (gather + first order + FM + tower + sigmoid) over one batch of --batch rows of that
set; successive steps walk the set.  --workload xdeepfm runs configs[2] (CIN 200,200,200).

Multi-GPU: one process per GPU (torch.distributed.run); every rank owns a replica of the 1M-row
table and its own batches (replicas only: the V = 1M forward has no exchange step), so
scaling is weak and value = sum of all ranks' examples / max rank time.

Prints ONE JSON line (rank 0).  Only the cpu_baseline leg touches oracle/ (the checker).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))

F, K, V = 39, 16, 1_000_000
FC = [400, 400, 400]
CIN = [200, 200, 200]
ROWS = 1 << 20  # the "1M-row synthetic" set
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75

# Peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0
PEAK_FP32_TFLOPS = 157.3
PEAK_BF16_TFLOPS = 2500.0  # dense
# fp32 GEMMs on the exact 3-way bf16 split (csrc/k_gemm_s3.hip): 6 bf16 MFMAs per fp32 product,
# so the ceiling of that arithmetic is the dense bf16 peak / 6 in fp32-equivalent FLOP/s
PEAK_S3_TFLOPS = PEAK_BF16_TFLOPS / 6
# stages whose GEMMs run on the split (f32_split on): priced against its peak.  The backward stages
# (dW and dX on the split; the CIN backward's rocBLAS part is fp32) take the higher peak too.
S3_STAGES = ("tower_layer", "cin_layer", "tower_back", "cin_back")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=["deepfm", "xdeepfm", "deepfm_sharded", "dcn_bf16", "pnn_bf16",
                                           "deepfm_train", "xdeepfm_train"],
                    default="deepfm")
    ap.add_argument("--vocab", type=int, default=0, help="table rows (default 1M; 100M for deepfm_sharded)")
    ap.add_argument("--batch", type=int, default=0, help="rows per step per GPU (default per workload)")
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="Zipf exponent of the ids within a field (SURVEY.md §8d secondary; 0 = uniform)")
    ap.add_argument("--no-dedupe", action="store_true", help="deepfm_sharded: skip the distinct-id step (default: auto)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--set", default="", help="kernel knobs before building the model, k=v,k=v (rmx_set_tuning)")
    return ap.parse_args()


def stage_work(workload, stage, B):
    """Algorithmic work of one launch of a stage: ('flop'|'byte', amount)."""
    D = F * K
    P = F * (F - 1) // 2
    es = 2 if workload.endswith("bf16") else 4  # table element bytes
    if stage == "shard_exchange":  # ids out + (k+1)-float rows back, all ranks' shares incl. self
        return "byte", B * F * (4 + 4 + (K + 1) * 4 * 2)
    if stage == "encoder_fm":  # ids + w + emb rows + y  (2,812 B / example)
        return "byte", B * (F * 4 + F * es + F * K * es + 4)
    if stage == "first_order":
        return "byte", B * (F * 4 + F * es + 4)
    if stage == "cross":  # ids + rows + pre2
        return "byte", B * (F * 4 + F * K * es + 4)
    if stage == "product":  # ids + rows + the [x | ip] row written
        return "byte", B * (F * 4 + F * K * es + (D + P) * es)
    k1 = D + P if workload.startswith("pnn") else D
    # backward (the *_train workloads): dW and dX GEMMs of every Linear, 2 x 2 B K N
    if stage == "tower_back1":
        return "flop", 4.0 * B * k1 * FC[0]
    if stage == "tower_back2":
        return "flop", 4.0 * B * FC[0] * FC[1]
    if stage == "tower_back3":
        return "flop", 4.0 * B * FC[1] * FC[2]
    if stage == "cin_back":  # dC_l and dZ_l GEMMs of every CIN layer
        hps = [F] + CIN[:-1]
        return "flop", sum(4.0 * B * K * F * hp * h for hp, h in zip(hps, CIN))
    if stage == "gather_x":
        return "byte", B * (F * 4 + F * K * es + D * 4)
    if stage == "tower_layer1":
        return "flop", 2.0 * B * k1 * FC[0]
    if stage == "tower_layer2":
        return "flop", 2.0 * B * FC[0] * FC[1]
    if stage == "tower_layer3":
        return "flop", 2.0 * B * FC[1] * FC[2] + 2.0 * B * FC[2]
    if stage.startswith("cin_layer"):
        idx = {"cin_layer1": 0, "cin_layer2": 1, "cin_layer3+": 2}[stage]
        hp = F if idx == 0 else CIN[idx - 1]
        return "flop", 2.0 * B * K * F * hp * CIN[idx]
    return None, 0


def cpu_baseline(workload, budget_s, threads):
    """Oracle (C restatement, OpenMP) on the host cores: examples/s on bounded batches."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ctypes as oc
    if workload == "dcn_bf16":
        om = oc.make_model(oc.DCN, F, K, fc=tuple(FC), cross_depth=3)
        B = 4096
    elif workload == "pnn_bf16":
        om = oc.make_model(oc.PNN, F, K, fc=tuple(FC))
        B = 4096
    elif workload != "xdeepfm":  # deepfm_sharded: same per-example CPU work (V = 1M table on the host)
        om = oc.make_model(oc.DEEPFM, F, K, fc=tuple(FC))
        B = 4096
    else:
        om = oc.make_model(oc.XDEEPFM, F, K, fc=tuple(FC), cin=tuple(CIN))
        B = 16
    mats = oc.init_mats(om, SEED_MATS)
    # the table slice for the rows we touch is regenerated on the host (same generator)
    done, t_tot, row0 = 0, 0.0, 0
    wt, et = oc.gen_table(SEED_TAB, V, K)
    while t_tot < budget_s:
        ids = oc.gen_ids(SEED_IDS, row0, B, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, ids)  # makeWeights / makeEmbeddings are part of the CPU path
        index = np.repeat(np.arange(B, dtype=np.int64), F)
        t0 = time.perf_counter()
        w, e = oc.gather(wt, et, 1, ids)
        oc.forward(om, B, index, np.array([0.01], np.float32), w, e, mats, 0, threads)
        t_tot += time.perf_counter() - t0
        done += B
        row0 += B
    return {"value": done / t_tot, "unit": "examples/s", "cores": threads, "kind": "port",
            "sample": "%d rows (%d batches of %d) of the same synthetic %s workload, fp32 oracle "
                      "(oracle/rmx_oracle.c, OpenMP, gather + forward), %.1f s"
                      % (done, done // B, B, workload, t_tot)}


def parity_check(workload, got, row0, n=512):
    """The checker beside the CPU baseline: GPU probabilities of rows [row0, row0 + n) of the bench
    set against the oracle on the same rows (fp64 oracle; bf16 workloads: the oracle's bf16-storage
    emulation, precision 2)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ctypes as oc
    base = workload
    if base == "xdeepfm":
        om = oc.make_model(oc.XDEEPFM, F, K, fc=tuple(FC), cin=tuple(CIN))
        n = min(n, 64)
    elif base == "dcn_bf16":
        om = oc.make_model(oc.DCN, F, K, fc=tuple(FC), cross_depth=3)
    elif base == "pnn_bf16":
        om = oc.make_model(oc.PNN, F, K, fc=tuple(FC))
    else:
        om = oc.make_model(oc.DEEPFM, F, K, fc=tuple(FC))
    mats = oc.init_mats(om, SEED_MATS)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    ids = oc.gen_ids(SEED_IDS, row0, n, F, V).astype(np.int64)
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(n, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    if workload.endswith("bf16"):
        ref = oc.forward(om, n, index, bias, oc.round_bf16(w), oc.round_bf16(e), mats, 2)
        tol, against = 2e-4, "oracle bf16-storage emulation (precision 2)"
    else:
        ref = oc.forward(om, n, index, bias, w, e, mats, 1)
        tol, against = 1e-5, "fp64 oracle"
    err = float(np.abs(got[:n] - ref).max())
    return {"rows": n, "max_abs_diff": err, "tol": tol, "against": against, "ok": err <= tol}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_sweep(workload, budget_s, threads):
    """All-core baseline (the reported value) + 1 and 2 threads (Spark local[1] / local[2]
    analogues) on shorter bounded samples."""
    res = cpu_baseline(workload, budget_s, threads)
    res["by_threads"] = {str(threads): round(res["value"], 1)}
    for t in (1, 2):
        if t < threads:
            res["by_threads"][str(t)] = round(cpu_baseline(workload, max(2.0, budget_s * 0.3), t)["value"], 1)
    res["cpu_model"] = cpu_model()
    res["nproc"] = os.cpu_count()
    return res


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # CPU (gloo) barrier / max only: the GPU work is librmx
        dist.init_process_group("gloo")
    import rmx
    for kv in filter(None, args.set.split(",")):
        k_, v_ = kv.split("=")
        rmx.set_tuning(k_, int(v_))

    train = args.workload.endswith("_train")
    base = args.workload[:-len("_train")] if train else args.workload
    B = args.batch or ({"xdeepfm": 16384, "xdeepfm_train": 4096}.get(args.workload, 65536))
    sharded = args.workload == "deepfm_sharded"
    Vw = args.vocab or (100_000_000 if sharded else V)
    # one rank per GPU; fewer GPUs than ranks (a rehearsal on a 1-GPU box) wraps ranks onto them
    # (torch.cuda.device_count() does not initialise the GPU on this image)
    ndev = 1
    if world > 1:
        import torch
        ndev = max(1, torch.cuda.device_count())
    if sharded and world > ndev:
        raise SystemExit("deepfm_sharded needs one GPU per rank (RCCL rejects ranks sharing a GPU)")
    rmx.set_device(local % ndev)
    ctx = rmx.default_context()
    stream = ctx.stream
    bf16 = args.workload.endswith("bf16")
    if base == "xdeepfm":
        model = rmx.XDeepFM(Vw, F, K, FC, CIN, ctx=ctx)
    elif args.workload == "dcn_bf16":  # configs[4]: DCN depth 3 + fcDims 400^3, bf16 table / weights
        model = rmx.DCN(Vw, F, K, 3, FC, ctx=ctx)
    elif args.workload == "pnn_bf16":  # configs[4]: PNN (IPNN) D1 = 400, fcDims 400^3, bf16
        model = rmx.PNN(Vw, F, K, FC, ctx=ctx)
    else:
        model = rmx.DeepFM(Vw, F, K, FC, ctx=ctx)
    if bf16:
        model.setPrecision(rmx.DTYPE_BF16)
    if sharded:
        # configs[3]: table hash-sharded over the ranks, RCCL exchange per batch
        # RCCL prints its version banner on fd 1 at init; keep stdout for the one JSON line
        sys.stdout.flush()
        saved_fd1 = os.dup(1)
        os.dup2(2, 1)
        try:
            uid = rmx.comm_unique_id() if rank == 0 else None
            if dist:
                box = [uid]
                dist.broadcast_object_list(box, src=0)
                uid = box[0]
            table = rmx.ShardedTable(ctx, Vw, K, world, rank, uid)
        finally:
            sys.stdout.flush()
            os.dup2(saved_fd1, 1)
            os.close(saved_fd1)
        table.set_dedupe(False if args.no_dedupe else "auto")
    else:
        table = rmx.EmbeddingTable(ctx, Vw, K, rmx.DTYPE_BF16 if bf16 else rmx.DTYPE_F32)
    table.fill_synthetic(SEED_TAB)
    model.setMats(model.initMats(SEED_MATS))
    model.setBias(0.01)
    nrows = max(ROWS, B)
    ids = rmx.DeviceArray(ctx, nrows * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, rank * nrows, nrows, F, Vw, ids, zipf=args.zipf)
    out = rmx.DeviceArray(ctx, nrows, np.float32)
    ctx.sync()
    nb = nrows // B
    import ctypes

    views = [(ids.view(s * B * F, B * F), out.view(s * B, B)) for s in range(nb)]
    if train:
        # synthetic labels Bernoulli(0.25), resident before timing; gradient outputs
        labels = (np.random.default_rng(SEED_IDS).random(nrows) < 0.25).astype(np.float32)
        tgt = rmx.DeviceArray(ctx, nrows, np.float32)
        tgt.upload(labels)
        g_b = rmx.DeviceArray(ctx, 1, np.float32)
        g_w = rmx.DeviceArray(ctx, B * F, np.float32)
        g_e = rmx.DeviceArray(ctx, B * F * K, np.float32)
        g_m = rmx.DeviceArray(ctx, model.matsLength(), np.float32)
        g_loss = rmx.DeviceArray(ctx, 1, np.float32)
        tviews = [tgt.view(s * B, B) for s in range(nb)]

    def step(i):
        ids_v, out_v = views[i % nb]
        if train:
            model.backward_ids(table, B, ids_v, tviews[i % nb], g_b, g_w, g_e, g_m, g_loss, stream)
        elif sharded:
            model.forward_ids_sharded(table, B, ids_v, out_v, stream)
        else:
            model.forward_ids(table, B, ids_v, out_v, stream)

    for i in range(args.warmup):
        step(i)
    ctx.sync()

    ev0, ev1 = ctypes.c_void_p(), ctypes.c_void_p()
    rmx._lib.lib.rmx_event_create(ctypes.byref(ev0))
    rmx._lib.lib.rmx_event_create(ctypes.byref(ev1))
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    rmx._lib.lib.rmx_event_record(ev0, stream)
    for i in range(args.steps):
        step(args.warmup + i)
    rmx._lib.lib.rmx_event_record(ev1, stream)
    ctx.sync()
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    ms = ctypes.c_float()
    rmx._lib.lib.rmx_event_elapsed_ms(ev0, ev1, ctypes.byref(ms))
    t_rank = max(wall, ms.value / 1e3)
    if dist:
        import torch
        t = torch.tensor([t_rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_rank = float(t.item())
    value = world * B * args.steps / t_rank

    # ---- roofline of the dominant kernel: per-stage HIP events on the launch stream ----
    model.set_timing(True)
    nt = max(5, min(args.steps, 20))
    for i in range(nt):
        step(i)
    ctx.sync()
    stages, calls = model.get_timing()
    model.set_timing(False)
    split = not bf16 and rmx.get_tuning("f32_split", 1) != 0

    def peak_of(stage):
        if bf16:
            return PEAK_BF16_TFLOPS
        return PEAK_S3_TFLOPS if split and stage.startswith(S3_STAGES) else PEAK_FP32_TFLOPS

    per_stage = {}
    for name, tot in stages.items():
        avg_ms = tot / max(calls, 1)
        kind, work = stage_work(args.workload, name, B)
        ent = {"avg_ms": round(avg_ms, 4)}
        if kind == "flop":
            ent["tflops"] = round(work / (avg_ms / 1e3) / 1e12, 2)
            ent["frac_mfma_peak"] = round(ent["tflops"] / peak_of(name), 3)
        elif kind == "byte":
            ent["gbs"] = round(work / (avg_ms / 1e3) / 1e9, 1)
            ent["frac_hbm_peak"] = round(ent["gbs"] / PEAK_HBM_GBS, 3)
        per_stage[name] = ent
    dom = max(stages.items(), key=lambda kv: kv[1])[0]
    kind, work = stage_work(args.workload, dom, B)
    avg_s = stages[dom] / max(calls, 1) / 1e3
    if kind == "byte":
        roof = {"bound": "hbm", "achieved": round(work / avg_s / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s"}
    else:
        roof = {"bound": "mfma", "achieved": round(work / avg_s / 1e12, 2), "peak": round(peak_of(dom), 1),
                "unit": "TFLOP/s"}
        if split and dom.startswith(S3_STAGES):
            roof["peak_basis"] = ("fp32 GEMM on the exact 3-way bf16 split: dense bf16 MFMA peak 2500 TF / 6 "
                                  "products (algorithmic fp32 FLOPs counted once)")
    roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
    # HBM bytes per launch of the same kernel from the committed rocprofv3 PMC passes
    # (FETCH_SIZE x 2 + WRITE_SIZE, tools/pmc_summary.py --stages); null when not profiled
    roof["traffic"] = None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):
        ent = json.load(open(tpath)).get(args.workload, {}).get(dom if not dom.startswith("cin") else "cin_layer")
        if ent and ent.get("batch") == B:
            roof["traffic"] = ent["hbm_bytes"]
            roof["traffic_source"] = "profiles/traffic.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE)"
    roof["kernel"] = dom
    roof["algorithmic_per_launch"] = work

    # predict loop over the whole resident row set + AUC (ParRecModel.predict, the examples' metric)
    pa = None
    if not train and not sharded:
        labels = (np.random.default_rng(SEED_IDS).random(nrows) < 0.25).astype(np.float32)
        dl = rmx.DeviceArray(ctx, nrows, np.float32)
        dl.upload(labels)
        ctx.sync()
        t0 = time.perf_counter()
        model.predict_ids(table, nrows, ids, out, batch=B, stream=stream)
        ctx.sync()
        t1 = time.perf_counter()
        a = rmx.auc(ctx, dl, out, stream=stream)
        t2 = time.perf_counter()
        pa = {"rows": nrows, "predict_ms": round((t1 - t0) * 1e3, 3), "auc_ms": round((t2 - t1) * 1e3, 3),
              "auc": round(a, 6), "labels": "Bernoulli(0.25), independent of the scores (AUC ~ 0.5)"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not train:
        threads = min(16, os.cpu_count() or 1)
        cpu = cpu_baseline_sweep(args.workload, args.cpu_seconds, threads)
        if not sharded and Vw == V and not args.zipf:
            # out holds the predict loop's probabilities of the whole rank-0 row set
            cpu["parity_check"] = parity_check(args.workload, out.numpy(), 0)

    if rank == 0:
        line = {
            "metric": ("CTR-train examples/sec (forward + RecModel.backward gradients; the optimizer lives on "
                       "the parameter server, out of scope)") if train else
                      "CTR-forward examples/sec on Criteo-shaped batch, DeepFM & xDeepFM, 1/2/4/8 GPU",
            "value": round(value, 1),
            "unit": "examples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_rank * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16 (fp32 accumulate)" if bf16 else "f32",
            **({"gemm_arith": "fp32 operands and accumulation; products on v_mfma_f32_16x16x32_bf16 via the exact "
                              "3-way bf16 split (6 products, dropped terms <= 2^-24 |xy|; parity vs the fp64 oracle "
                              "identical to the f32 MFMA engine)"} if split else {}),
            "data": "synthetic (splitmix64 Criteo-shaped ids, U(-0.05,0.05) table, Xavier mats)",
            "config": {"workload": "%s%s_F39_V%s_k16_fc400x3%s_B%d" % (
                args.workload, "" if bf16 else "_fp32",
                ("%dM" % (Vw // 1_000_000)) if Vw % 1_000_000 == 0 else str(Vw),
                {"xdeepfm": "_cin200x3", "dcn_bf16": "_cross3"}.get(base, ""), B),
                "global_batch": world * B, "rows_per_gpu_set": nrows,
                "ids": ("zipf%g" % args.zipf) if args.zipf else "uniform",
                "parallelism": ("hashshard%d_rccl" % world) if sharded else "replicas%d" % world},
            **({"exchange": {"dedupe": "off" if args.no_dedupe else "auto", "ids_sent_last_step": table.last_sent(),
                             "nnz_per_step": B * F}} if sharded else {}),
            "roofline": roof,
            "cpu_baseline": cpu,
            **({"predict_auc": pa} if pa else {}),
            "stages": per_stage,
        }
        if not train:
            # BASELINE.json asks for the HBM-roofline fraction too: the whole forward's algorithmic
            # bytes per example (ids + first-order weights + embedding rows + output)
            es = 2 if bf16 else 4
            bpe = F * 4 + F * es + F * K * es + 4
            line["forward_hbm"] = {"algorithmic_bytes_per_example": bpe,
                                   "gbs": round(value * bpe / 1e9, 1), "peak": PEAK_HBM_GBS,
                                   "frac": round(value * bpe / 1e9 / PEAK_HBM_GBS, 4),
                                   "note": "compute-bound: the dense tower / CIN, not the gather, sets the rate"}
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
