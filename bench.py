#!/usr/bin/env python3
"""CTR-forward examples/sec on a Criteo-shaped synthetic batch (BASELINE.json metric).

Workload (default, configs[1]): DeepFM fp32, 39 fields / 1M vocab / k = 16, fcDims 400,400,400,
over a 1M-row synthetic set whose ids and table live in HBM before timing starts.  One step =
one forward (gather + first order + FM + tower + sigmoid) over one batch of --batch rows of that
set; successive steps walk the set.  The default line also carries an "models.xdeepfm" sub-record
(configs[2], CIN 200,200,200 at B = 16,384): BASELINE.json's metric names DeepFM and xDeepFM.
Other workloads: xdeepfm, deepfm_sharded (configs[3]), dcn_bf16 / pnn_bf16 (configs[4]),
lr_plumbing (configs[0]: LIBSVM text -> parse -> LR predict -> AUC), deepfm_train / xdeepfm_train.

Multi-GPU: one process per GPU.  `bench.py --gpus N` launches its N ranks itself (fresh child
processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT; the launching parent makes
no GPU call and imports nothing of librmx), or runs as one rank of an external
`torch.distributed.run` (WORLD_SIZE set).  Every rank owns a replica of the 1M-row table and its own
batches (replicas only: the V = 1M forward has no exchange step), so scaling is weak and value = sum
of all ranks' examples / max rank time; deepfm_sharded hash-shards the 100M-row table over the ranks
(RCCL exchange per batch).  At N > 1 every rank checks its own bench rows against the oracle after
timing (`parity_check_ranks`).

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
CIN1 = [200]  # xdeepfm_cin1: the only CIN the reference can run (CINEncoder.scala:150-176; L > 1 mis-shapes)


def cin_of(workload):
    return CIN1 if workload.startswith("xdeepfm_cin1") else CIN
ROWS = 1 << 20  # the "1M-row synthetic" set
SEED_IDS, SEED_TAB, SEED_MATS, SEED_LAB = 0x5EED2026, 0x7AB1E, 0x3A75, 0x1AB3
PLUMB_ROWS, PLUMB_BATCH = 1000, 100  # configs[0]: 1k-row LIBSVM slice, batchSize 100 (LRLocalExample.scala:16)

# Peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0
PEAK_FP32_TFLOPS = 157.3
PEAK_BF16_TFLOPS = 2500.0  # dense
# fp32 GEMMs on the exact 3-way bf16 split (csrc/k_gemm_s3.hip): 6 bf16 MFMAs per fp32 product,
# so the ceiling of that arithmetic is the dense bf16 peak / 6 in fp32-equivalent FLOP/s
PEAK_S3_TFLOPS = PEAK_BF16_TFLOPS / 6
# stages whose GEMMs run on the split (f32_split on): priced against its peak.  The backward stages
# (dW and dX on the split; the CIN backward's rocBLAS part is fp32) take the higher peak too.
S3_STAGES = ("tower_layer", "tower_tail", "tower_small", "tower_fused", "cin", "tower_back", "head_x")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=["deepfm", "xdeepfm", "xdeepfm_cin1", "deepfm_sharded", "dcn_bf16",
                                           "pnn_bf16", "deepfm_train", "xdeepfm_train", "lr_plumbing", "encoder"],
                    default="deepfm")
    ap.add_argument("--no-encoder-record", action="store_true",
                    help="deepfm: skip the encoder sub-record (gather + first order + FM alone at V = 1M and 100M)")
    ap.add_argument("--enc-table", choices=["row", "line", "both"], default="both",
                    help="encoder workload: time the [V][k] row table, the [V][32] line table or both (a PMC pass "
                         "profiles one layout per run: the kernel instantiation is the same)")
    ap.add_argument("--no-la-record", action="store_true",
                    help="deepfm: skip the L-A record (rmx_forward with host arrays at B = 100 / 4,096 / 65,536)")
    ap.add_argument("--no-companion", action="store_true",
                    help="deepfm: skip the xDeepFM sub-record (BASELINE.json's metric names both models)")
    ap.add_argument("--no-sharded-companion", action="store_true",
                    help="deepfm at N > 1 (one GPU per rank): skip the configs[3] sub-record (the 100M-row table "
                         "hash-sharded over the ranks, RCCL exchange)")
    ap.add_argument("--sharded-companion", action="store_true",
                    help="deepfm: add the sharded sub-record at N = 1 too (a rehearsal of the N > 1 path)")
    ap.add_argument("--companion-timeout", type=float, default=240.0,
                    help="seconds the sharded sub-record may take before a watchdog aborts its communicator and "
                         "the line is printed with the sub-record marked as timed out")
    ap.add_argument("--vocab", type=int, default=0, help="table rows (default 1M; 100M for deepfm_sharded)")
    ap.add_argument("--batch", type=int, default=0, help="rows per step per GPU (default per workload)")
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="Zipf exponent of the ids within a field (SURVEY.md §8d secondary; 0 = uniform)")
    ap.add_argument("--no-dedupe", action="store_true", help="deepfm_sharded: skip the distinct-id step (default: auto)")
    ap.add_argument("--dedupe-on", action="store_true", help="deepfm_sharded: always run the distinct-id step")
    ap.add_argument("--no-overlap", action="store_true",
                    help="deepfm_sharded: exchange and forward on one stream (default: batch i + 1's exchange "
                         "on a second stream beside batch i's forward)")
    ap.add_argument("--settle-ms", type=float, default=400.0,
                    help="untimed steps run back to back for this long before the W warm-up steps, so the GPU "
                         "leaves its idle clock state first (0 = off)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="bounded CPU-baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-only", action="store_true",
                    help="no CPU timing, but the parity check of the predicted rows against the fp64 oracle (grids)")
    ap.add_argument("--set", default="", help="kernel knobs before building the model, k=v,k=v (rmx_set_tuning)")
    return ap.parse_args()


def stage_work(workload, stage, B, direct=False):
    """Algorithmic work of one launch of a stage: ('flop'|'byte', amount).  direct: the
    one-rank sharded table read in place (the "exchange" maps the batch's ids to partition rows)."""
    D = F * K
    P = F * (F - 1) // 2
    es = 2 if workload.endswith("bf16") else 4  # table element bytes
    if stage == "first_order_sigmoid":  # LR: ids + w + p
        return "byte", B * (F * 4 + F * es + 4)
    if stage == "shard_exchange":
        if direct:  # ids in, partition rows out
            return "byte", B * F * 8
        # ids out + (k+1)-float rows back, all ranks' shares incl. self
        return "byte", B * F * (4 + 4 + (K + 1) * 4 * 2)
    if stage == "encoder_fm":  # ids + w + emb rows + y  (2,812 B / example)
        return "byte", B * (F * 4 + F * es + F * K * es + 4)
    if stage == "first_order":
        return "byte", B * (F * 4 + F * es + 4)
    if stage == "encoder_fm_x":  # training: the same reads + the gathered rows stored as fp32 x
        return "byte", B * (F * 4 + F * es + F * K * es + 4 + D * 4)
    if stage == "first_order_x":  # training: ids + w + rows + y + x
        return "byte", B * (F * 4 + F * es + F * K * es + 4 + D * 4)
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
    cin = cin_of(workload)
    if stage == "cin_back":  # dC_l and dZ_l GEMMs of every CIN layer
        hps = [F] + cin[:-1]
        return "flop", sum(4.0 * B * K * F * hp * h for hp, h in zip(hps, cin))
    if stage == "gather_x":
        return "byte", B * (F * 4 + F * K * es + D * 4)
    if stage in ("tower_layer1", "head_x"):  # head_x: training's encoder + layer 1 (k_head_s3.hip XS), the GEMM
        return "flop", 2.0 * B * k1 * FC[0]
    if stage == "tower_layer2":
        return "flop", 2.0 * B * FC[0] * FC[1]
    if stage == "tower_layer3":
        return "flop", 2.0 * B * FC[1] * FC[2] + 2.0 * B * FC[2]
    if stage in ("tower_small", "tower_fused"):  # the whole tower (+ the output dot) in one launch
        # (csrc/k_small_s3.hip, k_fused_s3.hip; the first order + FM sums ride along, not counted)
        return "flop", 2.0 * B * (k1 * FC[0] + FC[0] * FC[1] + FC[1] * FC[2] + FC[2])
    if stage == "tower_tail":  # layers 2 and 3 + the output dot in one launch (csrc/k_tail.hip, k_tail_s3.hip)
        return "flop", 2.0 * B * FC[0] * FC[1] + 2.0 * B * FC[1] * FC[2] + 2.0 * B * FC[2]
    if stage.startswith("cin_layer"):
        idx = {"cin_layer1": 0, "cin_layer2": 1, "cin_layer3+": 2}[stage]
        hp = F if idx == 0 else cin[idx - 1]
        return "flop", 2.0 * B * K * F * hp * cin[idx]
    return None, 0


def cin_exec_chunks(Fn, hp, first):
    """16-wide K chunks the split CIN executes for one layer (csrc/k_gemm.hip cin_chunk_map): per h-chunk of
    16 maps, one chunk per field -- layer 1 keeps fields f >= 16 hc only (the folded h <= f triangle) -- and an
    h-chunk with <= 8 live maps carries two fields per chunk."""
    n = 0
    for hc in range((hp + 15) // 16):
        live = min(16, hp - 16 * hc)
        nf = Fn - 16 * hc if first else Fn
        n += (nf + 1) // 2 if live <= 8 else nf
    return n


def stage_exec_flop(workload, stage, B):
    """FLOP the matrix cores execute per launch of a split-GEMM stage, padding and the chunk map included (the
    MFMA tiles issued, counted once per fp32 product like the algorithmic figure): beside stage_work's
    algorithmic FLOP, it tells the executed-MFMA fraction of the peak (the folded CIN layer 1
    runs 66 of its 117 K chunks, so its algorithmic rate overstates the hardware rate)."""
    np16 = lambda n: (n + 15) // 16 * 16
    if stage == "tower_fused":
        return 2.0 * B * ((F * K + 31) // 32 * 32 * np16(FC[0]) + 32 * ((FC[0] + 31) // 32) * np16(FC[1])
                          + 32 * ((FC[1] + 31) // 32) * np16(FC[2]))
    if stage.startswith("cin_layer"):
        cin = cin_of(workload)
        idx = {"cin_layer1": 0, "cin_layer2": 1, "cin_layer3+": 2}[stage]
        hp = F if idx == 0 else cin[idx - 1]
        return 2.0 * B * K * 16 * cin_exec_chunks(F, hp, idx == 0) * np16(cin[idx])
    return None


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ctypes as oc
    return oc


def _oracle_model(oc, workload):
    if workload.startswith("xdeepfm"):
        return oc.make_model(oc.XDEEPFM, F, K, fc=tuple(FC), cin=tuple(cin_of(workload)))
    if workload == "dcn_bf16":
        return oc.make_model(oc.DCN, F, K, fc=tuple(FC), cross_depth=3)
    if workload == "pnn_bf16":
        return oc.make_model(oc.PNN, F, K, fc=tuple(FC))
    return oc.make_model(oc.DEEPFM, F, K, fc=tuple(FC))


def cpu_baseline(workload, budget_s, threads):
    """Oracle (C restatement, OpenMP) on the host cores: examples/s on bounded batches, the gather
    (makeWeights / makeEmbeddings) included.  deepfm_sharded runs the same per-example CPU work on
    the V = 1M table (the host cannot hold the sharded table's point: it is the same math)."""
    oc = _oracle()
    if workload == "lr_plumbing":
        return cpu_baseline_plumbing(oc, budget_s, threads)
    om = _oracle_model(oc, workload)
    # the oracle parallelises over 8-row blocks (oracle/rmx_oracle.c RB): xDeepFM (~45 rows/s per thread)
    # takes 8 rows per thread per batch so every thread has a block
    B = 8 * max(threads, 1) if workload == "xdeepfm" else (64 * max(threads, 1) if workload == "xdeepfm_cin1" else 4096)
    mats = oc.init_mats(om, SEED_MATS)
    done, t_tot, row0 = 0, 0.0, 0
    wt, et = oc.gen_table(SEED_TAB, V, K)
    bf16 = workload.endswith("bf16")
    while t_tot < budget_s:
        ids = oc.gen_ids(SEED_IDS, row0, B, F, V).astype(np.int64)
        index = np.repeat(np.arange(B, dtype=np.int64), F)
        t0 = time.perf_counter()
        w, e = oc.gather(wt, et, 1, ids)
        oc.forward(om, B, index, np.array([0.01], np.float32), w, e, mats, 0, threads)
        t_tot += time.perf_counter() - t0
        done += B
        row0 += B
    return {"value": done / t_tot, "unit": "examples/s", "cores": threads, "kind": "port",
            "sample": "%d rows (%d batches of %d) of the same synthetic %s workload, fp32 oracle "
                      "(oracle/rmx_oracle.c, OpenMP, gather + forward%s), %.1f s"
                      % (done, done // B, B, workload, "; fp32 arithmetic on the bf16 model's shapes" if bf16 else "",
                         t_tot)}


def cpu_baseline_plumbing(oc, budget_s, threads):
    """configs[0] on the host: the Python restatement of SampleParser (tests/ref_parser.py) + the
    oracle's makeWeights gather and LR forward per 100-line batch + the AUC, over the 1k-row slice."""
    import ref_parser
    from test_metric import auc_ref
    from rmx import synthetic
    text, _, _ = synthetic.libsvm_text(SEED_IDS, SEED_LAB, 0, PLUMB_ROWS, F, V)
    lines = text.splitlines()
    wt, _ = oc.gen_table(SEED_TAB, V, 0)
    om = oc.make_model(oc.LR)
    bias = np.array([0.01], np.float32)
    done, t_tot = 0, 0.0
    while t_tot < budget_s:
        t0 = time.perf_counter()
        rows, cols, _, targets, _ = ref_parser.parse(lines)
        scores = np.zeros(PLUMB_ROWS, np.float32)
        for b0 in range(0, PLUMB_ROWS, PLUMB_BATCH):
            lo, hi = np.searchsorted(rows, [b0, b0 + PLUMB_BATCH])
            w, _ = oc.gather(wt, np.zeros((V, 0), np.float32), 1, cols[lo:hi])
            scores[b0:b0 + PLUMB_BATCH] = oc.forward(om, PLUMB_BATCH, rows[lo:hi] - b0, bias, w, None, None, 0,
                                                     threads)
        auc_ref(targets, scores)
        t_tot += time.perf_counter() - t0
        done += PLUMB_ROWS
    return {"value": done / t_tot, "unit": "examples/s", "cores": threads, "kind": "port",
            "sample": "%d passes over the 1k-row LIBSVM slice: Python SampleParser restatement "
                      "(tests/ref_parser.py) + oracle makeWeights + LR forward per 100-line batch "
                      "(oracle/rmx_oracle.c) + Mann-Whitney AUC, %.1f s" % (done // PLUMB_ROWS, t_tot)}


def parity_check(workload, got, row0, n=512, vocab=V, ids_host=None):
    """The checker beside the CPU baseline: GPU probabilities of rows [row0, row0 + n) of the bench
    set against the oracle on the same rows (fp64 oracle; bf16 workloads: the oracle's bf16-storage
    emulation, precision 2).  A V = 100M table is not materialised on the host: the
    oracle generates just the rows the checked ids use (same generator as the device)."""
    oc = _oracle()
    om = _oracle_model(oc, workload)
    if workload == "xdeepfm":
        n = min(n, 64)
    if workload == "xdeepfm_cin1":
        n = min(n, 256)
    mats = oc.init_mats(om, SEED_MATS)
    # (ids_host: the bench's own ids read back, e.g. the Zipf(1.1) set, which the oracle has no generator for)
    ids = (ids_host[:n * F] if ids_host is not None else oc.gen_ids(SEED_IDS, row0, n, F, vocab)).astype(np.int64)
    if vocab == V:
        wt, et = oc.gen_table(SEED_TAB, V, K)
        w, e = oc.gather(wt, et, 1, ids)
    else:
        w, e = oc.gen_rows(SEED_TAB, vocab, K, ids)
    index = np.repeat(np.arange(n, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    if workload.endswith("bf16"):
        ref = oc.forward(om, n, index, bias, oc.round_bf16(w), oc.round_bf16(e), mats, 2)
        tol, against = 2e-4, "oracle bf16-storage emulation (precision 2)"
    else:
        ref = oc.forward(om, n, index, bias, w, e, mats, 1)
        tol, against = 1e-5, "fp64 oracle"
    err = float(np.abs(got[:n] - ref).max())
    return {"rows": n, "row0": row0, "max_abs_diff": err, "tol": tol, "against": against, "ok": err <= tol}


# exit status of a rank whose line reports a failed check (after the line is printed): the driver and
# launch_ranks see it, not only a string inside the line
STATUS_PARITY_MISS = 5
STATUS_COMPANION_FAILED = 6
STATUS_RECORD_ERROR = 7
STATUS_REASON = {STATUS_PARITY_MISS: "parity miss", STATUS_COMPANION_FAILED: "sharded sub-record failed",
                 STATUS_RECORD_ERROR: "encoder / L-A sub-record raised"}


def _pc_ok(p):
    """one rank's parity record: {"ok": ...} or {"deepfm": {...}, "xdeepfm": {...}}"""
    if p is None:
        return True
    return p["ok"] if "ok" in p else all(q["ok"] for q in p.values())


def job_status(parity_ranks=None, sub=None, cpu=None, cpu2=None):
    """The status every rank exits with once the line is out: STATUS_PARITY_MISS when any rank's rows missed
    the oracle (the main workload, its xDeepFM companion or the sharded sub-record), STATUS_COMPANION_FAILED
    when the sharded sub-record raised (its watchdog exits 124 itself), else 0.  parity_ranks and the
    sub-record's checks are gathered over the ranks, so every rank computes the same status."""
    if parity_ranks and not all(_pc_ok(p) for p in parity_ranks):
        return STATUS_PARITY_MISS
    for c in (cpu, cpu2):
        if c and c.get("parity_check") and not c["parity_check"]["ok"]:
            return STATUS_PARITY_MISS
    if sub is not None:
        if "error" in sub:
            return STATUS_COMPANION_FAILED
        if not sub.get("parity_ok", True):
            return STATUS_PARITY_MISS
    return 0


def record_status(*recs):
    """Status of rank 0's encoder / L-A sub-records ({"V1M": {...}, ...} or {"B100": {...}, ...}): an entry
    that raised is STATUS_RECORD_ERROR (not a parity miss), a failed check STATUS_PARITY_MISS."""
    st = 0
    for rec in recs:
        for k_, e in (rec or {}).items():
            if not isinstance(e, dict):
                continue
            if "error" in e:
                return STATUS_RECORD_ERROR
            pc = e.get("parity_check", {})
            if not (pc.get("bitwise_equal", False) if k_.startswith("V") else pc.get("ok", False)):
                st = STATUS_PARITY_MISS
    return st


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_counts():
    """(logical CPUs of the machine, CPUs this process may run on, cgroup CPU quota or None, physical
    cores): the box shows the whole machine's CPUs while its cgroup grants a share of them."""
    logical = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = logical
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    phys = set()
    try:
        pid = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                pid = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
                phys.add((pid, core))
    except OSError:
        pass
    return logical, avail, quota, len(phys) or None


def cpu_baseline_sweep(workload, budget_s, short=False):
    """The baseline at all the cores this job may use (the reported value), plus 1 and 2 threads
    (Spark local[1] / local[2] analogues) on shorter bounded samples."""
    logical, avail, quota, phys = cpu_counts()
    allc = min(avail, quota) if quota else avail
    if workload == "lr_plumbing":
        res = cpu_baseline(workload, budget_s, 2)  # configs[0] is the Spark local[2] run
        res["by_threads"] = {"2": round(res["value"], 1)}
    else:
        res = cpu_baseline(workload, budget_s, allc)
        res["by_threads"] = {str(allc): round(res["value"], 1)}
        for t in (() if short else (1, 2)):
            if t < allc:
                res["by_threads"][str(t)] = round(cpu_baseline(workload, max(2.0, budget_s * 0.3), t)["value"], 1)
    res["cpu_model"] = cpu_model()
    res["logical_cpus"] = logical
    res["physical_cores"] = phys
    res["cpus_in_affinity"] = avail
    res["cgroup_cpu_quota"] = quota
    res["cores_note"] = ("all cores available to this job: min(affinity, cgroup quota)"
                         if workload != "lr_plumbing" else "Spark local[2]: 2 threads")
    return res


def make_model(rmx, workload, Vw, ctx):
    base = workload[:-len("_train")] if workload.endswith("_train") else workload
    if base in ("xdeepfm", "xdeepfm_cin1"):
        return rmx.XDeepFM(Vw, F, K, FC, cin_of(base), ctx=ctx)
    if base == "dcn_bf16":  # configs[4]: DCN depth 3 + fcDims 400^3, bf16 table / weights
        return rmx.DCN(Vw, F, K, 3, FC, ctx=ctx)
    if base == "pnn_bf16":  # configs[4]: PNN (IPNN) D1 = 400, fcDims 400^3, bf16
        return rmx.PNN(Vw, F, K, FC, ctx=ctx)
    if base == "lr_plumbing":
        return rmx.LR(Vw, F, ctx=ctx)
    return rmx.DeepFM(Vw, F, K, FC, ctx=ctx)


def run_plumbing(args, rmx, ctx, rank, world, dist, steps, warmup):
    """configs[0]: one step = one pass over a 1k-row LIBSVM slice (example/LRLocalExample.scala:13-58):
    native parse at 2 threads (Spark local[2]) -> ids + labels to HBM -> LR predict loop of
    100-row forwards (ParRecModel.predict, batchSize 100) -> device AUC."""
    from rmx import synthetic
    text, _, _ = synthetic.libsvm_text(SEED_IDS, SEED_LAB, rank * PLUMB_ROWS, PLUMB_ROWS, F, V)
    blob = text.encode()
    model = make_model(rmx, "lr_plumbing", V, ctx)
    table = rmx.EmbeddingTable(ctx, V, 0)
    table.fill_synthetic(SEED_TAB)
    model.setBias(0.01)
    ids = rmx.DeviceArray(ctx, PLUMB_ROWS * F, np.int32)
    lab = rmx.DeviceArray(ctx, PLUMB_ROWS, np.float32)
    scores = rmx.DeviceArray(ctx, PLUMB_ROWS, np.float32)
    stream = ctx.stream
    res = {}

    def step():
        s = rmx.Samples(blob, rmx.FORMAT_LIBSVM, 2)
        ids.upload(s.ids(F))
        lab.upload(s.targets)
        model.predict_ids(table, PLUMB_ROWS, ids, scores, batch=PLUMB_BATCH, stream=stream)
        res["auc"] = rmx.auc(ctx, lab, scores, stream=stream)  # synchronises

    for _ in range(warmup):
        step()
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    t_rank = time.perf_counter() - t0
    if dist:
        dist.barrier()
    t_rank = max_over_ranks(dist, t_rank)
    model.set_timing(True)
    step()
    stages, calls = model.get_timing()
    model.set_timing(False)
    B = PLUMB_ROWS
    per_stage = {n: {"avg_ms_per_pass": round(t, 4)} for n, t in stages.items()}
    kind, work = stage_work("lr_plumbing", "first_order_sigmoid", PLUMB_BATCH)
    launches = PLUMB_ROWS // PLUMB_BATCH
    avg_s = stages.get("first_order_sigmoid", 0.0) / 1e3 / launches
    roof = {"bound": "hbm", "achieved": round(work / avg_s / 1e9, 2) if avg_s else None, "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(work / avg_s / 1e9 / PEAK_HBM_GBS, 6) if avg_s else None,
            "traffic": None, "kernel": "first_order_sigmoid", "algorithmic_per_launch": work,
            "note": "100-row launches: latency-bound plumbing (the parse on the host dominates the pass)"}
    return {"value": world * B * steps / t_rank, "ms_per_step": t_rank * 1e3 / steps, "B": B, "Vw": V,
            "nrows": PLUMB_ROWS, "roofline": roof, "stages": per_stage, "auc": res.get("auc"),
            "out": scores.numpy()}


def max_over_ranks(dist, t):
    if not dist:
        return t
    import torch
    x = torch.tensor([t], dtype=torch.float64)
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    return float(x.item())


ENC_VOCABS = (1_000_000, 100_000_000)


def run_encoder(args, rmx, ctx, steps, warmup, Vw, B=65536):
    """The encoder alone (rmx_encoder_ids: gather + first order + FM of DeepFM, encoder_k16v2_kernel) at
    vocabulary Vw, with the [V][k] row table + [V] weights and with the [V][32] line copy (one 128-B line per
    id: knob table_lines), timed with HIP events on its stream: examples/s, algorithmic GB/s (2,812 B per
    example) against the 8 TB/s HBM peak, and the 128-B line rate (a random 64-B row or 4-B
    weight costs one full line: profiles/r02/fetch_calib.txt).  Bit-exact parity of y against the oracle's
    first order + FM on rows of the first batch (V = 1M: the host table; V = 100M: the generated rows)."""
    import ctypes
    m = rmx.DeepFM(Vw, F, K, FC, ctx=ctx)
    table = rmx.EmbeddingTable(ctx, Vw, K)
    table.fill_synthetic(SEED_TAB)
    nb = 16
    ids = rmx.DeviceArray(ctx, nb * B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, nb * B, F, Vw, ids)
    y = rmx.DeviceArray(ctx, nb * B, np.float32)
    ctx.sync()
    stream = ctx.stream
    lib = rmx._lib.lib
    ev0, ev1 = ctypes.c_void_p(), ctypes.c_void_p()
    lib.rmx_event_create(ctypes.byref(ev0))
    lib.rmx_event_create(ctypes.byref(ev1))
    bpe = F * 4 + F * 4 + F * K * 4 + 4
    rec = {"kernel": ("encoder_k16v2_kernel (enc_u %d)" % rmx.get_tuning("enc_u", 20)) if rmx.get_tuning("enc_u", 20)
           else "encoder_k16_kernel<1, float>", "batch": B, "vocab": Vw,
           "algorithmic_bytes_per_example": bpe, "peak_gbs": PEAK_HBM_GBS}
    saved = rmx.get_tuning("table_lines", 0)
    layouts = {"row": (0,), "line": (1,)}.get(getattr(args, "enc_table", "both"), (0, 1))
    try:
        for lines in layouts:
            rmx.set_tuning("table_lines", lines)
            table.refresh_lines()
            ctx.sync()
            t_end = time.perf_counter() + 0.3
            i = 0
            while time.perf_counter() < t_end:  # clock settle
                for _ in range(8):
                    m.encoder_ids(table, B, ids.view((i % nb) * B * F, B * F), y.view((i % nb) * B, B), stream)
                    i += 1
                ctx.sync()
            for j in range(warmup):
                m.encoder_ids(table, B, ids.view((j % nb) * B * F, B * F), y.view((j % nb) * B, B), stream)
            lib.rmx_event_record(ev0, stream)
            for j in range(steps):
                m.encoder_ids(table, B, ids.view((j % nb) * B * F, B * F), y.view((j % nb) * B, B), stream)
            lib.rmx_event_record(ev1, stream)
            ctx.sync()
            ms = ctypes.c_float()
            lib.rmx_event_elapsed_ms(ev0, ev1, ctypes.byref(ms))
            avg_s = ms.value / 1e3 / steps
            lines_per_ex = F if lines else 2 * F  # + the ids' own lines (156 B per example, streamed)
            ent = {"avg_ms": round(avg_s * 1e3, 4), "examples_per_s": round(B / avg_s, 1),
                   "achieved_gbs": round(B * bpe / avg_s / 1e9, 1),
                   "frac": round(B * bpe / avg_s / 1e9 / PEAK_HBM_GBS, 4),
                   "lines_per_example": lines_per_ex,
                   "line_gbs": round(B * (lines_per_ex * 128 + F * 4 + 4) / avg_s / 1e9, 1),
                   "line_frac": round(B * (lines_per_ex * 128 + F * 4 + 4) / avg_s / 1e9 / PEAK_HBM_GBS, 4)}
            # HBM bytes per launch from the committed rocprofv3 PMC passes of this exact record
            # (tools/gpu_check.sh pmcenc, tools/pmc_summary.py --stages: FETCH_SIZE x 2 + WRITE_SIZE)
            tkey = "encoder_V%dM_%s" % (Vw // 1_000_000, "line" if lines else "row")
            tent = _traffic(tkey, "encoder", B)
            ent["traffic"] = tent["hbm_bytes"] if tent else None
            if tent:
                ent["traffic_per_example"] = round(tent["hbm_bytes"] / B, 1)
                ent["traffic_over_algorithmic"] = round(tent["hbm_bytes"] / (B * bpe), 3)
                ent["traffic_source"] = "profiles/traffic.json %s (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE)" % tkey
                if "avg_ns" in tent:  # the same launches' kernel-trace duration under the profiler
                    ent["pmc_pass_avg_ms"] = round(tent["avg_ns"] / 1e6, 4)
            rec["line_table" if lines else "row_table"] = ent
        # parity (bit-exact) on the layout timed last: rows [0, n) of the first batch, y = y1 + y2 from the
        # oracle's own gather + sums
        m.encoder_ids(table, B, ids.view(0, B * F), y.view(0, B), stream)
        ctx.sync()
    finally:
        rmx.set_tuning("table_lines", saved)
    got = y.numpy()[:256]
    oc = _oracle()
    n = 256
    h_ids = ids.numpy()[:n * F].astype(np.int64)
    if Vw == V:
        wt, et = oc.gen_table(SEED_TAB, V, K)
        w, e = oc.gather(wt, et, 1, h_ids)
    else:
        w, e = oc.gen_rows(SEED_TAB, Vw, K, h_ids)
    ref = (oc.first_order(n, np.repeat(np.arange(n, dtype=np.int64), F), w) + oc.fm(n, F, K, e)).astype(np.float32)
    rec["parity_check"] = {"rows": n, "bitwise_equal": bool(np.array_equal(got, ref)),
                           "max_abs_diff": float(np.abs(got - ref).max()), "against": "oracle first order + FM (fp32)"}
    table.close()
    return rec


def _traffic(workload, stage, B):
    """profiles/traffic.json entry of (workload, stage) when it was profiled at batch B, else None."""
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(tpath):
        return None
    ent = json.load(open(tpath)).get(workload, {}).get(stage)
    return ent if ent and ent.get("batch") == B else None


def encoder_record(args, rmx, ctx, steps, warmup):
    """models.encoder of the default line: the encoder alone at V = 1M (Infinity-Cache resident) and 100M."""
    out = {"note": ("the DeepFM forward fuses this encoder into tower layer 1 (k_fused_s3.hip); timed alone here "
                    "for its HBM roofline (north_star, SURVEY.md §8d)")}
    for Vw in ENC_VOCABS:
        try:
            out["V%dM" % (Vw // 1_000_000)] = run_encoder(args, rmx, ctx, steps, warmup, Vw)
        except Exception as e:
            out["V%dM" % (Vw // 1_000_000)] = {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}
    return out


LA_BATCHES = (100, 4096, 65536)  # 100 = the reference's batchSize (example/DeepFMLocalExample.scala:16)


def run_la(args, rmx, ctx, B, calls):
    """L-A: rmx_forward, the exact RecModel.forward host-array contract (RecModel.scala:37-48,
    ParRecModel.scala:555-567) -- COO index / feats, the gathered first-order weights [nnz] and embeddings
    [nnz][k], and the whole mats array with EVERY call, as the Scala side would hand them over through JNI
    (pageable host memory) -- timed end to end on the host clock (arrays in, probabilities out), plus its
    stages from HIP events: la_mats (mats H2D + pack), la_h2d (rows / weights H2D), the forward's kernels
    and la_d2h.  The host arrays are the device table's own rows (rmx_gather), so the forward sees the same
    inputs as the L-B line; parity against the fp64 oracle, and bitwise against L-B on the same rows."""
    m = rmx.DeepFM(V, F, K, FC, ctx=ctx)
    mats = m.initMats(SEED_MATS)
    sizes = np.asarray(m.getMatsSize(), np.int32)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    nnz = B * F
    ids = rmx.DeviceArray(ctx, nnz, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    w_d = rmx.DeviceArray(ctx, nnz, np.float32)
    e_d = rmx.DeviceArray(ctx, nnz * K, np.float32)
    table.gather(ids, nnz, w_d, e_d)
    ctx.sync()
    feats = ids.numpy().astype(np.int64)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    w, e = w_d.numpy(), e_d.numpy()
    bias = np.array([0.01], np.float32)
    batch = rmx.CooLongFloatMatrix(index, feats)

    def call():
        return m.forward(B, batch, bias, w, e, K, mats, sizes)

    for _ in range(max(3, calls // 10)):
        out = call()
    t0 = time.perf_counter()
    for _ in range(calls):
        out = call()
    wall = (time.perf_counter() - t0) / calls
    m.set_timing(True)
    nt = max(3, min(calls, 20))
    for _ in range(nt):
        call()
    stages, ncalls = m.get_timing()
    m.set_timing(False)
    st = {n: round(t / max(ncalls, 1), 4) for n, t in stages.items()}
    kern = sum(v for n, v in st.items() if not n.startswith("la_"))
    # L-B on the same rows and table (forward_ids), for the bitwise comparison
    m.setMats(mats)
    m.setBias(0.01)
    o_d = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids, o_d)
    ctx.sync()
    lb = o_d.numpy()
    mats_b = 4 * len(mats)
    rows_b = 4 * nnz * (K + 1)
    pc = parity_check("deepfm", out, 0, n=min(B, 512))
    rec = {"batch": B, "calls": calls, "wall_ms_per_call": round(wall * 1e3, 4),
           "examples_per_s": round(B / wall, 1), "stages_ms": st, "kernels_ms": round(kern, 4),
           "h2d_bytes_per_call": {"mats": mats_b, "rows_and_weights": rows_b},
           "h2d_gbs": round((mats_b + rows_b) / ((st.get("la_mats", 0) + st.get("la_h2d", 0)) / 1e3) / 1e9, 1)
           if st.get("la_h2d") else None,
           "pcie_cap_examples_per_s": round(63e9 / (4 * F * (K + 1)), 1),
           "parity_check": pc, "bitwise_vs_lb": bool(np.array_equal(out, lb))}
    table.close()
    m.close()
    return rec


def la_record(args, rmx, ctx):
    """models.deepfm_la of the default line: the L-A drop-in (host arrays) at B = 100 / 4,096 / 65,536."""
    out = {"note": ("rmx_forward: the RecModel.forward host-array contract through librmx (what the JNI shim "
                    "calls); SURVEY.md §8b prices its cap at PCIe: (16 + 1) x 4 B x 39 per example at 63 GB/s "
                    "= 23.8 M examples/s, before the per-call mats")}
    for B in LA_BATCHES:
        try:
            out["B%d" % B] = run_la(args, rmx, ctx, B, {100: 200, 4096: 50}.get(B, 10))
        except Exception as e:
            out["B%d" % B] = {"error": "%s: %s" % (type(e).__name__, str(e)[:300])}
    return out


LIVE_SHARDS = []  # sharded tables of this process (the companion watchdog aborts their communicators)


def run(args, workload, rmx, ctx, rank, world, dist, steps, warmup, B=0):
    """Builds the workload, times K steps after W warm-up steps (max over ranks), then measures the
    per-stage kernel times (HIP events on the launch stream) for the roofline of the dominant kernel."""
    if workload == "lr_plumbing":
        return run_plumbing(args, rmx, ctx, rank, world, dist, steps, warmup)
    train = workload.endswith("_train")
    B = B or args.batch or ({"xdeepfm": 16384, "xdeepfm_cin1": 65536, "xdeepfm_train": 4096}.get(workload, 65536))
    sharded = workload == "deepfm_sharded"
    Vw = args.vocab or (100_000_000 if sharded else V)
    stream = ctx.stream
    bf16 = workload.endswith("bf16")
    model = make_model(rmx, workload, Vw, ctx)
    if bf16:
        model.setPrecision(rmx.DTYPE_BF16)
    table = None
    if sharded:
        # configs[3]: table hash-sharded over the ranks, RCCL exchange per batch
        # RCCL prints its version banner on fd 1 at init; keep stdout for the one JSON line
        with stdout_to_stderr():
            uid = rmx.comm_unique_id() if rank == 0 else None
            if dist:
                box = [uid]
                dist.broadcast_object_list(box, src=0)
                uid = box[0]
            table = rmx.ShardedTable(ctx, Vw, K, world, rank, uid)
            LIVE_SHARDS.append(table)
        table.set_dedupe(False if args.no_dedupe else (True if args.dedupe_on else "auto"))
        table.set_batch_hint(B * F)  # every rank the same B: the first exchange skips the overflow round
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

    # deepfm_sharded, overlapped (default): rmx_shard_pull of batch j + 1 into the other pull slot on
    # a second stream while rmx_forward_pulled runs batch j; every step still does one exchange and
    # one forward (the first batch's pull happens in the step before it)
    overlap = sharded and not args.no_overlap
    pipe = {"j": 0, "pulled": False}
    ctx_x = rmx.Context(ctx.device) if overlap else None

    def step_overlap():
        # forward j is enqueued first, so the host-side part of pull j + 1 (at N > 1 the counts round
        # trip and its stream sync) runs while the GPU computes batch j
        j = pipe["j"]
        if not pipe["pulled"]:
            table.pull(views[j % nb][0], B * F, j % 2, ctx_x.stream)
        model.forward_pulled(table, B, j % 2, views[j % nb][1], stream)
        table.pull(views[(j + 1) % nb][0], B * F, (j + 1) % 2, ctx_x.stream)
        pipe["j"], pipe["pulled"] = j + 1, True

    def drain():
        if overlap and pipe["pulled"]:
            j = pipe["j"]
            model.forward_pulled(table, B, j % 2, views[j % nb][1], stream)
            pipe["j"], pipe["pulled"] = j + 1, False
            ctx.sync()
            ctx_x.sync()

    def step(i):
        ids_v, out_v = views[i % nb]
        if train:
            model.backward_ids(table, B, ids_v, tviews[i % nb], g_b, g_w, g_e, g_m, g_loss, stream)
        elif overlap:
            step_overlap()
        elif sharded:
            model.forward_ids_sharded(table, B, ids_v, out_v, stream)
        else:
            model.forward_ids(table, B, ids_v, out_v, stream)

    # clock settle: an idle MI355X ramps its clocks over the first ~0.1-0.3 s of load, so 5 warm-up
    # steps (~2 ms) leave the timed steps on a cold clock.  Untimed, before the W
    # warm-up steps; the K timed steps are unchanged.
    settle = 0
    if args.settle_ms > 0:
        ctx.sync()
        t_s = time.perf_counter()
        # every sharded step at N > 1 is a collective (the exchange): the ranks must run the same
        # number of them, so they agree each round on going on (any rank still under the budget)
        agree = sharded and dist is not None
        while True:
            more = (time.perf_counter() - t_s) * 1e3 < args.settle_ms
            if agree:
                more = max_over_ranks(dist, 1.0 if more else 0.0) > 0.5
            if not more:
                break
            for _ in range(8):
                step(settle)
                settle += 1
            ctx.sync()
    for i in range(warmup):
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
    for i in range(steps):
        step(warmup + i)
    rmx._lib.lib.rmx_event_record(ev1, stream)
    ctx.sync()
    if overlap:
        ctx_x.sync()
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    ms = ctypes.c_float()
    rmx._lib.lib.rmx_event_elapsed_ms(ev0, ev1, ctypes.byref(ms))
    t_rank = max_over_ranks(dist, max(wall, ms.value / 1e3))
    value = world * B * steps / t_rank

    drain()  # (overlap) the pull of the batch after the last timed one
    # ---- roofline of the dominant kernel: per-stage HIP events on the launch stream ----
    # (deepfm_sharded: measured on the one-stream path, exchange and forward in sequence)
    model.set_timing(True)
    if overlap:
        overlap, saved = False, overlap
    nt = max(5, min(steps, 20))
    for i in range(nt):
        step(i)
    ctx.sync()
    stages, calls = model.get_timing()
    model.set_timing(False)
    if sharded and not args.no_overlap:
        overlap = saved
    split = not bf16 and rmx.get_tuning("f32_split", 1) != 0

    def peak_of(stage):
        if bf16:
            return PEAK_BF16_TFLOPS
        return PEAK_S3_TFLOPS if split and stage.startswith(S3_STAGES) else PEAK_FP32_TFLOPS

    # one rank without dedupe: the sharded table is read in place (csrc/shard.hip direct_eligible)
    direct = sharded and world == 1 and not args.dedupe_on
    per_stage = {}
    for name, tot in stages.items():
        avg_ms = tot / max(calls, 1)
        kind, work = stage_work(workload, name, B, direct)
        ent = {"avg_ms": round(avg_ms, 4)}
        if kind == "flop":
            ent["tflops"] = round(work / (avg_ms / 1e3) / 1e12, 2)
            ent["frac_mfma_peak"] = round(ent["tflops"] / peak_of(name), 3)
            ex = stage_exec_flop(workload, name, B) if split else None
            if ex:
                ent["executed_tflops"] = round(ex / (avg_ms / 1e3) / 1e12, 2)
                ent["executed_frac"] = round(ent["executed_tflops"] / peak_of(name), 3)
        elif kind == "byte":
            ent["gbs"] = round(work / (avg_ms / 1e3) / 1e9, 1)
            ent["frac_hbm_peak"] = round(ent["gbs"] / PEAK_HBM_GBS, 3)
        per_stage[name] = ent
    stage_sum = sum(stages.values()) / max(calls, 1)
    dom = max(stages.items(), key=lambda kv: kv[1])[0]
    kind, work = stage_work(workload, dom, B, direct)
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
    ent = _traffic(workload, dom, B) or (_traffic(workload, "cin_layer", B) if dom.startswith("cin_layer") else None)
    if ent:
        roof["traffic"] = ent["hbm_bytes"]
        roof["traffic_source"] = "profiles/traffic.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE), %s" % ent.get(
            "source", "")
        roof["traffic_kernel"] = ent.get("kernel")
        if "mfma_util" in ent:  # measured matrix-pipe occupancy of the same kernel (profiled run)
            roof["mfma_util_pmc"] = ent["mfma_util"]
            roof["mfma_util_source"] = ("rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs), "
                                        "%s" % ent.get("source", ""))
            if "clock_ghz" in ent:
                roof["pmc_clock_ghz"] = ent["clock_ghz"]
    roof["kernel"] = dom
    roof["algorithmic_per_launch"] = work
    if "executed_frac" in per_stage.get(dom, {}):
        roof["executed_frac"] = per_stage[dom]["executed_frac"]
        roof["executed_note"] = ("the MFMA tiles the kernel issues (K / N padding, the CIN chunk map) over the same "
                                 "time, against the same peak; frac counts the algorithmic FLOP only")

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
    elif sharded:
        model.forward_ids_sharded(table, B, views[0][0], views[0][1], stream)  # rows [0, B) again, for parity
        ctx.sync()
    res = {"value": value, "ms_per_step": t_rank * 1e3 / steps, "B": B, "Vw": Vw, "nrows": nrows,
           "roofline": roof, "stages": per_stage, "stage_sum_ms": round(stage_sum, 4), "predict_auc": pa,
           "settle_steps": settle,
           "out": out.numpy()[:512], "bf16": bf16, "split": split,
           "ids_head": ids.numpy()[:512 * F] if args.zipf else None}
    if sharded:
        res["exchange"] = {"dedupe": "off" if args.no_dedupe else ("on" if args.dedupe_on else "auto"),
                           "mode": ("one rank: the batch's ids map to partition rows p(id) and the forward reads "
                                    "the [emb | w | pad] lines in place (no exchange, no row copy)") if direct else
                                   "RCCL exchange (ids to owners, rows back)",
                           "owner_map": "keyed Feistel permutation p (rmx.OWNER_HASH_DEFAULT): owner = p(id) mod N",
                           "ids_sent_last_step": table.last_sent(),
                           "nnz_per_step": B * F,
                           "overlap": ("batch i + 1's exchange (rmx_shard_pull) on a second stream beside batch i's "
                                       "forward (rmx_forward_pulled)") if not args.no_overlap else "none (one stream)",
                           "table_rows": "[emb 16 | w | pad] fp32, 128 B: one memory line per id"}
    return res


def config_of(workload, r, world, zipf):
    base = workload[:-len("_train")] if workload.endswith("_train") else workload
    Vw, B = r["Vw"], r["B"]
    if workload == "lr_plumbing":
        return {"workload": "lr_plumbing_F39_V1M_libsvm1k_B100", "global_batch": world * PLUMB_BATCH,
                "rows_per_gpu_set": PLUMB_ROWS, "ids": "uniform", "parallelism": "replicas%d" % world,
                "step": "parse (2 threads) + ids to HBM + 10 LR forwards of 100 rows + AUC"}
    return {"workload": "%s%s_F39_V%s_k16_fc400x3%s_B%d" % (
        workload, "" if r["bf16"] else "_fp32",
        ("%dM" % (Vw // 1_000_000)) if Vw % 1_000_000 == 0 else str(Vw),
        {"xdeepfm": "_cin200x3", "xdeepfm_cin1": "_cin200x1", "dcn_bf16": "_cross3"}.get(base, ""), B),
        "global_batch": world * B, "rows_per_gpu_set": r["nrows"],
        "ids": ("zipf%g" % zipf) if zipf else "uniform",
        "parallelism": ("hashshard%d_rccl" % world) if workload == "deepfm_sharded" else "replicas%d" % world}


class stdout_to_stderr:
    """fd 1 -> fd 2 for a block (library banners: gloo, RCCL), so stdout carries only the JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv, script=None, grace_s=10.0):
    """`--gpus N` without an external launcher: start N fresh rank processes of `script` (this file)
    with the torch.distributed env (RANK, LOCAL_RANK = rank, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a
    free MASTER_PORT), relay rank 0's stdout (the one JSON line) and return the job's exit status: 0
    when every rank exits 0, else the first failing rank's status, after the other ranks are stopped
    (SIGTERM, then SIGKILL after grace_s).  Only child processes are started (no exec) and this
    process touches no GPU: each rank initialises its own device."""
    import signal
    import subprocess
    import threading
    script = os.path.abspath(script or __file__)
    port = _free_port()
    procs, out0 = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))

    def pump():  # rank 0's stdout, read while it runs (a full pipe would block the rank)
        for line in procs[0].stdout:
            out0.append(line)

    def forward(signum, _frame):  # a launcher stopped by its caller stops (and reaps) its ranks: no orphans
        for pr in procs:
            if pr.poll() is None:
                pr.send_signal(signum)
        t_end = time.time() + grace_s
        for pr in procs:
            try:
                pr.wait(max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                pr.kill()
                pr.wait()
        raise SystemExit(128 + signum)
    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    status = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                sys.stderr.write("bench.py: rank %d exited with status %d; stopping the other ranks\n" % (r, rc))
                for q in live:
                    procs[q].send_signal(signal.SIGTERM)
                t_end = time.time() + grace_s
                for q in list(live):
                    try:
                        procs[q].wait(max(0.1, t_end - time.time()))
                    except subprocess.TimeoutExpired:
                        procs[q].kill()
                        procs[q].wait()
                live.clear()
                break
        time.sleep(0.05)
    th.join(5.0)
    for line in out0:
        sys.stdout.write(line.decode(errors="replace"))
    sys.stdout.flush()
    return status


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # this process is the launcher only: the ranks are fresh children (no GPU call here)
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # CPU (gloo) barrier / max only: the GPU work is librmx
        with stdout_to_stderr():  # gloo prints a connection banner on fd 1: stdout is the JSON line
            dist.init_process_group("gloo")
    import rmx
    for kv in filter(None, args.set.split(",")):
        k_, v_ = kv.split("=")
        rmx.set_tuning(k_, int(v_))

    train = args.workload.endswith("_train")
    # one rank per GPU; fewer GPUs than ranks (a rehearsal on a 1-GPU box) wraps ranks onto them
    # (torch.cuda.device_count() does not initialise the GPU on this image)
    ndev = 1
    if world > 1:
        import torch
        ndev = max(1, torch.cuda.device_count())
    if args.workload == "deepfm_sharded" and world > ndev:
        sys.stderr.write("bench.py: deepfm_sharded needs one GPU per rank (%d ranks, %d GPU(s) visible): RCCL "
                         "rejects ranks sharing a GPU\n" % (world, ndev))
        if dist:
            dist.destroy_process_group()
        raise SystemExit(3)
    rmx.set_device(local % ndev)
    ctx = rmx.default_context()

    if args.workload == "encoder":
        # the encoder alone (profiling / its own line): V = --vocab (default 100M), B = --batch (65,536)
        Vw = args.vocab or 100_000_000
        rec = run_encoder(args, rmx, ctx, args.steps, args.warmup, Vw, B=args.batch or 65536)
        if rank == 0:
            lay = "row_table" if "row_table" in rec else "line_table"
            ent = rec[lay]
            print(json.dumps({
                "metric": "encoder (gather + first order + FM) examples/sec", "value": ent["examples_per_s"],
                "unit": "examples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": ent["avg_ms"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "f32", "data": "synthetic", "config": {"workload": "encoder_fp32_F39_V%s_k16_B%d_%s" % (
                    ("%dM" % (Vw // 1_000_000)) if Vw % 1_000_000 == 0 else Vw, rec["batch"], lay)},
                "roofline": {"bound": "hbm", "achieved": ent["achieved_gbs"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": ent["frac"], "traffic": ent.get("traffic"), "kernel": rec["kernel"]},
                "encoder": rec}), flush=True)
        if dist:
            dist.destroy_process_group()
        raise SystemExit(0 if rec["parity_check"]["bitwise_equal"] else STATUS_PARITY_MISS)
    r = run(args, args.workload, rmx, ctx, rank, world, dist, args.steps, args.warmup)
    # BASELINE.json's metric names DeepFM AND xDeepFM: the default line measures both (xDeepFM as a
    # sub-record with its own steps, roofline, parity and CPU baseline; configs[2])
    companion = None
    if args.workload == "deepfm" and not args.no_companion:
        companion = run(args, "xdeepfm", rmx, ctx, rank, world, dist, args.steps, args.warmup, B=16384)
    cpu = cpu2 = None
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline and not train and not args.parity_only
    if rank == 0 and world == 1 and args.parity_only and not train and args.workload != "lr_plumbing":
        cpu = {"parity_check": parity_check(args.workload, r["out"], 0, vocab=r["Vw"], ids_host=r.get("ids_head"))}
        if companion:
            cpu2 = {"parity_check": parity_check("xdeepfm", companion["out"], 0)}
    if want_cpu:
        cpu = cpu_baseline_sweep(args.workload, args.cpu_seconds)
        if args.workload == "lr_plumbing":
            pass
        elif args.workload == "deepfm_sharded" and not args.zipf:
            cpu["parity_check"] = parity_check(args.workload, r["out"], 0, vocab=r["Vw"])
        elif r["Vw"] == V and not args.zipf:
            # out holds the predict loop's probabilities of the whole rank-0 row set
            cpu["parity_check"] = parity_check(args.workload, r["out"], 0)
        if companion:
            cpu2 = cpu_baseline_sweep("xdeepfm", max(3.0, args.cpu_seconds * 0.5))
            cpu2["parity_check"] = parity_check("xdeepfm", companion["out"], 0)

    # N > 1: every rank checks rows of its own bench set against the oracle (after timing), rank 0
    # reports them all
    parity_ranks = None
    if world > 1 and not train and args.workload != "lr_plumbing" and not args.zipf:
        pc = parity_check(args.workload, r["out"], rank * r["nrows"], vocab=r["Vw"])
        if companion:
            pc = {"deepfm": pc, "xdeepfm": parity_check("xdeepfm", companion["out"], rank * companion["nrows"])}
        parity_ranks = [None] * world
        dist.all_gather_object(parity_ranks, pc)

    if rank == 0:
        line = {
            "metric": ("CTR-train examples/sec (forward + RecModel.backward gradients; the optimizer lives on "
                       "the parameter server, out of scope)") if train else
                      "CTR-forward examples/sec on Criteo-shaped batch, DeepFM & xDeepFM, 1/2/4/8 GPU",
            "value": round(r["value"], 1),
            "unit": "examples/s",
            "n_gpus": world,
            **({"gpus_visible": ndev, "note_ranks": "%d ranks share %d visible GPU(s) (rehearsal, not a "
                                                    "scaling point)" % (world, ndev)} if world > ndev else {}),
            "steps": args.steps,
            "warmup": args.warmup,
            **({"settle": {"ms": args.settle_ms, "untimed_steps": r["settle_steps"]}} if "settle_steps" in r else {}),
            "ms_per_step": round(r["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16 (fp32 accumulate)" if r.get("bf16") else "f32",
            **({"gemm_arith": "fp32 operands and accumulation; products on v_mfma_f32_16x16x32_bf16 via the exact "
                              "3-way bf16 split (6 products, dropped terms <= 2^-24 |xy|; parity vs the fp64 oracle "
                              "identical to the f32 MFMA engine)"} if r.get("split") else {}),
            "data": ("synthetic (splitmix64 Criteo-shaped ids, U(-0.05,0.05) table, Xavier mats)"
                     + ("; LIBSVM text of the same ids, Bernoulli(0.25) labels" if args.workload == "lr_plumbing"
                        else "")),
            "config": config_of(args.workload, r, world, args.zipf),
            **({"table_layout": "[V][32] fp32 line rows [emb 16 | w | pad]: one 128-B memory line per id "
                                "(rmx_table::line, knob table_lines)"}
               if args.workload == "deepfm" and rmx.get_tuning("table_lines", 0) else {}),
            **({"exchange": r["exchange"]} if "exchange" in r else {}),
            "roofline": r["roofline"],
            "cpu_baseline": cpu,
            **({"parity_check_ranks": parity_ranks,
                "parity_ok": all(_pc_ok(p) for p in parity_ranks)}
               if parity_ranks else {}),
            **({"predict_auc": r["predict_auc"]} if r.get("predict_auc") else {}),
            **({"auc": r["auc"]} if "auc" in r else {}),
            "stages": r["stages"],
            **({"stage_sum_ms": r["stage_sum_ms"]} if "stage_sum_ms" in r else {}),
        }
        if companion:
            line["models"] = {"xdeepfm": {
                "config": config_of("xdeepfm", companion, world, args.zipf),
                "value": round(companion["value"], 1), "unit": "examples/s",
                "ms_per_step": round(companion["ms_per_step"], 4), "steps": args.steps, "warmup": args.warmup,
                "roofline": companion["roofline"], "stages": companion["stages"],
                "stage_sum_ms": companion["stage_sum_ms"], "cpu_baseline": cpu2,
                **({"predict_auc": companion["predict_auc"]} if companion.get("predict_auc") else {})}}
        if not train and args.workload != "lr_plumbing":
            # BASELINE.json asks for the HBM-roofline fraction too: the whole forward's algorithmic
            # bytes per example (ids + first-order weights + embedding rows + output)
            es = 2 if r.get("bf16") else 4
            bpe = F * 4 + F * es + F * K * es + 4
            line["forward_hbm"] = {"algorithmic_bytes_per_example": bpe,
                                   "gbs": round(r["value"] * bpe / 1e9, 1), "peak": PEAK_HBM_GBS,
                                   "frac": round(r["value"] * bpe / 1e9 / PEAK_HBM_GBS, 4),
                                   "note": "compute-bound: the dense tower / CIN, not the gather, sets the rate"}
    # configs[3] at N > 1 (one GPU per rank): the 100M-row table hash-sharded over the ranks, one RCCL
    # exchange per batch, as a sub-record of the default line -- so the driver's multi-GPU runs execute
    # and check the exchange.  A watchdog bounds it: past --companion-timeout it aborts the RCCL
    # communicator, prints the line with the sub-record marked as timed out and ends the process.
    sub = None
    if (args.workload == "deepfm" and not args.no_companion and not args.no_sharded_companion and not args.zipf
            and ((world > 1 and world <= ndev) or args.sharded_companion)):
        sub = sharded_companion(args, rmx, ctx, rank, world, dist, line if rank == 0 else None)
        if rank == 0:
            line.setdefault("models", {})["deepfm_sharded"] = sub
    # rank 0's own sub-records, after the sharded one (whose watchdog budget they would otherwise eat at
    # N > 1): the encoder alone (gather + first order + FM) at V = 1M and 100M, its HBM
    # roofline, and the L-A drop-in (host arrays) at the reference's batch sizes
    enc = la = None
    if args.workload == "deepfm" and not args.zipf and rank == 0:
        if not args.no_encoder_record:
            enc = encoder_record(args, rmx, ctx, max(20, min(args.steps, 100)), max(5, args.warmup))
            line.setdefault("models", {})["encoder"] = enc
        if not args.no_la_record:
            la = la_record(args, rmx, ctx)
            line.setdefault("models", {})["deepfm_la"] = la
    status = job_status(parity_ranks, sub, cpu, cpu2) or record_status(enc, la)
    if rank == 0:
        if status:
            line["status"] = {"exit": status, "reason": STATUS_REASON[status]}
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    if status:
        sys.stderr.write("bench.py: rank %d exits %d (%s)\n" % (rank, status, STATUS_REASON[status]))
        raise SystemExit(status)


def sharded_companion(args, rmx, ctx, rank, world, dist, line):
    """The deepfm_sharded sub-record (rank 0 returns it; every rank takes part): run() on the sharded
    workload with min(K, 20) / min(W, 5) steps, then every rank's parity on its own rows."""
    import threading
    t_lim = args.companion_timeout
    out_fd = os.dup(1)  # the real stdout: the watchdog may fire inside stdout_to_stderr (RCCL init)

    closing = threading.Event()  # set before the shards are closed: the watchdog then only exits

    def expire():
        sys.stderr.write("bench.py: the sharded sub-record passed %.0f s; aborting its communicator\n" % t_lim)
        if not closing.is_set():  # (ShardedTable.abort / close are also ordered by the table's lock)
            for t in list(LIVE_SHARDS):
                try:
                    t.abort()
                except Exception:
                    pass
        if line is not None:
            out = dict(line)
            out.setdefault("models", {})["deepfm_sharded"] = {
                "error": "timed out after %.0f s (watchdog aborted the RCCL communicator)" % t_lim}
            os.write(out_fd, (json.dumps(out) + "\n").encode())
        # the line (with the main measurement) is out; the non-zero status tells launch_ranks and the
        # driver that the multi-GPU exchange hung
        os._exit(124)
    wd = threading.Timer(t_lim, expire)
    wd.daemon = True
    wd.start()
    try:
        rs = run(args, "deepfm_sharded", rmx, ctx, rank, world, dist, min(args.steps, 20), min(args.warmup, 5))
        pc = parity_check("deepfm_sharded", rs["out"], rank * rs["nrows"], vocab=rs["Vw"])
        pcs = [pc]
        if dist:
            pcs = [None] * world
            dist.all_gather_object(pcs, pc)
        sub = {"config": config_of("deepfm_sharded", rs, world, 0), "value": round(rs["value"], 1),
               "unit": "examples/s", "ms_per_step": round(rs["ms_per_step"], 4), "steps": min(args.steps, 20),
               "warmup": min(args.warmup, 5), "exchange": rs["exchange"], "roofline": rs["roofline"],
               "stages": rs["stages"], "parity_check_ranks": pcs, "parity_ok": all(p["ok"] for p in pcs)}
    except Exception as e:  # recorded in the line; the main measurement stands
        sub = {"error": "%s: %s" % (type(e).__name__, str(e)[:400])}
        for t in LIVE_SHARDS:  # a failed exchange may leave RCCL kernels waiting on peers
            try:
                t.abort()
            except Exception:
                pass
    closing.set()
    for t in LIVE_SHARDS:  # (still under the watchdog: destroy synchronises the device)
        t.close()
    del LIVE_SHARDS[:]
    wd.cancel()
    os.close(out_fd)
    return sub


if __name__ == "__main__":
    main()
