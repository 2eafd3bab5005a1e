"""Hash-sharded table (include/rmx.h rmx_shard_*, csrc/shard.hip; BASELINE.json configs[3]).

CPU (gloo, world_size 2): the exchange protocol restated in tests/shard_ref.py over a real
torch.distributed all-to-all reproduces the global table's rows bit-exactly and the same forward.
GPU: librmx's sharded path gives BITWISE the outputs of the replicated table -- the exchange only
copies rows -- for
  * exchange-group shards (rmx_group: N virtual ranks, one thread + context + stream each, on one
    GPU): the product's N > 1 schedule -- counts, ids to owners, owner gather, rows back, the
    own-bucket skip and the peer-only owner buffers -- with device copies as the transport;
  * loopback shards (N partitions in one shard: routing / owner gather at N > 1, single thread);
  * an RCCL communicator of one rank (no exchange: route + the own-bucket gather, sized on the
    device).
"""
import os
import socket

import numpy as np
import pytest

import oracle_ctypes as oc

F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_exchange_protocol_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    import shard_ref
    V, k, B, F_ = 5003, 8, 37, 5
    mp.spawn(shard_ref.worker, args=(2, _free_port(), V, k, B, F_, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        ok = np.load(os.path.join(tmp_path, "rank%d.npy" % r))
        assert ok.tolist() == [1, 1, 1], (r, ok)


def test_route_is_a_bijection():
    import shard_ref
    ids = np.random.default_rng(0).integers(0, 1000, 5000)
    for N in (1, 2, 3, 8):
        counts, send_ids, perm = shard_ref.route(ids, N)
        assert counts.sum() == len(ids) and sorted(perm.tolist()) == list(range(len(ids)))
        owner_of_slot = np.repeat(np.arange(N), counts)
        assert np.array_equal(owner_of_slot[perm], ids % N)
        assert np.array_equal(send_ids[perm] * N + ids % N, ids)
        # keyed owner map: slot owners follow p(id), the local rows invert back to the ids
        counts, send_ids, perm = shard_ref.route(ids, N, shard_ref.OWNER_HASH_DEFAULT, 1000)
        p = shard_ref.owner_perm(ids, shard_ref.OWNER_HASH_DEFAULT, 1000)
        assert np.array_equal(np.repeat(np.arange(N), counts)[perm], p % N)
        assert np.array_equal(send_ids[perm] * N + p % N, p)


@pytest.mark.parametrize("V,N", [(5003, 2), (100_003, 8), (1 << 20, 3), (100_000_000, 8)])
def test_owner_hash_host_matches_numpy_restatement(V, N):
    """rmx_owner_hash (the C function every route kernel inlines) against the numpy restatement of
    the keyed Feistel permutation; the default key is on (configs[3] hash-shards), key 0 = id mod N."""
    import rmx
    import shard_ref
    ids = np.random.default_rng(V).integers(0, V, 2000)
    ids[:3] = [0, V - 1, V // 2]
    for key in (rmx.OWNER_HASH_DEFAULT, 0, 99):
        p = shard_ref.owner_perm(ids, key, V)
        got = [rmx.owner_hash(key, V, N, int(i)) for i in ids]
        assert [o for o, _ in got] == (p % N).tolist()
        assert [l for _, l in got] == (p // N).tolist()
    assert rmx.OWNER_HASH_DEFAULT == shard_ref.OWNER_HASH_DEFAULT
    with pytest.raises(ValueError):
        rmx.owner_hash(rmx.OWNER_HASH_DEFAULT, V, N, V)  # outside [0, V): no owner


def test_owner_hash_is_a_bijection_and_balances():
    import shard_ref
    V = 100_003
    p = shard_ref.owner_perm(np.arange(V), shard_ref.OWNER_HASH_DEFAULT, V)
    assert np.array_equal(np.sort(p), np.arange(V))
    assert np.array_equal(shard_ref.owner_perm(p, shard_ref.OWNER_HASH_DEFAULT, V, inverse=True), np.arange(V))
    strided = np.arange(0, V, 8)  # all multiples of 8: one owner under id mod 8
    c = np.bincount(shard_ref.owner_perm(strided, shard_ref.OWNER_HASH_DEFAULT, V) % 8, minlength=8)
    assert c.min() > 0.9 * len(strided) / 8 and c.max() < 1.1 * len(strided) / 8


# ------------------------------------------------------------------ GPU ----
def _setup(ctx, V, B, seed_row=0, zipf=0.0):
    import rmx
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, seed_row, B, F, V, ids, zipf=zipf)
    return table, ids


@pytest.mark.gpu
@pytest.mark.parametrize("dedupe", [True, False])
@pytest.mark.parametrize("zipf", [0.0, 1.1])
@pytest.mark.parametrize("N", [1, 2, 3, 8])
def test_loopback_shard_gather_bit_exact(N, zipf, dedupe):
    import rmx
    ctx = rmx.default_context()
    V, B = 100_003, 300
    _, ids = _setup(ctx, V, B, zipf=zipf)
    sh = rmx.ShardedTable(ctx, V, K, N)
    sh.set_dedupe(dedupe)
    sh.fill_synthetic(SEED_TAB)
    n = B * F
    w = rmx.DeviceArray(ctx, n, np.float32)
    e = rmx.DeviceArray(ctx, n * K, np.float32)
    sh.gather(ids, n, w, e)
    ctx.sync()
    h_ids = ids.numpy().astype(np.int64)
    wt, et = oc.gen_table(SEED_TAB, V, K)
    w_ref, e_ref = oc.gather(wt, et, 1, h_ids)
    assert np.array_equal(w.numpy(), w_ref) and np.array_equal(e.numpy(), e_ref)
    # step 0 sends each distinct id once
    assert sh.last_sent() == (len(np.unique(h_ids)) if dedupe else n)


@pytest.mark.gpu
@pytest.mark.parametrize("zipf", [0.0, 1.1])
def test_loopback_shard_dedupe_auto(zipf):
    """dedupe "auto" (the default): the first batch is deduplicated; when that removed < 10 % of the
    ids (uniform ids over a large V) the next batches skip the step, with heavy reuse (Zipf) they keep
    it -- the gathered rows are bit-exact either way."""
    import rmx
    ctx = rmx.default_context()
    V, B, N = 5_000_011, 300, 4
    _, ids = _setup(ctx, V, B, zipf=zipf)
    sh = rmx.ShardedTable(ctx, V, K, N)
    sh.set_dedupe("auto")
    sh.fill_synthetic(SEED_TAB)
    n = B * F
    h_ids = ids.numpy().astype(np.int64)
    distinct = len(np.unique(h_ids))
    wt, et = oc.gen_table(SEED_TAB, V, K)
    w_ref, e_ref = oc.gather(wt, et, 1, h_ids)
    w = rmx.DeviceArray(ctx, n, np.float32)
    e = rmx.DeviceArray(ctx, n * K, np.float32)
    sent = []
    for _ in range(3):
        sh.gather(ids, n, w, e)
        ctx.sync()
        assert np.array_equal(w.numpy(), w_ref) and np.array_equal(e.numpy(), e_ref)
        sent.append(sh.last_sent())
    assert sent[0] == distinct
    if distinct * 10 > n * 9:
        assert sent[1:] == [n, n]
    else:
        assert sent[1:] == [distinct, distinct]


@pytest.mark.gpu
def test_gen_ids_zipf_shape():
    """Zipf-like ids: inside each field's range, deterministic, rank 0 the most frequent."""
    import rmx
    ctx = rmx.default_context()
    V, B = 1_000_000, 4096
    per = V // F
    a = rmx.DeviceArray(ctx, B * F, np.int32)
    b = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, a, zipf=1.1)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, b, zipf=1.1)
    ctx.sync()
    x = a.numpy().reshape(B, F).astype(np.int64)
    assert np.array_equal(x, b.numpy().reshape(B, F))
    r = x - np.arange(F)[None, :] * per
    assert r.min() >= 0 and r.max() < per
    cnt = np.bincount(r.ravel(), minlength=per)
    assert cnt[0] == cnt.max() and cnt[0] > 0.05 * B * F
    assert len(np.unique(x)) < 0.5 * B * F  # heavy reuse (the point of the dedupe step)


def _models():
    import rmx
    V = 100_003
    return {
        "deepfm": lambda: rmx.DeepFM(V, F, K, [400, 400, 400]),
        "xdeepfm": lambda: rmx.XDeepFM(V, F, K, [64, 32], [48, 32]),
        "dcn": lambda: rmx.DCN(V, F, K, 3, [64, 32]),
        "pnn": lambda: rmx.PNN(V, F, K, [48, 32]),
        "lr": lambda: rmx.LR(V, F),
    }


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "xdeepfm", "dcn", "pnn", "lr"])
@pytest.mark.parametrize("N,zipf,dedupe", [(1, 0.0, True), (4, 0.0, True), (8, 0.0, True), (8, 1.1, True),
                                           (4, 1.1, False)])
def test_sharded_forward_bitwise_equals_replicated(kind, N, zipf, dedupe):
    import rmx
    ctx = rmx.default_context()
    V, B = 100_003, 1000
    table, ids = _setup(ctx, V, B, seed_row=11, zipf=zipf)
    m = _models()[kind]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    sh = rmx.ShardedTable(ctx, V, K, N)
    sh.set_dedupe(dedupe)
    sh.fill_synthetic(SEED_TAB)
    ref = rmx.DeviceArray(ctx, B, np.float32)
    got = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids, ref)
    m.forward_ids_sharded(sh, B, ids, got)
    ctx.sync()
    assert np.array_equal(got.numpy(), ref.numpy())


@pytest.mark.gpu
def test_rccl_single_rank_shard_matches_replicated():
    """A one-rank RCCL communicator: no exchange (route + the own-bucket gather, no RCCL op and no
    host sync); the group tests above run the N > 1 schedule."""
    import rmx
    ctx = rmx.default_context()
    V, B = 200_000, 2048
    table, ids = _setup(ctx, V, B, seed_row=3)
    m = rmx.DeepFM(V, F, K, [400, 400, 400])
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    sh = rmx.ShardedTable(ctx, V, K, 1, 0, rmx.comm_unique_id())
    sh.fill_synthetic(SEED_TAB)
    ref = rmx.DeviceArray(ctx, B, np.float32)
    got = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids, ref)
    for _ in range(2):  # buffers are reused across batches
        m.forward_ids_sharded(sh, B, ids, got)
    ctx.sync()
    assert np.array_equal(got.numpy(), ref.numpy())
    n = 777
    w = rmx.DeviceArray(ctx, n, np.float32)
    e = rmx.DeviceArray(ctx, n * K, np.float32)
    sh.gather(ids, n, w, e)
    ctx.sync()
    wt, et = oc.gen_table(SEED_TAB, V, K)
    w_ref, e_ref = oc.gather(wt, et, 1, ids.numpy()[:n].astype(np.int64))
    assert np.array_equal(w.numpy(), w_ref) and np.array_equal(e.numpy(), e_ref)


@pytest.mark.gpu
def test_rccl_shard_abort():
    """rmx_shard_abort tears the RCCL communicator down without a lock (a watchdog's call): a second
    abort is a no-op, the one-rank path (no RCCL op) still serves batches bitwise, and destroy
    afterwards skips the aborted communicator.  A loopback shard has none: abort is a no-op."""
    import rmx
    ctx = rmx.default_context()
    V, B = 200_000, 1024
    table, ids = _setup(ctx, V, B, seed_row=5)
    m = rmx.DeepFM(V, F, K, [64, 32])
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    ref = rmx.DeviceArray(ctx, B, np.float32)
    got = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids, ref)
    sh = rmx.ShardedTable(ctx, V, K, 1, 0, rmx.comm_unique_id())
    sh.fill_synthetic(SEED_TAB)
    sh.abort()
    sh.abort()
    m.forward_ids_sharded(sh, B, ids, got)
    ctx.sync()
    assert np.array_equal(got.numpy(), ref.numpy())
    sh.close()
    lb = rmx.ShardedTable(ctx, V, K, 2, 0)
    lb.abort()
    lb.close()


@pytest.mark.gpu
def test_shard_bad_args():
    import rmx
    ctx = rmx.default_context()
    with pytest.raises(rmx.RmxError):
        rmx.ShardedTable(ctx, 10, K, 0)
    with pytest.raises(rmx.RmxError):
        rmx.ShardedTable(ctx, 10, K, 2, 2)


# --------------------------------------------------- exchange group (N virtual ranks) ----
def _run_ranks(N, fn, timeout=300):
    """fn(rank) on N threads (each rank drives its own context / stream, like N processes)."""
    import threading
    res, errs = [None] * N, []

    def run(r):
        try:
            res[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 -- re-raised below with the rank
            errs.append((r, e))

    ts = [threading.Thread(target=run, args=(r,)) for r in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    if errs:
        raise AssertionError("rank %d failed: %r" % errs[0])
    return res


def _group_forward(kind, N, V, B, zipf, dedupe, reps=2):
    import rmx
    g = rmx.ExchangeGroup(N)

    def rank(r):
        ctx = rmx.Context(0)
        sh = rmx.ShardedTable(ctx, V, K, N, r, group=g)
        sh.set_dedupe(dedupe)
        sh.fill_synthetic(SEED_TAB)
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        rmx.gen_ids(ctx, SEED_IDS, 11 + r * B, B, F, V, ids, zipf=zipf)
        m = _models_v(V)[kind]()
        m.setMats(m.initMats(SEED_MATS))
        m.setBias(0.01)
        got = rmx.DeviceArray(ctx, B, np.float32)
        for _ in range(reps):  # buffers are reused across batches
            m.forward_ids_sharded(sh, B, ids, got, ctx.stream)
        ctx.sync()
        out = (got.numpy(), ids.numpy(), sh.last_sent())
        sh.close()
        return out

    return _run_ranks(N, rank)


def _models_v(V):
    import rmx
    return {
        "deepfm": lambda: rmx.DeepFM(V, F, K, [400, 400, 400]),
        "xdeepfm": lambda: rmx.XDeepFM(V, F, K, [64, 32], [48, 32]),
        "dcn": lambda: rmx.DCN(V, F, K, 3, [64, 32]),
        "pnn": lambda: rmx.PNN(V, F, K, [48, 32]),
        "lr": lambda: rmx.LR(V, F),
    }


@pytest.mark.gpu
@pytest.mark.parametrize("dedupe", [True, False])
@pytest.mark.parametrize("zipf", [0.0, 1.1])
@pytest.mark.parametrize("N", [2, 4, 8])
def test_group_exchange_forward_bitwise_equals_replicated(N, zipf, dedupe):
    """The product's N > 1 exchange schedule (csrc/shard.hip steps 2-5) at N virtual ranks: every
    rank's DeepFM forward is bitwise the replicated table's, and the ids it sent are its distinct ids
    (dedupe) or all of them."""
    import rmx
    V, B = 100_003, 1000
    outs = _group_forward("deepfm", N, V, B, zipf, dedupe)
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    m = _models_v(V)["deepfm"]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    for r, (got, h_ids, sent) in enumerate(outs):
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        ids.upload(h_ids)
        ref = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(table, B, ids, ref)
        ctx.sync()
        rv = ref.numpy()
        bad = np.flatnonzero(got != rv)
        assert bad.size == 0, "rank %d: %d rows differ (first %s, max |d| %.3g)" % (
            r, bad.size, bad[:8].tolist(), float(np.abs(got - rv).max()))
        assert sent == (len(np.unique(h_ids)) if dedupe else B * F), r


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["xdeepfm", "dcn", "pnn", "lr"])
def test_group_exchange_every_model(kind):
    import rmx
    V, B, N = 100_003, 600, 4
    outs = _group_forward(kind, N, V, B, 1.1, True, reps=1)
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    m = _models_v(V)[kind]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    for got, h_ids, _ in outs:
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        ids.upload(h_ids)
        ref = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(table, B, ids, ref)
        ctx.sync()
        assert np.array_equal(got, ref.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("N", [2, 8])
def test_group_exchange_gather_ragged(N):
    """rmx_shard_gather through the group with different id counts per rank (one rank sends none):
    the received rows are the generator's, bit for bit."""
    import rmx
    V = 50_021
    g = rmx.ExchangeGroup(N)
    wt, et = oc.gen_table(SEED_TAB, V, K)

    def rank(r):
        ctx = rmx.Context(0)
        sh = rmx.ShardedTable(ctx, V, K, N, r, group=g)
        sh.set_dedupe(r % 2 == 0)
        sh.fill_synthetic(SEED_TAB)
        n = 0 if r == 1 else 997 * (r + 1)
        h_ids = np.random.default_rng(r).integers(0, V, max(n, 1)).astype(np.int32)[:n]
        ids = rmx.DeviceArray(ctx, max(n, 1), np.int32)
        if n:
            ids.upload(h_ids)
        w = rmx.DeviceArray(ctx, max(n, 1), np.float32)
        e = rmx.DeviceArray(ctx, max(n, 1) * K, np.float32)
        for _ in range(2):
            sh.gather(ids, n, w, e, ctx.stream)
        ctx.sync()
        out = (h_ids, w.numpy()[:n], e.numpy()[:n * K])
        sh.close()
        return out

    for h_ids, w, e in _run_ranks(N, rank):
        w_ref, e_ref = oc.gather(wt, et, 1, h_ids.astype(np.int64))
        assert np.array_equal(w, w_ref) and np.array_equal(e, e_ref)


@pytest.mark.gpu
def test_group_of_one_rank_dedupe_device_count():
    """One rank: no exchange; with dedupe on, the gather is sized by the device-side distinct count
    (no host sync) and last_sent reads it back."""
    V, B = 100_003, 700
    (got, h_ids, sent), = _group_forward("deepfm", 1, V, B, 1.1, True)
    assert sent == len(np.unique(h_ids))


@pytest.mark.gpu
def test_group_exchange_100m_rows_vs_fp64_oracle():
    """configs[3] at full size: V = 100M rows hash-sharded over 4 virtual ranks, B = 65,536 rows per
    rank; head and tail slices of every rank's probabilities against the fp64 oracle, whose table rows
    come from the same generator (only the rows the slices use are generated)."""
    V, B, N = 100_000_000, 65536, 4
    outs = _group_forward("deepfm", N, V, B, 0.0, "auto", reps=1)
    om = oc.make_model(oc.DEEPFM, F, K, fc=(400, 400, 400))
    mats = oc.init_mats(om, SEED_MATS)
    n = 64
    for got, h_ids, _ in outs:
        ids2 = h_ids.reshape(B, F)
        for rows in (slice(0, n), slice(B - n, B)):
            sl = ids2[rows].astype(np.int64).ravel()
            w, e = oc.gen_rows(SEED_TAB, V, K, sl)
            index = np.repeat(np.arange(n, dtype=np.int64), F)
            ref = oc.forward(om, n, index, np.array([0.01], np.float32), w, e, mats, 1)
            err = float(np.abs(got[rows] - ref).max())
            assert err <= 1e-5, err


# ------------------------------------------- pull / forward_pulled (exchange beside forward) ----
def _pipelined(m, sh, ids_all, B, nb, ctx, ctx_x):
    """Batches 0..nb-1: pull(i + 1) on the exchange stream beside forward_pulled(i) on the main one.
    ctx_x may be a pair of contexts: slot q's pulls then run on ctx_x[q]'s stream (the
    overflow round of a slot runs on that slot's stream, the next exchange on the other one)."""
    import rmx
    xs = list(ctx_x) if isinstance(ctx_x, (list, tuple)) else [ctx_x, ctx_x]
    outs = [rmx.DeviceArray(ctx, B, np.float32) for _ in range(nb)]
    sh.pull(ids_all.view(0, B * F), B * F, 0, xs[0].stream)
    for i in range(nb):
        if i + 1 < nb:
            sh.pull(ids_all.view((i + 1) * B * F, B * F), B * F, (i + 1) % 2, xs[(i + 1) % 2].stream)
        m.forward_pulled(sh, B, i % 2, outs[i], ctx.stream)
    ctx.sync()
    for x in xs:
        x.sync()
    return [o.numpy() for o in outs]


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 4])
def test_pull_pipeline_bitwise_equals_replicated(N):
    """rmx_shard_pull into alternating slots on a second stream while rmx_forward_pulled runs the
    previous batch: every batch's output is bitwise the replicated table's (loopback N = 4, one-rank
    RCCL N = 1)."""
    import rmx
    ctx, ctx_x = rmx.default_context(), rmx.Context(0)
    V, B, nb = 100_003, 1000, 5
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, nb * B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 5, nb * B, F, V, ids)
    m = rmx.DeepFM(V, F, K, [400, 400, 400])
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    sh = rmx.ShardedTable(ctx, V, K, N, 0, rmx.comm_unique_id() if N == 1 else None)
    sh.fill_synthetic(SEED_TAB)
    ctx.sync()
    got = _pipelined(m, sh, ids, B, nb, ctx, ctx_x)
    ref = rmx.DeviceArray(ctx, B, np.float32)
    for i in range(nb):
        m.forward_ids(table, B, ids.view(i * B * F, B * F), ref)
        ctx.sync()
        assert np.array_equal(got[i], ref.numpy()), i
    # the one-stream path still works after pipelined use (slot 0 ordered behind its last forward)
    m.forward_ids_sharded(sh, B, ids.view(0, B * F), ref)
    ctx.sync()
    assert np.array_equal(ref.numpy(), got[0])


@pytest.mark.gpu
def test_pull_slot_misuse_raises():
    import rmx
    ctx = rmx.default_context()
    V, B = 10_007, 64
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    m = rmx.DeepFM(V, F, K, [32])
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    sh = rmx.ShardedTable(ctx, V, K, 2)
    sh.fill_synthetic(SEED_TAB)
    out = rmx.DeviceArray(ctx, B, np.float32)
    with pytest.raises(rmx.RmxError):
        m.forward_pulled(sh, B, 1, out)  # nothing pulled
    sh.pull(ids, B * F, 1)
    with pytest.raises(rmx.RmxError):
        sh.pull(ids, B * F, 1)  # slot still holds an unconsumed pull
    with pytest.raises(rmx.RmxError):
        m.forward_pulled(sh, B - 1, 1, out)  # batch * nFields differs from the pull
    m.forward_pulled(sh, B, 1, out)
    with pytest.raises(rmx.RmxError):
        sh.pull(ids, B * F, 2)
    ctx.sync()


@pytest.mark.gpu
def test_group_pull_pipeline(N=2):
    """The pipelined calls through the N > 1 group schedule: each rank pulls on its exchange stream."""
    import rmx
    V, B, nb = 100_003, 500, 3
    g = rmx.ExchangeGroup(N)

    def rank(r):
        ctx, ctx_x = rmx.Context(0), rmx.Context(0)
        sh = rmx.ShardedTable(ctx, V, K, N, r, group=g)
        sh.fill_synthetic(SEED_TAB)
        ids = rmx.DeviceArray(ctx, nb * B * F, np.int32)
        rmx.gen_ids(ctx, SEED_IDS, 100 + r * nb * B, nb * B, F, V, ids)
        m = _models_v(V)["deepfm"]()
        m.setMats(m.initMats(SEED_MATS))
        m.setBias(0.01)
        ctx.sync()
        got = _pipelined(m, sh, ids, B, nb, ctx, ctx_x)
        out = (got, ids.numpy())
        sh.close()
        return out

    outs = _run_ranks(N, rank)
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    m = _models_v(V)["deepfm"]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    for got, h_ids in outs:
        ids = rmx.DeviceArray(ctx, nb * B * F, np.int32)
        ids.upload(h_ids)
        ref = rmx.DeviceArray(ctx, B, np.float32)
        for i in range(nb):
            m.forward_ids(table, B, ids.view(i * B * F, B * F), ref)
            ctx.sync()
            assert np.array_equal(got[i], ref.numpy()), i


# ------------------------------------------------- keyed owner permutation (set_owner_hash) ----
@pytest.mark.gpu
@pytest.mark.parametrize("N", [3, 8])
def test_owner_hash_balances_strided_ids_and_stays_bitwise(N):
    """Ids that are all multiples of N land on one owner under id mod N; the keyed Feistel permutation
    spreads them within +-15 %, and the sharded forward (loopback) stays bitwise the replicated one."""
    import rmx
    ctx = rmx.default_context()
    V, B = 100_003, 1000
    sh = rmx.ShardedTable(ctx, V, K, N)
    sh.set_owner_hash(0x1234ABCD)
    strided = range(0, V, N)
    cnt = np.bincount([sh.owner_of(i) for i in strided], minlength=N)
    assert cnt.min() > 0.85 * len(strided) / N and cnt.max() < 1.15 * len(strided) / N
    plain = rmx.ShardedTable(ctx, V, K, N)
    plain.set_owner_hash(0)  # the identity: owner = id mod N
    assert all(plain.owner_of(i) == 0 for i in range(0, 3000, N))
    dflt = rmx.ShardedTable(ctx, V, K, N)  # hash-sharded by default
    assert all(dflt.owner_of(i) == rmx.owner_hash(rmx.OWNER_HASH_DEFAULT, V, N, i)[0] for i in range(0, 3000, 7))
    sh.fill_synthetic(SEED_TAB)
    with pytest.raises(rmx.RmxError):
        sh.set_owner_hash(7)  # fixed once the rows are filled
    table, ids = _setup(ctx, V, B, seed_row=21)
    m = rmx.DeepFM(V, F, K, [400, 400, 400])
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    ref = rmx.DeviceArray(ctx, B, np.float32)
    got = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids, ref)
    m.forward_ids_sharded(sh, B, ids, got)
    ctx.sync()
    assert np.array_equal(got.numpy(), ref.numpy())
    n = 500
    w = rmx.DeviceArray(ctx, n, np.float32)
    e = rmx.DeviceArray(ctx, n * K, np.float32)
    sh.gather(ids, n, w, e)
    ctx.sync()
    wt, et = oc.gen_table(SEED_TAB, V, K)
    w_ref, e_ref = oc.gather(wt, et, 1, ids.numpy()[:n].astype(np.int64))
    assert np.array_equal(w.numpy(), w_ref) and np.array_equal(e.numpy(), e_ref)


@pytest.mark.gpu
def test_group_exchange_owner_hash(N=4):
    """The N > 1 group schedule with the keyed owner permutation: bitwise the replicated forward."""
    import rmx
    V, B = 100_003, 800
    g = rmx.ExchangeGroup(N)

    def rank(r):
        ctx = rmx.Context(0)
        sh = rmx.ShardedTable(ctx, V, K, N, r, group=g)
        sh.set_owner_hash(99)
        sh.fill_synthetic(SEED_TAB)
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        rmx.gen_ids(ctx, SEED_IDS, 7 + r * B, B, F, V, ids)
        m = _models_v(V)["deepfm"]()
        m.setMats(m.initMats(SEED_MATS))
        m.setBias(0.01)
        got = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids_sharded(sh, B, ids, got, ctx.stream)
        ctx.sync()
        out = (got.numpy(), ids.numpy())
        sh.close()
        return out

    outs = _run_ranks(N, rank)
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    m = _models_v(V)["deepfm"]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    for got, h_ids in outs:
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        ids.upload(h_ids)
        ref = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(table, B, ids, ref)
        ctx.sync()
        assert np.array_equal(got, ref.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 4])
def test_pull_slots_grow_independently(N):
    """a pull into slot 1 with a LARGER batch than the pending pull in slot 0 grows only
    slot 1's buffers -- slot 0's rows survive and both forwards stay bitwise the replicated table's."""
    import rmx
    ctx, ctx_x = rmx.default_context(), rmx.Context(0)
    V = 100_003
    Bs = (300, 1300, 2100)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    m = rmx.DeepFM(V, F, K, [64, 32])
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    sh = rmx.ShardedTable(ctx, V, K, N, 0, rmx.comm_unique_id() if N == 1 else None)
    sh.fill_synthetic(SEED_TAB)
    ids = [rmx.DeviceArray(ctx, B * F, np.int32) for B in Bs]
    for i, B in enumerate(Bs):
        rmx.gen_ids(ctx, SEED_IDS, 1000 * i, B, F, V, ids[i])
    outs = [rmx.DeviceArray(ctx, B, np.float32) for B in Bs]
    ctx.sync()
    sh.pull(ids[0], Bs[0] * F, 0, ctx_x.stream)
    sh.pull(ids[1], Bs[1] * F, 1, ctx_x.stream)   # grows slot 1 while slot 0 is pending
    m.forward_pulled(sh, Bs[0], 0, outs[0], ctx.stream)
    sh.pull(ids[2], Bs[2] * F, 0, ctx_x.stream)   # grows slot 0 while slot 1 is pending
    m.forward_pulled(sh, Bs[1], 1, outs[1], ctx.stream)
    m.forward_pulled(sh, Bs[2], 0, outs[2], ctx.stream)
    ctx.sync()
    ctx_x.sync()
    for i, B in enumerate(Bs):
        ref = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(table, B, ids[i], ref)
        ctx.sync()
        assert np.array_equal(outs[i].numpy(), ref.numpy()), i


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 3])
def test_out_of_range_ids_do_not_hang_the_route(N):
    """with the keyed owner map an id outside [0, V) has no finite cycle walk; routing
    gives it no owner (a defined in-range slot, a zero row at one rank), so the exchange returns and
    every sample that holds only valid ids is bitwise the replicated forward."""
    import rmx
    ctx = rmx.default_context()
    V, B = 100_003, 400
    table, ids = _setup(ctx, V, B, seed_row=31)
    h = ids.numpy().reshape(B, F).copy()
    bad_rows = [0, 7, B - 1]
    h[0, 3], h[7, 0], h[B - 1, F - 1] = V + 5, -2, (1 << 30)
    bad = rmx.DeviceArray(ctx, B * F, np.int32)
    bad.upload(h.ravel())
    m = rmx.DeepFM(V, F, K, [64, 32])
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    sh = rmx.ShardedTable(ctx, V, K, N, 0, rmx.comm_unique_id() if N == 1 else None)
    sh.fill_synthetic(SEED_TAB)
    got = rmx.DeviceArray(ctx, B, np.float32)
    ref = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids_sharded(sh, B, bad, got)
    m.forward_ids(table, B, ids, ref)
    ctx.sync()
    keep = np.setdiff1d(np.arange(B), bad_rows)
    assert np.array_equal(got.numpy()[keep], ref.numpy()[keep])
    assert np.isfinite(got.numpy()).all()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["deepfm", "xdeepfm", "dcn", "pnn", "lr"])
def test_rccl_single_rank_reads_partition_in_place(kind):
    """One rank (no dedupe): no exchange and no row copy -- the batch's ids map to partition rows p(id)
    and DeepFM / DNN / LR read the [emb | w | pad] lines in place; the other models copy the mapped
    rows out first.  Every model bitwise equals the replicated table, one-shot and pipelined."""
    import rmx
    ctx, ctx_x = rmx.default_context(), rmx.Context(0)
    V, B = 100_003, 700
    table, ids = _setup(ctx, V, B, seed_row=41)
    m = _models()[kind]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    sh = rmx.ShardedTable(ctx, V, K, 1, 0, rmx.comm_unique_id())
    sh.fill_synthetic(SEED_TAB)
    ref = rmx.DeviceArray(ctx, B, np.float32)
    got = rmx.DeviceArray(ctx, B, np.float32)
    got2 = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids, ref)
    m.forward_ids_sharded(sh, B, ids, got)
    ctx.sync()
    sh.pull(ids, B * F, 1, ctx_x.stream)
    m.forward_pulled(sh, B, 1, got2, ctx.stream)
    ctx.sync()
    assert np.array_equal(got.numpy(), ref.numpy()) and np.array_equal(got2.numpy(), ref.numpy())


# ------------------------------------ fixed-capacity exchange: overflow round, zero rows (round 4) ----
def _group_forward_stats(kind, N, V, B, zipf, dedupe, h_ids_of=None, pipelined=False, nbp=3):
    """_group_forward, also returning every rank's overflow-round count; h_ids_of(r) overrides the ids.
    pipelined = "alt": the pulls of the two slots on two different streams."""
    import rmx
    g = rmx.ExchangeGroup(N)

    def rank(r):
        ctx, ctx_x = rmx.Context(0), rmx.Context(0)
        if pipelined == "alt":
            ctx_x = (ctx_x, rmx.Context(0))
        sh = rmx.ShardedTable(ctx, V, K, N, r, group=g)
        sh.set_dedupe(dedupe)
        sh.fill_synthetic(SEED_TAB)
        nb = nbp if pipelined else 1
        ids = rmx.DeviceArray(ctx, nb * B * F, np.int32)
        if h_ids_of is not None:
            ids.upload(h_ids_of(r))
        else:
            rmx.gen_ids(ctx, SEED_IDS, 11 + r * nb * B, nb * B, F, V, ids, zipf=zipf)
        m = _models_v(V)[kind]()
        m.setMats(m.initMats(SEED_MATS))
        m.setBias(0.01)
        ctx.sync()
        if pipelined:
            got = _pipelined(m, sh, ids, B, nb, ctx, ctx_x)
        else:
            o = rmx.DeviceArray(ctx, B, np.float32)
            for _ in range(2):  # buffers reused across batches
                m.forward_ids_sharded(sh, B, ids, o, ctx.stream)
            ctx.sync()
            got = [o.numpy()]
        out = (got, ids.numpy(), sh.overflow_rounds())
        sh.close()
        return out

    return _run_ranks(N, rank)


def _replicated(kind, V, h_ids, B, nb):
    import rmx
    ctx = rmx.default_context()
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    m = _models_v(V)[kind]()
    m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    ids = rmx.DeviceArray(ctx, nb * B * F, np.int32)
    ids.upload(h_ids)
    res = []
    for i in range(nb):
        ref = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(table, B, ids.view(i * B * F, B * F), ref)
        ctx.sync()
        res.append(ref.numpy())
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("N,zipf,cap_pct", [(2, 0.0, 110), (8, 0.0, 110), (4, 1.1, 110), (8, 1.1, 110),
                                            (4, 0.0, 30), (8, 0.0, 60)])
def test_fixed_exchange_overflow_round_bitwise(N, zipf, cap_pct, pipelined):
    """The N > 1 exchange with fixed-capacity buckets (~1.1 nnz / N per peer, no host sync): uniform ids
    never overflow; Zipf(1.1) ids without dedupe pile onto the hot ids' owners, and a small capacity
    (shard_cap_pct 30 / 60) overflows every bucket -- every rank then runs the counted overflow round
    (the same number of collectives on every rank), and every forward stays bitwise the replicated
    table's, through forward_ids_sharded and through the pull / forward_pulled pipeline."""
    import rmx
    V, B = 100_003, 1000
    rmx.set_tuning("shard_cap_pct", cap_pct)
    try:
        outs = _group_forward_stats("deepfm", N, V, B, zipf, False, pipelined=pipelined)
    finally:
        rmx.set_tuning("shard_cap_pct", None)
    rounds = {o[2] for o in outs}
    assert len(rounds) == 1, rounds  # every rank ran the same rounds
    n_ex = 3 if pipelined else 2  # exchanges per rank
    # the first exchange has no agreed capacity yet (cap 0): it always runs the overflow round
    if zipf == 0.0 and cap_pct >= 110:
        assert rounds == {1}
    if cap_pct < 100:
        assert rounds == {n_ex}
    nb = 3 if pipelined else 1
    for r, (got, h_ids, _) in enumerate(outs):
        ref = _replicated("deepfm", V, h_ids, B, nb)
        for i in range(nb):
            assert np.array_equal(got[i], ref[i]), (r, i)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [2, 4])
def test_fixed_exchange_overflow_round_alternating_pull_streams(N):
    """every bucket overflows (shard_cap_pct 30), so every exchange runs its overflow round on its
    slot's stream -- and the two slots' pulls run on two different streams.  The next exchange's route
    rewrites the overflow scratch the previous round sends from; it must wait for that round (the shard's
    ovf_done event).  Every forward stays bitwise the replicated table's."""
    import rmx
    V, B, nb = 100_003, 1000, 6
    rmx.set_tuning("shard_cap_pct", 30)
    try:
        outs = _group_forward_stats("deepfm", N, V, B, 0.0, False, pipelined="alt", nbp=nb)
    finally:
        rmx.set_tuning("shard_cap_pct", None)
    assert {o[2] for o in outs} == {nb}
    for r, (got, h_ids, _) in enumerate(outs):
        ref = _replicated("deepfm", V, h_ids, B, nb)
        for i in range(nb):
            assert np.array_equal(got[i], ref[i]), (r, i)


@pytest.mark.gpu
def test_fixed_exchange_zipf_without_dedupe_overflows():
    """Zipf(1.1) ids at N = 8 without dedupe: the hot ids' owners get far more than 1.1 nnz / N, so the
    overflow round runs in the second exchange too (the first always runs it; results bitwise, above)."""
    outs = _group_forward_stats("deepfm", 8, 100_003, 2000, 1.1, False)
    assert all(o[2] == 2 for o in outs), [o[2] for o in outs]


@pytest.mark.gpu
@pytest.mark.parametrize("N,dedupe", [(1, True), (3, False), (3, True)])
def test_out_of_range_ids_read_zero_rows(N, dedupe):
    """an id outside [0, V) reads a zero row (zero embedding, zero first-order weight) on
    every routed path -- the fixed exchange, a dedupe route, one rank -- instead of another id's row:
    the affected samples match the fp64 oracle fed zero rows, the others are bitwise the replicated
    forward."""
    import rmx
    V, B = 100_003, 400
    bad = {(0, 3): V + 5, (7, 0): -2, (B - 1, F - 1): 1 << 30, (9, 5): -1}

    def ids_of(r):
        h = oc.gen_ids(SEED_IDS, 77 + r * B, B, F, V).reshape(B, F).copy()
        for (i, f), v in bad.items():
            h[i, f] = v
        return h.ravel().astype(np.int32)

    outs = _group_forward_stats("deepfm", N, V, B, 0.0, dedupe, h_ids_of=ids_of)
    om = oc.make_model(oc.DEEPFM, F, K, fc=(400, 400, 400))
    wt, et = oc.gen_table(SEED_TAB, V, K)
    bad_rows = sorted({i for i, _ in bad})
    for r, (got, h_ids, _) in enumerate(outs):
        h = h_ids.reshape(B, F)
        good = np.setdiff1d(np.arange(B), bad_rows)
        fixed = h.copy()
        fixed[bad_rows] = 0
        ref = _replicated("deepfm", V, fixed.ravel(), B, 1)[0]
        assert np.array_equal(got[0][good], ref[good]), r
        sl = h[bad_rows].astype(np.int64)
        ok = (sl >= 0) & (sl < V)
        w, e = oc.gather(wt, et, 1, np.where(ok, sl, 0).ravel())
        w = np.where(ok.ravel(), w, 0).astype(np.float32)
        e = np.where(np.repeat(ok.ravel(), K), e, 0).astype(np.float32)
        n = len(bad_rows)
        p = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e,
                       oc.init_mats(om, SEED_MATS), 1)
        assert np.abs(got[0][bad_rows] - p).max() <= 1e-5, r


@pytest.mark.gpu
@pytest.mark.parametrize("N", [2, 4])
def test_group_batch_hint_first_exchange_needs_no_overflow_round(N):
    """rmx_shard_set_batch_hint: with the same hint on every rank, the first fixed
    exchange of uniform ids fits its buckets -- no overflow round -- and stays bitwise the replicated
    forward; without it the first exchange takes the counted round."""
    import rmx
    V, B = 100_003, 1000
    for hint in (True, False):
        g = rmx.ExchangeGroup(N)

        def rank(r):
            ctx = rmx.Context(0)
            sh = rmx.ShardedTable(ctx, V, K, N, r, group=g)
            sh.set_dedupe(False)
            if hint:
                sh.set_batch_hint(B * F)
            sh.fill_synthetic(SEED_TAB)
            ids = rmx.DeviceArray(ctx, B * F, np.int32)
            rmx.gen_ids(ctx, SEED_IDS, 5 + r * B, B, F, V, ids)
            m = _models_v(V)["deepfm"]()
            m.setMats(m.initMats(SEED_MATS))
            m.setBias(0.01)
            got = rmx.DeviceArray(ctx, B, np.float32)
            m.forward_ids_sharded(sh, B, ids, got, ctx.stream)
            ctx.sync()
            out = (got.numpy(), ids.numpy(), sh.overflow_rounds())
            sh.close()
            return out

        outs = _run_ranks(N, rank)
        ctx = rmx.default_context()
        table = rmx.EmbeddingTable(ctx, V, K)
        table.fill_synthetic(SEED_TAB)
        m = _models_v(V)["deepfm"]()
        m.setMats(m.initMats(SEED_MATS))
        m.setBias(0.01)
        for r, (got, h_ids, rounds) in enumerate(outs):
            assert rounds == (0 if hint else 1), (hint, r, rounds)
            ids = rmx.DeviceArray(ctx, B * F, np.int32)
            ids.upload(h_ids)
            ref = rmx.DeviceArray(ctx, B, np.float32)
            m.forward_ids(table, B, ids, ref)
            ctx.sync()
            assert np.array_equal(got, ref.numpy()), (hint, r)
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fixed", [1, 0])
def test_group_failed_exchange_fails_every_later_exchange(fixed):
    """include/rmx.h: an exchange that fails on a rank at nranks > 1 fails every later exchange on the shard
    at once, on the fixed path and on the counted one (the counted path did not mark the shard).
    Rank 1's route fails by the test hook; rank 0 sees its peer post nothing."""
    import rmx
    N, V, B = 2, 50_021, 256
    g = rmx.ExchangeGroup(N)
    rmx.set_tuning("shard_fixed", fixed)
    rmx.set_tuning("shard_debug_fail_rank", 2)  # rank 1

    def rank(r):
        ctx = rmx.Context(0)
        sh = rmx.ShardedTable(ctx, V, K, N, r, group=g)
        sh.set_dedupe(False)
        sh.fill_synthetic(SEED_TAB)
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        rmx.gen_ids(ctx, SEED_IDS, r * B, B, F, V, ids)
        w = rmx.DeviceArray(ctx, B * F, np.float32)
        e = rmx.DeviceArray(ctx, B * F * K, np.float32)
        errs = []
        for _ in range(2):
            try:
                sh.gather(ids, B * F, w, e, ctx.stream)
                ctx.sync()
                errs.append(None)
            except rmx.RmxError as ex:
                errs.append(str(ex))
        ctx.sync()
        sh.close()
        return errs

    try:
        res = _run_ranks(N, rank, timeout=200)
    finally:
        rmx.set_tuning("shard_debug_fail_rank", None)
        rmx.set_tuning("shard_fixed", None)
        g.close()
    for r, errs in enumerate(res):
        assert errs[0] is not None, (r, errs)
        assert errs[1] is not None and "earlier exchange failed" in errs[1], (r, errs)
    assert "injected" in res[1][0]
