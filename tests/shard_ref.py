"""Host restatement of the sharded-table exchange protocol (TEST INFRASTRUCTURE ONLY).

Mirrors recommendation-models_amd/csrc/shard.hip step by step with numpy arrays and a real
torch.distributed all-to-all (gloo on CPU): owner(id) = p(id) mod N, local row = p(id) div N with p
the keyed Feistel permutation of [0, V) (restated below; key 0 = identity), bucket the batch's ids by
owner, exchange counts, ids to owners, owner gather, rows back, un-permute.  Used by
tests/test_shard.py to run the N > 1 protocol over 2 CPU ranks; the GPU path is checked against the
replicated table on the device.
"""
import os

import numpy as np

import oracle_ctypes as oc

OWNER_HASH_DEFAULT = 0x5EED5A4D0C7A11ED  # include/rmx.h RMX_OWNER_HASH_DEFAULT
_M64 = (1 << 64) - 1


def _round_keys(key):
    z, rk = key, []
    for _ in range(4):  # splitmix64 of the key, successive states
        z = (z + 0x9E3779B97F4A7C15) & _M64
        x = z
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
        rk.append((x ^ (x >> 31)) & 0xFFFFFFFF)
    return rk


def _side(V):
    a = int(np.sqrt(max(V, 1)))
    while a * a < V:
        a += 1
    while a > 1 and (a - 1) * (a - 1) >= V:
        a -= 1
    return a


def _round(x, rk, a):
    """F_r(x) = mulhi(fmix32(x ^ k_r), a): uniform in [0, a) (shard.hip owner_round)."""
    h = (x ^ np.uint64(rk)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return (h * np.uint64(a)) >> np.uint64(32)


def owner_perm(ids, key, V, inverse=False):
    """p(ids) (shard.hip owner_perm): 4 Feistel rounds on Z_a x Z_a (a = ceil(sqrt(V))), each
    (L, R) -> (R, (L + F_r(R)) mod a), cycle-walked back into [0, V); key 0 = identity."""
    ids = np.asarray(ids, np.int64)
    if not key:
        return ids.copy()
    a = _side(V)
    rk = _round_keys(key)
    A = np.uint64(a)

    def once(x):
        x = x.astype(np.uint64)
        L, R = x // A, x % A
        if not inverse:
            for r in range(4):
                L, R = R, (L + _round(R, rk[r], a)) % A
        else:
            for r in range(3, -1, -1):
                L, R = (R + A - _round(L, rk[r], a)) % A, L
        return (L * A + R).astype(np.int64)

    y = once(ids)
    out = y >= V
    while out.any():
        y[out] = once(y[out])
        out = y >= V
    return y


def partition(w_table, e_table, N, rank, key=OWNER_HASH_DEFAULT):
    """Rows owned by `rank` in local-row order: local row l holds the id with p(id) = l N + rank."""
    V = len(w_table)
    rows_per = (V + N - 1) // N
    pid = np.arange(rows_per, dtype=np.int64) * N + rank
    gid = owner_perm(pid[pid < V], key, V, inverse=True)
    w = np.zeros(rows_per, w_table.dtype)
    e = np.zeros((rows_per,) + e_table.shape[1:], e_table.dtype)
    w[:len(gid)], e[:len(gid)] = w_table[gid], e_table[gid]
    return w, e


def route(ids, N, key=0, V=None):
    p = owner_perm(ids, key, V if V is not None else int(np.max(ids)) + 1)
    owner = p % N
    order = np.argsort(owner, kind="stable")          # bucket order (any order within a bucket works)
    counts = np.bincount(owner, minlength=N).astype(np.int64)
    send_ids = (p[order] // N).astype(np.int32)       # local rows on the owner
    perm = np.empty(len(ids), np.int64)
    perm[order] = np.arange(len(ids))                 # slot of id n
    return counts, send_ids, perm


def dedupe(ids):
    """Step 0 (ParRecModel.distinctIntIndices, ParRecModel.scala:337-345): distinct ids + inverse."""
    uniq, inv = np.unique(ids, return_inverse=True)
    return uniq, inv


def exchange(dist, torch, ids, w_loc, e_loc, N, k, V, use_dedupe=True, key=OWNER_HASH_DEFAULT):
    if use_dedupe:
        uniq, inv = dedupe(ids)
        w_u, e_u = exchange(dist, torch, uniq, w_loc, e_loc, N, k, V, use_dedupe=False, key=key)
        return w_u[inv], e_u[inv]
    counts, send_ids, perm = route(ids, N, key, V)
    rc = torch.zeros(N, dtype=torch.int64)
    dist.all_to_all_single(rc, torch.from_numpy(counts))
    rcounts = rc.numpy()
    recv_ids = torch.zeros(int(rcounts.sum()), dtype=torch.int32)
    dist.all_to_all_single(recv_ids, torch.from_numpy(send_ids), rcounts.tolist(), counts.tolist())
    rows = recv_ids.numpy()
    send_rows = np.concatenate([e_loc[rows], w_loc[rows][:, None]], axis=1).astype(np.float32)  # owner gather
    back = torch.zeros((len(ids), k + 1), dtype=torch.float32)
    dist.all_to_all_single(back, torch.from_numpy(send_rows), counts.tolist(), rcounts.tolist())
    back = back.numpy()[perm]                         # un-permute to id order
    return back[:, k].copy(), back[:, :k].copy()


def worker(rank, world, port, V, k, B, F, out_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wt, et = oc.gen_table(0x7AB1E, V, k)
    w_loc, e_loc = partition(wt, et, world, rank)
    ids = oc.gen_ids(0x5EED2026, rank * B, B, F, V).astype(np.int64)
    ids[::3] = ids[0]  # repeated ids: the dedupe step has work to do
    w, e = exchange(dist, torch, ids, w_loc, e_loc, world, k, V)
    w2, e2 = exchange(dist, torch, ids, w_loc, e_loc, world, k, V, use_dedupe=False)
    w0, e0 = partition(wt, et, world, rank, key=0)  # the identity owner map (id mod N)
    w3, e3 = exchange(dist, torch, ids, w0, e0, world, k, V, use_dedupe=False, key=0)
    ok_rows = (np.array_equal(w, wt[ids]) and np.array_equal(e, et[ids]) and np.array_equal(w2, w)
               and np.array_equal(e2, e) and np.array_equal(w3, w) and np.array_equal(e3, e))
    m = oc.make_model(oc.DEEPFM, F, k, fc=(16,))
    mats = oc.init_mats(m, 3)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    p_shard = oc.forward(m, B, index, bias, w, e, mats, 0, 1)
    w_ref, e_ref = oc.gather(wt, et, 1, ids)
    p_ref = oc.forward(m, B, index, bias, w_ref, e_ref, mats, 0, 1)
    # the time reduction of bench.py: max over ranks
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    np.save(os.path.join(out_dir, "rank%d.npy" % rank),
            np.array([ok_rows, np.array_equal(p_shard, p_ref), t.item() == world], dtype=np.int64))
    dist.destroy_process_group()
