"""Host restatement of the sharded-table exchange protocol (TEST INFRASTRUCTURE ONLY).

Mirrors recommendation-models_amd/csrc/shard.hip step by step with numpy arrays and a real
torch.distributed all-to-all (gloo on CPU): owner(id) = id mod N, local row = id div N, bucket the
batch's ids by owner, exchange counts, ids to owners, owner gather, rows back, un-permute.  Used by
tests/test_shard.py to run the N > 1 protocol over 2 CPU ranks; the GPU path is checked against the
replicated table on the device.
"""
import os

import numpy as np

import oracle_ctypes as oc


def partition(w_table, e_table, N, rank):
    """Rows owned by `rank` (ids rank, rank + N, ...), in local-row order."""
    return w_table[rank::N].copy(), e_table[rank::N].copy()


def route(ids, N):
    owner = ids % N
    order = np.argsort(owner, kind="stable")          # bucket order (any order within a bucket works)
    counts = np.bincount(owner, minlength=N).astype(np.int64)
    send_ids = (ids[order] // N).astype(np.int32)     # local rows on the owner
    perm = np.empty(len(ids), np.int64)
    perm[order] = np.arange(len(ids))                 # slot of id n
    return counts, send_ids, perm


def dedupe(ids):
    """Step 0 (ParRecModel.distinctIntIndices, ParRecModel.scala:337-345): distinct ids + inverse."""
    uniq, inv = np.unique(ids, return_inverse=True)
    return uniq, inv


def exchange(dist, torch, ids, w_loc, e_loc, N, k, use_dedupe=True):
    if use_dedupe:
        uniq, inv = dedupe(ids)
        w_u, e_u = exchange(dist, torch, uniq, w_loc, e_loc, N, k, use_dedupe=False)
        return w_u[inv], e_u[inv]
    counts, send_ids, perm = route(ids, N)
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
    w, e = exchange(dist, torch, ids, w_loc, e_loc, world, k)
    w2, e2 = exchange(dist, torch, ids, w_loc, e_loc, world, k, use_dedupe=False)
    ok_rows = (np.array_equal(w, wt[ids]) and np.array_equal(e, et[ids]) and np.array_equal(w2, w)
               and np.array_equal(e2, e))
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
