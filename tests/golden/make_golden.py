"""Writes the golden fixtures of tests/golden/ (TEST INFRASTRUCTURE ONLY).

The reference cannot run anywhere here and ships no vectors, so each fixture
is produced by the oracle (oracle/rmx_oracle.c, fp32 in BigDL op order and fp64) AND checked
against the independent numpy re-expression (tests/ref_numpy.py) before it is written; a case
where the two disagree beyond 1e-7 (fp64) aborts.  Inputs are the reference's RecModel.forward
flat arrays (RecModel.scala:37-63): COO row index, gathered weights / embeddings, bias, mats.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ctypes as oc  # noqa: E402
import ref_numpy as rn  # noqa: E402

CASES = [
    # name, type, F, k, kwargs, B, V
    ("lr_f39", oc.LR, 39, 16, {}, 24, 4000),
    ("deepfm_f39k16", oc.DEEPFM, 39, 16, dict(fc=(40, 24)), 24, 4000),
    ("deepfm_f5k4", oc.DEEPFM, 5, 4, dict(fc=(8,)), 9, 100),
    ("dnn_f39k16", oc.DNN, 39, 16, dict(fc=(32,)), 24, 4000),
    ("xdeepfm1_f39k16", oc.XDEEPFM, 39, 16, dict(fc=(16, 8), cin=(20,)), 16, 4000),
    ("xdeepfm3_f39k16", oc.XDEEPFM, 39, 16, dict(fc=(16, 8), cin=(12, 20, 8)), 16, 4000),
    ("dcn_f39k16", oc.DCN, 39, 16, dict(fc=(16, 8), cross_depth=3), 16, 4000),
    ("pnn_f39k16", oc.PNN, 39, 16, dict(fc=(24, 8)), 16, 4000),
    ("pnn_f6k4", oc.PNN, 6, 4, dict(fc=(5,)), 7, 60),
]
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75


def ref_kind(t):
    return {oc.LR: "lr", oc.DEEPFM: "deepfm", oc.DNN: "dnn", oc.XDEEPFM: "xdeepfm", oc.DCN: "dcn",
            oc.PNN: "pnn"}[t]


def main():
    for name, t, F, k, kw, B, V in CASES:
        m = oc.make_model(t, F, k, **kw)
        ids = oc.gen_ids(SEED_IDS, 0, B, F, V).astype(np.int64)
        wt, et = oc.gen_table(SEED_TAB, V, k)
        w, e = oc.gather(wt, et, 1, ids)
        index = np.repeat(np.arange(B, dtype=np.int64), F)
        mats = oc.init_mats(m, SEED_MATS) if t != oc.LR else np.zeros(0, np.float32)
        bias = np.array([0.01], np.float32)
        emb = e if t != oc.LR else None
        p32 = oc.forward(m, B, index, bias, w, emb, mats if t != oc.LR else None, 0)
        p64 = oc.forward(m, B, index, bias, w, emb, mats if t != oc.LR else None, 1)
        ref = rn.forward(ref_kind(t), B, F, k, index, bias, w, emb, mats, fc=kw.get("fc", ()),
                         cin=kw.get("cin", ()), cross_depth=kw.get("cross_depth", 0))
        err = float(np.abs(p64 - ref).max())
        if err > 1e-7:
            raise SystemExit("%s: oracle fp64 vs numpy restatement differ by %g" % (name, err))
        y1 = oc.first_order(B, index, w)
        y2 = oc.fm(B, F, k, e) if t != oc.LR else np.zeros(B, np.float32)
        sizes = oc.mats_sizes(m) if t != oc.LR else np.zeros(0, np.int32)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"),
            model=np.array([t, F, k, kw.get("cross_depth", 0)], np.int32),
            fc=np.array(kw.get("fc", ()), np.int32), cin=np.array(kw.get("cin", ()), np.int32),
            batch_size=np.int32(B), num_rows=np.int64(V), ids=ids, index=index, bias=bias, weights=w,
            embedding=e, mats=mats, mat_sizes=sizes.astype(np.int32),
            y1=y1, y2=y2, p32=p32, p64=p64)
        print("%-18s B=%-3d mats=%-7d max|p64-numpy|=%.2g" % (name, B, len(mats), err))
    # gather fixture: reference PS layout k x V (ParRecModel.scala:95-101, :300-306)
    V, k = 257, 16
    wt, et = oc.gen_table(SEED_TAB, V, k)
    feats = oc.gen_ids(SEED_IDS, 0, 20, 13, V).astype(np.int64)
    w, e = oc.gather(wt, np.ascontiguousarray(et.T), 0, feats)
    if not np.array_equal(e.reshape(-1, k), et[feats]) or not np.array_equal(w, wt[feats]):
        raise SystemExit("gather fixture: k-major gather disagrees with row indexing")
    np.savez_compressed(os.path.join(HERE, "gather_kmajor.npz"), w_table=wt, emb_table_kmajor=et.T.copy(),
                        feats=feats, w=w, e=e)
    print("gather_kmajor      V=%d nnz=%d" % (V, len(feats)))


if __name__ == "__main__":
    main()
