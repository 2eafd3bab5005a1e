"""Which rows of the whole-tower kernel (k_small_s3.hip) differ from the engine, per batch and RT.
usage: diag_small.py B[,B...] [zero_wo]"""
import sys
import numpy as np
sys.path.insert(0, "recommendation-models_amd")
import rmx

F, K, V = 39, 16, 50000
WO_OFF = 624 * 400 + 400 + 2 * (400 * 400 + 400)
ctx = rmx.default_context()
m = rmx.DeepFM(V, F, K, [400, 400, 400])
mats = np.array(m.initMats(0x3A75), np.float32)
if len(sys.argv) > 2 and sys.argv[2] == "zero_wo":
    mats[WO_OFF:WO_OFF + 400] = 0.0
m.setMats(mats)
m.setBias(0.01)
table = rmx.EmbeddingTable(ctx, V, K)
table.fill_synthetic(0x7AB1E)
for B in [int(b) for b in sys.argv[1].split(",")]:
    for rt in (1, 2):
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        rmx.gen_ids(ctx, 0x5A11, 0, B, F, V, ids)
        out = rmx.DeviceArray(ctx, B, np.float32)
        rmx.set_tuning("s3_small_rt", rt)
        res = []
        for knob in (0, 2, 2, 2):
            rmx.set_tuning("s3_small", knob)
            m.forward_ids(table, B, ids, out)
            ctx.sync()
            res.append(out.numpy().copy())
        for i in (1, 2, 3):
            bad = np.flatnonzero(np.abs(res[i] - res[0]) > 1e-6)
            blocks = sorted(set((bad // (16 * rt)).tolist()))
            print("B=%d RT=%d run %d: bad rows %d, rows in block %s, blocks %s" % (
                B, rt, i, bad.size, sorted(set((bad % (16 * rt)).tolist()))[:40], blocks[:64]), flush=True)
            if bad.size:
                print("   first bad: engine %s small %s" % (res[0][bad[:4]], res[i][bad[:4]]))
