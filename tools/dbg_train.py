"""Debug helper: device backward vs oracle per array for a grid of shapes (prints error ratios)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "recommendation-models_amd"))
import numpy as np
import rmx
import oracle_ctypes as oc
import test_train as tt

kind = sys.argv[1] if len(sys.argv) > 1 else "pnn"
ctx = rmx.default_context()
V, F, K = 20_000, 39, 16
shapes = [(512, (400, 400)), (512, (400, 400)), (480, (400, 400)), (448, (400, 400)), (443, (400, 400)),
          (442, (400, 400))]
for B, fc in shapes:
    if True:
        m = tt._gpu_model(rmx, kind, V, F, K, fc)
        mats = m.initMats(tt.SEED_MATS)
        m.setMats(mats)
        m.setBias(0.01)
        t = rmx.EmbeddingTable(ctx, V, K)
        t.fill_synthetic(tt.SEED_TAB)
        ids = rmx.DeviceArray(ctx, B * F, np.int32)
        rmx.gen_ids(ctx, tt.SEED_IDS, 3, B, F, V, ids)
        tg = (np.random.default_rng(5).random(B) > 0.7).astype(np.float32)
        targets = rmx.DeviceArray(ctx, B, np.float32)
        targets.upload(tg)
        ml = len(mats)
        g_b = rmx.DeviceArray(ctx, 1, np.float32)
        g_w = rmx.DeviceArray(ctx, B * F, np.float32)
        g_e = rmx.DeviceArray(ctx, B * F * K, np.float32)
        g_m = rmx.DeviceArray(ctx, ml, np.float32)
        loss = rmx.DeviceArray(ctx, 1, np.float32)
        m.backward_ids(t, B, ids, targets, g_b, g_w, g_e, g_m, loss)
        ctx.sync()
        wt, et = oc.gen_table(tt.SEED_TAB, V, K)
        w, e = oc.gather(wt, et, 1, ids.numpy().astype(np.int64))
        index = np.repeat(np.arange(B), F).astype(np.int64)
        ref = oc.backward(tt._orc_model(kind, F, K, fc), B, index, np.array([0.01], np.float32), w, e, mats, tg)
        def r(a, b):
            b = np.asarray(b, np.float64)
            return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-12))
        ge = g_e.numpy().reshape(B, F, K)
        re = ref["embedding"].reshape(B, F, K)
        err = np.abs(ge - re).max(axis=2)
        bi, fi = np.unravel_index(np.argmax(err), err.shape)
        print(B, fc, "loss %.2e emb %.2e mats %.2e w %.2e  worst emb at b=%d f=%d" % (
            abs(loss.numpy()[0] - ref["loss"]) / ref["loss"], r(ge, re), r(g_m.numpy(), ref["mats"]),
            r(g_w.numpy(), ref["weights"]), bi, fi), flush=True)
        sizes = m.getMatsSize()
        off, segs = 0, []
        gm = g_m.numpy()
        for i in range(0, len(sizes), 2):
            n = int(sizes[i]) * int(sizes[i + 1])
            segs.append("%.1e" % r(gm[off:off + n], ref["mats"][off:off + n]))
            off += n
        print("   mats segments:", " ".join(segs), flush=True)
        bad = np.where(err.max(axis=1) > 1e-5 * np.abs(re).max())[0]
        print("   bad samples:", bad[:20].tolist(), "count", len(bad), flush=True)
        out = rmx.DeviceArray(ctx, B, np.float32)
        m.forward_ids(t, B, ids, out)
        ctx.sync()
        pf = oc.forward(tt._orc_model(kind, F, K, fc), B, index, np.array([0.01], np.float32), w, e, mats, 1)
        perr = np.abs(out.numpy() - pf)
        print("   forward max |p - ref| %.3g at %d" % (perr.max(), int(np.argmax(perr))), flush=True)
