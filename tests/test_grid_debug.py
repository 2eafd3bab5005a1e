"""(debug, temporary) which column group of the NT = 7 grid tower is off."""
import numpy as np
import pytest

import rmx

pytestmark = pytest.mark.gpu
F, K, FC = 39, 16, (400, 400, 400)


def test_grid_nt7_groups():
    ctx = rmx.default_context()
    B, V = 128, 50000
    base = rmx.DeepFM(V, F, K, list(FC))
    mats0 = np.array(base.initMats(0x3A75), np.float32)
    wo = len(mats0) - 401
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(0x7AB1E)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, 0x6A1D, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    for nt in (4, 7):
        for lo, hi in ((0, 112), (112, 224), (224, 336), (336, 400), (0, 400)):
            mats = mats0.copy()
            keep = mats[wo + lo:wo + hi].copy()
            mats[wo:wo + 400] = 0.0
            mats[wo + lo:wo + hi] = keep
            m = rmx.DeepFM(V, F, K, list(FC))
            m.setMats(mats)
            m.setBias(0.01)
            res = []
            for grid in (0, 1):
                rmx.set_tuning("s3_grid", 2 if grid else 0)
                rmx.set_tuning("s3_grid_nt", nt)
                rmx.set_tuning("s3_small", 0)
                rmx.set_tuning("s3_fused", 2)
                m.forward_ids(table, B, ids, out)
                ctx.sync()
                res.append(out.numpy().copy())
            d = np.abs(res[0] - res[1])
            print("nt=%d wo cols [%d, %d): max %.3g, rows off %d, first %s" % (
                nt, lo, hi, d.max(), int((d > 1e-6).sum()), np.flatnonzero(d > 1e-6)[:10].tolist()))
    for k in ("s3_grid", "s3_grid_nt", "s3_small", "s3_fused"):
        rmx.set_tuning(k, None)
