"""The bench configurations checked across the whole batch.

The other full-batch tests compare a few slices of a bench batch with the oracle.  Here a strided
sample touches every row block and every iteration of the persistent row-owner loops: every 32nd row
of B = 65,536 (DeepFM configs[1], xDeepFM CIN 1x200 reference-exact, DCN / PNN bf16 configs[4]) and
every 16th row of B = 16,384 (xDeepFM CIN 3x200, configs[2]).  A 128-row block of the row-owner
kernels then holds four checked rows (eight for xDeepFM's 256-row CIN tiles), whichever CU and loop
iteration ran it.  fp32 models are held to |p_gpu - p_oracle| <= 1e-5 against BOTH the fp64 oracle and
the fp32 oracle in BigDL's summation order (precision 0); bf16 models to 2e-4 against the oracle's
bf16-storage emulation (precision 2).  The ids are bench.py's (same seeds, same set)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

F, K, V = 39, 16, 1_000_000
FC = [400, 400, 400]
SEED_IDS, SEED_TAB, SEED_MATS = 0x5EED2026, 0x7AB1E, 0x3A75
TOL, TOL_BF16 = 1e-5, 2e-4


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(scope="module")
def host_table():
    return oc.gen_table(SEED_TAB, V, K)


CASES = {
    # name: (rmx model, oracle model, B, stride, bf16)
    "deepfm": (lambda: rmx.DeepFM(V, F, K, FC), lambda: oc.make_model(oc.DEEPFM, F, K, fc=tuple(FC)), 65536, 32,
               False),
    "xdeepfm": (lambda: rmx.XDeepFM(V, F, K, FC, [200, 200, 200]),
                lambda: oc.make_model(oc.XDEEPFM, F, K, fc=tuple(FC), cin=(200, 200, 200)), 16384, 16, False),
    "xdeepfm_cin1": (lambda: rmx.XDeepFM(V, F, K, FC, [200]),
                     lambda: oc.make_model(oc.XDEEPFM, F, K, fc=tuple(FC), cin=(200,)), 65536, 32, False),
    "dcn_bf16": (lambda: rmx.DCN(V, F, K, 3, FC), lambda: oc.make_model(oc.DCN, F, K, fc=tuple(FC), cross_depth=3),
                 65536, 32, True),
    "pnn_bf16": (lambda: rmx.PNN(V, F, K, FC), lambda: oc.make_model(oc.PNN, F, K, fc=tuple(FC)), 65536, 32, True),
}


@pytest.mark.parametrize("name", list(CASES))
def test_bench_config_strided_rows(ctx, host_table, name):
    mk, mko, B, stride, bf16 = CASES[name]
    m = mk()
    if bf16:
        m.setPrecision(rmx.DTYPE_BF16)
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16 if bf16 else rmx.DTYPE_F32)
    table.fill_synthetic(SEED_TAB)
    ids_dev = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids_dev)
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids_dev, out)
    ctx.sync()
    got = out.numpy().copy()
    assert np.isfinite(got).all()
    h_ids = ids_dev.numpy().reshape(B, F)
    assert np.array_equal(h_ids, oc.gen_ids(SEED_IDS, 0, B, F, V).reshape(B, F))
    rows = np.arange(0, B, stride)
    rows = np.union1d(rows, [B - 1])  # and the batch's last row
    n = rows.size
    ids = h_ids[rows].astype(np.int64).ravel()
    wt, et = host_table
    w, e = oc.gather(wt, et, 1, ids)
    index = np.repeat(np.arange(n, dtype=np.int64), F)
    bias = np.array([0.01], np.float32)
    om = mko()
    if bf16:
        ref = oc.forward(om, n, index, bias, oc.round_bf16(w), oc.round_bf16(e), mats, 2)
        err = float(np.abs(got[rows] - ref).max())
        print("%s: %d strided rows, max|p - p_bf16_emulation| = %.3g" % (name, n, err))
        assert err <= TOL_BF16
    else:
        ref64 = oc.forward(om, n, index, bias, w, e, mats, 1)
        ref32 = oc.forward(om, n, index, bias, w, e, mats, 0)
        e64 = float(np.abs(got[rows] - ref64).max())
        e32 = float(np.abs(got[rows] - ref32).max())
        print("%s: %d strided rows, max|p - p_fp64| = %.3g, max|p - p_fp32| = %.3g" % (name, n, e64, e32))
        assert e64 <= TOL and e32 <= TOL
    # every row block holds a checked row: the largest gap between checked rows is the stride
    assert np.diff(rows).max() <= stride
