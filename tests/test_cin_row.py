"""GPU parity of xDeepFM's CIN stack as one row-owner kernel (csrc/k_cin_row.hip): every CIN layer of a
sample in one wave, the maps u_l kept in registers, the output dot of the pooled maps summed on the fly
(xdeepfm/CINEncoder.scala:135-176, XDeepFM.scala:62-86).

Each case runs xDeepFM with the kernel forced on (knob cin_row 2) and off (0: one split-GEMM launch per layer,
u_l through HBM) on the same inputs.  Both use the same split arithmetic (three bf16 planes, six products
per K step); the K order differs (padded chunk pairs), so the two agree to fp32 rounding, and both are held
to the fp64 oracle at the north-star 1e-5 on head / tail slices."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

TOL = 1e-5
ROW_VS_ENGINE = 3e-6
K = 16
SEED_IDS, SEED_TAB, SEED_MATS = 0xC1A, 0x7AB1E, 0x3A75


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    rmx.set_tuning("cin_row", None)


def _run(ctx, F, cin, fc, B, V):
    m = rmx.XDeepFM(V, F, K, list(fc), list(cin))
    mats = m.initMats(SEED_MATS)
    m.setMats(mats)
    m.setBias(0.01)
    table = rmx.EmbeddingTable(ctx, V, K)
    table.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res, stages = {}, {}
    for knob in (0, 2):
        rmx.set_tuning("cin_row", knob)
        m.set_timing(True)
        m.forward_ids(table, B, ids, out)
        ctx.sync()
        st, _ = m.get_timing()
        m.set_timing(False)
        res[knob] = out.numpy().copy()
        stages[knob] = set(st)
    return res, stages, mats


def _oracle_errs(res, F, cin, fc, mats, B, V, n=48):
    om = oc.make_model(oc.XDEEPFM, F, K, fc=tuple(fc), cin=tuple(cin))
    wt, et = oc.gen_table(SEED_TAB, V, K)
    errs = []
    for r0 in sorted({0, max(0, B - n)}):
        nn = min(n, B - r0)
        h = oc.gen_ids(SEED_IDS, r0, nn, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, h)
        ref = oc.forward(om, nn, np.repeat(np.arange(nn, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats,
                         1, 16)
        errs.append(max(float(np.abs(r[r0:r0 + nn] - ref).max()) for r in res.values()))
    return errs


@pytest.mark.parametrize("B", [1, 9, 1000, 16384])
def test_cin_row_headline_config(ctx, B):
    """configs[2]'s CIN (200, 200, 200) over F = 39; B = 1 and 9 leave most of a group of 8 samples empty."""
    F, cin, fc, V = 39, (200, 200, 200), (400, 400, 400), 100_000
    res, stages, mats = _run(ctx, F, cin, fc, B, V)
    assert "cin" in stages[2] and "cin" not in stages[0], stages
    d = float(np.abs(res[2] - res[0]).max())
    errs = _oracle_errs(res, F, cin, fc, mats, B, V)
    print("xDeepFM B=%d |row - engine| %.3g, vs fp64 %s" % (B, d, errs))
    assert d <= ROW_VS_ENGINE
    assert max(errs) <= TOL


@pytest.mark.parametrize("F,cin", [(17, (208,)), (40, (200,)), (13, (200, 200)), (24, (200, 200)),
                                   (39, (200, 200, 200, 200))])
def test_cin_row_other_shapes(ctx, F, cin):
    """Layer 1 with 1, 2 or 3 h-chunks (F = 13, 17 / 24, 39 / 40), a single 208-map layer (no pair chunk),
    four layers."""
    B, V, fc = 700, 20_011, (64,)
    res, stages, mats = _run(ctx, F, cin, fc, B, V)
    assert "cin" in stages[2], stages
    assert float(np.abs(res[2] - res[0]).max()) <= ROW_VS_ENGINE
    assert max(_oracle_errs(res, F, cin, fc, mats, B, V, n=32)) <= TOL


def test_cin_row_falls_back_for_unequal_layers(ctx):
    """Unequal layer widths keep the per-layer engine, bitwise."""
    res, stages, _ = _run(ctx, 39, (200, 196, 208), (64,), 300, 5000)
    assert "cin" not in stages[2]
    assert np.array_equal(res[2], res[0])
