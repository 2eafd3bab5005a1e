"""GPU parity of PNN's tower layer 1 with the inner products generated on chip (csrc/k_pnn_head.hip),
BASELINE.json configs[4] (bf16): Linear([x || ip] -> N1) + ReLU, x the gathered rows and ip the pair dot
products (pnn/ProductEncoder.scala:72-120, bnn/DotProduct2.scala:16-26, HigherOrderEncoder.scala:34-59),
without the [x || ip] row in HBM.

Each case runs PNN bf16 with the kernel forced on (knob pnn_head 2) and off (0: product16_kernel + the
column-sliced GEMM) on the same inputs.  The two compute ip in fp32 in different orders (v_dot2 pairs vs
MFMA) and both round it to bf16 once, so an ip can differ by one bf16 ulp where the fp32 sums straddle a
rounding boundary; the layer's K order differs too (quads vs lexicographic).  Bars: 1e-4 between the
paths, and the build-defined bf16 bar of test_bf16.py (2e-4) against the bf16 oracle (precision 2:
rows, ip and activations rounded to bf16 at the same points) on head / tail slices."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

K = 16
TOL_BF16 = 2e-4
HEAD_VS_ENGINE = 1e-4
SEED_IDS, SEED_TAB, SEED_MATS = 0x9A1E, 0x7AB1E, 0x3A75


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    rmx.set_tuning("pnn_head", None)


def _run(ctx, F, fc, B, V, knobs=(0, 2)):
    m = rmx.PNN(V, F, K, list(fc))
    om = oc.make_model(oc.PNN, F, K, fc=tuple(fc))
    mats = oc.round_bf16(m.initMats(SEED_MATS))
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res, stages = {}, {}
    for knob in knobs:
        rmx.set_tuning("pnn_head", knob)
        m.set_timing(True)
        m.forward_ids(t, B, ids, out)
        ctx.sync()
        st, _ = m.get_timing()
        m.set_timing(False)
        res[knob] = out.numpy().copy()
        stages[knob] = set(st)
    return res, stages, om, mats


def _oracle_errs(res, om, mats, F, B, V):
    wt, et = oc.gen_table(SEED_TAB, V, K)
    wt, et = oc.round_bf16(wt), oc.round_bf16(et)
    errs = []
    for r0 in sorted({0, max(0, B - 200)}):
        n = min(200, B - r0)
        h = oc.gen_ids(SEED_IDS, r0, n, F, V).astype(np.int64)
        w, e = oc.gather(wt, et, 1, h)
        ref = oc.forward(om, n, np.repeat(np.arange(n, dtype=np.int64), F), np.array([0.01], np.float32), w, e, mats, 2)
        errs.append(max(float(np.abs(r[r0:r0 + n] - ref).max()) for r in res.values()))
    return errs


@pytest.mark.parametrize("B", [1, 37, 1000, 19217, 65536])
def test_pnn_head_matches_engine_and_oracle(ctx, B):
    F, V = 39, 50_003
    res, stages, om, mats = _run(ctx, F, (400, 400, 400), B, V)
    assert "product" in stages[0] and "product" not in stages[2], stages
    d = float(np.abs(res[2] - res[0]).max())
    errs = _oracle_errs(res, om, mats, F, B, V)
    print("PNN bf16 F=39 B=%d |head - engine| %.3g, vs bf16 oracle %s" % (B, d, errs))
    assert d <= HEAD_VS_ENGINE
    assert max(errs) <= TOL_BF16


@pytest.mark.parametrize("F", [2, 3, 8, 17, 26, 40])
def test_pnn_head_other_field_counts(ctx, F):
    """The quad order, the packed K order and the DMA schedule are built per F (odd F: the last x step
    carries one field and a zero row; F = 40: the whole 40-field image)."""
    V, B = 20_011, 3001
    res, stages, om, mats = _run(ctx, F, (400, 400), B, V)
    assert "product" not in stages[2], stages
    assert float(np.abs(res[2] - res[0]).max()) <= HEAD_VS_ENGINE
    assert max(_oracle_errs(res, om, mats, F, B, V)) <= TOL_BF16


def test_pnn_head_not_taken_for_narrow_layer(ctx):
    """A 64-wide layer 1 (Npad != 416) keeps the unfused path, bitwise."""
    res, stages, _, _ = _run(ctx, 39, (64,), 517, 5000)
    assert "product" in stages[2]
    assert np.array_equal(res[2], res[0])
