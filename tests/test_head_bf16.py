"""GPU parity of the bf16 row-owner tower layer 1 (csrc/k_head_bf16.hip), BASELINE.json configs[4] DCN:
the gathered Linear(624 -> 400) + ReLU with the cross stack's dot products as raw extra columns
(dcn/CrossEncoder.scala:40-55, DESIGN.md §4's closed form) and the first order (bnn/Scatter.scala:17-36)
fused into one persistent launch.

Each case runs DCN bf16 with the kernel forced on (knob bf16_head 2) and off (0: the column-sliced bf16
GEMM) on the same inputs.  Both compute every output as the same chain of 32-wide bf16 MFMA steps in K
order, so they agree far inside the bf16 bar (5e-5 on p, the logit's summation order aside); both are held
to the bf16 oracle (precision 2) at the build-defined 2e-4 of test_bf16.py on head / tail slices."""
import numpy as np
import pytest

import oracle_ctypes as oc
import rmx

pytestmark = pytest.mark.gpu

F, K = 39, 16
TOL_BF16 = 2e-4
HEAD_VS_ENGINE = 5e-5
SEED_IDS, SEED_TAB, SEED_MATS = 0xB16EAD, 0x7AB1E, 0x3A75


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    for k in ("bf16_head", "bf16_tail"):
        rmx.set_tuning(k, None)


def _run(ctx, kind, B, V, tails=(None,)):
    if kind == "dcn":
        m = rmx.DCN(V, F, K, 3, [400, 400, 400])
        om = oc.make_model(oc.DCN, F, K, fc=(400, 400, 400), cross_depth=3)
    else:
        m = rmx.DNN(V, F, K, [400, 400])
        om = oc.make_model(oc.DNN, F, K, fc=(400, 400))
    mats = oc.round_bf16(m.initMats(SEED_MATS))
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(mats)
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = {}
    for head in (0, 2):
        for tail in tails:
            rmx.set_tuning("bf16_head", head)
            rmx.set_tuning("bf16_tail", tail)
            m.set_timing(True)
            m.forward_ids(t, B, ids, out)
            ctx.sync()
            stages, _ = m.get_timing()
            m.set_timing(False)
            res[(head, tail)] = out.numpy().copy()
    return res, om, mats


def _oracle_errs(res, om, mats, B, V):
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
def test_bf16_head_matches_engine_and_oracle(ctx, B):
    V = 50_003
    res, om, mats = _run(ctx, "dcn", B, V, tails=(0, 1))
    d = max(float(np.abs(res[(2, t)] - res[(0, t)]).max()) for t in (0, 1))
    errs = _oracle_errs(res, om, mats, B, V)
    print("DCN bf16 B=%d |head - engine| %.3g (bitwise %s), vs bf16 oracle %s"
          % (B, d, all(np.array_equal(res[(2, t)], res[(0, t)]) for t in (0, 1)), errs))
    assert d <= HEAD_VS_ENGINE
    assert max(errs) <= TOL_BF16


def test_bf16_head_dnn_without_cross_or_first_order(ctx):
    """DNN has neither cross columns nor a first order: the kernel runs with xcol = fm_y = null."""
    B, V = 4099, 50_003
    res, om, mats = _run(ctx, "dnn", B, V)
    assert float(np.abs(res[(2, None)] - res[(0, None)]).max()) <= HEAD_VS_ENGINE
    assert max(_oracle_errs(res, om, mats, B, V)) <= TOL_BF16


def test_bf16_head_auto_selection(ctx):
    """knob 1 (auto) takes the kernel only when the row blocks fill every CU: at B = 65,536 its predictions
    are bitwise knob 2's, at B = 1,000 bitwise knob 0's (the column-sliced GEMM)."""
    V = 50_003
    m = rmx.DCN(V, F, K, 3, [400, 400, 400])
    m.setPrecision(rmx.DTYPE_BF16)
    m.setMats(oc.round_bf16(m.initMats(SEED_MATS)))
    m.setBias(0.01)
    t = rmx.EmbeddingTable(ctx, V, K, rmx.DTYPE_BF16)
    t.fill_synthetic(SEED_TAB)
    B = 65536
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    got = {}
    for knob in (0, 1, 2):
        for b in (1000, B):
            rmx.set_tuning("bf16_head", knob)
            m.forward_ids(t, b, ids, out)
            ctx.sync()
            got[(knob, b)] = out.numpy()[:b].copy()
    assert np.array_equal(got[(1, B)], got[(2, B)])
    assert np.array_equal(got[(1, 1000)], got[(0, 1000)])
