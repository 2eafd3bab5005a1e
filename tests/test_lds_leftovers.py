"""No kernel of the forward reads LDS it did not write (csrc/*: the engine, the row-owner head / tail, the
bf16 tail, the whole-tower kernel, the CIN layers).

Each case fills every CU's LDS (rmx_debug_fill_lds: one 160-KiB workgroup per CU, four rounds) with a
pattern -- a NaN, an infinity, 1.0 -- right before the forward and compares the output with the one after
a fill of zeros: bitwise equal and finite.  A kernel that read a never-written pad (padding columns whose
weights are zero, say) would see 0 x NaN = NaN, which a ReLU turns into a silently wrong 0; the fill makes
that visible whatever ran before on the CU.  Models: every tower model at the fp32 and the bf16 settings
of BASELINE.json configs[1], [2] and [4], at a small, a ragged and the bench batch."""
import numpy as np
import pytest

import rmx

pytestmark = pytest.mark.gpu

F, K = 39, 16
SEED_IDS, SEED_TAB, SEED_MATS = 0x1DF5, 0x7AB1E, 0x3A75
PATTERNS = (0x7FC00000, 0x7F800000, 0x3F800000)


@pytest.fixture(scope="module")
def ctx():
    return rmx.default_context()


KNOBS = ("s3_head", "s3_tail", "s3_fused")


@pytest.fixture(autouse=True)
def _restore_knobs():
    yield
    for k in KNOBS:
        rmx.set_tuning(k, None)


def _model(kind, V):
    fc = [400, 400, 400]
    return {
        "deepfm": lambda: rmx.DeepFM(V, F, K, fc),
        "dnn": lambda: rmx.DNN(V, F, K, fc),
        "xdeepfm": lambda: rmx.XDeepFM(V, F, K, fc, [200, 200, 200]),
        "dcn": lambda: rmx.DCN(V, F, K, 3, fc),
        "pnn": lambda: rmx.PNN(V, F, K, fc),
        "lr": lambda: rmx.LR(V, F),
    }[kind]()


def _check(ctx, kind, B, bf16=False, knobs=()):
    V = 100_003
    for k, v in knobs:
        rmx.set_tuning(k, v)
    m = _model(kind, V)
    dt = rmx.DTYPE_BF16 if bf16 else rmx.DTYPE_F32
    t = rmx.EmbeddingTable(ctx, V, K, dt)
    t.fill_synthetic(SEED_TAB)
    if bf16:
        m.setPrecision(rmx.DTYPE_BF16)
    if kind != "lr":
        m.setMats(m.initMats(SEED_MATS))
    m.setBias(0.01)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    rmx.gen_ids(ctx, SEED_IDS, 0, B, F, V, ids)
    out = rmx.DeviceArray(ctx, B, np.float32)
    res = []
    for pat in (0,) + PATTERNS:
        rmx.debug_fill_lds(ctx, pat)
        m.forward_ids(t, B, ids, out)
        ctx.sync()
        res.append(out.numpy().copy())
    for pat, r in zip(PATTERNS, res[1:]):
        assert np.isfinite(r).all(), hex(pat)
        bad = np.flatnonzero(r != res[0])
        assert bad.size == 0, "pattern %s: %d rows differ (first %s, max |d| %.3g)" % (
            hex(pat), bad.size, bad[:8].tolist(), float(np.abs(r - res[0]).max()))


@pytest.mark.parametrize("B", [1000, 4096, 8192, 19217, 65536])
@pytest.mark.parametrize("kind", ["deepfm", "dnn", "dcn", "pnn", "lr"])
def test_fp32_forward_ignores_lds_leftovers(ctx, kind, B):
    _check(ctx, kind, B)


@pytest.mark.parametrize("B", [19217, 65536])
def test_deepfm_head_and_tail_ignore_lds_leftovers(ctx, B):
    """DeepFM on the head + tail pair (s3_fused 0) instead of the default fused tower."""
    _check(ctx, "deepfm", B, knobs=(("s3_fused", 0),))


@pytest.mark.parametrize("B", [1000, 16384])
def test_xdeepfm_forward_ignores_lds_leftovers(ctx, B):
    _check(ctx, "xdeepfm", B)


@pytest.mark.parametrize("B", [1000, 19217, 65536])
@pytest.mark.parametrize("kind", ["dcn", "pnn", "deepfm"])
def test_bf16_forward_ignores_lds_leftovers(ctx, kind, B):
    _check(ctx, kind, B, bf16=True)
