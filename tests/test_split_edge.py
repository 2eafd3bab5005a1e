"""The 3-way bf16 split (csrc/k_gemm.hpp split3, k_gemm_s3.hip pack_split3_kernel) outside the normal
range: tests/test_split_math.py covers exactness on normal fp32 values; here zeros, subnormals,
values near FLT_MAX, infinities and NaNs (host restatement of the device arithmetic: RNE casts, fp32
subtraction), and on the GPU a split-GEMM layer fed such inputs against the fp64 oracle."""
import numpy as np
import pytest


def _bf16(x):
    """round-to-nearest-even fp32 -> bf16 -> fp32 (NaN stays NaN), as v_cvt_pk_bf16_f32."""
    x = np.asarray(x, np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(np.float32)
    return np.where(np.isnan(x), np.float32(np.nan), out).astype(np.float32)


def _split3(x):
    x = np.asarray(x, np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        hi = _bf16(x)
        r = (x - hi).astype(np.float32)
        mid = _bf16(r)
        lo = _bf16((r - mid).astype(np.float32))
    return hi, mid, lo


def test_split_zero_and_subnormals_exact():
    """Zeros and the smallest normal split exactly; a subnormal loses only its bits below the bf16
    subnormal quantum 2^-133 (bf16 has fp32's exponent range but 7 stored bits): absolute error
    <= 2^-134 per element, far below one fp32 rounding of any normal-range dot product."""
    rng = np.random.default_rng(0)
    tiny = np.float32(np.finfo(np.float32).tiny)
    sub = rng.integers(1, 1 << 23, 20000).astype(np.uint32).view(np.float32)
    vals = np.concatenate([[0.0, -0.0, tiny, -tiny, 2 * tiny], sub, -sub]).astype(np.float32)
    hi, mid, lo = _split3(vals)
    rec = hi.astype(np.float64) + mid + lo
    err = np.abs(rec - vals.astype(np.float64))
    assert (err[:5] == 0).all()
    assert err.max() <= 2.0 ** -134
    q = vals.astype(np.float64) / 2.0 ** -133  # multiples of the quantum split exactly
    on_grid = q == np.round(q)
    assert (err[on_grid] == 0).all()


def test_split_near_max_and_specials():
    big = np.float32(np.finfo(np.float32).max)
    vals = np.array([big, -big, big * np.float32(0.75), np.inf, -np.inf, np.nan], np.float32)
    hi, mid, lo = _split3(vals)
    # |x| close to FLT_MAX: the bf16 rounding of hi may overflow to inf (hi*w then inf): documented limit
    assert np.isinf(hi[0]) or (hi[0] + np.float64(mid[0]) + lo[0] == np.float64(big))
    assert np.isinf(hi[3]) and np.isinf(hi[4])
    assert np.isnan(hi[5])  # a NaN input stays NaN through the split (products NaN, like fp32 sgemm)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["subnormal", "zeros", "nan", "inf"])
def test_split_gemm_special_inputs_vs_oracle(case):
    """DNN layer on the split GEMM with table rows holding subnormals / zeros / NaN / inf: outputs match
    the fp64 oracle (subnormal, zeros) or propagate NaN like an fp32 sgemm would (nan, inf -> NaN or
    saturated sigmoid)."""
    import oracle_ctypes as oc
    import rmx
    ctx = rmx.default_context()
    V, F, K, B = 1000, 39, 16, 300
    m = rmx.DNN(V, F, K, [400, 400])
    mats = m.initMats(0x3A75)
    m.setMats(mats)
    m.setBias(0.01)
    wt, et = oc.gen_table(0x7AB1E, V, K)
    et = et.copy()
    if case == "subnormal":
        et[:50] = (np.float32(1e-40) * np.sign(et[:50])).astype(np.float32)
    elif case == "zeros":
        et[:500] = 0.0
    elif case == "nan":
        et[7, 3] = np.nan
    else:
        et[7, 3] = np.inf
    table = rmx.EmbeddingTable(ctx, V, K)
    table.upload(wt, et)
    ids_h = oc.gen_ids(0x5EED2026, 0, B, F, V).astype(np.int64)
    ids = rmx.DeviceArray(ctx, B * F, np.int32)
    ids.upload(ids_h.astype(np.int32))
    out = rmx.DeviceArray(ctx, B, np.float32)
    m.forward_ids(table, B, ids, out)
    ctx.sync()
    got = out.numpy()
    w, e = oc.gather(wt, et, 1, ids_h)
    index = np.repeat(np.arange(B, dtype=np.int64), F)
    with np.errstate(invalid="ignore", over="ignore"):
        ref = oc.forward(oc.make_model(oc.DNN, F, K, fc=(400, 400)), B, index, np.array([0.01], np.float32), w, e,
                         mats, 1)
    hit = (ids_h.reshape(B, F) == 7).any(axis=1)
    if case in ("subnormal", "zeros"):
        assert np.abs(got - ref).max() <= 1e-5
    else:
        # rows that gathered the special row: NaN in the oracle -> NaN (or the same saturated value)
        assert np.array_equal(np.isnan(got[hit]), np.isnan(ref[hit]))
        assert np.abs(got[~hit] - ref[~hit]).max() <= 1e-5
