"""CPU check of the arithmetic behind the split fp32 GEMM (csrc/k_gemm_s3.hip): every normal fp32
x is exactly hi + mid + lo with three bf16 parts (round-to-nearest-even at each step, as
v_cvt_pk_bf16_f32 does), and the six kept products leave out at most ~2^-24 |x y| (|mid| <= 2^-8 |x|, |lo| <= 2^-17 |x|,
so mid*lo + lo*mid + lo*lo <= (2^-24 + 2^-34) |x y|): the size of one fp32 rounding."""
import numpy as np


def bf16_rne(x):
    b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = (b + 0x7FFF + ((b >> 16) & 1)) & 0xFFFF0000
    return r.astype(np.uint32).view(np.float32)


def split3(x):
    hi = bf16_rne(x)
    r = (x - hi).astype(np.float32)
    mid = bf16_rne(r)
    lo = bf16_rne((r - mid).astype(np.float32))
    return hi, mid, lo


def test_split_is_exact():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(200000).astype(np.float32),
                        (rng.random(100000) * 1e-3).astype(np.float32),
                        rng.uniform(-0.05, 0.05, 100000).astype(np.float32)])
    hi, mid, lo = split3(x)
    # every part is a bf16 value, and the sum (in fp64, exact) reproduces x bit for bit
    for part in (hi, mid, lo):
        assert np.array_equal(bf16_rne(part), part)
    assert np.array_equal((hi.astype(np.float64) + mid + lo).astype(np.float32), x)
    assert np.all(hi.astype(np.float64) + mid + lo == x.astype(np.float64))


def test_dropped_products_below_fp32_rounding():
    rng = np.random.default_rng(1)
    x = rng.standard_normal(100000).astype(np.float32)
    y = rng.standard_normal(100000).astype(np.float32)
    xh, xm, xl = (p.astype(np.float64) for p in split3(x))
    yh, ym, yl = (p.astype(np.float64) for p in split3(y))
    kept = xh * yh + xh * ym + xm * yh + xh * yl + xl * yh + xm * ym
    exact = x.astype(np.float64) * y.astype(np.float64)
    rel = np.abs(kept - exact) / np.abs(exact)
    assert rel.max() <= 2.0 ** -24 * (1 + 2.0 ** -9)
    # each kept product of two bf16 values is exact in fp32 (8 x 8 significand bits)
    for a, b in ((xh, yh), (xh, ym), (xm, yh), (xh, yl), (xl, yh), (xm, ym)):
        prod = a * b
        assert np.array_equal(prod.astype(np.float32).astype(np.float64), prod)
