"""CPU: the numerics of the fp16 hi/lo split GEMMs the fused kernels run (csrc/hpe_common.h split8 /
mfma3: a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi with fp16 halves, fp32 accumulate), emulated in numpy
on the shapes of the path (K = 96 channels forward, K = 32 rows per tile for dW1).  Products of fp16
values are exact in fp32, so the emulation is exact up to the accumulation order inside one MFMA.
Bar: the split dot's error against float64 stays within 4x the error of a plain fp32 fma chain (the
exact-fp32 MFMA's numerics) on the same data, and below 2^-20 of sum |a.b|."""
import numpy as np


def split(v):
    hi = v.astype(np.float16)
    lo = (v - hi.astype(np.float32)).astype(np.float16)
    return hi, lo


def split_dot(a, b, kstep=16):
    """rows of a (M, K) . columns of b (K, N) the way mfma3 accumulates: per K-step of 16, the
    three products (lo.hi, hi.lo, hi.hi) are each added to the fp32 accumulator."""
    ah, al = split(a)
    bh, bl = split(b)
    acc = np.zeros((a.shape[0], b.shape[1]), np.float32)
    for k0 in range(0, a.shape[1], kstep):
        s = slice(k0, k0 + kstep)
        for x, y in ((al, bh), (ah, bl), (ah, bh)):
            acc = (acc.astype(np.float64) + x[:, s].astype(np.float64) @ y[s].astype(np.float64)).astype(np.float32)
    return acc


def fp32_chain(a, b):
    acc = np.zeros((a.shape[0], b.shape[1]), np.float32)
    for k in range(a.shape[1]):
        acc = (acc + a[:, k:k + 1] * b[k:k + 1]).astype(np.float32)
    return acc


def _check(a, b):
    ref = a.astype(np.float64) @ b.astype(np.float64)
    mag = np.abs(a.astype(np.float64)) @ np.abs(b.astype(np.float64))
    e_split = np.max(np.abs(split_dot(a, b) - ref) / mag)
    e_fp32 = np.max(np.abs(fp32_chain(a, b) - ref) / mag)
    assert e_split <= max(4 * e_fp32, 2.0 ** -22), (e_split, e_fp32)
    assert e_split < 2.0 ** -20, e_split
    return e_split, e_fp32


def test_forward_gemm_96_channels():
    rng = np.random.default_rng(0)
    x = np.maximum(0.0, 0.6 * rng.standard_normal((256, 96)) - 0.3).astype(np.float32)
    w = (0.1 * rng.standard_normal((96, 64))).astype(np.float32)
    _check(x, w)


def test_dw1_gemm_unnormalised_gradients():
    # X^T (96 channels x 32 rows) . dZ1 (32 rows x 64 units), dZ1 = 2 (p - y) W2 act' ~ O(1..100)
    rng = np.random.default_rng(1)
    xt = np.maximum(0.0, 0.6 * rng.standard_normal((96, 32)) - 0.3).astype(np.float32)
    dz = (40.0 * rng.standard_normal((32, 64)) * rng.random((32, 64))).astype(np.float32)
    _check(xt, dz)


def test_small_magnitudes_absolute_floor():
    # values around 1e-3 put the lo halves in fp16's subnormal range: the absolute floor (2^-24 per
    # lo term) keeps the error at the fp32 level relative to sum |a.b|
    rng = np.random.default_rng(2)
    a = (1e-3 * rng.random((64, 96))).astype(np.float32)
    b = (1e-2 * rng.standard_normal((96, 32))).astype(np.float32)
    ref = a.astype(np.float64) @ b.astype(np.float64)
    mag = np.abs(a.astype(np.float64)) @ np.abs(b.astype(np.float64))
    assert np.max(np.abs(split_dot(a, b) - ref) / mag) < 2.0 ** -14


def test_fp16_range_overflow_is_non_finite():
    # |x| >= 65520 overflows the hi half: the accumulator becomes non-finite, which is what the
    # kernels' guard word detects before handing the launch to the exact-fp32 kernel
    a = np.ones((1, 16), np.float32)
    a[0, 3] = 1.0e5
    b = np.full((16, 1), 0.5, np.float32)
    with np.errstate(over='ignore', invalid='ignore'):
        assert not np.isfinite(split_dot(a, b)).all()
