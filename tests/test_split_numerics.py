"""CPU: the numerics of the exponent-shifted fp16 split GEMMs the fused kernels run
(csrc/hpe_common.h split_w8 / split_d8 / mfma3_dw), emulated in numpy on the shapes of the path
(K = 96 channels forward, K = 32 rows per tile for dW1).  Products of fp16 values are exact in fp32,
so the emulation is exact up to the accumulation order inside one MFMA.

Scheme (C = 2^SPLIT_SHIFT = 1024): weight side h = fp16(w), cl = fp16(C (w - h)); data side
ch = fp16(C d), cl = fp16(C d - ch), h = fp16(d); acc += ch.h_w + h.cl_w + cl.h_w (= C d.w), the
consumer multiplies by 1/C.  Keeping the lo halves scaled by C keeps them normal fp16 numbers down to
|v| ~ 2.4e-4, where the unshifted split (lo = fp16(v - hi), subnormal below |v| ~ 0.1) loses bits.

Bar: the split's error against float64, relative to sum |a.b| per element
(floored at 2^-24 of the largest), stays within 4x the error of a plain fp32 fma chain (the
exact-fp32 MFMA's numerics) on the same data — including the small-magnitude
weights of a trained L2 = 0.1 checkpoint (sqnu665j) on the reference's own features."""
import os

import numpy as np
import pytest

C = np.float32(1024.0)
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def split_w(v):
    h = v.astype(np.float16)
    cl = ((v - h.astype(np.float32)) * C).astype(np.float16)
    return h, cl


def split_d(v):
    s = (v * C).astype(np.float32)
    ch = s.astype(np.float16)
    cl = (s - ch.astype(np.float32)).astype(np.float16)
    return ch, cl, v.astype(np.float16)


def pow2_scale(m, t):
    """hpe_common.h pow2_scale: power of two s with m s in [2^t, 2^(t+1)); 1 for m == 0"""
    m = np.asarray(m, np.float64)
    e = np.frexp(np.where(m > 0, m, 1.0))[1]
    return np.where(m > 0, np.ldexp(1.0, t + 1 - np.clip(e, -100, 100)), 1.0).astype(np.float32)


def split_dot(d, w, kstep=16, t=13):
    """rows of the data d (M, K) . columns of the weights w (K, N) the way mfma3_dw accumulates: each
    weight column enters scaled by s = pow2_scale(max |column|, t) (the kernels' per-column weight
    exponent); per K-step of 16 the three products (cl.h, h.cl, ch.h) are each added to the fp32
    accumulator, which holds C s x the result; the consumer's 1/(C s) is exact (power of two)."""
    sc = pow2_scale(np.abs(w).max(axis=0), t) if t is not None else np.ones(w.shape[1], np.float32)
    ch, cl, h = split_d(d)
    wh, wcl = split_w((w * sc).astype(np.float32))
    acc = np.zeros((d.shape[0], w.shape[1]), np.float32)
    for k0 in range(0, d.shape[1], kstep):
        s = slice(k0, k0 + kstep)
        for x, y in ((cl, wh), (h, wcl), (ch, wh)):
            acc = (acc.astype(np.float64) + x[:, s].astype(np.float64) @ y[s].astype(np.float64)).astype(np.float32)
    return acc / (C * sc)


def unshifted_dot(a, b, kstep=16):
    """round-1 scheme (lo = fp16(v - hi), no shift), kept to show what the shift fixes"""
    ah = a.astype(np.float16)
    al = (a - ah.astype(np.float32)).astype(np.float16)
    bh = b.astype(np.float16)
    bl = (b - bh.astype(np.float32)).astype(np.float16)
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


def _errs(d, w, fn=split_dot):
    ref = d.astype(np.float64) @ w.astype(np.float64)
    mag = np.abs(d.astype(np.float64)) @ np.abs(w.astype(np.float64))
    # elements whose whole |a|.|b| sum is below fp32's epsilon of the largest one are compared on
    # that floor: a weight of 1e-35 (L2-decayed) has no fp16 fragment, its product is an absolute
    # 1e-35 off, which no consumer of the sum can see
    mag = np.maximum(mag, 2.0 ** -24 * mag.max())
    return float(np.max(np.abs(fn(d, w) - ref) / mag)), float(np.max(np.abs(fp32_chain(d, w) - ref) / mag))


def _check(d, w):
    e_split, e_fp32 = _errs(d, w)
    assert e_split <= 4 * e_fp32, (e_split, e_fp32)
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


@pytest.mark.parametrize('wscale', [1e-2, 1e-3, 3e-4])
def test_small_magnitudes_fp32_level(wscale):
    # data ~1e-3 and weights down to 3e-4: the unshifted split's lo halves are fp16 subnormals here
    # (error ~2^-14 relative); the shifted split stays within 4x the fp32 chain
    rng = np.random.default_rng(2)
    a = (1e-3 * rng.random((64, 96))).astype(np.float32)
    b = (wscale * rng.standard_normal((96, 32))).astype(np.float32)
    e_split, e_fp32 = _check(a, b)
    e_old, _ = _errs(a, b, unshifted_dot)
    assert e_old > 8 * e_split, (e_old, e_split)
    # the exponent shift alone (no per-column weight exponent) already holds the bar down to 1e-3
    if wscale >= 1e-3:
        e_nosc, _ = _errs(a, b, lambda p, q: split_dot(p, q, t=None))
        assert e_nosc <= 4 * e_fp32, (e_nosc, e_fp32)


def test_trained_l2_checkpoint_weights_on_reference_features():
    # sqnu665j: create_model(360) trained with l2 0.1 (Model-96/Trained-Models-96-ReshapedInput-
    # NoFlatten), its W1 (96 x 360, |w| ~ 1e-3 .. 1e-1) on the reference's AFLW2000 features
    w = dict(np.load(os.path.join(GOLD, 'models', 'sqnu665j.npz')))
    k = [v for n, v in w.items() if n.endswith('kernel') and v.size == 96 * 360][0].reshape(96, 360)
    x = np.load(os.path.join(GOLD, 'data', 'AFLW2000_features_96_0.7_1.npz'))['features'][:256].astype(np.float32)
    assert np.median(np.abs(k)) < 0.05
    _check(x, k.astype(np.float32))
    # and the dW1 shape: X^T of 32 rows against a dZ1 whose columns carry tiny factors (saturated
    # tanh units, tiny W2 rows: |dZ1| from 1e-7 to 10); the kernel's dZ1 column exponent (from W2,
    # t = 2) keeps those columns' hi halves normal
    rng = np.random.default_rng(3)
    dz = (2.0 * rng.standard_normal((32, 360)) * np.abs(k[:32])).astype(np.float32)
    for t in (2, 13):
        e_split, e_fp32 = _errs(np.ascontiguousarray(x[:32].T), dz, lambda a, b: split_dot(a, b, t=t))
        assert e_split <= 4 * e_fp32, (t, e_split, e_fp32)


def test_data_side_overflow_is_non_finite():
    # |d| >= 65520 / C (64) overflows the data side's ch fragment: the accumulator becomes
    # non-finite, which is what the kernels' guard word detects before handing the launch to the
    # exact-fp32 kernel; the reference's features stay below 10.4
    a = np.ones((1, 16), np.float32)
    a[0, 3] = 70.0
    b = np.full((16, 1), 0.5, np.float32)
    with np.errstate(over='ignore', invalid='ignore'):
        assert not np.isfinite(split_dot(a, b)).all()
    a[0, 3] = 60.0
    assert np.isfinite(split_dot(a, b)).all()
