"""Numpy emulator of the row-program semantics (csrc/hpe_prog.h) — TEST INFRASTRUCTURE.

Executes the same op words the HIP kernel interprets, element by element in float64, so the
compiler's lowering (fusion, backward construction, in-place slot reuse) is checked on CPU
against the oracle before the GPU checks the kernel against both.  Not importable by the product.
"""
import struct

import numpy as np

import hpe.compiler as C


def _i2f(i):
    return struct.unpack('<f', struct.pack('<i', int(i)))[0]


def _act(a, z):
    if a == 0:
        return z
    if a == 1:
        return np.tanh(z)
    if a == 2:
        return np.maximum(z, 0)
    if a == 3:
        return z / (1 + np.abs(z))
    if a == 4:
        return 1 / (1 + np.exp(-z))
    if a == 5:
        return np.where(z > 0, z, np.expm1(z))
    if a == 6:
        return 1.0507009873554805 * np.where(z > 0, z, 1.6732632423543772 * np.expm1(z))
    if a == 7:
        return z / (1 + np.exp(-z))
    if a == 8:
        return np.where(z > 20, z, np.log1p(np.exp(np.minimum(z, 20))))
    if a == 9:
        return np.where(z > 0, z, 0.2 * z)
    raise ValueError(a)


def _dact(a, v, z):
    if a == 0:
        return np.ones_like(v)
    if a == 1:
        return 1 - v * v
    if a == 2:
        return (v > 0).astype(v.dtype)
    if a == 3:
        return (1 - np.abs(v)) ** 2
    if a == 4:
        return v * (1 - v)
    if a == 5:
        return np.where(v > 0, 1, v + 1)
    if a == 6:
        return np.where(v > 0, 1.0507009873554805, v + 1.0507009873554805 * 1.6732632423543772)
    if a == 7:
        s = 1 / (1 + np.exp(-z))
        return s * (1 + z * (1 - s))
    if a == 8:
        return -np.expm1(-v)
    if a == 9:
        return np.where(v > 0, 1, 0.2)
    raise ValueError(a)


def _hash(seed, did, img, ch):
    """csrc/hpe_common.h drop_hash: 64-bit splitmix of (seed, ordinal, image), 32-bit finaliser of
    (its high word, channel)."""
    with np.errstate(over='ignore'):
        x = np.uint64((int(seed) + 0x9E3779B97F4A7C15 * (1 + int(did))) & ((1 << 64) - 1))
        x = x ^ (img.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9))
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
        b = (x >> np.uint64(32)).astype(np.uint32)
        h = b ^ (ch.astype(np.uint32) * np.uint32(0x9E3779B9))
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x85EBCA6B)
        h = h ^ (h >> np.uint32(13))
        h = h * np.uint32(0xC2B2AE35)
        h = h ^ (h >> np.uint32(16))
        return h.astype(np.uint32)


def run(prog, params, x_rows, P=1, y_img=None, inv_count=1.0, seed=0, img_off=0):
    """Returns dict(out=..., grad=flat gradient (n_train), sse, sae)."""
    w = prog.words.astype(np.int64)
    hdr = w[:C.H_WORDS]
    nslots, nops = int(hdr[C.H_NSLOTS]), int(hdr[C.H_NOPS])
    so, oo = int(hdr[C.H_SLOTS_OFF]), int(hdr[C.H_OPS_OFF])
    slots = [w[so + 4 * i: so + 4 * i + 4] for i in range(nslots)]
    ops = [w[oo + C.O_WORDS * i: oo + C.O_WORDS * (i + 1)] for i in range(nops)]
    mode = int(hdr[C.H_MODE])
    R = x_rows.shape[0]
    p = np.asarray(params, dtype=np.float64)
    pt = C.build_mirror(prog, np.asarray(params[:prog.n_train], np.float32)).astype(np.float64)
    S = [np.zeros((R, int(s[1]))) for s in slots]
    S[int(hdr[C.H_IN_SLOT])] = np.asarray(x_rows, dtype=np.float64).copy()
    img = np.arange(R) // P + img_off
    grad = np.zeros(prog.n_train)
    sse = sae = 0.0

    def epi(o):
        return (int(o[C.O_EACT]), int(o[C.O_EDROP]), int(o[C.O_ETHR]) & 0xFFFFFFFF,
                _i2f(o[C.O_EKEEP]), int(o[C.O_EZ]))

    def mask(did, thr, n):
        ch = np.arange(n)[None, :]
        return _hash(seed, did, img[:, None], ch) >= np.uint32(thr)

    def efwd(o, z):
        a, did, thr, keep, zs = epi(o)
        v = _act(a, z)
        if did >= 0:
            v = np.where(mask(did, thr, z.shape[1]), v / keep, 0.0)
        return v

    def ebwd(o, g, val):
        a, did, thr, keep, zs = epi(o)
        z = S[zs] if zs >= 0 else None
        if did >= 0:
            m = mask(did, thr, g.shape[1])
            g = np.where(m, g / keep, 0.0)
            val = val * keep
        return g if a == 0 else g * _dact(a, val, z)

    def W(o, K, N, transposed_buf=False):
        off = int(o[C.O_W])
        src = pt if (int(o[C.O_WSEL]) != transposed_buf) else p
        return src[off:off + K * N].reshape(K, N)

    def dst(o, d, v):
        mode_ = int(o[C.O_MODE])
        if mode_ == C.DST_STORE:
            S[d][:] = v
        elif mode_ == C.DST_ACCUM:
            S[d][:] += v
        else:
            vs = int(o[C.O_AUX0])
            S[d][:] = ebwd(o, v, S[vs].copy())

    for o in ops:
        t = int(o[C.O_TYPE])
        a, b, out = int(o[C.O_A]), int(o[C.O_B]), int(o[C.O_OUT])
        K, N = int(o[C.O_K]), int(o[C.O_N])
        if t in (C.OP_DENSE, C.OP_TDENSE):
            z = S[a] @ W(o, K, N)
            if o[C.O_BIAS] >= 0:
                z = z + p[int(o[C.O_BIAS]):int(o[C.O_BIAS]) + N]
            if o[C.O_EZ] >= 0:
                S[int(o[C.O_EZ])][:] = z
            S[out][:] = efwd(o, z)
        elif t == C.OP_EW:
            fl = int(o[C.O_FLAGS])
            f0, f1 = _i2f(o[C.O_F0]), _i2f(o[C.O_F1])
            Cc = S[out].shape[1]
            if fl & C.EW_MUL:
                v = S[a] * S[b]
            else:
                v = f0 * S[a] + (f1 * S[b] if fl & C.EW_HAS_B else 0)
            if fl & C.EW_AFFINE:
                v = v * p[int(o[C.O_AUX0]):int(o[C.O_AUX0]) + Cc]
                if o[C.O_AUX1] >= 0:
                    v = v + p[int(o[C.O_AUX1]):int(o[C.O_AUX1]) + Cc]
            if o[C.O_EZ] >= 0:
                S[int(o[C.O_EZ])][:] = v
            S[out][:] = efwd(o, v)
        elif t == C.OP_LN:
            x = S[a]
            mu = x.mean(1, keepdims=True)
            var = ((x - mu) ** 2).mean(1, keepdims=True)
            rs = 1 / np.sqrt(var + _i2f(o[C.O_F0]))
            xh = (x - mu) * rs
            y = xh.copy()
            Cc = x.shape[1]
            if o[C.O_AUX0] >= 0:
                y = y * p[int(o[C.O_AUX0]):int(o[C.O_AUX0]) + Cc]
            if o[C.O_AUX1] >= 0:
                y = y + p[int(o[C.O_AUX1]):int(o[C.O_AUX1]) + Cc]
            S[out][:] = efwd(o, y)
            if o[C.O_AUX2] >= 0:
                S[int(o[C.O_AUX2])][:] = xh
            if o[C.O_AUX3] >= 0:
                S[int(o[C.O_AUX3])][:] = rs
        elif t == C.OP_LOSS:
            pr = S[a]
            e = pr - y_img[img - img_off]
            sse += float((e * e).sum())
            sae += float(np.abs(e).sum())
            if mode == C.MODE_TRAIN:
                S[out][:] = ebwd(o, 2 * e * inv_count, pr.copy())
        elif t == C.OP_EPIGRAD:
            S[out][:] = ebwd(o, S[out].copy(), S[a].copy())
        elif t == C.OP_DW:
            off = int(o[C.O_W])
            grad[off:off + K * N] += (S[a].T @ S[b]).ravel()
        elif t == C.OP_TACC:
            tm = int(o[C.O_AUX3])
            off = int(o[C.O_W])
            if tm == C.TACC_GEMM:
                grad[off:off + K * N] += (S[a].T @ S[b]).ravel()
            elif tm == C.TACC_BIAS:
                grad[off:off + N] += S[b].sum(0)
            else:
                grad[off:off + N] += (S[a] * S[b]).sum(0)
        elif t == C.OP_DIN:
            wt = W(o, N, K, True)    # mirror (params_t) holds W^T [N][K]
            dst(o, out, S[a] @ wt)
        elif t == C.OP_TDIN:
            wk = W(o, K, N)
            dst(o, out, S[a] @ wk.T)
        elif t == C.OP_EWB:
            fl = int(o[C.O_FLAGS])
            f0, f1 = _i2f(o[C.O_F0]), _i2f(o[C.O_F1])
            g = S[out].copy()
            Cc = g.shape[1]
            if fl & C.EW_AFFINE:
                g = g * p[int(o[C.O_AUX2]):int(o[C.O_AUX2]) + Cc]
            if fl & C.EW_MUL:
                g0, g1 = g * S[b], g * S[a]
            else:
                g0, g1 = f0 * g, f1 * g
            m = int(o[C.O_MODE])
            d0, d1 = int(o[C.O_AUX0]), int(o[C.O_AUX1])
            if d0 >= 0:
                S[d0][:] = (S[d0] + g0) if m & 1 else g0
            if d1 >= 0:
                S[d1][:] = (S[d1] + g1) if m & 2 else g1
        elif t == C.OP_LNB:
            xh, g = S[a], S[b]
            Cc = g.shape[1]
            gam = p[int(o[C.O_AUX0]):int(o[C.O_AUX0]) + Cc] if o[C.O_AUX0] >= 0 else 1.0
            dxh = g * gam
            m1 = dxh.mean(1, keepdims=True)
            m2 = (dxh * xh).mean(1, keepdims=True)
            rs = S[int(o[C.O_AUX1])][:, :1]
            v = rs * (dxh - m1 - xh * m2)
            if int(o[C.O_MODE]) == C.DST_ACCUM:
                S[out][:] += v
            else:
                S[out][:] = v
        else:
            raise ValueError('op %d' % t)
    return {'out': S[int(hdr[C.H_OUT_SLOT])], 'grad': grad, 'sse': sse, 'sae': sae}


def run_chain(prog, params, x_rows):
    """KIND_CHAIN program (csrc/hpe_chain.hip): x -> dense F1 -> [dense F2] -> dense 3, from the op
    words alone (field map in csrc/hpe_prog.h OP_CHAIN)."""
    w = prog.words.astype(np.int64)
    o = w[int(w[C.H_OPS_OFF]):]
    assert int(o[C.O_TYPE]) == C.OP_CHAIN
    p = np.asarray(params, dtype=np.float64)
    cin, f1, f2 = int(o[C.O_K]), int(o[C.O_N]), int(o[C.O_AUX3])

    def dense(x, wo, bo, k, n, act):
        z = x @ p[wo:wo + k * n].reshape(k, n)
        if bo >= 0:
            z = z + p[bo:bo + n]
        return _act(act, z)
    h = dense(np.asarray(x_rows, np.float64), int(o[C.O_W]), int(o[C.O_BIAS]), cin, f1, int(o[C.O_EACT]))
    fh = f1
    if f2 > 0:
        h = dense(h, int(o[C.O_AUX0]), int(o[C.O_AUX1]), f1, f2, int(o[C.O_FLAGS]))
        fh = f2
    return dense(h, int(o[C.O_AUX2]), int(o[C.O_TBASE]), fh, int(o[C.O_TCOUNT]), int(o[C.O_MODE]))
