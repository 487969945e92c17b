"""Numpy emulator of the BlazeFace plan words (csrc/hpe_prog.h BFO_*) — TEST INFRASTRUCTURE.

Executes exactly what csrc/hpe_blaze.hip computes from the plan (padded channel strides, the stem's
6-row W^T table, depthwise tables, split head epilogue) in float64, so the plan builder's parameter
packing is checked against the oracle on CPU before the GPU runs the kernels.
"""
import numpy as np

from hpe import blazeface as B


def _f(words, i):
    o = int(words[B.BFH_OPS_OFF]) + i * B.BFO_WORDS
    return [int(v) for v in words[o:o + B.BFO_WORDS]]


def run(plan, images):
    words, P = plan['words'], plan['params'].astype(np.float64)
    n = images.shape[0]
    bufs = {B.BUF_IMG: images.astype(np.float64)}
    for i in range(int(words[B.BFH_NOPS])):
        f = _f(words, i)
        if f[B.BFO_KIND] in (B.BF_STAGE, B.BF_FRONT):   # execution records: their ops follow as ordinary records
            continue
        x = bufs[f[B.BFO_SRC]]
        H, W, Ho, Wo = f[B.BFO_H], f[B.BFO_W], f[B.BFO_HO], f[B.BFO_WO]
        if f[B.BFO_KIND] == B.BF_STEM:
            wt = P[f[B.BFO_PWW]:f[B.BFO_PWW] + 32 * 90].reshape(32, 6, 5, 3)
            b = P[f[B.BFO_PWB]:f[B.BFO_PWB] + 32]
            pt, pl = f[B.BFO_PADT], f[B.BFO_PADL]
            xp = np.zeros((n, 2 * Ho + 6, 2 * Wo + 5, 3))
            xp[:, pt:pt + H, pl:pl + W] = x
            y = np.zeros((n, Ho, Wo, 32))
            for ky in range(6):
                for kx in range(5):
                    win = xp[:, ky:ky + 2 * Ho:2, kx:kx + 2 * Wo:2, :]      # (n,Ho,Wo,3)
                    y += win @ wt[:, ky, kx, :].T
            y = np.maximum(y + b, 0)[..., :f[B.BFO_COUT]]
            bufs[f[B.BFO_DST]] = y
            continue
        cinp, cout, coutp = f[B.BFO_CINP], f[B.BFO_COUT], f[B.BFO_COUTP]
        s = f[B.BFO_STRIDE]
        xin = x.reshape(n, H, W, -1)
        if xin.shape[-1] < cinp:
            xin = np.concatenate([xin, np.zeros(xin.shape[:3] + (cinp - xin.shape[-1],))], -1)
        if f[B.BFO_DW]:
            tab = P[f[B.BFO_DWW]:f[B.BFO_DWW] + 10 * cinp].reshape(10, cinp)
            pt, pl = f[B.BFO_PADT], f[B.BFO_PADL]
            xp = np.zeros((n, (Ho - 1) * s + 3, (Wo - 1) * s + 3, cinp))
            hh = min(H, xp.shape[1] - pt)
            ww = min(W, xp.shape[2] - pl)
            xp[:, pt:pt + hh, pl:pl + ww] = xin[:, :hh, :ww]
            a = np.broadcast_to(tab[9], (n, Ho, Wo, cinp)).copy()
            for t in range(9):
                dy, dx = divmod(t, 3)
                a += xp[:, dy:dy + (Ho - 1) * s + 1:s, dx:dx + (Wo - 1) * s + 1:s] * tab[t]
        else:
            a = xin
        wt = P[f[B.BFO_PWW]:f[B.BFO_PWW] + coutp * cinp].reshape(coutp, cinp)
        z = a @ wt.T + P[f[B.BFO_PWB]:f[B.BFO_PWB] + coutp]
        if f[B.BFO_RES] == B.RES_ID:
            z[..., :cinp] += xin
        elif f[B.BFO_RES] == B.RES_MAXPOOL:
            mp = np.maximum(np.maximum(xin[:, 0::2, 0::2], xin[:, 0::2, 1::2]),
                            np.maximum(xin[:, 1::2, 0::2], xin[:, 1::2, 1::2]))
            z[..., :cinp] += mp
        if f[B.BFO_RELU]:
            z = np.maximum(z, 0)
        sp = f[B.BFO_SPLIT]
        if sp:
            bufs[f[B.BFO_DST]] = z[..., :sp]
            bufs[f[B.BFO_DST2]] = z[..., sp:cout]
        else:
            bufs[f[B.BFO_DST]] = z[..., :f[B.BFO_OSTRIDE]]
    return bufs
