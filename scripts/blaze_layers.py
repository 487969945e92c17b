"""Per-layer HBM roofline of the BlazeFace forward (configs[4]) from a rocprofv3 kernel trace of
scripts/time_blaze.py: dispatches of the bf_* kernels are matched in order to the plan's ops, each
op's algorithmic bytes (its input map + its output map as stored, fp32; hpe.blazeface) divided by
its mean duration.  Writes profiles/<tag>_blaze_layers.csv.

Usage: python scripts/blaze_layers.py gpurun_out/prof_blaze/run_kernel_trace.csv r05 [batch]
(HPE_BF_STAGE=0 HPE_BF_FRONT=0 for a trace of the per-op plan: profiles/<tag>_blaze_layers_perop.csv)
"""
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from hpe import blazeface as B  # noqa: E402
from util import fixture  # noqa: E402

PEAK = 8.0e12


def launches(plan):
    """The bf_* launches of one forward in order: (label, out map, algorithmic bytes per frame).
    A stage record (bf_stage_kernel) is ONE launch over its NI records: its bytes are the stage's
    input map, the taps and the head outputs (the maps in between stay in LDS)."""
    wd = np.asarray(plan['words'])
    nops, off = int(wd[B.BFH_NOPS]), int(wd[B.BFH_OPS_OFF])
    recs = [[int(v) for v in wd[off + i * B.BFO_WORDS: off + (i + 1) * B.BFO_WORDS]] for i in range(nops)]
    out = []
    i = 0
    while i < nops:
        f = recs[i]
        if f[B.BFO_KIND] == B.BF_FRONT:
            sub = recs[i + 1:i + 1 + f[B.BFO_NI]]
            last = sub[-1]
            nb = 4 * sub[0][B.BFO_H] * sub[0][B.BFO_W] * 3 + 4 * last[B.BFO_HO] * last[B.BFO_WO] * last[B.BFO_OSTRIDE]
            out.append(('front: stem + %d blocks (128x128 -> %dx%d)' % (len(sub) - 1, last[B.BFO_HO], last[B.BFO_WO]),
                        '%dx%d' % (last[B.BFO_HO], last[B.BFO_WO]), nb))
            i += 1 + f[B.BFO_NI]
            continue
        if f[B.BFO_KIND] == B.BF_STAGE:
            ni = f[B.BFO_NI]
            sub = recs[i + 1:i + 1 + ni]
            nb = 4 * sub[0][B.BFO_H] * sub[0][B.BFO_W] * sub[0][B.BFO_CINP]
            for g in sub:
                if g[B.BFO_DST] >= B.BUF_OUT0:
                    out_c = g[B.BFO_COUT] if g[B.BFO_SPLIT] else g[B.BFO_OSTRIDE]
                    nb += 4 * g[B.BFO_HO] * g[B.BFO_WO] * out_c
            out.append(('stage: %d blocks + heads (%dx%d -> %dx%d)' % (
                ni, sub[0][B.BFO_H], sub[0][B.BFO_W], sub[-1][B.BFO_HO], sub[-1][B.BFO_WO]),
                '%dx%d' % (sub[-1][B.BFO_HO], sub[-1][B.BFO_WO]), nb))
            i += 1 + ni
            continue
        hw_in, hw_out = f[B.BFO_H] * f[B.BFO_W], f[B.BFO_HO] * f[B.BFO_WO]
        if f[B.BFO_KIND] == B.BF_STEM:
            nb = 4 * (hw_in * 3 + hw_out * f[B.BFO_COUTP])
            what = 'stem 5x5 s2 3->%d' % f[B.BFO_COUT]
        else:
            out_c = f[B.BFO_COUT] if f[B.BFO_SPLIT] else f[B.BFO_OSTRIDE]
            nb = 4 * (hw_in * f[B.BFO_CINP] + hw_out * out_c)
            what = ('dw3x3 s%d + pw %d->%d' % (f[B.BFO_STRIDE], f[B.BFO_CIN], f[B.BFO_COUT])
                    if f[B.BFO_DW] else 'heads pw %d->%d' % (f[B.BFO_CIN], f[B.BFO_COUT]))
        out.append((what, '%dx%d' % (f[B.BFO_HO], f[B.BFO_WO]), nb))
        i += 1
    return out


def main(trace, tag, batch=1024, stage=True, front=True):
    mc, w = fixture('reg1-stoqa9pt-reg2-hrchr82r-selected')
    plan = B.build_plan(mc, w, stage=stage, front=front)
    ops = [(what, hw, nb * batch) for what, hw, nb in launches(plan)]
    nops = len(ops)
    rows = [r for r in csv.DictReader(open(trace)) if r['Kernel_Name'].startswith(('bf_', 'void bf_'))]
    durs = [[] for _ in ops]
    for i, r in enumerate(rows):
        durs[i % nops].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9)
    out = os.path.join(ROOT, 'profiles', '%s_blaze_layers%s.csv' % (tag, '' if stage and front else '_perop'))
    tot_t = tot_b = 0.0
    with open(out, 'w') as fh:
        wr = csv.writer(fh)
        wr.writerow(['launch', 'layer', 'out_map', 'bytes_per_launch', 'mean_us', 'achieved_GBps', 'frac_hbm_peak'])
        for i, ((what, hw, nb), d) in enumerate(zip(ops, durs)):
            t = float(np.mean(d[2:] if len(d) > 4 else d))
            tot_t += t
            tot_b += nb
            wr.writerow([i, what, hw, nb, '%.1f' % (t * 1e6), '%.0f' % (nb / t / 1e9), '%.3f' % (nb / t / PEAK)])
            print('%2d %-44s %6s %7.1f us %6.0f GB/s %5.1f%%' % (i, what, hw, t * 1e6, nb / t / 1e9,
                                                                100 * nb / t / PEAK))
        wr.writerow(['all', 'backbone + detector heads (bf_* launches)', '', int(tot_b), '%.1f' % (tot_t * 1e6),
                     '%.0f' % (tot_b / tot_t / 1e9), '%.3f' % (tot_b / tot_t / PEAK)])
    print('total %.1f us, %.0f GB/s (%.1f%% of 8 TB/s) -> %s' % (tot_t * 1e6, tot_b / tot_t / 1e9,
                                                               100 * tot_b / tot_t / PEAK, out))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else 'r05',
         int(sys.argv[3]) if len(sys.argv) > 3 else 1024, os.environ.get('HPE_BF_STAGE', '1') != '0',
         os.environ.get('HPE_BF_FRONT', '1') != '0')
