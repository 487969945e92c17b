"""Quick look at the PMC passes of one bench line (gpurun_out/pmc_<tag>_<line>_*): per kernel (name,
grid) the mean of every counter over its dispatches, plus the derived fractions the DESIGN tables
use.  Read-only: writes nothing under profiles/ (scripts/summarize_profile.py does that)."""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import summarize_profile as S  # noqa: E402

tag, line = sys.argv[1], sys.argv[2]
ctr = {}
for p in sorted(glob.glob(os.path.join(S.OUT, 'pmc_%s_%s_*' % (tag, line)))):
    f = S._one(os.path.join(p, '**', '*counter_collection.csv'))
    if not f:
        continue
    for key, cs in S.counter_groups(f).items():
        for c, vals in cs.items():
            ctr.setdefault(key, {})[c] = S.mean(vals[1:] if len(vals) > 1 else vals)
for key, v in sorted(ctr.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0))[:3]:
    print(key[0][:80], key[1])
    cyc = v.get('GRBM_GUI_ACTIVE', 0) / 8.0
    wc = v.get('SQ_WAVE_CYCLES', 0) or 1
    out = {k: round(x) for k, x in v.items()}
    print('  ', out)
    if cyc:
        print('   mfma_busy %.3f' % (v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * S.N_SIMD)))
    for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS',
              'SQ_WAIT_INST_LDS'):
        if c in v:
            print('   %s / wave cycles %.3f' % (c, v[c] / wc))
    if 'SQ_INSTS_LDS' in v and 'SQ_LDS_BANK_CONFLICT' in v:
        print('   bank conflict cycles per LDS instr %.2f' % (v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_INSTS_LDS'])))
