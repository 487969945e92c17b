"""Turn the per-line profiles of scripts/gpu_evidence.sh (kernel trace) and scripts/pmc_line.sh (PMC passes)
into committed evidence under profiles/.

Every bench line is profiled in its OWN process (``bench.py --only <line>``), so a line's dispatches
never mix with another line's launches of the same kernel name (the round-1 summariser averaged the
infer launch together with BlazeFace's small regressor launches).  Within one line, dispatches are
keyed by (kernel name, grid size) and the line's dominant key is the one with the largest total time.

Inputs (gpurun_out/, merged back by gpurun):
  prof_<tag>_<line>/**/*kernel_stats.csv        rocprofv3 --kernel-trace --stats
  prof_<tag>_<line>/**/*kernel_trace.csv        per-dispatch trace (durations keyed by grid)
  pmc_<tag>_<line>_<pass>/**/*counter_collection.csv   rocprofv3 --pmc, one pass per counter group
Timed region only: rocprofv3's own --stats summary averages every dispatch of a
process, including the bench's untimed warm-up launches (the first one cold), so its average can
exceed the bench's step time.  The per-line averages here keep only the LAST ``timed`` iterations'
dispatches of each (kernel, grid) group, where ``timed`` / ``warm`` are the bench line's own loop
counts for ``bench.py --only <line> --steps S --warmup W`` (``loop_counts``); a group launched k times
per iteration keeps its last k * timed dispatches.

Outputs:
  profiles/<tag>_<line>_kernel_stats.csv        copy of rocprofv3's stats summary (all dispatches)
  profiles/<tag>_<line>_kernel_stats_timed.csv  the same columns over the timed-region dispatches
  profiles/<tag>_<line>_pmc.csv                 per (kernel, grid): dispatches, mean of every counter
  profiles/traffic.json                         per line: dominant kernel, avg duration, HBM bytes per
                                                launch, SQ-derived utilisation; read by bench.py

gfx950 corrections (MI355X_MICROARCH.md §HBM / §PMC): FETCH_SIZE (KiB) reports half the bytes of a
wide coalesced 16-B/lane stream -> bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact for 16-B
stores -> 1024 * WRITE_SIZE.  SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_WAIT_* count quad-cycles;
SQ_VALU_MFMA_BUSY_CYCLES counts cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'gpurun_out')
PROF = os.path.join(ROOT, 'profiles')
N_SIMD = 256 * 4


def _one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    return hits[-1] if hits else None


def short(name):
    return name.split('(')[0].replace('void ', '')


def trace_groups(path):
    """(kernel, grid) -> list of dispatch durations in ns."""
    g = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            gx = r.get('Grid_Size_X') or r.get('Grid_Size') or '0'
            key = (short(r['Kernel_Name']), int(float(gx)))
            g[key].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    return g


def counter_groups(path):
    """(kernel, grid) -> {counter: [value per dispatch]}."""
    per = defaultdict(lambda: defaultdict(dict))
    with open(path) as fh:
        for r in csv.DictReader(fh):
            key = (short(r['Kernel_Name']), int(float(r.get('Grid_Size') or 0)))
            did = r.get('Dispatch_Id') or r.get('Correlation_Id')
            c = r['Counter_Name']
            per[key][c][did] = per[key][c].get(did, 0.0) + float(r['Counter_Value'])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def mean(v):
    return sum(v) / len(v) if v else 0.0


def loop_counts(line, steps, warmup):
    """(warm-up iterations, timed iterations) of ``bench.py --only <line> --steps steps --warmup
    warmup`` -- mirrors the loops in bench.py (train: run_train(steps, warmup); train88: 2 warm-ups,
    max(5, min(steps, 20)) timed; infer: 3 / max(10, steps); blazeface and attn: 3 / max(10, steps)
    forwards)."""
    if line == 'train':
        return warmup, steps
    if line == 'train88':
        return 2, max(5, min(steps, 20))
    if line in ('infer', 'blazeface', 'attn'):
        return 3, max(10, steps)
    return 0, None


def timed_only(groups, warm, timed):
    """Keep each group's dispatches of the last ``timed`` iterations (k per iteration when the
    group's count is a multiple of warm + timed; a group that does not repeat per iteration, e.g.
    one-off setup launches, is dropped)."""
    if timed is None:
        return dict(groups)
    out = {}
    it = warm + timed
    for key, v in groups.items():
        if len(v) >= it and len(v) % it == 0:
            k = len(v) // it
            out[key] = v[-k * timed:]
    return out


def write_stats(path, groups):
    """rocprofv3 --stats columns, one row per kernel name (grids merged), sorted by total time."""
    by = defaultdict(list)
    for (name, _grid), v in groups.items():
        by[name].extend(v)
    tot_all = sum(sum(v) for v in by.values()) or 1
    with open(path, 'w', newline='') as fh:
        wr = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        wr.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs'])
        for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            wr.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot_all, min(v), max(v)])


def summarize_line(tag, line, steps=10, warmup=2, pmc_steps=5, pmc_warmup=1):
    tdir = os.path.join(OUT, 'prof_%s_%s' % (tag, line))
    stats = _one(os.path.join(tdir, '**', '*kernel_stats.csv'))
    trace = _one(os.path.join(tdir, '**', '*kernel_trace.csv'))
    res = {}
    if stats:
        shutil.copy(stats, os.path.join(PROF, '%s_%s_kernel_stats.csv' % (tag, line)))
    all_groups = trace_groups(trace) if trace else {}
    warm, timed = loop_counts(line, steps, warmup)
    groups = timed_only(all_groups, warm, timed)
    if groups:
        write_stats(os.path.join(PROF, '%s_%s_kernel_stats_timed.csv' % (tag, line)), groups)
    ctr = defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(OUT, 'pmc_%s_%s_*' % (tag, line)))):
        f = _one(os.path.join(p, '**', '*counter_collection.csv'))
        if not f:
            continue
        pw, pt = loop_counts(line, pmc_steps, pmc_warmup)
        for key, cs in counter_groups(f).items():
            for c, vals in cs.items():
                vals = timed_only({key: vals}, pw, pt).get(key) or vals
                ctr[key][c] = (len(vals), mean(vals))
    if ctr:
        names = sorted({c for v in ctr.values() for c in v})
        with open(os.path.join(PROF, '%s_%s_pmc.csv' % (tag, line)), 'w') as fh:
            wr = csv.writer(fh)
            wr.writerow(['kernel', 'grid', 'dispatches'] + names)
            for key in sorted(ctr):
                n = max(v[0] for v in ctr[key].values())
                wr.writerow([key[0][:140], key[1], n] + ['%.6g' % ctr[key][c][1] if c in ctr[key] else ''
                                                         for c in names])
    if not groups:
        return res
    if line == 'blazeface':
        # one forward = every launch of the graph; forwards = dispatches of the stem (timed only)
        nfwd = max(1, min(len(v) for k, v in groups.items() if k[0].startswith(('bf_stem', 'bf_front'))))
        tot_ns = sum(sum(v) for v in groups.values()) / nfwd
        fb = wb = 0.0
        for key, cs in ctr.items():
            if key[0].startswith(('at::', '__amd_rocclr')):   # the bench's synthetic frames / copies
                continue
            if 'FETCH_SIZE' in cs:
                fb += 2 * 1024 * cs['FETCH_SIZE'][1] * cs['FETCH_SIZE'][0]
            if 'WRITE_SIZE' in cs:
                wb += 1024 * cs['WRITE_SIZE'][1] * cs['WRITE_SIZE'][0]
        res = {'kernel': 'all launches of one forward (bf_* + head GEMMs + regressor programs)',
               'avg_ns': tot_ns, 'forwards': nfwd, 'timed_region_only': True}
        if ctr:
            # the PMC passes run their own step counts: their forwards are their own front dispatches
            pf = [max(v[0] for v in cs.values()) for k, cs in ctr.items() if k[0].startswith(('bf_stem', 'bf_front'))]
            npf = max(1, min(pf)) if pf else nfwd
            res.update({'fetch_bytes': fb / npf, 'write_bytes': wb / npf, 'hbm_bytes_per_launch': (fb + wb) / npf,
                        'pmc_forwards': npf})
        return res
    key = max(groups, key=lambda k: sum(groups[k]))
    d = groups[key]
    res = {'kernel': key[0], 'grid': key[1], 'dispatches': len(d), 'avg_ns': mean(d),
           'min_ns': min(d), 'timed_region_only': timed is not None,
           'avg_ns_all_dispatches': mean(all_groups[key]),
           'share_of_line_time': sum(d) / sum(sum(v) for v in groups.values())}
    cs = ctr.get(key)
    if cs:
        if 'FETCH_SIZE' in cs:
            res['fetch_bytes'] = 2 * 1024 * cs['FETCH_SIZE'][1]
        if 'WRITE_SIZE' in cs:
            res['write_bytes'] = 1024 * cs['WRITE_SIZE'][1]
        if 'fetch_bytes' in res and 'write_bytes' in res:
            res['hbm_bytes_per_launch'] = res['fetch_bytes'] + res['write_bytes']
        v = {c: x[1] for c, x in cs.items()}
        if 'GRBM_GUI_ACTIVE' in v:
            cyc = v['GRBM_GUI_ACTIVE'] / 8.0          # kernel cycles (summed over the 8 XCDs)
            res['clock_ghz'] = cyc / res['avg_ns'] if res['avg_ns'] else None
            if 'SQ_VALU_MFMA_BUSY_CYCLES' in v:
                # fraction of all SIMD-cycles the MFMA pipe was busy
                res['mfma_busy_frac'] = v['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * N_SIMD)
        if 'SQ_WAVE_CYCLES' in v and v['SQ_WAVE_CYCLES']:
            wc = v['SQ_WAVE_CYCLES']
            for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU',
                      'SQ_ACTIVE_INST_LDS', 'SQ_WAIT_INST_LDS'):
                if c in v:
                    res[c.lower().replace('sq_', '') + '_frac_of_wave_cycles'] = v[c] / wc
        for c in ('SQ_INSTS_VALU_MFMA_MOPS_F16', 'SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT',
                  'SQ_INSTS_SALU', 'SQ_INSTS_VMEM'):
            if c in v:
                res[c] = v[c]
    return res


def profiled_step_ms(tag, line):
    """the bench line's own ms per step / batch as printed by the PROFILED process itself
    (gpurun_out/prof_<tag>_<line>.log): the like-for-like bound for the trace average (a separate
    un-profiled bench run clocks higher)"""
    p = os.path.join(OUT, 'prof_%s_%s.log' % (tag, line))
    if not os.path.exists(p):
        return None
    for ln in open(p):
        if ln.startswith('{'):
            try:
                d = json.loads(ln)
            except ValueError:
                continue
            v = d if line == 'train' else d.get(line, {})
            if isinstance(v, dict):
                return v.get('ms_per_step', v.get('ms_per_batch'))
    return None


def main(tag, lines, steps=10, warmup=2):
    os.makedirs(PROF, exist_ok=True)
    path = os.path.join(PROF, 'traffic.json')
    out = {}
    if os.path.exists(path):
        with open(path) as fh:
            out = json.load(fh)
        if out.get('tag') != tag:      # never mix an older round's numbers into this one
            out = {}
    for line in lines:
        r = summarize_line(tag, line, steps, warmup)
        if r:
            r['source'] = ('profiles/%s_%s_kernel_stats_timed.csv (timed-region dispatches of %s_%s_kernel_'
                           'stats.csv), %s_%s_pmc.csv' % (tag, line, tag, line, tag, line))
            ms = profiled_step_ms(tag, line)
            if ms is not None:
                r['profiled_process_ms_per_step'] = ms
            out[line] = r
    out['tag'] = tag
    out['note'] = ('per bench line, profiled in its own process (bench.py --only <line> --steps %d --warmup %d); '
                   'avg_ns over the timed-region dispatches only; FETCH_SIZE x 2 x 1024, WRITE_SIZE x 1024 '
                   '(gfx950, MI355X_MICROARCH.md); mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / '
                   '(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)' % (steps, warmup))
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    tag = sys.argv[1] if len(sys.argv) > 1 else 'r03'
    lines = sys.argv[2].split(',') if len(sys.argv) > 2 else ['train', 'infer', 'train88', 'blazeface', 'p1', 'attn']
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    warmup = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    main(tag, lines, steps, warmup)
