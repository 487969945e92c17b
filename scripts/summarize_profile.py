"""Turn a scripts/profile.sh run (gpurun_out/prof_*) into committed evidence under profiles/:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of bench.py
  profiles/<tag>_traffic.csv        per-kernel FETCH_SIZE / WRITE_SIZE (separate --pmc passes)
  profiles/traffic.json             HBM bytes per launch of the bench's train / infer kernels,
                                    read back by bench.py as roofline.traffic

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half the bytes of a wide
coalesced 16-B/lane stream -> bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE exact for 16-B stores ->
1024 * WRITE_SIZE.  Only dispatches of the bench's timed kernels are averaged.
"""
import csv
import re
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'gpurun_out')
PROF = os.path.join(ROOT, 'profiles')


def counters(path, name):
    agg = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r['Counter_Name'] == name:
                agg[r['Kernel_Name']].append(float(r['Counter_Value']))
    return agg


def main(tag):
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, 'prof_trace', 'trace_kernel_stats.csv'),
                os.path.join(PROF, '%s_kernel_stats.csv' % tag))
    fetch = counters(os.path.join(OUT, 'prof_fetch', 'fetch_counter_collection.csv'), 'FETCH_SIZE')
    write = counters(os.path.join(OUT, 'prof_write', 'write_counter_collection.csv'), 'WRITE_SIZE')
    rows = []
    res = {}
    per = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else 0.0
        wb = 1024 * sum(w) / len(w) if w else 0.0
        rows.append((k[:120], len(f), fb, wb, fb + wb))
        per[k.split('(')[0]] = (fb, wb, len(f))

    def put(key, short):
        fb, wb, _ = per[short]
        res[key] = {'kernel': short, 'fetch_bytes': fb, 'write_bytes': wb, 'hbm_bytes_per_launch': fb + wb}

    # bench lines -> their dominant kernels (template args: <KH, ACT1, DROP, NWM, SPLIT>; ACT 1 = tanh,
    # 3 = softsign).  The exact-fp32 instantiations (SPLIT false) are the guarded fallbacks that exit
    # at once unless the split launch flagged an overflow; the split ones carry the traffic.
    split = os.environ.get('HPE_EXACT_FP32') != '1'
    for short in per:
        if short.startswith('void mlp2_kernel<48') and ', 1, false, 12, %s>' % str(split).lower() in short:
            put('train', short)
        elif short.startswith('void mlp2_kernel<44') and ', true, 4, %s>' % str(split).lower() in short:
            put('train88', short)
        elif ('chain_split' if split else 'chain_fwd') in short:
            put('infer', short)
    # BlazeFace forward = every bf_* launch of one forward (one dispatch each per forward per kernel
    # name, except the 64x64/32x32 block kernels that run several blocks): bytes per forward
    bf = [(s, v) for s, v in per.items() if re.match(r'(void )?bf_', s)]
    if bf:
        nfwd = min(v[2] for s, v in bf if 'stem' in s) if any('stem' in s for s, _ in bf) else 1
        tot_f = sum(v[0] * v[2] for _, v in bf) / nfwd
        tot_w = sum(v[1] * v[2] for _, v in bf) / nfwd
        res['blazeface'] = {'kernel': 'bf_* (one forward)', 'fetch_bytes': tot_f, 'write_bytes': tot_w,
                            'hbm_bytes_per_launch': tot_f + tot_w}
    with open(os.path.join(PROF, '%s_traffic.csv' % tag), 'w') as fh:
        wr = csv.writer(fh)
        wr.writerow(['kernel', 'dispatches', 'fetch_bytes_per_launch(x2 gfx950)', 'write_bytes_per_launch', 'hbm_bytes_per_launch'])
        for r in rows:
            wr.writerow(r)
    res['source'] = '%s_traffic.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)' % tag
    with open(os.path.join(PROF, 'traffic.json'), 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'r01')
