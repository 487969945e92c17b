"""CPU: scripts/summarize_profile.py keys dispatches per bench line and per (kernel, grid), so one
line's launches never mix with another's, and applies the gfx950 FETCH_SIZE x 2 correction (the
round-1 summariser averaged BlazeFace's small regressor launches into the infer line)."""
import csv
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location('summarize_profile', os.path.join(ROOT, 'scripts', 'summarize_profile.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _write(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, 'w', newline='') as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_dominant_kernel_keyed_by_grid(tmp_path):
    m = _mod()
    m.OUT, m.PROF = str(tmp_path / 'out'), str(tmp_path / 'prof')
    os.makedirs(m.PROF)
    tr = m.OUT + '/prof_t_infer/host/trace_kernel_trace.csv'
    rows = []
    t = 0
    # the line's big launch (grid 196608, 200 us; 3 warm-ups, the first cold at 900 us, then 10
    # timed) and a small launch of the same kernel name twice per iteration
    for grid, dur in [(196608, 900000)] + [(196608, 200000)] * 12 + [(1024, 5000)] * 26:
        rows.append({'Kernel_Name': 'void chain_split_kernel<1>(Args)', 'Grid_Size_X': grid,
                     'Start_Timestamp': t, 'End_Timestamp': t + dur})
        t += dur + 10
    _write(tr, rows)
    _write(m.OUT + '/prof_t_infer/host/trace_kernel_stats.csv', [{'Name': 'x', 'Calls': 1}])
    fetch = [{'Kernel_Name': 'void chain_split_kernel<1>(Args)', 'Grid_Size': g, 'Dispatch_Id': i,
              'Counter_Name': 'FETCH_SIZE', 'Counter_Value': v}
             for i, (g, v) in enumerate([(196608, 999000.0)] + [(196608, 456000.0)] * 12 + [(1024, 10.0)] * 26)]
    _write(m.OUT + '/pmc_t_infer_fetch/host/pmc_counter_collection.csv', fetch)
    write = [dict(r, Counter_Name='WRITE_SIZE', Counter_Value=27648.0 if r['Grid_Size'] == 196608 else 1.0) for r in fetch]
    _write(m.OUT + '/pmc_t_infer_write/host/pmc_counter_collection.csv', write)
    r = m.summarize_line('t', 'infer', steps=10, warmup=2, pmc_steps=10, pmc_warmup=2)
    # timed region only: the cold warm-up dispatch is not in the average
    assert r['grid'] == 196608 and r['dispatches'] == 10 and r['timed_region_only']
    assert abs(r['avg_ns'] - 200000) < 1e-6
    assert r['avg_ns_all_dispatches'] > r['avg_ns']
    with open(os.path.join(m.PROF, 't_infer_kernel_stats_timed.csv')) as fh:
        rows = list(csv.DictReader(fh))
    assert rows[0]['Calls'] == '30' and abs(float(rows[0]['AverageNs']) - (10 * 200000 + 20 * 5000) / 30) < 1e-6
    assert r['fetch_bytes'] == 2 * 1024 * 456000.0          # gfx950: FETCH_SIZE counts half
    assert r['hbm_bytes_per_launch'] == 2 * 1024 * 456000.0 + 1024 * 27648.0
    assert os.path.exists(os.path.join(m.PROF, 't_infer_pmc.csv'))
    m.main('t', ['infer'], 10, 2)
    with open(os.path.join(m.PROF, 'traffic.json')) as fh:
        assert json.load(fh)['infer']['grid'] == 196608
