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
    # the line's big launch (grid 196608, 200 us) and a small launch of the same kernel name
    for grid, dur in [(196608, 200000)] * 5 + [(1024, 5000)] * 20:
        rows.append({'Kernel_Name': 'void chain_split_kernel<1>(Args)', 'Grid_Size_X': grid,
                     'Start_Timestamp': t, 'End_Timestamp': t + dur})
        t += dur + 10
    _write(tr, rows)
    _write(m.OUT + '/prof_t_infer/host/trace_kernel_stats.csv', [{'Name': 'x', 'Calls': 1}])
    fetch = [{'Kernel_Name': 'void chain_split_kernel<1>(Args)', 'Grid_Size': g, 'Dispatch_Id': i,
              'Counter_Name': 'FETCH_SIZE', 'Counter_Value': v}
             for i, (g, v) in enumerate([(196608, 456000.0)] * 5 + [(1024, 10.0)] * 20)]
    _write(m.OUT + '/pmc_t_infer_fetch/host/pmc_counter_collection.csv', fetch)
    write = [dict(r, Counter_Name='WRITE_SIZE', Counter_Value=27648.0 if r['Grid_Size'] == 196608 else 1.0) for r in fetch]
    _write(m.OUT + '/pmc_t_infer_write/host/pmc_counter_collection.csv', write)
    r = m.summarize_line('t', 'infer')
    assert r['grid'] == 196608 and r['dispatches'] == 5
    assert abs(r['avg_ns'] - 200000) < 1e-6
    assert r['fetch_bytes'] == 2 * 1024 * 456000.0          # gfx950: FETCH_SIZE counts half
    assert r['hbm_bytes_per_launch'] == 2 * 1024 * 456000.0 + 1024 * 27648.0
    assert os.path.exists(os.path.join(m.PROF, 't_infer_pmc.csv'))
    m.main('t', ['infer'])
    with open(os.path.join(m.PROF, 'traffic.json')) as fh:
        assert json.load(fh)['infer']['grid'] == 196608
