"""Concurrent sweeps: hpe.sweep runs sweep.yaml trials as separate processes, one
per GPU slot, and reads each trial's metric from its run record.  CPU: a stand-in program (no GPU)
exercises scheduling, flag passing, GPU pinning and the grid / random / bayes proposals.  GPU: two
real train_96.py trials on synthetic feature maps."""
import os
import sys
import textwrap

import numpy as np
import pytest

from hpe import sweep

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'head-pose-estimation-model_amd')
SPEC = os.path.join(PKG, 'Model-96', 'sweep.yaml')

FAKE = textwrap.dedent('''
    import argparse, os, sys
    sys.path.insert(0, %r)
    from hpe import runlog
    ap = argparse.ArgumentParser()
    ap.add_argument('--dropout_rate', type=float)
    ap.add_argument('--regularizer_rate', type=float)
    ap.add_argument('--num_filters', type=int)
    a = ap.parse_args()
    run = runlog.init(project='fake', config=vars(a))
    run.summary['test_AFLW2000_mae'] = ((a.num_filters - 128) / 100.0) ** 2 + 10 * a.dropout_rate + a.regularizer_rate
    run.summary['gpu'] = os.environ['HIP_VISIBLE_DEVICES']
    run.finish()
''') % PKG


def _fake(tmp_path):
    p = tmp_path / 'fake_train.py'
    p.write_text(FAKE)
    return str(p)


def _f(p):
    return ((p['num_filters'] - 128) / 100.0) ** 2 + 10 * float(p['dropout_rate']) + float(p['regularizer_rate'])


def test_reference_sweep_spec_parses():
    spec = sweep.load_spec(SPEC)
    s = sweep.Search(spec)
    assert s.method == 'bayes' and spec['count'] == 50 and s.metric == 'test_AFLW2000_mae'
    assert s.names == ['dropout_rate', 'num_filters', 'regularizer_rate']
    assert len(s.grid) == 8 * 5 * 8
    assert os.path.exists(os.path.join(spec['_dir'], spec['program']))


def test_grid_sweep_two_slots(tmp_path):
    spec = dict(sweep.load_spec(SPEC), method='grid')
    trials = sweep.run_sweep(spec, gpus=[0, 1], count=6, program=_fake(tmp_path),
                             run_dir=str(tmp_path / 'runs'), log=lambda *a: None, poll=0.05)
    assert len(trials) == 6
    assert len({tuple(t['combo']) for t in trials}) == 6
    for t in trials:
        assert t['returncode'] == 0
        assert t['metric'] == pytest.approx(_f(t['params']))
    summ = [sweep.runlog.read_summary(str(tmp_path / 'runs' / (t['run_id'] + '.jsonl'))) for t in trials]
    assert {s['gpu'] for s in summ} == {'0', '1'}
    assert all(s['gpu'] == str(t['gpu']) for s, t in zip(summ, trials))
    assert os.path.exists(tmp_path / 'runs' / 'sweep.json')


def test_bayes_sweep_finds_a_good_region(tmp_path):
    spec = sweep.load_spec(SPEC)
    # one slot: every proposal sees all earlier results, so the outcome does not depend on which of
    # several concurrent trials happens to finish first on a loaded host
    trials = sweep.run_sweep(spec, gpus=[0], count=15, program=_fake(tmp_path),
                             run_dir=str(tmp_path / 'runs'), seed=1, log=lambda *a: None, poll=0.02)
    assert len({tuple(t['combo']) for t in trials}) == 15       # never repeats while untried remain
    b = sweep.best_trial(trials)
    # 320 combinations, optimum 0.0 at (num_filters 128, dropout 0, l2 0); random 15 rarely gets < 0.02
    assert b['metric'] < 0.3
    s = sweep.Search(spec, seed=1)
    done = [(tuple(t['combo']), t['metric']) for t in trials]
    c1, c2 = s.propose(done), sweep.Search(spec, seed=1).propose(done)
    assert c1 == c2 and c1 not in {d[0] for d in done}


def test_failed_trial_is_recorded(tmp_path):
    bad = tmp_path / 'bad.py'
    bad.write_text('import sys; sys.exit(3)\n')
    trials = sweep.run_sweep(dict(sweep.load_spec(SPEC), method='random'), gpus=[0], count=2,
                             program=str(bad), run_dir=str(tmp_path / 'r'), log=lambda *a: None, poll=0.05)
    assert [t['returncode'] for t in trials] == [3, 3] and sweep.best_trial(trials) is None


@pytest.mark.gpu
def test_gpu_sweep_runs_train96_trials(tmp_path):
    d = tmp_path / 'maps'
    d.mkdir()
    rng = np.random.default_rng(0)
    for name, n in (('BIWI_train_features_96.npz', 300), ('BIWI_test_features_96.npz', 80),
                    ('AFLW2000_features_96_0.7_1.npz', 80)):
        np.savez(d / name, features=np.maximum(0, rng.standard_normal((n, 96)) * .6 - .3).astype(np.float32),
                 poses=rng.standard_normal((n, 3)) * 20)
    prog = tmp_path / 'trial96.py'
    prog.write_text(textwrap.dedent('''
        import sys
        sys.path.insert(0, %r)
        import train_96
        train_96.config['total_epochs'] = 3
        train_96.main(sys.argv[1:])
    ''') % os.path.join(PKG, 'Model-96'))
    env = {'FEATUREMAPS_DIR_PATH': str(d) + '/', 'TRAINED_MODELS_96_RESHAPEDINPUT_NOFLATTEN_PATH': str(tmp_path / 'ck')}
    trials = sweep.run_sweep(sweep.load_spec(SPEC), gpus=[0], count=2, program=str(prog),
                             run_dir=str(tmp_path / 'runs'), extra_env=env, log=lambda *a: None)
    out = [open(tmp_path / 'runs' / (t['run_id'] + '.out')).read()[-2000:] for t in trials]
    assert all(t['returncode'] == 0 for t in trials), out
    assert all(t['metric'] is not None and np.isfinite(t['metric']) for t in trials)
    assert len(list((tmp_path / 'ck').glob('*.h5'))) == 2


def test_child_device_pins_within_the_visible_set():
    """under ROCR_VISIBLE_DEVICES=4,5 a child must be pinned to position 0 / 1 (HIP counts
    HIP_VISIBLE_DEVICES inside the inherited ROCR filter), and a parent HIP list (ids or UUIDs) is
    passed through entry by entry."""
    assert sweep.child_device(1, {'ROCR_VISIBLE_DEVICES': '4,5'}) == '1'
    assert sweep.child_device(0, {'HIP_VISIBLE_DEVICES': '6,7'}) == '6'
    assert sweep.child_device(1, {'HIP_VISIBLE_DEVICES': 'GPU-aa,GPU-bb', 'ROCR_VISIBLE_DEVICES': '2,3'}) == 'GPU-bb'
    assert sweep.child_device(3, {}) == '3'
    with pytest.raises(ValueError):
        sweep.child_device(2, {'HIP_VISIBLE_DEVICES': '6,7'})
    old = {k: os.environ.pop(k, None) for k in ('HIP_VISIBLE_DEVICES', 'ROCR_VISIBLE_DEVICES')}
    try:
        os.environ['ROCR_VISIBLE_DEVICES'] = 'GPU-x,GPU-y,GPU-z'
        assert sweep.visible_gpus() == [0, 1, 2]
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
