"""Concurrent hyper-parameter sweeps, one trial per GPU.

Replaces the wandb sweep agent the reference drives with Model-96/sweep.yaml (method bayes, count
50, metric test_AFLW2000_mae minimised over dropout_rate / regularizer_rate / num_filters, program
train_96.py).  As the agent does, every trial runs the program as its own process with the sampled
values as ``--name=value`` flags; here the controller keeps one trial running on each GPU of the
node (``HIP_VISIBLE_DEVICES`` pins it; the trial's fit loop is the hot path on that GPU) and reads
the trial's metric back from its run record (hpe.runlog, ``HPE_RUN_ID`` / ``HPE_RUN_DIR``: the
``wandb.run.summary`` entries of train_96.py:191-196).  The controller itself never touches a GPU.

Search methods (wandb's names): ``grid`` (every combination, in order), ``random`` (uniform over
the value lists, seeded), ``bayes`` — Gaussian-process expected improvement over the grid of
``values`` (Matern 5/2 on each parameter's rank in its list, as wandb's bayes treats categorical
values; the first ``n_initial`` trials random).  Proposals never repeat a finished or running
combination while untried ones remain.
"""
import argparse
import itertools
import json
import math
import os
import subprocess
import sys
import time
import uuid

import numpy as np

from . import runlog


def load_spec(path):
    import yaml
    with open(path) as fh:
        spec = yaml.safe_load(fh)
    spec['_dir'] = os.path.dirname(os.path.abspath(path))
    return spec


def _num(v):
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


class Search:
    def __init__(self, spec, seed=0, n_initial=3):
        self.spec = spec
        self.method = spec.get('method', 'grid')
        if self.method not in ('grid', 'random', 'bayes'):
            raise ValueError('sweep method %r not supported (grid, random, bayes)' % self.method)
        params = spec.get('parameters') or {}
        self.names = sorted(params)
        self.values = []
        for n in self.names:
            p = params[n]
            if 'values' in p:
                self.values.append(list(p['values']))
            elif 'value' in p:
                self.values.append([p['value']])
            else:
                raise ValueError('parameter %s: only "values" / "value" lists are supported' % n)
        m = spec.get('metric') or {}
        self.metric = m.get('name')
        self.sign = -1.0 if m.get('goal', 'minimize') == 'maximize' else 1.0
        self.rng = np.random.default_rng(seed)
        self.n_initial = n_initial
        self.grid = list(itertools.product(*[range(len(v)) for v in self.values]))

    def params(self, combo):
        return {n: self.values[i][c] for i, (n, c) in enumerate(zip(self.names, combo))}

    def _x(self, combo):
        return np.array([c / max(len(self.values[i]) - 1, 1) for i, c in enumerate(combo)])

    def propose(self, done, busy=()):
        """done: [(combo, metric or None)], busy: [combo] -> next combo (tuple of indices)."""
        taken = {tuple(c) for c, _ in done} | {tuple(c) for c in busy}
        free = [g for g in self.grid if g not in taken]
        if not free:
            free = list(self.grid)
        if self.method == 'grid':
            return free[0]
        scored = [(c, y) for c, y in done if y is not None and math.isfinite(y)]
        if self.method == 'random' or len(scored) < self.n_initial:
            return free[int(self.rng.integers(len(free)))]
        from sklearn.gaussian_process import GaussianProcessRegressor
        from sklearn.gaussian_process.kernels import ConstantKernel, Matern, WhiteKernel
        X = np.stack([self._x(c) for c, _ in scored])
        y = self.sign * np.array([v for _, v in scored], np.float64)
        gp = GaussianProcessRegressor(kernel=ConstantKernel() * Matern(nu=2.5) + WhiteKernel(1e-6),
                                      normalize_y=True, random_state=int(self.rng.integers(1 << 31)))
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')   # kernel-bound convergence notes on tiny histories
            gp.fit(X, y)
        Xf = np.stack([self._x(c) for c in free])
        mu, sd = gp.predict(Xf, return_std=True)
        best = y.min()
        sd = np.maximum(sd, 1e-12)
        z = (best - mu) / sd
        from scipy.stats import norm
        ei = (best - mu) * norm.cdf(z) + sd * norm.pdf(z)
        return free[int(np.argmax(ei))]


def _flags(params):
    return ['--%s=%s' % (k, v) for k, v in params.items()]


def run_sweep(spec, gpus, count=None, program=None, run_dir='sweep_runs', seed=0, python=None,
              extra_env=None, poll=0.2, log=print):
    """Run ``count`` trials of ``program`` with at most one per entry of ``gpus`` at a time.
    Returns the trials [{'params', 'run_id', 'gpu', 'returncode', 'metric', 'seconds'}] in start
    order; the best one is ``best_trial(...)``."""
    if isinstance(spec, str):
        spec = load_spec(spec)
    search = Search(spec, seed=seed)
    count = int(count if count is not None else spec.get('count', len(search.grid)))
    prog = program or spec.get('program')
    if prog is None:
        raise ValueError('sweep has no program')
    if not os.path.isabs(prog):
        prog = os.path.join(spec.get('_dir', os.getcwd()), prog)
    if not os.path.exists(prog):
        raise FileNotFoundError(prog)
    os.makedirs(run_dir, exist_ok=True)
    gpus = list(gpus)
    if not gpus:
        raise ValueError('no GPUs to run trials on')
    trials, running = [], {}   # gpu -> (trial, Popen)
    while len(trials) < count or running:
        for g in gpus:
            if g in running or len(trials) >= count:
                continue
            done = [(t['combo'], t['metric']) for t in trials if t['returncode'] is not None]
            busy = [t['combo'] for t, _ in running.values()]
            combo = search.propose(done, busy)
            rid = uuid.uuid4().hex[:8]
            env = dict(os.environ)
            env.update(extra_env or {})
            env.update(HIP_VISIBLE_DEVICES=child_device(g), HPE_RUN_ID=rid, HPE_RUN_DIR=os.path.abspath(run_dir))
            t = dict(combo=combo, params=search.params(combo), run_id=rid, gpu=g, returncode=None,
                     metric=None, start=time.time())
            out = open(os.path.join(run_dir, rid + '.out'), 'w')
            p = subprocess.Popen([python or sys.executable, prog] + _flags(t['params']), env=env,
                                 cwd=os.path.dirname(prog), stdout=out, stderr=subprocess.STDOUT)
            p._hpe_out = out
            running[g] = (t, p)
            trials.append(t)
            log('[sweep] trial %d/%d %s on GPU %s: %s' % (len(trials), count, rid, g, t['params']))
        time.sleep(poll)
        for g in list(running):
            t, p = running[g]
            rc = p.poll()
            if rc is None:
                continue
            p._hpe_out.close()
            t['returncode'] = rc
            t['seconds'] = time.time() - t.pop('start')
            summ = runlog.read_summary(os.path.join(run_dir, t['run_id'] + '.jsonl'))
            v = summ.get(search.metric)
            t['metric'] = float(v) if rc == 0 and _num(v) is not None else None
            del running[g]
            log('[sweep] trial %s done rc=%d %s=%s (%.1fs)' % (t['run_id'], rc, search.metric, t['metric'],
                                                             t['seconds']))
    for t in trials:
        t['combo'] = list(t['combo'])
    with open(os.path.join(run_dir, 'sweep.json'), 'w') as fh:
        json.dump({'spec': {k: v for k, v in spec.items() if k != '_dir'}, 'trials': trials}, fh, indent=1,
                  default=str)
    return trials


def best_trial(trials, goal='minimize'):
    ok = [t for t in trials if t['metric'] is not None]
    if not ok:
        return None
    return (min if goal == 'minimize' else max)(ok, key=lambda t: t['metric'])


def visible_gpus():
    """Logical GPU positions 0..n-1 within this process's visible set (device count only: no HIP
    context is created here).  ``child_device`` turns a position into the child's pin."""
    env = os.environ.get('HIP_VISIBLE_DEVICES') or os.environ.get('ROCR_VISIBLE_DEVICES')
    if env:
        return list(range(len([x for x in env.split(',') if x.strip()])))
    import torch
    return list(range(torch.cuda.device_count()))


def child_device(pos, environ=None):
    """HIP_VISIBLE_DEVICES value that pins a child to logical position ``pos`` of the parent's
    visible set.  HIP counts HIP_VISIBLE_DEVICES inside the ROCR_VISIBLE_DEVICES filter, which the
    child inherits: with a parent HIP list the child gets that list's entry (index or UUID, kept as
    text); with only a ROCR filter (e.g. ROCR_VISIBLE_DEVICES=4,5) the child gets the position
    (0 or 1), never the raw ROCR id."""
    environ = os.environ if environ is None else environ
    hip = [x.strip() for x in (environ.get('HIP_VISIBLE_DEVICES') or '').split(',') if x.strip()]
    if hip:
        if not 0 <= pos < len(hip):
            raise ValueError('GPU position %d outside HIP_VISIBLE_DEVICES=%s' % (pos, ','.join(hip)))
        return hip[pos]
    return str(pos)


def main(argv=None):
    ap = argparse.ArgumentParser(description='run a sweep.yaml with one trial per GPU')
    ap.add_argument('sweep')
    ap.add_argument('--gpus', default=None, help='comma-separated GPU positions within the visible set (default: all visible)')
    ap.add_argument('--count', type=int, default=None)
    ap.add_argument('--run-dir', default='sweep_runs')
    ap.add_argument('--seed', type=int, default=0)
    a = ap.parse_args(argv)
    spec = load_spec(a.sweep)
    gpus = [int(x) for x in a.gpus.split(',')] if a.gpus else visible_gpus()
    trials = run_sweep(spec, gpus, count=a.count, run_dir=a.run_dir, seed=a.seed)
    b = best_trial(trials, (spec.get('metric') or {}).get('goal', 'minimize'))
    print(json.dumps({'best': b, 'n_trials': len(trials)}, default=str))
    return 0 if b is not None else 1


if __name__ == '__main__':
    sys.exit(main())
