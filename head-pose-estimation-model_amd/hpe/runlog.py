"""Offline stand-in for the wandb calls of the reference's drivers (wandb.init / log /
run.summary / run.id: Model-96/train_96.py:115-120,191-209, utilities.py:23-29).  wandb is not
part of this image; records go to JSON lines under $HPE_RUN_DIR (default ./runs)."""
import json
import os
import random
import string
import time


class _Run:
    def __init__(self, project, config, notes, tags):
        # a sweep controller (hpe.sweep) names the run so it can read the summary back
        self.id = os.environ.get('HPE_RUN_ID') or ''.join(
            random.Random(time.time_ns()).choice(string.ascii_lowercase + string.digits) for _ in range(8))
        self.project, self.config, self.notes, self.tags = project, dict(config or {}), notes, tags
        self.summary = {}
        d = os.environ.get('HPE_RUN_DIR', 'runs')
        os.makedirs(d, exist_ok=True)
        self.path = os.path.join(d, '%s.jsonl' % self.id)
        self._write({'event': 'init', 'project': project, 'config': self.config, 'notes': notes,
                     'tags': tags})

    def _write(self, rec):
        with open(self.path, 'a') as fh:
            fh.write(json.dumps(rec, default=float) + '\n')

    def log(self, d):
        self._write({'event': 'log', **d})

    def finish(self):
        self._write({'event': 'summary', **self.summary})


run = None


def init(project=None, config=None, notes='', tags=None, **kw):
    global run
    run = _Run(project, config, notes, tags)
    return run


def log(d):
    if run is not None:
        run.log(d)


def read_summary(path):
    """The last summary record of a run's JSON-lines file ({} if the run never finished)."""
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as fh:
        for line in fh:
            try:
                rec = json.loads(line)
            except ValueError:
                continue
            if rec.get('event') == 'summary':
                out = {k: v for k, v in rec.items() if k != 'event'}
    return out
