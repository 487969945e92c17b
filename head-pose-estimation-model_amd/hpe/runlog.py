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
        self.id = ''.join(random.Random(time.time_ns()).choice(string.ascii_lowercase + string.digits)
                          for _ in range(8))
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
