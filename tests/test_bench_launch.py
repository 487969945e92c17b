"""bench.py --gpus N: the N-rank launch is decided before anything touches a GPU, runs as a child
torchrun job (never an exec), and fails cleanly when fewer GPUs are visible (this CPU container)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_launch_plan_is_pure_and_device_free():
    import bench
    cmd = bench.launch_plan(4, ['--gpus', '4', '--steps', '5'], {})
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node' in cmd and cmd[cmd.index('--nproc-per-node') + 1] == '4'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-3:] == ['--gpus', '4', '--steps', '5'][-3:]
    assert os.path.samefile(cmd[cmd.index('--master-port') + 2], os.path.join(ROOT, 'bench.py'))
    # already a torchrun rank, or a single GPU: this process is the job
    assert bench.launch_plan(4, [], {'WORLD_SIZE': '4'}) is None
    assert bench.launch_plan(1, [], {}) is None
    assert not torch.cuda.is_initialized()


def test_gpus_2_without_gpus_fails_cleanly():
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--no-cpu'],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, (r.returncode, r.stdout[-500:], r.stderr[-2000:])
    assert 'GPU(s) visible' in r.stderr
    assert r.stdout.strip() == ''
