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


def _kfd(tmp_path, kinds):
    for i, simd in enumerate(kinds):
        d = tmp_path / str(i)
        d.mkdir()
        (d / 'properties').write_text('cpu_cores_count 0\nsimd_count %d\nlds_size_in_kb 160\n' % simd)
    return str(tmp_path)


def test_visible_gpus_counts_without_hip(tmp_path, monkeypatch):
    """the launcher counts GPUs from KFD sysfs / the visible-devices env; torch's device
    count (which can initialise HIP in the parent) is never called."""
    import bench

    def boom(*a, **k):
        raise AssertionError('launcher touched the HIP runtime')
    monkeypatch.setattr(torch.cuda, 'device_count', boom)
    monkeypatch.setattr(torch.cuda, 'is_available', boom)
    kfd = _kfd(tmp_path, [0, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024])  # 1 CPU + 8 GPU nodes
    assert bench.visible_gpus({}, kfd) == 8
    assert bench.visible_gpus({'HIP_VISIBLE_DEVICES': '0,1'}, kfd) == 2
    assert bench.visible_gpus({'ROCR_VISIBLE_DEVICES': '3', 'HIP_VISIBLE_DEVICES': '0,1'}, kfd) == 1
    assert bench.visible_gpus({'CUDA_VISIBLE_DEVICES': ''}, kfd) == 0
    assert bench.visible_gpus({}, str(tmp_path / 'absent')) == 0
    monkeypatch.setattr(bench, 'KFD_NODES', kfd)
    calls = []
    monkeypatch.setattr(bench.subprocess, 'call', lambda cmd, env=None: calls.append(cmd) or 0)
    monkeypatch.delenv('HIP_VISIBLE_DEVICES', raising=False)
    monkeypatch.delenv('ROCR_VISIBLE_DEVICES', raising=False)
    monkeypatch.delenv('CUDA_VISIBLE_DEVICES', raising=False)
    monkeypatch.setattr(bench, 'visible_gpus', lambda env=None, kfd=kfd: 8)
    assert bench.spawn_ranks(8, ['--gpus', '8']) == 0
    assert calls and calls[0][2] == 'torch.distributed.run'
    assert not torch.cuda.is_initialized()
