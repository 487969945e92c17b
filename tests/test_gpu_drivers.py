"""GPU: the drop-in drivers end to end (train_96 / train_88 / evaluate_head_pose_model) and the
data-parallel fit path with two ranks on one device (gloo transport, same code path as RCCL)."""
import importlib.util
import os
import socket
import sys

import numpy as np
import pytest
import torch

import hpe
from util import DATA, features, fixture, labels

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'head-pose-estimation-model_amd')


def _load(rel, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, rel))
    mod = importlib.util.module_from_spec(spec)
    sys.path.insert(0, os.path.dirname(os.path.join(PKG, rel)))
    spec.loader.exec_module(mod)
    return mod


def test_train96_driver_end_to_end(tmp_path, monkeypatch):
    d = tmp_path / 'maps'
    d.mkdir()
    rng = np.random.default_rng(0)
    for name, n in (('BIWI_train_features_96.npz', 400), ('BIWI_test_features_96.npz', 100)):
        np.savez(d / name, features=np.maximum(0, rng.standard_normal((n, 96)) * .6 - .3).astype(np.float32),
                 poses=rng.standard_normal((n, 3)) * 20)
    import shutil
    shutil.copy(os.path.join(DATA, 'AFLW2000_features_96_0.7_1.npz'), d / 'AFLW2000_features_96_0.7_1.npz')
    ck = tmp_path / 'ckpt'
    monkeypatch.setenv('FEATUREMAPS_DIR_PATH', str(d) + '/')
    monkeypatch.setenv('TRAINED_MODELS_96_RESHAPEDINPUT_NOFLATTEN_PATH', str(ck))
    monkeypatch.setenv('HPE_RUN_DIR', str(tmp_path / 'runs'))
    t96 = _load('Model-96/train_96.py', 't96drv')
    t96.config['total_epochs'] = 3
    model, hist = t96.main(['--dropout_rate', '0.05', '--regularizer_rate', '0.001',
                            '--num_filters', '64'])
    assert len(hist.history['loss']) == 3 and np.isfinite(hist.history['val_loss']).all()
    saved = list(ck.glob('*.h5'))
    assert len(saved) == 1
    tmod = _load('Model-96/test.py', 'test96')
    m = tmod.evaluate_head_pose_model(str(saved[0]), os.path.join(DATA, 'AFLW2000_features_96_0.7_1.npz'))
    assert set(m['MAE']) == {'yaw', 'pitch', 'roll', 'average'}


def test_evaluate_head_pose_model_on_reference_checkpoint():
    tmod = _load('Model-96/test.py', 'test96b')
    m = tmod.evaluate_head_pose_model(os.path.join(ROOT, 'tests/golden/models/hrchr82r'),
                                      os.path.join(DATA, 'AFLW2000_features_96_0.7_1.npz'))
    assert abs(m['MAE']['average'] - 8.0307) < 1.5e-4


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, out):
    for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import hpe as H
    from hpe import keras as kk
    from util import features as f_, fixture as fx, labels as lb
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mc, w = fx('sqnu665j')
    res = {}
    # the step loop in C (hpe_fit_steps_dp, all-reduce hook per step) and the Python loop
    # (HPE_FIT_STEPS=0) from the same state: bit-identical weights
    for mode in ('1', '0'):
        os.environ['HPE_FIT_STEPS'] = mode
        H.set_seed(3)
        m = H.model_from_config(mc, w).distribute()
        m.compile(optimizer=kk.optimizers.Adam(learning_rate=1e-3), loss='mse', metrics=['mae'])
        h = m.fit(f_(160, 96, seed=21), lb(160, seed=22), batch_size=64, epochs=2, shuffle=True, verbose=0)
        res[mode] = (np.asarray(h.history['loss']), m.weights_dict())
        # 129 rows at batch 64 on 2 ranks: the last batch has ONE row, so rank 0's share
        # is empty (hpe_fit_steps_dp's zeroed-gradient branch) while rank 1 trains on it
        H.set_seed(4)
        m2 = H.model_from_config(mc, w).distribute()
        m2.compile(optimizer=kk.optimizers.Adam(learning_rate=1e-3), loss='mse', metrics=['mae'])
        h2 = m2.fit(f_(129, 96, seed=23), lb(129, seed=24), batch_size=64, epochs=2, shuffle=True, verbose=0)
        res[mode + 'r'] = (np.asarray(h2.history['loss']), m2.weights_dict())
        assert m2._eng().iterations == 6
    os.environ.pop('HPE_FIT_STEPS')
    same = True
    for key in ('', 'r'):
        same = same and all(np.array_equal(res['1' + key][1][k], v) for k, v in res['0' + key][1].items())
        same = same and np.array_equal(res['1' + key][0], res['0' + key][0])
    if rank == 0:
        h, wd = res['1']
        np.savez(out, loss=h, c_equals_python=same, **{k.replace('/', '|'): v for k, v in wd.items()})
    dist.destroy_process_group()


def test_data_parallel_fit_matches_single_device(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / 'dp.npz')
    mp.spawn(_dp_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    dp = np.load(out)
    assert bool(dp['c_equals_python'])   # hpe_fit_steps_dp == the Python DP step loop, bit for bit
    mc, w = fixture('sqnu665j')
    hpe.set_seed(3)
    m = hpe.model_from_config(mc, w)
    m.compile(optimizer=hpe.keras.optimizers.Adam(learning_rate=1e-3), loss='mse', metrics=['mae'])
    h = m.fit(features(160, 96, seed=21), labels(160, seed=22), batch_size=64, epochs=2, shuffle=True,
              verbose=0)
    np.testing.assert_allclose(dp['loss'], h.history['loss'], rtol=1e-5)
    for k, v in m.weights_dict().items():
        np.testing.assert_allclose(dp[k.replace('/', '|')], v, rtol=1e-4, atol=1e-6, err_msg=k)


def _bench_worker(rank, world, port, out):
    for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import bench
    import hpe as H
    from hpe import keras as kk
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    H.set_seed(42)
    kk.backend.clear_session()
    m = bench.build_train_model(kk)
    eng = m._eng()
    dev = torch.device('cuda', 0)
    P, n_loc = 64, 12
    x, y = bench.synth(n_loc * world, 7, dev, P=P)   # the global batch; this rank takes its slice
    xs, ys = x[rank * n_loc * P:(rank + 1) * n_loc * P].contiguous(), y[rank * n_loc:(rank + 1) * n_loc].contiguous()
    dt, kms, mse, dom = bench.run_train(eng, m.optimizer, xs, ys, P, n_loc, n_loc * world, rank, world, 3, 1, dist)
    if rank == 0:
        np.savez(out, mse=mse, dt=dt, **{k.replace('/', '|'): v for k, v in m.weights_dict().items()})
    dist.destroy_process_group()


def test_bench_run_train_two_ranks_matches_one(tmp_path):
    """bench.run_train itself (the timed loop of the headline / strong lines) on
    2 gloo ranks sharing one GPU, each taking its slice of the global batch, gives the weights of
    one rank training on the whole batch (one all-reduce of the flat gradient per step)."""
    import torch.multiprocessing as mp
    import bench
    out = str(tmp_path / 'b.npz')
    mp.spawn(_bench_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    dp = np.load(out)
    hpe.set_seed(42)
    hpe.keras.backend.clear_session()
    m = bench.build_train_model(hpe.keras)
    dev = torch.device('cuda', 0)
    P, n = 64, 24
    x, y = bench.synth(n, 7, dev, P=P)
    _, _, mse, dom = bench.run_train(m._eng(), m.optimizer, x, y, P, n, n, 0, 1, 3, 1, None)
    assert 0.0 < dom < 1e3, dom   # the dominant kernel alone, HIP events recorded by libhpe.so
    assert float(dp['mse']) == pytest.approx(mse, rel=1e-4)
    for k, v in m.weights_dict().items():
        np.testing.assert_allclose(dp[k.replace('/', '|')], v, rtol=1e-4, atol=1e-6, err_msg=k)


def _rccl_worker(rank, port, out):
    for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
        sys.path.insert(0, p)
    import ctypes
    import torch.distributed as dist
    import hpe as H
    from hpe import _lib
    from hpe import engine as E
    from hpe import keras as kk
    from util import features as f_, fixture as fx, labels as lb
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    lib = _lib.load()
    # the library's own communicator over the group's one rank: its sum is the identity
    comm = E.rccl_comm(dist, None, dev)
    buf = torch.randn(1001, device=dev)
    ref = buf.clone()
    rc = lib.hpe_rccl_allreduce(ctypes.c_void_p(buf.data_ptr()), buf.numel(),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), comm)
    torch.cuda.synchronize()
    identity = comm is not None and rc == 0 and torch.equal(buf, ref)
    # the data-parallel step loop (hpe_fit_steps_dp) on the one-rank group: the native RCCL hook
    # against the torch.distributed hook, and against the single-rank step loop
    mc, w = fx('sqnu665j')
    os.environ['HPE_FIT_FUSED'] = '0'
    res = {}
    for mode in ('native', 'torch', 'single'):
        os.environ['HPE_NATIVE_RCCL'] = '1' if mode == 'native' else '0'
        os.environ['HPE_FIT_DP_ONE_RANK'] = '0' if mode == 'single' else '1'
        H.set_seed(3)
        m = H.model_from_config(mc, w).distribute()
        m.compile(optimizer=kk.optimizers.Adam(learning_rate=1e-3), loss='mse', metrics=['mae'])
        h = m.fit(f_(160, 96, seed=21), lb(160, seed=22), batch_size=64, epochs=2, shuffle=True, verbose=0)
        res[mode] = (np.asarray(h.history['loss']), m.weights_dict())
    same = all(np.array_equal(res['native'][1][k], v) for k, v in res['torch'][1].items())
    same = same and np.array_equal(res['native'][0], res['torch'][0])
    ncomm = len(E._RCCL_COMMS)
    E.release_rccl_comms()
    dist.destroy_process_group()
    np.savez(out, identity=identity, same=same, ncomm=ncomm, loss=res['native'][0], loss1=res['single'][0],
             **{'n|' + k.replace('/', '|'): v for k, v in res['native'][1].items()},
             **{'s|' + k.replace('/', '|'): v for k, v in res['single'][1].items()})


def test_native_rccl_allreduce_one_rank(tmp_path):
    """hpe_fit_steps_dp with the library's own RCCL all-reduce as its per-step
    hook (hpe_rccl_allreduce, enqueued on the step's stream; no Python per step) on an nccl group of
    ONE rank — the one RCCL configuration a one-GPU box can run: the communicator is made (id
    broadcast over the group), its sum is the identity, and the native hook gives the torch.distributed
    hook's weights bit for bit (and the single-rank loop's within float tolerance).  Across GPUs it is
    unexercised until an 8-GPU run."""
    import torch.multiprocessing as mp
    out = str(tmp_path / 'rccl.npz')
    mp.spawn(_rccl_worker, args=(_free_port(), out), nprocs=1, join=True)
    r = np.load(out)
    assert bool(r['identity'])
    assert int(r['ncomm']) == 1          # the native hook was the one used
    assert bool(r['same'])
    np.testing.assert_allclose(r['loss'], r['loss1'], rtol=1e-5)
    for k in r.files:
        if k.startswith('n|'):
            np.testing.assert_allclose(r[k], r['s|' + k[2:]], rtol=1e-4, atol=1e-6, err_msg=k)
