"""CPU, world_size 2 over gloo: the data-parallel decomposition of a training step (per-rank
contiguous batch slices, gradient normalised by the global element count, one all-reduce of the
flat gradient + loss sums) reproduces the single-device gradient.  Per-rank gradients come from
the row-program emulator running the same compiled program the HIP kernel runs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hpe.parallel import batch_slice


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat(prog, w):
    p = np.zeros(prog.n_params)
    for k, (o, shp) in prog.param_index.items():
        p[o:o + int(np.prod(shp))] = w[k].ravel()
    return p


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), 'head-pose-estimation-model_amd'), here):
        sys.path.insert(0, p)
    import hpe.compiler as C
    import rowprog_emu as EMU
    from hpe.parallel import all_reduce_grad, batch_slice as bs
    from util import features, fixture, labels
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mc, w = fixture('stoqa9pt')
    prog = C.compile_graph(mc, w, 'train', fused=False)
    x = features(37, 88, seed=11)
    y = labels(37, seed=12)
    r0, r1 = bs(0, 37, rank, world)
    r = EMU.run(prog, _flat(prog, w), x[r0:r1].reshape(r1 - r0, 88), y_img=y[r0:r1].astype(np.float64),
                inv_count=1.0 / (37 * 3), seed=5, img_off=r0)
    g = torch.tensor(np.concatenate([r['grad'], [r['sse'], r['sae']]]), dtype=torch.float64)
    all_reduce_grad(g)
    if rank == 0:
        torch.save(g, out)
    dist.destroy_process_group()


def test_batch_slice_partitions():
    for nb in (1, 2, 7, 128, 513):
        for world in (1, 2, 3, 8):
            spans = [batch_slice(10, 10 + nb, r, world) for r in range(world)]
            assert spans[0][0] == 10 and spans[-1][1] == 10 + nb
            for a, b in zip(spans, spans[1:]):
                assert a[1] == b[0]
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_two_rank_gradient_equals_single(tmp_path):
    import hpe.compiler as C
    import rowprog_emu as EMU
    from util import features, fixture, labels
    out = str(tmp_path / 'g.pt')
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    g2 = torch.load(out, weights_only=True).numpy()
    mc, w = fixture('stoqa9pt')
    prog = C.compile_graph(mc, w, 'train', fused=False)
    x = features(37, 88, seed=11)
    y = labels(37, seed=12)
    r = EMU.run(prog, _flat(prog, w), x.reshape(37, 88), y_img=y.astype(np.float64),
                inv_count=1.0 / (37 * 3), seed=5)
    g1 = np.concatenate([r['grad'], [r['sse'], r['sae']]])
    np.testing.assert_allclose(g2, g1, rtol=1e-10, atol=1e-12)


def _rccl_gate_worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), 'head-pose-estimation-model_amd'), here):
        sys.path.insert(0, p)
    from hpe import engine as E
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    # gloo group (or no GPU device): the native RCCL hook is not used, the torch.distributed
    # callback stays; nothing is created (no device touched)
    res = [E.rccl_comm(dist, None, torch.device('cuda', 0)) is None,
           E.rccl_comm(dist, None, None) is None,
           E.rccl_comm(dist, None, torch.device('cpu')) is None,
           len(E._RCCL_COMMS) == 0]
    if rank == 0:
        torch.save(torch.tensor(res), out)
    dist.destroy_process_group()


def test_native_rccl_hook_gated_to_nccl_groups(tmp_path):
    """hpe.engine.rccl_comm: the library's RCCL communicator is made only for nccl (RCCL) groups on
    a GPU device; gloo ranks keep the torch.distributed per-step hook (two gloo ranks on CPU)."""
    out = str(tmp_path / 'gate.pt')
    mp.spawn(_rccl_gate_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert bool(torch.load(out, weights_only=True).all())
