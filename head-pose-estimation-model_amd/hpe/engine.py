"""Device-side execution of one model: compiled row programs, parameter / optimizer buffers, and
the per-step launch sequence (train_step -> reduce -> [RCCL all-reduce] -> optimizer).

PyTorch is used only for device memory, the current HIP stream and torch.distributed (RCCL); every
arithmetic op of the hot path runs in libhpe.so (csrc/hpe_rowprog.hip) through the C ABI.
"""
import ctypes
import os
import warnings

import numpy as np
import torch

from . import _lib
from .compiler import build_mirror, compile_graph

OPT_KIND = {'sgd': 0, 'adam': 1, 'adamax': 2}


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_RCCL_COMMS = {}   # (group, device) -> the library's RCCL communicator for hpe_fit_steps_dp


def rccl_comm(mod, grp, device, nranks=None, rank=None):
    """The library's own RCCL communicator over the ranks of process group `grp` (one per group and
    device, made once: rank 0's hpe_rccl_unique_id broadcast over the group, then
    hpe_rccl_comm_init on every rank's current device), or None when the group is not an nccl
    (RCCL) group on a GPU, librccl does not load, or HPE_NATIVE_RCCL=0 — the caller then keeps
    the torch.distributed hook.  nranks / rank default to the group's."""
    if os.environ.get('HPE_NATIVE_RCCL', '1') == '0' or device is None or torch.device(device).type != 'cuda':
        return None
    if str(mod.get_backend(grp)).lower() != 'nccl':
        return None
    lib = _lib.load()
    if not lib.hpe_rccl_available():
        return None
    device = torch.device(device)
    if device.index is None:
        device = torch.device('cuda', torch.cuda.current_device())
    pg = grp if grp is not None else mod.group.WORLD   # the group object itself: a re-initialised
    key = (pg, device.index)                           # default group gets its own communicator
    if key not in _RCCL_COMMS:
        nranks = mod.get_world_size(grp) if nranks is None else nranks
        rank = mod.get_rank(grp) if rank is None else rank
        uid = ctypes.create_string_buffer(_lib.RCCL_ID_BYTES)
        if rank == 0:
            _lib.check(lib.hpe_rccl_unique_id(uid), 'hpe_rccl_unique_id')
        obj = [bytes(uid.raw) if rank == 0 else None]
        mod.broadcast_object_list(obj, group=grp, group_src=0)
        uid = ctypes.create_string_buffer(obj[0], _lib.RCCL_ID_BYTES)
        comm = ctypes.c_void_p()
        with torch.cuda.device(device):
            _lib.check(lib.hpe_rccl_comm_init(uid, int(nranks), int(rank), ctypes.byref(comm)), 'hpe_rccl_comm_init')
        _RCCL_COMMS[key] = comm
    return _RCCL_COMMS[key]


def release_rccl_comms():
    """Destroy every communicator rccl_comm made (before its process group is destroyed)."""
    lib = _lib.load()
    while _RCCL_COMMS:
        _, comm = _RCCL_COMMS.popitem()
        _lib.check(lib.hpe_rccl_comm_destroy(comm), 'hpe_rccl_comm_destroy')


class _Compiled:
    def __init__(self, prog):
        self.prog = prog
        lib = _lib.load()
        h = ctypes.c_void_p()
        w = np.ascontiguousarray(prog.words, dtype=np.int32)
        _lib.check(lib.hpe_program_create(w.ctypes.data_as(ctypes.c_void_p), w.size, ctypes.byref(h)),
                   'hpe_program_create')
        self.h = h
        self.ws = None
        self.ws_rows = -1

    def workspace(self, n_rows, device):
        lib = _lib.load()
        need = lib.hpe_workspace_size(self.h, n_rows)
        if self.ws is None or self.ws.numel() * 4 < need:
            # zero once: slab entries no op owns stay zero for ever
            self.ws = torch.zeros(max(need // 4, 4), dtype=torch.float32, device=device)
        return self.ws

    def __del__(self):
        try:
            if self.h:
                _lib.load().hpe_program_destroy(self.h)
        except Exception:
            pass


class Engine:
    """Parameters live on the device as one flat fp32 vector in Keras trainable_weights order
    (+ inference constants), plus the transposed mirror the backward GEMMs read."""

    def __init__(self, model_config, weights, device=None, fused=None):
        if not torch.cuda.is_available():
            raise _lib.HPEError('hpe needs a ROCm GPU (MI355X / gfx950); torch.cuda is unavailable')
        self.device = torch.device(device or 'cuda')
        self.model_config = model_config
        self.weights = dict(weights)
        self.progs = {}
        import os
        self.fused = (os.environ.get('HPE_FUSED', '1') != '0') if fused is None else fused
        base = compile_graph(model_config, self.weights, mode='fwd', fused=False)
        self.layout = base
        flat = np.zeros(base.n_train, dtype=np.float32)
        for k, (o, shp) in base.param_index.items():
            flat[o:o + int(np.prod(shp))] = np.asarray(self.weights[k], dtype=np.float32).ravel()
        self.n_train = base.n_train
        self.params = torch.from_numpy(np.concatenate([flat, base.consts])).to(self.device)
        self.params_t = torch.from_numpy(build_mirror(base, flat)).to(self.device)
        self.l2 = torch.from_numpy(base.l2).to(self.device)
        self.tpos = torch.from_numpy(base.tpos).to(self.device)
        self.m = None
        self._pending = None   # (program, rows, workspace) of a gradient awaiting its fused reduce
        self.v = None
        self._fit_ws = None
        self.iterations = 0
        self.grad = torch.zeros(self.n_train + 4, dtype=torch.float32, device=self.device)

    # -- programs -----------------------------------------------------------------------------
    def program(self, mode, P=1):
        key = (mode, P == 1)
        if key not in self.progs:
            prog = compile_graph(self.model_config, self.weights, mode=mode, P=P, fused=self.fused)
            if prog.n_train != self.n_train:
                raise RuntimeError('parameter layout mismatch between programs')
            if prog.consts.size and self.params.numel() != self.n_train + prog.consts.size:
                self.params = torch.cat([self.params[:self.n_train],
                                         torch.from_numpy(prog.consts).to(self.device)])
            self.progs[key] = _Compiled(prog)
        return self.progs[key]

    # -- host <-> device weights --------------------------------------------------------------
    def get_weights(self):
        flat = self.params[:self.n_train].detach().cpu().numpy()
        out = {}
        for k, (o, shp) in self.layout.param_index.items():
            out[k] = flat[o:o + int(np.prod(shp))].reshape(shp).copy()
        return out

    def set_weights(self, wdict):
        if hasattr(self, '_spatial'):
            del self._spatial  # rebuilt from the new weights on the next H x W > 1 forward
        flat = self.params[:self.n_train].detach().cpu().numpy().copy()
        for k, a in wdict.items():
            o, shp = self.layout.param_index[k]
            a = np.asarray(a, dtype=np.float32)
            if a.shape != tuple(shp):
                raise ValueError('weight %s: shape %s != %s' % (k, a.shape, tuple(shp)))
            flat[o:o + a.size] = a.ravel()
        self.params[:self.n_train].copy_(torch.from_numpy(flat))
        self.params_t.copy_(torch.from_numpy(build_mirror(self.layout, flat)))
        self.weights.update({k: np.asarray(v, dtype=np.float32) for k, v in wdict.items()})

    # -- compute ------------------------------------------------------------------------------
    def spatial(self):
        """Staged executor for graphs with ops that are not row-local on H x W > 1 maps (SE gate,
        spatial MHA, terminal GAP: hpe/spatial.py), or None."""
        if not hasattr(self, '_spatial'):
            from .spatial import SpatialHead, is_spatial
            self._spatial = SpatialHead(self.model_config, self.get_weights(), self.device) \
                if is_spatial(self.model_config) else None
        return self._spatial

    def forward(self, x, P, idx=None, out=None):
        """x: device fp32 [n_images*P, C_in] (rows); returns [n_images*P, C_out] ([n_images, C_out]
        for a graph ending in GlobalAveragePooling2D at P > 1)."""
        if P > 1 and self.spatial() is not None:
            if idx is not None:
                raise ValueError('gathered batches of attention heads on H x W > 1 maps are not supported')
            return self._spatial.forward(x, P, out=out)
        c = self.program('fwd', P)
        n_img = x.shape[0] // P if idx is None else idx.numel()
        if out is None:
            out = torch.empty((n_img * P, c.prog.C_out), dtype=torch.float32, device=self.device)
        lib = _lib.load()
        _lib.check(lib.hpe_forward(c.h, _ptr(self.params), _ptr(self.params_t), _ptr(x), n_img, P,
                                   _ptr(idx), _ptr(out), _stream()), 'hpe_forward')
        return out

    def loss_sums(self, x, y, P, idx=None, n_images=None):
        """Eval pass: returns device tensor [sum e^2, sum |e|, ...] (grad buffer layout)."""
        if P > 1 and self.spatial() is not None:
            raise ValueError('evaluate / fit of attention heads runs on 1x1 maps (the reference '
                             'trains them at P = 1, train_88.py:270-305); use predict on H x W maps')
        c = self.program('eval', P)
        n_img = n_images if n_images is not None else (x.shape[0] // P if idx is None else idx.numel())
        lib = _lib.load()
        ws = c.workspace(n_img * P, self.device)
        _lib.check(lib.hpe_train_step(c.h, _ptr(self.params), _ptr(self.params_t), _ptr(x), _ptr(y),
                                      n_img, P, _ptr(idx), 0, 1.0, 0, _ptr(ws), _stream()),
                   'hpe_train_step(eval)')
        out = torch.empty(self.n_train + 4, dtype=torch.float32, device=self.device)
        _lib.check(lib.hpe_reduce(c.h, n_img * P, _ptr(ws), _ptr(out), _stream()), 'hpe_reduce')
        return out[self.n_train:self.n_train + 2]

    # per-step launches whose persistent grid is at most this many workgroups hand the slab
    # reduction to the optimizer launch (hpe_reduce_optim_step: one launch fewer per step)
    FUSED_REDUCE_MAX_GRID = 16

    def gradient(self, x, y, P, idx, n_images, inv_count, seed, img_off=0, defer_reduce=False, x_bound=0.0):
        """fwd + loss + bwd over this rank's images; self.grad = [dL/dparams..., sse, sae, 0, 0].
        defer_reduce: a single-rank fit step whose next call is optimizer_step may leave the
        per-workgroup slabs unreduced; optimizer_step then reduces and updates in one launch
        (self.grad is written by that launch, bit-identical to hpe_reduce's).  x_bound: a known
        bound on max |x| (fit: once per call over the resident dataset; 0 = unknown) that lets the
        fp16-split kernels skip their exact-fp32 twin launch (hpe_train_step_bounded)."""
        if P > 1 and self.spatial() is not None:
            raise ValueError('fit of attention heads runs on 1x1 maps (train_88.py:270-305)')
        c = self.program('train', P)
        lib = _lib.load()
        rows = n_images * P
        ws = c.workspace(rows, self.device)
        _lib.check(lib.hpe_train_step_bounded(c.h, _ptr(self.params), _ptr(self.params_t), _ptr(x), _ptr(y),
                                              n_images, P, _ptr(idx), img_off, float(inv_count),
                                              int(seed) & 0xFFFFFFFFFFFFFFFF, float(x_bound), _ptr(ws),
                                              _stream()),
                   'hpe_train_step')
        self._pending = None
        if defer_reduce and lib.hpe_launch_grid(c.h, rows) <= self.FUSED_REDUCE_MAX_GRID:
            self._pending = (c, rows, ws)
            return None
        _lib.check(lib.hpe_reduce(c.h, rows, _ptr(ws), _ptr(self.grad), _stream()), 'hpe_reduce')
        return self.grad

    def optimizer_step(self, opt, stats, grad_scale=1.0):
        kind = OPT_KIND[opt.kind]
        if kind and self.m is None:
            self.m = torch.zeros(self.n_train, dtype=torch.float32, device=self.device)
            self.v = torch.zeros(self.n_train, dtype=torch.float32, device=self.device)
        self.iterations += 1
        lib = _lib.load()
        pend = getattr(self, '_pending', None)
        if pend is not None:
            self._pending = None
            c, rows, ws = pend
            _lib.check(lib.hpe_reduce_optim_step(c.h, rows, _ptr(ws), _ptr(self.grad), kind,
                                                 float(opt.learning_rate), float(opt.beta_1),
                                                 float(opt.beta_2), float(opt.epsilon), self.iterations,
                                                 float(grad_scale), _ptr(self.params), _ptr(self.params_t),
                                                 _ptr(self.m), _ptr(self.v), _ptr(self.l2), _ptr(self.tpos),
                                                 self.n_train, _ptr(stats), _stream()),
                       'hpe_reduce_optim_step')
            return
        _lib.check(lib.hpe_optim_step(kind, float(opt.learning_rate), float(opt.beta_1),
                                      float(opt.beta_2), float(opt.epsilon), self.iterations,
                                      float(grad_scale), _ptr(self.params), _ptr(self.params_t),
                                      _ptr(self.m), _ptr(self.v), _ptr(self.grad), _ptr(self.l2),
                                      _ptr(self.tpos), self.n_train, _ptr(stats), _stream()),
                   'hpe_optim_step')

    def optim_grid(self):
        return _lib.load().hpe_optim_grid(self.n_train)

    # the all-reduce hook hpe_fit_steps_dp calls once per step (int (*)(float*, int64, void*, void*)):
    # hpe_rccl_allreduce on GPU ranks of an nccl (RCCL) group, else this Python callback
    ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p)

    def fit_steps(self, opt, x, y, perm, batch, stats, seed_base, x_bound=0.0, P=1, dist=None):
        """One epoch of fit's per-step path as ONE C call: hpe_fit_steps issues, per step, the
        launches gradient(defer_reduce=True) + optimizer_step issue from Python, with the same
        arguments (bit-identical results) and no Python round trip between steps.  dist = (module,
        group) of a data-parallel fit: hpe_fit_steps_dp runs this rank's share of every batch and
        calls back once per step for the all-reduce of [gradient | loss sums] (torch.distributed:
        RCCL on GPU ranks), the launches of the Python DP loop in the same order."""
        if P > 1 and self.spatial() is not None:
            raise ValueError('fit of attention heads runs on 1x1 maps (train_88.py:270-305)')
        kind = OPT_KIND[opt.kind]
        if kind and self.m is None:
            self.m = torch.zeros(self.n_train, dtype=torch.float32, device=self.device)
            self.v = torch.zeros(self.n_train, dtype=torch.float32, device=self.device)
        c = self.program('train', P)
        lib = _lib.load()
        n = int(perm.numel())
        steps = (n + batch - 1) // batch
        ws = c.workspace(min(batch, n) * P, self.device)
        if dist is not None and (dist[0].get_world_size(dist[1]) > 1 or os.environ.get('HPE_FIT_DP_ONE_RANK') == '1'):
            mod, grp = dist
            errors = []
            comm = rccl_comm(mod, grp, self.device)
            if comm is not None:
                # GPU ranks: the library's own RCCL sum on the step's stream, no Python per step
                hook, user = ctypes.cast(lib.hpe_rccl_allreduce, ctypes.c_void_p), comm
            else:
                def allreduce(_buf, _n, _stream, _user):
                    try:
                        mod.all_reduce(self.grad, group=grp)
                        return 0
                    except Exception as e:   # surfaces as HPE_ERUNTIME from the C loop, re-raised below
                        errors.append(e)
                        return 1
                hook, user = self.ALLREDUCE_FN(allreduce), None
            done = ctypes.c_int64(0)
            rc = lib.hpe_fit_steps_dp(c.h, _ptr(self.params), _ptr(self.params_t), _ptr(self.m), _ptr(self.v),
                                      _ptr(self.l2), _ptr(self.tpos), self.n_train, _ptr(x), _ptr(y), _ptr(perm),
                                      n, int(batch), int(P), float(x_bound), kind, float(opt.learning_rate),
                                      float(opt.beta_1), float(opt.beta_2), float(opt.epsilon),
                                      int(seed_base) & 0xFFFFFFFFFFFFFFFF, int(self.iterations), _ptr(ws),
                                      _ptr(self.grad), _ptr(stats), int(stats.shape[1]),
                                      mod.get_rank(grp), mod.get_world_size(grp),
                                      ctypes.cast(hook, ctypes.c_void_p), user, ctypes.byref(done), _stream())
            # the steps whose optimizer update was applied advance the iteration count even when
            # the epoch stopped early (Adam's bias correction and the dropout seeds of a retry stay
            # in step with params / m / v)
            self._pending = None
            self.iterations += int(done.value)
            if errors:
                raise errors[0]
            _lib.check(rc, 'hpe_fit_steps_dp')
            return
        _lib.check(lib.hpe_fit_steps(c.h, _ptr(self.params), _ptr(self.params_t), _ptr(self.m), _ptr(self.v),
                                     _ptr(self.l2), _ptr(self.tpos), self.n_train, _ptr(x), _ptr(y), _ptr(perm),
                                     n, int(batch), int(P), float(x_bound), kind, float(opt.learning_rate),
                                     float(opt.beta_1), float(opt.beta_2), float(opt.epsilon),
                                     int(seed_base) & 0xFFFFFFFFFFFFFFFF, int(self.iterations), _ptr(ws),
                                     _ptr(self.grad), _ptr(stats), int(stats.shape[1]), _stream()),
                   'hpe_fit_steps')
        self._pending = None
        self.iterations += steps

    # -- whole-epoch launch (P = 1, one rank): csrc/hpe_fit.hip ----------------------------------
    # batches above this run the per-step path unless HPE_FIT_FUSED=1: the epoch kernel computes
    # on one XCD's workgroups (hidden units split over <= 32 CUs), which wins while a step is
    # latency-bound (b128: 16.5 vs 41.7 us / step) and loses once it is not (b512: 56.1 vs 46.2 us,
    # profiles/r03c_bench.json p1 lines, MI355X)
    FIT_FUSED_AUTO_MAX = 256

    def fit_epoch_supported(self, batch, P=1, world=1):
        """True when fit's epoch can run as ONE hpe_fit_epoch launch: the reference's regime (1x1
        maps, the 2-layer create_model family, one rank) at batch <= FIT_FUSED_AUTO_MAX;
        HPE_FIT_FUSED=0 forces the per-step path, HPE_FIT_FUSED=1 the fused one wherever the
        kernel supports the batch (<= 512)."""
        env = os.environ.get('HPE_FIT_FUSED')
        if world != 1 or P != 1 or env == '0':
            return False
        if env is None and batch > self.FIT_FUSED_AUTO_MAX:
            return False
        if getattr(self, '_fit_disabled', False):   # an earlier epoch launch timed out
            return False
        c = self.program('train', 1)
        return c.prog.kind in ('mlp2', 'res') and _lib.load().hpe_fit_supported(c.h, int(batch)) == 1

    def fit_groups(self):
        """Workgroups of the whole-epoch launch: one per 32 hidden units (create_model family); one
        for the residual stacks (csrc/hpe_res.hip: stats [sse, sae, regularisation loss])."""
        prog = self.program('train', 1).prog
        if prog.kind == 'res':
            return 1
        return -(-int(prog.info['F']) // 32)

    def _alphas(self, opt, steps):
        """Per-iteration optimizer step sizes, computed exactly as hpe_optim_step does (double
        arithmetic on the float32 hyper-parameters, rounded to float32)."""
        t = (self.iterations + 1 + np.arange(steps)).astype(np.float64)
        lr = float(np.float32(opt.learning_rate))
        b1 = float(np.float32(opt.beta_1))
        b2 = float(np.float32(opt.beta_2))
        if opt.kind == 'adam':
            a = lr * np.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)
        elif opt.kind == 'adamax':
            a = lr / (1.0 - b1 ** t)
        else:
            a = np.full(steps, lr)
        return torch.from_numpy(a.astype(np.float32)).to(self.device)

    def _restore(self, saved):
        for dst, src in zip([t for t in (self.params, self.params_t, self.m, self.v) if t is not None], saved):
            dst.copy_(src)

    def fit_epoch(self, opt, x, y, perm, batch, stats, seed_base):
        """One epoch of fit: ceil(n / batch) steps over rows perm (device int32) of x / y in one
        launch; stats: device [steps, >= 2 + G].  A flagged fp16-split overflow re-runs the epoch
        on the exact-fp32 path from the saved state.  A workgroup-exchange timeout (flag 2: the G
        workgroups were not all resident, e.g. another job held CUs) leaves workgroups at different
        steps, so the saved parameters / Adam state are restored, the fused path is disabled for this
        engine, and None is returned: the caller re-runs the epoch on the per-step path."""
        c = self.program('train', 1)
        lib = _lib.load()
        kind = OPT_KIND[opt.kind]
        if kind and self.m is None:
            self.m = torch.zeros(self.n_train, dtype=torch.float32, device=self.device)
            self.v = torch.zeros(self.n_train, dtype=torch.float32, device=self.device)
        n = int(perm.numel())
        steps = -(-n // int(batch))
        alpha = self._alphas(opt, steps)
        need = lib.hpe_fit_workspace_size(c.h, int(batch))
        if getattr(self, '_fit_ws', None) is None or self._fit_ws.numel() * 4 < need:
            self._fit_ws = torch.zeros(max(need // 4, 16), dtype=torch.float32, device=self.device)
        saved = [t.clone() for t in (self.params, self.params_t, self.m, self.v) if t is not None]

        def launch(exact):
            _lib.check(lib.hpe_fit_epoch(
                c.h, _ptr(self.params), _ptr(self.params_t), _ptr(self.m), _ptr(self.v), _ptr(self.l2),
                _ptr(self.tpos), _ptr(x), _ptr(y), _ptr(perm), n, int(batch), kind, float(opt.learning_rate),
                float(opt.beta_1), float(opt.beta_2), float(opt.epsilon), _ptr(alpha),
                int(seed_base) & 0xFFFFFFFFFFFFFFFF, int(self.iterations), _ptr(stats), int(stats.shape[1]),
                int(exact), _ptr(self._fit_ws), _stream()), 'hpe_fit_epoch')
            return int(self._fit_ws[:2].view(torch.int32)[1].item())

        flags = launch(0)
        if flags & 1:  # fp16 range exceeded somewhere: redo the epoch exactly
            self._restore(saved)
            flags = launch(1)
        if flags & 2:
            self._restore(saved)
            self._fit_disabled = True
            warnings.warn('hpe_fit_epoch: workgroup exchange timed out; epoch re-run on the per-step path')
            return None
        self.iterations += steps
        return steps
