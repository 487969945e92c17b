"""ctypes binding of libhpe.so (include/hpe.h).  The library is built in-tree by
``__graft_entry__.build()`` (hipcc --offload-arch=gfx950); there is no fallback: every compute
call goes through these symbols, and a missing library raises at first use."""
import ctypes
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('HPE_LIB') or os.path.join(_HERE, 'libhpe.so')  # HPE_LIB: debug builds

# symbol -> (restype, argtypes), exactly the declarations of include/hpe.h
_vp, _i32, _i64, _f, _u64, _sz = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float,
                                  ctypes.c_uint64, ctypes.c_size_t)
SIGNATURES = {
    'hpe_program_create': (ctypes.c_int, [_vp, _i64, ctypes.POINTER(_vp)]),
    'hpe_program_destroy': (ctypes.c_int, [_vp]),
    'hpe_launch_grid': (ctypes.c_int, [_vp, _i64]),
    'hpe_workspace_size': (_sz, [_vp, _i64]),
    'hpe_forward': (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp]),
    'hpe_train_step': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _f, _u64,
                                      _vp, _vp]),
    'hpe_train_step_bounded': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _f, _u64,
                                              _f, _vp, _vp]),
    'hpe_reduce': (ctypes.c_int, [_vp, _i64, _vp, _vp, _vp]),
    'hpe_optim_step': (ctypes.c_int, [_i32, _f, _f, _f, _f, _i64, _f, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _vp, _i64, _vp, _vp]),
    'hpe_optim_grid': (ctypes.c_int, [_i64]),
    'hpe_reduce_optim_step': (ctypes.c_int, [_vp, _i64, _vp, _vp, _i32, _f, _f, _f, _f, _i64, _f, _vp, _vp, _vp,
                                             _vp, _vp, _vp, _i64, _vp, _vp]),
    'hpe_fit_steps': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _i32,
                                     _f, _i32, _f, _f, _f, _f, _u64, _i64, _vp, _vp, _vp, _i32, _vp]),
    'hpe_fit_steps_dp': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i64, _i32, _i32,
                                        _f, _i32, _f, _f, _f, _f, _u64, _i64, _vp, _vp, _vp, _i32, _i32, _i32,
                                        _vp, _vp, _vp, _vp]),
    'hpe_fit_supported': (ctypes.c_int, [_vp, _i32]),
    'hpe_fit_workspace_size': (_sz, [_vp, _i32]),
    'hpe_fit_epoch': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _f,
                                     _f, _f, _f, _vp, _u64, _i64, _vp, _i32, _i32, _vp, _vp]),
    'hpe_blazeface_create': (ctypes.c_int, [_vp, _i64, ctypes.POINTER(_vp)]),
    'hpe_blazeface_destroy': (ctypes.c_int, [_vp]),
    'hpe_blazeface_workspace_size': (_sz, [_vp, _i64]),
    'hpe_blazeface_forward': (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    'hpe_detect': (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _f, _f, _i32, _vp, _vp, _vp, _vp,
                                  _vp, _vp, _vp]),
    'hpe_gather_features': (ctypes.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _i32, _vp, _i32, _vp, _vp,
                                           _vp, _vp]),
    'hpe_se_gate': (ctypes.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp, _i32, _i32, _vp, _vp, _i32,
                                   _vp]),
    'hpe_seg_mean': (ctypes.c_int, [_vp, _vp, _i64, _i32, _i32, _vp]),
    'hpe_mha': (ctypes.c_int, [_vp, _i32, _i32, _vp, _i32, _i64, _i32, _i32, _i32, _vp]),
    'hpe_mha_xg': (ctypes.c_int, [_vp, _i32, _vp, _i32, _vp, _i32, _i64, _i32, _i32, _i32, _vp]),
    'hpe_attn_tail_supported': (ctypes.c_int, [_vp]),
    'hpe_attn_tail': (ctypes.c_int, [_vp, _i32, _vp, _i32, _i64, _vp, _vp, _vp, _vp]),
    'hpe_last_error': (ctypes.c_char_p, []),
    'hpe_build_id': (ctypes.c_char_p, []),
    'hpe_guard_peek': (ctypes.c_int, [_vp, _vp]),
    'hpe_kernel_timing': (ctypes.c_int, [_i32]),
    'hpe_kernel_times': (ctypes.c_int, [_vp, _i32]),
    'hpe_set_exact_fp32': (ctypes.c_int, [ctypes.c_int]),
    'hpe_act_probe': (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_void_p]),
    'hpe_rccl_available': (ctypes.c_int, []),
    'hpe_rccl_unique_id': (ctypes.c_int, [_vp]),
    'hpe_rccl_comm_init': (ctypes.c_int, [_vp, _i32, _i32, ctypes.POINTER(_vp)]),
    'hpe_rccl_comm_destroy': (ctypes.c_int, [_vp]),
    'hpe_rccl_allreduce': (ctypes.c_int, [_vp, _i64, _vp, _vp]),
}
RCCL_ID_BYTES = 128   # HPE_RCCL_ID_BYTES

_lib = None
_CSRC = os.path.join(os.path.dirname(_HERE), 'csrc')
_HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), 'include', 'hpe.h')


def source_hash():
    """The src= field csrc/Makefile stamps into libhpe.so: sha256 of the .hip / .h sources in name
    order, include/hpe.h and the Makefile (first 16 hex digits); None without the sources."""
    if not os.path.isdir(_CSRC):
        return None
    names = sorted(f for f in os.listdir(_CSRC) if f.endswith('.hip') or f.endswith('.h'))
    h = hashlib.sha256()
    for path in [os.path.join(_CSRC, f) for f in names] + [_HEADER, os.path.join(_CSRC, 'Makefile')]:
        with open(path, 'rb') as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_id():
    return load().hpe_build_id().decode()


class HPEError(RuntimeError):
    pass


def load():
    """Load libhpe.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HPEError('libhpe.so not found at %s: run __graft_entry__.build() (hipcc gfx950)'
                       % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # the library must be built from the sources of this tree (HPE_ALLOW_STALE=1: debug builds)
    want = source_hash()
    got = lib.hpe_build_id().decode()
    if want and 'src=%s ' % want not in got + ' ' and os.environ.get('HPE_ALLOW_STALE') != '1' \
            and not os.environ.get('HPE_LIB'):
        raise HPEError('libhpe.so (%s) was built from other sources than this tree (src=%s): '
                       'rebuild with __graft_entry__.build()' % (got, want))
    _lib = lib
    return lib


def check(rc, what=''):
    if rc == 0:
        return
    msg = load().hpe_last_error().decode(errors='replace')
    if rc == 1:
        raise ValueError('%s: %s' % (what, msg))
    raise HPEError('%s: %s' % (what, msg))
