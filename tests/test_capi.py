"""CPU: the C-ABI library (built by __graft_entry__.build) loads and exports exactly the entry
points include/hpe.h declares.  No compute call is made without a GPU."""
import ctypes
import os
import re

import pytest

from hpe import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(ROOT, 'include', 'hpe.h')) as fh:
        src = fh.read()
    return set(re.findall(r'^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(hpe_[a-z_0-9]+)\s*\(', src, re.M))


def test_header_declares_expected_entry_points():
    assert _declared() == set(_lib.SIGNATURES)


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason='libhpe.so not built')
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason='libhpe.so not built')
def test_error_path_without_gpu():
    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.hpe_program_create(None, 0, ctypes.byref(h))
    assert rc == 1
    assert b'null' in lib.hpe_last_error()


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason='libhpe.so not built')
def test_build_stamp_matches_tree_sources():
    """libhpe.so carries the hash of the sources it was built from
    (csrc/Makefile hpe_build.o) and the binding refuses a library built from other sources, so the
    kernels a run loads are this checkout's."""
    bid = _lib.build_id()
    assert bid.startswith('src=') and ' git=' in bid
    assert bid.split()[0] == 'src=' + _lib.source_hash()


def _complex():
    import importlib.util
    import hpe
    from hpe import keras
    path = os.path.join(ROOT, 'head-pose-estimation-model_amd', 'Model-88', 'attention_model.py')
    spec = importlib.util.spec_from_file_location('hpe_attention_model_88_capi', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    keras.backend.clear_session()
    hpe.set_seed(88)
    m = mod.create_model_complex(1e-6, 1e-4)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse')
    return m


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason='libhpe.so not built')
def test_fused_kernel_programs_pass_host_validation():
    """train_88.py's create_model_complex at P = 1 compiles to the residual-stack kernel (KIND_RES)
    and hpe_program_create's host-side validation accepts it: with no GPU the call gets as far as
    the device allocation (rc 2), never a geometry rejection (rc 1)."""
    import numpy as np
    from hpe import compiler
    m = _complex()
    prog = compiler.compile_graph(m.model_config, m.weights_dict(), mode='train', P=1)
    assert prog.kind == 'res' and prog.info['blocks'] == 3
    lib = _lib.load()
    w = np.ascontiguousarray(prog.words, np.int32)
    h = ctypes.c_void_p()
    rc = lib.hpe_program_create(w.ctypes.data_as(ctypes.c_void_p), w.size, ctypes.byref(h))
    assert rc != 1, lib.hpe_last_error()


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason='libhpe.so not built')
def test_rccl_hook_argument_checks_without_gpu():
    """hpe_rccl_*: argument errors come back as HPE_EINVAL with a message, before any RCCL or
    device call (the hook itself runs in tests/test_gpu_drivers.py on a one-rank nccl group)."""
    lib = _lib.load()
    assert lib.hpe_rccl_available() in (0, 1)
    assert lib.hpe_rccl_allreduce(None, 16, None, None) == 1
    assert b'hpe_rccl_allreduce' in lib.hpe_last_error()
    comm = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(_lib.RCCL_ID_BYTES)
    assert lib.hpe_rccl_comm_init(uid, 0, 0, ctypes.byref(comm)) == 1
    assert lib.hpe_rccl_comm_init(uid, 2, 2, ctypes.byref(comm)) == 1 and not comm.value
    assert lib.hpe_rccl_comm_init(None, 1, 0, ctypes.byref(comm)) == 1
    assert lib.hpe_rccl_unique_id(None) == 1
    assert lib.hpe_rccl_comm_destroy(None) == 0
