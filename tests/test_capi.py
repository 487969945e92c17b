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


def _m88(F):
    import hpe
    from hpe import keras
    keras.backend.clear_session()
    hpe.set_seed(88)
    reg = keras.regularizers.l2(1e-6)
    inp = keras.Input(shape=(None, None, 88))
    h = keras.layers.SpatialDropout2D(1e-4)(keras.layers.Conv2D(F, 1, activation='softsign', kernel_regularizer=reg)(inp))
    o = keras.layers.SpatialDropout2D(1e-4)(keras.layers.Conv2D(3, 1, kernel_regularizer=reg)(h))
    m = keras.Model(inp, o)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse')
    return m


@pytest.mark.parametrize('F', [16, 32, 48, 64])
def test_fused_kernel_programs_pass_host_validation(F, monkeypatch):
    """train_88.py's create_model at P = 1 compiles (HPE_WIDE=1) to the wide residual-stack kernel
    (KIND_RES, no blocks) and hpe_program_create's host-side validation accepts it — with no GPU the call gets as
    far as the device allocation (rc 2), never a geometry rejection (rc 1).  Regression: F = 64
    (5,891 parameters) once exceeded the kernels' LDS parameter capacity."""
    import numpy as np
    from hpe import compiler
    monkeypatch.setenv('HPE_WIDE', '1')
    m = _m88(F)
    prog = compiler.compile_graph(m.model_config, m.weights_dict(), mode='train', P=1)
    assert prog.kind == 'res' and prog.info['blocks'] == 0
    lib = _lib.load()
    w = np.ascontiguousarray(prog.words, np.int32)
    h = ctypes.c_void_p()
    rc = lib.hpe_program_create(w.ctypes.data_as(ctypes.c_void_p), w.size, ctypes.byref(h))
    assert rc != 1, lib.hpe_last_error()
