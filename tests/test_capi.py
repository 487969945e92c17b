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
