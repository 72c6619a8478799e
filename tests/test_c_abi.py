"""The drop-in boundary: libvampgpu.so loads and exports exactly what include/vamp_gpu.h
declares (no compute calls -- this runs without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "vamp_gpu.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*\**(vgpu_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    from vamp_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "mr-vamp_amd")])
    return _lib.load()


def test_header_declares_api():
    names = declared()
    assert "vgpu_validate_motions" in names and "vgpu_fkcc" in names and "vgpu_sphere_fk" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol(lib):
    for name in declared():
        assert hasattr(lib, name), name


def test_python_binding_covers_header():
    from vamp_amd import _lib
    assert sorted(_lib.SIGNATURES) == declared()


def test_exports_are_c_abi():
    from vamp_amd import _lib
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for name in declared():
        assert name in exported, f"{name} not exported unmangled"


def test_errors_without_context(lib):
    # argument validation paths need no device
    assert lib.vgpu_sync(None) == -1
    assert lib.vgpu_ctx_set_stream(None, None) == -1
    assert lib.vgpu_robot_info(99, None, None, None) == -4
    d, r, n = C.c_int32(), C.c_int32(), C.c_int32()
    assert lib.vgpu_robot_info(1, C.byref(d), C.byref(r), C.byref(n)) == 0
    assert (d.value, r.value, n.value) == (7, 32, 59)
