"""The drop-in boundary: libvampgpu.so loads and exports exactly what include/vamp_gpu.h
declares (no compute calls -- this runs without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "vamp_gpu.h")
CAGE = [(0.55, 0, 0.25), (0.35, 0.35, 0.25), (0, 0.55, 0.25), (-0.55, 0, 0.25), (-0.35, -0.35, 0.25),
        (0, -0.55, 0.25), (0.35, -0.35, 0.25), (0.35, 0.35, 0.8), (0, 0.55, 0.8), (-0.35, 0.35, 0.8),
        (-0.55, 0, 0.8), (-0.35, -0.35, 0.8), (0, -0.55, 0.8), (0.35, -0.35, 0.8)]


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|float|const char \*|vgpu_ctx \*)\s*\**(vgpu_\w+)\s*\(", txt, re.M)))


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


def test_no_exception_crosses_the_abi():
    """Every multi-statement int entry point of the host runtime is a function-try-block ending in
    VGPU_ABI_CATCH (mr-vamp_amd/csrc/vgpu_abi.hh): a C++ exception inside the library comes back as
    VGPU_ERR_OOM / VGPU_ERR_INTERNAL instead of terminating the caller's process."""
    csrc = os.path.join(ROOT, "mr-vamp_amd", "csrc")
    files = ["vgpu_api.cpp", "vgpu_multi.cpp", "cpu/vcpu.cpp", "cpu/vcpu_roadmap.cpp", "cpu/vcpu_rrtc.cpp"]
    seen = 0
    for f in files:
        lines = open(os.path.join(csrc, f)).read().split("\n")
        for i, l in enumerate(lines):
            if not l.startswith('extern "C" int ') or l.rstrip().endswith(";") or "{" in l:
                continue
            j = i
            while lines[j] not in ("{", "try {"):
                assert not lines[j].rstrip().endswith(";"), (f, i)
                j += 1
            assert lines[j] == "try {", f"{f}:{i + 1}: {l.strip()} is not a function-try-block"
            k = j + 1
            while not lines[k].startswith("}"):
                k += 1
            assert lines[k] == "} VGPU_ABI_CATCH", f"{f}:{k + 1}"
            seen += 1
    assert seen >= 80


def test_errors_without_context(lib):
    # argument validation paths need no device
    assert lib.vgpu_sync(None) == -1
    assert lib.vgpu_ctx_set_stream(None, None) == -1
    assert lib.vgpu_robot_info(99, None, None, None) == -4
    d, r, n = C.c_int32(), C.c_int32(), C.c_int32()
    assert lib.vgpu_robot_info(1, C.byref(d), C.byref(r), C.byref(n)) == 0
    assert (d.value, r.value, n.value) == (7, 32, 59)


def _build_example(out_dir):
    exe = os.path.join(out_dir, "validate_edges")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "examples", "validate_edges.cpp"),
                           "-L", os.path.join(ROOT, "mr-vamp_amd", "vamp_amd"), "-lvampgpu",
                           "-Wl,-rpath," + os.path.join(ROOT, "mr-vamp_amd", "vamp_amd"), "-o", exe])
    return exe


def test_cpp_mirror_compiles_and_links(lib, tmp_path):
    """include/vamp_gpu.hpp (the C++ mirror of vamp::robots / vamp::planning) builds against
    the shipped library with -Wall -Werror."""
    exe = _build_example(str(tmp_path))
    assert os.access(exe, os.X_OK)


@pytest.mark.gpu
def test_cpp_mirror_validate_matches_oracle(lib, tmp_path, oracle):
    """The C++ mirror's planning::validate_motions<Panda_0_0> on the sphere cage equals the
    oracle's validate_motion on the same edges (margin-free: random edges; any disagreement
    here would also show in test_gpu_parity): bit-exact."""
    import numpy as np
    exe = _build_example(str(tmp_path))
    rng = np.random.default_rng(7)
    n = 2000
    s = rng.random((n, 7), dtype=np.float32)
    g = rng.random((n, 7), dtype=np.float32)
    edges = np.concatenate([s, g], axis=1).astype(np.float32)
    src, dst = tmp_path / "e.f32", tmp_path / "o.u8"
    edges.tofile(src)
    r = subprocess.run([exe, str(src), str(dst)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    got = np.fromfile(dst, np.uint8).astype(bool)
    # bit-identical to the Python binding over the same C ABI
    import vamp_amd
    env = vamp_amd.Environment()
    for c in CAGE:
        env.add_sphere(vamp_amd.Sphere(c, 0.2))
    py_ok, _ = vamp_amd.panda_0_0.validate_batch(s, g, env)
    assert np.array_equal(got, np.asarray(py_ok, bool))
    want, _ = oracle.validate_motions(oracle.sphere_cage_env(), s, g)
    assert np.array_equal(got, want)  # same host, same rsqrt table: bit-exact


def test_attachment_host_pose_identity():
    """Attachment.set_ee_pose (attachments.hh:75-122) at the identity end-effector pose and an
    identity relative frame leaves the spheres where they are; a pure translation adds."""
    import numpy as np
    import vamp_amd
    a = vamp_amd.Attachment((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))
    a.add_spheres([vamp_amd.Sphere((0.1, -0.2, 0.3), 0.05), vamp_amd.Sphere((0.0, 0.0, 1.0), 0.01)])
    a.set_ee_pose((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))
    assert np.array_equal(np.float32([s.center for s in a.posed_spheres]), np.float32([s.center for s in a.spheres]))
    a.set_ee_pose((1.0, 2.0, 3.0), (0.0, 0.0, 0.0, 1.0))
    assert np.allclose([s.center for s in a.posed_spheres], [[1.1, 1.8, 3.3], [1.0, 2.0, 4.0]])
    # a quarter turn about z maps x to y
    h = np.float32(np.sqrt(0.5))
    a.set_ee_pose((0.0, 0.0, 0.0), (0.0, 0.0, h, h))
    assert np.allclose(a.posed_spheres[0].center, [0.2, 0.1, 0.3], atol=1e-6)
    assert a.relative_frame == ([0.0, 0.0, 0.0], [0.0, 0.0, 0.0, 1.0])


def test_roadmap_host_functions_errors_and_order():
    """vgpu_prm_neighbor_params / vgpu_roadmap_assemble are host code (no GPU): argument errors
    come back as VGPU_ERR_INVALID_ARG, and the assembly replays pairs in the reference's append
    order (prm.hh:270-275)."""
    import ctypes as C
    import numpy as np
    from vamp_amd import _lib, roadmap
    lib = _lib.load()
    k = np.zeros(4, np.uint32)
    r = np.zeros(4, np.float32)
    assert lib.vgpu_prm_neighbor_params(0, 1.0, 2.0, 4, k.ctypes.data_as(_lib.U32P), r.ctypes.data_as(_lib.F32P)) == -1
    off = np.zeros(4, np.uint64)
    adj = np.zeros(8, np.uint32)
    bad = np.array([[2, 7]], np.uint32)  # neighbour index outside the 3 vertices
    assert lib.vgpu_roadmap_assemble(3, bad.ctypes.data_as(_lib.U32P), 1, off.ctypes.data_as(C.POINTER(C.c_size_t)),
                                     adj.ctypes.data_as(_lib.U32P), None) == -1
    # vertex 2 connects to 0 then 1; vertex 3 to 1: lists 0:[2] 1:[2,3] 2:[0,1] 3:[1]
    o, a, comp = roadmap.assemble(5, np.array([[2, 0], [2, 1], [3, 1]], np.int32))
    assert [a[o[i]:o[i + 1]].tolist() for i in range(5)] == [[2], [2, 3], [0, 1], [1], []]
    assert comp.tolist() == [0, 0, 0, 0, 4]
