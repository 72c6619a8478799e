"""The C++ mirror as a template drop-in: examples/robot_concept.cpp is written
against the reference's Robot concept -- validate_motion<Robot, 8, Robot::resolution>(start, goal,
env), Robot::fkcc<8>(env, block), sphere_fk<8>, scale_/descale_configuration[_block], eefk,
RRTC<Robot, 8, res>::solve -- and instantiated on vamp_gpu::robots::Panda_0_0 with a host-only
environment (CPU rake, no GPU).  Its results must equal the oracle's."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

F = np.float32


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    from vamp_amd import _lib
    _lib.load()
    out = str(tmp_path_factory.mktemp("concept") / "robot_concept")
    lib_dir = os.path.join(ROOT, "mr-vamp_amd", "vamp_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "examples", "robot_concept.cpp"), "-L", lib_dir, "-lvampgpu",
                           "-Wl,-rpath," + lib_dir, "-o", out])
    return out


def test_reference_shaped_templates_match_oracle(exe, oracle, tmp_path):
    rng = np.random.default_rng(17)
    env = oracle.sphere_cage_env()
    pool = oracle.scale(rng.random((4000, 7), dtype=F))
    valid = oracle.fkcc(env, pool)
    s = oracle.scale(rng.random((400, 7), dtype=F))
    g = oracle.scale(rng.random((400, 7), dtype=F))
    g = (s + (g - s) * F(0.15)).astype(F)
    s[:2], g[:2] = pool[valid][:2], pool[valid][2:4]  # edge 0's start and edge 1's goal: the RRTC problem
    np.concatenate([s, g], 1).astype(F).tofile(tmp_path / "e.f32")
    r = subprocess.run([exe, str(tmp_path / "e.f32"), str(tmp_path / "o.txt")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    lines = open(tmp_path / "o.txt").read().splitlines()
    vm = np.array([int(x.split()[0]) for x in lines[:400]], bool)
    fk = np.array([int(x.split()[1]) for x in lines[:400]], bool)
    want, _ = oracle.validate_motions(env, s, g, (0, 0, 0))
    assert np.array_equal(vm, want)
    blocks = np.stack([s[(np.arange(8) + e) % 400] for e in range(400)]).reshape(-1, 7)
    assert np.array_equal(fk, oracle.fkcc(env, blocks, (0, 0, 0), G=8))  # 8 distinct lanes: group semantics
    rt = [float(x) for x in lines[400].split()[1:]]
    assert abs(rt[0] - s[0][0]) < 1e-6 and abs(rt[1] - s[0][0]) < 1e-6
    pose = np.array([float(x) for x in lines[401].split()[1:]], F)
    import vamp_amd
    assert np.allclose(pose, vamp_amd.panda_0_0.eefk_batch(s[:1])[0], atol=1e-7)
    sph = np.array([float(x) for x in lines[402].split()[1:]], F)
    assert np.allclose(sph, oracle.sphere_fk(s[:1], (0, 0, 0))[0][0], atol=1e-7)
    n_path, iters, n_sizes, path_ok, rng_index = (int(x) for x in lines[403].split()[1:])
    res = vamp_amd.panda_0_0.rrtc(s[0], g[1], vamp_amd_env(vamp_amd), vamp_amd.RRTCSettings(range=1.0))
    assert n_path == len(res.path) > 0 and iters == res.iterations and n_sizes == 2
    assert path_ok == 1 and rng_index >= 1


def vamp_amd_env(vamp):
    from test_c_abi import CAGE
    e = vamp.Environment()
    for c in CAGE:
        e.add_sphere(vamp.Sphere(c, 0.2))
    return e
