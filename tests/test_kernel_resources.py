"""Register budgets of the hot staged kernels, read from the built library's gfx950 code objects (CPU test).

A kernel whose VGPR budget (its __launch_bounds__ waves/EU) is below what its code needs spills to scratch:
per-lane private memory that costs HBM traffic and latency on every spill and reload (GB of
scratch writes per call in the Fetch and composite kernels).  This test reads each kernel's
.private_segment_fixed_size and .vgpr_spill_count from the AMDGPU metadata note of the shipped
libvampgpu.so (tools/kernel_resources.py: clang offload bundles -> llvm-readelf --notes) and fails when a
listed hot kernel has either non-zero.  The list covers the staged pipelines the bench workloads run
(vgpu_staged.hh bound / lead / children kernels): the Panda (configs[1], [2]), the Fetch (configs[3]), the
two-Panda composite's arm and inter-arm passes (configs[4]) and the point-cloud (EXT) Panda kernels of the
CAPT workload (configs[2]).
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

LIB = os.path.join(ROOT, "mr-vamp_amd", "vamp_amd", "libvampgpu.so")


def staged(robot, ext, lead=False):
    """regexes of a robot's staged bound / children (/ lead) kernels (vgpu_staged.hh); robot is a regex over the
    robot type's name, ext = the point-cloud instantiations"""
    R = robot
    e = "true" if ext else "false"
    src = rf"vgpu::Src(?:\w+)<{R} ?>"
    return [rf"vgpu::bound_kernel<{R}, {src}, {e}>", rf"vgpu::children_kernel<{R}, {src}, {e}, \d>"] + \
        ([rf"vgpu::lead_kernel<{R}, {src} ?>"] if lead else [])


# (description, regexes over the demangled kernel names); every match must have 0 scratch and 0 VGPR spills.
# Not listed: the Fetch's point-cloud children kernels (no bench workload runs them), where 2-5 VGPRs (8-16 B
# per lane) still spill in four kernels even at 128-168 VGPRs (vgpu_fetch_staged.hip kExtClassWaves)
HOT = [
    ("Panda staged, primitive environments (configs[1])", staged(r"vgpu::PandaR", False, lead=True)),
    ("Panda staged, point clouds (CAPT, configs[2])", staged(r"vgpu::PandaR", True)),
    ("Fetch staged, primitive environments (configs[3])", staged(r"vgpu::FetchR", False)),
    ("composite arm passes (configs[4])", staged(r"vgpu::PairArmR<\d>", False) + staged(r"vgpu::PairArmR<\d>", True)),
    ("composite inter-arm passes (configs[4])", staged(r"vgpu::PairInterR<\d>", False) + staged(r"vgpu::PairInterR<\d>", True)),
]


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("libvampgpu.so not built (make -C mr-vamp_amd)")
    import kernel_resources
    return kernel_resources.kernels(LIB)


def test_library_has_kernel_metadata(kernels):
    ours = [k for k in kernels if "vgpu::" in k["name"].split("(")[0]]
    assert len(ours) > 100
    assert all(k["vgpr"] > 0 for k in ours)


@pytest.mark.parametrize("desc,patterns", HOT, ids=[h[0] for h in HOT])
def test_hot_kernels_do_not_spill(kernels, desc, patterns):
    hit = []
    for pattern in patterns:
        rx = re.compile(pattern)
        got = [k for k in kernels if rx.search(k["name"])]
        assert got, f"no kernel matches {pattern}"
        hit += got
    bad = [(k["name"][:120], k["vgpr"], k["vgpr_spill"], k["scratch"]) for k in hit
           if k["scratch"] or k["vgpr_spill"]]
    assert not bad, f"{desc}: kernels with scratch / VGPR spills: {bad}"
