import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "mr-vamp_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def golden(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


ALT = os.path.join(GOLD, "alt_rsqrt")


def host_fixture(name, oracle):
    """A reference-DAG fixture as evaluated under THIS host's rsqrt cull: the primary file (made on
    the build container's host) or, when this host's _mm256_rsqrt_ps table differs, the primary
    inputs overlaid with tests/golden/alt_rsqrt/<name> -- the same inputs evaluated under that
    host's table (tools/make_golden.py --lut; the GPU box's EPYC 9575F is one).  Returns a dict with
    the rsqrt_lut/rsqrt_kbits it was made with (fixtures without them take fkcc_panda_cage's)."""
    fx = dict(golden(name))
    if "rsqrt_lut" not in fx:
        ref = golden("fkcc_panda_cage.npz")
        fx["rsqrt_lut"], fx["rsqrt_kbits"] = ref["rsqrt_lut"], ref["rsqrt_kbits"]
    lut, kb = oracle.rsqrt_probe()
    if kb == int(fx["rsqrt_kbits"]) and np.array_equal(lut, fx["rsqrt_lut"]):
        return fx
    alt = os.path.join(ALT, name)
    if os.path.exists(alt):
        z = np.load(alt, allow_pickle=False)
        if kb == int(z["rsqrt_kbits"]) and np.array_equal(lut, z["rsqrt_lut"]):
            fx.update({k: z[k] for k in z.files})
    return fx


# Reference-fixture coverage records (tests/test_oracle.py:fixture_check): how much of each
# reference-DAG fixture the margin filter keeps on THIS host and how many results flip outside
# it.  Printed at the end of every session so the GPU box's log carries the numbers.
COVERAGE = []


def pytest_terminal_summary(terminalreporter):
    if not COVERAGE:
        return
    terminalreporter.section("reference-fixture coverage on this host")
    for rec in COVERAGE:
        terminalreporter.write_line(
            f"{rec['name']}: compared {rec['kept']}/{rec['total']} (coverage {rec['coverage']:.4f}, "
            f"cull filter {'off' if rec['same_rsqrt'] else 'on'}), flips inside {rec['flips_kept']}, "
            f"flips outside {rec['flips_dropped']}")
    path = os.environ.get("VGPU_COVERAGE_JSON")
    if path:
        import json
        with open(path, "w") as f:
            json.dump(COVERAGE, f, indent=1)


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    oracle_py.build()
    return oracle_py


# Debug builds (make -C mr-vamp_amd DEBUG=1, selected with VAMP_AMD_LIB=.../libvampgpu_debug.so): after
# every GPU test, the bounds-check counters of the default context and of every live environment copy
# must be zero (vgpu_debug_violations; SURVEY §5 "race detection / sanitizers").
DEBUG_CHECKED = []


@pytest.fixture(autouse=True)
def _debug_bounds(request):
    yield
    if "gpu" not in request.keywords:
        return
    import ctypes as C
    try:
        from vamp_amd._lib import load
        lib = load()
        if not lib.vgpu_debug_build():
            return
        import vamp_amd
    except Exception:
        return
    ctx = vamp_amd.context(0)
    out = (C.c_uint32 * 2)()
    found = []
    assert lib.vgpu_debug_violations(ctx.h, None, out) == 0
    if out[0]:
        found.append(("context", out[0], out[1]))
    for env in list(vamp_amd._ENVS):
        for key, h in list(env._handles.items()):
            if key != ctx.h.value:  # copies on other (possibly closed) contexts are skipped
                continue
            assert lib.vgpu_debug_violations(C.c_void_p(key), h, out) == 0
            if out[0]:
                found.append(("environment", out[0], out[1]))
    DEBUG_CHECKED.append(request.node.nodeid)
    assert not found, f"debug bounds violations (where, count, first site): {found}"
