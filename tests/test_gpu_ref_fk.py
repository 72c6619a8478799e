"""GPU sphere_fk (the HBM-bound FK output kernel and the FK inside every collision kernel, bit-identical to the
oracle -- tests/test_gpu_parity.py) against the reference's sphere_fk COMPILED with its release flags
(tests/golden/ref_fk_compiled.npz, tests/test_ref_fk.py): within 1e-6 m on every centre of every robot, 10x inside
north_star's 1e-5 (the release build's reassociations are not reproducible op for op)."""
import numpy as np
import pytest

from conftest import golden
from test_ref_fk import FK_TOL, OBSERVED_TOL, report

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("robot,key", [("panda_0_0", "panda_xyz_b000"), ("panda", "panda_xyz_b220"),
                                       ("fetch", "fetch_xyz"), ("ur5", "ur5_xyz"), ("baxter", "baxter_xyz")])
def test_gpu_sphere_fk_vs_compiled_reference(robot, key):
    import vamp_amd as vamp
    assert vamp.context(0) is not None
    ref = golden("ref_fk_compiled.npz")
    q = ref[key.split("_")[0] + "_q"]
    got = getattr(vamp, robot).sphere_fk_batch(q)
    d = report(f"GPU {key}", got, ref[key])
    assert d <= FK_TOL and d <= OBSERVED_TOL
