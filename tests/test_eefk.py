"""Robot::eefk (panda/fk.hh:11399-11650, fetch/fk.hh:30993, ur5/fk.hh:5868; bound as
vamp.<robot>.eefk, bindings/common.hh:342-352) on the CPU: equal to the reference's generated eefk
evaluated in double (tools/eefk_ref.py -> tests/golden/eefk.npz).  Tolerance: the north_star FK
tolerance, 1e-5 absolute; observed bit-identical."""
import numpy as np
import pytest

from conftest import golden

FK_TOL = 1e-5


@pytest.fixture(scope="module")
def vamp():
    import vamp_amd
    return vamp_amd


@pytest.mark.parametrize("robot", ["panda", "fetch", "ur5"])
def test_eefk_vs_reference(vamp, robot):
    fx = golden("eefk.npz")
    rob = vamp.panda_0_0 if robot == "panda" else getattr(vamp, robot)
    got = rob.eefk_batch(fx[f"{robot}_q"])
    assert np.abs(got - fx[f"{robot}_pose"]).max() <= FK_TOL
    assert np.array_equal(got, fx[f"{robot}_pose"])  # observed: bit-identical
    pos, quat = rob.eefk(fx[f"{robot}_q"][0])
    assert np.array_equal(np.concatenate([pos, quat]), got[0])
    assert np.allclose(np.linalg.norm(got[:, 3:], axis=1), 1.0, atol=1e-5)


def test_eefk_base_independent_and_unsupported(vamp):
    from vamp_amd import VgpuError
    q = golden("eefk.npz")["panda_q"][:16]
    assert np.array_equal(vamp.panda.eefk_batch(q), vamp.panda_0_0.eefk_batch(q))  # panda::eefk takes no base
    with pytest.raises(VgpuError):
        vamp.baxter.eefk_batch(np.zeros((1, 14), np.float32))
    with pytest.raises(VgpuError):
        vamp.panda_pair.eefk_batch(np.zeros((1, 14), np.float32))
