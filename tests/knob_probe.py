"""Helper of tests/test_gpu_knobs.py (run as a subprocess, so each A/B knob is read at context creation):
validates the same seeded set-A and set-B cage edges and fkcc configurations, and writes the results to
the .npz path given."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(out):
    import vamp_amd
    from test_c_abi import CAGE
    rng = np.random.default_rng(11)
    env = vamp_amd.Environment()
    for c in CAGE:
        env.add_sphere(vamp_amd.Sphere(c, 0.2))
    robot = vamp_amd.panda_0_0
    n = 1 << 14
    # set A: raw pairs of uniform configurations; set B-like: short edges around valid-ish starts
    sa = rng.random((n, 7), dtype=np.float32)
    ga = rng.random((n, 7), dtype=np.float32)
    sb = rng.random((n, 7), dtype=np.float32)
    gb = np.clip(sb + rng.normal(0, 0.05, (n, 7)).astype(np.float32), 0, 1).astype(np.float32)
    res = {}
    for tag, s, g in (("A", sa, ga), ("B", sb, gb)):
        ok, nb = robot.validate_batch(s, g, env)
        res["ok" + tag] = np.asarray(ok, bool)
    res["fkcc"] = np.asarray(robot.fkcc_batch(sa, env), bool) if hasattr(robot, "fkcc_batch") else np.zeros(0, bool)
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1])
