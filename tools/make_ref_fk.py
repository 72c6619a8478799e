#!/usr/bin/env python3
"""Fixture source (build container only: needs /root/reference): the reference's generated `sphere_fk` and `eefk`
COMPILED with its release flags (oracle/_ref/fk_probe, built by `make -C oracle ref` from the fk.hh text as it
lies, oracle/extract_fk.sh) on the configurations of the interpreted-DAG fixtures, into
tests/golden/ref_fk_compiled.npz:

  <robot>_q [n][dim], <robot>_xyz [n][n_spheres][3]  (panda: panda_xyz_b000 / panda_xyz_b220, PandaBase<0,0,0> and
  <200,200,0>), <robot>_eefk_q / <robot>_eefk [n][7] (Baxter's eefk is empty in the reference: none)

    python tools/make_ref_fk.py        # (after make -C oracle ref)
"""
import os
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "oracle", "_ref", "fk_probe")
G = os.path.join(ROOT, "tests", "golden")
NS = {"panda": 59, "fetch": 111, "ur5": 36, "baxter": 75}


def probe(args, q, cols):
    with tempfile.TemporaryDirectory() as d:
        qi, qo = os.path.join(d, "q.bin"), os.path.join(d, "o.bin")
        np.ascontiguousarray(q, np.float32).tofile(qi)
        subprocess.check_call([PROBE] + args + [qi, qo])
        return np.fromfile(qo, np.float32).reshape(len(q), *cols)


def main():
    out = {}
    for robot in NS:
        q = np.load(os.path.join(G, f"fk_{robot}.npz"))["q"].astype(np.float32)
        out[f"{robot}_q"] = q
        bases = [(0, 0, 0), (200, 200, 0)] if robot == "panda" else [(0, 0, 0)]
        for b in bases:
            xyz = probe(["sphere_fk", robot, *map(str, b)], q, (NS[robot], 3))
            key = f"{robot}_xyz" + (f"_b{b[0] // 100}{b[1] // 100}{b[2] // 100}" if robot == "panda" else "")
            out[key] = xyz
    e = np.load(os.path.join(G, "eefk.npz"))
    for robot in ("panda", "fetch", "ur5"):
        q = e[f"{robot}_q"].astype(np.float32)
        out[f"{robot}_eefk_q"] = q
        out[f"{robot}_eefk"] = probe(["eefk", robot], q, (7,))
    np.savez_compressed(os.path.join(G, "ref_fk_compiled.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
