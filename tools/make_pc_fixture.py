#!/usr/bin/env python3
"""Fixture for the MotionBenchMaker point-cloud harness tests: the problem dict of
table_pick_panda scene0001 (resources/panda/problems.tar.bz2, parsed with yaml.safe_load;
data only) -> tests/golden/mbm_table_pick_panda_0001.json.  Needs /root/reference (this
container only); the tests read the committed JSON.

    python tools/make_pc_fixture.py
"""
import json
import os
import sys
import tarfile

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mr-vamp_amd"))
from vamp_amd.pointcloud import scene_to_problem_dict  # noqa: E402


def main():
    with tarfile.open("/root/reference/resources/panda/problems.tar.bz2") as t:
        scene = yaml.safe_load(t.extractfile("problems/table_pick_panda/scene0001.yaml").read().decode())
    d = scene_to_problem_dict(scene, "table_pick")
    out = os.path.join(ROOT, "tests", "golden", "mbm_table_pick_panda_0001.json")
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(out, len(d["box"]), "boxes", len(d["cylinder"]), "cylinders")


if __name__ == "__main__":
    main()
