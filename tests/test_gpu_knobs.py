"""The staged pipeline's A/B knobs change only how the work is scheduled, never a result:
the lead pass on / off / also for configurations, the heads' compacted list on / off, the children's near sets on / off, every source kind as one round or as rounds, explicit
rounds, and the monolithic kernels give the same validate (set A, set-B-like) and fkcc answers as the
default schedule on the same seeded inputs.  Each setting runs in its own process (the knobs are read
at context creation)."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

SETTINGS = {
    "lead_off": {"VAMP_AMD_LEAD": "0"},
    "head_list_off": {"VAMP_AMD_HEAD_LIST": "0"},
    "near_off": {"VAMP_AMD_NEAR": "0"},
    "lead_configs": {"VAMP_AMD_LEAD": "5"},
    "rounds_per_batch_everywhere": {"VAMP_AMD_ONE_ROUND": "0"},
    "one_round_everywhere": {"VAMP_AMD_ONE_ROUND": "0x1f"},
    "explicit_rounds": {"VAMP_AMD_ROUNDS": "0x8043091f,0x7fbcf6e0"},
    "monolithic": {"VAMP_AMD_STAGED": "0"},
}


def run(tmp_path, name, extra):
    out = str(tmp_path / f"{name}.npz")
    env = dict(os.environ)
    for k in ("VAMP_AMD_LEAD", "VAMP_AMD_HEAD_LIST", "VAMP_AMD_NEAR", "VAMP_AMD_ONE_ROUND", "VAMP_AMD_ROUNDS", "VAMP_AMD_STAGED"):
        env.pop(k, None)
    env.update(extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "knob_probe.py"), out], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict(np.load(out, allow_pickle=False))


@pytest.mark.gpu
def test_knobs_change_no_result(tmp_path):
    base = run(tmp_path, "default", {})
    assert base["okA"].size == 1 << 14 and 0 < base["okB"].mean() < 1
    for name, extra in SETTINGS.items():
        got = run(tmp_path, name, extra)
        print(f"knobs {name}: {extra} -> same results", flush=True)
        for k in base:
            assert np.array_equal(got[k], base[k]), (name, k, int((got[k] != base[k]).sum()))
