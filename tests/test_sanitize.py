"""ASan/UBSan build of the CPU restatement (VERDICT r01 "missing: the ASan/UBSan build").

`make -C oracle sanitize` compiles oracle/vamp_oracle.c and the product's host-only CAPT build
(mr-vamp_amd/csrc/vgpu_capt.cpp) with -fsanitize=address,undefined -fno-sanitize-recover=all and
links oracle/sanitize_main.cc, which drives every oracle entry-point family on small seeded inputs
(all robots' FK / fkcc / validate incl. attachments, zero-length and long edges, the composite, CAPT
build + queries cross-checked against the host build, Halton, the PRM neighbour query, the
point-cloud filter with and without culling).  Any sanitizer report aborts with a non-zero exit.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="no host compiler")
def test_oracle_and_capt_build_under_asan_ubsan():
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True, text=True)
    assert b.returncode == 0, b.stdout + b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_build", "sanitize_check")], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize_check: ok" in r.stdout
