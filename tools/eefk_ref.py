"""Evaluate the reference's generated eefk (robots/<robot>/fk.hh `inline auto eefk(...)`) in IEEE
double, as the reference computes it (its temporaries are `auto` of float * double literals, so
double, with std::sin / std::cos), narrowed to float32 at the return -- a fixture source for
tests/test_eefk.py (build container only: reads /root/reference)."""
import math
import re

import numpy as np


def eefk_body(robot, ref_root="/root/reference"):
    src = open(f"{ref_root}/src/impl/vamp/robots/{robot}/fk.hh").read()
    m = re.search(r"inline auto eefk\(const std::array<float, (\d+)> &q\) noexcept -> std::array<float, 7>\s*\{", src)
    if not m:
        raise ValueError(f"no eefk in {robot}/fk.hh")
    i, depth = m.end(), 1
    j = i
    while depth:
        depth += {"{": 1, "}": -1}.get(src[j], 0)
        j += 1
    body = src[i:j - 1]
    stmts = re.findall(r"auto (\w+) = ([^;]+);", body)
    ret = re.search(r"return \{([^}]*)\};", body)
    if not stmts or not ret:
        raise ValueError(f"{robot}: eefk has no body (e.g. Baxter's is empty)")
    return int(m.group(1)), stmts, [x.strip() for x in ret.group(1).split(",")]


def make_eval(robot):
    dim, stmts, ret = eefk_body(robot)
    lines = ["def f(q):"]
    for name, expr in stmts:
        expr = expr.replace("std::sin", "math.sin").replace("std::cos", "math.cos")
        expr = re.sub(r"q\[(\d+)\]", r"float(q[\1])", expr)
        lines.append(f"    {name} = {expr}")
    lines.append(f"    return [{', '.join(ret)}]")
    ns = {"math": math}
    exec("\n".join(lines), ns)  # the reference's own expression DAG, evaluated in Python float (double)
    f = ns["f"]

    def run(Q):
        return np.array([f(q) for q in np.asarray(Q, np.float32)], np.float64).astype(np.float32)

    return dim, run
