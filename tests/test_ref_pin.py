"""The C restatement (oracle/) against outputs of the reference's own code.

tests/golden/ref_pins.npz was produced by oracle/_ref/ref_probe, compiled from the
reference's vector layer and random/halton.hh with the reference release flags
(tools/make_golden.py).  These are the bit-level semantics every other layer inherits.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import golden

F = np.float32


@pytest.fixture(scope="module")
def pins():
    return golden("ref_pins.npz")


def test_sincos_bit_exact(oracle, pins):
    """FloatVector::sin()/cos() of q*0.5 (vector/interface.hh:438-469, fk.hh:182-185)."""
    L = oracle.lib()
    q = pins["sincos_q"]
    h = (q * F(0.5)).astype(F)
    s = np.array([L.vo_sin(float(x)) for x in h], F)
    c = np.array([L.vo_cos(float(x)) for x in h], F)
    assert (s.view(np.uint32) == pins["sin"].view(np.uint32)).all()
    assert (c.view(np.uint32) == pins["cos"].view(np.uint32)).all()


def test_extent_bit_exact(oracle, pins):
    """max_extent = v*rsqrt(v) + r with dot_3 contracted (validity.hh:55-59).  The value
    depends on the host CPU's rsqrt table, so this pin holds where the table matches the
    one recorded with the fixture (any Intel host); elsewhere the table-emulated path is
    checked against this host's native rsqrt instead (test_rsqrt_table_emulation)."""
    lut, kb = oracle.rsqrt_probe()
    if kb != int(pins["rsqrt_kbits"]) or not np.array_equal(lut, pins["rsqrt_lut"]):
        pytest.skip("host rsqrt table differs from the fixture host's (non-Intel CPU)")
    L = oracle.lib()
    x = pins["extent_in"]
    me = np.array([L.vo_max_extent(*map(float, row)) for row in x], F)
    ref = pins["extent"]
    both_nan = np.isnan(me) & np.isnan(ref)
    assert (both_nan | (me.view(np.uint32) == ref.view(np.uint32))).all()
    assert np.isnan(ref[:8]).all() and np.signbit(ref[:8]).all()  # 0*rsqrt(0): sign-set NaN, no cull


def test_rsqrt_table_emulation(oracle):
    """The (parity, top-K mantissa) table + exponent shift reproduces this host's
    _mm_rsqrt_ss; that emulation is what the GPU kernels run."""
    lut, kb = oracle.rsqrt_probe()
    L = oracle.lib()
    rng = np.random.default_rng(7)
    v = np.concatenate([rng.uniform(1e-6, 10.0, 20000), rng.uniform(0, 3.0, 20000), [0.0, 1e-40, 1.0, 4.0]]).astype(F)
    lp = lut.ctypes.data_as(C.POINTER(C.c_uint32))
    emu = np.array([L.vo_sqrt_lut(float(x), lp, kb) for x in v], F)
    nat = np.array([F(x) * F(L.vo_rsqrt_native(float(x))) for x in v], F)
    ok = (emu.view(np.uint32) == nat.view(np.uint32)) | (np.isnan(emu) & np.isnan(nat))
    assert ok.all()


def test_rake_bit_exact(oracle, pins):
    """validate_motion's distance, n, first block and back-steps (validate.hh:31-56)."""
    s, g, out = pins["rake_starts"], pins["rake_goals"], pins["rake_out"]
    NB = int(pins["rake_blocks"])
    L = oracle.lib()
    for e in range(s.shape[0]):
        v = (g[e] - s[e]).astype(F)
        d = F(L.vo_l2_norm7(v.ctypes.data_as(C.POINTER(C.c_float))))
        assert d.view(np.uint32) == out[e, 0].view(np.uint32)
        n = max(np.ceil(F(d / F(8) * F(32))), F(1))
        assert n == out[e, 1]
        pct = (np.arange(1, 9, dtype=F) / F(8)).astype(F)
        # fma(v, pct, s): exact product in float64, one rounding (validate.hh:37 as compiled)
        blk = ((v[:, None].astype(np.float64) * pct[None, :].astype(np.float64)) + s[e][:, None]).astype(F)
        back = (v / F(8 * int(n))).astype(F)
        for b in range(min(NB, int(n))):
            if b:
                blk = (blk - back[:, None]).astype(F)
            ref = out[e, 2 + b * 56: 2 + (b + 1) * 56].reshape(7, 8)
            assert (blk.view(np.uint32) == ref.view(np.uint32)).all(), (e, b)


def test_halton_bit_exact(oracle, pins):
    """rng::Halton<7>/<8>::next() (random/halton.hh:73-104) incl. the 1e6-draw base rotation."""
    for dim in (7, 8):
        ks = pins[f"halton{dim}_k"]
        ref = pins[f"halton{dim}"]
        got = oracle.halton(dim, ks)
        assert (got.view(np.uint32) == ref.view(np.uint32)).all(), dim


# ---- point-cloud (CAPT) and heightfield expression pins (tests/golden/ref_pins_ext.npz) ----
@pytest.fixture(scope="module")
def ext():
    return golden("ref_pins_ext.npz")


def _f3(a):
    a = np.ascontiguousarray(a, F)
    return a.ctypes.data_as(C.POINTER(C.c_float)), a


def test_sql2_bit_exact(oracle, ext):
    """collision::sql2_3 on FloatVector (math.hh:29-42), compiled from the reference header:
    the CAPT affordance distance (capt.hh:528-534)."""
    L = oracle.lib()
    x = ext["sql2_in"]
    got = np.array([L.vo_sql2_3(*map(float, row)) for row in x], F)
    assert (got.view(np.uint32) == ext["sql2"].view(np.uint32)).all()


def test_capt_box_forms_bit_exact(oracle, ext):
    """collides_simd leaf-box distance (capt.hh:505-521) and Volume::distsq_to /
    contained_by_internal_ball (capt.hh:70-86) as the reference release build evaluates them."""
    L = oracle.lib()
    x = ext["box_in"]
    vec, dist, ball = [], [], []
    for row in x:
        c, _a = _f3(row[0:3])
        lo, _b = _f3(row[3:6])
        up, _c = _f3(row[6:9])
        vec.append(L.vo_capt_box_vec(c, lo, up))
        dist.append(L.vo_capt_vol_distsq(c, lo, up))
        ball.append(L.vo_capt_vol_ball(c, lo, up))
    for got, key in ((vec, "box_vec"), (dist, "vol_distsq"), (ball, "vol_ball")):
        got = np.array(got, F)
        ref = ext[key]
        assert ((got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))).all(), key
    rr = (x[:, 9] + x[:, 10]).astype(F)
    assert ((rr * rr).astype(F) == ext["box_rc"]).all()


def test_heightfield_bit_exact(oracle, ext):
    """sphere_heightfield (sphere_heightfield.hh:9-30): every in-range query bit-exact; the
    out-of-range ones (a gather past the data in the reference) are flagged, not compared."""
    L = oracle.lib()
    h = ext["hf_hdr"]
    data = np.ascontiguousarray(ext["hf_data"], F)
    hf = oracle.VoHeightfield(*map(float, h[:6]), int(h[6]), int(h[7]), data.ctypes.data_as(C.POINTER(C.c_float)))
    q, ref = ext["hf_q"], ext["hf"]
    oob = C.c_int(0)
    n_in = 0
    for row, want in zip(q, ref):
        v = F(L.vo_sphere_heightfield(C.byref(hf), *map(float, row), C.byref(oob)))
        if oob.value:
            continue
        n_in += 1
        assert v.view(np.uint32) == want.view(np.uint32)
    assert n_in > 0.9 * len(q)


def test_scale_configuration_bit_exact(oracle, ext):
    """Robot::scale_configuration q * s_m + s_a (robots/panda/fk.hh:34-37) compiles to one fma
    per joint; the Halton -> configuration step of the sampling path."""
    got = oracle.scale(ext["scale_u"])
    assert np.array_equal(got.view(np.uint32), ext["scale_q"].view(np.uint32))


def test_sql2_scalar_bit_exact(oracle):
    """filter_robot_from_pointcloud's robot-sphere test (bindings/common.hh:71-72): the scalar float
    sphere_sphere_sql2 as the reference's release build contracts it -- fma(xs, xs, ys*ys) +
    fma(zs, zs, -(rs*rs)) -- on 65536 inputs, half of them within 1e-6 of contact
    (tests/golden/ref_pins_sql2s.npz, tools/make_golden.py --sql2s)."""
    z = golden("ref_pins_sql2s.npz")
    L = oracle.lib()
    L.vo_sql2_scalar.restype = C.c_float
    L.vo_sql2_scalar.argtypes = [C.c_float] * 8
    got = np.array([L.vo_sql2_scalar(*map(float, row)) for row in z["sql2s_in"]], F)
    assert (got.view(np.uint32) == z["sql2s"].view(np.uint32)).all()
    assert 0.2 < np.signbit(z["sql2s"]).mean() < 0.8
