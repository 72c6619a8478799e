// ref_probe.cc -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Drives the parts of the reference that compile in this container WITHOUT any
// stand-in headers: the AVX2 vector layer (/root/reference/src/impl/vamp/vector.hh
// and vector/{interface,avx,utils}.hh) and the Halton sampler
// (/root/reference/src/impl/vamp/random/halton.hh).  Everything else on the hot
// path (shapes.hh, validity.hh, robots/*/fk.hh, validate.hh) includes <Eigen/...>
// or <pdqsort.h>, which this image does not have, so it is NOT built here (see
// DESIGN.md "Oracle and parity").
//
// Built by oracle/Makefile with the reference's own release flags
// (cmake/CompilerSettings.cmake:3,12-15,27) into oracle/_ref/ref_probe.
// The outputs pin the bit-level semantics that the C restatement
// (oracle/vamp_oracle.c) and the HIP kernels must reproduce:
//   * FloatVector::sin()/cos() polynomial approximations  (vector/interface.hh:438-469)
//   * collision::sqrt == v * rsqrt(v)                      (vector/avx.hh:411-415, collision/math.hh:55-59)
//   * l2_norm / hsum lane order                             (vector/interface.hh:402-410, avx.hh:441-452)
//   * the validate_vector rake arithmetic                   (planning/validate.hh:31-56; the two loops
//     are restated below with the reference's own FloatVector types because
//     validate.hh itself includes environment.hh -> Eigen)
//   * rng::Halton<dim>::next                                (random/halton.hh:73-104)
//   * collision::sql2_3 on FloatVector (collision/math.hh:29-42), the CAPT affordance test, and the
//     scalar sphere_sphere_sql2 of filter_robot_from_pointcloud (bindings/common.hh:71-72)
//   * expression probes for code whose header cannot be compiled here (capt.hh needs
//     <pdqsort.h>, sphere_heightfield.hh needs shapes.hh -> Eigen): the CAPT leaf-box test
//     (capt.hh:505-521), Volume::distsq_to / contained_by_internal_ball (capt.hh:70-89) and
//     sphere_heightfield (sphere_heightfield.hh:9-30) are restated below with the reference's
//     own FloatVector/IntVector types and compiled with its flags, so the contraction and
//     association the release compiler picks for those expression shapes is observed.
//
// Usage: ref_probe <mode> <in.bin> <out.bin> [args]   (raw little-endian float32)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>

#include <vamp/vector.hh>
#include <vamp/random/halton.hh>
#include <vamp/collision/math.hh>   // <algorithm>/<cmath> only: compiled as is

using namespace vamp;

static std::vector<float> read_f32(const char *path)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    std::fseek(f, 0, SEEK_END);
    long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<float> v(sz / 4);
    if (std::fread(v.data(), 4, v.size(), f) != v.size()) { std::exit(2); }
    std::fclose(f);
    return v;
}

static void write_f32(const char *path, const std::vector<float> &v)
{
    FILE *f = std::fopen(path, "wb");
    if (!f) { std::perror(path); std::exit(2); }
    std::fwrite(v.data(), 4, v.size(), f);
    std::fclose(f);
}

// Opaque barrier so each probe sees the same "value loaded from memory" context
// the generated FK code has (INPUT_k = q[k]; DIV = INPUT * 0.5; .sin()).
template <typename T>
__attribute__((noinline)) static T launder(T v) { asm volatile("" : "+m"(v)); return v; }

// sin/cos of q*0.5, exactly the expression shape of robots/panda/fk.hh:182-185
__attribute__((noinline)) static void probe_sincos(const float *q, float *s, float *c)
{
    FloatVector<8> in(q);
    auto half = in * 0.5;
    auto sv = half.sin();
    auto cv = half.cos();
    sv.to_array(s);
    cv.to_array(c);
}

// max_extent of validity.hh:55-59 (sqrt(dot_3(s,s)) + r, r a scalar broadcast)
__attribute__((noinline)) static void
probe_extent(const float *x, const float *y, const float *z, float r, float *ext, float *root)
{
    FloatVector<8> sx(x), sy(y), sz(z);
    FloatVector<8> sr(r);
    auto d3 = (sx * sx) + (sy * sy) + (sz * sz);   // collision/math.hh:17-27 dot_3
    auto rt = d3.sqrt();                           // collision/math.hh:55-59 -> avx.hh:411-415
    auto me = rt + sr;
    me.to_array(ext);
    rt.to_array(root);
}

// collision::sql2_3 with a broadcast centre (capt.hh:528-534 affordance scan)
__attribute__((noinline)) static void
probe_sql2(const float *ax, const float *ay, const float *az, float bx, float by, float bz, float *out)
{
    FloatVector<8> X(ax), Y(ay), Z(az);
    const auto xc = FloatVector<8>::fill(bx), yc = FloatVector<8>::fill(by), zc = FloatVector<8>::fill(bz);
    collision::sql2_3(X, Y, Z, xc, yc, zc).to_array(out);
}

// leaf-box distance of collides_simd (capt.hh:505-521): c - clamp(c, lo, up), summed squares,
// and rc_sq = (r + r_point)^2
__attribute__((noinline)) static void probe_capt_box(const float *c, const float *lo, const float *up,
                                                     const float *r, float rp, float *out, float *rc)
{
    FloatVector<8> c0(c), c1(c + 8), c2(c + 16), rr(r);
    FloatVector<8> l0(lo), l1(lo + 8), l2(lo + 16), u0(up), u1(up + 8), u2(up + 16);
    auto d0 = c0 - c0.clamp(l0, u0);
    auto d1 = c1 - c1.clamp(l1, u1);
    auto d2 = c2 - c2.clamp(l2, u2);
    auto dist = d0 * d0 + d1 * d1 + d2 * d2;
    rr = rr + rp;
    auto rcs = rr * rr;
    dist.to_array(out);
    rcs.to_array(rc);
}

// Volume::distsq_to (capt.hh:79-86) and contained_by_internal_ball's sum (capt.hh:70-77), scalar
__attribute__((noinline)) static float probe_vol_distsq(const float *p, const float *lo, const float *up)
{
    const float d0 = p[0] - std::clamp(p[0], lo[0], up[0]);
    const float d1 = p[1] - std::clamp(p[1], lo[1], up[1]);
    const float d2 = p[2] - std::clamp(p[2], lo[2], up[2]);
    return d0 * d0 + d1 * d1 + d2 * d2;
}
__attribute__((noinline)) static float probe_vol_ball(const float *p, const float *lo, const float *up)
{
    const float d0 = std::max(p[0] - lo[0], up[0] - p[0]);
    const float d1 = std::max(p[1] - lo[1], up[1] - p[1]);
    const float d2 = std::max(p[2] - lo[2], up[2] - p[2]);
    return d0 * d0 + d1 * d1 + d2 * d2;
}

// sphere_heightfield (sphere_heightfield.hh:9-30); hf = {x, y, z, xs, ys, zs, xd, yd}
__attribute__((noinline)) static void probe_hf(const float *x, const float *y, const float *z, float r,
                                               const float *hf, const float *data, float *out)
{
    using IndexT = IntVector<8>;
    const std::size_t xd = (std::size_t)hf[6], yd = (std::size_t)hf[7];
    const std::size_t xd2 = xd / 2, yd2 = yd / 2;
    FloatVector<8> X(x), Y(y), Z(z), R(r);
    FloatVector<8> hx(hf[0]), hy(hf[1]), hz(hf[2]), hxs(hf[3]), hys(hf[4]), hzs(hf[5]);
    auto xo = hx - X;
    auto yo = hy - Y;
    auto xs = (hxs * xo + xd2).clamp(0.F, static_cast<float>(xd)).floor();
    auto ys = (hys * yo + yd2).clamp(0.F, static_cast<float>(yd)).floor();
    auto index = ys * xd + xs;
    IndexT indices = index.template to<IndexT>();
    auto zh = FloatVector<8>::gather(data, indices);
    auto zhs = hzs * zh + hz;
    (Z - R - zhs).to_array(out);
}

// filter_robot_from_pointcloud's sphere test (bindings/common.hh:71-72): scalar float
// collision::sphere_sphere_sql2 = sql2_3<float>(a, b) - (ar + br)^2 (sphere_sphere.hh:20-22; that
// header includes shapes.hh -> Eigen, so its two lines are restated over the reference's own sql2_3)
__attribute__((noinline)) static float probe_sql2_scalar(const float *a, const float *b)
{
    auto sum = collision::sql2_3(a[0], a[1], a[2], b[0], b[1], b[2]);
    auto rs = a[3] + b[3];
    return sum - rs * rs;
}

// Robot::scale_configuration shape (robots/panda/fk.hh:34-37): q * s_m + s_a on FloatVector<7>
// with the Panda constants restated from fk.hh:14-30 (fk.hh itself needs Eigen via its includes)
__attribute__((noinline)) static void probe_scale(const float *q, float *out)
{
    alignas(32) static const std::array<float, 7> sm{5.9342f, 3.6652f, 5.9342f, 3.2289f, 5.9342f, 3.9096f, 5.9342f};
    alignas(32) static const std::array<float, 7> sa{-2.9671f, -1.8326f, -2.9671f, -3.1416f, -2.9671f, -0.0873f,
                                                      -2.9671f};
    const FloatVector<7> s_m(sm), s_a(sa);
    alignas(32) float buf[8] = {0};
    std::memcpy(buf, q, 28);
    FloatVector<7> v(buf);
    v = v * s_m + s_a;
    v.to_array(buf);
    std::memcpy(out, buf, 28);
}

int main(int argc, char **argv)
{
    if (argc < 4) { std::fprintf(stderr, "usage: ref_probe mode in out [args]\n"); return 2; }
    const std::string mode = argv[1];

    if (mode == "sincos")
    {
        // in: N q values (N multiple of 8). out: N sin(q/2) then N cos(q/2)
        auto q = read_f32(argv[2]);
        const size_t n = q.size();
        std::vector<float> out(2 * n);
        alignas(32) float s[8], c[8], qq[8];
        for (size_t i = 0; i < n; i += 8)
        {
            std::memcpy(qq, &q[i], 32);
            probe_sincos(launder(qq), s, c);
            std::memcpy(&out[i], s, 32);
            std::memcpy(&out[n + i], c, 32);
        }
        write_f32(argv[3], out);
    }
    else if (mode == "extent")
    {
        // in: N x 4 (x,y,z,r) with r constant per group of 8. out: N ext, N root
        auto in = read_f32(argv[2]);
        const size_t n = in.size() / 4;
        std::vector<float> out(2 * n);
        alignas(32) float x[8], y[8], z[8], e[8], r8[8];
        for (size_t i = 0; i < n; i += 8)
        {
            for (int l = 0; l < 8; ++l)
            {
                x[l] = in[4 * (i + l) + 0];
                y[l] = in[4 * (i + l) + 1];
                z[l] = in[4 * (i + l) + 2];
            }
            probe_extent(launder(x), y, z, in[4 * i + 3], e, r8);
            std::memcpy(&out[i], e, 32);
            std::memcpy(&out[n + i], r8, 32);
        }
        write_f32(argv[3], out);
    }
    else if (mode == "rake")
    {
        // in: E x 14 (start[7], goal[7]); arg: max blocks B.
        // out per edge: [distance, n, then B blocks x 7 rows x 8 lanes] (unused blocks = NaN)
        // Mirrors planning/validate.hh:67-75 (validate_motion) and :23-56 (rake + back-steps),
        // with Robot::dimension = 7, rake = 8, resolution = 32 (robots/panda_base.hh:20-21).
        auto in = read_f32(argv[2]);
        const size_t nb = argc > 4 ? std::strtoul(argv[4], nullptr, 10) : 4;
        const size_t E = in.size() / 14;
        const size_t rec = 2 + nb * 56;
        std::vector<float> out(E * rec, __builtin_nanf(""));
        constexpr std::size_t rake = 8, resolution = 32, dim = 7;
        alignas(32) float sbuf[8] = {0}, gbuf[8] = {0};
        const float pct_a[8] = {1.f / 8, 2.f / 8, 3.f / 8, 4.f / 8, 5.f / 8, 6.f / 8, 7.f / 8, 8.f / 8};
        for (size_t e = 0; e < E; ++e)
        {
            for (size_t j = 0; j < dim; ++j) { sbuf[j] = in[14 * e + j]; gbuf[j] = in[14 * e + 7 + j]; }
            FloatVector<7> start(launder(sbuf)), goal(gbuf);
            auto vector = goal - start;
            float distance = vector.l2_norm();
            std::array<float, 8> pa;
            std::copy(pct_a, pct_a + 8, pa.begin());
            const auto percents = FloatVector<rake>(pa);
            FloatVector<rake, dim> block;
            for (auto i = 0U; i < dim; ++i)
                block[i] = start.broadcast(i) + (vector.broadcast(i) * percents);
            const std::size_t n =
                std::max(std::ceil(distance / static_cast<float>(rake) * resolution), 1.F);
            const auto backstep = vector / (rake * n);
            float *o = &out[e * rec];
            o[0] = distance;
            o[1] = static_cast<float>(n);
            for (size_t b = 0; b < nb && b < n; ++b)
            {
                if (b > 0)
                    for (auto j = 0U; j < dim; ++j) block[j] = block[j] - backstep.broadcast(j);
                alignas(32) float row[8];
                for (size_t j = 0; j < dim; ++j)
                {
                    block[j].to_array(row);
                    std::memcpy(o + 2 + b * 56 + j * 8, row, 32);
                }
            }
        }
        write_f32(argv[3], out);
    }
    else if (mode == "l2norm")
    {
        // in: E x dim vectors (goal - start); arg: dim (7, 8 or 14).  out: E distances
        // FloatVector<dim>::l2_norm (interface.hh:402-410): lane-wise sum of the registers
        // (utils.hh:53-62), then the AVX hsum (avx.hh:441-452), then std::sqrt.
        auto in = read_f32(argv[2]);
        const int dim = std::atoi(argv[4]);
        const size_t E = in.size() / dim;
        std::vector<float> out(E);
        alignas(32) float buf[16] = {0};
        for (size_t e = 0; e < E; ++e)
        {
            for (int j = 0; j < dim; ++j) buf[j] = in[dim * e + j];
            if (dim == 7) out[e] = FloatVector<7>(launder(buf)).l2_norm();
            else if (dim == 8) out[e] = FloatVector<8>(launder(buf)).l2_norm();
            else if (dim == 14) out[e] = FloatVector<14>(launder(buf)).l2_norm();
            else { std::fprintf(stderr, "l2norm: dim %d unsupported\n", dim); return 2; }
        }
        write_f32(argv[3], out);
    }
    else if (mode == "halton")
    {
        // args: dim count skip.  out: count x dim samples (after `skip` draws)
        const int dim = std::atoi(argv[4]);
        const size_t count = std::strtoul(argv[5], nullptr, 10);
        const size_t skip = std::strtoul(argv[6], nullptr, 10);
        std::vector<float> out;
        out.reserve(count * dim);
        alignas(32) float buf[16];
        if (dim == 8)
        {
            rng::Halton<8> h;
            for (size_t i = 0; i < skip; ++i) (void)h.next();
            for (size_t i = 0; i < count; ++i)
            {
                h.next().to_array(buf);
                out.insert(out.end(), buf, buf + 8);
            }
        }
        else if (dim == 7)
        {
            rng::Halton<7> h;
            for (size_t i = 0; i < skip; ++i) (void)h.next();
            for (size_t i = 0; i < count; ++i)
            {
                h.next().to_array(buf);
                out.insert(out.end(), buf, buf + 7);
            }
        }
        else
        {
            std::fprintf(stderr, "dim must be 7 or 8\n");
            return 2;
        }
        write_f32(argv[3], out);
    }
    else if (mode == "scale")
    {
        // in: N x 7 unit-cube samples.  out: N x 7 scaled configurations
        auto in = read_f32(argv[2]);
        const size_t n = in.size() / 7;
        std::vector<float> out(7 * n);
        for (size_t i = 0; i < n; ++i) probe_scale(launder(&in[7 * i]), &out[7 * i]);
        write_f32(argv[3], out);
    }
    else if (mode == "sql2")
    {
        // in: N x 6 (ax ay az bx by bz), b constant per group of 8.  out: N sql2_3
        auto in = read_f32(argv[2]);
        const size_t n = in.size() / 6;
        std::vector<float> out(n);
        alignas(32) float ax[8], ay[8], az[8], o[8];
        for (size_t i = 0; i < n; i += 8)
        {
            for (int l = 0; l < 8; ++l)
            {
                ax[l] = in[6 * (i + l) + 0];
                ay[l] = in[6 * (i + l) + 1];
                az[l] = in[6 * (i + l) + 2];
            }
            probe_sql2(launder(ax), ay, az, in[6 * i + 3], in[6 * i + 4], in[6 * i + 5], o);
            std::memcpy(&out[i], o, 32);
        }
        write_f32(argv[3], out);
    }
    else if (mode == "sql2s")
    {
        // in: N x 8 (ax ay az ar bx by bz br).  out: N scalar sphere_sphere_sql2 values
        auto in = read_f32(argv[2]);
        const size_t n = in.size() / 8;
        std::vector<float> out(n);
        for (size_t i = 0; i < n; ++i) out[i] = probe_sql2_scalar(launder(&in[8 * i]), &in[8 * i + 4]);
        write_f32(argv[3], out);
    }
    else if (mode == "capt_box")
    {
        // in: N x 11 (c[3] lo[3] up[3] r rp), rp constant per group of 8.
        // out: N simd leaf distsq, N rc_sq, N scalar distsq_to, N scalar ball sum
        auto in = read_f32(argv[2]);
        const size_t n = in.size() / 11;
        std::vector<float> out(4 * n);
        alignas(32) float c[24], lo[24], up[24], r[8], o[8], rc[8];
        for (size_t i = 0; i < n; i += 8)
        {
            for (int l = 0; l < 8; ++l)
            {
                const float *row = &in[11 * (i + l)];
                for (int k = 0; k < 3; ++k)
                {
                    c[8 * k + l] = row[k];
                    lo[8 * k + l] = row[3 + k];
                    up[8 * k + l] = row[6 + k];
                }
                r[l] = row[9];
                out[2 * n + i + l] = probe_vol_distsq(launder(row), row + 3, row + 6);
                out[3 * n + i + l] = probe_vol_ball(launder(row), row + 3, row + 6);
            }
            probe_capt_box(launder(c), lo, up, r, in[11 * i + 10], o, rc);
            std::memcpy(&out[i], o, 32);
            std::memcpy(&out[n + i], rc, 32);
        }
        write_f32(argv[3], out);
    }
    else if (mode == "hf")
    {
        // in: header [8] (x y z xs ys zs xd yd), data[xd*yd], then N x 4 (x y z r), r constant
        // per group of 8.  out: N test values (z - r - zh_scaled)
        auto in = read_f32(argv[2]);
        const size_t cells = (size_t)in[6] * (size_t)in[7];
        const float *data = &in[8];
        const float *q = &in[8 + cells];
        const size_t n = (in.size() - 8 - cells) / 4;
        std::vector<float> out(n);
        alignas(32) float x[8], y[8], z[8], o[8];
        for (size_t i = 0; i < n; i += 8)
        {
            for (int l = 0; l < 8; ++l)
            {
                x[l] = q[4 * (i + l)];
                y[l] = q[4 * (i + l) + 1];
                z[l] = q[4 * (i + l) + 2];
            }
            probe_hf(launder(x), y, z, q[4 * i + 3], in.data(), data, o);
            std::memcpy(&out[i], o, 32);
        }
        write_f32(argv[3], out);
    }
    else
    {
        std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    return 0;
}
