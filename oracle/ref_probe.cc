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
//
// Usage: ref_probe <mode> <in.bin> <out.bin> [args]   (raw little-endian float32)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>

#include <vamp/vector.hh>
#include <vamp/random/halton.hh>

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
    else
    {
        std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    return 0;
}
