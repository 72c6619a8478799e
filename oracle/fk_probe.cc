// fk_probe.cc -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// The reference's own generated forward kinematics, compiled here with its release flags
// (cmake/CompilerSettings.cmake:3,12-15,27: -O3 -march=native -ffp-contract=fast -fassociative-math ...):
// oracle/extract_fk.sh copies `sphere_fk` and `eefk` out of robots/<robot>/fk.hh UNCHANGED into oracle/_ref/
// (dropping only the collision includes those two functions never use), and this driver runs them.  So the FK
// that the collision masks rest on is pinned against the compiled reference -- its contractions and
// reassociations as the release compiler actually picks them -- not only against tools/fkhh_interp.py's
// uncontracted evaluation of the same text.
//
//   fk_probe sphere_fk <robot> <bx100> <by100> <bz100> <q.bin> <out.bin>
//       q: [n][dim] float32, n a multiple of 8 (rake-8 blocks, robots/<robot>.hh: ConfigurationBlock<8>);
//       out: [n][n_spheres][3] float32, world-frame centres (the Panda's base offsets are template parameters
//       of its sphere_fk: (0,0,0) and (200,200,0) are instantiated; the other robots have none)
//   fk_probe eefk <robot> <q.bin> <out.bin>          out: [n][7] (x y z qx qy qz qw)
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "_ref/fk_panda.hh"
#include "_ref/fk_fetch.hh"
#include "_ref/fk_ur5.hh"
#include "_ref/fk_baxter.hh"

using namespace vamp;

static std::vector<float> read_f32(const char *path)
{
    FILE *f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<float> v(sz / 4);
    if (std::fread(v.data(), 4, v.size(), f) != v.size()) std::exit(2);
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

// rake-8 blocks of q through Fn(block, spheres) -> out[n][NS][3]
template <std::size_t DIM, std::size_t NS, class Spheres, class Fn>
static std::vector<float> run_blocks(const std::vector<float> &q, Fn fn)
{
    constexpr std::size_t rake = 8;
    const std::size_t n = q.size() / DIM;
    if (n % rake) { std::fprintf(stderr, "n must be a multiple of 8\n"); std::exit(2); }
    std::vector<float> out(n * NS * 3);
    for (std::size_t b = 0; b < n; b += rake) {
        FloatVector<rake, DIM> block;
        for (std::size_t j = 0; j < DIM; ++j) {
            std::array<float, rake> col;
            for (std::size_t l = 0; l < rake; ++l) col[l] = q[(b + l) * DIM + j];
            block[j] = FloatVector<rake>(col);
        }
        Spheres s;
        fn(block, s);
        for (std::size_t k = 0; k < NS; ++k) {
            alignas(32) float x[rake], y[rake], z[rake];
            s.x[k].to_array(x);
            s.y[k].to_array(y);
            s.z[k].to_array(z);
            for (std::size_t l = 0; l < rake; ++l) {
                float *o = &out[((b + l) * NS + k) * 3];
                o[0] = x[l];
                o[1] = y[l];
                o[2] = z[l];
            }
        }
    }
    return out;
}

template <std::size_t DIM, class Fn>
static std::vector<float> run_eefk(const std::vector<float> &q, Fn fn)
{
    const std::size_t n = q.size() / DIM;
    std::vector<float> out(n * 7);
    for (std::size_t i = 0; i < n; ++i) {
        std::array<float, DIM> c;
        for (std::size_t j = 0; j < DIM; ++j) c[j] = q[i * DIM + j];
        const std::array<float, 7> e = fn(c);
        for (int j = 0; j < 7; ++j) out[i * 7 + j] = e[j];
    }
    return out;
}

int main(int argc, char **argv)
{
    if (argc < 5) { std::fprintf(stderr, "usage: see the header\n"); return 2; }
    const std::string mode = argv[1], robot = argv[2];
    if (mode == "sphere_fk") {
        if (argc != 8) return 2;
        const int bx = std::atoi(argv[3]), by = std::atoi(argv[4]), bz = std::atoi(argv[5]);
        const std::vector<float> q = read_f32(argv[6]);
        std::vector<float> out;
        if (robot == "panda") {
            using S = robots::panda::Spheres<8>;
            if (bx == 0 && by == 0 && bz == 0)
                out = run_blocks<7, 59, S>(q, [](const auto &b, S &s) { robots::panda::sphere_fk<8, 0, 0, 0>(b, s); });
            else if (bx == 200 && by == 200 && bz == 0)
                out = run_blocks<7, 59, S>(q, [](const auto &b, S &s) { robots::panda::sphere_fk<8, 200, 200, 0>(b, s); });
            else { std::fprintf(stderr, "panda base not instantiated\n"); return 2; }
        } else if (robot == "fetch") {
            using S = robots::fetch::Spheres<8>;
            out = run_blocks<8, 111, S>(q, [](const auto &b, S &s) { robots::fetch::sphere_fk<8>(b, s); });
        } else if (robot == "ur5") {
            using S = robots::ur5::Spheres<8>;
            out = run_blocks<6, 36, S>(q, [](const auto &b, S &s) { robots::ur5::sphere_fk<8>(b, s); });
        } else if (robot == "baxter") {
            using S = robots::baxter::Spheres<8>;
            out = run_blocks<14, 75, S>(q, [](const auto &b, S &s) { robots::baxter::sphere_fk<8>(b, s); });
        } else return 2;
        write_f32(argv[7], out);
        return 0;
    }
    if (mode == "eefk") {
        const std::vector<float> q = read_f32(argv[3]);
        std::vector<float> out;
        if (robot == "panda") out = run_eefk<7>(q, [](const auto &c) { return robots::panda::eefk(c); });
        else if (robot == "fetch") out = run_eefk<8>(q, [](const auto &c) { return robots::fetch::eefk(c); });
        else if (robot == "ur5") out = run_eefk<6>(q, [](const auto &c) { return robots::ur5::eefk(c); });
        else return 2;
        write_f32(argv[4], out);
        return 0;
    }
    return 2;
}
