// sanitize_main.cc -- TEST INFRASTRUCTURE ONLY (SURVEY §5 "ASan/UBSan build of the CPU restatement").
//
// Built by `make -C oracle sanitize` with -fsanitize=address,undefined -fno-sanitize-recover into
// oracle/_build/sanitize_check, from the oracle's C restatement (vamp_oracle.c) and the product's
// host-only CAPT construction (mr-vamp_amd/csrc/vgpu_capt.cpp).  It drives every oracle entry point
// family on small seeded inputs -- every robot's FK / fkcc / validate (incl. attachments, zero-length
// and long edges), the composite, CAPT build + both queries against the host build, Halton, the PRM
// neighbour query, the point-cloud filter with and without culling -- and cross-checks the two CAPT
// builds.  Any out-of-bounds access, use-after-free, leak or UB aborts with a non-zero exit
// (tests/test_sanitize.py).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mr-vamp_amd/csrc/vgpu_capt.hh"
#include "vamp_oracle.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static float uni(float lo, float hi)
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return lo + (hi - lo) * (float)((rng_state >> 40) * (1.0 / 16777216.0));
}

#define CHECK(cond)                                                                  \
    do {                                                                             \
        if (!(cond)) {                                                               \
            std::fprintf(stderr, "sanitize_check: %s failed (line %d)\n", #cond, __LINE__); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

static void add_sphere(std::vector<float>& s, float x, float y, float z, float r)
{
    s.insert(s.end(), {x, y, z, r, vo_sphere_min_distance(x, y, z, r)});
}

int main()
{
    // environment: spheres (sorted by min_distance), one cuboid, one capsule, one heightfield,
    // one point cloud
    std::vector<float> spheres;
    for (int i = 0; i < 12; ++i) add_sphere(spheres, uni(-0.8f, 0.8f), uni(-0.8f, 0.8f), uni(0.0f, 1.2f), uni(0.05f, 0.2f));
    std::vector<int> order(12);
    for (int i = 0; i < 12; ++i) order[i] = i;
    for (int i = 0; i < 12; ++i)
        for (int j = i + 1; j < 12; ++j)
            if (spheres[5 * order[j] + 4] < spheres[5 * order[i] + 4]) std::swap(order[i], order[j]);
    std::vector<float> sorted;
    for (int i : order) sorted.insert(sorted.end(), spheres.begin() + 5 * i, spheres.begin() + 5 * i + 5);
    float cub[16] = {0.6f, 0.0f, 0.3f, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0.1f, 0.2f, 0.05f, 0};
    cub[15] = vo_cuboid_min_distance(cub);
    float cap[9] = {-0.5f, 0.3f, 0.2f, 0.0f, 0.0f, 0.4f, 0.06f, 0, 0};
    cap[7] = 1.0f / (cap[3] * cap[3] + cap[4] * cap[4] + cap[5] * cap[5]);
    cap[8] = vo_capsule_min_distance(cap);
    std::vector<float> hdata(16 * 12);
    for (auto& h : hdata) h = uni(0.0f, 1.0f);
    vo_heightfield hf{-1.0f, -1.0f, -0.5f, 1.0f / 2.0f, 1.0f / 2.0f, 1.0f / 0.3f, 16, 12, hdata.data()};

    std::vector<float> pts;
    for (int i = 0; i < 600; ++i) pts.insert(pts.end(), {uni(0.3f, 0.7f), uni(-0.4f, 0.4f), uni(0.0f, 0.6f)});
    vo_capt capt{};
    CHECK(vo_capt_build(pts.data(), 600, 0.01f, 0.08f, 0.005f, &capt) == 0);
    vgpu::CaptTree host;
    vgpu::capt_build(pts.data(), 600, 0.01f, 0.08f, 0.005f, host);
    CHECK(host.nlog2 == capt.nlog2 && host.n_aff() == capt.n_aff);
    CHECK(std::memcmp(host.tests.data(), capt.tests, host.tests.size() * 4) == 0);
    CHECK(std::memcmp(host.aff.data(), capt.aff, host.aff.size() * 4) == 0);
    std::vector<float> qc(3 * 256), qr(256);
    for (int i = 0; i < 256; ++i) {
        qc[3 * i] = uni(0.0f, 1.0f), qc[3 * i + 1] = uni(-0.6f, 0.6f), qc[3 * i + 2] = uni(-0.1f, 0.8f);
        qr[i] = uni(0.01f, 0.08f);
    }
    std::vector<uint8_t> o0(256), o1(256);
    vo_capt_collides_batch(&capt, qc.data(), qr.data(), 256, 0, o0.data(), nullptr);
    vo_capt_collides_batch(&capt, qc.data(), qr.data(), 256, 1, o1.data(), nullptr);

    vo_env env{};
    env.n_spheres = 12;
    env.spheres = sorted.data();
    env.n_cuboids = 1;
    env.cuboids = cub;
    env.n_capsules = 1;
    env.capsules = cap;
    env.n_heightfields = 1;
    env.heightfields = &hf;
    env.n_pointclouds = 1;
    env.pointclouds = &capt;

    const float att_spheres[8] = {0.0f, 0.0f, 0.05f, 0.03f, 0.0f, 0.02f, 0.1f, 0.02f};
    vo_attachment att{{0.0f, 0.0f, 0.1f, 0.0f, 0.0f, 0.0f, 1.0f}, 2, att_spheres};
    const int robots[4] = {VO_ROBOT_PANDA, VO_ROBOT_FETCH, VO_ROBOT_UR5, VO_ROBOT_BAXTER};
    for (int r : robots) {
        const int dim = vo_robot_dim(r);
        const int ns = vo_robot_nspheres(r);
        CHECK(dim > 0 && dim <= 16 && ns > 0);
        const size_t n = 64;
        std::vector<float> q((n + 1) * dim), g((n + 1) * dim);
        for (auto& x : q) x = uni(0.0f, 1.0f);
        for (auto& x : g) x = uni(0.0f, 1.0f);
        for (size_t i = 0; i <= n; ++i) vo_robot_scale(r, &q[i * dim]), vo_robot_scale(r, &g[i * dim]);
        std::memcpy(&g[0], &q[0], dim * sizeof(float));  // a zero-length edge
        for (int j = 0; j < dim; ++j) g[dim + j] = q[dim + j] + 3.0f * ((j & 1) ? 1.0f : -1.0f);  // a long edge
        std::vector<float> xyz((size_t)ns * 3);
        vo_robot_sphere_fk(r, q.data(), 0, 0, 0, (float(*)[3])xyz.data());
        std::vector<uint8_t> valid(n), ok(n);
        std::vector<int32_t> nb(n);
        vo_stats st{};
        (void)vo_robot_fkcc_block(r, &env, q.data(), 8, 0, 0, 0, &st);
        vo_robot_fkcc_configs(r, &env, q.data(), n, 0, 0, 0, valid.data(), 2);
        vo_robot_validate_motions(r, &env, q.data(), g.data(), n, 0, 0, 0, ok.data(), nb.data(), 2);
        CHECK(nb[0] == 1);
        int n_out = 0;
        const int v1 = vo_robot_validate_motion(r, &env, q.data() + dim, g.data() + dim, 0, 0, 0, &n_out, &st);
        CHECK(v1 == ok[1] && n_out == nb[1]);
        if (vo_robot_fkcc_attach_block(r, &env, &att, q.data(), 8, 0, 0, 0, &st) >= 0) {
            vo_robot_fkcc_attach_configs(r, &env, &att, q.data(), n, 0, 0, 0, valid.data(), 2);
            vo_robot_validate_motions_att(r, &env, &att, q.data(), g.data(), n, 0, 0, 0, ok.data(), nb.data(), 2);
        }
        // PRM neighbour query over these configurations
        std::vector<uint32_t> nbr(n * 8), cnt(n);
        std::vector<float> dist(n * 8);
        vo_roadmap_knn(dim, q.data(), n, 1.0, 1.0, 8, nbr.data(), dist.data(), cnt.data(), 2);
        for (size_t i = 0; i < n; ++i) CHECK(cnt[i] <= 8 && cnt[i] <= i);
    }
    // composite
    {
        const int ba[3] = {0, 0, 0}, bb[3] = {0, 80, 0};
        std::vector<float> q(16 * 14), g(16 * 14);
        for (int i = 0; i < 16; ++i)
            for (int h = 0; h < 2; ++h) {
                float* a = &q[14 * i + 7 * h];
                float* b = &g[14 * i + 7 * h];
                for (int j = 0; j < 7; ++j) a[j] = uni(0.0f, 1.0f), b[j] = uni(0.0f, 1.0f);
                vo_panda_scale(a), vo_panda_scale(b);
            }
        std::vector<uint8_t> valid(16), ok(16);
        std::vector<int32_t> nb(16);
        vo_pair_fkcc_configs(&env, q.data(), 16, ba, bb, valid.data(), 2);
        vo_pair_validate_motions(&env, q.data(), g.data(), 16, ba, bb, ok.data(), nb.data(), 2);
    }
    // Halton
    for (int d = 2; d <= 16; ++d) {
        float h[16];
        vo_halton(d, 1, h);
        vo_halton(d, 999999, h);
        for (int j = 0; j < d; ++j) CHECK(h[j] >= 0.0f && h[j] < 1.0f);
    }
    // point-cloud filter, with and without culling (most points outside the workspace)
    {
        const size_t n = 4096;
        std::vector<float> pc(3 * n);
        for (auto& x : pc) x = uni(-3.0f, 3.0f);
        std::vector<uint32_t> idx(n);
        const float origin[3] = {0, 0, 0.5f}, lo[3] = {-1.2f, -1.2f, -1.2f}, hi[3] = {1.2f, 1.2f, 1.2f};
        for (int cull = 0; cull < 2; ++cull) {
            const size_t k = vo_filter_pointcloud(pc.data(), n, 0.05f, 1.5f, origin, lo, hi, cull, idx.data());
            CHECK(k >= 1 && k <= n);
            for (size_t i = 0; i < k; ++i) CHECK(idx[i] < n);
        }
        CHECK(vo_filter_pointcloud(pc.data(), 1, 0.05f, 1.5f, origin, lo, hi, 1, idx.data()) == 1);
    }
    vo_capt_free(&capt);
    std::printf("sanitize_check: ok\n");
    return 0;
}
