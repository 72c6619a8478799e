// examples/robot_concept.cpp -- code written against the reference's Robot concept, re-pointed at
// vamp_gpu::robots: generic templates instantiate
//   planning::validate_motion<Robot, 8, Robot::resolution>(start, goal, env)   (validate.hh:67-75)
//   Robot::template fkcc<8>(env, block), sphere_fk<8>, scale_/descale_configuration[_block], eefk
//   planning::RRTC<Robot, 8, Robot::resolution>::solve(...)                    (rrtc.hh:33-248)
// exactly as the reference's planners do; no GPU is needed (host-only environment, CPU rake).
//
//   g++ -std=c++17 -O2 -Wall -Werror -Iinclude examples/robot_concept.cpp -Lmr-vamp_amd/vamp_amd
//       -lvampgpu -Wl,-rpath,$PWD/mr-vamp_amd/vamp_amd -o build/robot_concept      (one command)
//   build/robot_concept edges.f32 out.txt     (edges.f32 = n x 14 float32: Panda start[7], goal[7])
// out.txt: one line per edge "<validate_motion> <fkcc of the 8 starts from this edge on>", then
// the scale round trip, eefk and sphere_fk of edge 0, and an RRT-Connect solve.
#include <cstdio>
#include <vector>

#include "vamp_gpu.hpp"

using namespace vamp_gpu;

// a reference-style generic helper: any Robot with the concept
template <typename Robot>
static auto path_is_valid(const std::vector<typename Robot::Configuration> &path,
                          const collision::Environment &env) -> bool
{
    for (std::size_t i = 0; i + 1 < path.size(); ++i)
        if (!planning::validate_motion<Robot, 8, Robot::resolution>(path[i], path[i + 1], env)) return false;
    return true;
}

template <typename Robot>
static auto block_of(const std::vector<typename Robot::Configuration> &q, std::size_t first) ->
    typename Robot::template ConfigurationBlock<8>
{
    typename Robot::template ConfigurationBlock<8> b;
    for (std::size_t l = 0; l < 8; ++l)
        for (std::size_t j = 0; j < Robot::dimension; ++j) b[j][l] = q[(first + l) % q.size()][j];
    return b;
}

int main(int argc, char **argv)
{
    if (argc < 3)
    {
        std::fprintf(stderr, "usage: %s edges.f32 out.txt\n", argv[0]);
        return 2;
    }
    using Robot = robots::Panda_0_0;
    std::FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<Robot::Configuration> starts, goals;
    float buf[14];
    while (std::fread(buf, sizeof(float), 14, f) == 14)
    {
        starts.emplace_back(buf);
        goals.emplace_back(buf + 7);
    }
    std::fclose(f);
    if (starts.empty()) return 2;
    try
    {
        collision::Environment env;  // host-only: the CPU rake
        const float cage[14][3] = {{0.55f, 0.0f, 0.25f}, {0.35f, 0.35f, 0.25f}, {0.0f, 0.55f, 0.25f},
                                   {-0.55f, 0.0f, 0.25f}, {-0.35f, -0.35f, 0.25f}, {0.0f, -0.55f, 0.25f},
                                   {0.35f, -0.35f, 0.25f}, {0.35f, 0.35f, 0.8f}, {0.0f, 0.55f, 0.8f},
                                   {-0.35f, 0.35f, 0.8f}, {-0.55f, 0.0f, 0.8f}, {-0.35f, -0.35f, 0.8f},
                                   {0.0f, -0.55f, 0.8f}, {0.35f, -0.35f, 0.8f}};
        for (const auto &c : cage) env.add_sphere({c[0], c[1], c[2]}, 0.2f);
        std::FILE *o = std::fopen(argv[2], "w");
        for (std::size_t e = 0; e < starts.size(); ++e)
        {
            const bool v = planning::validate_motion<Robot, 8, Robot::resolution>(starts[e], goals[e], env);
            const bool b = Robot::fkcc<8>(env, block_of<Robot>(starts, e));
            std::fprintf(o, "%d %d\n", v ? 1 : 0, b ? 1 : 0);
        }
        // scale / descale round trip of edge 0's start, the block forms, eefk, sphere_fk
        auto q = starts[0];
        Robot::descale_configuration(q);
        Robot::scale_configuration(q);
        auto blk = block_of<Robot>(starts, 0);
        Robot::descale_configuration_block(blk);
        Robot::scale_configuration_block(blk);
        const auto pose = Robot::eefk(starts[0].to_array());
        Robot::Spheres<8> sph;
        Robot::sphere_fk<8>(block_of<Robot>(starts, 0), sph);
        std::fprintf(o, "roundtrip %.9g %.9g\n", q[0], blk[0][0]);
        std::fprintf(o, "eefk %.9g %.9g %.9g %.9g %.9g %.9g %.9g\n", pose[0], pose[1], pose[2], pose[3], pose[4],
                     pose[5], pose[6]);
        std::fprintf(o, "sphere0 %.9g %.9g %.9g\n", sph.x[0][0], sph.y[0][0], sph.z[0][0]);
        // RRT-Connect from edge 0's start to edge 1's goal (the caller's checks: path_is_valid)
        rng::Halton<Robot::dimension> rng;
        planning::RRTCSettings settings;
        settings.range = 1.0f;
        const auto res = planning::RRTC<Robot, 8, Robot::resolution>::solve(starts[0], goals[1 % goals.size()], env,
                                                                             settings, rng);
        std::fprintf(o, "rrtc %zu %zu %zu %d %llu\n", res.path.size(), res.iterations, res.size.size(),
                     path_is_valid<Robot>(res.path, env) ? 1 : 0, (unsigned long long)rng.index);
        std::fclose(o);
        return 0;
    }
    catch (const Error &e)
    {
        std::fprintf(stderr, "vamp_gpu error %d: %s\n", e.code, e.what());
        return 1;
    }
}
