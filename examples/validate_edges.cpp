// examples/validate_edges.cpp -- the C++ mirror used the way a reference planner would use
// vamp::planning::validate_motion, on a batch: the sphere cage of the reference's collision
// benchmark (scripts/cpp/benchmark_collision_checks.cc:33-51), edges read from a binary file.
//
//   g++ -std=c++17 -O2 -Iinclude examples/validate_edges.cpp -Lmr-vamp_amd/vamp_amd -lvampgpu
//       -Wl,-rpath,$PWD/mr-vamp_amd/vamp_amd -o build/validate_edges     (one command)
//   build/validate_edges edges.f32 out.u8      (edges.f32 = n x 14 float32: start[7], goal[7])
#include <cstdio>
#include <vector>

#include "vamp_gpu.hpp"

using namespace vamp_gpu;

// The other robot types of the mirror, instantiated so the header's templates are compiled
// (-Wall -Werror in tests/test_c_abi.py): Fetch and the two-Panda composite.
[[maybe_unused]] static auto other_robots(collision::Environment &env) -> std::size_t
{
    const robots::Fetch::Configuration qf{0.1f, 0.0f, 0.5f, 0.0f, 1.0f, 0.0f, 1.0f, 0.0f};
    const robots::Panda_Pair::Configuration qp{};
    const bool a = robots::Fetch::fkcc_batch(env, {qf})[0] != 0;
    const auto b = planning::validate_motions<robots::Fetch>(env, {qf}, {qf});
    const bool c = planning::validate_motion<robots::Panda_Pair, 8, 32>(qp, qp, env);
    const bool d = robots::UR5::fkcc_batch(env, {robots::UR5::Configuration{}})[0] != 0;
    const bool e = planning::validate_motion<robots::Baxter, 8, 64>(robots::Baxter::Configuration{},
                                                                    robots::Baxter::Configuration{}, env);
    return (a ? 1u : 0u) + b.size() + (c ? 1u : 0u) + (d ? 1u : 0u) + (e ? 1u : 0u);
}

// An attached object (Environment::attach) and the PRM edge stage (build_roadmap's graph).
[[maybe_unused]] static auto attach_and_roadmap(collision::Environment &env) -> std::size_t
{
    collision::Attachment held({0.0f, 0.0f, 0.1f}, {0.0f, 0.0f, 0.0f, 1.0f});
    held.add_sphere({0.0f, 0.0f, 0.05f}, 0.03f);
    env.attach(held);
    const auto m = robots::Panda_0_0::fkcc_attach_batch(env, std::vector<robots::Panda_0_0::Configuration>(4));
    env.detach();
    const auto rm = planning::build_roadmap_edges<robots::Fetch>(
        env, std::vector<robots::Fetch::Configuration>(16), 269832.265625);
    return m.size() + rm.edges.size();
}

int main(int argc, char **argv)
{
    if (argc < 3)
    {
        std::fprintf(stderr, "usage: %s edges.f32 out.u8\n", argv[0]);
        return 2;
    }
    std::FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<float> raw;
    float buf[14];
    while (std::fread(buf, sizeof(float), 14, f) == 14) raw.insert(raw.end(), buf, buf + 14);
    std::fclose(f);
    using Robot = robots::Panda_0_0;
    std::vector<Robot::Configuration> starts(raw.size() / 14), goals(raw.size() / 14);
    for (std::size_t e = 0; e < starts.size(); ++e)
        for (std::size_t j = 0; j < Robot::dimension; ++j)
        {
            starts[e][j] = raw[14 * e + j];
            goals[e][j] = raw[14 * e + 7 + j];
        }
    try
    {
        Context ctx(0);
        collision::Environment env(ctx);
        const float cage[14][3] = {{0.55f, 0.0f, 0.25f}, {0.35f, 0.35f, 0.25f}, {0.0f, 0.55f, 0.25f},
                                   {-0.55f, 0.0f, 0.25f}, {-0.35f, -0.35f, 0.25f}, {0.0f, -0.55f, 0.25f},
                                   {0.35f, -0.35f, 0.25f}, {0.35f, 0.35f, 0.8f}, {0.0f, 0.55f, 0.8f},
                                   {-0.35f, 0.35f, 0.8f}, {-0.55f, 0.0f, 0.8f}, {-0.35f, -0.35f, 0.8f},
                                   {0.0f, -0.55f, 0.8f}, {0.35f, -0.35f, 0.8f}};
        for (const auto &c : cage) env.add_sphere({c[0], c[1], c[2]}, 0.2f);
        std::vector<int32_t> n;
        const auto ok = planning::validate_motions<Robot>(env, starts, goals, &n);
        std::size_t valid = 0;
        for (auto v : ok) valid += v;
        // the reference-shaped single edge: the CPU rake (same result as the GPU batch)
        const bool single = planning::validate_motion<Robot, 8, Robot::resolution>(starts[0], goals[0], env);
        std::FILE *o = std::fopen(argv[2], "wb");
        std::fwrite(ok.data(), 1, ok.size(), o);
        std::fclose(o);
        std::printf("edges %zu valid %zu first %d single %d\n", ok.size(), valid, (int)ok[0], (int)single);
        return single == (ok[0] != 0) ? 0 : 1;
    }
    catch (const Error &e)
    {
        std::fprintf(stderr, "vamp_gpu error %d: %s\n", e.code, e.what());
        return 1;
    }
}
