// vamp_gpu.hpp -- C++ host mirror of the reference's hot-path API over the C ABI (vamp_gpu.h).
//
// Mirrors the names and argument meaning of the reference (jamesmotes/mr-vamp):
//   vamp::collision::Environment<float> + add_* routing     collision/environment.hh:12-66,
//                                                          bindings/environment.cc:107-146
//   vamp::robots::PandaBase<X100,Y100,Z100>, Panda          robots/panda_base.hh:15-75,
//                                                          robots/panda_grid.hh:10-41
//   vamp::planning::validate_motion<Robot, rake, res>       planning/validate.hh:67-75
// so a planner written against the reference can swap its batch edge checks to the GPU.  As in
// the reference, collision results are plain bools (true = valid); infrastructure failures
// (no device, HIP error, bad arguments) throw vamp_gpu::Error, since the C ABI reports them
// as status codes.
#pragma once

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "vamp_gpu.h"

namespace vamp_gpu
{
    struct Error : std::runtime_error
    {
        int code;
        Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
    };

    inline void check(int rc, const vgpu_ctx *ctx, const char *what)
    {
        if (rc != VGPU_OK)
        {
            throw Error(rc, std::string(what) + ": " + (ctx ? vgpu_last_error(ctx) : "no context"));
        }
    }

    // One HIP device + stream; probes the host CPU's rsqrt approximation on creation.
    class Context
    {
    public:
        explicit Context(int device = 0)
        {
            const int rc = vgpu_ctx_create(device, &h_);
            if (rc != VGPU_OK)
            {
                throw Error(rc, "vgpu_ctx_create failed");
            }
        }
        ~Context() { vgpu_ctx_destroy(h_); }
        Context(const Context &) = delete;
        Context &operator=(const Context &) = delete;
        auto handle() const noexcept -> vgpu_ctx * { return h_; }
        void sync() { check(vgpu_sync(h_), h_, "vgpu_sync"); }
        void set_stream(void *hip_stream) { check(vgpu_ctx_set_stream(h_, hip_stream), h_, "set_stream"); }

    private:
        vgpu_ctx *h_ = nullptr;
    };

    namespace collision
    {
        using Point = std::array<float, 3>;

        // vamp::collision::Attachment<float> (collision/attachments.hh:14-123): spheres (x y z r)
        // relative to a frame (x y z, quaternion x y z w) held at the end effector
        struct Attachment
        {
            Attachment(const Point &center, const std::array<float, 4> &quaternion_xyzw)
              : frame{center[0], center[1], center[2], quaternion_xyzw[0], quaternion_xyzw[1],
                      quaternion_xyzw[2], quaternion_xyzw[3]}
            {
            }
            void add_sphere(const Point &center, float radius)
            {
                spheres.push_back({center[0], center[1], center[2], radius});
            }
            std::array<float, 7> frame;
            std::vector<std::array<float, 4>> spheres;
        };

        // vamp::collision::Environment<float>: obstacles are routed and sorted exactly like the
        // reference (axis_3_z == 1 -> z-aligned cuboid, xv == yv == 0 -> z-aligned capsule,
        // each list by min_distance); the device copy is made lazily on first use.
        class Environment
        {
        public:
            explicit Environment(Context &ctx) : ctx_(ctx)
            {
                check(vgpu_env_create(ctx.handle(), &h_), ctx.handle(), "vgpu_env_create");
            }
            ~Environment() { vgpu_env_destroy(h_); }
            Environment(const Environment &) = delete;
            Environment &operator=(const Environment &) = delete;

            void add_sphere(const Point &center, float radius)
            {
                check(vgpu_env_add_sphere(h_, center.data(), radius), ctx_.handle(), "add_sphere");
            }
            // factory::cuboid::array(center, euler_xyz, half_extents) (factory.hh:26-95)
            void add_cuboid(const Point &center, const Point &euler_xyz, const Point &half_extents)
            {
                check(vgpu_env_add_cuboid_euler(h_, center.data(), euler_xyz.data(), half_extents.data()),
                      ctx_.handle(), "add_cuboid");
            }
            // Cuboid<float> field constructor (shapes.hh:71-105)
            void add_cuboid(const Point &center, const Point &a1, const Point &a2, const Point &a3,
                            const Point &half_extents)
            {
                check(vgpu_env_add_cuboid_axes(h_, center.data(), a1.data(), a2.data(), a3.data(),
                                               half_extents.data()),
                      ctx_.handle(), "add_cuboid");
            }
            // factory::cylinder::endpoints (factory.hh:104-121)
            void add_capsule(const Point &p1, const Point &p2, float radius)
            {
                check(vgpu_env_add_capsule_endpoints(h_, p1.data(), p2.data(), radius), ctx_.handle(),
                      "add_capsule");
            }
            // factory::cylinder::center (factory.hh:149-173)
            void add_capsule(const Point &center, const Point &euler_xyz, float radius, float length)
            {
                check(vgpu_env_add_capsule_euler(h_, center.data(), euler_xyz.data(), radius, length),
                      ctx_.handle(), "add_capsule");
            }
            // Environment::attach(Attachment) / detach (bindings/environment.cc:161-163):
            // validate_motion then runs its first rake block through Robot::fkcc_attach
            void attach(const Attachment &a)
            {
                check(vgpu_env_attach(h_, a.frame.data(), a.spheres.empty() ? nullptr : a.spheres[0].data(),
                                      a.spheres.size()),
                      ctx_.handle(), "attach");
            }
            void detach() { check(vgpu_env_detach(h_), ctx_.handle(), "detach"); }
            auto handle() const noexcept -> vgpu_env * { return h_; }
            auto context() const noexcept -> Context & { return ctx_; }

        private:
            Context &ctx_;
            vgpu_env *h_ = nullptr;
        };
    }  // namespace collision

    namespace robots
    {
        // The batched calls every robot type shares (Derived provides c_robot(), dimension,
        // n_spheres and Configuration).
        template <typename Derived>
        struct RobotOps
        {
            // fkcc<rake> of one configuration broadcast to the rake == validate(q) without the
            // joint-limit check (bindings/common.hh:172-182)
            template <typename Configuration>
            static auto fkcc(collision::Environment &env, const Configuration &q) -> bool
            {
                return fkcc(env, std::vector<Configuration>{q})[0] != 0;
            }

            template <typename Configuration>
            static auto fkcc(collision::Environment &env, const std::vector<Configuration> &q)
                -> std::vector<uint8_t>
            {
                std::vector<uint8_t> out(q.size());
                const vgpu_robot r = Derived::c_robot();
                vgpu_ctx *c = env.context().handle();
                check(vgpu_fkcc_host(c, &r, env.handle(), q.empty() ? nullptr : q[0].data(), q.size(),
                                     out.data()),
                      c, "vgpu_fkcc_host");
                return out;
            }

            // fkcc_attach<rake> of each configuration (robots/panda_base.hh:61-65, fetch.hh:42,
            // ur5.hh:43; the Baxter's is its fkcc): the environment's attachment posed at the
            // end effector
            template <typename Configuration>
            static auto fkcc_attach(collision::Environment &env, const std::vector<Configuration> &q)
                -> std::vector<uint8_t>
            {
                std::vector<uint8_t> out(q.size());
                const vgpu_robot r = Derived::c_robot();
                vgpu_ctx *c = env.context().handle();
                check(vgpu_fkcc_attach_host(c, &r, env.handle(), q.empty() ? nullptr : q[0].data(), q.size(),
                                            out.data()),
                      c, "vgpu_fkcc_attach_host");
                return out;
            }

            // sphere_fk<1>: world-frame centres of the collision spheres (radii are constants)
            template <typename Configuration>
            static auto sphere_fk(Context &ctx, const Configuration &q)
            {
                constexpr std::size_t ns = Derived::n_spheres;
                std::vector<float> soa(3 * ns);
                const vgpu_robot r = Derived::c_robot();
                check(vgpu_sphere_fk_host(ctx.handle(), &r, q.data(), 1, soa.data()), ctx.handle(),
                      "vgpu_sphere_fk_host");
                std::array<std::array<float, 3>, ns> out{};
                for (std::size_t s = 0; s < ns; ++s)
                    for (int c = 0; c < 3; ++c) out[s][c] = soa[c * ns + s];
                return out;
            }
        };

        // vamp::robots::PandaBase<X100, Y100, Z100> (robots/panda_base.hh:15-75)
        template <int BaseX100, int BaseY100, int BaseZ100>
        struct PandaBase : RobotOps<PandaBase<BaseX100, BaseY100, BaseZ100>>
        {
            static constexpr auto name = "panda";
            static constexpr std::size_t dimension = 7;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 59;
            static constexpr float base_x = static_cast<float>(BaseX100) / 100.0f;
            static constexpr float base_y = static_cast<float>(BaseY100) / 100.0f;
            static constexpr float base_z = static_cast<float>(BaseZ100) / 100.0f;

            using Configuration = std::array<float, dimension>;
            using Spheres = std::array<std::array<float, 3>, n_spheres>;  // centres; radii are constants

            static auto c_robot() noexcept -> vgpu_robot
            {
                return vgpu_robot{VGPU_ROBOT_PANDA, BaseX100, BaseY100, BaseZ100, 0, 0, 0};
            }
        };

        // vamp::robots::Fetch (robots/fetch.hh:8-48): 8 dof (prismatic torso first), 111 spheres
        struct Fetch : RobotOps<Fetch>
        {
            static constexpr auto name = "fetch";
            static constexpr std::size_t dimension = 8;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 111;
            using Configuration = std::array<float, dimension>;
            using Spheres = std::array<std::array<float, 3>, n_spheres>;

            static auto c_robot() noexcept -> vgpu_robot { return vgpu_robot{VGPU_ROBOT_FETCH, 0, 0, 0, 0, 0, 0}; }
        };

        // vamp::robots::UR5 (robots/ur5.hh): 6 dof, 36 spheres
        struct UR5 : RobotOps<UR5>
        {
            static constexpr auto name = "ur5";
            static constexpr std::size_t dimension = 6;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 36;
            using Configuration = std::array<float, dimension>;
            static auto c_robot() noexcept -> vgpu_robot { return vgpu_robot{VGPU_ROBOT_UR5, 0, 0, 0, 0, 0, 0}; }
        };

        // vamp::robots::Baxter (robots/baxter.hh): 14-dof dual arm, 75 spheres, resolution 64
        struct Baxter : RobotOps<Baxter>
        {
            static constexpr auto name = "baxter";
            static constexpr std::size_t dimension = 14;
            static constexpr std::size_t resolution = 64;
            static constexpr std::size_t n_spheres = 75;
            using Configuration = std::array<float, dimension>;
            static auto c_robot() noexcept -> vgpu_robot { return vgpu_robot{VGPU_ROBOT_BAXTER, 0, 0, 0, 0, 0, 0}; }
        };

        // Two Pandas as one 14-dof robot (BASELINE configs[4]; no reference counterpart):
        // joints 0..6 = PandaBase<A>, 7..13 = PandaBase<B>; valid = fkcc_A && fkcc_B && no A-B
        // sphere overlap.  fkcc and validate_motions only (sphere_fk: use each arm's type).
        template <int AX, int AY, int AZ, int BX, int BY, int BZ>
        struct PandaPair : RobotOps<PandaPair<AX, AY, AZ, BX, BY, BZ>>
        {
            static constexpr auto name = "panda_pair";
            static constexpr std::size_t dimension = 14;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 118;
            using Configuration = std::array<float, dimension>;

            static auto c_robot() noexcept -> vgpu_robot
            {
                return vgpu_robot{VGPU_ROBOT_PANDA_PAIR, AX, AY, AZ, BX, BY, BZ};
            }
        };

        // robots/panda_grid.hh:10-41 -- this fork's default Panda stands at (2, 2, 0)
        struct Panda : PandaBase<200, 200, 0> {};
        struct Panda_0_0 : PandaBase<0, 0, 0> { static constexpr auto name = "panda_0_0"; };
        struct Panda_1_0 : PandaBase<100, 0, 0> { static constexpr auto name = "panda_1_0"; };
        struct Panda_2_2 : PandaBase<200, 200, 0> { static constexpr auto name = "panda_2_2"; };
        // the configs[4] composite: arms 1 m apart along x
        using Panda_Pair = PandaPair<0, 0, 0, 100, 0, 0>;
    }  // namespace robots

    namespace planning
    {
        // validate_motion<Robot, 8, Robot::resolution> for a batch of edges (validate.hh:67-75);
        // n_blocks receives n_e (interpolants = 8 * n_e) when given.
        template <typename Robot>
        inline auto validate_motions(collision::Environment &env,
                                     const std::vector<typename Robot::Configuration> &starts,
                                     const std::vector<typename Robot::Configuration> &goals,
                                     std::vector<int32_t> *n_blocks = nullptr) -> std::vector<uint8_t>
        {
            if (starts.size() != goals.size())
            {
                throw Error(VGPU_ERR_INVALID_ARG, "validate_motions: starts/goals differ in size");
            }
            std::vector<uint8_t> ok(starts.size());
            std::vector<int32_t> n(starts.size());
            const vgpu_robot r = Robot::c_robot();
            vgpu_ctx *c = env.context().handle();
            check(vgpu_validate_motions_host(c, &r, env.handle(), starts.empty() ? nullptr : starts[0].data(),
                                             goals.empty() ? nullptr : goals[0].data(), starts.size(), ok.data(),
                                             n.data()),
                  c, "vgpu_validate_motions_host");
            if (n_blocks) *n_blocks = std::move(n);
            return ok;
        }

        // validate_motion<Robot, 8, res>(start, goal, env): one edge (prefer the batch form)
        template <typename Robot>
        inline auto validate_motion(collision::Environment &env, const typename Robot::Configuration &start,
                                    const typename Robot::Configuration &goal) -> bool
        {
            return validate_motions<Robot>(env, {start}, {goal})[0] != 0;
        }

        // Roadmap<dim> (prm.hh:285-299): vertices and, per vertex, its neighbours in the order
        // build_roadmap appended them; component = smallest vertex index of its component
        template <typename Robot>
        struct Roadmap
        {
            std::vector<typename Robot::Configuration> vertices;
            std::vector<std::vector<std::size_t>> edges;
            std::vector<uint32_t> component;
        };

        // Roadmap::build_roadmap's graph (prm.hh:197-299) over a vertex sequence (start, goal,
        // then the valid samples in draw order): every vertex's PRM* neighbour query
        // (PRMStarNeighborParams(dim, space_measure) with gamma_scale, roadmap.hh:42-77) and
        // validate_motion of every candidate edge on the GPU
        template <typename Robot>
        inline auto build_roadmap_edges(collision::Environment &env,
                                        const std::vector<typename Robot::Configuration> &vertices,
                                        double space_measure, double gamma_scale = 2.0) -> Roadmap<Robot>
        {
            const std::size_t n = vertices.size();
            std::vector<uint32_t> k(n);
            std::vector<float> r(n);
            check(vgpu_prm_neighbor_params(static_cast<int>(Robot::dimension), space_measure, gamma_scale, n, k.data(),
                                           r.data()),
                  nullptr, "vgpu_prm_neighbor_params");
            std::size_t cap = 0;
            for (uint32_t v : k) cap += 2 * static_cast<std::size_t>(v);
            std::vector<std::size_t> offsets(n + 1, 0);
            std::vector<uint32_t> adj(cap > 0 ? cap : 1);
            Roadmap<Robot> out{vertices, std::vector<std::vector<std::size_t>>(n), std::vector<uint32_t>(n)};
            std::size_t n_adj = 0;
            const vgpu_robot rb = Robot::c_robot();
            vgpu_ctx *c = env.context().handle();
            check(vgpu_build_roadmap_host(c, &rb, env.handle(), n ? vertices[0].data() : nullptr, n, space_measure,
                                          gamma_scale, offsets.data(), adj.data(), adj.size(), &n_adj,
                                          out.component.data()),
                  c, "vgpu_build_roadmap_host");
            for (std::size_t i = 0; i < n; ++i) out.edges[i].assign(adj.begin() + offsets[i], adj.begin() + offsets[i + 1]);
            return out;
        }
    }  // namespace planning
}  // namespace vamp_gpu
