// vamp_gpu.hpp -- C++ mirror of the reference's hot-path API over the C ABI (vamp_gpu.h).
//
// The reference's template boundary (robots/panda_base.hh:15-75, fetch.hh:8-48,
// planning/validate.hh:23-75, planning/rrtc.hh:16-249): a Robot type with static name,
// dimension, resolution, n_spheres, space_measure(), Configuration, ConfigurationArray,
// ConfigurationBuffer, ConfigurationBlock<rake>, Spheres<rake>, scale_/descale_configuration[_block],
// fkcc<rake>(env, block), fkcc_attach<rake>(env, block), sphere_fk<rake>(block, out), eefk(q); and
// the generic consumers validate_vector / validate_motion<Robot, rake, resolution>(...) and
// RRTC<Robot, rake, resolution>::solve(...).  A planner templated on vamp::robots::Panda can be
// re-pointed at vamp_gpu::robots::Panda unchanged: the single-block / single-edge calls run on the
// host CPU rake (AVX2, bit-identical to the GPU kernels -- a GPU launch costs far more than one
// edge), and the *batch* calls (fkcc_batch, planning::validate_motions, build_roadmap_edges) run on
// the MI355X.
//
// Collision results are plain bools (true = valid), as in the reference; infrastructure failures
// (no device, HIP error, bad arguments) throw vamp_gpu::Error, since the C ABI reports them as
// status codes.  The CPU rake supports rake = 8 (one AVX2 register per block, the reference's
// FloatVectorWidth); other rakes are rejected at compile time.
#pragma once

#include <array>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
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
            throw Error(rc, std::string(what) + ": " + (ctx ? vgpu_last_error(ctx) : "vamp_gpu error"));
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

    // FloatVector<dim> as the planners use a Configuration (vector/interface.hh): element access,
    // lane-wise + - * /, scalar * /, and l2_norm in the AVX lane order (vgpu_l2_norm).
    template <std::size_t dim>
    struct FloatVector
    {
        static constexpr std::size_t num_scalars = dim;
        static constexpr std::size_t num_scalars_rounded = (dim + 7) / 8 * 8;
        std::array<float, dim> v{};

        FloatVector() = default;
        FloatVector(const std::array<float, dim> &a) : v(a) {}  // NOLINT: implicit, as the reference's
        template <typename... T, typename = std::enable_if_t<sizeof...(T) == dim && (dim > 1)>>
        FloatVector(T... x) : v{{static_cast<float>(x)...}}  // NOLINT: brace lists of dim scalars
        {
        }
        explicit FloatVector(const float *p)
        {
            for (std::size_t i = 0; i < dim; ++i) v[i] = p[i];
        }
        auto operator[](std::size_t i) noexcept -> float & { return v[i]; }
        auto operator[](std::size_t i) const noexcept -> float { return v[i]; }
        auto data() noexcept -> float * { return v.data(); }
        auto data() const noexcept -> const float * { return v.data(); }
        auto to_array() const -> std::array<float, dim> { return v; }
        void to_array(float *out) const
        {
            for (std::size_t i = 0; i < dim; ++i) out[i] = v[i];
        }
        auto broadcast(std::size_t i) const noexcept -> float { return v[i]; }

#define VAMP_GPU_LANEWISE(OP)                                                        \
    friend auto operator OP(const FloatVector &a, const FloatVector &b) -> FloatVector \
    {                                                                                \
        FloatVector r;                                                               \
        for (std::size_t i = 0; i < dim; ++i) r.v[i] = a.v[i] OP b.v[i];             \
        return r;                                                                    \
    }                                                                                \
    friend auto operator OP(const FloatVector &a, float s) -> FloatVector            \
    {                                                                                \
        FloatVector r;                                                               \
        for (std::size_t i = 0; i < dim; ++i) r.v[i] = a.v[i] OP s;                  \
        return r;                                                                    \
    }
        VAMP_GPU_LANEWISE(+)
        VAMP_GPU_LANEWISE(-)
        VAMP_GPU_LANEWISE(*)
        VAMP_GPU_LANEWISE(/)
#undef VAMP_GPU_LANEWISE

        // (in the library, compiled without contraction: a caller's -ffp-contract=fast could fuse the
        // squares into the lane sums)
        auto l2_norm() const -> float { return vgpu_l2_norm(v.data(), static_cast<int>(dim)); }
        auto distance(const FloatVector &o) const -> float { return (*this - o).l2_norm(); }
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
        // reference (axis_3_z == 1 -> z-aligned cuboid, xv == yv == 0 -> z-aligned capsule, each
        // list by min_distance).  Environment() is host-only (the CPU rake: single blocks/edges and
        // planners); Environment(ctx) also serves the GPU batch calls (device copy made lazily).
        class Environment
        {
        public:
            Environment() { check(vgpu_env_create(nullptr, &h_), nullptr, "vgpu_env_create"); }
            explicit Environment(Context &ctx) : ctx_(&ctx)
            {
                check(vgpu_env_create(ctx.handle(), &h_), ctx.handle(), "vgpu_env_create");
            }
            ~Environment() { vgpu_env_destroy(h_); }
            Environment(const Environment &) = delete;
            Environment &operator=(const Environment &) = delete;

            void add_sphere(const Point &center, float radius)
            {
                check(vgpu_env_add_sphere(h_, center.data(), radius), ctxh(), "add_sphere");
            }
            // factory::cuboid::array(center, euler_xyz, half_extents) (factory.hh:26-95)
            void add_cuboid(const Point &center, const Point &euler_xyz, const Point &half_extents)
            {
                check(vgpu_env_add_cuboid_euler(h_, center.data(), euler_xyz.data(), half_extents.data()), ctxh(),
                      "add_cuboid");
            }
            // Cuboid<float> field constructor (shapes.hh:71-105)
            void add_cuboid(const Point &center, const Point &a1, const Point &a2, const Point &a3,
                            const Point &half_extents)
            {
                check(vgpu_env_add_cuboid_axes(h_, center.data(), a1.data(), a2.data(), a3.data(),
                                               half_extents.data()),
                      ctxh(), "add_cuboid");
            }
            // factory::cylinder::endpoints (factory.hh:104-121)
            void add_capsule(const Point &p1, const Point &p2, float radius)
            {
                check(vgpu_env_add_capsule_endpoints(h_, p1.data(), p2.data(), radius), ctxh(), "add_capsule");
            }
            // factory::cylinder::center (factory.hh:149-173)
            void add_capsule(const Point &center, const Point &euler_xyz, float radius, float length)
            {
                check(vgpu_env_add_capsule_euler(h_, center.data(), euler_xyz.data(), radius, length), ctxh(),
                      "add_capsule");
            }
            // Environment::add_pointcloud (bindings/environment.cc:148-158): builds a CAPT
            auto add_pointcloud(const std::vector<Point> &pts, float r_min, float r_max, float r_point) -> int64_t
            {
                int64_t ns = 0;
                check(vgpu_env_add_pointcloud(h_, pts.empty() ? nullptr : pts[0].data(), pts.size(), r_min, r_max,
                                              r_point, &ns),
                      ctxh(), "add_pointcloud");
                return ns;
            }
            // Environment::attach(Attachment) / detach (bindings/environment.cc:161-163):
            // validate_motion then runs its first rake block through Robot::fkcc_attach
            void attach(const Attachment &a)
            {
                check(vgpu_env_attach(h_, a.frame.data(), a.spheres.empty() ? nullptr : a.spheres[0].data(),
                                      a.spheres.size()),
                      ctxh(), "attach");
                attached_ = true;
            }
            void detach()
            {
                check(vgpu_env_detach(h_), ctxh(), "detach");
                attached_ = false;
            }
            // Environment::attachments (environment.hh:21) is set
            auto attached() const noexcept -> bool { return attached_; }
            auto handle() const noexcept -> vgpu_env * { return h_; }
            auto context() const -> Context &
            {
                if (!ctx_) throw Error(VGPU_ERR_INVALID_ARG, "host-only environment: construct it with a Context");
                return *ctx_;
            }

        private:
            auto ctxh() const noexcept -> vgpu_ctx * { return ctx_ ? ctx_->handle() : nullptr; }
            Context *ctx_ = nullptr;
            bool attached_ = false;
            vgpu_env *h_ = nullptr;
        };
    }  // namespace collision

    namespace robots
    {
        // The Robot concept of the reference over the C ABI.  Derived provides name, dimension,
        // resolution, n_spheres, kind and (Pandas) the base offset.
        template <typename Derived, std::size_t dim, std::size_t spheres>
        struct RobotBase
        {
            using Configuration = FloatVector<dim>;
            using ConfigurationArray = std::array<float, dim>;
            struct alignas(32) ConfigurationBuffer : std::array<float, Configuration::num_scalars_rounded>
            {
            };
            // ConfigurationBlock<rake>: dim rows of rake lanes (lane l = interpolant l), as
            // FloatVector<rake, dim> (panda/fk.hh:11-12)
            template <std::size_t rake>
            struct ConfigurationBlock
            {
                std::array<std::array<float, rake>, dim> rows{};
                auto operator[](std::size_t i) noexcept -> std::array<float, rake> & { return rows[i]; }
                auto operator[](std::size_t i) const noexcept -> const std::array<float, rake> & { return rows[i]; }
                auto data() const noexcept -> const float * { return rows[0].data(); }
            };
            // Spheres<rake> (panda/fk.hh:94-102): world-frame centres per sphere and lane
            template <std::size_t rake>
            struct Spheres
            {
                std::array<std::array<float, rake>, spheres> x{}, y{}, z{};
            };

            static auto c_robot() noexcept -> vgpu_robot { return Derived::c_robot(); }

            // scale_configuration q * s_m + s_a (contracted to one fma per joint by the reference
            // release build, pinned by ref_probe "scale"); descale (q - s_a) * d_m
            static void scale_configuration(Configuration &q)
            {
                const auto &p = params();
                for (std::size_t j = 0; j < dim; ++j) q[j] = std::fma(q[j], p.s_m[j], p.s_a[j]);
            }
            static void descale_configuration(Configuration &q)
            {
                const auto &p = params();
                for (std::size_t j = 0; j < dim; ++j) q[j] = (q[j] - p.s_a[j]) * p.d_m[j];
            }
            template <std::size_t rake>
            static void scale_configuration_block(ConfigurationBlock<rake> &q)
            {
                const auto &p = params();
                for (std::size_t j = 0; j < dim; ++j)
                    for (std::size_t l = 0; l < rake; ++l) q[j][l] = std::fma(q[j][l], p.s_m[j], p.s_a[j]);
            }
            template <std::size_t rake>
            static void descale_configuration_block(ConfigurationBlock<rake> &q)
            {
                const auto &p = params();
                for (std::size_t j = 0; j < dim; ++j)
                    for (std::size_t l = 0; l < rake; ++l) q[j][l] = p.d_m[j] * (q[j][l] - p.s_a[j]);
            }

            // Robot::fkcc<rake>(env, block): true when every lane is collision-free (CPU rake)
            template <std::size_t rake>
            static auto fkcc(const collision::Environment &env, const ConfigurationBlock<rake> &q) -> bool
            {
                static_assert(rake == 8, "the CPU rake evaluates 8-lane blocks (FloatVectorWidth)");
                const vgpu_robot r = c_robot();
                int valid = 0;
                check(vgpu_cpu_fkcc_block(&r, env.handle(), q.data(), &valid), nullptr, "vgpu_cpu_fkcc_block");
                return valid != 0;
            }
            // Robot::fkcc_attach<rake>(env, block)
            template <std::size_t rake>
            static auto fkcc_attach(const collision::Environment &env, const ConfigurationBlock<rake> &q) -> bool
            {
                static_assert(rake == 8, "the CPU rake evaluates 8-lane blocks (FloatVectorWidth)");
                const vgpu_robot r = c_robot();
                int valid = 0;
                check(vgpu_cpu_fkcc_attach_block(&r, env.handle(), q.data(), &valid), nullptr,
                      "vgpu_cpu_fkcc_attach_block");
                return valid != 0;
            }
            // Robot::sphere_fk<rake>(block, out)
            template <std::size_t rake>
            static void sphere_fk(const ConfigurationBlock<rake> &q, Spheres<rake> &out)
            {
                static_assert(rake == 8, "the CPU rake evaluates 8-lane blocks (FloatVectorWidth)");
                const vgpu_robot r = c_robot();
                std::vector<float> soa(3 * spheres * rake);
                check(vgpu_cpu_sphere_fk_block(&r, q.data(), soa.data()), nullptr, "vgpu_cpu_sphere_fk_block");
                for (std::size_t s = 0; s < spheres; ++s)
                    for (std::size_t l = 0; l < rake; ++l)
                    {
                        out.x[s][l] = soa[(0 * spheres + s) * rake + l];
                        out.y[s][l] = soa[(1 * spheres + s) * rake + l];
                        out.z[s][l] = soa[(2 * spheres + s) * rake + l];
                    }
            }
            // Robot::eefk(q): end-effector position, quaternion x y z w (robot frame)
            static auto eefk(const ConfigurationArray &q) -> std::array<float, 7>
            {
                const vgpu_robot r = c_robot();
                std::array<float, 7> out{};
                check(vgpu_cpu_eefk(&r, q.data(), 1, out.data()), nullptr, "vgpu_cpu_eefk");
                return out;
            }

            // ---- batches on the MI355X (a Context-bound environment) ----
            // fkcc<8> of each configuration broadcast to the rake (validate(q) without the joint-limit
            // check, bindings/common.hh:172-182)
            static auto fkcc_batch(collision::Environment &env, const std::vector<Configuration> &q)
                -> std::vector<uint8_t>
            {
                std::vector<uint8_t> out(q.size());
                const vgpu_robot r = c_robot();
                vgpu_ctx *c = env.context().handle();
                check(vgpu_fkcc_host(c, &r, env.handle(), q.empty() ? nullptr : q[0].data(), q.size(), out.data()), c,
                      "vgpu_fkcc_host");
                return out;
            }
            static auto fkcc_attach_batch(collision::Environment &env, const std::vector<Configuration> &q)
                -> std::vector<uint8_t>
            {
                std::vector<uint8_t> out(q.size());
                const vgpu_robot r = c_robot();
                vgpu_ctx *c = env.context().handle();
                check(vgpu_fkcc_attach_host(c, &r, env.handle(), q.empty() ? nullptr : q[0].data(), q.size(),
                                            out.data()),
                      c, "vgpu_fkcc_attach_host");
                return out;
            }

        private:
            struct Params
            {
                std::array<float, dim> s_m{}, s_a{}, d_m{};
            };
            static auto params() -> const Params &
            {
                static const Params p = [] {
                    Params q;
                    const vgpu_robot r = Derived::c_robot();
                    check(vgpu_robot_scale_params(&r, q.s_m.data(), q.s_a.data(), q.d_m.data()), nullptr,
                          "vgpu_robot_scale_params");
                    return q;
                }();
                return p;
            }
        };

        // vamp::robots::PandaBase<X100, Y100, Z100> (robots/panda_base.hh:15-75)
        template <int BaseX100, int BaseY100, int BaseZ100>
        struct PandaBase : RobotBase<PandaBase<BaseX100, BaseY100, BaseZ100>, 7, 59>
        {
            static constexpr auto name = "panda";
            static constexpr std::size_t dimension = 7;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 59;
            static constexpr float base_x = static_cast<float>(BaseX100) / 100.0f;
            static constexpr float base_y = static_cast<float>(BaseY100) / 100.0f;
            static constexpr float base_z = static_cast<float>(BaseZ100) / 100.0f;
            static auto space_measure() noexcept -> float { return 878819.1112640093f; }  // panda/fk.hh:88-91
            static auto c_robot() noexcept -> vgpu_robot
            {
                return vgpu_robot{VGPU_ROBOT_PANDA, BaseX100, BaseY100, BaseZ100, 0, 0, 0};
            }
        };

        // vamp::robots::Fetch (robots/fetch.hh:8-48): 8 dof (prismatic torso first), 111 spheres
        struct Fetch : RobotBase<Fetch, 8, 111>
        {
            static constexpr auto name = "fetch";
            static constexpr std::size_t dimension = 8;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 111;
            static auto space_measure() noexcept -> float { return 269832.2635954135f; }
            static auto c_robot() noexcept -> vgpu_robot { return vgpu_robot{VGPU_ROBOT_FETCH, 0, 0, 0, 0, 0, 0}; }
        };

        // vamp::robots::UR5 (robots/ur5.hh): 6 dof, 36 spheres
        struct UR5 : RobotBase<UR5, 6, 36>
        {
            static constexpr auto name = "ur5";
            static constexpr std::size_t dimension = 6;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 36;
            static auto space_measure() noexcept -> float { return 700852.7173113511f; }
            static auto c_robot() noexcept -> vgpu_robot { return vgpu_robot{VGPU_ROBOT_UR5, 0, 0, 0, 0, 0, 0}; }
        };

        // vamp::robots::Baxter (robots/baxter.hh): 14-dof dual arm, 75 spheres, resolution 64
        // (its reference eefk is empty: eefk throws)
        struct Baxter : RobotBase<Baxter, 14, 75>
        {
            static constexpr auto name = "baxter";
            static constexpr std::size_t dimension = 14;
            static constexpr std::size_t resolution = 64;
            static constexpr std::size_t n_spheres = 75;
            static auto space_measure() noexcept -> float { return 89641415145.821f; }
            static auto c_robot() noexcept -> vgpu_robot { return vgpu_robot{VGPU_ROBOT_BAXTER, 0, 0, 0, 0, 0, 0}; }
        };

        // Two Pandas as one 14-dof robot (BASELINE configs[4]; no reference counterpart):
        // joints 0..6 = PandaBase<A>, 7..13 = PandaBase<B>; valid = fkcc_A && fkcc_B && no A-B
        // sphere overlap.  No fkcc_attach / eefk.
        template <int AX, int AY, int AZ, int BX, int BY, int BZ>
        struct PandaPair : RobotBase<PandaPair<AX, AY, AZ, BX, BY, BZ>, 14, 118>
        {
            static constexpr auto name = "panda_pair";
            static constexpr std::size_t dimension = 14;
            static constexpr std::size_t resolution = 32;
            static constexpr std::size_t n_spheres = 118;
            static auto space_measure() noexcept -> float { return 878819.1112640093f * 878819.1112640093f; }
            static auto c_robot() noexcept -> vgpu_robot
            {
                return vgpu_robot{VGPU_ROBOT_PANDA_PAIR, AX, AY, AZ, BX, BY, BZ};
            }
        };

        // robots/panda_grid.hh:10-41 -- this fork's default Panda stands at (2, 2, 0)
        struct Panda : PandaBase<200, 200, 0>
        {
        };
        struct Panda_0_0 : PandaBase<0, 0, 0>
        {
            static constexpr auto name = "panda_0_0";
        };
        struct Panda_1_0 : PandaBase<100, 0, 0>
        {
            static constexpr auto name = "panda_1_0";
        };
        struct Panda_2_2 : PandaBase<200, 200, 0>
        {
            static constexpr auto name = "panda_2_2";
        };
        // the configs[4] composite: arms 1 m apart along x
        using Panda_Pair = PandaPair<0, 0, 0, 100, 0, 0>;
    }  // namespace robots

    namespace rng
    {
        // rng::Halton<dim> (random/halton.hh:73-104) as a handle on the draw index; the planners
        // draw through the C ABI (vgpu_cpu_rrtc), which restates next() in closed form
        template <std::size_t dim>
        struct Halton
        {
            uint64_t index = 1;  // 1-based index of the next draw
            void reset() noexcept { index = 1; }
            void skip(uint64_t n) noexcept { index += n; }
        };
    }  // namespace rng

    namespace planning
    {
        // validate_vector<Robot, rake, resolution>(start, vector, distance, env) (validate.hh:23-65),
        // restated over Robot::fkcc<rake>: block = start + vector * (l + 1) / rake (contracted to an
        // fma by the reference release build), n = max(ceil(distance / rake * resolution), 1), the
        // first block through fkcc_attach when the environment has an attachment, then n - 1
        // back-steps block -= vector / (rake * n), early exit on the first invalid block.
        template <typename Robot, std::size_t rake, std::size_t resolution>
        inline auto validate_vector(const typename Robot::Configuration &start,
                                    const typename Robot::Configuration &vector, float distance,
                                    const collision::Environment &environment) -> bool
        {
            typename Robot::template ConfigurationBlock<rake> block;
            for (std::size_t i = 0; i < Robot::dimension; ++i)
                for (std::size_t l = 0; l < rake; ++l)
                    block[i][l] = std::fma(vector[i], static_cast<float>(l + 1) / static_cast<float>(rake), start[i]);
            const float nf = std::ceil(distance / static_cast<float>(rake) * static_cast<float>(resolution));
            const std::size_t n = nf > 1.0f ? static_cast<std::size_t>(nf) : 1;
            const bool valid = environment.attached() ? Robot::template fkcc_attach<rake>(environment, block)
                                                      : Robot::template fkcc<rake>(environment, block);
            if (!valid || n == 1) return valid;
            const auto backstep = vector / static_cast<float>(rake * n);
            for (std::size_t i = 1; i < n; ++i)
            {
                for (std::size_t j = 0; j < Robot::dimension; ++j)
                    for (std::size_t l = 0; l < rake; ++l) block[j][l] = block[j][l] - backstep[j];
                if (!Robot::template fkcc<rake>(environment, block)) return false;
            }
            return true;
        }

        // validate_motion<Robot, rake, resolution>(start, goal, env) (validate.hh:67-75)
        template <typename Robot, std::size_t rake, std::size_t resolution>
        inline auto validate_motion(const typename Robot::Configuration &start,
                                    const typename Robot::Configuration &goal,
                                    const collision::Environment &environment) -> bool
        {
            const auto vector = goal - start;
            return validate_vector<Robot, rake, resolution>(start, vector, vector.l2_norm(), environment);
        }

        // validate_motion<Robot, 8, Robot::resolution> for a batch of edges on the MI355X;
        // n_blocks receives n_e (interpolants = 8 * n_e) when given
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

        // RRTCSettings (planning/rrtc_settings.hh:5-20)
        struct RRTCSettings
        {
            float range = 2.;
            bool dynamic_domain = true;
            float radius = 4.;
            float alpha = 0.0001;
            float min_radius = 1.;
            bool balance = true;
            float tree_ratio = 1.;
            std::size_t max_iterations = 100000;
            std::size_t max_samples = 100000;
            bool start_tree_first = true;
        };

        // PlanningResult<dim> (planning/plan.hh)
        template <std::size_t dim>
        struct PlanningResult
        {
            std::vector<FloatVector<dim>> path;
            float cost = 0.0f;
            std::size_t nanoseconds = 0;
            std::size_t iterations = 0;
            std::vector<std::size_t> size;
        };

        // RRTC<Robot, rake, resolution>::solve (planning/rrtc.hh:16-249) on the CPU rake
        template <typename Robot, std::size_t rake, std::size_t resolution>
        struct RRTC
        {
            static_assert(rake == 8 && resolution == Robot::resolution,
                          "the CPU planner runs the robot's own rake 8 / resolution");
            using Configuration = typename Robot::Configuration;
            static constexpr auto dimension = Robot::dimension;

            static auto solve(const Configuration &start, const std::vector<Configuration> &goals,
                              const collision::Environment &environment, const RRTCSettings &settings,
                              rng::Halton<dimension> &rng) -> PlanningResult<dimension>
            {
                const vgpu_robot r = Robot::c_robot();
                const vgpu_rrtc_settings s{settings.range, settings.dynamic_domain, settings.radius,
                                           settings.alpha, settings.min_radius, settings.balance,
                                           settings.tree_ratio, settings.max_iterations, settings.max_samples,
                                           settings.start_tree_first};
                std::vector<float> g;
                for (const auto &x : goals) g.insert(g.end(), x.data(), x.data() + dimension);
                vgpu_plan_result res{};
                std::vector<float> path(4096 * dimension);
                for (;;)
                {
                    uint64_t idx = rng.index;
                    const int rc = vgpu_cpu_rrtc(&r, environment.handle(), start.data(), g.data(), goals.size(), &s,
                                                 &idx, path.data(), path.size() / dimension, &res);
                    if (rc == VGPU_OK)
                    {
                        rng.index = idx;
                        break;
                    }
                    if (res.path_len * dimension <= path.size()) check(rc, nullptr, "vgpu_cpu_rrtc");
                    path.resize(res.path_len * dimension);
                }
                PlanningResult<dimension> out;
                for (std::size_t i = 0; i < res.path_len; ++i) out.path.emplace_back(path.data() + i * dimension);
                out.cost = res.cost;
                out.nanoseconds = static_cast<std::size_t>(res.nanoseconds);
                out.iterations = res.iterations;
                out.size = {res.size[0], res.size[1]};
                return out;
            }
            static auto solve(const Configuration &start, const Configuration &goal,
                              const collision::Environment &environment, const RRTCSettings &settings,
                              rng::Halton<dimension> &rng) -> PlanningResult<dimension>
            {
                return solve(start, std::vector<Configuration>{goal}, environment, settings, rng);
            }
        };

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
        // validate_motion of every candidate edge on the MI355X
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
