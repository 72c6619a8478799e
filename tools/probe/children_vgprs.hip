// Development probe (tools/probe_children_vgprs.py): the VGPRs each of a robot's checks needs in a staged
// children kernel when compiled ALONE -- a robot type whose class 0 is that one check (the rest class 1),
// instantiated per check without an occupancy bound, so the code object's per-kernel .vgpr_count is the
// check's own need.  Not part of the library.
#include "../../mr-vamp_amd/csrc/vgpu_rake.hh"
#include "../../mr-vamp_amd/csrc/vgpu_staged.hh"

#include "../../mr-vamp_amd/csrc/gen/fetch_fk.inc"

namespace vgpu {
template <int C>
struct ProbeR {
    static constexpr int D = 8;
    static constexpr int kRes = 32;
    static constexpr int kChecks = fetch_n_checks;
    static constexpr int kWavesPerEU = 1;
    static constexpr int kChildWavesPerEU = 1;
    static constexpr unsigned kSourceKinds = 0x8u;  // validate tails
    using Mask = fetch_mask_t;
    static constexpr Mask kEnvChecks = fetch_env_check_bits;
    static constexpr int kClasses = 2;
    static constexpr int kClassOf[kChecks] = {
#define X(i) (i == C ? 0 : 1)
        X(0), X(1), X(2), X(3), X(4), X(5), X(6), X(7), X(8), X(9), X(10), X(11), X(12), X(13), X(14), X(15),
        X(16), X(17), X(18), X(19), X(20), X(21), X(22), X(23), X(24), X(25), X(26), X(27), X(28), X(29), X(30),
        X(31), X(32), X(33), X(34), X(35), X(36), X(37), X(38), X(39), X(40), X(41), X(42), X(43), X(44), X(45),
        X(46), X(47), X(48), X(49), X(50), X(51), X(52), X(53), X(54), X(55), X(56), X(57), X(58), X(59), X(60),
        X(61), X(62)
#undef X
    };
    static constexpr int kClassWaves[kClasses] = {1, 1};
    __device__ static __forceinline__ void sample(uint64_t, float v[8]) {}
    __device__ static __forceinline__ void head(const float* s, const float* g, int lane, float v[8])
    {
        const RakeD<8> rk = rake_setup_d<8, kRes>(s, g);
        rake_block_d<8>(s, rk, lane, 0, v);
    }
    __device__ static __forceinline__ void tail(const float* s, const float* g, int lane, int k, float v[8])
    {
        const RakeD<8> rk = rake_setup_d<8, kRes>(s, g);
        rake_block_d<8>(s, rk, lane, k, v);
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ Mask bound(const float* v, const EnvView& env, const Bases&)
    {
        return 0;
    }
    template <class Grp, bool EXT>
    __device__ static __forceinline__ bool children(int c, const float* v, const EnvView& env, const Bases&)
    {
        return fetch_children<Grp, EXT>(c, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], env, 0.0f, 0.0f, 0.0f);
    }
};
}  // namespace vgpu

template <int C>
void probe_one(const void* plan, const uint32_t* items, const EnvView* env, uint8_t* valid)
{
    using R = vgpu::ProbeR<C>;
    vgpu::SrcTailT<R> src{nullptr, nullptr, nullptr, nullptr};
    hipLaunchKernelGGL((vgpu::children_kernel<R, vgpu::SrcTailT<R>, false, 0>), dim3(1), dim3(256), 0, 0, src,
                       (const vgpu::StagedPlan*)plan, items, *env, Bases{}, valid);
}

template <int... C>
void probe_all(std::integer_sequence<int, C...>, const void* plan, const uint32_t* items, const EnvView* env,
               uint8_t* valid)
{
    (probe_one<C>(plan, items, env, valid), ...);
}

extern "C" void probe_children(const void* plan, const uint32_t* items, const EnvView* env, uint8_t* valid)
{
    probe_all(std::make_integer_sequence<int, fetch_n_checks>{}, plan, items, env, valid);
}
