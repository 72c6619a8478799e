// vgpu_device.hh -- CDNA4 device primitives of the motion-validation rake.
//
// Semantics follow the reference AVX2 path bit for bit (see DESIGN.md "Numerics"):
//   * vamp_sin/vamp_cos: FloatVector::sin()/cos() (reference vector/interface.hh:438-469)
//     in the Horner/FMA form the reference release build compiles them to;
//   * sqrt_host: collision::sqrt = v * rsqrt(v) (vector/avx.hh:411-415) where rsqrt is the
//     HOST CPU's _mm256_rsqrt_ps, emulated from a table probed on the host at context
//     creation (vgpu_api.cpp: probe_host_rsqrt);
//   * the collision predicate is the sign bit of the test value (avx.hh:385-389 testz);
//   * a rake group of G lanes (G = 8: one reference block; G = 1: one broadcast
//     configuration) shares its decisions: an obstacle loop stops when ALL lanes of the
//     group are culled, a check fires when ANY lane's test is negative
//     (collision/validity.hh:46-150).  For G = 8 the group is 8 consecutive lanes of a
//     wave64 (a DPP half-row) and the reductions are three DPP shuffles.
//
// Compiled with -ffp-contract=off: every fmaf below is intended, nothing else fuses.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define VGPU_CONST __attribute__((address_space(4)))

// ---- debug bounds checks (make DEBUG=1 -> -DVGPU_DEBUG; SURVEY §5 "race detection / sanitizers") ----
// Data-dependent indices (staged item lists, CAPT nodes / leaves / affordance ranges / grid cells, kNN
// tiles and candidates) are checked against their ranges.  A failed check adds 1 to dbg[0] and leaves its
// site id in dbg[1] (the first one); the kernel goes on with the index clamped, so a violation is counted
// and reported (vgpu_debug_violations) instead of faulting the GPU.  dbg: the environment blob's first
// two words (EnvView::base) or the kNN pool's.  Release builds compile the checks out.
enum : uint32_t {
    DBG_QUEUE_SLOT = 1, DBG_CHILD_GROUP, DBG_CHILD_ITEM, DBG_CAPT_CELL, DBG_CAPT_NODE, DBG_CAPT_LEAF,
    DBG_CAPT_AFF, DBG_DEFER_SLOT, DBG_DEFER_CLOUD, DBG_KNN_TILE, DBG_KNN_SUPER, DBG_KNN_VERTEX, DBG_KNN_QUERY
};
#ifdef VGPU_DEBUG
__device__ __forceinline__ uint32_t vgpu_dcheck(const void* dbg, bool ok, uint32_t site, uint32_t v, uint32_t hi)
{
    if (!ok && dbg) {
        uint32_t* w = (uint32_t*)dbg;
        atomicAdd(w, 1u);
        atomicCAS(w + 1, 0u, site);
    }
    return ok ? v : (hi ? hi - 1u : 0u);
}
#define VGPU_DCHECK(dbg, cond, site) (void)vgpu_dcheck((dbg), (cond), (site), 0u, 0u)
#define VGPU_DCLAMP(dbg, v, hi, site) vgpu_dcheck((dbg), (uint32_t)(v) < (uint32_t)(hi), (site), (uint32_t)(v), (uint32_t)(hi))
#else
#define VGPU_DCHECK(dbg, cond, site) ((void)0)
#define VGPU_DCLAMP(dbg, v, hi, site) (v)
#endif
constexpr int kDbgWords = 16;  // floats reserved at the start of an environment blob (debug words + padding)

// ---- group reductions -----------------------------------------------------------------
// A rake group is G consecutive lanes of a wave64 (G = 8 -> one DPP half-row).  The
// reductions are VALU DPP shuffles (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror), so the
// scalar unit stays free for loop control and obstacle loads.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

struct Grp1 {
    static constexpr int G = 1;
    __device__ static __forceinline__ uint32_t or_bits(uint32_t b) { return b; }
    __device__ static __forceinline__ bool any(bool p) { return p; }
    __device__ static __forceinline__ bool any_bits(uint32_t b) { return (b >> 31) != 0u; }
    __device__ static __forceinline__ float max(float v) { return v; }
};

struct Grp8 {
    static constexpr int G = 8;
    // OR of a small bit mask over the group's 8 lanes
    __device__ static __forceinline__ uint32_t or_bits(uint32_t b)
    {
        int x = (int)b;
        x |= dpp_i<0xB1>(x);
        x |= dpp_i<0x4E>(x);
        x |= dpp_i<0x141>(x);
        return (uint32_t)x;
    }
    // any lane of the group with its sign bit set (bits OR-reduced over the DPP half-row)
    __device__ static __forceinline__ bool any_bits(uint32_t b)
    {
        int x = (int)b;
        x |= dpp_i<0xB1>(x);
        x |= dpp_i<0x4E>(x);
        x |= dpp_i<0x141>(x);
        return x < 0;
    }
    __device__ static __forceinline__ bool any(bool p)
    {
        int x = p ? 1 : 0;
        x |= dpp_i<0xB1>(x);   // quad_perm [1,0,3,2]
        x |= dpp_i<0x4E>(x);   // quad_perm [2,3,0,1]
        x |= dpp_i<0x141>(x);  // row_half_mirror
        return x != 0;
    }
    // max of NON-NEGATIVE floats (max_extent = |c| + r > 0, or +inf): their bit patterns
    // order like the values, so an unsigned max folds into one v_max_u32_dpp per step.
    __device__ static __forceinline__ float max(float v)
    {
        uint32_t u = __float_as_uint(v);
        u = umax(u, (uint32_t)dpp_i<0xB1>((int)u));
        u = umax(u, (uint32_t)dpp_i<0x4E>((int)u));
        u = umax(u, (uint32_t)dpp_i<0x141>((int)u));
        return __uint_as_float(u);
    }
};

// Groups of the staged kernels with a point cloud: CAPT queries the cell grid cannot decide are
// queued per wave and resolved in batches (capt_defer_* below) instead of inline.  TAG = the queue
// tag of env_bits calls that pass none: -1 resolves them inline (bound kernels: their generated
// calls pass the check's bit), kChildTag marks "a child of this lane hit" (children kernels).
template <class G, int TAG>
struct Deferred : G {
    static constexpr int kDeferTag = TAG;
};
template <class G, class = void>
struct DeferTagOf {
    static constexpr bool on = false;
    static constexpr int tag = -1;
};
template <class G>
struct DeferTagOf<G, std::void_t<decltype(G::kDeferTag)>> {
    static constexpr bool on = true;
    static constexpr int tag = G::kDeferTag;
};
constexpr int kChildTag = 63;
constexpr int kTagDefault = -2;  // env_bits: the group type's default tag

// ---- FloatVector::sin()/cos() -----------------------------------------------------------
__device__ __forceinline__ float vamp_sin(float x)
{
    const float c1 = -0x1.ea200ap-2f;  // (float)-0.478637850138
    const float c2 = 0x1.80f17p+0f;    // (float) 1.503684069359
    const float c3 = 0x1.7c019ap-7f;   // (float) 0.011596870476
    const float c4 = 0x1.1ec4f2p-3f;   // (float) 0.140024078368
    const float c5 = 0x1.54952ep-1f;   // (float) 0.665200679751
    const float p = x * __builtin_fmaf(__builtin_fabsf(x), c1, c2);
    const float ap = __builtin_fabsf(p);
    return p * __builtin_fmaf(ap, __builtin_fmaf(ap, c3, c4), c5);
}

__device__ __forceinline__ float vamp_cos(float x)
{
    const float PI = 0x1.921fb6p+1f;       // (float)3.14159265359
    const float HALF_PI = 0x1.921fb6p+0f;  // (float)(PI / 2.)
    const float TWO_PI = 0x1.921fb6p+2f;   // (float)(2 * PI)
    float v = x + HALF_PI;
    v = v - ((v >= PI) ? TWO_PI : 0.0f);
    return vamp_sin(v);
}

// ---- rng::Halton<dim>::next (random/halton.hh:73-104), closed form ------------------------------
// Draw k (1-based: the k-th next() of a fresh sampler).  The reference restarts its numerators
// every 1,000,000 draws and rotates the bases left; since the reset sets iterations = 0 after
// the increment, every cycle after the first is 1,000,001 draws long.  Within a cycle, draw i
// has coordinate d = radical inverse of i in base primes[(d + cycle) % dim], and the
// reference's n / d are exact float integers, so one float division reproduces it.
constexpr uint32_t kHaltonPrimes[16] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59};
constexpr uint64_t kHaltonCycle = 1000000u;

__device__ __forceinline__ void halton_index(uint64_t k, uint32_t& idx, uint32_t& cycle)
{
    if (k <= kHaltonCycle) {
        idx = (uint32_t)k;
        cycle = 0;
    } else {
        const uint64_t kk = k - kHaltonCycle - 1;
        cycle = (uint32_t)(1 + kk / (kHaltonCycle + 1));
        idx = (uint32_t)(kk % (kHaltonCycle + 1)) + 1u;
    }
}

// Radical inverse of idx (< 2^24: idx <= 1,000,001 within a cycle) in base b.  The digit
// division uses a float reciprocal estimate of idx / b (exact float operands; |error| < 1) and one
// integer correction step, so every quotient and remainder is the exact integer one -- no
// hardware integer divide (a ~40-instruction sequence on CDNA) per digit.
__device__ __forceinline__ float halton_coord(uint32_t idx, uint32_t b)
{
    const float inv = 1.0f / (float)b;
    uint32_t num = 0, den = 1;
    while (idx) {
        uint32_t q = (uint32_t)((float)idx * inv);
        int32_t r = (int32_t)(idx - q * b);
        if (r < 0) {
            q -= 1u;
            r += (int32_t)b;
        } else if (r >= (int32_t)b) {
            q += 1u;
            r -= (int32_t)b;
        }
        num = num * b + (uint32_t)r;
        den *= b;
        idx = q;
    }
    return (float)num / (float)den;
}

// ---- environment view ----------------------------------------------------------------------
// collision::Environment<float> on the device: one section per obstacle type, each sorted
// ascending by min_distance (environment.hh:40-66) and terminated by kObsPad sentinel records
// whose min_distance is +inf (never evaluated; lets the loops prefetch past the end).
// Records (float32, field 0 = min_distance):
//   sphere   pair blocks of 16: md_a md_b x_a x_b y_a y_b z_a z_b r_a r_b (records 2k, 2k + 1; scan_spheres)
//   capsule  stride 16: md x1 y1 z1 xv yv zv r rdv | bx by bz bR            (z-capsule: same)
//   cuboid   stride 20: md x y z a1x a1y a1z a2x a2y a2z a3x a3y a3z r1 r2 r3 | bx by bz bR   (z-cuboid: same)
// (bx by bz bR: the record's bounding sphere, vgpu_api.cpp obstacle_bound -- not part of the reference's record;
// scan_type skips a record for a wave none of whose live lanes' spheres reach it)
enum : int { OBS_SPHERE = 0, OBS_CAPSULE = 1, OBS_ZCAPSULE = 2, OBS_CUBOID = 3, OBS_ZCUBOID = 4, OBS_TYPES = 5 };
constexpr int kObsStride[OBS_TYPES] = {8, 16, 16, 20, 20};  // spheres: 16 floats per PAIR of records
constexpr int kSphereBlock = 16;
constexpr int kObsBound[OBS_TYPES] = {-1, 9, 9, 16, 16};  // first bounding-sphere field (-1: none)
constexpr int kObsPad = 8;  // >= 2 * VGPU_SCAN_UNROLL - 1 (the loop's prefetch reach)

struct EnvView {
    const VGPU_CONST float* obs[OBS_TYPES];
    const uint32_t* lut;  // host rsqrt table, 2 << kbits entries
    int n[OBS_TYPES];
    int kbits;
    // heightfields and point clouds (no cull; evaluated after the five primitive types,
    // validity.hh:133-148).  Headers are kExtHdr floats each (layouts below); data / tree
    // arrays are addressed as float offsets from `base` (the environment's device buffer).
    const VGPU_CONST float* hf;
    const VGPU_CONST float* pc;
    const float* base;
    int n_hf, n_pc;
    // the environment's attachment (Environment::attachments, environment.hh:21): frame tf =
    // x y z qx qy qz qw (+1 pad), then n_att spheres x y z r relative to it (kAttHdr floats in)
    const VGPU_CONST float* att;
    int n_att;
    // levels of the first point cloud's split tree staged in this workgroup's LDS by
    // capt_stage_lds (0: none -- the host-built view, and kernels that do not stage)
    int pc_lds_levels;
    // near sets (env_near / env_bits_near): nonzero when the primitive records number at most kNearMax; record i
    // of type t is bit near_base[t] + i
    int near_ok;
    int near_base[OBS_TYPES];
};
constexpr int kNearMax = 64;
constexpr int kAttHdr = 8;
constexpr int kExtHdr = 32;
// heightfield header: x y z xs ys zs xd yd xd2 yd2 (floats) | data_off cells (uint32 bits)
enum : int { HF_X = 0, HF_Y, HF_Z, HF_XS, HF_YS, HF_ZS, HF_XD, HF_YD, HF_XD2, HF_YD2, HF_OFF, HF_CELLS };
// point-cloud (CAPT) header: top lower xyz, top upper xyz, r_point | nlog2, tests_off, aabbs_off,
// starts_off, aff_off (uint32 bits).  aff = [n_aff][3][8] floats (x8 y8 z8), 16-B aligned.
// Device copies add the cell grid (vgpu_capt_grid.hip): origin xyz, 1/h, cell counts (uint32 and
// float), the bound unit, and cells_off (0 = no grid; the cell bounds, see PC_GNODES and capt_cell_index).
enum : int {
    PC_TOP = 0, PC_RPOINT = 6, PC_NLOG2 = 7, PC_TESTS, PC_AABBS, PC_STARTS, PC_AFF,
    PC_GX = 12, PC_GY, PC_GZ, PC_GINVH, PC_GNX, PC_GNY, PC_GNZ, PC_GNXF, PC_GNYF, PC_GNZF, PC_GUNIT, PC_GCELLS,
    PC_GBRICK,  // 1: cells stored in 4 x 4 x 4 bricks (capt_cell_index), 0: x-fastest rows
    PC_GNODES   // 0: one uint2 {bounds, node} per cell; else the offset of a separate node plane (one uint32 per
                // cell) and cells_off holds the bounds alone, one uint32 per cell
};
// storage index of cell (ix, iy, iz): x-fastest rows, or 4 x 4 x 4 bricks of 64 consecutive cells (brick-major,
// x-fastest bricks; every count a multiple of 4) -- a sphere's next children fall in the same or a nearby brick
__host__ __device__ __forceinline__ uint32_t capt_cell_index(uint32_t ix, uint32_t iy, uint32_t iz, uint32_t nx,
                                                             uint32_t ny, bool brick)
{
    if (!brick) return (iz * ny + iy) * nx + ix;
    return ((((iz >> 2) * (ny >> 2) + (iy >> 2)) * (nx >> 2) + (ix >> 2)) << 6) | ((iz & 3u) << 4) | ((iy & 3u) << 2) |
           (ix & 3u);
}
// Cell bounds are scaled by these before they decide a query (vgpu_capt_grid.hip: the float
// rounding of the distance and of the bound itself is < 1e-6 relative)
constexpr float kGridLoFac = 0.9999f, kGridHiFac = 1.0001f;

// Robot base offsets of a staged pass (robots/panda/fk.hh:109-111, added to world-frame centres):
// x y z of the robot -- and of the second arm, for the two-Panda composite's inter-arm checks
struct Bases {
    float x, y, z, x2, y2, z2;
};

__device__ __forceinline__ bool signbit_f(float v) { return (__float_as_uint(v) >> 31) != 0u; }

// v * rsqrt_host(v); returns a NaN with the sign bit (x86 "indefinite") for 0 / denormal v,
// exactly what v * _mm256_rsqrt_ps(v) gives on the host (rsqrt(0) = +inf, 0 * inf).
__device__ __forceinline__ float sqrt_host(float v, const uint32_t* __restrict__ lut, int kbits)
{
    const uint32_t b = __float_as_uint(v);
    const int e = (int)((b >> 23) & 0xFFu);
    const uint32_t p = (uint32_t)e & 1u;
    const uint32_t idx = (p << kbits) | ((b & 0x7FFFFFu) >> (23 - kbits));
    const uint32_t t = lut[idx];
    const int shift = (e - (int)(126u + p)) / 2;
    const float r = __uint_as_float(t - ((uint32_t)shift << 23));
    // x86: rsqrt(0 / denormal) = +inf -> 0*inf = default NaN (sign set), denormal*inf = +inf;
    // inf/NaN inputs give NaN.  All of these mean "no cull" to the caller.
    if (e == 0) return (b & 0x7FFFFFFFu) == 0u ? __uint_as_float(0xFFC00000u) : __uint_as_float(0x7F800000u);
    return (e == 255) ? __uint_as_float(0xFFC00000u) : v * r;
}

// dot_3 / dot_2 (reference collision/math.hh:10-27) in the release build's contracted form
__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2)
{
    return __builtin_fmaf(a0, b0, __builtin_fmaf(a2, b2, a1 * b1));
}
__device__ __forceinline__ float dot2(float a0, float a1, float b0, float b1)
{
    return __builtin_fmaf(a0, b0, a1 * b1);
}

// sphere_sphere_sql2 (sphere_sphere.hh:10-22)
__device__ __forceinline__ float sphere_sphere(float ax, float ay, float az, float ar, float bx, float by,
                                               float bz, float br)
{
    const float xs = ax - bx, ys = ay - by, zs = az - bz;
    const float rs = ar + br;
    return __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
}

__device__ __forceinline__ float max0(float v) { return (v > 0.0f) ? v : 0.0f; }

// sphere_environment_in_collision (collision/validity.hh:46-150) for one lane of a rake group.
//
// Returns this lane's hit over exactly the obstacles the reference evaluates for the whole
// group; the group result (the reference's return value) is Grp::any() of it, taken by the
// caller.  Reference loop per type: `if (all lanes: min_distance - max_extent >= +0) break;
// if (any lane: test < 0) return true;`.  Since the float difference of two floats is >= +0
// exactly when min_distance >= max_extent, "all lanes culled" == min_distance >= the group
// maximum of max_extent (a NaN/inf extent -- 0 or denormal |c|^2 -- never culls: +inf).  The
// `return true` only ends work early: a lane stops at its own first hit, which leaves the
// group OR unchanged.
// One obstacle type: evaluates records while md < emax (this lane's group prefix), two per
// iteration, the next pair's scalar loads issued before the current pair is tested.  The
// body is branch-free per lane; the loop exits when no lane of the wave has anything left.
#ifndef VGPU_SCAN_UNROLL
#define VGPU_SCAN_UNROLL 2  // records per loop trip (A/B on MI355X: 1 -> 5.15 ms, 2 -> 4.97, 4 -> 5.17)
#endif
static_assert(kObsPad >= 2 * VGPU_SCAN_UNROLL - 1, "sentinel padding must cover the prefetch");
// (round 5, A/B on MI355X: loading the next trip's whole sphere records ahead as well -- the tests no longer
// waiting on their own records' scalar loads -- was slower: set B 2.32 -> 2.39-2.41 ms, profiles/r05d_ab.log)
template <int S>
struct ObsRec {
    float v[S];
};
// obstacle records are read through the scalar cache (address space 4, s_load): every lane of a wave reads
// the same record, one s_load into SGPRs the tests use directly (a per-workgroup LDS copy measured 7-11 %
// slower in round 3: a ds_read broadcast per field plus the copy and barrier)
// Records with a bounding sphere (kObsBound) are tested only when some live lane's sphere (x, y, z, r)
// reaches it: |p - b| <= r + bR is implied by the test firing (obstacle_bound), so a wave-uniform skip of
// the others leaves acc bit-identical.  VGPU_OBS_PREFILTER=0 restores the unconditional tests (A/B).
#ifndef VGPU_OBS_PREFILTER
#define VGPU_OBS_PREFILTER 1
#endif
template <int TYPE, class TestFn>
__device__ __forceinline__ uint32_t scan_type(const VGPU_CONST float* o, float emax, uint32_t acc, TestFn test,
                                              float x, float y, float z, float r)
{
    // The lane state is kept as VALU bit masks (acc: sign bit = hit) instead of per-lane bools:
    // combining divergent bools costs a 64-bit SALU op each, and the scalar unit -- shared by
    // the waves of a SIMD -- was the busiest pipe of these kernels.
    constexpr int S = kObsStride[TYPE];
    constexpr int U = VGPU_SCAN_UNROLL;
    constexpr int B = VGPU_OBS_PREFILTER ? kObsBound[TYPE] : -1;
    using Rec = ObsRec<S>;  // one record: a single s_load per field group
    const VGPU_CONST Rec* p = (const VGPU_CONST Rec*)o;
    float md[U];
#pragma unroll
    for (int u = 0; u < U; ++u) md[u] = p[u].v[0];
    for (;;) {
        uint32_t live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) live[u] = (md[u] < emax) ? 0xFFFFFFFFu : 0u;
        // md is sorted: live[u] implies live[0].  ballot of an opaque value: otherwise
        // instcombine folds the test back into an i1 AND, which the backend lowers as
        // compare -> v_cndmask -> compare
        uint32_t pend = live[0] & ~acc;
        __asm__("" : "+v"(pend));
        if (__builtin_amdgcn_ballot_w64((int)pend < 0) == 0) break;
        float nmd[U];
#pragma unroll
        for (int u = 0; u < U; ++u) nmd[u] = p[U + u].v[0];  // prefetch (sentinel-padded)
        uint32_t hit = 0u;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (B >= 0) {
                const float dx = x - p[u].v[B], dy = y - p[u].v[B + 1], dz = z - p[u].v[B + 2];
                const float lim = r + p[u].v[B + 3];
                // NaN distances count as near (the exact test decides them)
                uint32_t near = (dot3(dx, dy, dz, dx, dy, dz) > lim * lim) ? 0u : live[u] & ~acc;
                __asm__("" : "+v"(near));
                if (__builtin_amdgcn_ballot_w64((int)near < 0) != 0) hit |= __float_as_uint(test(p[u].v)) & live[u];
            } else {
                hit |= __float_as_uint(test(p[u].v)) & live[u];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) md[u] = nmd[u];
        acc |= hit;
        p += U;
    }
    return acc;
}

// Spheres, two records per block and per loop trip: one s_load brings both records' fields.  The two tests
// are sphere_sphere's operations in its order (bit-identical values).  VGPU_SPHERE_PACKED=1 runs them as
// packed FP32 (v_pk_add / v_pk_mul / v_pk_fma_f32 on the block's SGPR pairs: 7 VALU instructions for two
// records instead of 14) -- measured SLOWER on MI355X (set B 2.29-2.31 vs 2.22-2.25 ms unpacked,
// profiles/r05g_panda_ab.log): a packed FP32 instruction costs the issue of two (MI355X_MICROARCH.md), and
// the duplicated lane operands cost VGPRs.
typedef float f2v __attribute__((ext_vector_type(2)));
struct SphereBlk {
    f2v md, x, y, z, r, pad[3];
};
static_assert(sizeof(SphereBlk) == kSphereBlock * 4, "sphere block layout");
#ifndef VGPU_SPHERE_PACKED
#define VGPU_SPHERE_PACKED 0
#endif
__device__ __forceinline__ uint32_t scan_spheres(const VGPU_CONST float* o, float emax, uint32_t acc, float x, float y,
                                                 float z, float r)
{
    const VGPU_CONST SphereBlk* p = (const VGPU_CONST SphereBlk*)o;
    f2v md = p->md;
    if constexpr (VGPU_SPHERE_PACKED) {
        const f2v X = {x, x}, Y = {y, y}, Z = {z, z}, R = {r, r};
        for (;;) {
            const uint32_t la = (md.x < emax) ? 0xFFFFFFFFu : 0u, lb = (md.y < emax) ? 0xFFFFFFFFu : 0u;
            uint32_t pend = la & ~acc;  // sorted: lb implies la
            __asm__("" : "+v"(pend));
            if (__builtin_amdgcn_ballot_w64((int)pend < 0) == 0) break;
            const f2v nmd = p[1].md;  // prefetch (sentinel-padded)
            const f2v xs = p->x - X, ys = p->y - Y, zs = p->z - Z, rs = p->r + R;
            f2v d = ys * ys;  // sphere_sphere: fma(-rs, rs, fma(xs, xs, fma(zs, zs, ys * ys)))
            d = __builtin_elementwise_fma(zs, zs, d);
            d = __builtin_elementwise_fma(xs, xs, d);
            d = __builtin_elementwise_fma(-rs, rs, d);
            acc |= (__float_as_uint(d.x) & la) | (__float_as_uint(d.y) & lb);
            md = nmd;
            ++p;
        }
    } else {
        for (;;) {
            const uint32_t la = (md.x < emax) ? 0xFFFFFFFFu : 0u, lb = (md.y < emax) ? 0xFFFFFFFFu : 0u;
            uint32_t pend = la & ~acc;
            __asm__("" : "+v"(pend));
            if (__builtin_amdgcn_ballot_w64((int)pend < 0) == 0) break;
            const f2v nmd = p[1].md;
            const f2v bx = p->x, by = p->y, bz = p->z, br = p->r;
            const uint32_t ha = __float_as_uint(sphere_sphere(bx.x, by.x, bz.x, br.x, x, y, z, r));
            const uint32_t hb = __float_as_uint(sphere_sphere(bx.y, by.y, bz.y, br.y, x, y, z, r));
            acc |= (ha & la) | (hb & lb);
            md = nmd;
            ++p;
        }
    }
    return acc;
}

// _mm256_max_ps / _mm256_min_ps operand semantics (a NaN first operand yields the second)
__device__ __forceinline__ float mm_max(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float mm_min(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t hdr_u(const VGPU_CONST float* h, int i) { return __float_as_uint(h[i]); }

// sphere_heightfield (sphere_heightfield.hh:9-30) in the release build's form (ref_probe "hf"):
// xs = floor(clamp(fma(xs, hx - x, xd2), 0, xd)), index = fma(ys, xd, xs), value = (z - r) -
// fma(zs, data[index], hz).  An index outside the data (undefined in the reference, whose
// gather reads past the array) is reported as a collision.
__device__ __forceinline__ bool hf_lane(const VGPU_CONST float* h, const float* __restrict__ base, float x, float y,
                                        float z, float r)
{
    const float xo = h[HF_X] - x, yo = h[HF_Y] - y;
    const float xs = __builtin_floorf(mm_min(mm_max(__builtin_fmaf(h[HF_XS], xo, h[HF_XD2]), 0.0f), h[HF_XD]));
    const float ys = __builtin_floorf(mm_min(mm_max(__builtin_fmaf(h[HF_YS], yo, h[HF_YD2]), 0.0f), h[HF_YD]));
    const float fi = __builtin_fmaf(ys, h[HF_XD], xs);
    const uint32_t cells = hdr_u(h, HF_CELLS);
    if (!(fi >= 0.0f && fi < (float)cells)) return true;
    const uint32_t idx = (uint32_t)__builtin_rintf(fi);
    if (idx >= cells) return true;
    const float zh = base[hdr_u(h, HF_OFF) + idx];
    return signbit_f((z - r) - __builtin_fmaf(h[HF_ZS], zh, h[HF_Z]));
}

// The top VGPU_CAPT_LDS_LEVELS levels of a point cloud's split tree (tests[0 .. 2^L - 2]) staged in
// LDS per workgroup: the descent's first L dependent loads become LDS reads instead of divergent
// L2 gathers (SURVEY §8(a) a10 / north_star: "CAPT split planes staged in LDS").
#ifndef VGPU_CAPT_LDS_LEVELS
#define VGPU_CAPT_LDS_LEVELS 0  // with the cell grid; 12 measured best without it (r02)
#endif
constexpr uint32_t kCaptLdsNodes = VGPU_CAPT_LDS_LEVELS > 0 ? (1u << VGPU_CAPT_LDS_LEVELS) - 1u : 1u;

__device__ __forceinline__ float* capt_lds()
{
    __shared__ float top[kCaptLdsNodes];  // one per workgroup of every kernel that stages
    return top;
}

// Cooperative copy of the first point cloud's top levels; every thread of the workgroup must call
// it (it ends in a barrier) before any early return.
__device__ __forceinline__ void capt_stage_lds(EnvView& env)
{
    if (VGPU_CAPT_LDS_LEVELS > 0 && env.n_pc > 0) {
        const uint32_t nlog2 = hdr_u(env.pc, PC_NLOG2);
        const uint32_t L = nlog2 < (uint32_t)VGPU_CAPT_LDS_LEVELS ? nlog2 : (uint32_t)VGPU_CAPT_LDS_LEVELS;
        const uint32_t nodes = (1u << L) - 1u;
        const float* __restrict__ t = env.base + hdr_u(env.pc, PC_TESTS);
        float* top = capt_lds();
        for (uint32_t i = threadIdx.x; i < nodes; i += blockDim.x) top[i] = t[i];
        env.pc_lds_levels = (int)L;
    }
    __syncthreads();
}

// one lane of CAPT::collides_simd (capt.hh:457-541): top-box test inflated by r, descent of
// the implicit split tree (axis cycles x, y, z), leaf point-volume box test with
// (r + r_point)^2, then the leaf's affordance vectors, inclusive distance test.  Sums of
// squares in the FloatVector form fma(d0, d0, fma(d2, d2, d1 * d1)) (ref_probe "sql2").
//
// Cell grid (device copies, vgpu_capt_grid.hip): the centre's cell holds [lo, hi] -- over every
// leaf the cell can descend to, the least distance from the cell to an affordance of that leaf,
// and the largest over those leaves of the least farthest-corner distance to one -- and the
// deepest split node whose region contains the whole cell.  (r + r_point)^2 below lo^2 is a miss
// and above hi^2 a hit, whatever leaf the centre reaches (the leaf box always contains its
// affordances, so its test never decides alone); anything between descends from that node.
// Same answer as the reference's traversal, for ~5x fewer dependent loads per query.
// lds_levels > 0: the tree's first lds_levels levels are read from capt_lds().
// Top box + cell grid: 0 = miss, 1 = hit, 2 = undecided -- node = the split node the traversal
// starts from (0: the root, without a grid or outside it).
__device__ __forceinline__ int capt_decide(const VGPU_CONST float* h, float x, float y, float z, float r,
                                           const float* __restrict__ base, uint32_t& node)
{
    node = 0u;
    if (!((x + r >= h[0]) && (x - r <= h[3]) && (y + r >= h[1]) && (y - r <= h[4]) && (z + r >= h[2]) &&
          (z - r <= h[5])))
        return 0;
    const uint32_t goff = hdr_u(h, PC_GCELLS);
    if (goff) {
        const float fx = (x - h[PC_GX]) * h[PC_GINVH];
        const float fy = (y - h[PC_GY]) * h[PC_GINVH];
        const float fz = (z - h[PC_GZ]) * h[PC_GINVH];
        if (fx >= 0.0f && fy >= 0.0f && fz >= 0.0f && fx < h[PC_GNXF] && fy < h[PC_GNYF] && fz < h[PC_GNZF]) {
            uint32_t cell = capt_cell_index((uint32_t)fx, (uint32_t)fy, (uint32_t)fz, hdr_u(h, PC_GNX), hdr_u(h, PC_GNY),
                                            hdr_u(h, PC_GBRICK) != 0u);
            cell = VGPU_DCLAMP(base, cell, hdr_u(h, PC_GNX) * hdr_u(h, PC_GNY) * hdr_u(h, PC_GNZ), DBG_CAPT_CELL);
            const uint32_t noff = hdr_u(h, PC_GNODES);
            const uint32_t rec = noff ? ((const uint32_t*)(base + goff))[cell] : ((const uint2*)(base + goff))[cell].x;
            const float rr = r + h[PC_RPOINT];
            const float rc = rr * rr;
            const float lo = (float)(rec & 0xFFFFu) * h[PC_GUNIT];
            if (rc < lo * lo * kGridLoFac) return 0;
            const uint32_t hq = rec >> 16;
            const float hi = (float)hq * h[PC_GUNIT];
            if (hq != 0xFFFFu && rc > hi * hi * kGridHiFac) return 1;
            node = noff ? ((const uint32_t*)(base + noff))[cell] : ((const uint2*)(base + goff))[cell].y;
        }
    }
    return 2;
}

// The reference's traversal below `node` (whose region contains the centre): descent, leaf box,
// affordance scan.
__device__ __forceinline__ bool capt_resolve(const VGPU_CONST float* h, const float* __restrict__ base, float x,
                                             float y, float z, float r, uint32_t node, int lds_levels = 0)
{
    const int nlog2 = (int)hdr_u(h, PC_NLOG2);
    const float* __restrict__ tests = base + hdr_u(h, PC_TESTS);
    const float rr = r + h[PC_RPOINT];
    const float rc = rr * rr;
    // node: a split node or, when the whole grid cell lies in one leaf's region, that leaf
    uint32_t idx = VGPU_DCLAMP(base, node, (2u << nlog2) - 1u, DBG_CAPT_NODE);
    int i = 31 - __builtin_clz(idx + 1u);  // the node's level; the axis of level i is i % 3
    const int rot = i % 3;
    float a = rot == 0 ? x : (rot == 1 ? y : z);
    float b = rot == 0 ? y : (rot == 1 ? z : x);
    float c = rot == 0 ? z : (rot == 1 ? x : y);
    if (lds_levels > i) {
        const float* top = capt_lds();
        for (; i < lds_levels; ++i) {
            idx = 2u * idx + 1u + ((a >= top[idx]) ? 1u : 0u);
            const float t = a;
            a = b;
            b = c;
            c = t;
        }
    }
    for (; i < nlog2; ++i) {
        idx = 2u * idx + 1u + ((a >= tests[idx]) ? 1u : 0u);
        const float t = a;
        a = b;
        b = c;
        c = t;
    }
    uint32_t leaf = nlog2 ? idx - ((1u << nlog2) - 1u) : 0u;
    leaf = VGPU_DCLAMP(base, leaf, 1u << nlog2, DBG_CAPT_LEAF);
    const float* __restrict__ box = base + hdr_u(h, PC_AABBS) + 6u * leaf;
    const float d0 = x - mm_min(mm_max(x, box[0]), box[3]);
    const float d1 = y - mm_min(mm_max(y, box[1]), box[4]);
    const float d2 = z - mm_min(mm_max(z, box[2]), box[5]);
    if (!(__builtin_fmaf(d0, d0, __builtin_fmaf(d2, d2, d1 * d1)) <= rc)) return false;
    const uint32_t* __restrict__ starts = (const uint32_t*)(base + hdr_u(h, PC_STARTS));
    const uint32_t s = starts[leaf], e = starts[leaf + 1];
    VGPU_DCHECK(base, s <= e && e <= starts[1u << nlog2], DBG_CAPT_AFF);
    const float4* __restrict__ aff = (const float4*)(base + hdr_u(h, PC_AFF));
    for (uint32_t i = s; i < e; ++i) {
        const float4* v = aff + 6u * i;
        const float4 x0 = v[0], x1 = v[1], y0 = v[2], y1 = v[3], z0 = v[4], z1 = v[5];
        const float px[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const float py[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
        const float pz[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
        bool any = false;
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const float dx = px[l] - x, dy = py[l] - y, dz = pz[l] - z;
            any |= __builtin_fmaf(dx, dx, __builtin_fmaf(dz, dz, dy * dy)) <= rc;
        }
        if (any) return true;
    }
    return false;
}

__device__ __forceinline__ bool capt_lane(const VGPU_CONST float* h, const float* __restrict__ base, float x, float y,
                                          float z, float r, int lds_levels = 0)
{
    uint32_t node;
    const int d = capt_decide(h, x, y, z, r, base, node);
    return d == 2 ? capt_resolve(h, base, x, y, z, r, node, lds_levels) : d == 1;
}

// ---- deferred CAPT queries (staged kernels, kStagedBlock = 256 threads = 4 waves) ----------------
// A wave appends its undecided queries (centre, radius, start node, owner thread, tag, cloud) to
// its LDS queue; when a push would overflow, and at the end of the kernel's collision work, the
// whole wave resolves the queue one entry per lane (capt_defer_flush), OR-ing a hit into the
// owner's 64-bit tag mask.  Divergent single-lane traversals become full-wave batches.
constexpr int kDeferCap = 128;
constexpr int kDeferWaves = 4;
struct DeferQ {
    float x[kDeferCap], y[kDeferCap], z[kDeferCap], r[kDeferCap];
    uint32_t node[kDeferCap], meta[kDeferCap];  // meta: owner thread | tag << 8 | cloud << 14
};
__device__ __forceinline__ DeferQ* defer_q()
{
    __shared__ DeferQ q[kDeferWaves];
    return q;
}
__device__ __forceinline__ uint32_t* defer_cnt()
{
    __shared__ uint32_t c[kDeferWaves];
    return c;
}
__device__ __forceinline__ unsigned long long* defer_hits()
{
    __shared__ unsigned long long m[kDeferWaves * 64];
    return m;
}
// every thread of the block, before any return
__device__ __forceinline__ void capt_defer_init()
{
    defer_hits()[threadIdx.x] = 0ull;
    if ((threadIdx.x & 63) == 0) defer_cnt()[threadIdx.x >> 6] = 0u;
    __builtin_amdgcn_wave_barrier();
}
// the active lanes of the wave resolve every queued entry (once per kernel, at the end)
__device__ __forceinline__ void capt_defer_flush(const VGPU_CONST float* pc, const float* base, int lds_levels)
{
    const uint32_t w = threadIdx.x >> 6;
    DeferQ& q = defer_q()[w];
    const uint32_t cnt = (uint32_t)__builtin_amdgcn_readfirstlane((int)defer_cnt()[w]);
    const uint64_t act = __builtin_amdgcn_ballot_w64(true);
    const uint32_t na = (uint32_t)__builtin_popcountll(act);
    const uint32_t rk = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    for (uint32_t b = 0; b < cnt; b += na) {
        const uint32_t i = b + rk;
        if (i < cnt) {
            const uint32_t meta = q.meta[i];
            const uint32_t cloud = meta >> 14;
            if (capt_resolve(pc + kExtHdr * cloud, base, q.x[i], q.y[i], q.z[i], q.r[i], q.node[i],
                             cloud == 0 ? lds_levels : 0))
                atomicOr(&defer_hits()[(w << 6) | (meta & 63u)], 1ull << ((meta >> 8) & 63u));
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (rk == 0) defer_cnt()[w] = 0u;
    __builtin_amdgcn_wave_barrier();
}
// queue this lane's undecided query; returns its hit when the queue is full and it was resolved here
// instead (rare: no call, no flush inside the generated code -- a call would cost every kernel a stack)
__device__ __forceinline__ bool capt_defer_push(bool pend, int tag, int cloud, float x, float y, float z, float r,
                                                uint32_t node, const VGPU_CONST float* pc, const float* base,
                                                int lds_levels)
{
    const uint64_t pm = __builtin_amdgcn_ballot_w64(pend);
    if (pm == 0ull) return false;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)defer_cnt()[w]);
    const uint32_t np = (uint32_t)__builtin_popcountll(pm);
    if (c0 + np > (uint32_t)kDeferCap)
        return pend && capt_resolve(pc + kExtHdr * cloud, base, x, y, z, r, node, cloud == 0 ? lds_levels : 0);
    if (pend) {
        uint32_t pos = c0 + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
        pos = VGPU_DCLAMP(base, pos, (uint32_t)kDeferCap, DBG_DEFER_SLOT);
        DeferQ& q = defer_q()[w];
        q.x[pos] = x;
        q.y[pos] = y;
        q.z[pos] = z;
        q.r[pos] = r;
        q.node[pos] = node;
        q.meta[pos] = (threadIdx.x & 63u) | ((uint32_t)tag << 8) | ((uint32_t)cloud << 14);
    }
    __builtin_amdgcn_wave_barrier();
    defer_cnt()[w] = c0 + np;  // every active lane stores the same value
    __builtin_amdgcn_wave_barrier();
    return false;
}
// resolve what is left; this lane's tag mask
__device__ __forceinline__ uint64_t capt_defer_finish(const VGPU_CONST float* pc, const float* base, int lds_levels)
{
    const uint32_t w = threadIdx.x >> 6;
    if (__builtin_amdgcn_readfirstlane((int)defer_cnt()[w]) != 0) capt_defer_flush(pc, base, lds_levels);
    __builtin_amdgcn_wave_barrier();
    return defer_hits()[threadIdx.x];
}

template <int TYPE, class TestFn>
__device__ __forceinline__ uint32_t scan_env_type(const EnvView& env, float emax, uint32_t acc, TestFn test, float x,
                                                  float y, float z, float r)
{
    return scan_type<TYPE>(env.obs[TYPE], emax, acc, test, x, y, z, r);
}

// Conservative environment test of a mid-level sphere (tools/gen_kernels.py --mids): sign bit set when the
// sphere may touch an obstacle.  Its cull extent, (sqrt(|c|^2) + r) * 1.001, bounds from above the
// approximate extent the reference culls a contained child sphere with (|c_child| + r_child <= |c| + r - 1e-4,
// and v * rsqrt_host(v) is within 2^-11 relative of sqrt v), so no obstacle a child could be tested against
// is culled here; the predicates are the reference's, on a sphere that contains the child with a 0.1 mm
// margin (float rounding of the test values is far below it).  Primitive obstacles only (no EXT).
template <class Grp>
__device__ __forceinline__ uint32_t mid_env_bits(const EnvView& env, float x, float y, float z, float r,
                                                 uint32_t acc = 0u)
{
    const float d = dot3(x, y, z, x, y, z);
    float me = (__builtin_sqrtf(d) + r) * 1.001f + 1e-5f;
    if (me != me) me = __builtin_inff();
    const float emax = Grp::max(me);
    const float rsq = r * r;
    if (env.n[OBS_SPHERE]) acc = scan_spheres(env.obs[OBS_SPHERE], emax, acc, x, y, z, r);
    if (env.n[OBS_CAPSULE])
        acc = scan_env_type<OBS_CAPSULE>(env, emax, acc, [&](const auto* o) {
            const float dot = dot3(x - o[1], y - o[2], z - o[3], o[4], o[5], o[6]);
            const float cdf = fminf(fmaxf(dot * o[8], 0.0f), 1.0f);
            const float px = __builtin_fmaf(o[4], cdf, o[1]);
            const float py = __builtin_fmaf(o[5], cdf, o[2]);
            const float pz = __builtin_fmaf(o[6], cdf, o[3]);
            const float xs = x - px, ys = y - py, zs = z - pz;
            const float rs = r + o[7];
            return __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
        }, x, y, z, r);
    if (env.n[OBS_ZCAPSULE])
        acc = scan_env_type<OBS_ZCAPSULE>(env, emax, acc, [&](const auto* o) {
            const float dot = (z - o[3]) * o[6];
            const float cdf = fminf(fmaxf(dot * o[8], 0.0f), 1.0f);
            const float pz = __builtin_fmaf(o[6], cdf, o[3]);
            const float xs = x - o[1], ys = y - o[2], zs = z - pz;
            const float rs = r + o[7];
            return __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
        }, x, y, z, r);
    if (env.n[OBS_CUBOID])
        acc = scan_env_type<OBS_CUBOID>(env, emax, acc, [&](const auto* o) {
            const float xs = x - o[1], ys = y - o[2], zs = z - o[3];
            const float a1 = max0(__builtin_fabsf(dot3(o[4], o[5], o[6], xs, ys, zs)) - o[13]);
            const float a2 = max0(__builtin_fabsf(dot3(o[7], o[8], o[9], xs, ys, zs)) - o[14]);
            const float a3 = max0(__builtin_fabsf(dot3(o[10], o[11], o[12], xs, ys, zs)) - o[15]);
            return dot3(a1, a2, a3, a1, a2, a3) - rsq;
        }, x, y, z, r);
    if (env.n[OBS_ZCUBOID])
        acc = scan_env_type<OBS_ZCUBOID>(env, emax, acc, [&](const auto* o) {
            const float xs = x - o[1], ys = y - o[2], zs = z - o[3];
            const float a1 = max0(__builtin_fabsf(dot2(o[4], o[5], xs, ys)) - o[13]);
            const float a2 = max0(__builtin_fabsf(dot2(o[7], o[8], xs, ys)) - o[14]);
            const float a3 = max0(__builtin_fabsf(zs) - o[15]);
            return dot3(a1, a2, a3, a1, a2, a3) - rsq;
        }, x, y, z, r);
    return acc;
}

// Returns acc with this lane's hits OR-ed into the sign bit.  A lane entering with its sign
// bit already set (an earlier child hit) does not keep any obstacle loop alive.
// tag: the deferred-query tag (kTagDefault: the group type's; bound kernels pass the check's bit)
template <class Grp, bool EXT = false>
__device__ __forceinline__ uint32_t env_bits(const EnvView& env, float x, float y, float z, float r, uint32_t acc = 0u,
                                             int tag = kTagDefault)
{
    const float d = dot3(x, y, z, x, y, z);
    float me = sqrt_host(d, env.lut, env.kbits) + r;  // validity.hh:55-59
    const uint32_t dexp = __float_as_uint(d) & 0x7F800000u;
    if (dexp == 0u || dexp == 0x7F800000u || me != me) me = __builtin_inff();
    const float emax = Grp::max(me);
    const float rsq = r * r;

    if (env.n[OBS_SPHERE]) acc = scan_spheres(env.obs[OBS_SPHERE], emax, acc, x, y, z, r);  // sphere_sphere.hh:10-22
    if (env.n[OBS_CAPSULE])  // sphere_capsule.hh:9-22
        acc = scan_env_type<OBS_CAPSULE>(env, emax, acc, [&](const auto* o) {
            const float dot = dot3(x - o[1], y - o[2], z - o[3], o[4], o[5], o[6]);
            const float cdf = fminf(fmaxf(dot * o[8], 0.0f), 1.0f);
            const float px = __builtin_fmaf(o[4], cdf, o[1]);
            const float py = __builtin_fmaf(o[5], cdf, o[2]);
            const float pz = __builtin_fmaf(o[6], cdf, o[3]);
            const float xs = x - px, ys = y - py, zs = z - pz;
            const float rs = r + o[7];
            return __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
        }, x, y, z, r);
    if (env.n[OBS_ZCAPSULE])  // sphere_capsule.hh:30-43
        acc = scan_env_type<OBS_ZCAPSULE>(env, emax, acc, [&](const auto* o) {
            const float dot = (z - o[3]) * o[6];
            const float cdf = fminf(fmaxf(dot * o[8], 0.0f), 1.0f);
            const float pz = __builtin_fmaf(o[6], cdf, o[3]);
            const float xs = x - o[1], ys = y - o[2], zs = z - pz;
            const float rs = r + o[7];
            return __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
        }, x, y, z, r);
    if (env.n[OBS_CUBOID])  // sphere_cuboid.hh:9-27
        acc = scan_env_type<OBS_CUBOID>(env, emax, acc, [&](const auto* o) {
            const float xs = x - o[1], ys = y - o[2], zs = z - o[3];
            const float a1 = max0(__builtin_fabsf(dot3(o[4], o[5], o[6], xs, ys, zs)) - o[13]);
            const float a2 = max0(__builtin_fabsf(dot3(o[7], o[8], o[9], xs, ys, zs)) - o[14]);
            const float a3 = max0(__builtin_fabsf(dot3(o[10], o[11], o[12], xs, ys, zs)) - o[15]);
            return dot3(a1, a2, a3, a1, a2, a3) - rsq;
        }, x, y, z, r);
    if (env.n[OBS_ZCUBOID])  // sphere_cuboid.hh:35-52
        acc = scan_env_type<OBS_ZCUBOID>(env, emax, acc, [&](const auto* o) {
            const float xs = x - o[1], ys = y - o[2], zs = z - o[3];
            const float a1 = max0(__builtin_fabsf(dot2(o[4], o[5], xs, ys)) - o[13]);
            const float a2 = max0(__builtin_fabsf(dot2(o[7], o[8], xs, ys)) - o[14]);
            const float a3 = max0(__builtin_fabsf(zs) - o[15]);
            return dot3(a1, a2, a3, a1, a2, a3) - rsq;
        }, x, y, z, r);
    if constexpr (EXT) {
        bool hit = (acc >> 31) != 0u;
        for (int i = 0; i < env.n_hf; ++i)
            if (!hit) hit = hf_lane(env.hf + kExtHdr * i, env.base, x, y, z, r);
        const int dtag = tag == kTagDefault ? DeferTagOf<Grp>::tag : tag;
        if (DeferTagOf<Grp>::on && dtag >= 0) {
            // undecided queries are queued under dtag; a hit found later is OR-ed by the kernel
            for (int i = 0; i < env.n_pc; ++i) {
                uint32_t node = 0u;
                int d = 0;
                if (!hit) d = capt_decide(env.pc + kExtHdr * i, x, y, z, r, env.base, node);
                if (d == 1) hit = true;
                if (capt_defer_push(d == 2, dtag, i, x, y, z, r, node, env.pc, env.base, env.pc_lds_levels)) hit = true;
            }
        } else {
            for (int i = 0; i < env.n_pc; ++i)
                if (!hit) hit = capt_lane(env.pc + kExtHdr * i, env.base, x, y, z, r, i == 0 ? env.pc_lds_levels : 0);
        }
        if (hit) acc |= 0x80000000u;
    }
    return acc;
}

template <class Grp, bool EXT = false>
__device__ __forceinline__ bool env_lane(const EnvView& env, float x, float y, float z, float r)
{
    return (env_bits<Grp, EXT>(env, x, y, z, r) >> 31) != 0u;
}

// ---- near sets: the records a check's children can touch ----------------------------------------------
// A check's children are tested only after its bounding test fires, and each of them runs the full culled
// scan of every obstacle type above -- most of the validate step's time (the Panda's lead pass: 76 us for FK and
// the bounding test, 480 us with the 12 children's scans).  A child the reference reports hitting record O lies
// inside S, a sphere enclosing all of the check's children with a 0.1 mm margin (tools/gen_kernels.py NEAR), so
// O's test fires for S as well: every test value here measures a distance (sphere, capsule, orthonormal cuboid --
// the reference's closest-point forms), and the margin is ~300x the float error of the FK centres and of the
// test values.  env_near scans S once and keeps, per lane, the records whose S test fires (bit near_base[t] + i
// for record i of type t); env_bits_near then runs a child's scan over those records only, with the child's own
// cull and test -- the same records fire as in env_bits, so the sign bit is the reference's.
// S's cull is mid_env_bits' (it bounds from above the approximate extent the reference culls any child with),
// made infinite when S reaches the origin (a child centred there has an infinite reference extent).  Cuboids
// whose axes are not orthonormal (bounding sphere +inf, vgpu_api.cpp obstacle_bound) are always near: their test
// value is no distance.  Only environments of at most kNearMax primitive records (EnvView::near_ok) and without
// heightfields / point clouds use near sets; the others run env_bits.
struct NearSet {
    uint64_t lane, wave;  // this lane's records (wave: unused, 0)
};

// the reference's sphere-vs-primitive test values (sign bit = collision) on one record, as in env_bits
struct ObsTests {
    float x, y, z, r, rsq;
    __device__ __forceinline__ float capsule(const VGPU_CONST float* o) const  // sphere_capsule.hh:9-22
    {
        const float dot = dot3(x - o[1], y - o[2], z - o[3], o[4], o[5], o[6]);
        const float cdf = fminf(fmaxf(dot * o[8], 0.0f), 1.0f);
        const float px = __builtin_fmaf(o[4], cdf, o[1]);
        const float py = __builtin_fmaf(o[5], cdf, o[2]);
        const float pz = __builtin_fmaf(o[6], cdf, o[3]);
        const float xs = x - px, ys = y - py, zs = z - pz;
        const float rs = r + o[7];
        return __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
    }
    __device__ __forceinline__ float zcapsule(const VGPU_CONST float* o) const  // sphere_capsule.hh:30-43
    {
        const float dot = (z - o[3]) * o[6];
        const float cdf = fminf(fmaxf(dot * o[8], 0.0f), 1.0f);
        const float pz = __builtin_fmaf(o[6], cdf, o[3]);
        const float xs = x - o[1], ys = y - o[2], zs = z - pz;
        const float rs = r + o[7];
        return __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
    }
    __device__ __forceinline__ float cuboid(const VGPU_CONST float* o) const  // sphere_cuboid.hh:9-27
    {
        const float xs = x - o[1], ys = y - o[2], zs = z - o[3];
        const float a1 = max0(__builtin_fabsf(dot3(o[4], o[5], o[6], xs, ys, zs)) - o[13]);
        const float a2 = max0(__builtin_fabsf(dot3(o[7], o[8], o[9], xs, ys, zs)) - o[14]);
        const float a3 = max0(__builtin_fabsf(dot3(o[10], o[11], o[12], xs, ys, zs)) - o[15]);
        return dot3(a1, a2, a3, a1, a2, a3) - rsq;
    }
    __device__ __forceinline__ float zcuboid(const VGPU_CONST float* o) const  // sphere_cuboid.hh:35-52
    {
        const float xs = x - o[1], ys = y - o[2], zs = z - o[3];
        const float a1 = max0(__builtin_fabsf(dot2(o[4], o[5], xs, ys)) - o[13]);
        const float a2 = max0(__builtin_fabsf(dot2(o[7], o[8], xs, ys)) - o[14]);
        const float a3 = max0(__builtin_fabsf(zs) - o[15]);
        return dot3(a1, a2, a3, a1, a2, a3) - rsq;
    }
    __device__ __forceinline__ float sphere(const VGPU_CONST float* o) const  // o: md x y z r at stride 2
    {
        return sphere_sphere(o[2], o[4], o[6], o[8], x, y, z, r);  // sphere_sphere.hh:10-22, as scan_spheres
    }
};

// record i of a type's section (spheres: two records per kSphereBlock-float block, fields interleaved)
template <int TYPE>
__device__ __forceinline__ const VGPU_CONST float* obs_record(const VGPU_CONST float* o, int i)
{
    if constexpr (TYPE == OBS_SPHERE) return o + kSphereBlock * (i >> 1) + (i & 1);
    else return o + kObsStride[TYPE] * i;
}

template <int TYPE>
__device__ __forceinline__ float obs_test(const ObsTests& t, const VGPU_CONST float* o)
{
    if constexpr (TYPE == OBS_SPHERE) return t.sphere(o);
    else if constexpr (TYPE == OBS_CAPSULE) return t.capsule(o);
    else if constexpr (TYPE == OBS_ZCAPSULE) return t.zcapsule(o);
    else if constexpr (TYPE == OBS_CUBOID) return t.cuboid(o);
    else return t.zcuboid(o);
}

// S's bits over one type: records in md order until no lane of the wave reaches one (the next md loaded a trip
// ahead; the sections are sentinel-padded).  Spheres two records per trip, from their pair blocks (as scan_spheres).
template <int TYPE>
__device__ __forceinline__ uint64_t near_bits_type(const EnvView& env, const ObsTests& t, float emax, uint64_t lane)
{
    const VGPU_CONST float* o = env.obs[TYPE];
    const int n = env.n[TYPE], base = env.near_base[TYPE];
    if constexpr (TYPE == OBS_SPHERE) {
        const VGPU_CONST SphereBlk* p = (const VGPU_CONST SphereBlk*)o;
        f2v md = p->md;
        for (int i = 0; i < n; i += 2, ++p) {
            const bool la = md.x < emax, lb = md.y < emax;  // a pad record's md is +inf
            if (__builtin_amdgcn_ballot_w64(la) == 0ull) break;  // sorted by md: nothing later is reached either
            const f2v nmd = p[1].md;
            const float va = sphere_sphere(p->x.x, p->y.x, p->z.x, p->r.x, t.x, t.y, t.z, t.r);
            const float vb = sphere_sphere(p->x.y, p->y.y, p->z.y, p->r.y, t.x, t.y, t.z, t.r);
            const uint64_t on = (la && !(va >= 0.0f) ? 1ull : 0ull) | (lb && !(vb >= 0.0f) ? 2ull : 0ull);  // NaN: near
            lane |= on << (base + i);
            md = nmd;
        }
    } else {
        float md = obs_record<TYPE>(o, 0)[0];
        for (int i = 0; i < n; ++i) {
            const bool live = md < emax;
            if (__builtin_amdgcn_ballot_w64(live) == 0ull) break;
            const VGPU_CONST float* rec = obs_record<TYPE>(o, i);
            md = obs_record<TYPE>(o, i + 1)[0];
            const float v = obs_test<TYPE>(t, rec);
            bool near = !(v >= 0.0f);
            if constexpr (TYPE == OBS_CUBOID || TYPE == OBS_ZCUBOID) near = near || !(rec[kObsBound[TYPE] + 3] < __builtin_inff());
            if (live && near) lane |= 1ull << (base + i);
        }
    }
    return lane;
}

// S's near set; requires env.near_ok (the generated code branches on it: without near sets the children run
// env_bits)
template <class Grp>
__device__ __forceinline__ NearSet env_near(const EnvView& env, float x, float y, float z, float r)
{
    const float d = dot3(x, y, z, x, y, z);
    float me = (__builtin_sqrtf(d) + r) * 1.001f + 1e-5f;
    if (me != me || !(d > r * r * 1.001f)) me = __builtin_inff();  // NaN, or S reaches the origin
    const float emax = Grp::max(me);
    const ObsTests t{x, y, z, r, r * r};
    uint64_t b = 0ull;
    if (env.n[OBS_SPHERE]) b = near_bits_type<OBS_SPHERE>(env, t, emax, b);
    if (env.n[OBS_CAPSULE]) b = near_bits_type<OBS_CAPSULE>(env, t, emax, b);
    if (env.n[OBS_ZCAPSULE]) b = near_bits_type<OBS_ZCAPSULE>(env, t, emax, b);
    if (env.n[OBS_CUBOID]) b = near_bits_type<OBS_CUBOID>(env, t, emax, b);
    if (env.n[OBS_ZCUBOID]) b = near_bits_type<OBS_ZCUBOID>(env, t, emax, b);
    return NearSet{b, 0ull};
}

// a child's scan over one type's records in this lane's near set: each lane walks its OWN set (per-lane loads of
// the records, L1-resident), so a wave needs as many trips as its fullest lane has records -- not the union over
// the wave's 8 unrelated edges, which a scalar walk would take; the reference's cull (md < emax, the group's) and
// test per record
template <int TYPE>
__device__ __forceinline__ uint32_t near_scan_type(const EnvView& env, const NearSet& ns, const ObsTests& t, float emax,
                                                   uint32_t acc)
{
    const VGPU_CONST float* o = env.obs[TYPE];
    const int n = env.n[TYPE], base = env.near_base[TYPE];
    uint64_t m = ns.lane >> base;
    if (n < 64) m &= (1ull << n) - 1ull;
    if (acc >> 31) m = 0ull;  // this lane already hit
    while (__builtin_amdgcn_ballot_w64(m != 0ull) != 0ull) {
        if (m != 0ull) {
            const int i = __builtin_ctzll(m);
            m &= m - 1ull;
            const VGPU_CONST float* rec = obs_record<TYPE>(o, i);
            if (rec[0] < emax) acc |= __float_as_uint(obs_test<TYPE>(t, rec));
        }
    }
    return acc;
}

// a bounding test inside a near-set cluster (tools/gen_kernels.py --cluster): the walk over the cluster sphere's near
// records, or env_bits without near sets / with heightfields or point clouds
template <class Grp>
__device__ __forceinline__ uint32_t env_bits_near(const EnvView& env, const NearSet& ns, float x, float y, float z,
                                                  float r, uint32_t acc);
template <class Grp, bool EXT>
__device__ __forceinline__ uint32_t env_bits_e(const EnvView& env, const NearSet& ns, float x, float y, float z, float r,
                                               uint32_t acc = 0u, int tag = kTagDefault)
{
    if constexpr (!EXT) {
        if (env.near_ok) return env_bits_near<Grp>(env, ns, x, y, z, r, acc);
    }
    return env_bits<Grp, EXT>(env, x, y, z, r, acc, tag);
}

// env_bits of a child of the check whose near set is ns (same sign bit); primitive environments with near sets
template <class Grp>
__device__ __forceinline__ uint32_t env_bits_near(const EnvView& env, const NearSet& ns, float x, float y, float z,
                                                  float r, uint32_t acc)
{
    const float d = dot3(x, y, z, x, y, z);
    float me = sqrt_host(d, env.lut, env.kbits) + r;  // validity.hh:55-59, as env_bits
    const uint32_t dexp = __float_as_uint(d) & 0x7F800000u;
    if (dexp == 0u || dexp == 0x7F800000u || me != me) me = __builtin_inff();
    const float emax = Grp::max(me);
    const ObsTests t{x, y, z, r, r * r};
    if (env.n[OBS_SPHERE]) acc = near_scan_type<OBS_SPHERE>(env, ns, t, emax, acc);
    if (env.n[OBS_CAPSULE]) acc = near_scan_type<OBS_CAPSULE>(env, ns, t, emax, acc);
    if (env.n[OBS_ZCAPSULE]) acc = near_scan_type<OBS_ZCAPSULE>(env, ns, t, emax, acc);
    if (env.n[OBS_CUBOID]) acc = near_scan_type<OBS_CUBOID>(env, ns, t, emax, acc);
    if (env.n[OBS_ZCUBOID]) acc = near_scan_type<OBS_ZCUBOID>(env, ns, t, emax, acc);
    return acc;
}

// Attachment::pose (collision/attachments.hh:75-122) at the end-effector pose p (position,
// quaternion x y z w): the composed rotation's basis and translation, float32 left to right
// exactly as the oracle's pose_attachment (oracle/vamp_oracle.c).
struct AttPose {
    float xx, xy, xz, yx, yy, yz, zx, zy, zz, tx, ty, tz;
};
__device__ __forceinline__ AttPose att_pose(const EnvView& env, float p_tx, float p_ty, float p_tz, float p_rx,
                                            float p_ry, float p_rz, float p_rw)
{
    const VGPU_CONST float* tf = env.att;
    const float t_tx = tf[0], t_ty = tf[1], t_tz = tf[2], t_rx = tf[3], t_ry = tf[4], t_rz = tf[5], t_rw = tf[6];
    const float rx = p_rw * t_rx + p_rx * t_rw + p_ry * t_rz - p_rz * t_ry;
    const float ry = p_rw * t_ry - p_rx * t_rz + p_ry * t_rw + p_rz * t_rx;
    const float rz = p_rw * t_rz + p_rx * t_ry - p_ry * t_rx + p_rz * t_rw;
    const float rw = p_rw * t_rw - p_rx * t_rx - p_ry * t_ry - p_rz * t_rz;
    const float x0 = p_ry * t_tz - p_rz * t_ty;
    const float x1 = p_rx * t_ty - p_ry * t_tx;
    const float x2 = p_rx * t_tz - p_rz * t_tx;
    AttPose a;
    a.tx = p_tx + 2.0f * (p_rw * x0 + p_ry * x1 + p_rz * x2) + t_tx;
    a.ty = p_ty + 2.0f * (-p_rw * x2 - p_rx * x1 + p_rz * x0) + t_ty;
    a.tz = p_tz + 2.0f * (p_rw * x1 - p_rx * x2 - p_ry * x0) + t_tz;
    const float bx0 = ry * ry, bx1 = rz * rz, bx2 = rw * rz, bx3 = rw * ry, bx4 = rx * rx;
    const float bx5 = rw * rx, bx6 = rx * ry, bx7 = rx * rz, bx8 = ry * rz;
    a.xx = -2.0f * (bx0 + bx1) + 1.0f;
    a.xy = 2.0f * (bx6 + bx2);
    a.xz = 2.0f * (bx7 - bx3);
    a.yx = 2.0f * (bx6 - bx2);
    a.yy = -2.0f * (bx1 + bx4) + 1.0f;
    a.yz = 2.0f * (bx8 + bx5);
    a.zx = 2.0f * (bx7 + bx3);
    a.zy = 2.0f * (bx8 - bx5);
    a.zz = -2.0f * (bx0 + bx4) + 1.0f;
    return a;
}
// posed centre of attached sphere k (attachments.hh:112-120)
__device__ __forceinline__ void att_sphere(const EnvView& env, const AttPose& a, int k, float& X, float& Y, float& Z,
                                           float& R)
{
    const VGPU_CONST float* c = env.att + kAttHdr + 4 * k;
    X = c[0] * a.xx + c[1] * a.yx + c[2] * a.zx + a.tx;
    Y = c[0] * a.xy + c[1] * a.yy + c[2] * a.zy + a.ty;
    Z = c[0] * a.xz + c[1] * a.yz + c[2] * a.zz + a.tz;
    R = c[3];
}

// sphere_sphere_self_collision (collision/validity.hh:13-44)
// (per lane; the group result is Grp::any of it).  self_bits returns the raw test-value
// bits so a block of children reduces with one v_or per child (sign bit = collision).
__device__ __forceinline__ uint32_t self_bits(float ax, float ay, float az, float ar, float bx, float by, float bz,
                                              float br)
{
    return __float_as_uint(sphere_sphere(ax, ay, az, ar, bx, by, bz, br));
}
__device__ __forceinline__ bool self_lane(float ax, float ay, float az, float ar, float bx, float by, float bz,
                                          float br)
{
    return signbit_f(sphere_sphere(ax, ay, az, ar, bx, by, bz, br));
}
