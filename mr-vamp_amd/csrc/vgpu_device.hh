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
//     wave64 and the reductions are one ballot + scalar bit-twiddling + inverse ballot.
//
// Compiled with -ffp-contract=off: every fmaf below is intended, nothing else fuses.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define VGPU_CONST __attribute__((address_space(4)))

// ---- group reductions -----------------------------------------------------------------
struct Grp1 {
    static constexpr int G = 1;
    __device__ static __forceinline__ bool any(bool p) { return p; }
    __device__ static __forceinline__ bool all(bool p) { return p; }
};

struct Grp8 {
    static constexpr int G = 8;
    __device__ static __forceinline__ bool any(bool p)
    {
        unsigned long long t = __ballot(p);
        t |= t >> 1;
        t |= t >> 2;
        t |= t >> 4;
        t &= 0x0101010101010101ull;
        return __builtin_amdgcn_inverse_ballot_w64(t * 0xFFull);
    }
    __device__ static __forceinline__ bool all(bool p)
    {
        unsigned long long t = __ballot(p);
        t &= t >> 1;
        t &= t >> 2;
        t &= t >> 4;
        t &= 0x0101010101010101ull;
        return __builtin_amdgcn_inverse_ballot_w64(t * 0xFFull);
    }
};

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

// ---- environment view ----------------------------------------------------------------------
// Obstacle rows (float32), each list sorted ascending by min_distance (last field):
//   sphere [5] x y z r md | capsule [9] x1 y1 z1 xv yv zv r rdv md | cuboid [16] x y z a1 a2 a3 r1 r2 r3 md
struct EnvView {
    const VGPU_CONST float* spheres;
    const VGPU_CONST float* capsules;
    const VGPU_CONST float* zcapsules;
    const VGPU_CONST float* cuboids;
    const VGPU_CONST float* zcuboids;
    const uint32_t* lut;  // host rsqrt table, 2 << kbits entries
    int n_spheres, n_capsules, n_zcapsules, n_cuboids, n_zcuboids;
    int kbits;
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

// sphere_environment_in_collision (collision/validity.hh:46-150), one rake group
#ifndef VGPU_ENV_INLINE
#define VGPU_ENV_ATTR __noinline__
#else
#define VGPU_ENV_ATTR __forceinline__
#endif
template <class Grp>
__device__ VGPU_ENV_ATTR bool env_collide(const EnvView& env, float x, float y, float z, float r)
{
    const float d = dot3(x, y, z, x, y, z);
    const float me = sqrt_host(d, env.lut, env.kbits) + r;  // validity.hh:55-59
    const uint32_t dexp = __float_as_uint(d) & 0x7F800000u;
    const bool nocull = dexp == 0u || dexp == 0x7F800000u;  // 0/denormal/inf/NaN: NaN extent

    for (int j = 0; j < env.n_spheres; ++j) {
        const VGPU_CONST float* o = env.spheres + 5 * j;
        const bool cull = !nocull && !signbit_f(o[4] - me);
        if (Grp::all(cull)) break;
        const float v = sphere_sphere(o[0], o[1], o[2], o[3], x, y, z, r);
        if (Grp::any(signbit_f(v))) return true;
    }
    for (int j = 0; j < env.n_capsules; ++j) {  // sphere_capsule.hh:9-22
        const VGPU_CONST float* o = env.capsules + 9 * j;
        const bool cull = !nocull && !signbit_f(o[8] - me);
        if (Grp::all(cull)) break;
        const float dot = dot3(x - o[0], y - o[1], z - o[2], o[3], o[4], o[5]);
        const float cdf = fminf(fmaxf(dot * o[7], 0.0f), 1.0f);
        const float px = __builtin_fmaf(o[3], cdf, o[0]);
        const float py = __builtin_fmaf(o[4], cdf, o[1]);
        const float pz = __builtin_fmaf(o[5], cdf, o[2]);
        const float xs = x - px, ys = y - py, zs = z - pz;
        const float rs = r + o[6];
        const float v = __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
        if (Grp::any(signbit_f(v))) return true;
    }
    for (int j = 0; j < env.n_zcapsules; ++j) {  // sphere_capsule.hh:30-43
        const VGPU_CONST float* o = env.zcapsules + 9 * j;
        const bool cull = !nocull && !signbit_f(o[8] - me);
        if (Grp::all(cull)) break;
        const float dot = (z - o[2]) * o[5];
        const float cdf = fminf(fmaxf(dot * o[7], 0.0f), 1.0f);
        const float pz = __builtin_fmaf(o[5], cdf, o[2]);
        const float xs = x - o[0], ys = y - o[1], zs = z - pz;
        const float rs = r + o[6];
        const float v = __builtin_fmaf(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
        if (Grp::any(signbit_f(v))) return true;
    }
    const float rsq = r * r;
    for (int j = 0; j < env.n_cuboids; ++j) {  // sphere_cuboid.hh:9-27
        const VGPU_CONST float* o = env.cuboids + 16 * j;
        const bool cull = !nocull && !signbit_f(o[15] - me);
        if (Grp::all(cull)) break;
        const float xs = x - o[0], ys = y - o[1], zs = z - o[2];
        const float a1 = max0(__builtin_fabsf(dot3(o[3], o[4], o[5], xs, ys, zs)) - o[12]);
        const float a2 = max0(__builtin_fabsf(dot3(o[6], o[7], o[8], xs, ys, zs)) - o[13]);
        const float a3 = max0(__builtin_fabsf(dot3(o[9], o[10], o[11], xs, ys, zs)) - o[14]);
        const float v = dot3(a1, a2, a3, a1, a2, a3) - rsq;
        if (Grp::any(signbit_f(v))) return true;
    }
    for (int j = 0; j < env.n_zcuboids; ++j) {  // sphere_cuboid.hh:35-52
        const VGPU_CONST float* o = env.zcuboids + 16 * j;
        const bool cull = !nocull && !signbit_f(o[15] - me);
        if (Grp::all(cull)) break;
        const float xs = x - o[0], ys = y - o[1], zs = z - o[2];
        const float a1 = max0(__builtin_fabsf(dot2(o[3], o[4], xs, ys)) - o[12]);
        const float a2 = max0(__builtin_fabsf(dot2(o[6], o[7], xs, ys)) - o[13]);
        const float a3 = max0(__builtin_fabsf(zs) - o[14]);
        const float v = dot3(a1, a2, a3, a1, a2, a3) - rsq;
        if (Grp::any(signbit_f(v))) return true;
    }
    return false;
}

// sphere_sphere_self_collision (collision/validity.hh:13-44)
template <class Grp>
__device__ __forceinline__ bool self_collide(float ax, float ay, float az, float ar, float bx, float by, float bz,
                                             float br)
{
    return Grp::any(signbit_f(sphere_sphere(ax, ay, az, ar, bx, by, bz, br)));
}
