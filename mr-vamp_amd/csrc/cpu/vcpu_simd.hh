// vcpu_simd.hh -- the CPU rake block: one reference ConfigurationBlock<8> in one AVX2 register.
//
// This is the host half of the build (single-edge planner calls stay on the
// CPU, GPU launch latency >> 2 us/edge) and the CPU baseline timed next to the GPU (§8(d)).
// The generated robot code (tools/gen_kernels.py --cpu -> csrc/gen/cpu/*.inc) is the SAME
// expression text as the HIP kernels' (csrc/gen/*.inc), with `float` -> V and the per-lane
// check bits `uint32_t` -> VB; this header gives those names their AVX2 meaning:
//   * V  = 8 lanes of float32 (one rake block: lane l = interpolant l of the block), every
//          operator one IEEE float op (the TU is compiled -ffp-contract=off; each fma below is
//          an explicit _mm256_fmadd_ps mirroring a contraction of the reference release build);
//   * VB = per-lane sign-bit masks (a test value's bits, or a compare result): a lane fires
//          when its sign bit is set (reference avx.hh:385-389 testz on the sign);
//   * Grp (GrpBlock) = the whole block: any_bits = movemask != 0 (validity.hh "any lane").
// The environment loop is the reference's own formulation (collision/validity.hh:46-150): per
// obstacle type in ascending min_distance, `break` when every lane has md - max_extent >= +0,
// `return` at the first obstacle any lane hits; max_extent = v * _mm256_rsqrt_ps(v) + r with the
// host's own rsqrt (the GPU emulates the same instruction from a table probed on this host).
#pragma once

#include <immintrin.h>
#include <stdint.h>

#include <cmath>
#include <cstring>

#define VCPU_INLINE static inline __attribute__((always_inline))

namespace vcpu {

struct V {
    __m256 v;
    V() : v(_mm256_setzero_ps()) {}
    V(__m256 x) : v(x) {}
    V(float x) : v(_mm256_set1_ps(x)) {}  // scalar literals / base offsets broadcast (validity.hh:55-58)
};
VCPU_INLINE V operator+(V a, V b) { return _mm256_add_ps(a.v, b.v); }
VCPU_INLINE V operator-(V a, V b) { return _mm256_sub_ps(a.v, b.v); }
VCPU_INLINE V operator*(V a, V b) { return _mm256_mul_ps(a.v, b.v); }
VCPU_INLINE V operator-(V a) { return _mm256_xor_ps(a.v, _mm256_set1_ps(-0.0f)); }
VCPU_INLINE V fma(V a, V b, V c) { return _mm256_fmadd_ps(a.v, b.v, c.v); }
VCPU_INLINE V vabs(V a) { return _mm256_andnot_ps(_mm256_set1_ps(-0.0f), a.v); }
// _mm256_max_ps / _mm256_min_ps operand semantics (a NaN first operand yields the second)
VCPU_INLINE V vmax(V a, V b) { return _mm256_max_ps(a.v, b.v); }
VCPU_INLINE V vmin(V a, V b) { return _mm256_min_ps(a.v, b.v); }

struct VB {
    __m256 v;
    VB() : v(_mm256_setzero_ps()) {}
    VB(__m256 x) : v(x) {}
    VB(V x) : v(x.v) {}  // a test value: its sign bit is the lane's hit
};
VCPU_INLINE VB operator|(VB a, VB b) { return _mm256_or_ps(a.v, b.v); }
VCPU_INLINE VB& operator|=(VB& a, VB b) { a.v = _mm256_or_ps(a.v, b.v); return a; }
VCPU_INLINE VB operator&&(VB a, VB b) { return _mm256_and_ps(a.v, b.v); }
VCPU_INLINE VB operator!(VB a) { return _mm256_xor_ps(a.v, _mm256_castsi256_ps(_mm256_set1_epi32(-1))); }
VCPU_INLINE VB operator>=(V a, V b) { return _mm256_cmp_ps(a.v, b.v, _CMP_GE_OQ); }
VCPU_INLINE VB operator<=(V a, V b) { return _mm256_cmp_ps(a.v, b.v, _CMP_LE_OQ); }
VCPU_INLINE int signmask(VB a) { return _mm256_movemask_ps(a.v); }
VCPU_INLINE int signmask(V a) { return _mm256_movemask_ps(a.v); }

// the rake group of the reference: the whole 8-lane block
struct GrpBlock {
    static constexpr int G = 8;
    VCPU_INLINE bool any_bits(VB b) { return signmask(b) != 0; }
    VCPU_INLINE bool any(VB b) { return signmask(b) != 0; }
};

// ---- FloatVector::sin()/cos() (vector/interface.hh:438-469), release-build Horner/FMA form ----
VCPU_INLINE V vamp_sin(V x)
{
    const V c1 = -0x1.ea200ap-2f, c2 = 0x1.80f17p+0f, c3 = 0x1.7c019ap-7f, c4 = 0x1.1ec4f2p-3f,
            c5 = 0x1.54952ep-1f;
    const V p = x * fma(vabs(x), c1, c2);
    const V ap = vabs(p);
    return p * fma(ap, fma(ap, c3, c4), c5);
}
VCPU_INLINE V vamp_cos(V x)
{
    const V PI = 0x1.921fb6p+1f, HALF_PI = 0x1.921fb6p+0f, TWO_PI = 0x1.921fb6p+2f;
    V v = x + HALF_PI;
    v = v - V(_mm256_and_ps(_mm256_cmp_ps(v.v, PI.v, _CMP_GE_OQ), TWO_PI.v));
    return vamp_sin(v);
}

// dot_3 / dot_2 (collision/math.hh:10-27) in the release build's contracted form
VCPU_INLINE V dot3(V a0, V a1, V a2, V b0, V b1, V b2) { return fma(a0, b0, fma(a2, b2, a1 * b1)); }
VCPU_INLINE V dot2(V a0, V a1, V b0, V b1) { return fma(a0, b0, a1 * b1); }

// sphere_sphere_sql2 (sphere_sphere.hh:10-22)
VCPU_INLINE V sphere_sphere(V ax, V ay, V az, V ar, V bx, V by, V bz, V br)
{
    const V xs = ax - bx, ys = ay - by, zs = az - bz;
    const V rs = ar + br;
    return fma(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
}

// ---- environment view: the same blob layout as the device buffer (vgpu_device.hh EnvView) ----
enum : int { OBS_SPHERE = 0, OBS_CAPSULE = 1, OBS_ZCAPSULE = 2, OBS_CUBOID = 3, OBS_ZCUBOID = 4, OBS_TYPES = 5 };
constexpr int kObsStride[OBS_TYPES] = {8, 16, 16, 20, 20};  // = vgpu_device.hh (bounding spheres unused here)
constexpr int kSphereBlock = 16;  // spheres: pair blocks md_a md_b x_a x_b y_a y_b z_a z_b r_a r_b (vgpu_device.hh)
constexpr int kAttHdr = 8;
constexpr int kExtHdr = 32;  // = vgpu_device.hh (the host view leaves the device-only cell grid fields 0)
enum : int { HF_X = 0, HF_Y, HF_Z, HF_XS, HF_YS, HF_ZS, HF_XD, HF_YD, HF_XD2, HF_YD2, HF_OFF, HF_CELLS };
enum : int { PC_TOP = 0, PC_RPOINT = 6, PC_NLOG2 = 7, PC_TESTS, PC_AABBS, PC_STARTS, PC_AFF };

struct EnvView {
    const float* obs[OBS_TYPES];
    int n[OBS_TYPES];
    const float* hf;
    const float* pc;
    const float* base;
    int n_hf, n_pc;
    const float* att;
    int n_att;
};

inline uint32_t hdr_u(const float* h, int i)
{
    uint32_t u;
    std::memcpy(&u, h + i, 4);
    return u;
}
inline float mm_max(float a, float b) { return a > b ? a : b; }
inline float mm_min(float a, float b) { return a < b ? a : b; }

// sphere_heightfield (sphere_heightfield.hh:9-30), release-build form (ref_probe "hf"); an index
// outside the data (undefined in the reference) is reported as a collision, as on the GPU
inline bool hf_lane(const float* h, const float* base, float x, float y, float z, float r)
{
    const float xo = h[HF_X] - x, yo = h[HF_Y] - y;
    const float xs = std::floor(mm_min(mm_max(std::fma(h[HF_XS], xo, h[HF_XD2]), 0.0f), h[HF_XD]));
    const float ys = std::floor(mm_min(mm_max(std::fma(h[HF_YS], yo, h[HF_YD2]), 0.0f), h[HF_YD]));
    const float fi = std::fma(ys, h[HF_XD], xs);
    const uint32_t cells = hdr_u(h, HF_CELLS);
    if (!(fi >= 0.0f && fi < (float)cells)) return true;
    const uint32_t idx = (uint32_t)std::nearbyint(fi);
    if (idx >= cells) return true;
    const float zh = base[hdr_u(h, HF_OFF) + idx];
    const float v = (z - r) - std::fma(h[HF_ZS], zh, h[HF_Z]);
    return std::signbit(v);
}

// CAPT::collides_simd (capt.hh:457-541) for one lane: top box inflated by r, descent of the
// implicit split tree, leaf box with (r + r_point)^2, then the leaf's affordance vectors -- 8
// points per AVX2 register, inclusive distance test, sums of squares fma(d0,d0,fma(d2,d2,d1*d1))
inline bool capt_lane(const float* h, const float* base, float x, float y, float z, float r)
{
    if (!((x + r >= h[0]) && (x - r <= h[3]) && (y + r >= h[1]) && (y - r <= h[4]) && (z + r >= h[2]) &&
          (z - r <= h[5])))
        return false;
    const int nlog2 = (int)hdr_u(h, PC_NLOG2);
    const float* tests = base + hdr_u(h, PC_TESTS);
    uint32_t idx = 0;
    float a = x, b = y, c = z;
    for (int i = 0; i < nlog2; ++i) {
        idx = 2u * idx + 1u + ((a >= tests[idx]) ? 1u : 0u);
        const float t = a;
        a = b;
        b = c;
        c = t;
    }
    const uint32_t leaf = nlog2 ? idx - ((1u << nlog2) - 1u) : 0u;
    const float* box = base + hdr_u(h, PC_AABBS) + 6u * leaf;
    const float rr = r + h[PC_RPOINT];
    const float rc = rr * rr;
    const float d0 = x - mm_min(mm_max(x, box[0]), box[3]);
    const float d1 = y - mm_min(mm_max(y, box[1]), box[4]);
    const float d2 = z - mm_min(mm_max(z, box[2]), box[5]);
    if (!(std::fma(d0, d0, std::fma(d2, d2, d1 * d1)) <= rc)) return false;
    const uint32_t* starts = (const uint32_t*)(base + hdr_u(h, PC_STARTS));
    const uint32_t s = starts[leaf], e = starts[leaf + 1];
    const float* aff = base + hdr_u(h, PC_AFF);
    const V X = x, Y = y, Z = z, RC = rc;
    for (uint32_t i = s; i < e; ++i) {
        const float* v = aff + 24u * i;
        const V dx = V(_mm256_loadu_ps(v)) - X, dy = V(_mm256_loadu_ps(v + 8)) - Y, dz = V(_mm256_loadu_ps(v + 16)) - Z;
        if (signmask(VB(_mm256_cmp_ps(fma(dx, dx, fma(dz, dz, dy * dy)).v, RC.v, _CMP_LE_OQ)))) return true;
    }
    return false;
}

// sphere_environment_in_collision (collision/validity.hh:46-150) for one 8-lane block: returns
// acc with the lanes' hits in the sign bits.  Entering with any lane already hit, the block's
// result is already a collision (the reference returned at that child): nothing more to do.
// Out of line: an fkcc calls it ~80 times, and one copy per call site makes the generated
// functions too large for the compiler (V arguments travel in ymm registers).
template <class Grp, bool EXT>
__attribute__((noinline)) static VB env_bits(const EnvView& env, V x, V y, V z, float r, VB acc = VB())
{
    if (signmask(acc)) return acc;
    const V d = dot3(x, y, z, x, y, z);
    const V me = d * V(_mm256_rsqrt_ps(d.v)) + V(r);  // validity.hh:55-59, the host rsqrt
    const V R = r, RSQ = r * r;
    // one obstacle type: ascending min_distance; stop when all lanes are culled
#define VCPU_SCAN(TYPE, TEST)                                                        \
    {                                                                                \
        const float* o = env.obs[TYPE];                                              \
        for (int j = 0; j < env.n[TYPE]; ++j, o += kObsStride[TYPE]) {               \
            if (signmask(V(o[0]) - me) == 0) break;                                  \
            const V t = TEST;                                                        \
            if (signmask(t)) return acc | VB(t);                                     \
        }                                                                            \
    }
    {  // sphere_sphere.hh:10-22; record j is half j & 1 of pair block j / 2
        const float* s = env.obs[OBS_SPHERE];
        for (int j = 0; j < env.n[OBS_SPHERE]; ++j) {
            const float* o = s + (j >> 1) * kSphereBlock + (j & 1);
            if (signmask(V(o[0]) - me) == 0) break;
            const V t = sphere_sphere(o[2], o[4], o[6], o[8], x, y, z, R);
            if (signmask(t)) return acc | VB(t);
        }
    }
    VCPU_SCAN(OBS_CAPSULE, ([&] {                                              // sphere_capsule.hh:9-22
                  const V dot = dot3(x - o[1], y - o[2], z - o[3], o[4], o[5], o[6]);
                  const V cdf = vmin(vmax(dot * o[8], 0.0f), 1.0f);
                  const V px = fma(o[4], cdf, o[1]), py = fma(o[5], cdf, o[2]), pz = fma(o[6], cdf, o[3]);
                  const V xs = x - px, ys = y - py, zs = z - pz;
                  const V rs = R + o[7];
                  return fma(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
              }()))
    VCPU_SCAN(OBS_ZCAPSULE, ([&] {  // sphere_capsule.hh:30-43
                  const V dot = (z - o[3]) * o[6];
                  const V cdf = vmin(vmax(dot * o[8], 0.0f), 1.0f);
                  const V pz = fma(o[6], cdf, o[3]);
                  const V xs = x - o[1], ys = y - o[2], zs = z - pz;
                  const V rs = R + o[7];
                  return fma(-rs, rs, dot3(xs, ys, zs, xs, ys, zs));
              }()))
    VCPU_SCAN(OBS_CUBOID, ([&] {  // sphere_cuboid.hh:9-27
                  const V xs = x - o[1], ys = y - o[2], zs = z - o[3];
                  const V a1 = vmax(vabs(dot3(o[4], o[5], o[6], xs, ys, zs)) - o[13], 0.0f);
                  const V a2 = vmax(vabs(dot3(o[7], o[8], o[9], xs, ys, zs)) - o[14], 0.0f);
                  const V a3 = vmax(vabs(dot3(o[10], o[11], o[12], xs, ys, zs)) - o[15], 0.0f);
                  return dot3(a1, a2, a3, a1, a2, a3) - RSQ;
              }()))
    VCPU_SCAN(OBS_ZCUBOID, ([&] {  // sphere_cuboid.hh:35-52
                  const V xs = x - o[1], ys = y - o[2], zs = z - o[3];
                  const V a1 = vmax(vabs(dot2(o[4], o[5], xs, ys)) - o[13], 0.0f);
                  const V a2 = vmax(vabs(dot2(o[7], o[8], xs, ys)) - o[14], 0.0f);
                  const V a3 = vmax(vabs(zs) - o[15], 0.0f);
                  return dot3(a1, a2, a3, a1, a2, a3) - RSQ;
              }()))
#undef VCPU_SCAN
    if constexpr (EXT) {  // heightfields, then point clouds: no cull (validity.hh:133-148)
        alignas(32) float lx[8], ly[8], lz[8];
        _mm256_store_ps(lx, x.v);
        _mm256_store_ps(ly, y.v);
        _mm256_store_ps(lz, z.v);
        for (int i = 0; i < env.n_hf; ++i)
            for (int l = 0; l < 8; ++l)
                if (hf_lane(env.hf + kExtHdr * i, env.base, lx[l], ly[l], lz[l], r)) return VB(V(-1.0f));
        for (int i = 0; i < env.n_pc; ++i)
            for (int l = 0; l < 8; ++l)
                if (capt_lane(env.pc + kExtHdr * i, env.base, lx[l], ly[l], lz[l], r)) return VB(V(-1.0f));
    }
    return acc;
}

// sphere_sphere_self_collision (collision/validity.hh:13-44): the test value's bits per lane
VCPU_INLINE VB self_bits(V ax, V ay, V az, float ar, V bx, V by, V bz, float br)
{
    return VB(sphere_sphere(ax, ay, az, ar, bx, by, bz, br));
}
VCPU_INLINE VB self_lane(V ax, V ay, V az, float ar, V bx, V by, V bz, float br)
{
    return self_bits(ax, ay, az, ar, bx, by, bz, br);
}

// Attachment::pose (collision/attachments.hh:75-122) at the end-effector pose (position,
// quaternion x y z w) per lane: float32, left to right, as the oracle's pose_attachment
struct AttPose {
    V xx, xy, xz, yx, yy, yz, zx, zy, zz, tx, ty, tz;
};
VCPU_INLINE AttPose att_pose(const EnvView& env, V p_tx, V p_ty, V p_tz, V p_rx, V p_ry, V p_rz, V p_rw)
{
    const float* tf = env.att;
    const V t_tx = tf[0], t_ty = tf[1], t_tz = tf[2], t_rx = tf[3], t_ry = tf[4], t_rz = tf[5], t_rw = tf[6];
    const V rx = p_rw * t_rx + p_rx * t_rw + p_ry * t_rz - p_rz * t_ry;
    const V ry = p_rw * t_ry - p_rx * t_rz + p_ry * t_rw + p_rz * t_rx;
    const V rz = p_rw * t_rz + p_rx * t_ry - p_ry * t_rx + p_rz * t_rw;
    const V rw = p_rw * t_rw - p_rx * t_rx - p_ry * t_ry - p_rz * t_rz;
    const V x0 = p_ry * t_tz - p_rz * t_ty;
    const V x1 = p_rx * t_ty - p_ry * t_tx;
    const V x2 = p_rx * t_tz - p_rz * t_tx;
    const V two = 2.0f, mtwo = -2.0f, one = 1.0f;
    AttPose a;
    a.tx = p_tx + two * (p_rw * x0 + p_ry * x1 + p_rz * x2) + t_tx;
    a.ty = p_ty + two * (-p_rw * x2 - p_rx * x1 + p_rz * x0) + t_ty;
    a.tz = p_tz + two * (p_rw * x1 - p_rx * x2 - p_ry * x0) + t_tz;
    const V bx0 = ry * ry, bx1 = rz * rz, bx2 = rw * rz, bx3 = rw * ry, bx4 = rx * rx;
    const V bx5 = rw * rx, bx6 = rx * ry, bx7 = rx * rz, bx8 = ry * rz;
    a.xx = mtwo * (bx0 + bx1) + one;
    a.xy = two * (bx6 + bx2);
    a.xz = two * (bx7 - bx3);
    a.yx = two * (bx6 - bx2);
    a.yy = mtwo * (bx1 + bx4) + one;
    a.yz = two * (bx8 + bx5);
    a.zx = two * (bx7 + bx3);
    a.zy = two * (bx8 - bx5);
    a.zz = mtwo * (bx0 + bx4) + one;
    return a;
}
VCPU_INLINE void att_sphere(const EnvView& env, const AttPose& a, int k, V& X, V& Y, V& Z, float& R)
{
    const float* c = env.att + kAttHdr + 4 * k;
    const V c0 = c[0], c1 = c[1], c2 = c[2];
    X = c0 * a.xx + c1 * a.yx + c2 * a.zx + a.tx;
    Y = c0 * a.xy + c1 * a.yy + c2 * a.zy + a.ty;
    Z = c0 * a.xz + c1 * a.yz + c2 * a.zz + a.tz;
    R = c[3];
}

}  // namespace vcpu
