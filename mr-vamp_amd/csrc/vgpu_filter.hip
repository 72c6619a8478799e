// vgpu_filter.hip -- the point-cloud filter (reference collision/filter.hh:175-268) on the GPU.
//
// The reference runs six space-filling-curve passes on one core: Morton-key every surviving
// point, pdqsort by key, then a sequential scan that keeps a point only if it lies farther than
// min_dist from the LAST KEPT point.  That scan is a chain (kept_{k+1} = next(kept_k) with
// next(i) = first j > i farther than min_dist from i), so per pass the GPU
//   1. keys every point (remap_point + morton_pdep, filter.hh:101-127) and reduces the pass's
//      coordinate min/max for the next pass's bounds,
//   2. radix-sorts (key, index) pairs (stable: ties keep the previous pass's order),
//   3. computes next(i) for every sorted position in parallel (a short forward scan in Morton
//      order, where close points are adjacent),
//   4. marks the chain from position 0 by pointer doubling (ceil(log2 len) rounds),
//   5. compacts the marked positions in order.
// The result equals the sequential scan for every input; the order among equal keys follows
// the stable sort (the reference's pdqsort is unstable there: parity unpinned on ties).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <mutex>

// the block reductions below (shuffle offsets 32..1, one leader per 64 lanes) assume wave64,
// which gfx950 always runs; any other device target is refused at compile time
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "vgpu_filter.hip: the min/max reductions are written for wave64 gfx950"
#endif

namespace {

struct Bounds {
    float mn, mx;    // the pass's remap range
    float nmn, nmx;  // running min/max of coordinates over the pass (filter.hh:225-233)
};

__device__ inline float sql2_3(float ax, float ay, float az, float bx, float by, float bz)
{
    // sql2_3 as the oracle restates it for the reference's compiled code (math.hh:17-42 under
    // -ffp-contract=fast, oracle/vamp_oracle.c sumsq_vec): fmaf(dx, dx, fmaf(dz, dz, dy*dy))
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    return __builtin_fmaf(dx, dx, __builtin_fmaf(dz, dz, dy * dy));
}

__device__ inline uint32_t remap_point(float x, float mn, float mx)
{
    const float q = __fmul_rn(__fdiv_rn(x - mn, mx - mn), 1000.0f);
    if (!(q > -9.2233715e18f && q < 9.2233715e18f)) return 0u;
    return (uint32_t)(uint64_t)(int64_t)q;  // GCC x86-64 float -> uint32 (low word of cvttss2si)
}

__device__ inline uint32_t spread3(uint32_t v, int nbits, int lane)
{
    uint32_t out = 0;
    for (int i = 0; i < nbits; ++i) out |= ((v >> i) & 1u) << (3 * i + lane);
    return out;
}

__device__ inline uint32_t morton(uint32_t x, uint32_t y, uint32_t z)
{
    // _pdep_u32 with MORTON_X/Y/Z_MASK: 11, 11 and 10 low bits deposited
    return spread3(x, 11, 0) | spread3(y, 11, 1) | spread3(z, 10, 2);
}

__global__ void cull_kernel(const float* __restrict__ pc, uint32_t n, float sqrange, float ox, float oy, float oz,
                            float lx, float ly, float lz, float ux, float uy, float uz, int cull,
                            uint8_t* __restrict__ flag)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* p = pc + 3 * (size_t)i;
    const float x = p[0], y = p[1], z = p[2];
    flag[i] = !cull || (sql2_3(x, y, z, ox, oy, oz) < sqrange && lx <= x && x <= ux && ly <= y && y <= uy &&
                        lz <= z && z <= uz);
}

__global__ void iota_kernel(uint32_t* __restrict__ v, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// keys of the current list under coordinate permutation (c0, c1, c2); each block's coordinate
// min/max to part[2 * blockIdx.x + {0, 1}] (no same-address atomics)
__global__ __launch_bounds__(256) void key_kernel(const float* __restrict__ pc, const uint32_t* __restrict__ idx,
                                                  uint32_t len, int c0, int c1, int c2, const Bounds* b,
                                                  float* __restrict__ part, uint32_t* __restrict__ key)
{
    __shared__ float slo[4], sup[4];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const float mn = b->mn, mx = b->mx;
    float lo = 3.4e38f, up = -3.4e38f;
    if (i < len) {
        const float* p = pc + 3 * (size_t)idx[i];
        key[i] = morton(remap_point(p[c0], mn, mx), remap_point(p[c1], mn, mx), remap_point(p[c2], mn, mx));
        lo = fminf(p[0], fminf(p[1], p[2]));
        up = fmaxf(p[0], fmaxf(p[1], p[2]));
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, off));
        up = fmaxf(up, __shfl_xor(up, off));
    }
    if ((threadIdx.x & 63) == 0) {
        slo[threadIdx.x >> 6] = lo;
        sup[threadIdx.x >> 6] = up;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = fminf(fminf(slo[0], slo[1]), fminf(slo[2], slo[3]));
        part[2 * blockIdx.x + 1] = fmaxf(fmaxf(sup[0], sup[1]), fmaxf(sup[2], sup[3]));
    }
}

// the next pass's bounds (filter.hh:262-263) from the block partials: nmn starts at mx, nmx at mn
__global__ __launch_bounds__(1024) void bounds_kernel(Bounds* b, const float* __restrict__ part, uint32_t nparts)
{
    __shared__ float slo[16], sup[16];
    float lo = 3.4e38f, up = -3.4e38f;
    for (uint32_t k = threadIdx.x; k < nparts; k += blockDim.x) {
        lo = fminf(lo, part[2 * k]);
        up = fmaxf(up, part[2 * k + 1]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, off));
        up = fmaxf(up, __shfl_xor(up, off));
    }
    if ((threadIdx.x & 63) == 0) {
        slo[threadIdx.x >> 6] = lo;
        sup[threadIdx.x >> 6] = up;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) {
            lo = fminf(lo, slo[w]);
            up = fmaxf(up, sup[w]);
        }
        lo = fminf(slo[0], lo);
        up = fmaxf(sup[0], up);
        const float nmn = fminf(b->mx, lo), nmx = fmaxf(b->mn, up);
        const float mx = (float)((double)(nmx + b->mx) / 2.0), mn = (float)((double)(nmn + b->mn) / 2.0);
        b->mn = mn;
        b->mx = mx;
    }
}

// next(i): first sorted position j > i farther than min_dist from i, else len
__global__ void next_kernel(const float* __restrict__ pc, const uint32_t* __restrict__ sidx, uint32_t len,
                            float sqd, uint32_t* __restrict__ jump, uint8_t* __restrict__ on)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const float* a = pc + 3 * (size_t)sidx[i];
    const float ax = a[0], ay = a[1], az = a[2];
    uint32_t j = i + 1;
    for (; j < len; ++j) {
        const float* p = pc + 3 * (size_t)sidx[j];
        if (sql2_3(p[0], p[1], p[2], ax, ay, az) > sqd) break;
    }
    jump[i] = j;
    on[i] = (i == 0);
}

// one doubling round: chain flags only ever go 0 -> 1 (in place; a flag set earlier in the same
// round only marks chain nodes sooner), jump pointers double into the other buffer
__global__ void double_kernel(const uint32_t* __restrict__ jin, uint32_t* __restrict__ jout, uint8_t* on,
                              uint32_t len)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const uint32_t j = jin[i];
    if (on[i] && j < len) on[j] = 1;
    jout[i] = j < len ? jin[j] : len;
}

inline unsigned blocks(size_t n) { return (unsigned)((n + 255) / 256); }

constexpr int kMaxDevices = 64;
struct Pool {
    char* base = nullptr;
    size_t cap = 0;
};
Pool g_pools[kMaxDevices];
std::mutex g_pool_mu[kMaxDevices];  // one lock per device: calls on different devices run concurrently

}  // namespace

#define FCHK(x)                                   \
    do {                                          \
        hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) { release(); return e_; } \
    } while (0)

// d_pc: n x 3 f32 on the device; d_out: n u32 on the device (kept indices, final order);
// *count: number kept.  Synchronous on `s`.
extern "C" hipError_t vgpu_filter_pointcloud_run(const float* d_pc, size_t n, float min_dist, float max_range,
                                      const float origin[3], const float ws_min[3], const float ws_max[3], int cull,
                                      uint32_t* d_out, size_t* count, hipStream_t s)
{
    *count = 0;
    if (n == 0) return hipSuccess;
    if (n > 0x7fffffffu) return hipErrorInvalidValue;
    const uint32_t N = (uint32_t)n;
    // scratch: one grow-only pool per device, reused across calls (calls are synchronous and
    // serialised per device by that device's pool lock)
    int dev = 0;
    {
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    }
    std::lock_guard<std::mutex> lock(g_pool_mu[dev]);
    auto release = []() {};
    size_t tsel = 0, tsort = 0;
    FCHK(hipcub::DeviceSelect::Flagged(nullptr, tsel, (uint32_t*)nullptr, (uint8_t*)nullptr, (uint32_t*)nullptr,
                                       (uint32_t*)nullptr, N, s));
    FCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tsort, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                            (uint32_t*)nullptr, (uint32_t*)nullptr, N, 0, 32, s));
    const size_t tbytes = tsel > tsort ? tsel : tsort;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t sizes[11] = {4 * n, 4 * n, 4 * n, 4 * n, 4 * n, 4 * n, n, 4, sizeof(Bounds), 8 * (size_t)blocks(n),
                              tbytes};
    size_t total = 0;
    for (size_t v : sizes) total += al(v ? v : 1);
    Pool& pool = g_pools[dev];
    if (pool.cap < total) {
        if (pool.base) FCHK(hipFree(pool.base));
        pool.base = nullptr;
        pool.cap = 0;
        FCHK(hipMalloc((void**)&pool.base, total));
        pool.cap = total;
    }
    void* ptr[11];
    {
        char* q = pool.base;
        for (int k = 0; k < 11; ++k) {
            ptr[k] = q;
            q += al(sizes[k] ? sizes[k] : 1);
        }
    }
    uint32_t *idx = (uint32_t*)ptr[0], *key = (uint32_t*)ptr[1], *skey = (uint32_t*)ptr[2], *sidx = (uint32_t*)ptr[3];
    uint32_t *j0 = (uint32_t*)ptr[4], *j1 = (uint32_t*)ptr[5], *nsel = (uint32_t*)ptr[7];
    uint8_t* on0 = (uint8_t*)ptr[6];
    Bounds* b = (Bounds*)ptr[8];
    float* part = (float*)ptr[9];
    void* tmp = ptr[10];

    // step 1 (filter.hh:194-214): kept indices first, the rest of the n-long list names point 0
    const float sqd = min_dist * min_dist, sqr = max_range * max_range;
    cull_kernel<<<blocks(n), 256, 0, s>>>(d_pc, N, sqr, origin[0], origin[1], origin[2], ws_min[0], ws_min[1],
                                         ws_min[2], ws_max[0], ws_max[1], ws_max[2], cull, on0);
    FCHK(hipGetLastError());
    iota_kernel<<<blocks(n), 256, 0, s>>>(key, N);
    FCHK(hipGetLastError());
    size_t tb = tbytes;
    FCHK(hipcub::DeviceSelect::Flagged(tmp, tb, key, on0, idx, nsel, N, s));
    uint32_t hi = 0;
    FCHK(hipMemcpyAsync(&hi, nsel, 4, hipMemcpyDeviceToHost, s));
    FCHK(hipStreamSynchronize(s));
    // The reference's list keeps length n, its unfilled tail naming point 0 (filter.hh:194-214).
    // Those N - hi copies share one key, so the stable sort keeps them consecutive, and the scan
    // keeps at most the first of them (the rest are at distance 0 from it, or from the same last
    // kept point); they add nothing to the pass's min/max either.  One copy is therefore exact,
    // and it avoids an O((N - hi)^2) next-scan over a run of identical points.
    uint32_t len = N;
    if (hi < N) {
        FCHK(hipMemsetAsync(idx + hi, 0, 4, s));
        len = hi + 1;
    }

    auto fmin3 = [](float a, float b2, float c) { float m = a; if (b2 < m) m = b2; if (c < m) m = c; return m; };
    Bounds hb;
    hb.mn = fmin3(origin[0] - max_range, origin[1] - max_range, origin[2] - max_range);
    hb.mx = fmin3(origin[0] + max_range, origin[1] + max_range, origin[2] + max_range);  // sic, filter.hh:192
    hb.nmn = hb.nmx = 0.f;
    FCHK(hipMemcpyAsync(b, &hb, sizeof hb, hipMemcpyHostToDevice, s));

    static const int perms[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
    for (int pi = 0; pi < 6; ++pi) {
        key_kernel<<<blocks(len), 256, 0, s>>>(d_pc, idx, len, perms[pi][0], perms[pi][1], perms[pi][2], b, part,
                                               key);
        FCHK(hipGetLastError());
        bounds_kernel<<<1, 1024, 0, s>>>(b, part, blocks(len));
        FCHK(hipGetLastError());
        tb = tbytes;
        FCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, skey, idx, sidx, len, 0, 32, s));
        next_kernel<<<blocks(len), 256, 0, s>>>(d_pc, sidx, len, sqd, j0, on0);
        FCHK(hipGetLastError());
        uint32_t *ja = j0, *jb = j1;
        for (uint32_t reach = 1; reach < len; reach <<= 1) {
            double_kernel<<<blocks(len), 256, 0, s>>>(ja, jb, on0, len);
            FCHK(hipGetLastError());
            uint32_t* tj = ja; ja = jb; jb = tj;
        }
        tb = tbytes;
        FCHK(hipcub::DeviceSelect::Flagged(tmp, tb, sidx, on0, idx, nsel, len, s));
        FCHK(hipMemcpyAsync(&len, nsel, 4, hipMemcpyDeviceToHost, s));
        FCHK(hipStreamSynchronize(s));
    }
    FCHK(hipMemcpyAsync(d_out, idx, 4 * (size_t)len, hipMemcpyDeviceToDevice, s));
    FCHK(hipStreamSynchronize(s));
    *count = len;
    release();
    return hipSuccess;
}
