// vgpu_capt_grid.hip -- the cell grid of a device point cloud: an acceleration structure over the
// CAPT (collision/capt.hh:91-398) that decides most queries with one 8-byte load and starts the
// rest below the root.  It changes no answer: every bound is taken over exactly the affordances
// the reference's traversal can reach from the cell, and query_lane (vgpu_device.hh capt_lane)
// falls back to that traversal whenever a bound does not decide.
//
// Grid: a box of nx * ny * nz cubic cells of side h = 1 / inv_h from (x0, y0, z0) (the CAPT's top
// box grown by r_max + r_point on every side).  A centre x lands in cell floor((x - x0) * inv_h)
// evaluated in float; that is within 3e-5 cells of the exact quotient for up to ~1000 cells per
// axis, so the EXPANDED cell [i - kSlack, i + 1 + kSlack] * h (kSlack = 1e-3) contains every
// centre the device puts in cell i.  Per cell, one thread, in double:
//   node  the deepest split node whose region contains the whole expanded cell: every split above
//         it sends the whole cell one way (a >= t for all a when lo >= t; a < t for all when
//         hi < t or t is NaN -- the device's `a >= t` is false on NaN), so a descent from it
//         reaches the same leaf as one from the root;
//   lo    min over the leaves the cell can reach (both sides of each split it straddles) of the
//         least distance from the cell to an affordance of the leaf (point-to-box distance);
//   hi    max over those leaves of min over the leaf's affordances of the FARTHEST-corner
//         distance: some affordance of whichever leaf is reached lies within hi of any centre.
// lo is rounded down and hi up to multiples of unit = h / 256 (16 bits each; 0xFFFF = no bound:
// a cell with an empty leaf or more than kMaxLeaves reachable leaves).  The device tests
// (r + r_point)^2 < (lo)^2 * 0.9999 -> miss and > (hi)^2 * 1.0001 -> hit: the reference's
// fma sum-of-squares differs from the exact squared distance by < 1e-6 relative (all terms
// non-negative), and the float products of the bound by < 1e-6.
#include "vgpu_capt.hh"
#include "vgpu_device.hh"

namespace vgpu {

constexpr double kSlack = 1e-3;
constexpr int kMaxLeaves = 64;
constexpr int kGridBlock = 256;

// the float next to finite f toward -inf / +inf
__device__ __forceinline__ float next_down(float f)
{
    const uint32_t b = __float_as_uint(f);
    if (f == 0.0f) return -__uint_as_float(1u);
    return __uint_as_float(f > 0.0f ? b - 1u : b + 1u);
}
__device__ __forceinline__ float next_up(float f) { return -next_down(-f); }
__device__ __forceinline__ float round_down(double x)
{
    const float f = (float)x;
    return (double)f > x ? next_down(f) : f;
}
__device__ __forceinline__ float round_up(double x)
{
    const float f = (float)x;
    return (double)f < x ? next_up(f) : f;
}

// (Round 5: skipping a reachable leaf's affordance loop when a per-leaf box / representative-affordance test shows
// it cannot move either bound -- exact -- measured no gain on MI355X: 1.73 -> 1.79 ms for 2M cells plus 0.05 ms
// for the summaries, profiles/r05j_capt_rel_kernel_stats.csv; most cells reach one or two leaves, whose loops
// decide the bounds.)
// One thread per cell.  The walk's stack lives in LDS (a private array indexed by a variable would go to
// scratch memory), and the affordance loop runs in float over the expanded cell rounded OUTWARD to float
// (a larger box: lo can only shrink and hi only grow), so its float rounding (< 1e-6 relative on distances
// of a few metres) only loosens bounds that are then rounded by a further whole unit (h / 256) -- every
// bound stays conservative.  The descent and the choice of leaves compare the split values with the
// double cell bounds, as before.
// kStackDepth: a depth-first walk of a tree of depth nlog2 holds <= nlog2 + 1 nodes; the launcher takes the 16-deep
// stack (16 KB of LDS per block instead of 32 KB) for trees of depth < 16.
template <int kStackDepth>
__global__ __launch_bounds__(kGridBlock) void capt_grid_kernel(float* __restrict__ base, CaptGridArgs g)
{
    __shared__ uint32_t stk[kStackDepth][kGridBlock];
    const uint32_t cell = blockIdx.x * (uint32_t)kGridBlock + threadIdx.x;
    const uint32_t n_cells = g.nx * g.ny * g.nz;
    if (cell >= n_cells) return;
    uint32_t ix, iy, iz;  // the cell whose bounds this thread writes at storage index `cell`
    if (g.brick) {
        const uint32_t b = cell >> 6, l = cell & 63u, nbx = g.nx >> 2, nby = g.ny >> 2;
        ix = (b % nbx) * 4u + (l & 3u);
        iy = ((b / nbx) % nby) * 4u + ((l >> 2) & 3u);
        iz = (b / (nbx * nby)) * 4u + (l >> 4);
    } else {
        ix = cell % g.nx;
        iy = (cell / g.nx) % g.ny;
        iz = cell / (g.nx * g.ny);
    }
    const double h = 1.0 / (double)g.inv_h;
    const double o[3] = {(double)g.x0, (double)g.y0, (double)g.z0};
    const uint32_t ic[3] = {ix, iy, iz};
    double L[3], U[3];
    float Lf[3], Uf[3];
    for (int k = 0; k < 3; ++k) {
        L[k] = o[k] + ((double)ic[k] - kSlack) * h;
        U[k] = o[k] + ((double)ic[k] + 1.0 + kSlack) * h;
        Lf[k] = round_down(L[k]);
        Uf[k] = round_up(U[k]);
    }
    const float* __restrict__ tests = base + g.tests_off;
    const uint32_t* __restrict__ starts = (const uint32_t*)(base + g.starts_off);
    const float* __restrict__ aff = base + g.aff_off;
    const int nlog2 = g.nlog2;

    // the deepest node containing the whole expanded cell
    uint32_t node = 0;
    for (int lv = 0; lv < nlog2; ++lv) {
        const float t = tests[node];
        const int ax = lv % 3;
        if (L[ax] >= (double)t) node = 2u * node + 2u;                 // every a >= t
        else if (U[ax] < (double)t || t != t) node = 2u * node + 1u;  // no a >= t
        else break;
    }
    // the leaves reachable from it, depth first
    float lo2 = __builtin_inff(), hi2 = 0.0f;
    int leaves = 0;
    bool bounded = nlog2 < kStackDepth;
    int sp = 0;
    const uint32_t tx = threadIdx.x;
    stk[sp++][tx] = node;
    const uint32_t first_leaf = (1u << nlog2) - 1u;
    while (sp > 0 && bounded) {
        const uint32_t n = stk[--sp][tx];
        if (n >= first_leaf) {
            if (++leaves > kMaxLeaves) {
                bounded = false;
                break;
            }
            const uint32_t leaf = n - first_leaf;
            float lmin = __builtin_inff(), hmin = __builtin_inff();
            for (uint32_t j = starts[leaf], e = starts[leaf + 1]; j < e; ++j) {
                const float* v = aff + 24u * j;
#pragma unroll
                for (int l = 0; l < 8; ++l) {
                    // no finiteness test: the +inf padding gives dn = df = +inf (no effect on either min), and a
                    // NaN coordinate gives dn = 0 (max ignores NaN: lo only shrinks) and df = NaN (min ignores it)
                    const float p[3] = {v[l], v[8 + l], v[16 + l]};
                    float dn = 0.0f, df = 0.0f;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const float a = Lf[k] - p[k], b = p[k] - Uf[k];
                        const float near = fmaxf(fmaxf(a, b), 0.0f);  // v_max3
                        const float far = fmaxf(fabsf(a), fabsf(b));   // |p - Lf|, |p - Uf|: abs source modifiers
                        dn = __builtin_fmaf(near, near, dn);
                        df = __builtin_fmaf(far, far, df);
                    }
                    lmin = fminf(lmin, dn);
                    hmin = fminf(hmin, df);
                }
            }
            lo2 = fminf(lo2, lmin);
            hi2 = fmaxf(hi2, hmin);  // an empty leaf: +inf, no hit bound
            continue;
        }
        const int lv = 31 - __builtin_clz(n + 1u);
        const float t = tests[n];
        const int ax = lv % 3;
        if (sp + 2 > kStackDepth) {
            bounded = false;
            break;
        }
        if (U[ax] >= (double)t) stk[sp++][tx] = 2u * n + 2u;             // some a >= t
        if (L[ax] < (double)t || t != t) stk[sp++][tx] = 2u * n + 1u;    // some a < t (or NaN t)
    }
    uint32_t lq = 0u, hq = 0xFFFFu;
    if (bounded) {
        // float rounding of the squared sums and of sqrt: < 4e-7 relative; taken off lo and added to hi
        // before the extra whole unit below
        const double u = (double)g.unit;
        const double lo = sqrt((double)lo2) * (1.0 - 1e-6) / u, hi = sqrt((double)hi2) * (1.0 + 1e-6) / u;
        // round lo down and hi up by one extra unit
        lq = lo >= 65535.0 ? 65535u : (uint32_t)fmax(floor(lo) - 1.0, 0.0);
        hq = hi + 1.0 < 65535.0 ? (uint32_t)ceil(hi) + 1u : 0xFFFFu;
    }
    if (g.nodes_off) {
        ((uint32_t*)(base + g.cells_off))[cell] = lq | (hq << 16);
        ((uint32_t*)(base + g.nodes_off))[cell] = node;
    } else {
        ((uint2*)(base + g.cells_off))[cell] = make_uint2(lq | (hq << 16), node);
    }
}

}  // namespace vgpu

extern "C" hipError_t vgpu_launch_capt_grid(float* base, const vgpu::CaptGridArgs* g, hipStream_t st)
{
    const uint64_t n = (uint64_t)g->nx * g->ny * g->nz;
    if (n == 0) return hipSuccess;
    if (n >= ((uint64_t)1 << 31)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((n + vgpu::kGridBlock - 1) / vgpu::kGridBlock)), block(vgpu::kGridBlock);
    if (g->nlog2 < 16)
        hipLaunchKernelGGL(vgpu::capt_grid_kernel<16>, grid, block, 0, st, base, *g);
    else
        hipLaunchKernelGGL(vgpu::capt_grid_kernel<32>, grid, block, 0, st, base, *g);
    return hipGetLastError();
}
