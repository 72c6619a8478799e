// vgpu_roadmap_assemble.hip -- Roadmap::build_roadmap's adjacency (planning/prm.hh:270-275) and connected
// components on the device, from the valid (vertex i, neighbour j) pairs in query order (i ascending,
// nearest first) that the edge stage leaves in HBM.  Same output as the host vgpu_roadmap_assemble:
//   adjacency  vertex v's list = its own pairs' j in pair order, then the later vertices i whose pair
//              names v, ascending.  The pairs expand to entries [(i, j), (j, i)] in pair order and a
//              STABLE radix sort by the first element groups them per vertex in that order: v's own
//              pairs all precede any later pair naming v, because pairs come in ascending i.
//   offsets    an atomic histogram of the entries' first elements, exclusive-scanned (widened to 64 bits).
//   component  the smallest vertex index of v's component: hooking by atomicMin of the larger root
//              onto the smaller one (a parent is never above its child, so a root is its tree's minimum)
//              plus pointer jumping, repeated until no pair joins two trees.
// At the configs[3] size (2.68M vertices, ~108M valid pairs) this replaces 1.3 s of host assembly.
#include <hipcub/hipcub.hpp>

#include "vgpu_device.hh"

namespace vgpu {
namespace asmb {

__global__ __launch_bounds__(256) void expand_kernel(const uint32_t* __restrict__ pairs, size_t m, uint32_t n,
                                                     uint32_t* __restrict__ key, uint32_t* __restrict__ val,
                                                     uint32_t* __restrict__ bad)
{
    const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= m) return;
    const uint32_t i = pairs[2 * p], j = pairs[2 * p + 1];
    if (i >= n || j >= n) {
        *bad = 1u;
        key[2 * p] = key[2 * p + 1] = 0u;  // keeps the sort and the histogram in bounds; the call fails
        val[2 * p] = val[2 * p + 1] = 0u;
        return;
    }
    key[2 * p] = i;
    val[2 * p] = j;
    key[2 * p + 1] = j;
    val[2 * p + 1] = i;
}

// offsets from the SORTED keys: off[v] = the first position whose key is >= v (the exclusive scan of the
// per-vertex counts, without 2m random atomics -- 10 ms of the 2.68M-vertex step in round 4's profile); each
// position writes the offsets of the vertices between its predecessor's key and its own, the last one the tail
__global__ __launch_bounds__(256) void bounds_kernel(const uint32_t* __restrict__ key, size_t e, uint32_t n,
                                                     unsigned long long* __restrict__ off)
{
    const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (p > e) return;
    const uint32_t lo = p == 0 ? 0u : key[p - 1] + 1u;  // vertices lo .. hi start at position p
    const uint32_t hi = p == e ? n : key[p];
    for (uint32_t v = lo; v <= hi; ++v) off[v] = p;
}

__global__ __launch_bounds__(256) void widen_kernel(const uint32_t* __restrict__ off32, uint32_t n1,
                                                    unsigned long long* __restrict__ off64)
{
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v < n1) off64[v] = off32[v];
}

__global__ __launch_bounds__(256) void iota_kernel(uint32_t n, uint32_t* __restrict__ parent)
{
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v < n) parent[v] = v;
}

__device__ __forceinline__ uint32_t root_of(const uint32_t* parent, uint32_t x)
{
    for (uint32_t p = parent[x]; p != x; p = parent[x]) x = p;
    return x;
}

__global__ __launch_bounds__(256) void hook_kernel(const uint32_t* __restrict__ pairs, size_t m, uint32_t* parent,
                                                   uint32_t* __restrict__ changed)
{
    const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= m) return;
    const uint32_t a = root_of(parent, pairs[2 * p]), b = root_of(parent, pairs[2 * p + 1]);
    if (a == b) return;
    atomicMin(&parent[a > b ? a : b], a < b ? a : b);
    *changed = 1u;
}

__global__ __launch_bounds__(256) void jump_kernel(uint32_t n, uint32_t* parent)
{
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v < n) parent[v] = root_of(parent, v);
}

}  // namespace asmb
}  // namespace vgpu

extern "C" {

static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

static int bits_of(uint32_t n)
{
    int b = 1;
    while (b < 32 && ((uint64_t)1 << b) < n) ++b;
    return b;
}

// scratch bytes of vgpu_launch_roadmap_assemble (0: unsupported size)
size_t vgpu_roadmap_assemble_bytes(uint32_t n, size_t m)
{
    if (2 * m >= ((size_t)1 << 31)) return 0;
    const int e = (int)(2 * m);
    size_t ts = 0, tc = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, ts, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, e, 0, bits_of(n)) != hipSuccess)
        return 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, tc, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n + 1) != hipSuccess)
        return 0;
    return 3 * al256(2 * m * 4) + 2 * al256(((size_t)n + 1) * 4) + al256(16) + al256(std::max(ts, tc));  // (cnt unused)
}

// pairs[m][2], offsets[n + 1], adj[2m], component[n] (optional): device memory.  *flags (host) gets
// bit 0 = a pair index >= n (nothing else is then written).  Host syncs: one after the expansion, one per
// hooking round, one at the end.
hipError_t vgpu_launch_roadmap_assemble(uint32_t n, const uint32_t* pairs, size_t m, unsigned long long* offsets,
                                        uint32_t* adj, uint32_t* component, void* tmp, size_t tmp_bytes,
                                        uint32_t* flags, hipStream_t st)
{
    using namespace vgpu::asmb;
    *flags = 0;
    if (n == 0) return hipSuccess;
    char* t = (char*)tmp;
    const size_t e = 2 * m;
    uint32_t* key = (uint32_t*)t;
    t += al256(e * 4);
    uint32_t* key2 = (uint32_t*)t;
    t += al256(e * 4);
    uint32_t* val = (uint32_t*)t;
    t += al256(e * 4);
    uint32_t* cnt = (uint32_t*)t;
    t += al256(((size_t)n + 1) * 4);
    uint32_t* off32 = (uint32_t*)t;
    t += al256(((size_t)n + 1) * 4);
    uint32_t* dflag = (uint32_t*)t;  // [0] = bad pair, [1] = changed
    t += al256(16);
    void* work = t;
    const size_t work_bytes = tmp_bytes - (size_t)(t - (char*)tmp);
    hipError_t err;
    (void)cnt;
    (void)off32;
    if ((err = hipMemsetAsync(dflag, 0, 16, st)) != hipSuccess) return err;
    if (m) {
        hipLaunchKernelGGL(expand_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, pairs, m, n, key, val,
                           dflag);
        if ((err = hipGetLastError()) != hipSuccess) return err;
        uint32_t bad = 0;  // an index >= n would send the hooking below out of bounds: fail first
        if ((err = hipMemcpyAsync(&bad, dflag, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return err;
        if ((err = hipStreamSynchronize(st)) != hipSuccess) return err;
        if (bad) {
            *flags = 1u;
            return hipSuccess;
        }
        size_t wb = work_bytes;
        if ((err = hipcub::DeviceRadixSort::SortPairs(work, wb, key, key2, val, adj, (int)e, 0, bits_of(n), st)) !=
            hipSuccess)
            return err;
    }
    hipLaunchKernelGGL(bounds_kernel, dim3((unsigned)((e + 1 + 255) / 256)), dim3(256), 0, st, key2, e, n, offsets);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    if (component) {
        hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, component);
        if ((err = hipGetLastError()) != hipSuccess) return err;
        while (m) {  // each round with a change joins at least two trees: <= n rounds, a few in practice
            if ((err = hipMemsetAsync(dflag + 1, 0, 4, st)) != hipSuccess) return err;
            hipLaunchKernelGGL(hook_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, pairs, m, component,
                               dflag + 1);
            hipLaunchKernelGGL(jump_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, component);
            if ((err = hipGetLastError()) != hipSuccess) return err;
            uint32_t changed = 0;
            if ((err = hipMemcpyAsync(&changed, dflag + 1, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return err;
            if ((err = hipStreamSynchronize(st)) != hipSuccess) return err;
            if (!changed) break;
        }
    }
    return hipStreamSynchronize(st);
}

}  // extern "C"
