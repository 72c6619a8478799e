// vcpu_roadmap.cpp -- the PRM edge stage's neighbour queries on the host CPU: an exact k-d tree over the
// roadmap's vertices (the role nigh's KD-tree plays in the reference, planning/nn.hh:89-95, a CPM
// dependency absent from the image), answering build_roadmap's causal query for vertex i (prm.hh:264-266):
// the k(i) nearest of vertices 0 .. i-1 within r(i) (PRMStarNeighborParams, roadmap.hh:42-77), by
// Space<dim>::distance = (a - b).l2_norm() in the reference's AVX lane order (nn.hh:53-57, vgpu_l2_norm).
// The result is the same list the GPU kernels produce (vgpu_roadmap_knn): the k smallest (distance,
// index) keys with distance <= r, ascending.
//
// The tree is static and built once over all n vertices; every node keeps the smallest vertex index of
// its subtree, so the query for vertex i skips subtrees holding only later vertices (the incremental
// insertion order of the reference is recovered without rebuilding).  Subtrees are pruned with a double
// precision box distance against the current admission threshold widened by a relative 1e-5 (the float
// distance of a point may undercut its exact one by a few ulps): pruning is exact, the admitted keys are
// the float distances of the candidates.  Queries are spread over threads (dynamic chunks).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "../../../include/vamp_gpu.h"
#include "../vgpu_abi.hh"
#include "vcpu_robot.hh"

namespace {

constexpr int kLeaf = 16;
constexpr int kMaxD = 16;

struct KdNode {
    int lo, hi;            // range of the permutation (leaf) or of the subtree
    int left, right;       // children (-1 at a leaf)
    uint32_t min_index;    // smallest vertex index in the subtree
    float bmin[kMaxD], bmax[kMaxD];
};

struct KdTree {
    int dim = 0;
    const float* V = nullptr;
    std::vector<uint32_t> perm;
    std::vector<KdNode> nodes;

    int build(int lo, int hi)
    {
        KdNode nd;
        nd.lo = lo;
        nd.hi = hi;
        nd.left = nd.right = -1;
        nd.min_index = 0xFFFFFFFFu;
        for (int d = 0; d < dim; ++d) {
            nd.bmin[d] = INFINITY;
            nd.bmax[d] = -INFINITY;
        }
        for (int i = lo; i < hi; ++i) {
            const float* p = V + (size_t)perm[i] * dim;
            nd.min_index = std::min(nd.min_index, perm[i]);
            for (int d = 0; d < dim; ++d) {
                nd.bmin[d] = std::min(nd.bmin[d], p[d]);
                nd.bmax[d] = std::max(nd.bmax[d], p[d]);
            }
        }
        const int id = (int)nodes.size();
        nodes.push_back(nd);
        if (hi - lo > kLeaf) {
            int ax = 0;
            float w = -1.0f;
            for (int d = 0; d < dim; ++d)
                if (nd.bmax[d] - nd.bmin[d] > w) w = nd.bmax[d] - nd.bmin[d], ax = d;
            const int mid = (lo + hi) / 2;
            std::nth_element(perm.begin() + lo, perm.begin() + mid, perm.begin() + hi, [&](uint32_t a, uint32_t b) {
                const float pa = V[(size_t)a * dim + ax], pb = V[(size_t)b * dim + ax];
                return pa < pb || (pa == pb && a < b);
            });
            const int l = build(lo, mid);
            const int r = build(mid, hi);
            nodes[id].left = l;
            nodes[id].right = r;
        }
        return id;
    }
};

struct Key {
    float d;
    uint32_t i;
    bool operator<(const Key& o) const { return d < o.d || (d == o.d && i < o.i); }
};

// the k smallest keys within r among vertices < q (max-heap of the admitted keys)
void query(const KdTree& T, uint32_t q, uint32_t k, float r, std::vector<Key>& heap)
{
    heap.clear();
    if (k == 0 || q == 0) return;
    const int dim = T.dim;
    const float* x = T.V + (size_t)q * dim;
    float diff[kMaxD];
    struct Item {
        double lb;
        int node;
    };
    Item stack[128];
    int sp = 0;
    stack[sp++] = {0.0, 0};
    auto thr = [&]() -> double { return heap.size() < k ? (double)r : (double)heap.front().d; };
    while (sp) {
        const Item it = stack[--sp];
        const KdNode& nd = T.nodes[it.node];
        if (nd.min_index >= q) continue;
        if (it.lb > thr() * (1.0 + 1e-5) + 1e-7) continue;
        if (nd.left < 0) {
            for (int j = nd.lo; j < nd.hi; ++j) {
                const uint32_t v = T.perm[j];
                if (v >= q) continue;
                const float* p = T.V + (size_t)v * dim;
                for (int d = 0; d < dim; ++d) diff[d] = p[d] - x[d];  // Space::distance(a, b) = (b - a) norm
                const float dist = vcpu::l2_norm(diff, dim);
                if (!(dist <= r)) continue;
                const Key key{dist, v};
                if (heap.size() < k) {
                    heap.push_back(key);
                    std::push_heap(heap.begin(), heap.end());
                } else if (key < heap.front()) {
                    std::pop_heap(heap.begin(), heap.end());
                    heap.back() = key;
                    std::push_heap(heap.begin(), heap.end());
                }
            }
            continue;
        }
        // children nearest-box first (pushed last)
        double lb[2];
        const int ch[2] = {nd.left, nd.right};
        for (int c = 0; c < 2; ++c) {
            const KdNode& cn = T.nodes[ch[c]];
            double s = 0.0;
            for (int d = 0; d < dim; ++d) {
                const double v = x[d];
                const double e = v < cn.bmin[d] ? cn.bmin[d] - v : (v > cn.bmax[d] ? v - cn.bmax[d] : 0.0);
                s += e * e;
            }
            lb[c] = std::sqrt(s);
        }
        const int first = lb[0] <= lb[1] ? 0 : 1;
        if (sp + 2 > 128) continue;  // depth is log2(n / 16) < 40: never
        stack[sp++] = {lb[1 - first], ch[1 - first]};
        stack[sp++] = {lb[first], ch[first]};
    }
}

}  // namespace

// Neighbour lists of build_roadmap's causal queries for the listed vertices (queries[m] vertex indices,
// any order): nbr/dist [m][kmax], cnt[m] (row m = queries[m]); k[i], r[i] indexed by vertex.  threads <= 0:
// every hardware thread.
extern "C" int vgpu_cpu_roadmap_knn(int dim, const float* V, size_t n, const uint32_t* queries, size_t m,
                                    const uint32_t* k, const float* r, uint32_t kmax, uint32_t* nbr, float* dist,
                                    uint32_t* cnt, int threads)
try {
    if (dim < 1 || dim > kMaxD || n >= 0x7FFFFFFFu || kmax < 1) return VGPU_ERR_INVALID_ARG;
    if (m == 0) return VGPU_OK;
    if (!V || !queries || !k || !r || !nbr || !dist || !cnt) return VGPU_ERR_INVALID_ARG;
    for (size_t j = 0; j < m; ++j)
        if (queries[j] >= n) return VGPU_ERR_INVALID_ARG;
    KdTree T;
    T.dim = dim;
    T.V = V;
    T.perm.resize(n);
    for (size_t i = 0; i < n; ++i) T.perm[i] = (uint32_t)i;
    T.nodes.reserve(2 * (n / kLeaf + 1));
    if (n) T.build(0, (int)n);
    unsigned nt = threads > 0 ? (unsigned)threads : std::max(1u, std::thread::hardware_concurrency());
    nt = (unsigned)std::min<size_t>(nt, m);
    std::atomic<size_t> next{0};
    auto work = [&]() {
        std::vector<Key> heap;
        heap.reserve(kmax);
        for (;;) {
            const size_t lo = next.fetch_add(256);
            if (lo >= m) break;
            const size_t hi = std::min(m, lo + 256);
            for (size_t j = lo; j < hi; ++j) {
                const uint32_t q = queries[j];
                query(T, q, std::min(k[q], kmax), r[q], heap);
                std::sort_heap(heap.begin(), heap.end());
                cnt[j] = (uint32_t)heap.size();
                for (size_t t = 0; t < heap.size(); ++t) {
                    nbr[j * kmax + t] = heap[t].i;
                    dist[j * kmax + t] = heap[t].d;
                }
            }
        }
    };
    std::vector<std::thread> pool;  // workers take rows from a shared counter: fewer threads only take longer
    try {
        for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work);
    } catch (...) {
    }
    work();
    for (auto& th : pool) th.join();
    return VGPU_OK;
} VGPU_ABI_CATCH
