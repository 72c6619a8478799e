// vgpu_capt.cpp -- CAPT construction (collision/capt.hh:137-398), host side.
//
// Output arrays are identical to the reference's CAPT members (tests, aabbs, aff_starts,
// affordances) for tie-free point sets.  Floating-point forms follow the reference release
// build (pinned by oracle/_ref/ref_probe "capt_box"): scalar sums of squares compile to
// fma(d2, d2, fma(d0, d0, d1 * d1)); compiled here with -ffp-contract=off and explicit fmaf.
#include "vgpu_capt.hh"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <numeric>

namespace vgpu {
namespace {

constexpr float kInf = std::numeric_limits<float>::infinity();

struct Box {
    float lo[3], up[3];
    void grow(const float* p)  // Volume::extend (capt.hh:60-68)
    {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            up[k] = std::max(up[k], p[k]);
        }
    }
    float dist2(const float* p) const  // Volume::distsq_to (capt.hh:79-86)
    {
        float d[3];
        for (int k = 0; k < 3; ++k) d[k] = p[k] - std::clamp(p[k], lo[k], up[k]);
        return std::fmaf(d[2], d[2], std::fmaf(d[0], d[0], d[1] * d[1]));
    }
    bool inside_ball(const float* p, float r2) const  // contained_by_internal_ball (capt.hh:70-77)
    {
        float d[3];
        for (int k = 0; k < 3; ++k) d[k] = std::max(p[k] - lo[k], up[k] - p[k]);
        return std::fmaf(d[2], d[2], std::fmaf(d[0], d[0], d[1] * d[1])) <= r2;
    }
};

struct Builder {
    const std::vector<float>& pts;  // padded to 2^nlog2 points
    std::vector<uint32_t> order;    // the reference's argsort
    float r_max, aff_l2, min_l2;
    CaptTree& t;
    Box top{{kInf, kInf, kInf}, {-kInf, -kInf, -kInf}};

    const float* P(uint32_t i) const { return &pts[3 * (size_t)i]; }

    void leaf(uint32_t begin, const std::vector<uint32_t>& afford, const Box& cell)
    {
        const float* rep = P(order[begin]);
        Box box{{rep[0], rep[1], rep[2]}, {rep[0], rep[1], rep[2]}};
        if (std::isfinite(rep[0])) {
            top.grow(rep);
            float v[24];
            std::fill(v, v + 24, 0.0f);
            int j = 0;
            auto put = [&](const float* p) {
                v[j] = p[0];
                v[8 + j] = p[1];
                v[16 + j] = p[2];
                if (++j == 8) {
                    t.aff.insert(t.aff.end(), v, v + 24);
                    j = 0;
                }
            };
            put(rep);  // the cell's representative comes first
            if (!cell.inside_ball(rep, min_l2))
                for (uint32_t id : afford)
                    if (cell.dist2(P(id)) <= aff_l2) {
                        box.grow(P(id));
                        put(P(id));
                    }
            if (j > 0) {
                for (int k = j; k < 8; ++k) v[k] = v[8 + k] = v[16 + k] = kInf;
                t.aff.insert(t.aff.end(), v, v + 24);
            }
        }
        t.aabbs.insert(t.aabbs.end(), {box.lo[0], box.lo[1], box.lo[2], box.up[0], box.up[1], box.up[2]});
        t.aff_starts.push_back((uint32_t)t.n_aff());
    }

    void split(uint32_t begin, uint32_t count, uint32_t node, std::vector<uint32_t> afford, Box cell, int axis)
    {
        if (count == 1) {
            leaf(begin, afford, cell);
            return;
        }
        auto first = order.begin() + begin;
        std::sort(first, first + count, [&](uint32_t a, uint32_t b) {
            const float va = P(a)[axis], vb = P(b)[axis];
            return va < vb || (!(vb < va) && a < b);
        });
        const uint32_t half = count / 2, mid = begin + half;
        // median_partition (capt.hh:137-154): float sum halved in double
        const float test = (float)((double)(P(order[mid - 1])[axis] + P(order[mid])[axis]) / 2.0);
        t.tests[node] = test;
        const float hi_lim = test + r_max, lo_lim = test - r_max;

        std::vector<uint32_t> lo_aff, hi_aff;
        lo_aff.reserve(afford.size());
        hi_aff.reserve(afford.size());
        for (uint32_t id : afford) {  // inherited candidates (capt.hh:245-256)
            const float c = P(id)[axis];
            if (c <= hi_lim) lo_aff.push_back(id);
            if (c >= lo_lim) hi_aff.push_back(id);
        }
        afford.clear();
        afford.shrink_to_fit();
        // new candidates (capt.hh:258-280).  The reference walks the low half from its LOWEST
        // point (not from the median) while points are >= test - r_max, so the upper child
        // only inherits low-half points when the run starting at the bottom qualifies; the
        // lower child walks the high half up from the median.  Reproduced as is.
        for (uint32_t k = begin; k < mid; ++k) {
            const float c = P(order[k])[axis];
            if (!(c >= lo_lim && std::isfinite(c))) break;
            hi_aff.push_back(order[k]);
        }
        for (uint32_t k = mid; k < begin + count; ++k) {
            const float c = P(order[k])[axis];
            if (!(c <= hi_lim && std::isfinite(c))) break;
            lo_aff.push_back(order[k]);
        }
        Box lo_cell = cell, hi_cell = cell;
        lo_cell.up[axis] = test;
        hi_cell.lo[axis] = test;
        const int next = (axis + 1) % 3;
        split(begin, half, 2 * node + 1, std::move(lo_aff), lo_cell, next);
        split(mid, half, 2 * node + 2, std::move(hi_aff), hi_cell, next);
    }
};

}  // namespace

void capt_build(const float* points, size_t n, float r_min, float r_max, float r_point, CaptTree& t)
{
    const auto t0 = std::chrono::steady_clock::now();
    t = CaptTree{};
    t.r_min = r_min;
    t.r_max = r_max;
    t.r_point = r_point;
    int nlog2 = 0;
    while (((size_t)1 << nlog2) < n) ++nlog2;
    t.nlog2 = nlog2;
    const size_t m = (size_t)1 << nlog2;
    std::vector<float> pts(points, points + 3 * n);
    pts.resize(3 * m, kInf);
    t.tests.assign(m - 1, std::numeric_limits<float>::quiet_NaN());
    t.aabbs.reserve(6 * m);
    t.aff_starts.reserve(m + 1);
    t.aff_starts.push_back(0);
    const float l1 = r_max + r_point;
    Builder b{pts, std::vector<uint32_t>(m), r_max, l1 * l1, (r_min + r_point) * (r_min + r_point), t};
    std::iota(b.order.begin(), b.order.end(), 0u);
    b.split(0, (uint32_t)m, 0, {}, Box{{-kInf, -kInf, -kInf}, {kInf, kInf, kInf}}, 0);
    std::copy(b.top.lo, b.top.lo + 3, t.top);
    std::copy(b.top.up, b.top.up + 3, t.top + 3);
    t.build_ns =
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

bool capt_grid_plan(const CaptTree& t, size_t cells, CaptGridArgs& g)
{
    g = CaptGridArgs{};
    if (t.aff_starts.empty() || t.aff.empty()) return false;
    const double m = (double)t.r_max + (double)t.r_point;
    double lo[3], ext[3], vol = 1.0;
    for (int k = 0; k < 3; ++k) {
        lo[k] = (double)t.top[k] - m;
        ext[k] = (double)t.top[3 + k] + m - lo[k];
        if (!std::isfinite(lo[k]) || !std::isfinite(ext[k]) || !(ext[k] > 0.0)) return false;
        vol *= ext[k];
    }
    if (cells == 0) cells = std::min<size_t>(std::max<size_t>((size_t)128 << t.nlog2, 1u << 12), 1u << 22);
    double h = std::cbrt(vol / (double)cells);
    uint32_t n[3];
    for (;;) {  // at most 1024 cells per axis (the device's cell index error bound), ~cells in all
        bool ok = true;
        for (int k = 0; k < 3; ++k) {
            const double c = std::ceil(ext[k] / h);
            if (c > 1024.0) ok = false;
            n[k] = (uint32_t)std::max(1.0, c);
        }
        if (ok) break;
        h *= 1.25;
    }
    // cells in 4 x 4 x 4 bricks (counts rounded up to multiples of 4: the grid box grows by < 4 cells per axis;
    // cells beyond the cloud get their bounds like any other).  A wave of the grid build then walks 64 neighbouring
    // cells, which reach the same few leaves: 1.75 -> 1.06 ms for the bench cloud's grid, queries unchanged
    // (profiles/r05q_capt.log).  VGPU_CAPT_BRICK=0 keeps plain x-fastest rows.
    const char* bv = std::getenv("VGPU_CAPT_BRICK");
    g.brick = (bv && std::atoi(bv) == 0) ? 0u : 1u;
    if (g.brick)
        for (int k = 0; k < 3; ++k) n[k] = (n[k] + 3u) & ~3u;
    // the 16-bit bounds in a plane of their own, the start nodes (read only by undecided queries) in another: half
    // the cache footprint for the decided queries.  VGPU_CAPT_SPLIT=0 keeps one uint2 per cell.
    const char* sv = std::getenv("VGPU_CAPT_SPLIT");
    g.split = (sv && std::atoi(sv) == 0) ? 0u : 1u;
    g.x0 = (float)lo[0];
    g.y0 = (float)lo[1];
    g.z0 = (float)lo[2];
    g.inv_h = (float)(1.0 / h);
    g.nx = n[0];
    g.ny = n[1];
    g.nz = n[2];
    g.unit = (float)(1.0 / (double)g.inv_h / 256.0);
    g.nlog2 = t.nlog2;
    return g.unit > 0.0f && std::isfinite(g.unit);
}

}  // namespace vgpu
