// vcpu_rrtc.cpp -- RRT-Connect on the CPU rake (BASELINE configs[0]: the reference's planner, CPU
// only, its per-edge checks being this build's validate_vector).
//
// Restates vamp::planning::RRTC<Robot, 8, Robot::resolution>::solve (planning/rrtc.hh:16-249) with
// RRTCSettings (rrtc_settings.hh:5-20) and rng::Halton<dim> (random/halton.hh:73-104):
//   * balanced, dynamic-domain bidirectional RRT: sample -> scale_configuration -> nearest in
//     tree A -> extend by at most `range` (validate_vector with the NN distance or the range as
//     its distance) -> connect greedily to tree B in ceil(d / range) equal increments;
//   * nearest neighbours: exact linear scan with Space<dim>::distance = FloatVector::l2_norm of the
//     difference in the reference's lane order (nn.hh:53-57).  The reference's nigh KD-tree is
//     exact as well; only its order among equal distances is unknown (parity unpinned on ties,
//     which continuous samples do not produce);
//   * float ops as the source states them: extension = v * (range / d), increment = v * (1 / n),
//     new = nearest + extension (the release build may contract a multiply into the following
//     add across these statements; rrtc.hh cannot be compiled here -- nigh is absent -- so that is
//     unpinned);
//   * PlanningResult: path, cost (sum of l2 segment lengths in the reference's accumulation
//     order), iterations, tree sizes, nanoseconds of steady_clock around the search.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <limits>
#include <vector>

#include "vcpu_robot.hh"
#include "../vgpu_abi.hh"

namespace vcpu {
namespace {

// rng::Halton<dim>::next for draw k (1-based) of a fresh sampler: closed form of the reference's
// incremental radical inverse, its numerators reset and bases rotated every 1,000,000 draws (the
// reset makes later cycles 1,000,001 long); n / d are exact float integers (vgpu_device.hh).
constexpr uint32_t kPrimes[16] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59};

float radical_inverse(uint32_t idx, uint32_t b)
{
    uint32_t num = 0, den = 1;
    while (idx) {
        num = num * b + idx % b;
        den *= b;
        idx /= b;
    }
    return (float)num / (float)den;
}

void halton_draw(int dim, uint64_t k, float* out)
{
    uint32_t idx, cycle;
    if (k <= 1000000u) {
        idx = (uint32_t)k;
        cycle = 0;
    } else {
        const uint64_t kk = k - 1000000u - 1;
        cycle = (uint32_t)(1 + kk / 1000001u);
        idx = (uint32_t)(kk % 1000001u) + 1u;
    }
    for (int d = 0; d < dim; ++d) out[d] = radical_inverse(idx, kPrimes[(d + cycle) % (uint32_t)dim]);
}

struct Tree {
    std::vector<uint32_t> nodes;  // indices into the configuration buffer, insertion order
};

}  // namespace
}  // namespace vcpu

using namespace vcpu;

extern "C" int vgpu_cpu_rrtc(const vgpu_robot* robot, vgpu_env* env, const float* start, const float* goals,
                             size_t n_goals, const vgpu_rrtc_settings* settings, uint64_t* rng_index, float* path,
                             size_t path_cap, vgpu_plan_result* result)
try {
    Bound b;
    Env e;
    if (!start || (n_goals && !goals) || !settings || !rng_index || !result || (path_cap && !path))
        return VGPU_ERR_INVALID_ARG;
    if (*rng_index == 0 || n_goals == 0) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (int rc = view(env, e)) return rc;
    if (e.attached && !b.R->fkcc_attach) return VGPU_ERR_UNSUPPORTED;
    const RobotCpu& R = *b.R;
    const int D = R.dim;
    const vgpu_rrtc_settings& S = *settings;
    constexpr float kMax = std::numeric_limits<float>::max();

    std::vector<float> buf;  // configurations, D floats each (rrtc.hh:48-53)
    std::vector<size_t> parents;
    std::vector<float> radii;
    auto config = [&](size_t i) -> float* { return buf.data() + i * (size_t)D; };
    auto push = [&](const float* q, size_t parent) -> size_t {
        const size_t i = parents.size();
        buf.insert(buf.end(), q, q + D);
        parents.push_back(parent == SIZE_MAX ? i : parent);
        radii.push_back(kMax);
        return i;
    };
    std::vector<float> out_path;
    float cost = 0.0f;
    uint64_t iter = 0;
    Tree start_tree, goal_tree;

    const auto t0 = std::chrono::steady_clock::now();
    auto elapsed = [&] {
        return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
            .count();
    };
    *result = vgpu_plan_result{};

    for (size_t gi = 0; gi < n_goals; ++gi) {  // rrtc.hh:61-73: a direct connection needs no search
        if (validate_one(b, e, start, goals + gi * (size_t)D, nullptr, nullptr)) {
            out_path.assign(start, start + D);
            out_path.insert(out_path.end(), goals + gi * (size_t)D, goals + (gi + 1) * (size_t)D);
            result->nanoseconds = elapsed();
            result->solved = 1;
            result->iterations = 0;
            result->size[0] = result->size[1] = 1;
            result->cost = 0.0f;
            result->path_len = 2;
            if (path_cap < 2) return VGPU_ERR_INVALID_ARG;
            std::copy(out_path.begin(), out_path.end(), path);
            return VGPU_OK;
        }
    }

    bool tree_a_is_start = !S.start_tree_first;  // rrtc.hh:76-78
    Tree* tree_a = S.start_tree_first ? &goal_tree : &start_tree;
    Tree* tree_b = S.start_tree_first ? &start_tree : &goal_tree;
    start_tree.nodes.push_back((uint32_t)push(start, SIZE_MAX));
    for (size_t gi = 0; gi < n_goals; ++gi) goal_tree.nodes.push_back((uint32_t)push(goals + gi * (size_t)D, SIZE_MAX));

    auto nearest = [&](const Tree& t, const float* q, float& dist) -> size_t {
        float diff[kMaxDim];
        size_t best = SIZE_MAX;
        dist = kMax;
        for (uint32_t i : t.nodes) {
            const float* c = config(i);
            for (int j = 0; j < D; ++j) diff[j] = q[j] - c[j];
            const float d = l2_norm(diff, D);
            if (best == SIZE_MAX || d < dist) {
                best = i;
                dist = d;
            }
        }
        return best;
    };

    float temp[kMaxDim], ext[kMaxDim], nc[kMaxDim], newc[kMaxDim], onv[kMaxDim], inc[kMaxDim], prior[kMaxDim],
        next[kMaxDim];
    while (iter++ < S.max_iterations && parents.size() < S.max_samples) {  // rrtc.hh:95
        const float asize = (float)tree_a->nodes.size(), bsize = (float)tree_b->nodes.size();
        const float ratio = std::abs(asize - bsize) / asize;
        if (!S.balance || ratio < S.tree_ratio) {  // rrtc.hh:101-105
            std::swap(tree_a, tree_b);
            tree_a_is_start = !tree_a_is_start;
        }
        halton_draw(D, (*rng_index)++, temp);  // rng->next(); Robot::scale_configuration (fma)
        for (int j = 0; j < D; ++j) temp[j] = std::fma(temp[j], R.s_m[j], R.s_a[j]);

        float nd;
        const size_t nn = nearest(*tree_a, temp, nd);
        const float nr = radii[nn];
        if (S.dynamic_domain && nr < nd) continue;  // rrtc.hh:125-128
        std::copy(config(nn), config(nn) + D, nc);
        const bool reach = nd < S.range;
        const float sc = S.range / nd;
        for (int j = 0; j < D; ++j) {
            const float v = temp[j] - nc[j];
            ext[j] = reach ? v : v * sc;  // rrtc.hh:132-136
        }
        if (validate_vector_one(b, e, nc, ext, reach ? nd : S.range, nullptr, nullptr)) {
            for (int j = 0; j < D; ++j) newc[j] = nc[j] + ext[j];
            const size_t ni = push(newc, nn);
            tree_a->nodes.push_back((uint32_t)ni);
            if (S.dynamic_domain && nr != kMax) radii[nn] *= (1 + S.alpha);  // rrtc.hh:156-159

            float od;  // extend to the other tree (rrtc.hh:161-191)
            const size_t on = nearest(*tree_b, newc, od);
            for (int j = 0; j < D; ++j) onv[j] = config(on)[j] - newc[j];
            const size_t n_ext = (size_t)std::ceil(od / S.range);
            const float inc_len = od / (float)n_ext;
            const float inv = 1.0F / (float)n_ext;
            for (int j = 0; j < D; ++j) inc[j] = onv[j] * inv;
            std::copy(newc, newc + D, prior);
            size_t i_ext = 0;
            for (; i_ext < n_ext && validate_vector_one(b, e, prior, inc, inc_len, nullptr, nullptr) &&
                   parents.size() < S.max_samples;
                 ++i_ext) {
                for (int j = 0; j < D; ++j) next[j] = prior[j] + inc[j];
                const size_t xi = push(next, parents.size() - 1);
                tree_a->nodes.push_back((uint32_t)xi);
                std::copy(next, next + D, prior);
            }
            if (i_ext == n_ext) {  // connected: both half-paths (rrtc.hh:193-226)
                auto dist_last_two = [&] {
                    float d[kMaxDim];
                    const size_t m = out_path.size() / D;
                    for (int j = 0; j < D; ++j) d[j] = out_path[(m - 1) * D + j] - out_path[(m - 2) * D + j];
                    return l2_norm(d, D);
                };
                size_t cur = parents.size() - 1;
                out_path.insert(out_path.end(), config(cur), config(cur) + D);
                while (parents[cur] != cur) {
                    const size_t p = parents[cur];
                    out_path.insert(out_path.end(), config(p), config(p) + D);
                    cost += dist_last_two();
                    cur = p;
                }
                const size_t half = out_path.size() / D;
                for (size_t i = 0; i < half / 2; ++i)
                    std::swap_ranges(out_path.begin() + i * D, out_path.begin() + (i + 1) * D,
                                     out_path.begin() + (half - 1 - i) * D);
                cur = on;
                while (parents[cur] != cur) {
                    const size_t p = parents[cur];
                    out_path.insert(out_path.end(), config(p), config(p) + D);
                    cost += dist_last_two();
                    cur = p;
                }
                if (!tree_a_is_start) {
                    const size_t m = out_path.size() / D;
                    for (size_t i = 0; i < m / 2; ++i)
                        std::swap_ranges(out_path.begin() + i * D, out_path.begin() + (i + 1) * D,
                                         out_path.begin() + (m - 1 - i) * D);
                }
                break;
            }
        } else if (S.dynamic_domain) {  // rrtc.hh:229-239
            if (nr == kMax)
                radii[nn] = S.radius;
            else
                radii[nn] = std::max(radii[nn] * (1.F - S.alpha), S.min_radius);
        }
    }
    result->nanoseconds = elapsed();
    result->iterations = iter;
    result->size[0] = start_tree.nodes.size();
    result->size[1] = goal_tree.nodes.size();
    result->cost = cost;
    result->path_len = out_path.size() / D;
    result->solved = out_path.empty() ? 0 : 1;
    if (result->path_len > path_cap) return VGPU_ERR_INVALID_ARG;
    std::copy(out_path.begin(), out_path.end(), path);
    return VGPU_OK;
} VGPU_ABI_CATCH
