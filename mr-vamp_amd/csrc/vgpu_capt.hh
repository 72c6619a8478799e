// vgpu_capt.hh -- host-side construction of CAPT point-cloud trees and heightfields for the
// device environment (collision/capt.hh:91-398, collision/shapes.hh:250-312).
//
// CAPT ("collision-affording point tree") is built on the host exactly like the reference
// (it "stays host") and uploaded as four flat arrays; the device only walks it.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace vgpu {

struct CaptTree {
    int nlog2 = 0;
    float r_min = 0, r_max = 0, r_point = 0;
    float top[6] = {0, 0, 0, 0, 0, 0};  // aabb_top: lower xyz, upper xyz (finite points only)
    std::vector<float> tests;            // 2^nlog2 - 1 split values (implicit binary tree)
    std::vector<float> aabbs;            // 2^nlog2 x 6 leaf point volumes
    std::vector<uint32_t> aff_starts;    // 2^nlog2 + 1
    std::vector<float> aff;              // n_aff x [x8 y8 z8]
    int64_t build_ns = 0;
    size_t n_aff() const { return aff.size() / 24; }
};

// CAPT::CAPT(points, r_min, r_max, r_point).  points: n x 3 floats.  Equal split coordinates
// are ordered by point index (the reference's pdqsort leaves that order unspecified).
void capt_build(const float* points, size_t n, float r_min, float r_max, float r_point, CaptTree& out);

// Cell grid of a device copy (vgpu_capt_grid.hip); offsets in floats into the environment blob.
struct CaptGridArgs {
    uint32_t tests_off, starts_off, aff_off;
    int nlog2;
    float x0, y0, z0, inv_h;
    uint32_t nx, ny, nz;
    float unit;
    uint32_t cells_off;
    uint32_t brick;  // cells in 4 x 4 x 4 bricks (vgpu_device.hh capt_cell_index; counts rounded up to 4)
    uint32_t split;      // bounds and nodes in separate planes (PC_GNODES)
    uint32_t nodes_off;  // the node plane (split), else 0
};

// Sizes the grid of tree t: the top box grown by r_max + r_point, cubic cells, about `cells`
// of them (0 = default: 128 per leaf, within [2^12, 2^22]; 8 B each: bounds + start node).  false: no grid (empty cloud).
bool capt_grid_plan(const CaptTree& t, size_t cells, CaptGridArgs& g);

struct Heightfield {
    float x, y, z, xs, ys, zs;  // offset and reciprocal scales (factory::heightfield::flat)
    size_t xd, yd;
    std::vector<float> data;    // row-major, xd * yd
};

}  // namespace vgpu
