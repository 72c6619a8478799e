// vgpu_api.cpp -- host runtime behind include/vamp_gpu.h.
//
// Owns: HIP device/stream selection, the host-rsqrt table probe + upload, the
// collision::Environment<float> builder (shape constructors of collision/shapes.hh and
// collision/factory.hh, the add_* routing of bindings/environment.cc:107-146 and the
// min_distance sort of collision/environment.hh:40-66), device-resident obstacle
// tables, argument validation and error reporting.  Kernels live in vgpu_kernels.hip.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vamp_gpu.h"
#include "vgpu_abi.hh"
#include "vgpu_capt.hh"
#include "vgpu_device.hh"
#include "vgpu_host_env.hh"
#include "vgpu_ops.hh"
#include "gen/radii.inc"

extern "C" {
hipError_t vgpu_launch_panda_sample(uint64_t first, size_t n, float* q, hipStream_t st);
hipError_t vgpu_launch_panda_sample_fkcc(uint64_t first, size_t n, const EnvView* env, float bx, float by, float bz,
                                         float* q, uint8_t* valid, hipStream_t st);
hipError_t vgpu_launch_halton(int dim, uint64_t first, size_t n, float* out, hipStream_t st);
hipError_t vgpu_filter_pointcloud_run(const float* d_pc, size_t n, float min_dist, float max_range,
                                      const float origin[3], const float ws_min[3], const float ws_max[3], int cull,
                                      uint32_t* d_out, size_t* count, hipStream_t s);
size_t vgpu_compact_bytes(size_t n);
hipError_t vgpu_launch_compact(const uint8_t* valid, size_t n, uint32_t* idx_out, uint32_t* count, void* tmp,
                               size_t tmp_bytes, hipStream_t st);
hipError_t vgpu_launch_gather_rows(const float* q, const uint32_t* idx, const uint32_t* count, size_t max_rows,
                                   int dim, float* out, hipStream_t st);
hipError_t vgpu_launch_scatter_items(const uint32_t* cnt, const uint32_t* off, size_t n_edges, uint32_t* item_edge,
                                     hipStream_t st);
hipError_t vgpu_launch_filter_robot(const float* pc, size_t n, float point_radius, const float* sph, int S,
                                   const EnvView* env, uint8_t* keep, hipStream_t st);
hipError_t vgpu_launch_total64(const uint32_t* cnt, size_t n, unsigned long long* out, hipStream_t st);
#define VGPU_STAGED_DECL(NAME)                                                                                       \
    int vgpu_##NAME##_staged_checks(void);                                                                           \
    uint64_t vgpu_##NAME##_staged_env_checks(void);                                                                  \
    int vgpu_##NAME##_staged_mask_bytes(void);                                                                       \
    int vgpu_##NAME##_staged_class(int c, int ext);                                                                  \
    size_t vgpu_##NAME##_staged_plan_bytes(void);                                                                    \
    uint32_t vgpu_##NAME##_staged_blocks(int kind, uint32_t n_groups);                                               \
    hipError_t vgpu_##NAME##_staged_bound(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          uint64_t first, uint32_t n_groups, const EnvView* env, const float* bases, \
                                          int chain, void* mask, uint8_t* valid, hipStream_t st);                    \
    hipError_t vgpu_##NAME##_staged_count(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          const void* mask, uint32_t n_groups, uint64_t set, const uint8_t* valid,   \
                                          uint32_t* counts, hipStream_t st);                                         \
    hipError_t vgpu_##NAME##_staged_plan(const uint32_t* offs, uint32_t nb, uint32_t W, uint64_t set,                \
                                         uint32_t n_groups, void* plan, int ext, hipStream_t st);                    \
    hipError_t vgpu_##NAME##_staged_queue(int kind, const void* s0, const void* s1, const void* s2, const void* s3,  \
                                          const void* mask, uint32_t n_groups, uint64_t set, const void* plan,       \
                                          const uint8_t* valid, const uint32_t* offs, uint32_t* items,               \
                                          const void* dbg, hipStream_t st);                                          \
    hipError_t vgpu_##NAME##_staged_children(int kind, const void* s0, const void* s1, const void* s2,               \
                                             const void* s3, uint64_t first, const void* plan, const uint32_t* ub,   \
                                             const uint32_t* items, const EnvView* env, const float* bases,          \
                                             uint8_t* valid, hipStream_t st);                                         \
    int vgpu_##NAME##_staged_lead_check(void);                                                                       \
    hipError_t vgpu_##NAME##_staged_lead(int kind, const void* s0, const void* s1, const void* s2, const void* s3,   \
                                         uint64_t first, uint32_t n_groups, const EnvView* env, const float* bases,  \
                                         uint8_t* valid, hipStream_t st);                                            \
    int vgpu_##NAME##_staged_head_list(void);
VGPU_STAGED_DECL(panda_p0)
VGPU_STAGED_DECL(panda_p1)
VGPU_STAGED_DECL(panda_p2)
VGPU_STAGED_DECL(panda_p3)
VGPU_STAGED_DECL(fetch_p0)
VGPU_STAGED_DECL(fetch_p1)
VGPU_STAGED_DECL(fetch_p2)
VGPU_STAGED_DECL(fetch_p3)
VGPU_STAGED_DECL(ur5)
VGPU_STAGED_DECL(pair_a)
VGPU_STAGED_DECL(pair_b)
VGPU_STAGED_DECL(pair_i0)
VGPU_STAGED_DECL(pair_i1)
VGPU_STAGED_DECL(baxter_c0)
VGPU_STAGED_DECL(baxter_c1)
VGPU_STAGED_DECL(baxter_c2)
VGPU_STAGED_DECL(baxter_c3)
VGPU_STAGED_DECL(baxter_c4)
VGPU_STAGED_DECL(baxter_c5)
VGPU_STAGED_DECL(baxter_c6)
hipError_t vgpu_launch_pair_tail_counts(const float* starts, const float* goals, size_t n_edges, const uint8_t* ok,
                                        int32_t* n_blocks, uint32_t* cnt, hipStream_t st);
const RobotOps* vgpu_ur5_ops(void);
const RobotOps* vgpu_baxter_ops(void);
hipError_t vgpu_launch_fetch_tail_counts(const float* starts, const float* goals, size_t n_edges, const uint8_t* ok,
                                         int32_t* n_blocks, uint32_t* cnt, hipStream_t st);
hipError_t vgpu_launch_mask_finish(size_t n_edges, const uint32_t* off, uint8_t* ok, uint8_t* block_ok, hipStream_t st);
hipError_t vgpu_launch_tail_counts(const float* starts, const float* goals, size_t n_edges, const uint8_t* ok,
                                   int32_t* n_blocks, uint32_t* cnt, hipStream_t st);
hipError_t vgpu_launch_capt_grid(float* base, const vgpu::CaptGridArgs* g, hipStream_t st);
hipError_t vgpu_launch_capt_query(const float* centers, const float* radii, size_t n, const EnvView* env, int index,
                                  int simd, uint8_t* out, hipStream_t st);
hipError_t vgpu_launch_panda_sphere_fk(const float* q, size_t n, float bx, float by, float bz, float* out,
                                       size_t ld, hipStream_t st);
hipError_t vgpu_launch_panda_fkcc(const float* q, size_t n, const EnvView* env, float bx, float by, float bz,
                                  uint8_t* valid, hipStream_t st);
hipError_t vgpu_launch_fetch_sphere_fk(const float* q, size_t n, float* out, size_t ld, hipStream_t st);
hipError_t vgpu_launch_fetch_fkcc(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st);
hipError_t vgpu_launch_fetch_sample(uint64_t first, size_t n, float* q, hipStream_t st);
hipError_t vgpu_launch_fetch_sample_fkcc(uint64_t first, size_t n, const EnvView* env, float* q, uint8_t* valid,
                                         hipStream_t st);
hipError_t vgpu_launch_fetch_validate_head(const float* starts, const float* goals, size_t n_edges,
                                           const EnvView* env, uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                           hipStream_t st);
hipError_t vgpu_launch_fetch_validate_tail(const float* starts, const float* goals, size_t n_items,
                                           const EnvView* env, uint8_t* ok, const uint32_t* off,
                                           const uint32_t* item_edge, hipStream_t st);
hipError_t vgpu_launch_pair_fkcc(const float* q, size_t n, const EnvView* env, const float base[6], uint8_t* valid,
                                 hipStream_t st);
hipError_t vgpu_launch_pair_validate_head(const float* starts, const float* goals, size_t n_edges, const EnvView* env,
                                          const float base[6], uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                          hipStream_t st);
hipError_t vgpu_launch_pair_validate_tail(const float* starts, const float* goals, size_t n_items, const EnvView* env,
                                          const float base[6], uint8_t* ok, const uint32_t* off,
                                          const uint32_t* item_edge, hipStream_t st);
size_t vgpu_validate_scan_bytes(size_t n_edges);
hipError_t vgpu_launch_scan(const uint32_t* cnt, uint32_t* off, size_t n_edges, void* scan_tmp, size_t scan_bytes,
                            hipStream_t st);
hipError_t vgpu_launch_panda_fkcc_attach(const float* q, size_t n, const EnvView* env, float bx, float by, float bz,
                                         uint8_t* valid, hipStream_t st);
hipError_t vgpu_launch_panda_validate_head_att(const float* starts, const float* goals, size_t n_edges,
                                               const EnvView* env, float bx, float by, float bz, uint8_t* ok,
                                               int32_t* n_blocks, uint32_t* cnt, hipStream_t st);
hipError_t vgpu_launch_fetch_fkcc_attach(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st);
hipError_t vgpu_launch_fetch_validate_head_att(const float* starts, const float* goals, size_t n_edges,
                                               const EnvView* env, uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                               hipStream_t st);
hipError_t vgpu_launch_ur5_fkcc_attach(const float* q, size_t n, const EnvView* env, uint8_t* valid, hipStream_t st);
hipError_t vgpu_launch_ur5_validate_head_att(const float* starts, const float* goals, size_t n_edges,
                                             const EnvView* env, uint8_t* ok, int32_t* n_blocks, uint32_t* cnt,
                                             hipStream_t st);
hipError_t vgpu_launch_panda_validate_head(const float* starts, const float* goals, size_t n_edges,
                                           const EnvView* env, float bx, float by, float bz, uint8_t* ok,
                                           int32_t* n_blocks, uint32_t* cnt, hipStream_t st);
hipError_t vgpu_launch_panda_validate_tail(const float* starts, const float* goals, size_t n_edges,
                                           size_t n_items, const EnvView* env, float bx, float by, float bz,
                                           uint8_t* ok, const uint32_t* cnt, const uint32_t* off,
                                           uint32_t* item_edge, hipStream_t st);
}

namespace {

constexpr int kPandaDim = 7;
constexpr int kPandaResolution = 32;  // robots/panda_base.hh:21
constexpr int kPandaSpheres = 59;     // robots/panda/fk.hh:93
constexpr int kFetchDim = 8;          // robots/fetch.hh:12
constexpr int kFetchResolution = 32;  // robots/fetch.hh:13
constexpr int kFetchSpheres = 111;    // robots/fetch/fk.hh:104
constexpr int kPairDim = 14;          // two Panda arms (BASELINE configs[4])

inline uint32_t f2u(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}
inline float u2f(uint32_t u)
{
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// Probe the host's _mm256_rsqrt_ps as a table over (exponent parity, top K mantissa bits)
// for inputs with biased exponent 126 + parity, plus the exact exponent-shift rule for all
// other exponents.  K is the smallest width that reproduces every input of the two
// reference binades (8..23; 23 = the full 2 x 2^23 table).
__attribute__((target("avx2"))) int probe_host_rsqrt(std::vector<uint32_t>& lut, int& kbits, std::string& err)
{
    std::vector<uint32_t> full((size_t)2 << 23);
    for (uint32_t p = 0; p < 2; ++p) {
        for (uint32_t m = 0; m < (1u << 23); m += 8) {
            alignas(32) float in[8], out[8];
            for (int l = 0; l < 8; ++l) in[l] = u2f(((126u + p) << 23) | (m + (uint32_t)l));
            _mm256_store_ps(out, _mm256_rsqrt_ps(_mm256_load_ps(in)));
            for (int l = 0; l < 8; ++l) full[((size_t)p << 23) | (m + (uint32_t)l)] = f2u(out[l]);
        }
    }
    int K = -1;
    for (int k = 8; k <= 23 && K < 0; ++k) {
        bool ok = true;
        const uint32_t lowmask = (1u << (23 - k)) - 1u;
        for (size_t i = 0; i < ((size_t)2 << 23) && ok; ++i) {
            const size_t rep = i & ~(size_t)lowmask;
            ok = full[i] == full[rep];
        }
        if (ok) K = k;
    }
    if (K < 0) {
        err = "host rsqrt is not a function of (parity, mantissa)";
        return VGPU_ERR_RSQRT;
    }
    lut.assign((size_t)2 << K, 0u);
    for (uint32_t p = 0; p < 2; ++p)
        for (uint32_t j = 0; j < (1u << K); ++j) lut[((size_t)p << K) | j] = full[((size_t)p << 23) | ((size_t)j << (23 - K))];
    // exponent-shift rule over every normal exponent (sampled)
    uint64_t s = 0x243F6A8885A308D3ull;
    for (int e = 1; e < 255; ++e) {
        for (int t = 0; t < 2048; ++t) {
            s ^= s << 13;
            s ^= s >> 7;
            s ^= s << 17;
            const float x = u2f(((uint32_t)e << 23) | (uint32_t)(s & 0x7FFFFF));
            const float want = _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x)));
            const uint32_t p = (uint32_t)e & 1u;
            const int shift = (e - (int)(126 + p)) / 2;
            const uint32_t tb = lut[((size_t)p << K) | ((f2u(x) & 0x7FFFFFu) >> (23 - K))];
            const int re = (int)((tb >> 23) & 0xFF) - shift;
            if (re <= 0 || re >= 255) continue;
            if (u2f(tb - ((uint32_t)shift << 23)) != want) {
                err = "host rsqrt exponent scaling is not exact";
                return VGPU_ERR_RSQRT;
            }
        }
    }
    kbits = K;
    return VGPU_OK;
}

}  // namespace

struct vgpu_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t cur = nullptr;
    std::string err;
    std::vector<uint32_t> lut;
    int kbits = 0;
    uint32_t* lut_dev = nullptr;
    // staging for the *_host conveniences
    void* stage = nullptr;
    size_t stage_bytes = 0;
    // validate workspace: cnt/off (n_edges + 1 each), scan temp, work items, pinned total
    void* ws = nullptr;
    size_t ws_bytes = 0;
    uint32_t* items = nullptr;
    size_t items_cap = 0;
    uint32_t* total_host = nullptr;  // pinned, 4 words: [0] the 32-bit scan total, [2..3] its 64-bit sum
    // compaction workspace (selected indices' count word + hipcub temp)
    void* aux = nullptr;
    size_t aux_bytes = 0;
    // staged checks (vgpu_staged.hip): bounding masks, per-check counts/cursors, item list
    bool staged = true;
    bool stats = false;  // print each staged pass's per-check bounding counts (VAMP_AMD_STAGED_STATS)
    std::vector<uint64_t> rounds;  // check sets run in order (staged); empty = chosen per batch
    long one_round = -1;           // A/B: source kinds run as one round (VAMP_AMD_ONE_ROUND), -1 = the robot's
    long lead = -1;                // A/B: source kinds that run the lead pass (VAMP_AMD_LEAD), -1 = the robot's
    bool head_list = true;         // A/B: validate heads after the lead pass over its compacted list (VAMP_AMD_HEAD_LIST)
    bool no_near = false;          // A/B: children scan every culled record, no near sets (VAMP_AMD_NEAR=0)
    uint32_t* st_list = nullptr;   // that list (edges still valid, ascending), its count word, the selection's temp
    size_t st_list_cap = 0;
    uint32_t* st_mask = nullptr;
    size_t st_mask_cap = 0;
    uint32_t* st_q = nullptr;  // staged sampling without a caller buffer: the drawn configurations
    size_t st_q_cap = 0;
    uint32_t* st_cnt = nullptr;   // per-(check, block) counts, then their exclusive scan, + scan temp
    size_t st_cnt_cap = 0;
    uint32_t* st_host = nullptr;  // pinned: the first round's segment boundaries of a staged pass
    uint32_t* st_items = nullptr;
    size_t st_items_cap = 0;
    // roadmap kNN chunk lists (vgpu_roadmap.hip)
    uint32_t* knn_part = nullptr;
    size_t knn_part_cap = 0;
    // roadmap kNN spatial index (vgpu_knn_index.hip): 0 auto (index from kKnnIndexMin vertices),
    // 1 brute force, 2 index; its scratch pool
    int knn_mode = 0;
    uint32_t* knn_idx = nullptr;
    size_t knn_idx_cap = 0;
    // filter_robot_from_pointcloud: the configuration, its sphere_fk<1> centres and the radii
    float* small = nullptr;
    // debug-check words of the kernels without an environment (kNN index): VGPU_DCHECK, make DEBUG=1
    uint32_t* dbg = nullptr;
    // optional phase timing
    bool prof = false;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    float acc[4] = {0, 0, 0, 0};
};

struct vgpu_env {
    vgpu_ctx* ctx = nullptr;
    std::vector<std::array<float, 5>> spheres;
    std::vector<std::array<float, 9>> capsules, zcapsules;
    std::vector<std::array<float, 16>> cuboids, zcuboids;
    std::vector<vgpu::Heightfield> heightfields;
    std::vector<vgpu::CaptTree> pointclouds;
    bool attached = false;  // Environment::attachments (environment.hh:21)
    std::array<float, 7> att_tf{};
    std::vector<std::array<float, 4>> att_spheres;
    struct Layout {  // section offsets (floats) of one copy of the blob
        size_t off[OBS_TYPES] = {0, 0, 0, 0, 0};
        int cnt[OBS_TYPES] = {0, 0, 0, 0, 0};
        size_t hf_off = 0, pc_off = 0, att_off = 0;
    };
    Layout dev_lay, host_lay;  // the device copy carries cell grids the host copy has not: offsets differ
    std::vector<vgpu::CaptGridArgs> pc_grid;  // device copy: each cloud's cell grid (cells_off 0 = none)
    bool dirty = true;       // device copy stale (obstacles, heightfields, attachment: the blob's tail)
    bool pc_dirty = true;    // device copy's point clouds stale (the blob's prefix: trees + cell grids)
    bool host_dirty = true;  // host copy (the CPU rake's view, csrc/cpu/) stale
    size_t tail_off = 0;     // first float of the tail section (device copy)
    uint64_t n_full = 0, n_tail = 0, n_grids = 0;  // device uploads: whole blob, tail only; grid builds
    std::vector<float> host_blob;
    std::mutex host_mu;
    float* dev = nullptr;
    size_t dev_floats = 0;
};

// A context's device made current for this thread, and the thread's last HIP error cleared: a HANDLED failure of an
// earlier call (e.g. vgpu_ctx_create on a device that does not exist) must not be read back by this call's first
// hipGetLastError() after a kernel launch and reported as this call's failure
#define ctx_device(c) (hipSetDevice((c)->device) == hipSuccess ? ((void)hipGetLastError(), hipSuccess) \
                                                                 : hipSetDevice((c)->device))
#define HIPCHK(ctx, expr)                                                                          \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                        \
            return VGPU_ERR_HIP;                                                                   \
        }                                                                                          \
    } while (0)

static int fail(vgpu_ctx* ctx, int code, const char* msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

// ---------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------
extern "C" int vgpu_ctx_create(int device, vgpu_ctx** out)
try {
    if (!out) return VGPU_ERR_INVALID_ARG;
    *out = nullptr;
    auto* c = new (std::nothrow) vgpu_ctx();
    if (!c) return VGPU_ERR_OOM;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        delete c;
        return VGPU_ERR_HIP;
    }
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();  // handled here: not a later call's failure
        delete c;
        return VGPU_ERR_HIP;
    }
    c->cur = c->own;
    if (const char* s = std::getenv("VAMP_AMD_STAGED")) c->staged = std::strcmp(s, "0") != 0;
    if (const char* s = std::getenv("VAMP_AMD_KNN")) c->knn_mode = std::atoi(s);
    if (const char* s = std::getenv("VAMP_AMD_STAGED_STATS")) c->stats = std::strcmp(s, "0") != 0;
    if (const char* s = std::getenv("VAMP_AMD_ONE_ROUND")) c->one_round = std::strtol(s, nullptr, 0);
    if (const char* s = std::getenv("VAMP_AMD_LEAD")) c->lead = std::strtol(s, nullptr, 0);
    if (const char* s = std::getenv("VAMP_AMD_HEAD_LIST")) c->head_list = std::strcmp(s, "0") != 0;
    if (const char* s = std::getenv("VAMP_AMD_NEAR")) c->no_near = std::strcmp(s, "0") == 0;
    if (const char* s = std::getenv("VAMP_AMD_ROUNDS")) {  // A/B: comma-separated check bit masks
        for (const char* p = s; *p;) {
            char* end = nullptr;
            const unsigned long long v = std::strtoull(p, &end, 0);
            if (end == p) break;
            c->rounds.push_back((uint64_t)v);
            p = (*end == ',') ? end + 1 : end;
        }
    }
    int rc = probe_host_rsqrt(c->lut, c->kbits, c->err);
    if (rc != VGPU_OK) {
        (void)hipStreamDestroy(c->own);
        delete c;
        return rc;
    }
    if (hipMalloc(&c->lut_dev, c->lut.size() * 4) != hipSuccess ||
        hipMemcpy(c->lut_dev, c->lut.data(), c->lut.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc((void**)&c->dbg, 16) != hipSuccess || hipMemset(c->dbg, 0, 16) != hipSuccess) {
        if (c->lut_dev) (void)hipFree(c->lut_dev);
        (void)hipStreamDestroy(c->own);
        delete c;
        return VGPU_ERR_HIP;
    }
    *out = c;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_debug_build(void)
try {
#ifdef VGPU_DEBUG
    return 1;
#else
    return 0;
#endif
} VGPU_ABI_CATCH

// The debug-check words (VGPU_DCHECK, debug builds): the context's (kNN index) and, when env is given, the
// environment copy's (staged and CAPT kernels).  out[0] = violations, out[1] = first site id; read and reset.
extern "C" int vgpu_debug_violations(vgpu_ctx* c, vgpu_env* e, uint32_t out[2])
try {
    if (!c || !out) return VGPU_ERR_INVALID_ARG;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    uint32_t a[2] = {0, 0}, b[2] = {0, 0};
    HIPCHK(c, hipMemcpy(a, c->dbg, 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemset(c->dbg, 0, 8));
    if (e && e->ctx == c && e->dev) {
        HIPCHK(c, hipMemcpy(b, e->dev, 8, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemset(e->dev, 0, 8));
    }
    out[0] = a[0] + b[0];
    out[1] = a[1] ? a[1] : b[1];
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" void vgpu_ctx_destroy(vgpu_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->own) (void)hipStreamSynchronize(c->own);
    if (c->lut_dev) (void)hipFree(c->lut_dev);
    if (c->stage) (void)hipFree(c->stage);
    if (c->ws) (void)hipFree(c->ws);
    if (c->items) (void)hipFree(c->items);
    if (c->aux) (void)hipFree(c->aux);
    if (c->st_mask) (void)hipFree(c->st_mask);
    if (c->st_q) (void)hipFree(c->st_q);
    if (c->st_cnt) (void)hipFree(c->st_cnt);
    if (c->st_items) (void)hipFree(c->st_items);
    if (c->st_list) (void)hipFree(c->st_list);
    if (c->st_host) (void)hipHostFree(c->st_host);
    if (c->knn_part) (void)hipFree(c->knn_part);
    if (c->knn_idx) (void)hipFree(c->knn_idx);
    if (c->small) (void)hipFree(c->small);
    if (c->dbg) (void)hipFree(c->dbg);
    if (c->total_host) (void)hipHostFree(c->total_host);
    for (auto& ev : c->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

extern "C" const char* vgpu_last_error(const vgpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" int vgpu_ctx_set_stream(vgpu_ctx* c, void* s)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    c->cur = s ? (hipStream_t)s : c->own;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_ctx_device(const vgpu_ctx* c, int* device)
try {
    if (!c || !device) return VGPU_ERR_INVALID_ARG;
    *device = c->device;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_sync(vgpu_ctx* c)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_ctx_set_profiling(vgpu_ctx* c, int enable)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    HIPCHK(c, ctx_device(c));
    for (auto& ev : c->ev)
        if (!ev) HIPCHK(c, hipEventCreate(&ev));
    c->prof = enable != 0;
    for (float& a : c->acc) a = 0.0f;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_phase_times(vgpu_ctx* c, float ms[4])
try {
    if (!c || !ms) return VGPU_ERR_INVALID_ARG;
    for (int i = 0; i < 4; ++i) {
        ms[i] = c->acc[i];
        c->acc[i] = 0.0f;
    }
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_rsqrt_table(const vgpu_ctx* c, int* kbits, const uint32_t** table)
try {
    if (!c || !kbits || !table) return VGPU_ERR_INVALID_ARG;
    *kbits = c->kbits;
    *table = c->lut.data();
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_rsqrt_table_set(vgpu_ctx* c, const uint32_t* table, int kbits)
try {
    if (!c || !table || kbits < 1 || kbits > 23) return fail(c, VGPU_ERR_INVALID_ARG, "bad rsqrt table");
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    c->lut.assign(table, table + ((size_t)2 << kbits));
    if (c->lut_dev) (void)hipFree(c->lut_dev);
    c->lut_dev = nullptr;
    HIPCHK(c, hipMalloc(&c->lut_dev, c->lut.size() * 4));
    HIPCHK(c, hipMemcpy(c->lut_dev, c->lut.data(), c->lut.size() * 4, hipMemcpyHostToDevice));
    c->kbits = kbits;
    return VGPU_OK;
} VGPU_ABI_CATCH

// ---------------------------------------------------------------------------------------
// environment: shapes.hh / factory.hh restated on the host (float, no contraction)
// ---------------------------------------------------------------------------------------
static float clampf(float v, float lo, float hi) { return std::max(std::min(v, hi), lo); }  // math.hh:50-53

static float sphere_min_distance(float x, float y, float z, float r)  // shapes.hh:238
{
    return std::sqrt(x * x + y * y + z * z) - r;
}

static float cuboid_min_distance(const float* c)  // shapes.hh:52-67
{
    const float x = c[0], y = c[1], z = c[2];
    const float *a1 = c + 3, *a2 = c + 6, *a3 = c + 9;
    const float d1 = -x * a1[0] + -y * a1[1] + -z * a1[2];
    const float d2 = -x * a2[0] + -y * a2[1] + -z * a2[2];
    const float d3 = -x * a3[0] + -y * a3[1] + -z * a3[2];
    const float v1 = clampf(d1, -c[12], c[12]);
    const float v2 = clampf(d2, -c[13], c[13]);
    const float v3 = clampf(d3, -c[14], c[14]);
    const float xn = x + a1[0] * v1 + a2[0] * v2 + a3[0] * v3;
    const float yn = y + a1[1] * v1 + a2[1] * v2 + a3[1] * v3;
    const float zn = z + a1[2] * v1 + a2[2] * v2 + a3[2] * v3;
    return std::sqrt(xn * xn + yn * yn + zn * zn);
}

static float capsule_min_distance(const float* c)  // shapes.hh:165-189
{
    const float x1 = c[0], y1 = c[1], z1 = c[2], xv = c[3], yv = c[4], zv = c[5], r = c[6], rdv = c[7];
    const float dot = clampf((-x1 * xv + -y1 * yv + -z1 * zv) * rdv, 0.f, 1.f);
    const float xp = x1 + xv * dot, yp = y1 + yv * dot, zp = z1 + zv * dot;
    float xo = -xp, yo = -yp, zo = -zp;
    const float ol = std::sqrt(xo * xo + yo * yo + zo * zo);
    xo = xo / ol;
    yo = yo / ol;
    zo = zo / ol;
    const float ro = clampf(ol, 0.f, r);
    const float xn = xp + ro * xo, yn = yp + ro * yo, zn = zp + ro * zo;
    return std::sqrt(xn * xn + yn * yn + zn * zn);
}

// Eigen::AngleAxisf(phi, Z) * AngleAxisf(theta, Y) * AngleAxisf(rho, X) (factory.hh:37-39):
// a product of AngleAxis is a quaternion; its rotation matrix columns are the cuboid axes.
// The exact float op order of Eigen is not reproduced (parity of Euler->axes is unpinned;
// fixtures pass resolved axes through vgpu_env_add_cuboid_axes).
static void euler_xyz_matrix(const float e[3], float R[3][3])
{
    const float hr = e[0] * 0.5f, ht = e[1] * 0.5f, hp = e[2] * 0.5f;
    const float cr = std::cos(hr), sr = std::sin(hr), ct = std::cos(ht), st = std::sin(ht), cp = std::cos(hp),
                sp = std::sin(hp);
    // q = qz(phi) * qy(theta) * qx(rho)
    const float w = cp * ct * cr + sp * st * sr;
    const float x = cp * ct * sr - sp * st * cr;
    const float y = cp * st * cr + sp * ct * sr;
    const float z = sp * ct * cr - cp * st * sr;
    R[0][0] = 1 - 2 * (y * y + z * z);
    R[0][1] = 2 * (x * y - w * z);
    R[0][2] = 2 * (x * z + w * y);
    R[1][0] = 2 * (x * y + w * z);
    R[1][1] = 1 - 2 * (x * x + z * z);
    R[1][2] = 2 * (y * z - w * x);
    R[2][0] = 2 * (x * z - w * y);
    R[2][1] = 2 * (y * z + w * x);
    R[2][2] = 1 - 2 * (x * x + y * y);
}

// c may be NULL: a host-only environment (build and inspect; it cannot be uploaded or used)
extern "C" int vgpu_env_create(vgpu_ctx* c, vgpu_env** out)
try {
    if (!out) return VGPU_ERR_INVALID_ARG;
    auto* e = new (std::nothrow) vgpu_env();
    if (!e) return fail(c, VGPU_ERR_OOM, "out of host memory");
    e->ctx = c;
    *out = e;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" void vgpu_env_destroy(vgpu_env* e)
{
    if (!e) return;
    if (e->dev) {
        (void)hipSetDevice(e->ctx->device);
        (void)hipStreamSynchronize(e->ctx->cur);
        (void)hipFree(e->dev);
    }
    delete e;
}

static bool finite3(const float* v) { return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]); }

extern "C" int vgpu_env_add_sphere(vgpu_env* e, const float c[3], float r)
try {
    if (!e || !c || !finite3(c) || !std::isfinite(r)) return VGPU_ERR_INVALID_ARG;
    e->spheres.push_back({c[0], c[1], c[2], r, sphere_min_distance(c[0], c[1], c[2], r)});
    e->dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_add_cuboid_axes(vgpu_env* e, const float c[3], const float a1[3], const float a2[3],
                                        const float a3[3], const float h[3])
try {
    if (!e || !c || !a1 || !a2 || !a3 || !h) return VGPU_ERR_INVALID_ARG;
    std::array<float, 16> row{c[0],  c[1],  c[2],  a1[0], a1[1], a1[2], a2[0], a2[1],
                              a2[2], a3[0], a3[1], a3[2], h[0],  h[1],  h[2],  0.0f};
    row[15] = cuboid_min_distance(row.data());
    if (row[11] == 1.0f)  // bindings/environment.cc:120 (axis_3_z == 1.)
        e->zcuboids.push_back(row);
    else
        e->cuboids.push_back(row);
    e->dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_add_cuboid_euler(vgpu_env* e, const float c[3], const float euler[3], const float h[3])
try {
    if (!e || !c || !euler || !h) return VGPU_ERR_INVALID_ARG;
    float R[3][3];
    euler_xyz_matrix(euler, R);
    const float a1[3] = {R[0][0], R[1][0], R[2][0]};
    const float a2[3] = {R[0][1], R[1][1], R[2][1]};
    const float a3[3] = {R[0][2], R[1][2], R[2][2]};
    return vgpu_env_add_cuboid_axes(e, c, a1, a2, a3, h);
} VGPU_ABI_CATCH

extern "C" int vgpu_env_add_capsule_endpoints(vgpu_env* e, const float p1[3], const float p2[3], float r)
try {
    if (!e || !p1 || !p2) return VGPU_ERR_INVALID_ARG;
    const float xv = p2[0] - p1[0], yv = p2[1] - p1[1], zv = p2[2] - p1[2];  // factory.hh:113-116
    const float dot = (xv * xv + yv * yv) + zv * zv;
    if (!(dot > 0.0f)) return fail(e->ctx, VGPU_ERR_INVALID_ARG, "degenerate capsule");
    std::array<float, 9> row{p1[0], p1[1], p1[2], xv, yv, zv, r, (float)(1.0 / (double)dot), 0.0f};
    row[8] = capsule_min_distance(row.data());
    if (xv == 0.0f && yv == 0.0f)  // bindings/environment.cc:134
        e->zcapsules.push_back(row);
    else
        e->capsules.push_back(row);
    e->dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_add_capsule_euler(vgpu_env* e, const float c[3], const float euler[3], float r, float len)
try {
    if (!e || !c || !euler) return VGPU_ERR_INVALID_ARG;
    float R[3][3];
    euler_xyz_matrix(euler, R);
    const float h = len / 2;  // factory.hh:168-171: p = T * (0, 0, +-len/2)
    const float p1[3] = {c[0] + R[0][2] * h, c[1] + R[1][2] * h, c[2] + R[2][2] * h};
    const float p2[3] = {c[0] - R[0][2] * h, c[1] - R[1][2] * h, c[2] - R[2][2] * h};
    return vgpu_env_add_capsule_endpoints(e, p1, p2, r);
} VGPU_ABI_CATCH

extern "C" int vgpu_env_counts(const vgpu_env* e, int32_t counts[5])
try {
    if (!e || !counts) return VGPU_ERR_INVALID_ARG;
    counts[0] = (int32_t)e->spheres.size();
    counts[1] = (int32_t)e->capsules.size();
    counts[2] = (int32_t)e->zcapsules.size();
    counts[3] = (int32_t)e->cuboids.size();
    counts[4] = (int32_t)e->zcuboids.size();
    return VGPU_OK;
} VGPU_ABI_CATCH

// HeightField via factory::heightfield::array / flat (factory.hh:365-423): reciprocal scales
extern "C" int vgpu_env_add_heightfield(vgpu_env* e, const float center[3], const float scale[3], size_t xd,
                                        size_t yd, const float* data)
try {
    if (!e || !center || !scale || (xd * yd && !data)) return VGPU_ERR_INVALID_ARG;
    if (xd == 0 || yd == 0 || xd * yd >= (1u << 24)) return fail(e->ctx, VGPU_ERR_INVALID_ARG, "heightfield size");
    vgpu::Heightfield h;
    h.x = center[0];
    h.y = center[1];
    h.z = center[2];
    h.xs = 1.0f / scale[0];
    h.ys = 1.0f / scale[1];
    h.zs = 1.0f / scale[2];
    h.xd = xd;
    h.yd = yd;
    h.data.assign(data, data + xd * yd);
    e->heightfields.push_back(std::move(h));
    e->dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

// Environment::add_pointcloud (bindings/environment.cc:148-158): builds the CAPT on the host
extern "C" int vgpu_env_add_pointcloud(vgpu_env* e, const float* points, size_t n, float r_min, float r_max,
                                       float r_point, int64_t* build_ns)
try {
    if (!e || (n && !points)) return VGPU_ERR_INVALID_ARG;
    if (n == 0 || n > ((size_t)1 << 26)) return fail(e->ctx, VGPU_ERR_INVALID_ARG, "point cloud size");
    for (size_t i = 0; i < 3 * n; ++i)
        if (!std::isfinite(points[i])) return fail(e->ctx, VGPU_ERR_INVALID_ARG, "non-finite point");
    e->pointclouds.emplace_back();
    vgpu::capt_build(points, n, r_min, r_max, r_point, e->pointclouds.back());
    if (build_ns) *build_ns = e->pointclouds.back().build_ns;
    e->dirty = e->pc_dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

namespace vgpu {
hipError_t capt_build_device(const float* points, size_t n, float r_min, float r_max, float r_point, hipStream_t st,
                             CaptTree& out);  // vgpu_capt_build.hip
}

extern "C" int vgpu_env_add_pointcloud_device(vgpu_ctx* c, vgpu_env* e, const float* points, size_t n, float r_min,
                                              float r_max, float r_point, int64_t* build_ns)
try {
    // env: this context's, or a host-only one (ctx NULL); the build runs on ctx's device and stream
    if (!c || !e || (e->ctx && e->ctx != c) || (n && !points))
        return fail(c, VGPU_ERR_INVALID_ARG, "bad add_pointcloud_device");
    if (n == 0 || n > ((size_t)1 << 26)) return fail(c, VGPU_ERR_INVALID_ARG, "point cloud size");
    HIPCHK(c, ctx_device(c));
    vgpu::CaptTree t;
    HIPCHK(c, vgpu::capt_build_device(points, n, r_min, r_max, r_point, c->cur, t));
    if (build_ns) *build_ns = t.build_ns;
    e->pointclouds.push_back(std::move(t));
    e->dirty = e->pc_dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

// A deep copy of src's obstacles, point clouds and attachment bound to context c (or host-only for NULL):
// the per-device environments of a multi-device batch (vgpu_multi.cpp)
extern "C" int vgpu_env_clone(const vgpu_env* src, vgpu_ctx* c, vgpu_env** out)
try {
    if (!src || !out) return VGPU_ERR_INVALID_ARG;
    *out = nullptr;
    auto* e = new (std::nothrow) vgpu_env();
    if (!e) return fail(c, VGPU_ERR_OOM, "out of host memory");
    e->ctx = c;
    e->spheres = src->spheres;
    e->capsules = src->capsules;
    e->zcapsules = src->zcapsules;
    e->cuboids = src->cuboids;
    e->zcuboids = src->zcuboids;
    e->heightfields = src->heightfields;
    e->pointclouds = src->pointclouds;
    e->attached = src->attached;
    e->att_tf = src->att_tf;
    e->att_spheres = src->att_spheres;
    *out = e;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_copy_pointcloud(vgpu_env* dst, const vgpu_env* src, int index)
try {
    if (!dst || !src || index < 0 || (size_t)index >= src->pointclouds.size()) return VGPU_ERR_INVALID_ARG;
    if (dst == src) {
        vgpu::CaptTree t = src->pointclouds[index];  // copy before the vector may reallocate
        dst->pointclouds.push_back(std::move(t));
    } else {
        dst->pointclouds.push_back(src->pointclouds[index]);
    }
    dst->dirty = dst->pc_dirty = dst->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_ext_counts(const vgpu_env* e, int32_t counts[2])
try {
    if (!e || !counts) return VGPU_ERR_INVALID_ARG;
    counts[0] = (int32_t)e->heightfields.size();
    counts[1] = (int32_t)e->pointclouds.size();
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_pointcloud_info(const vgpu_env* e, int index, int32_t* nlog2, size_t* n_aff, float top[6])
try {
    if (!e || index < 0 || (size_t)index >= e->pointclouds.size()) return VGPU_ERR_INVALID_ARG;
    const auto& t = e->pointclouds[index];
    if (nlog2) *nlog2 = t.nlog2;
    if (n_aff) *n_aff = t.n_aff();
    if (top) std::copy(t.top, t.top + 6, top);
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_pointcloud_arrays(const vgpu_env* e, int index, float* tests, float* aabbs,
                                          uint32_t* aff_starts, float* aff)
try {
    if (!e || index < 0 || (size_t)index >= e->pointclouds.size()) return VGPU_ERR_INVALID_ARG;
    const auto& t = e->pointclouds[index];
    if (tests) std::copy(t.tests.begin(), t.tests.end(), tests);
    if (aabbs) std::copy(t.aabbs.begin(), t.aabbs.end(), aabbs);
    if (aff_starts) std::copy(t.aff_starts.begin(), t.aff_starts.end(), aff_starts);
    if (aff) std::copy(t.aff.begin(), t.aff.end(), aff);
    return VGPU_OK;
} VGPU_ABI_CATCH

template <size_t W>
static void sort_md(std::vector<std::array<float, W>>& v)  // environment.hh:40-66
{
    std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a[W - 1] < b[W - 1]; });
}

// Device layout of EnvView (vgpu_device.hh): per type, records sorted by min_distance
// (environment.hh:40-66) followed by kObsPad sentinels with min_distance = +inf.
extern "C" int vgpu_env_attach(vgpu_env* e, const float tf[7], const float* spheres, size_t n)
try {
    if (!e || !tf || (n && !spheres)) return VGPU_ERR_INVALID_ARG;
    if (n > ((size_t)1 << 20)) return fail(e->ctx, VGPU_ERR_INVALID_ARG, "too many attached spheres");
    for (int i = 0; i < 7; ++i)
        if (!std::isfinite(tf[i])) return fail(e->ctx, VGPU_ERR_INVALID_ARG, "non-finite attachment frame");
    std::copy(tf, tf + 7, e->att_tf.begin());
    e->att_spheres.assign(n, {});
    for (size_t k = 0; k < n; ++k)
        for (int i = 0; i < 4; ++i) e->att_spheres[k][i] = spheres[4 * k + i];
    e->attached = true;
    e->dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_detach(vgpu_env* e)
try {
    if (!e) return VGPU_ERR_INVALID_ARG;
    e->attached = false;
    e->att_spheres.clear();
    e->dirty = e->host_dirty = true;
    return VGPU_OK;
} VGPU_ABI_CATCH

// The environment as one float blob: per obstacle type, records sorted by min_distance
// (environment.hh:40-66) followed by kObsPad sentinels (md = +inf), then heightfield / point-cloud
// headers and arrays, then the attachment.  The same layout serves the device (vgpu_env_upload)
// and the CPU rake (vgpu_env_host_view); offsets are recorded in the environment.
// Cells of the device point clouds' grids: VGPU_CAPT_GRID_CELLS unset = capt_grid_plan's default,
// 0 = no grid (the plain traversal, for A/B runs), N = about N cells.
static bool grid_cells(size_t& cells)
{
    const char* v = std::getenv("VGPU_CAPT_GRID_CELLS");
    cells = v ? (size_t)std::strtoull(v, nullptr, 10) : 0;
    return !(v && cells == 0);
}

// The blob in two sections.  Prefix: the point clouds (headers, then each cloud's arrays and, in device
// copies, its cell grid) -- rebuilt only when the set of clouds changes.  Tail (from tail_off): the five
// obstacle sections, heightfields, the attachment -- small, rewritten in place on add_sphere / attach /
// detach ... without touching the clouds or relaunching their grid builds (environment.cc:107-163 mutate
// the reference's environment in place just as cheaply).
// The cell grids are written by the device (vgpu_launch_capt_grid), so they are holes in the host copy of the
// prefix: `holes` receives (host position, device floats skipped) per grid, and every offset the prefix records
// is a device position (host position + the holes before it).  An upload then sends the host runs between
// the holes -- no zero-filled grid crosses PCIe (16 MB for the 10k-point cloud's 2M cells).
static void build_prefix(vgpu_env* e, vgpu_env::Layout& L, std::vector<float>& blob, bool device,
                         std::vector<std::pair<size_t, size_t>>* holes = nullptr)
{
    blob.assign(kDbgWords, 0.0f);  // the debug-check words (vgpu_device.hh VGPU_DCHECK), zero at every full upload
    if (device) e->pc_grid.clear();
    if (holes) holes->clear();
    size_t shift = 0;  // device floats of the holes so far (multiples of 16: host and device alignment agree)
    auto dpos = [&]() { return blob.size() + shift; };
    auto hdr_u = [](uint32_t u) { return u2f(u); };
    auto align16 = [&]() { while (blob.size() % 4) blob.push_back(0.0f); };
    L.pc_off = dpos();
    blob.resize(blob.size() + (size_t)kExtHdr * e->pointclouds.size(), 0.0f);
    for (size_t i = 0; i < e->pointclouds.size(); ++i) {
        const auto& t = e->pointclouds[i];
        align16();
        const size_t o_tests = dpos();
        blob.insert(blob.end(), t.tests.begin(), t.tests.end());
        align16();
        const size_t o_aabbs = dpos();
        blob.insert(blob.end(), t.aabbs.begin(), t.aabbs.end());
        align16();
        const size_t o_starts = dpos();
        for (uint32_t v : t.aff_starts) blob.push_back(u2f(v));
        align16();
        const size_t o_aff = dpos();
        blob.insert(blob.end(), t.aff.begin(), t.aff.end());
        float* hd = &blob[L.pc_off + kExtHdr * i];  // headers precede every hole: host == device position
        std::copy(t.top, t.top + 6, hd);
        hd[PC_RPOINT] = t.r_point;
        hd[PC_NLOG2] = hdr_u((uint32_t)t.nlog2);
        hd[PC_TESTS] = hdr_u((uint32_t)o_tests);
        hd[PC_AABBS] = hdr_u((uint32_t)o_aabbs);
        hd[PC_STARTS] = hdr_u((uint32_t)o_starts);
        hd[PC_AFF] = hdr_u((uint32_t)o_aff);
        // device copies: the cell grid, a hole filled by vgpu_launch_capt_grid after the upload
        vgpu::CaptGridArgs g{};
        size_t cells = 0;
        if (device && grid_cells(cells) && vgpu::capt_grid_plan(t, cells, g)) {
            while (blob.size() % 16) blob.push_back(0.0f);
            hd = &blob[L.pc_off + kExtHdr * i];  // the push_backs may have moved the blob
            g.tests_off = (uint32_t)o_tests;
            g.starts_off = (uint32_t)o_starts;
            g.aff_off = (uint32_t)o_aff;
            g.cells_off = (uint32_t)dpos();
            const size_t n_cells = (size_t)g.nx * g.ny * g.nz;
            g.nodes_off = g.split ? (uint32_t)(g.cells_off + ((n_cells + 15) & ~(size_t)15)) : 0u;
            const size_t hole = 2 * ((n_cells + 15) & ~(size_t)15);
            if (holes) holes->push_back({blob.size(), hole});
            shift += hole;
            const float gv[] = {g.x0, g.y0, g.z0, g.inv_h};
            std::copy(gv, gv + 4, hd + PC_GX);
            hd[PC_GNX] = hdr_u(g.nx);
            hd[PC_GNY] = hdr_u(g.ny);
            hd[PC_GNZ] = hdr_u(g.nz);
            hd[PC_GNXF] = (float)g.nx;
            hd[PC_GNYF] = (float)g.ny;
            hd[PC_GNZF] = (float)g.nz;
            hd[PC_GUNIT] = g.unit;
            hd[PC_GCELLS] = hdr_u(g.cells_off);
            hd[PC_GBRICK] = hdr_u(g.brick);
            hd[PC_GNODES] = hdr_u(g.nodes_off);
        }
        if (device) e->pc_grid.push_back(g);
    }
    while (blob.size() % 16) blob.push_back(0.0f);
}

// The bounding sphere of a capsule / cuboid record (vgpu_device.hh kObsBound): centre and a radius R such
// that the reference's test for a sphere (p, r) can only come out negative when |p - centre| <= r + R.
// Capsule: the segment's midpoint, |v| / 2 + radius (the closest point the test picks lies on the segment,
// sphere_capsule.hh:9-22; the z-capsule's test reads only the z component of v, :30-43).  Cuboid: the centre
// and the half diagonal |(r1, r2, r3)| -- the box distance is at least the centre distance less the half
// diagonal when the axes are orthonormal (sphere_cuboid.hh:9-52); other axes get R = +inf (never skipped).
// R is widened by 1e-5 of the record's scale (+ 1e-5) -- orders of magnitude above the float rounding of
// either test -- so the prefilter never skips a record whose test would fire.
static void obstacle_bound(int type, const float* row, float* out)
{
    double c[3], R;
    if (type == OBS_CAPSULE || type == OBS_ZCAPSULE) {
        const double vx = type == OBS_CAPSULE ? row[3] : 0.0, vy = type == OBS_CAPSULE ? row[4] : 0.0, vz = row[5];
        c[0] = row[0] + 0.5 * vx;
        c[1] = row[1] + 0.5 * vy;
        c[2] = row[2] + 0.5 * vz;
        R = 0.5 * std::sqrt(vx * vx + vy * vy + vz * vz) + std::fabs((double)row[6]);
    } else {
        for (int i = 0; i < 3; ++i) c[i] = row[i];
        double ax[3][3];
        for (int k = 0; k < 3; ++k)
            for (int i = 0; i < 3; ++i) ax[k][i] = row[3 + 3 * k + i];
        if (type == OBS_ZCUBOID) {  // the test uses a1, a2 in the xy plane and the z axis
            ax[0][2] = ax[1][2] = 0.0;
            ax[2][0] = ax[2][1] = 0.0;
            ax[2][2] = 1.0;
        }
        bool ortho = true;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                const double d = ax[a][0] * ax[b][0] + ax[a][1] * ax[b][1] + ax[a][2] * ax[b][2];
                ortho = ortho && std::fabs(d - (a == b ? 1.0 : 0.0)) <= 1e-6;
            }
        const double h0 = row[12], h1 = row[13], h2 = row[14];
        R = ortho ? std::sqrt(h0 * h0 + h1 * h1 + h2 * h2) : HUGE_VAL;
    }
    const double scale = std::fabs(c[0]) + std::fabs(c[1]) + std::fabs(c[2]) + R;
    R += 1e-5 * (1.0 + scale);
    for (int i = 0; i < 3; ++i) out[i] = (float)c[i];
    out[3] = std::isfinite(R) && std::isfinite(scale) && R < 3e38 ? std::nextafter((float)R, HUGE_VALF) : HUGE_VALF;
    if (!(std::isfinite(out[0]) && std::isfinite(out[1]) && std::isfinite(out[2]))) out[3] = HUGE_VALF;
}

// The tail section as its own vector; its offsets are recorded relative to the blob, starting at base.
static void build_tail(vgpu_env* e, vgpu_env::Layout& L, std::vector<float>& tail, size_t base)
{
    sort_md(e->spheres);
    sort_md(e->capsules);
    sort_md(e->zcapsules);
    sort_md(e->cuboids);
    sort_md(e->zcuboids);
    tail.clear();
    auto put = [&](auto& v, int type, int np) {
        const int S = kObsStride[type];
        L.off[type] = base + tail.size();
        L.cnt[type] = (int)v.size();
        if (type == OBS_SPHERE) {  // pair blocks (vgpu_device.hh scan_spheres), then sentinel blocks
            const size_t blocks = (v.size() + kObsPad + 1) / 2;
            for (size_t b = 0; b < blocks; ++b) {
                const size_t at = tail.size();
                tail.resize(at + kSphereBlock, 0.0f);
                for (int h = 0; h < 2; ++h) {
                    const size_t j = 2 * b + h;
                    if (j < v.size()) {
                        tail[at + h] = v[j][np];  // min_distance
                        for (int i = 0; i < np; ++i) tail[at + 2 + 2 * i + h] = v[j][i];
                    } else {
                        tail[at + h] = __builtin_inff();
                    }
                }
            }
            while (tail.size() % 16) tail.push_back(0.0f);
            return;
        }
        for (auto& row : v) {
            const size_t at = tail.size();
            tail.resize(at + S, 0.0f);
            tail[at] = row[np];  // min_distance is the last field of the host row
            for (int i = 0; i < np; ++i) tail[at + 1 + i] = row[i];
            if (kObsBound[type] >= 0) obstacle_bound(type, row.data(), &tail[at + kObsBound[type]]);
        }
        for (int k = 0; k < kObsPad; ++k) {
            const size_t at = tail.size();
            tail.resize(at + S, 0.0f);
            tail[at] = __builtin_inff();
        }
        while (tail.size() % 16) tail.push_back(0.0f);
    };
    put(e->spheres, OBS_SPHERE, 4);
    put(e->capsules, OBS_CAPSULE, 8);
    put(e->zcapsules, OBS_ZCAPSULE, 8);
    put(e->cuboids, OBS_CUBOID, 15);
    put(e->zcuboids, OBS_ZCUBOID, 15);
    // heightfields: kExtHdr-float headers, then their arrays (16-B aligned)
    auto hdr_u = [](uint32_t u) { return u2f(u); };
    auto align16 = [&]() { while (tail.size() % 4) tail.push_back(0.0f); };
    L.hf_off = base + tail.size();
    tail.resize(tail.size() + (size_t)kExtHdr * e->heightfields.size(), 0.0f);
    for (size_t i = 0; i < e->heightfields.size(); ++i) {
        const auto& h = e->heightfields[i];
        align16();
        const size_t data_off = base + tail.size();
        tail.insert(tail.end(), h.data.begin(), h.data.end());
        float* hd = &tail[L.hf_off - base + kExtHdr * i];
        const float v[HF_OFF] = {h.x, h.y, h.z, h.xs, h.ys, h.zs, (float)h.xd, (float)h.yd, (float)(h.xd / 2),
                                 (float)(h.yd / 2)};
        std::copy(v, v + HF_OFF, hd);
        hd[HF_OFF] = hdr_u((uint32_t)data_off);
        hd[HF_CELLS] = hdr_u((uint32_t)(h.xd * h.yd));
    }
    // the attachment: frame (7 floats + pad), then its spheres (16-B aligned)
    align16();
    L.att_off = base + tail.size();
    tail.resize(tail.size() + kAttHdr, 0.0f);
    std::copy(e->att_tf.begin(), e->att_tf.end(), tail.begin() + (L.att_off - base));
    for (const auto& sp : e->att_spheres) tail.insert(tail.end(), sp.begin(), sp.end());
}

// host: the whole blob; device (holes != NULL): the blob minus the grid holes, *dev_floats = its device size
static int build_blob(vgpu_env* e, std::vector<float>& blob, std::vector<std::pair<size_t, size_t>>* holes = nullptr,
                      size_t* dev_floats = nullptr)
{
    const bool device = holes != nullptr;
    vgpu_env::Layout& L = device ? e->dev_lay : e->host_lay;
    build_prefix(e, L, blob, device, holes);
    size_t shift = 0;
    if (holes)
        for (const auto& h : *holes) shift += h.second;
    std::vector<float> tail;
    const size_t base = blob.size() + shift;  // device position of the tail
    build_tail(e, L, tail, base);
    blob.insert(blob.end(), tail.begin(), tail.end());
    if (device) e->tail_off = base;
    if (dev_floats) *dev_floats = blob.size() + shift;
    if (blob.size() + shift >= ((size_t)1 << 32))
        return fail(e->ctx, VGPU_ERR_INVALID_ARG, "environment larger than 16 GiB");
    return VGPU_OK;
}

extern "C" int vgpu_env_upload(vgpu_env* e)
try {
    if (!e) return VGPU_ERR_INVALID_ARG;
    vgpu_ctx* c = e->ctx;
    if (!c) return VGPU_ERR_INVALID_ARG;  // host-only environment
    if (!e->dirty && !e->pc_dirty && e->dev) return VGPU_OK;
    std::lock_guard<std::mutex> lock(e->host_mu);  // the builds re-sort the host rows
    HIPCHK(c, ctx_device(c));
    if (e->dev && !e->pc_dirty) {  // the tail alone, in place, when it still fits the allocation
        std::vector<float> tail;
        build_tail(e, e->dev_lay, tail, e->tail_off);
        if (e->tail_off + tail.size() <= e->dev_floats) {
            HIPCHK(c, hipMemcpyAsync(e->dev + e->tail_off, tail.data(), tail.size() * sizeof(float),
                                     hipMemcpyHostToDevice, c->cur));
            HIPCHK(c, hipStreamSynchronize(c->cur));  // tail is a host temporary
            e->dirty = false;
            ++e->n_tail;
            return VGPU_OK;
        }
    }
    std::vector<float> blob;
    std::vector<std::pair<size_t, size_t>> holes;
    size_t total = 0;
    if (int rc = build_blob(e, blob, &holes, &total)) return rc;
    // room for the tail to grow in place (obstacles added later, an attachment)
    const size_t want = total + std::max<size_t>(total - e->tail_off, 4096);
    if (total > e->dev_floats) {
        if (e->dev) {
            HIPCHK(c, hipStreamSynchronize(c->cur));
            HIPCHK(c, hipFree(e->dev));
            e->dev = nullptr;
            e->dev_floats = 0;
        }
        HIPCHK(c, hipMalloc(&e->dev, want * sizeof(float)));
        e->dev_floats = want;
    }
    // the host runs between the grid holes
    size_t hpos = 0, dpos = 0;
    for (size_t k = 0; k <= holes.size(); ++k) {
        const size_t hend = k < holes.size() ? holes[k].first : blob.size();
        if (hend > hpos)
            HIPCHK(c, hipMemcpyAsync(e->dev + dpos, blob.data() + hpos, (hend - hpos) * sizeof(float),
                                     hipMemcpyHostToDevice, c->cur));
        dpos += hend - hpos;
        hpos = hend;
        if (k < holes.size()) dpos += holes[k].second;
    }
    for (const auto& g : e->pc_grid)
        if (g.cells_off) {
            HIPCHK(c, vgpu_launch_capt_grid(e->dev, &g, c->cur));
            ++e->n_grids;
        }
    HIPCHK(c, hipStreamSynchronize(c->cur));  // blob is a host temporary
    e->dirty = e->pc_dirty = false;
    ++e->n_full;
    return VGPU_OK;
} VGPU_ABI_CATCH

// The cell grid of point cloud `index` as its DEVICE header records it: out = {nx, ny, nz, cells_off} (all 0:
// no grid).  Reads the uploaded header back, so a layout slip that drops the grid shows up in a test.
extern "C" int vgpu_env_pointcloud_grid(vgpu_env* e, int index, uint32_t out[4])
try {
    if (!e || !out || !e->ctx || index < 0 || (size_t)index >= e->pointclouds.size()) return VGPU_ERR_INVALID_ARG;
    if (int rc = vgpu_env_upload(e)) return rc;
    vgpu_ctx* c = e->ctx;
    float hd[kExtHdr];
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    HIPCHK(c, hipMemcpy(hd, e->dev + e->dev_lay.pc_off + (size_t)kExtHdr * index, sizeof(hd), hipMemcpyDeviceToHost));
    const int f[4] = {PC_GNX, PC_GNY, PC_GNZ, PC_GCELLS};
    for (int k = 0; k < 4; ++k) std::memcpy(&out[k], &hd[f[k]], 4);
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_env_upload_stats(const vgpu_env* e, uint64_t out[3])
try {
    if (!e || !out) return VGPU_ERR_INVALID_ARG;
    out[0] = e->n_full;
    out[1] = e->n_tail;
    out[2] = e->n_grids;
    return VGPU_OK;
} VGPU_ABI_CATCH

// Host view for the CPU rake (csrc/cpu/vcpu.cpp): the same blob in host memory, rebuilt when the
// environment changed.  Offsets are identical to the device copy's.
int vgpu_env_host_view(vgpu_env* e, vgpu::HostEnvView* v)
{
    if (!e || !v) return VGPU_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lock(e->host_mu);
    if (e->host_dirty) {
        if (int rc = build_blob(e, e->host_blob)) return rc;
        e->host_dirty = false;
    }
    const float* b = e->host_blob.data();
    const vgpu_env::Layout& L = e->host_lay;
    for (int t = 0; t < OBS_TYPES; ++t) {
        v->obs[t] = b + L.off[t];
        v->n[t] = L.cnt[t];
    }
    v->hf = b + L.hf_off;
    v->pc = b + L.pc_off;
    v->base = b;
    v->n_hf = (int)e->heightfields.size();
    v->n_pc = (int)e->pointclouds.size();
    v->att = b + L.att_off;
    v->n_att = e->attached ? (int)e->att_spheres.size() : 0;
    v->attached = e->attached;
    return VGPU_OK;
}

static EnvView make_view(const vgpu_env* e)
{
    EnvView v{};
    const vgpu_env::Layout& L = e->dev_lay;
    for (int t = 0; t < OBS_TYPES; ++t) {
        v.obs[t] = (const VGPU_CONST float*)(e->dev + L.off[t]);
        v.n[t] = L.cnt[t];
    }
    v.lut = e->ctx->lut_dev;
    v.kbits = e->ctx->kbits;
    v.hf = (const VGPU_CONST float*)(e->dev + L.hf_off);
    v.pc = (const VGPU_CONST float*)(e->dev + L.pc_off);
    v.base = e->dev;
    v.n_hf = (int)e->heightfields.size();
    v.n_pc = (int)e->pointclouds.size();
    v.att = (const VGPU_CONST float*)(e->dev + L.att_off);
    v.n_att = e->attached ? (int)e->att_spheres.size() : 0;
    // near sets (vgpu_device.hh env_near): every primitive record has a bit
    int total = 0;
    for (int t = 0; t < OBS_TYPES; ++t) {
        v.near_base[t] = total;
        total += v.n[t];
    }
    v.near_ok = (total <= kNearMax && !e->ctx->no_near) ? 1 : 0;
    return v;
}

// ---------------------------------------------------------------------------------------
// batch entry points
// ---------------------------------------------------------------------------------------
static const RobotOps* generic_ops(int32_t kind);
static size_t dim_of(const vgpu_robot* r);

extern "C" int vgpu_robot_info(int32_t kind, int32_t* dim, int32_t* res, int32_t* ns)
try {
    if (const RobotOps* g = generic_ops(kind)) {
        if (dim) *dim = g->dim;
        if (res) *res = g->resolution;
        if (ns) *ns = g->n_spheres;
        return VGPU_OK;
    }
    if (kind == VGPU_ROBOT_PANDA_PAIR) {
        if (dim) *dim = kPairDim;
        if (res) *res = kPandaResolution;
        if (ns) *ns = 2 * kPandaSpheres;
        return VGPU_OK;
    }
    if (kind == VGPU_ROBOT_FETCH) {
        if (dim) *dim = kFetchDim;
        if (res) *res = kFetchResolution;
        if (ns) *ns = kFetchSpheres;
        return VGPU_OK;
    }
    if (kind != VGPU_ROBOT_PANDA) return VGPU_ERR_UNSUPPORTED;
    if (dim) *dim = kPandaDim;
    if (res) *res = kPandaResolution;
    if (ns) *ns = kPandaSpheres;
    return VGPU_OK;
} VGPU_ABI_CATCH

// both arms' bases of a VGPU_ROBOT_PANDA_PAIR, metres (panda/fk.hh:109-111 per arm)
static void pair_bases(const vgpu_robot* r, float pb[6])
{
    pb[0] = (float)r->base_x100 / 100.0f;
    pb[1] = (float)r->base_y100 / 100.0f;
    pb[2] = (float)r->base_z100 / 100.0f;
    pb[3] = (float)r->base2_x100 / 100.0f;
    pb[4] = (float)r->base2_y100 / 100.0f;
    pb[5] = (float)r->base2_z100 / 100.0f;
}

static int check_robot(vgpu_ctx* c, const vgpu_robot* r, float base[3])
{
    if (!r) return fail(c, VGPU_ERR_INVALID_ARG, "null robot");
    if (r->kind == VGPU_ROBOT_FETCH || generic_ops(r->kind)) {  // fetch.hh, ur5.hh, baxter.hh: no base offset
        if (r->base_x100 || r->base_y100 || r->base_z100)
            return fail(c, VGPU_ERR_INVALID_ARG, "this robot has no base offset (base_*100 must be 0)");
        base[0] = base[1] = base[2] = 0.0f;
        return VGPU_OK;
    }
    if (r->kind != VGPU_ROBOT_PANDA && r->kind != VGPU_ROBOT_PANDA_PAIR)
        return fail(c, VGPU_ERR_UNSUPPORTED, "unsupported robot kind");
    // robots/panda/fk.hh:109-111: static_cast<float>(base_x100) / 100.0f
    base[0] = (float)r->base_x100 / 100.0f;
    base[1] = (float)r->base_y100 / 100.0f;
    base[2] = (float)r->base_z100 / 100.0f;
    return VGPU_OK;
}

extern "C" int vgpu_sphere_fk(vgpu_ctx* c, const vgpu_robot* r, const float* q, size_t n, float* xyz, size_t ld)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    if (n && (!q || !xyz || ld < n)) return fail(c, VGPU_ERR_INVALID_ARG, "bad sphere_fk arguments");
    HIPCHK(c, ctx_device(c));
    if (r->kind == VGPU_ROBOT_FETCH) {
        HIPCHK(c, vgpu_launch_fetch_sphere_fk(q, n, xyz, ld, c->cur));
        return VGPU_OK;
    }
    if (const RobotOps* g = generic_ops(r->kind)) {
        HIPCHK(c, g->sphere_fk(q, n, xyz, ld, c->cur));
        return VGPU_OK;
    }
    if (r->kind == VGPU_ROBOT_PANDA_PAIR)
        return fail(c, VGPU_ERR_UNSUPPORTED, "sphere_fk of the composite: call it per arm (VGPU_ROBOT_PANDA)");
    HIPCHK(c, vgpu_launch_panda_sphere_fk(q, n, b[0], b[1], b[2], xyz, ld, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

// One staged pass (vgpu_staged.hip) over n groups of a source kind (0 configurations, 1 Halton
// samples, 2 validate head, 3 validate tail): bound -> counts to host -> queue -> children.
static int grow(vgpu_ctx* c, uint32_t** p, size_t* cap, size_t need)
{
    if (need <= *cap) return VGPU_OK;
    if (*p) {
        HIPCHK(c, hipStreamSynchronize(c->cur));
        HIPCHK(c, hipFree(*p));
        *p = nullptr;
    }
    const size_t n = std::max(need + need / 4, (size_t)1 << 16);
    HIPCHK(c, hipMalloc((void**)p, n * sizeof(uint32_t)));
    *cap = n;
    return VGPU_OK;
}

// the staged pipeline of one robot (vgpu_staged.hh instantiations)
struct StagedOps {
    int (*checks)(void);
    uint64_t (*env_checks)(void);
    int (*mask_bytes)(void);
    int (*child_class)(int, int);  // (check, point-cloud / heightfield environment)
    size_t (*plan_bytes)(void);
    uint32_t (*blocks)(int, uint32_t);
    hipError_t (*bound)(int, const void*, const void*, const void*, const void*, uint64_t, uint32_t, const EnvView*,
                        const float*, int, void*, uint8_t*, hipStream_t);
    hipError_t (*count)(int, const void*, const void*, const void*, const void*, const void*, uint32_t, uint64_t,
                        const uint8_t*, uint32_t*, hipStream_t);
    hipError_t (*plan)(const uint32_t*, uint32_t, uint32_t, uint64_t, uint32_t, void*, int, hipStream_t);
    hipError_t (*queue)(int, const void*, const void*, const void*, const void*, const void*, uint32_t, uint64_t,
                        const void*, const uint8_t*, const uint32_t*, uint32_t*, const void*, hipStream_t);
    hipError_t (*children)(int, const void*, const void*, const void*, const void*, uint64_t, const void*,
                           const uint32_t*, const uint32_t*, const EnvView*, const float*, uint8_t*, hipStream_t);
    // source kinds (bit k = kind k) run as ONE round of every check: there the rounds' bookkeeping costs
    // more than their early exit saves (A/B on MI355X, profiles/r04e_ab.log, r04f_rounds_ab.log: the Fetch
    // sampler 1.09 -> 1.02 ms per 4M draws, the composite 10.69-10.73 -> 10.53-10.55 ms per 2^20 edges;
    // the Panda keeps its rounds for heads and configurations: set B 2.53 vs 2.85 ms, set A 1.61 vs 2.95, CAPT
    // 0.52 vs 0.64; its validate tails, whose bound stage runs the mid-sphere tests, take one round: set B
    // 2.33-2.37 -> 2.32, set A 1.41-1.45 -> 1.40, profiles/r04l_ab.log)
    unsigned one_round_kinds;
    int (*lead_check)(void);  // the robot's lead check (vgpu_staged.hh lead_kernel), -1: none
    hipError_t (*lead)(int, const void*, const void*, const void*, const void*, uint64_t, uint32_t, const EnvView*,
                       const float*, uint8_t*, hipStream_t);
    // source kinds (bit k = kind k) that run the lead pass first: where its check invalidates most
    // groups, the chained bound stage skips them (the Panda's validate heads, A/B in DESIGN.md §5d)
    unsigned lead_kinds;
    int (*head_list)(void);  // 1: after the lead pass, validate heads run over the compacted list of live edges
    // a robot compiled as several translation units by source kind (vgpu_fetch_staged.hip VGPU_FETCH_PART):
    // by_kind[k] = the part whose exports run kind k (NULL: this table runs every kind)
    const struct StagedOps* const* by_kind = nullptr;
};
#define VGPU_STAGED_OPS(NAME, ONE_ROUND, LEAD)                                                                           \
    StagedOps                                                                                                        \
    {                                                                                                                \
        vgpu_##NAME##_staged_checks, vgpu_##NAME##_staged_env_checks, vgpu_##NAME##_staged_mask_bytes,               \
            vgpu_##NAME##_staged_class, vgpu_##NAME##_staged_plan_bytes, vgpu_##NAME##_staged_blocks,                \
            vgpu_##NAME##_staged_bound, vgpu_##NAME##_staged_count, vgpu_##NAME##_staged_plan,                       \
            vgpu_##NAME##_staged_queue, vgpu_##NAME##_staged_children, ONE_ROUND, vgpu_##NAME##_staged_lead_check,   \
            vgpu_##NAME##_staged_lead, LEAD, vgpu_##NAME##_staged_head_list                                          \
    }
static const StagedOps kPandaParts[4] = {VGPU_STAGED_OPS(panda_p0, (1u << 3) | (1u << 4), 1u << 2),
                                         VGPU_STAGED_OPS(panda_p1, (1u << 3) | (1u << 4), 1u << 2),
                                         VGPU_STAGED_OPS(panda_p2, (1u << 3) | (1u << 4), 1u << 2),
                                         VGPU_STAGED_OPS(panda_p3, (1u << 3) | (1u << 4), 1u << 2)};
static const StagedOps* const kPandaByKind[5] = {&kPandaParts[0], &kPandaParts[0], &kPandaParts[1], &kPandaParts[2],
                                                 &kPandaParts[3]};
static const StagedOps kPandaStaged = [] {
    StagedOps o = kPandaParts[0];
    o.by_kind = kPandaByKind;
    return o;
}();
// the Fetch: the sampler and the validate tails as one round (edge stage at 100k vertices 26.12-26.14 ->
// 25.81-25.97 ms per step, profiles/r04t_fetch_rounds_ab.log)
static const StagedOps kFetchParts[4] = {VGPU_STAGED_OPS(fetch_p0, (1u << 1) | (1u << 3) | (1u << 4), 0u),
                                         VGPU_STAGED_OPS(fetch_p1, (1u << 1) | (1u << 3) | (1u << 4), 0u),
                                         VGPU_STAGED_OPS(fetch_p2, (1u << 1) | (1u << 3) | (1u << 4), 0u),
                                         VGPU_STAGED_OPS(fetch_p3, (1u << 1) | (1u << 3) | (1u << 4), 0u)};
static const StagedOps* const kFetchByKind[5] = {&kFetchParts[0], &kFetchParts[0], &kFetchParts[1], &kFetchParts[2],
                                                 &kFetchParts[3]};
static const StagedOps kFetchStaged = [] {
    StagedOps o = kFetchParts[0];
    o.by_kind = kFetchByKind;
    return o;
}();
static const StagedOps kUr5Staged = VGPU_STAGED_OPS(ur5, 0u, 0u);
// the two-Panda composite: four chained passes (vgpu_pair_staged.hip) -- arm A, arm B, inter-arm chunks
static const StagedOps kPairStaged[4] = {VGPU_STAGED_OPS(pair_a, 0x1Fu, 0u), VGPU_STAGED_OPS(pair_b, 0x1Fu, 0u),
                                         VGPU_STAGED_OPS(pair_i0, 0x1Fu, 0u), VGPU_STAGED_OPS(pair_i1, 0x1Fu, 0u)};

// robots built from vgpu_robot.hh (one TU each): their launch table, or NULL
static const RobotOps* generic_ops(int32_t kind)
{
    switch (kind) {
    case VGPU_ROBOT_UR5: return vgpu_ur5_ops();
    case VGPU_ROBOT_BAXTER: return vgpu_baxter_ops();
    default: return nullptr;
    }
}
// the Baxter: its 388 checks in 7 chained chunks of <= 64 (vgpu_baxter_staged.hip)
static const StagedOps kBaxterStaged[7] = {VGPU_STAGED_OPS(baxter_c0, 0u, 0u), VGPU_STAGED_OPS(baxter_c1, 0u, 0u),
                                           VGPU_STAGED_OPS(baxter_c2, 0u, 0u), VGPU_STAGED_OPS(baxter_c3, 0u, 0u),
                                           VGPU_STAGED_OPS(baxter_c4, 0u, 0u), VGPU_STAGED_OPS(baxter_c5, 0u, 0u),
                                           VGPU_STAGED_OPS(baxter_c6, 0u, 0u)};
// A robot's staged pipeline: one pass, or several chained passes over the same groups (check lists
// beyond one 64-bit mask, the composite's arms and inter-arm checks)
struct StagedChain {
    const StagedOps* ops;
    int n;
};
static StagedChain generic_chain(int32_t kind)
{
    if (kind == VGPU_ROBOT_UR5) return {&kUr5Staged, 1};
    if (kind == VGPU_ROBOT_BAXTER) return {kBaxterStaged, 7};
    return {nullptr, 0};
}

// One staged pass (vgpu_staged.hh) over n groups:
//   bound -> count(all checks) -> scan -> [read back the per-check counts: the pass's ONE sync]
//   -> per round: (count -> scan, later rounds) -> plan -> queue -> children per class.
// The first round's per-check counts bound every later round's (groups only ever become invalid),
// so they size all item buffers and children grids; the exact per-round layout is computed on the
// device (plan_kernel) and read there by queue and children.
// b: the robot base (b[0..2]) -- and the composite's second arm (b[3..5]); chain != 0: a later pass
// over the same groups (the flags are ANDed into, groups already invalid skip every stage)
// masks_ready: this pass's masks were stored by the previous pass's bound kernel at c->st_mask + mask_off
// (vgpu_staged.hh BothChunks) -- its own bound kernel is skipped
static int staged_pass(vgpu_ctx* c, const StagedOps& ops_in, int kind, const void* s0, const void* s1, const void* s2,
                       const void* s3, uint64_t first, size_t n, const EnvView* v, const float b[3], uint8_t* valid,
                       int chain = 0, const float* b2 = nullptr, bool masks_ready = false, size_t mask_off = 0)
{
    if (kind < 0 || kind > 4) return fail(c, VGPU_ERR_INVALID_ARG, "staged pass: source kind");
    const StagedOps& ops = ops_in.by_kind ? *ops_in.by_kind[kind] : ops_in;
    const float bases[6] = {b[0], b[1], b[2], b2 ? b2[0] : 0.0f, b2 ? b2[1] : 0.0f, b2 ? b2[2] : 0.0f};
    if (n == 0) return VGPU_OK;
    if (n >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "too many groups in one call (< 2^31)");
    const int checks = ops.checks();
    const uint32_t W = (kind >= 2) ? 8u : 64u;  // items per wave: 64 lanes / group size
    const size_t nb = ops.blocks(kind, (uint32_t)n);
    const size_t cells = (size_t)checks * nb;
    const size_t scan_bytes = vgpu_validate_scan_bytes(cells);
    const size_t cells_al = (cells + 1 + 63) & ~(size_t)63;
    const size_t plan_words = ((ops.plan_bytes() + 3) / 4 + 63) & ~(size_t)63;  // keeps tmp 256-B aligned
    int rc;
    if (!masks_ready && (rc = grow(c, &c->st_mask, &c->st_mask_cap, n * (size_t)ops.mask_bytes() / 4))) return rc;
    uint32_t* const mask = c->st_mask + mask_off;
    if ((rc = grow(c, &c->st_cnt, &c->st_cnt_cap, 2 * cells_al + scan_bytes / 4 + 64 + plan_words))) return rc;
    if (!c->st_host) HIPCHK(c, hipHostMalloc((void**)&c->st_host, 128 * sizeof(uint32_t), hipHostMallocDefault));
    uint32_t* counts = c->st_cnt;
    uint32_t* offs = c->st_cnt + cells_al;
    void* plan = c->st_cnt + 2 * cells_al;
    void* tmp = c->st_cnt + 2 * cells_al + plan_words;
    HIPCHK(c, hipMemsetAsync(counts + cells, 0, sizeof(uint32_t), c->cur));
    // the lead pass: one check for every group first (it initialises the flags), the rest chained
    const int lead = ops.lead_check();
    const unsigned lead_kinds = c->lead >= 0 ? (unsigned)c->lead : ops.lead_kinds;
    const bool use_lead = lead >= 0 && !chain && ((lead_kinds >> kind) & 1u) && v->n_hf == 0 && v->n_pc == 0;
    // (round 5: the lead check fused into the bound kernel -- its children inside, no second FK -- measured
    // slower on MI355X, set B 2.33 -> 2.41 ms, set A 0.81 -> 0.90: profiles/r05c_ab.log; not kept)
    if (use_lead) {
        HIPCHK(c, ops.lead(kind, s0, s1, s2, s3, first, (uint32_t)n, v, bases, valid, c->cur));
        chain = 1;
        // validate heads: the rest of the pass runs over the edges the lead check left valid, compacted (a wave
        // of the bound stage otherwise carries the groups it killed -- ~40 % of set B's heads -- as idle lanes)
        if (kind == 2 && !s2 && c->head_list && ops.head_list()) {
            const size_t sel = vgpu_compact_bytes(n);
            const size_t list_words = (n + 63) & ~(size_t)63;
            if ((rc = grow(c, &c->st_list, &c->st_list_cap, list_words + 64 + (sel + 3) / 4))) return rc;
            uint32_t* const live = c->st_list + list_words;
            HIPCHK(c, vgpu_launch_compact(valid, n, c->st_list, live, live + 64, sel, c->cur));
            s2 = c->st_list;
            s3 = live;
        }
    }
    if (!masks_ready) HIPCHK(c, ops.bound(kind, s0, s1, s2, s3, first, (uint32_t)n, v, bases, chain, mask, valid, c->cur));
    uint64_t all = checks >= 64 ? ~0ull : ((1ull << checks) - 1ull);
    if (use_lead) all &= ~(1ull << lead);  // decided by the lead pass
    const uint64_t env_bits = ops.env_checks();
    const int ext = (v->n_hf > 0 || v->n_pc > 0) ? 1 : 0;  // the children kernels' EXT instantiation (class table)
    // every check's fired groups (groups still valid): segment boundaries offs[k * nb], k = 0..checks
    HIPCHK(c, ops.count(kind, s0, s1, s2, s3, mask, (uint32_t)n, all, valid, counts, c->cur));
    HIPCHK(c, vgpu_launch_scan(counts, offs, cells, tmp, scan_bytes, c->cur));
    HIPCHK(c, hipMemcpy2DAsync(c->st_host, sizeof(uint32_t), offs, nb * sizeof(uint32_t), sizeof(uint32_t), checks + 1,
                               hipMemcpyDeviceToHost, c->cur));
    if (c->stats && kind == 2 && s3)  // the compacted head list's live count (statistics only)
        HIPCHK(c, hipMemcpyAsync(c->st_host + 127, s3, sizeof(uint32_t), hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    uint32_t fired[64];
    for (int k = 0; k < checks; ++k) fired[k] = c->st_host[k + 1] - c->st_host[k];
    if (c->stats) {  // VAMP_AMD_STAGED_STATS=1: the pass's bounding statistics (development)
        std::fprintf(stderr, "staged kind=%d chain=%d groups=%zu", kind, chain, n);
        if (kind == 2 && s3) std::fprintf(stderr, " live=%u", c->st_host[127]);
        std::fprintf(stderr, " fired:");
        for (int k = 0; k < checks; ++k) std::fprintf(stderr, " %u", fired[k]);
        std::fprintf(stderr, "\n");
    }
    std::vector<uint64_t> rounds(c->rounds.begin(), c->rounds.end());
    const unsigned one_round = c->one_round >= 0 ? (unsigned)c->one_round : ops.one_round_kinds;
    if (rounds.empty() && ((one_round >> kind) & 1u)) rounds = {all};
    if (rounds.empty()) {
        // Rounds from this batch's bounding statistics: (1) the environment check that fires for
        // the most groups, alone (the Panda's link-5 sphere: it fires for ~every group of an
        // invalid-heavy batch and its children confirm 97 % of them there, so later rounds see few
        // groups), (3) self checks whose bounding spheres overlap for ~every group (adjacent links:
        // many children, rarely a hit), (2) everything else.  Later rounds only see the groups still
        // valid: the reference's early exit, recovered at round granularity.  A/B on MI355X
        // (profiles/r04k_rounds_ab.log) against round 1 = the first three environment checks that
        // fire: set A 1.61 -> 1.45 ms, set B 2.41 -> 2.36-2.39, fkcc 0.85 -> 0.855.
        uint64_t r1 = 0, r3 = 0;
        for (int k = 0, best = -1; k < checks; ++k)
            if (((env_bits >> k) & 1u) && fired[k] && (best < 0 || fired[k] > fired[best])) r1 = 1ull << k, best = k;
        for (int k = 0; k < checks; ++k)
            if (!((env_bits >> k) & 1u) && fired[k] >= n - n / 100) r3 |= 1ull << k;
        rounds = {r1, all & ~r1 & ~r3, r3};
    }
    size_t items_ub = 0;  // items of any round at most
    for (int k = 0; k < checks; ++k) items_ub += (fired[k] + W - 1) / W * W;
    if (items_ub >= ((size_t)1 << 32)) return fail(c, VGPU_ERR_INVALID_ARG, "staged pass: more than 2^32 items");
    if ((rc = grow(c, &c->st_items, &c->st_items_cap, items_ub + 1))) return rc;
    bool first_round = true;  // its counts are the ones read back
    for (uint64_t set : rounds) {
        set &= all;
        uint32_t ub[4] = {0, 0, 0, 0};  // per children class, from the first round's counts
        for (int k = 0; k < checks; ++k)
            if ((set >> k) & 1u) ub[ops.child_class(k, ext)] += (fired[k] + W - 1) / W * W;
        if (!(ub[0] | ub[1] | ub[2] | ub[3])) continue;
        if (!first_round) {
            HIPCHK(c, ops.count(kind, s0, s1, s2, s3, mask, (uint32_t)n, set, valid, counts, c->cur));
            HIPCHK(c, vgpu_launch_scan(counts, offs, cells, tmp, scan_bytes, c->cur));
        }
        first_round = false;
        HIPCHK(c, ops.plan(offs, (uint32_t)nb, W, set, (uint32_t)n, plan, ext, c->cur));
        HIPCHK(c, ops.queue(kind, s0, s1, s2, s3, mask, (uint32_t)n, set, plan, valid, offs, c->st_items, v->base,
                            c->cur));
        HIPCHK(c, ops.children(kind, s0, s1, s2, s3, first, plan, ub, c->st_items, v, bases, valid, c->cur));
    }
    return VGPU_OK;
}

// Chained staged passes over the same groups: the first initialises the flags, the later ones only
// clear them (a group already invalid skips every stage) -- the reference's result is an OR over checks.
static int chain_pass(vgpu_ctx* c, const StagedChain& ch, int kind, const void* s0, const void* s1, const void* s2,
                      const void* s3, uint64_t first, size_t n, const EnvView* v, const float b[3], uint8_t* valid,
                      const float* b2 = nullptr)
{
    for (int p = 0; p < ch.n; ++p)
        if (int rc = staged_pass(c, ch.ops[p], kind, s0, s1, s2, s3, first, n, v, b, valid, p, b2)) return rc;
    return VGPU_OK;
}

// The composite's validity fkcc_A && fkcc_B && !inter (vgpu_pair_staged.hip): arm A, arm B, inter-arm chunks
// (inter-arm chunk 0's bound kernel also stores chunk 1's masks, after its own: vgpu_pair_staged.hip PairInterR,
// so chunk 1 runs without a bound kernel of its own -- both arms' FK once for all 121 inter-arm bounding pairs)
static int pair_staged(vgpu_ctx* c, int kind, const void* s0, const void* s1, const void* s2, const void* s3, size_t n,
                       const EnvView* v, const float pb[6], uint8_t* valid)
{
    const bool both = kPairStaged[2].mask_bytes() == 2 * kPairStaged[3].mask_bytes();
    for (int p = 0; p < 4; ++p) {
        const bool ready = both && p == 3;
        const size_t off = ready ? n * (size_t)kPairStaged[3].mask_bytes() / 4 : 0;
        if (int rc = staged_pass(c, kPairStaged[p], kind, s0, s1, s2, s3, 0, n, v, pb, valid, p, pb + 3, ready, off))
            return rc;
    }
    return VGPU_OK;
}

extern "C" int vgpu_fkcc(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* q, size_t n, uint8_t* valid)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    if (n && (!q || !valid)) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    if ((rc = vgpu_env_upload(e))) return rc;
    const EnvView v = make_view(e);
    HIPCHK(c, ctx_device(c));
    if (const RobotOps* g = generic_ops(r->kind)) {
        if (c->staged && g->staged)
            return chain_pass(c, generic_chain(r->kind), 0, q, nullptr, nullptr, nullptr, 0, n, &v, b, valid);
        HIPCHK(c, g->fkcc(q, n, &v, valid, c->cur));
        return VGPU_OK;
    }
    if (r->kind == VGPU_ROBOT_FETCH) {
        if (c->staged) return staged_pass(c, kFetchStaged, 0, q, nullptr, nullptr, nullptr, 0, n, &v, b, valid);
        HIPCHK(c, vgpu_launch_fetch_fkcc(q, n, &v, valid, c->cur));
        return VGPU_OK;
    }
    if (r->kind == VGPU_ROBOT_PANDA_PAIR) {
        float pb[6];
        pair_bases(r, pb);
        if (c->staged) return pair_staged(c, 0, q, nullptr, nullptr, nullptr, n, &v, pb, valid);
        HIPCHK(c, vgpu_launch_pair_fkcc(q, n, &v, pb, valid, c->cur));
        return VGPU_OK;
    }
    if (c->staged) return staged_pass(c, kPandaStaged, 0, q, nullptr, nullptr, nullptr, 0, n, &v, b, valid);
    HIPCHK(c, vgpu_launch_panda_fkcc(q, n, &v, b[0], b[1], b[2], valid, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_fkcc_attach(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* q, size_t n,
                                uint8_t* valid)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    if (r->kind == VGPU_ROBOT_PANDA_PAIR) return fail(c, VGPU_ERR_UNSUPPORTED, "fkcc_attach: not for the composite");
    if (!e->attached) return fail(c, VGPU_ERR_INVALID_ARG, "fkcc_attach: the environment has no attachment");
    if (n && (!q || !valid)) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    if (r->kind == VGPU_ROBOT_BAXTER) return vgpu_fkcc(c, r, e, q, n, valid);  // Baxter::fkcc_attach = fkcc
    if ((rc = vgpu_env_upload(e))) return rc;
    const EnvView v = make_view(e);
    HIPCHK(c, ctx_device(c));
    if (r->kind == VGPU_ROBOT_FETCH)
        HIPCHK(c, vgpu_launch_fetch_fkcc_attach(q, n, &v, valid, c->cur));
    else if (r->kind == VGPU_ROBOT_UR5)
        HIPCHK(c, vgpu_launch_ur5_fkcc_attach(q, n, &v, valid, c->cur));
    else
        HIPCHK(c, vgpu_launch_panda_fkcc_attach(q, n, &v, b[0], b[1], b[2], valid, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

// The back-step item count of a validate call (cnt[0 .. n_edges) scanned into off): read back once,
// with its 64-bit sum -- the scan and the item indices are 32-bit, so a batch whose rake blocks do not
// fit (very long edges) is rejected before any offset is used.
static int item_total(vgpu_ctx* c, const uint32_t* cnt, const uint32_t* off, size_t n_edges, void* tmp,
                      size_t tmp_bytes, size_t* n_items)
{
    auto* t64 = (unsigned long long*)(((uintptr_t)tmp + tmp_bytes + 7) & ~(uintptr_t)7);
    HIPCHK(c, vgpu_launch_total64(cnt, n_edges, t64, c->cur));
    HIPCHK(c, hipMemcpyAsync(c->total_host, off + n_edges, sizeof(uint32_t), hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipMemcpyAsync(c->total_host + 2, t64, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    unsigned long long total = 0;
    std::memcpy(&total, c->total_host + 2, sizeof(total));
    if (total != (unsigned long long)c->total_host[0] || total + n_edges >= (1ull << 32))
        return fail(c, VGPU_ERR_INVALID_ARG, "edges too long: more than 2^32 rake blocks in one call (split the batch)");
    *n_items = (size_t)total;
    return VGPU_OK;
}

static int ensure_ws(vgpu_ctx* c, size_t n_edges, uint32_t** cnt, uint32_t** off, void** tmp, size_t* tmp_bytes)
{
    const size_t idx_bytes = ((n_edges + 1) * sizeof(uint32_t) + 255) & ~(size_t)255;
    *tmp_bytes = vgpu_validate_scan_bytes(n_edges);
    const size_t need = 2 * idx_bytes + *tmp_bytes + 256;
    if (need > c->ws_bytes) {
        if (c->ws) {
            HIPCHK(c, hipStreamSynchronize(c->cur));
            HIPCHK(c, hipFree(c->ws));
            c->ws = nullptr;
        }
        HIPCHK(c, hipMalloc(&c->ws, need));
        c->ws_bytes = need;
    }
    if (!c->total_host) HIPCHK(c, hipHostMalloc((void**)&c->total_host, 4 * sizeof(uint32_t), hipHostMallocDefault));
    char* p = (char*)c->ws;
    *cnt = (uint32_t*)p;
    *off = (uint32_t*)(p + idx_bytes);
    *tmp = p + 2 * idx_bytes;
    return VGPU_OK;
}

extern "C" int vgpu_validate_motions(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* starts,
                                     const float* goals, size_t n_edges, uint8_t* ok, int32_t* n_blocks)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    if (n_edges == 0) return VGPU_OK;
    if (!starts || !goals || !ok) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    if (n_edges >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "too many edges in one call (< 2^31)");
    // validate.hh:43: with an attachment the first block goes through fkcc_attach; the Baxter's
    // fkcc_attach is its plain fkcc (baxter.hh:44), so its attachment changes nothing
    const bool att = e->attached && r->kind != VGPU_ROBOT_BAXTER;
    if (att && r->kind == VGPU_ROBOT_PANDA_PAIR)
        return fail(c, VGPU_ERR_UNSUPPORTED, "attachments: no fkcc_attach for the composite");
    if ((rc = vgpu_env_upload(e))) return rc;
    const EnvView v = make_view(e);
    HIPCHK(c, ctx_device(c));
    uint32_t *cnt, *off;
    void* tmp;
    size_t tmp_bytes;
    if ((rc = ensure_ws(c, n_edges, &cnt, &off, &tmp, &tmp_bytes))) return rc;
    const bool pair_staged_path = r->kind == VGPU_ROBOT_PANDA_PAIR && c->staged;  // chained staged passes
    const bool pair = r->kind == VGPU_ROBOT_PANDA_PAIR && !c->staged;             // monolithic head/tail kernels
    const bool fetch = r->kind == VGPU_ROBOT_FETCH && !c->staged;
    const RobotOps* g = generic_ops(r->kind);
    const bool g_mono = g && !(c->staged && g->staged);
    const StagedChain chain = g ? (g->staged ? generic_chain(r->kind) : StagedChain{&kPandaStaged, 1})
                                : StagedChain{r->kind == VGPU_ROBOT_FETCH ? &kFetchStaged : &kPandaStaged, 1};
    float pb[6];
    pair_bases(r, pb);
    if (c->prof) HIPCHK(c, hipEventRecord(c->ev[0], c->cur));
    if (att) {
        if (r->kind == VGPU_ROBOT_FETCH)
            HIPCHK(c, vgpu_launch_fetch_validate_head_att(starts, goals, n_edges, &v, ok, n_blocks, cnt, c->cur));
        else if (r->kind == VGPU_ROBOT_UR5)
            HIPCHK(c, vgpu_launch_ur5_validate_head_att(starts, goals, n_edges, &v, ok, n_blocks, cnt, c->cur));
        else
            HIPCHK(c, vgpu_launch_panda_validate_head_att(starts, goals, n_edges, &v, b[0], b[1], b[2], ok, n_blocks,
                                                          cnt, c->cur));
    } else if (g_mono) {
        HIPCHK(c, g->validate_head(starts, goals, n_edges, &v, ok, n_blocks, cnt, c->cur));
    } else if (pair_staged_path) {
        if ((rc = pair_staged(c, 2, starts, goals, nullptr, nullptr, n_edges, &v, pb, ok))) return rc;
        HIPCHK(c, vgpu_launch_pair_tail_counts(starts, goals, n_edges, ok, n_blocks, cnt, c->cur));
    } else if (pair) {
        HIPCHK(c, vgpu_launch_pair_validate_head(starts, goals, n_edges, &v, pb, ok, n_blocks, cnt, c->cur));
    } else if (fetch) {
        HIPCHK(c, vgpu_launch_fetch_validate_head(starts, goals, n_edges, &v, ok, n_blocks, cnt, c->cur));
    } else if (c->staged) {
        if ((rc = chain_pass(c, chain, 2, starts, goals, nullptr, nullptr, 0, n_edges, &v, b, ok))) return rc;
        if (g)
            HIPCHK(c, g->tail_counts(starts, goals, n_edges, ok, n_blocks, cnt, c->cur));
        else if (r->kind == VGPU_ROBOT_FETCH)
            HIPCHK(c, vgpu_launch_fetch_tail_counts(starts, goals, n_edges, ok, n_blocks, cnt, c->cur));
        else
            HIPCHK(c, vgpu_launch_tail_counts(starts, goals, n_edges, ok, n_blocks, cnt, c->cur));
    } else {
        HIPCHK(c, vgpu_launch_panda_validate_head(starts, goals, n_edges, &v, b[0], b[1], b[2], ok, n_blocks, cnt,
                                                  c->cur));
    }
    if (c->prof) HIPCHK(c, hipEventRecord(c->ev[1], c->cur));
    HIPCHK(c, vgpu_launch_scan(cnt, off, n_edges, tmp, tmp_bytes, c->cur));
    // number of back-step work items: one read-back (the item buffer is sized from it)
    size_t n_items = 0;
    if ((rc = item_total(c, cnt, off, n_edges, tmp, tmp_bytes, &n_items))) return rc;
    if (n_items > c->items_cap) {
        if (c->items) HIPCHK(c, hipFree(c->items));
        c->items = nullptr;
        const size_t cap = std::max(n_items, (size_t)1 << 20);
        HIPCHK(c, hipMalloc(&c->items, cap * sizeof(uint32_t)));
        c->items_cap = cap;
    }
    if (c->prof) HIPCHK(c, hipEventRecord(c->ev[2], c->cur));
    if (fetch || pair || g_mono) {
        if (n_items) {
            HIPCHK(c, vgpu_launch_scatter_items(cnt, off, n_edges, c->items, c->cur));
            if (g_mono)
                HIPCHK(c, g->validate_tail(starts, goals, n_items, &v, ok, off, c->items, c->cur));
            else if (pair)
                HIPCHK(c, vgpu_launch_pair_validate_tail(starts, goals, n_items, &v, pb, ok, off, c->items, c->cur));
            else
                HIPCHK(c, vgpu_launch_fetch_validate_tail(starts, goals, n_items, &v, ok, off, c->items, c->cur));
        }
    } else if (pair_staged_path) {
        if (n_items) {
            HIPCHK(c, vgpu_launch_scatter_items(cnt, off, n_edges, c->items, c->cur));
            if ((rc = pair_staged(c, 3, starts, goals, c->items, off, n_items, &v, pb, ok))) return rc;
        }
    } else if (c->staged) {
        if (n_items) {
            HIPCHK(c, vgpu_launch_scatter_items(cnt, off, n_edges, c->items, c->cur));
            if ((rc = chain_pass(c, chain, 3, starts, goals, c->items, off, 0, n_items, &v, b, ok))) return rc;
        }
    } else {
        HIPCHK(c, vgpu_launch_panda_validate_tail(starts, goals, n_edges, n_items, &v, b[0], b[1], b[2], ok, cnt,
                                                  off, c->items, c->cur));
    }
    if (c->prof) {
        HIPCHK(c, hipEventRecord(c->ev[3], c->cur));
        HIPCHK(c, hipEventSynchronize(c->ev[3]));
        float t0 = 0, t1 = 0, t2 = 0;
        HIPCHK(c, hipEventElapsedTime(&t0, c->ev[0], c->ev[1]));
        HIPCHK(c, hipEventElapsedTime(&t1, c->ev[1], c->ev[2]));
        HIPCHK(c, hipEventElapsedTime(&t2, c->ev[2], c->ev[3]));
        c->acc[0] += t0;  // head kernel (one memset + panda_validate_head_kernel)
        c->acc[1] += t1;  // scan + the 4-byte D2H of the item count
        c->acc[2] += t2;  // scatter + panda_validate_tail_kernel
        c->acc[3] += 1.0f;
    }
    return VGPU_OK;
} VGPU_ABI_CATCH

// Full-mask mode (SURVEY §8(d) "full-mask: every interpolant evaluated"): every rake block of every
// edge is evaluated -- no early exit across an edge's blocks -- and each block's result is kept.
extern "C" int vgpu_validate_motions_mask(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* starts,
                                          const float* goals, size_t n_edges, uint8_t* ok, int32_t* n_blocks,
                                          uint8_t* block_ok, size_t block_cap, size_t* n_total)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    if (n_total) *n_total = 0;
    if (n_edges == 0) return VGPU_OK;
    if (!starts || !goals || !ok || !n_total) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    if (r->kind != VGPU_ROBOT_PANDA || !c->staged)
        return fail(c, VGPU_ERR_UNSUPPORTED, "full-mask validate: Panda (staged pipeline) only");
    if (e->attached) return fail(c, VGPU_ERR_UNSUPPORTED, "full-mask validate: no attachments");
    if (n_edges >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "too many edges in one call (< 2^31)");
    if ((rc = vgpu_env_upload(e))) return rc;
    const EnvView v = make_view(e);
    HIPCHK(c, ctx_device(c));
    uint32_t *cnt, *off;
    void* tmp;
    size_t tmp_bytes;
    if ((rc = ensure_ws(c, n_edges, &cnt, &off, &tmp, &tmp_bytes))) return rc;
    if ((rc = staged_pass(c, kPandaStaged, 2, starts, goals, nullptr, nullptr, 0, n_edges, &v, b, ok))) return rc;
    HIPCHK(c, vgpu_launch_tail_counts(starts, goals, n_edges, nullptr, n_blocks, cnt, c->cur));  // every back-step
    HIPCHK(c, vgpu_launch_scan(cnt, off, n_edges, tmp, tmp_bytes, c->cur));
    size_t n_items = 0;
    if ((rc = item_total(c, cnt, off, n_edges, tmp, tmp_bytes, &n_items))) return rc;
    *n_total = n_items + n_edges;
    if (!block_ok || block_cap < *n_total)
        return fail(c, VGPU_ERR_INVALID_ARG, "block_ok capacity < total blocks (*n_total)");
    if (n_items > c->items_cap) {
        if (c->items) HIPCHK(c, hipFree(c->items));
        c->items = nullptr;
        const size_t cap = std::max(n_items, (size_t)1 << 20);
        HIPCHK(c, hipMalloc(&c->items, cap * sizeof(uint32_t)));
        c->items_cap = cap;
    }
    if (n_items) {
        HIPCHK(c, vgpu_launch_scatter_items(cnt, off, n_edges, c->items, c->cur));
        if ((rc = staged_pass(c, kPandaStaged, 4, starts, goals, c->items, off, 0, n_items, &v, b, block_ok))) return rc;
    }
    HIPCHK(c, vgpu_launch_mask_finish(n_edges, off, ok, block_ok, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

// CAPT::collides (simd = 0, capt.hh:403-443) or one lane of CAPT::collides_simd (simd = 1,
// capt.hh:457-541) for n raw spheres against point cloud `index` of the environment.
extern "C" int vgpu_pointcloud_collides(vgpu_ctx* c, vgpu_env* e, int index, const float* centers,
                                        const float* radii, size_t n, int simd, uint8_t* out)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    if (index < 0 || (size_t)index >= e->pointclouds.size()) return fail(c, VGPU_ERR_INVALID_ARG, "bad index");
    if (n == 0) return VGPU_OK;
    if (!centers || !radii || !out) return fail(c, VGPU_ERR_INVALID_ARG, "null buffer");
    int rc = vgpu_env_upload(e);
    if (rc) return rc;
    const EnvView v = make_view(e);
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, vgpu_launch_capt_query(centers, radii, n, &v, index, simd, out, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

// filter_pointcloud (collision/filter.hh:175-268) on the device (vgpu_filter.hip)
extern "C" int vgpu_filter_pointcloud(vgpu_ctx* c, const float* pc, size_t n, float min_dist, float max_range,
                                      const float origin[3], const float ws_min[3], const float ws_max[3], int cull,
                                      uint32_t* out_idx, size_t* count)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (!count || !origin || !ws_min || !ws_max) return fail(c, VGPU_ERR_INVALID_ARG, "null argument");
    *count = 0;
    if (n == 0) return VGPU_OK;
    if (!pc || !out_idx || n > 0x7fffffffu) return fail(c, VGPU_ERR_INVALID_ARG, "bad filter_pointcloud arguments");
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, vgpu_filter_pointcloud_run(pc, n, min_dist, max_range, origin, ws_min, ws_max, cull, out_idx, count,
                                         c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

// filter_robot_from_pointcloud<Robot> (bindings/common.hh:36-87): sphere_fk<1> of the configuration
// (the robot's own sphere_fk kernel on one row), then one lane per point (vgpu_query.hip)
static const float* sphere_radii(int32_t kind, int* S)
{
    switch (kind) {
    case VGPU_ROBOT_PANDA: *S = panda_n_spheres_table; return panda_sphere_radii;
    case VGPU_ROBOT_FETCH: *S = fetch_n_spheres_table; return fetch_sphere_radii;
    case VGPU_ROBOT_UR5: *S = ur5_n_spheres_table; return ur5_sphere_radii;
    case VGPU_ROBOT_BAXTER: *S = baxter_n_spheres_table; return baxter_sphere_radii;
    default: *S = 0; return nullptr;
    }
}

extern "C" int vgpu_filter_robot_pointcloud(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* configuration,
                                            const float* pc, size_t n, float point_radius, uint8_t* keep)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    int S = 0;
    const float* radii = sphere_radii(r->kind, &S);
    if (!radii) return fail(c, VGPU_ERR_UNSUPPORTED, "filter_from_pointcloud: Panda, Fetch, UR5, Baxter");
    if (!configuration) return fail(c, VGPU_ERR_INVALID_ARG, "null configuration");
    if (n == 0) return VGPU_OK;
    if (!pc || !keep) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    if ((rc = vgpu_env_upload(e))) return rc;
    const EnvView v = make_view(e);
    HIPCHK(c, ctx_device(c));
    constexpr int kSmallFloats = 16 + 4 * 128;
    if (!c->small) HIPCHK(c, hipMalloc((void**)&c->small, kSmallFloats * sizeof(float)));
    // [0, 16) configuration, [16, 16 + 3S) sphere_fk centres (ld = 1), then the radii
    float host[kSmallFloats] = {};
    const int dim = (int)dim_of(r);
    std::memcpy(host, configuration, (size_t)dim * sizeof(float));
    std::memcpy(host + 16 + 3 * S, radii, (size_t)S * sizeof(float));
    HIPCHK(c, hipMemcpyAsync(c->small, host, kSmallFloats * sizeof(float), hipMemcpyHostToDevice, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));  // host is a stack buffer
    if ((rc = vgpu_sphere_fk(c, r, c->small, 1, c->small + 16, 1))) return rc;
    HIPCHK(c, vgpu_launch_filter_robot(pc, n, point_radius, c->small + 16, S, &v, keep, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

// ---- sampling (rng::Halton, Robot::scale_configuration) and compaction --------------------------
extern "C" int vgpu_halton(vgpu_ctx* c, int dim, uint64_t first, size_t n, float* out)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (dim < 1 || dim > 16 || first == 0) return fail(c, VGPU_ERR_INVALID_ARG, "dim must be 1..16, first >= 1");
    if (n == 0) return VGPU_OK;
    if (!out) return fail(c, VGPU_ERR_INVALID_ARG, "null buffer");
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, vgpu_launch_halton(dim, first, n, out, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_sample_configurations(vgpu_ctx* c, const vgpu_robot* r, uint64_t first, size_t n, float* q)
try {
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    if (first == 0) return fail(c, VGPU_ERR_INVALID_ARG, "draw indices start at 1");
    if (n == 0) return VGPU_OK;
    if (!q) return fail(c, VGPU_ERR_INVALID_ARG, "null buffer");
    HIPCHK(c, ctx_device(c));
    if (r->kind == VGPU_ROBOT_PANDA_PAIR) return fail(c, VGPU_ERR_UNSUPPORTED, "no sampler for the composite");
    if (const RobotOps* g = generic_ops(r->kind))
        HIPCHK(c, g->sample(first, n, q, c->cur));
    else if (r->kind == VGPU_ROBOT_FETCH)
        HIPCHK(c, vgpu_launch_fetch_sample(first, n, q, c->cur));
    else
        HIPCHK(c, vgpu_launch_panda_sample(first, n, q, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_sample_fkcc(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, uint64_t first, size_t n, float* q,
                                uint8_t* valid)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    float b[3];
    int rc = check_robot(c, r, b);
    if (rc) return rc;
    if (first == 0) return fail(c, VGPU_ERR_INVALID_ARG, "draw indices start at 1");
    if (n == 0) return VGPU_OK;
    if (!valid) return fail(c, VGPU_ERR_INVALID_ARG, "null buffer");
    if ((rc = vgpu_env_upload(e))) return rc;
    const EnvView v = make_view(e);
    HIPCHK(c, ctx_device(c));
    if (r->kind == VGPU_ROBOT_PANDA_PAIR) return fail(c, VGPU_ERR_UNSUPPORTED, "no sampler for the composite");
    if (c->staged && !q) {  // the children stage reads the bound stage's samples back
        int32_t dim = 0;
        vgpu_robot_info(r->kind, &dim, nullptr, nullptr);
        if ((rc = grow(c, &c->st_q, &c->st_q_cap, n * (size_t)dim))) return rc;
        q = (float*)c->st_q;
    }
    if (const RobotOps* g = generic_ops(r->kind)) {
        if (c->staged && g->staged)
            return chain_pass(c, generic_chain(r->kind), 1, q, nullptr, nullptr, nullptr, first, n, &v, b, valid);
        HIPCHK(c, g->sample_fkcc(first, n, &v, q, valid, c->cur));
        return VGPU_OK;
    }
    if (r->kind == VGPU_ROBOT_FETCH) {
        if (c->staged) return staged_pass(c, kFetchStaged, 1, q, nullptr, nullptr, nullptr, first, n, &v, b, valid);
        HIPCHK(c, vgpu_launch_fetch_sample_fkcc(first, n, &v, q, valid, c->cur));
        return VGPU_OK;
    }
    if (c->staged) return staged_pass(c, kPandaStaged, 1, q, nullptr, nullptr, nullptr, first, n, &v, b, valid);
    HIPCHK(c, vgpu_launch_panda_sample_fkcc(first, n, &v, b[0], b[1], b[2], q, valid, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_compact(vgpu_ctx* c, const float* rows, const uint8_t* valid, size_t n, int dim, float* rows_out,
                            uint32_t* index_out, size_t* count)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (dim < 1 || !count || n >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "bad compaction args");
    *count = 0;
    if (n == 0) return VGPU_OK;
    if (!valid || !index_out || (rows_out && !rows)) return fail(c, VGPU_ERR_INVALID_ARG, "null buffer");
    const size_t tmp = vgpu_compact_bytes(n);
    const size_t need = 256 + tmp;
    HIPCHK(c, ctx_device(c));
    if (need > c->aux_bytes) {
        if (c->aux) {
            HIPCHK(c, hipStreamSynchronize(c->cur));
            HIPCHK(c, hipFree(c->aux));
            c->aux = nullptr;
        }
        HIPCHK(c, hipMalloc(&c->aux, need));
        c->aux_bytes = need;
    }
    if (!c->total_host) HIPCHK(c, hipHostMalloc((void**)&c->total_host, 4 * sizeof(uint32_t), hipHostMallocDefault));
    uint32_t* cnt = (uint32_t*)c->aux;
    HIPCHK(c, vgpu_launch_compact(valid, n, index_out, cnt, (char*)c->aux + 256, tmp, c->cur));
    if (rows_out) HIPCHK(c, vgpu_launch_gather_rows(rows, index_out, cnt, n, dim, rows_out, c->cur));
    HIPCHK(c, hipMemcpyAsync(c->total_host, cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    *count = *c->total_host;
    return VGPU_OK;
} VGPU_ABI_CATCH

// ---- host conveniences ------------------------------------------------------------------
// Also makes the context's device current for the calling thread: the staging buffer and everything the
// *_host entry point enqueues after it belong to that device (HIP's current device is per thread).
static int stage(vgpu_ctx* c, size_t bytes, char** p)
{
    HIPCHK(c, ctx_device(c));
    if (bytes > c->stage_bytes) {
        if (c->stage) {
            HIPCHK(c, hipStreamSynchronize(c->cur));
            HIPCHK(c, hipFree(c->stage));
            c->stage = nullptr;
        }
        HIPCHK(c, hipMalloc(&c->stage, bytes));
        c->stage_bytes = bytes;
    }
    *p = (char*)c->stage;
    return VGPU_OK;
}

static size_t al(size_t b) { return (b + 255) & ~(size_t)255; }

// configuration width and sphere count of a robot selection (host staging sizes)
static size_t dim_of(const vgpu_robot* r)
{
    if (r)
        if (const RobotOps* g = generic_ops(r->kind)) return (size_t)g->dim;
    if (r && r->kind == VGPU_ROBOT_FETCH) return kFetchDim;
    if (r && r->kind == VGPU_ROBOT_PANDA_PAIR) return kPairDim;
    return kPandaDim;
}
static size_t spheres_of(const vgpu_robot* r)
{
    if (r)
        if (const RobotOps* g = generic_ops(r->kind)) return (size_t)g->n_spheres;
    return (r && r->kind == VGPU_ROBOT_FETCH) ? kFetchSpheres : kPandaSpheres;
}

extern "C" int vgpu_sphere_fk_host(vgpu_ctx* c, const vgpu_robot* r, const float* q, size_t n, float* xyz)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n == 0) return VGPU_OK;
    char* d;
    const size_t qb = al(n * dim_of(r) * 4), ob = (size_t)3 * spheres_of(r) * n * 4;
    int rc = stage(c, qb + ob, &d);
    if (rc) return rc;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipMemcpyAsync(d, q, n * dim_of(r) * 4, hipMemcpyHostToDevice, c->cur));
    if ((rc = vgpu_sphere_fk(c, r, (const float*)d, n, (float*)(d + qb), n))) return rc;
    HIPCHK(c, hipMemcpyAsync(xyz, d + qb, ob, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_fkcc_host(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* q, size_t n,
                              uint8_t* valid)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n == 0) return VGPU_OK;
    char* d;
    const size_t qb = al(n * dim_of(r) * 4);
    int rc = stage(c, qb + n, &d);
    if (rc) return rc;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipMemcpyAsync(d, q, n * dim_of(r) * 4, hipMemcpyHostToDevice, c->cur));
    if ((rc = vgpu_fkcc(c, r, e, (const float*)d, n, (uint8_t*)(d + qb)))) return rc;
    HIPCHK(c, hipMemcpyAsync(valid, d + qb, n, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_fkcc_attach_host(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* q, size_t n,
                                     uint8_t* valid)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n == 0) return VGPU_OK;
    char* d;
    const size_t qb = al(n * dim_of(r) * 4);
    int rc = stage(c, qb + n, &d);
    if (rc) return rc;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipMemcpyAsync(d, q, n * dim_of(r) * 4, hipMemcpyHostToDevice, c->cur));
    if ((rc = vgpu_fkcc_attach(c, r, e, (const float*)d, n, (uint8_t*)(d + qb)))) return rc;
    HIPCHK(c, hipMemcpyAsync(valid, d + qb, n, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_validate_motions_host(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, const float* starts,
                                          const float* goals, size_t n, uint8_t* ok, int32_t* n_blocks)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n == 0) return VGPU_OK;
    char* d;
    const size_t qb = al(n * dim_of(r) * 4);
    const size_t okb = al(n), nbb = al(n * 4);
    int rc = stage(c, 2 * qb + okb + nbb, &d);
    if (rc) return rc;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipMemcpyAsync(d, starts, n * dim_of(r) * 4, hipMemcpyHostToDevice, c->cur));
    HIPCHK(c, hipMemcpyAsync(d + qb, goals, n * dim_of(r) * 4, hipMemcpyHostToDevice, c->cur));
    uint8_t* okd = (uint8_t*)(d + 2 * qb);
    int32_t* nbd = (int32_t*)(d + 2 * qb + okb);
    if ((rc = vgpu_validate_motions(c, r, e, (const float*)d, (const float*)(d + qb), n, okd, nbd))) return rc;
    HIPCHK(c, hipMemcpyAsync(ok, okd, n, hipMemcpyDeviceToHost, c->cur));
    if (n_blocks) HIPCHK(c, hipMemcpyAsync(n_blocks, nbd, n * 4, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_filter_pointcloud_host(vgpu_ctx* c, const float* pc, size_t n, float min_dist, float max_range,
                                           const float origin[3], const float ws_min[3], const float ws_max[3],
                                           int cull, uint32_t* out_idx, size_t* count)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (!count) return fail(c, VGPU_ERR_INVALID_ARG, "null count");
    *count = 0;
    if (n == 0) return VGPU_OK;
    if (!pc || !out_idx) return fail(c, VGPU_ERR_INVALID_ARG, "null buffer");
    char* d;
    const size_t pb = al(n * 12);
    int rc = stage(c, pb + n * 4, &d);
    if (rc) return rc;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipMemcpyAsync(d, pc, n * 12, hipMemcpyHostToDevice, c->cur));
    if ((rc = vgpu_filter_pointcloud(c, (const float*)d, n, min_dist, max_range, origin, ws_min, ws_max, cull,
                                     (uint32_t*)(d + pb), count)))
        return rc;
    HIPCHK(c, hipMemcpyAsync(out_idx, d + pb, *count * 4, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_pointcloud_collides_host(vgpu_ctx* c, vgpu_env* e, int index, const float* centers,
                                             const float* radii, size_t n, int simd, uint8_t* out)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n == 0) return VGPU_OK;
    char* d;
    const size_t cb = al(n * 12), rb = al(n * 4);
    int rc = stage(c, cb + rb + n, &d);
    if (rc) return rc;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipMemcpyAsync(d, centers, n * 12, hipMemcpyHostToDevice, c->cur));
    HIPCHK(c, hipMemcpyAsync(d + cb, radii, n * 4, hipMemcpyHostToDevice, c->cur));
    if ((rc = vgpu_pointcloud_collides(c, e, index, (const float*)d, (const float*)(d + cb), n, simd,
                                       (uint8_t*)(d + cb + rb))))
        return rc;
    HIPCHK(c, hipMemcpyAsync(out, d + cb + rb, n, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_halton_host(vgpu_ctx* c, int dim, uint64_t first, size_t n, float* out)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n == 0) return VGPU_OK;
    char* d;
    int rc = stage(c, n * (size_t)dim * 4, &d);
    if (rc) return rc;
    if ((rc = vgpu_halton(c, dim, first, n, (float*)d))) return rc;
    HIPCHK(c, hipMemcpyAsync(out, d, n * (size_t)dim * 4, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_sample_fkcc_host(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e, uint64_t first, size_t n,
                                     float* q, uint8_t* valid)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n == 0) return VGPU_OK;
    char* d;
    const size_t qb = al(n * dim_of(r) * 4);
    int rc = stage(c, qb + n, &d);
    if (rc) return rc;
    if ((rc = vgpu_sample_fkcc(c, r, e, first, n, q ? (float*)d : nullptr, (uint8_t*)(d + qb)))) return rc;
    if (q) HIPCHK(c, hipMemcpyAsync(q, d, n * dim_of(r) * 4, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipMemcpyAsync(valid, d + qb, n, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

// ---------------------------------------------------------------------------------------
// PRM roadmap edge stage (planning/prm.hh:235-299; vgpu_roadmap.hip)
// ---------------------------------------------------------------------------------------
extern "C" size_t vgpu_knn_chunks(size_t n, uint32_t* S);
extern "C" hipError_t vgpu_launch_roadmap_knn(int dim, const float* V, uint32_t n, uint32_t q_first, uint32_t q_count,
                                              const uint32_t* k, const float* r, uint32_t kmax, uint32_t S,
                                              uint32_t C, float* pd, uint32_t* pi, uint32_t* pc, uint32_t* nbr,
                                              float* dist, uint32_t* cnt, hipStream_t st);
extern "C" hipError_t vgpu_launch_edge_gather(const float* V, uint32_t q_first, uint32_t q_count, int dim,
                                              const uint32_t* nbr, uint32_t kmax, const uint32_t* cnt,
                                              const uint32_t* off, float* starts, float* goals, hipStream_t st);

// PRMStarNeighborParams (roadmap.hh:42-77) for roadmap sizes 0 .. n-1, in double as the reference
extern "C" int vgpu_prm_neighbor_params(int dim, double space_measure, double gamma_scale, size_t n, uint32_t* k,
                                        float* r)
try {
    if (dim <= 0 || (n && (!k || !r))) return VGPU_ERR_INVALID_ARG;
    const double E = 2.718281828459045235360287471352662498;  // constants.hh:6
    const double PI = 3.141592653589793238462643383279502884;
    const double kc = E + (E / (double)dim);
    const double inv = 1.0 / (double)dim;
    const double ball = std::pow(std::sqrt(PI), (double)dim) / std::tgamma((double)dim / 2.0 + 1.0);
    const double prm = 2.0 * std::pow(1.0 + inv, inv) * std::pow(space_measure / ball, inv);
    auto fill = [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            if (i < 2) {  // start and goal are inserted without a query (prm.hh:228-233)
                k[i] = 0;
                r[i] = 0.0f;
                continue;
            }
            const double li = std::log((double)i);
            const double d = kc * li;
            const size_t s = (size_t)d;  // c_ceil (utils.hh:28-32)
            const size_t kk = d > (double)s ? s + 1 : s;
            k[i] = (uint32_t)std::min<size_t>(kk, 0xFFFFFFFFu);
            r[i] = (float)(gamma_scale * prm * std::pow(li / (double)i, inv));
        }
    };
    // each entry depends on i alone: large tables are filled by up to 16 host threads (a log and a pow per
    // entry, ~60 ns: 0.15 s single-threaded for the 2.68M-vertex roadmap), same values
    const size_t nt = n < 65536 ? 1 : std::min<size_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (nt == 1) {
        fill(0, n);
        return VGPU_OK;
    }
    // a thread that cannot be started (std::system_error) leaves its range and every later one to this thread:
    // no exception crosses the C ABI, and the table is complete either way
    std::vector<std::thread> th;
    size_t done = 0;  // ranges [0, done) have a thread
    try {
        th.reserve(nt);
        for (; done < nt; ++done) th.emplace_back(fill, n * done / nt, n * (done + 1) / nt);
    } catch (...) {
    }
    fill(n * done / nt, n);
    for (auto& x : th) x.join();
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" size_t vgpu_knn_index_bytes(int dim, uint32_t n, uint32_t q_count);
extern "C" hipError_t vgpu_launch_knn_index(int dim, const float* V, uint32_t n, uint32_t q_first, uint32_t q_count,
                                            const uint32_t* k, const float* r, uint32_t kmax, uint32_t* nbr,
                                            float* dist, uint32_t* cnt, void* pool, size_t pool_bytes, uint32_t* dbg,
                                            hipStream_t st);

static bool knn_dim_ok(int dim) { return dim == 6 || dim == 7 || dim == 8 || dim == 14; }

// below this many vertices the brute-force scan is faster (MI355X, Fetch Halton vertices,
// tools/knn_scale.py: 100k brute 11.8 / index 18.3 ms, 400k 95 / 104 ms, 2.7M index 1.40 s vs
// ~4.3 s extrapolated brute)
static constexpr size_t kKnnIndexMin = 65536;  // group-query index: 3.6 vs 11.8 ms (brute) at 100k Fetch vertices

extern "C" int vgpu_set_knn_mode(vgpu_ctx* c, int mode)
try {
    if (!c || mode < 0 || mode > 2) return VGPU_ERR_INVALID_ARG;
    c->knn_mode = mode;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_roadmap_knn_range(vgpu_ctx* c, int dim, const float* V, size_t n, size_t q_first, size_t q_count,
                                      const uint32_t* k, const float* r, uint32_t kmax, uint32_t* nbr, float* dist,
                                      uint32_t* cnt)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (q_first > n || q_count > n - q_first) return fail(c, VGPU_ERR_INVALID_ARG, "query range outside the vertices");
    if (!knn_dim_ok(dim)) return fail(c, VGPU_ERR_UNSUPPORTED, "roadmap kNN: dimension 6, 7, 8 or 14");
    if (kmax == 0 || kmax > 64) return fail(c, VGPU_ERR_UNSUPPORTED, "roadmap kNN: 1 <= kmax <= 64");
    if (n >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "too many vertices");
    if (n && (!V || !k || !r || !nbr || !dist || !cnt)) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    HIPCHK(c, ctx_device(c));
    if (q_count == 0) return VGPU_OK;
    int rc;
    const bool index = c->knn_mode == 2 || (c->knn_mode == 0 && n >= kKnnIndexMin);
    if (index) {
        const size_t bytes = vgpu_knn_index_bytes(dim, (uint32_t)n, (uint32_t)q_count);
        if (!bytes) return fail(c, VGPU_ERR_HIP, "roadmap kNN index: scratch size query failed");
        if ((rc = grow(c, &c->knn_idx, &c->knn_idx_cap, (bytes + 3) / 4))) return rc;
        HIPCHK(c, vgpu_launch_knn_index(dim, V, (uint32_t)n, (uint32_t)q_first, (uint32_t)q_count, k, r, kmax, nbr,
                                        dist, cnt, c->knn_idx, c->knn_idx_cap * 4, c->dbg, c->cur));
        return VGPU_OK;
    }
    uint32_t S = 0;
    const size_t C = vgpu_knn_chunks(n, &S);
    // chunk lists (context-owned, grown on demand): distances, indices, counts
    const size_t cells = q_count * C, need = cells * (2 * (size_t)kmax + 1);
    if ((rc = grow(c, &c->knn_part, &c->knn_part_cap, need))) return rc;
    float* pd = (float*)c->knn_part;
    uint32_t* pi = c->knn_part + cells * kmax;
    uint32_t* pc = c->knn_part + 2 * cells * kmax;
    HIPCHK(c, vgpu_launch_roadmap_knn(dim, V, (uint32_t)n, (uint32_t)q_first, (uint32_t)q_count, k, r, kmax, S,
                                      (uint32_t)C, pd, pi, pc, nbr, dist, cnt, c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_roadmap_knn(vgpu_ctx* c, int dim, const float* V, size_t n, const uint32_t* k, const float* r,
                                uint32_t kmax, uint32_t* nbr, float* dist, uint32_t* cnt)
try {
    return vgpu_roadmap_knn_range(c, dim, V, n, 0, n, k, r, kmax, nbr, dist, cnt);
} VGPU_ABI_CATCH

extern "C" int vgpu_roadmap_edge_gather(vgpu_ctx* c, int dim, const float* V, size_t q_first, size_t q_count,
                                        const uint32_t* nbr, uint32_t kmax, const uint32_t* cnt, const uint32_t* off,
                                        float* starts, float* goals)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (q_count && (!V || !nbr || !cnt || !off || !starts || !goals))
        return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, vgpu_launch_edge_gather(V, (uint32_t)q_first, (uint32_t)q_count, dim, nbr, kmax, cnt, off, starts, goals,
                                      c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH

namespace {
struct DevBufs {  // call-scoped device allocations
    std::vector<void*> p;
    ~DevBufs()
    {
        for (void* q : p) (void)hipFree(q);
    }
    template <class T>
    hipError_t get(T** out, size_t count)
    {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) p.push_back(q);
        *out = (T*)q;
        return e;
    }
};
}  // namespace

// Roadmap adjacency in build_roadmap's append order (prm.hh:270-275): when vertex i is inserted
// it gets its valid neighbours nearest first and each neighbour j < i gets i appended.  Replaying
// the valid pairs in query order therefore reproduces every list: a vertex's own neighbours,
// then the later vertices that connected to it, ascending.  Union-find for the components.
extern "C" int vgpu_roadmap_assemble(size_t n, const uint32_t* pairs, size_t m, size_t* offsets, uint32_t* adj,
                                     uint32_t* component)
try {
    if (!offsets || (m && (!pairs || !adj))) return VGPU_ERR_INVALID_ARG;
    for (size_t p = 0; p < 2 * m; ++p)
        if (pairs[p] >= n) return VGPU_ERR_INVALID_ARG;
    std::vector<size_t> fill(n + 1, 0);
    for (size_t p = 0; p < 2 * m; ++p) ++fill[pairs[p] + 1];
    offsets[0] = 0;
    for (size_t i = 0; i < n; ++i) offsets[i + 1] = offsets[i] + fill[i + 1];
    std::copy(offsets, offsets + n, fill.begin());
    for (size_t p = 0; p < m; ++p) {
        const uint32_t i = pairs[2 * p], j = pairs[2 * p + 1];
        adj[fill[i]++] = j;
        adj[fill[j]++] = i;
    }
    if (component) {  // each vertex's component = its smallest vertex index
        std::vector<uint32_t> parent(n);
        for (size_t i = 0; i < n; ++i) parent[i] = (uint32_t)i;
        auto find = [&](uint32_t a) {
            while (parent[a] != a) a = parent[a] = parent[parent[a]];
            return a;
        };
        for (size_t p = 0; p < m; ++p) {
            const uint32_t a = find(pairs[2 * p]), b = find(pairs[2 * p + 1]);
            if (a != b) parent[std::max(a, b)] = std::min(a, b);
        }
        for (size_t i = 0; i < n; ++i) component[i] = find((uint32_t)i);
    }
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" size_t vgpu_roadmap_assemble_bytes(uint32_t n, size_t m);
extern "C" hipError_t vgpu_launch_roadmap_assemble(uint32_t n, const uint32_t* pairs, size_t m, unsigned long long* offsets,
                                                   uint32_t* adj, uint32_t* component, void* tmp, size_t tmp_bytes,
                                                   uint32_t* flags, hipStream_t st);

extern "C" int vgpu_roadmap_assemble_device(vgpu_ctx* c, size_t n, const uint32_t* pairs, size_t m, uint64_t* offsets,
                                            uint32_t* adj, uint32_t* component)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (n >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "too many vertices");
    if (2 * m >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "too many pairs (2m must be < 2^31)");
    if (!offsets || (m && (!pairs || !adj))) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    if (m && n == 0) return fail(c, VGPU_ERR_INVALID_ARG, "pair index out of range");
    HIPCHK(c, ctx_device(c));
    const size_t bytes = vgpu_roadmap_assemble_bytes((uint32_t)n, m);
    if (!bytes) return fail(c, VGPU_ERR_HIP, "roadmap assembly: scratch size query failed");
    int rc;
    // the kNN index pool: free again once the edge stage's queries are done (same stream)
    if ((rc = grow(c, &c->knn_idx, &c->knn_idx_cap, (bytes + 3) / 4))) return rc;
    if (n == 0) {
        HIPCHK(c, hipMemsetAsync(offsets, 0, sizeof(uint64_t), c->cur));
        return VGPU_OK;
    }
    uint32_t flags = 0;
    HIPCHK(c, vgpu_launch_roadmap_assemble((uint32_t)n, pairs, m, (unsigned long long*)offsets, adj, component,
                                           c->knn_idx, c->knn_idx_cap * 4, &flags, c->cur));
    if (flags & 1u) return fail(c, VGPU_ERR_INVALID_ARG, "pair index out of range");
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_build_roadmap_host(vgpu_ctx* c, const vgpu_robot* robot, vgpu_env* e, const float* V, size_t n,
                                       double space_measure, double gamma_scale, size_t* offsets, uint32_t* adj,
                                       size_t adj_cap, size_t* n_adj, uint32_t* component)
try {
    if (!c || !e || e->ctx != c) return fail(c, VGPU_ERR_INVALID_ARG, "bad context/environment");
    float b[3];
    int rc = check_robot(c, robot, b);
    if (rc) return rc;
    const int dim = (int)dim_of(robot);
    if (!knn_dim_ok(dim)) return fail(c, VGPU_ERR_UNSUPPORTED, "roadmap: robot dimension");
    if (n && (!V || !offsets || !n_adj)) return fail(c, VGPU_ERR_INVALID_ARG, "null buffers");
    if (n >= ((size_t)1 << 31)) return fail(c, VGPU_ERR_INVALID_ARG, "too many vertices");
    if (n_adj) *n_adj = 0;
    if (n == 0) {
        if (offsets) offsets[0] = 0;
        return VGPU_OK;
    }
    std::vector<uint32_t> k(n);
    std::vector<float> r(n);
    if ((rc = vgpu_prm_neighbor_params(dim, space_measure, gamma_scale, n, k.data(), r.data()))) return rc;
    uint32_t kmax = 1;
    for (uint32_t v : k) kmax = std::max(kmax, v);
    kmax = std::min<uint32_t>(kmax, (uint32_t)n);
    if (kmax > 64) return fail(c, VGPU_ERR_UNSUPPORTED, "roadmap kNN: more than 64 neighbours per query");
    HIPCHK(c, ctx_device(c));
    DevBufs db;
    float *dV, *dr, *dd;
    uint32_t *dk, *dn, *dc, *doff;
    HIPCHK(c, db.get(&dV, n * dim));
    HIPCHK(c, db.get(&dk, n));
    HIPCHK(c, db.get(&dr, n));
    HIPCHK(c, db.get(&dn, n * kmax));
    HIPCHK(c, db.get(&dd, n * kmax));
    HIPCHK(c, db.get(&dc, n));
    HIPCHK(c, db.get(&doff, n + 1));
    HIPCHK(c, hipMemcpyAsync(dV, V, n * dim * sizeof(float), hipMemcpyHostToDevice, c->cur));
    HIPCHK(c, hipMemcpyAsync(dk, k.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, c->cur));
    HIPCHK(c, hipMemcpyAsync(dr, r.data(), n * sizeof(float), hipMemcpyHostToDevice, c->cur));
    if ((rc = vgpu_roadmap_knn(c, dim, dV, n, dk, dr, kmax, dn, dd, dc))) return rc;
    std::vector<uint32_t> cnt(n), off(n + 1);
    HIPCHK(c, hipMemcpyAsync(cnt.data(), dc, n * sizeof(uint32_t), hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    off[0] = 0;
    for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + cnt[i];
    const size_t E = off[n];
    std::vector<uint32_t> nb(n * (size_t)kmax);
    std::vector<uint8_t> ok(E);
    if (E) {
        float *ds, *dg;
        uint8_t* dok;
        HIPCHK(c, db.get(&ds, E * dim));
        HIPCHK(c, db.get(&dg, E * dim));
        HIPCHK(c, db.get(&dok, E));
        HIPCHK(c, hipMemcpyAsync(doff, off.data(), (n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, c->cur));
        HIPCHK(c, vgpu_launch_edge_gather(dV, 0, (uint32_t)n, dim, dn, kmax, dc, doff, ds, dg, c->cur));
        // validate_motion(neighbor, vertex) for every candidate (prm.hh:267-276)
        if ((rc = vgpu_validate_motions(c, robot, e, ds, dg, E, dok, nullptr))) return rc;
        HIPCHK(c, hipMemcpyAsync(ok.data(), dok, E, hipMemcpyDeviceToHost, c->cur));
        HIPCHK(c, hipMemcpyAsync(nb.data(), dn, n * (size_t)kmax * sizeof(uint32_t), hipMemcpyDeviceToHost, c->cur));
        HIPCHK(c, hipStreamSynchronize(c->cur));
    }
    // the valid pairs in query order, nearest first
    std::vector<uint32_t> pairs;
    pairs.reserve(2 * E);
    for (size_t i = 0; i < n; ++i)
        for (uint32_t m = 0; m < cnt[i]; ++m)
            if (ok[off[i] + m]) {
                pairs.push_back((uint32_t)i);
                pairs.push_back(nb[i * kmax + m]);
            }
    *n_adj = pairs.size();
    if (pairs.size() > adj_cap || (!pairs.empty() && !adj))
        return fail(c, VGPU_ERR_INVALID_ARG, "adjacency capacity too small (*n_adj = required entries)");
    if ((rc = vgpu_roadmap_assemble(n, pairs.data(), pairs.size() / 2, offsets, adj, component)))
        return fail(c, rc, "roadmap assembly");
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_filter_robot_pointcloud_host(vgpu_ctx* c, const vgpu_robot* r, vgpu_env* e,
                                                 const float* configuration, const float* pc, size_t n,
                                                 float point_radius, float* out, size_t* count)
try {
    if (!c) return VGPU_ERR_INVALID_ARG;
    if (!count) return fail(c, VGPU_ERR_INVALID_ARG, "null count");
    *count = 0;
    if (n == 0) return VGPU_OK;
    if (!pc || !out) return fail(c, VGPU_ERR_INVALID_ARG, "null buffer");
    if (n > 0x7fffffffu) return fail(c, VGPU_ERR_INVALID_ARG, "point cloud size");
    char* d;
    const size_t pb = al(n * 12), kb = al(n), ib = al(n * 4);
    int rc = stage(c, 2 * pb + kb + ib, &d);
    if (rc) return rc;
    HIPCHK(c, ctx_device(c));
    HIPCHK(c, hipMemcpyAsync(d, pc, n * 12, hipMemcpyHostToDevice, c->cur));
    uint8_t* keep = (uint8_t*)(d + pb);
    if ((rc = vgpu_filter_robot_pointcloud(c, r, e, configuration, (const float*)d, n, point_radius, keep))) return rc;
    // the kept points in input order (std::vector::emplace_back order, common.hh:80-83)
    if ((rc = vgpu_compact(c, (const float*)d, keep, n, 3, (float*)(d + pb + kb), (uint32_t*)(d + 2 * pb + kb), count)))
        return rc;
    HIPCHK(c, hipMemcpyAsync(out, d + pb + kb, *count * 12, hipMemcpyDeviceToHost, c->cur));
    HIPCHK(c, hipStreamSynchronize(c->cur));
    return VGPU_OK;
} VGPU_ABI_CATCH
