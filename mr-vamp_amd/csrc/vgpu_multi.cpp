// vgpu_multi.cpp -- multi-GPU entry points at the C level, for a C++ planner that does not
// run torch.distributed:
//
//   * one process, several devices (vgpu_multi_*): one vgpu_ctx per device and one host thread per device;
//     a batch is split into contiguous ranges (vgpu_shard_range), each device validates / samples its own
//     range from pinned host staging, results land in the caller's host arrays in range order.  No
//     collective: edges and draws are independent units.
//   * one process per GPU (vgpu_comm_*): RCCL communicators over xGMI, loaded at run time from
//     librccl.so.1 (no torch); vgpu_prm_vertices_allgather is the PRM vertex stage of BASELINE configs[3]
//     -- each rank samples its contiguous draw range (Halton -> scale -> fkcc, compaction on the device),
//     then ONE exchange: an all-gather of the per-rank counts and an all-gather of the count-padded rows
//     and draw indices, concatenated in rank order = build_roadmap's vertex sequence (prm.hh:235-254).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vamp_gpu.h"

extern "C" int vgpu_env_clone(const vgpu_env* src, vgpu_ctx* c, vgpu_env** out);

// ---- shard ranges ---------------------------------------------------------------------------------
extern "C" int vgpu_shard_range(size_t n, int rank, int world, size_t* first, size_t* count)
{
    if (world < 1 || rank < 0 || rank >= world || !first || !count) return VGPU_ERR_INVALID_ARG;
    const unsigned __int128 lo = (unsigned __int128)n * (unsigned)rank / (unsigned)world;
    const unsigned __int128 hi = (unsigned __int128)n * (unsigned)(rank + 1) / (unsigned)world;
    *first = (size_t)lo;
    *count = (size_t)(hi - lo);
    return VGPU_OK;
}

// ---- one process, several devices -------------------------------------------------------------------
struct vgpu_multi {
    std::vector<vgpu_ctx*> ctx;
    std::vector<int> device;
    std::string err;
};

extern "C" int vgpu_multi_create(const int* devices, int n, vgpu_multi** out)
{
    if (!out || n < 1 || !devices) return VGPU_ERR_INVALID_ARG;
    *out = nullptr;
    auto* m = new (std::nothrow) vgpu_multi();
    if (!m) return VGPU_ERR_OOM;
    for (int i = 0; i < n; ++i) {
        vgpu_ctx* c = nullptr;
        const int rc = vgpu_ctx_create(devices[i], &c);
        if (rc != VGPU_OK) {
            for (vgpu_ctx* x : m->ctx) vgpu_ctx_destroy(x);
            delete m;
            return rc;
        }
        m->ctx.push_back(c);
        m->device.push_back(devices[i]);
    }
    *out = m;
    return VGPU_OK;
}

extern "C" void vgpu_multi_destroy(vgpu_multi* m)
{
    if (!m) return;
    for (vgpu_ctx* c : m->ctx) vgpu_ctx_destroy(c);
    delete m;
}

extern "C" int vgpu_multi_size(const vgpu_multi* m) { return m ? (int)m->ctx.size() : 0; }

extern "C" vgpu_ctx* vgpu_multi_context(vgpu_multi* m, int i)
{
    return (m && i >= 0 && i < (int)m->ctx.size()) ? m->ctx[i] : nullptr;
}

extern "C" const char* vgpu_multi_last_error(const vgpu_multi* m) { return m ? m->err.c_str() : "null multi"; }

// envs[i] = src realised on device i (destroy each with vgpu_env_destroy)
extern "C" int vgpu_multi_env_create(vgpu_multi* m, const vgpu_env* src, vgpu_env** envs)
{
    if (!m || !src || !envs) return VGPU_ERR_INVALID_ARG;
    for (size_t i = 0; i < m->ctx.size(); ++i) {
        const int rc = vgpu_env_clone(src, m->ctx[i], &envs[i]);
        if (rc != VGPU_OK) {
            for (size_t j = 0; j < i; ++j) vgpu_env_destroy(envs[j]);
            return rc;
        }
    }
    return VGPU_OK;
}

// Runs fn(i) on one host thread per device; the first failure's code and message are returned.
template <class Fn>
static int per_device(vgpu_multi* m, Fn fn)
{
    std::vector<int> rc(m->ctx.size(), VGPU_OK);
    std::vector<std::thread> th;
    for (size_t i = 0; i < m->ctx.size(); ++i) th.emplace_back([&, i] { rc[i] = fn((int)i); });
    for (auto& t : th) t.join();
    for (size_t i = 0; i < rc.size(); ++i)
        if (rc[i] != VGPU_OK) {
            m->err = std::string("device ") + std::to_string(m->device[i]) + ": " + vgpu_last_error(m->ctx[i]);
            return rc[i];
        }
    return VGPU_OK;
}

static int robot_dim(const vgpu_robot* r)
{
    int32_t dim = 0;
    return (r && vgpu_robot_info(r->kind, &dim, nullptr, nullptr) == VGPU_OK) ? dim : -1;
}

// validate_motion of every edge, edges split into contiguous ranges over the devices (host in/out)
extern "C" int vgpu_multi_validate_motions_host(vgpu_multi* m, const vgpu_robot* r, vgpu_env* const* envs,
                                                const float* starts, const float* goals, size_t n, uint8_t* ok,
                                                int32_t* n_blocks)
{
    if (!m || !envs || (n && (!starts || !goals || !ok))) return VGPU_ERR_INVALID_ARG;
    const int dim = robot_dim(r);
    if (dim < 1) return VGPU_ERR_INVALID_ARG;
    const int w = (int)m->ctx.size();
    return per_device(m, [&](int i) {
        size_t lo, cnt;
        vgpu_shard_range(n, i, w, &lo, &cnt);
        if (!cnt) return VGPU_OK;
        return vgpu_validate_motions_host(m->ctx[i], r, envs[i], starts + lo * dim, goals + lo * dim, cnt, ok + lo,
                                          n_blocks ? n_blocks + lo : nullptr);
    });
}

// The PRM vertex stage over the devices: draws first .. first + n_draws - 1 split into contiguous ranges,
// each device's valid rows compacted on the device and copied back; rows_out[*count][dim] and draws_out
// (1-based draw indices) in draw order (capacity n_draws each).
extern "C" int vgpu_multi_sample_fkcc_host(vgpu_multi* m, const vgpu_robot* r, vgpu_env* const* envs, uint64_t first,
                                           size_t n_draws, float* rows_out, uint64_t* draws_out, size_t* count)
{
    if (!m || !envs || !count || (n_draws && (!rows_out || !draws_out)) || first == 0) return VGPU_ERR_INVALID_ARG;
    *count = 0;
    const int dim = robot_dim(r);
    if (dim < 1) return VGPU_ERR_INVALID_ARG;
    const int w = (int)m->ctx.size();
    std::vector<size_t> got(w, 0);
    std::vector<std::vector<float>> rows(w);
    std::vector<std::vector<uint32_t>> idx(w);
    const int rc = per_device(m, [&](int i) -> int {
        size_t lo, cnt;
        vgpu_shard_range(n_draws, i, w, &lo, &cnt);
        if (!cnt) return VGPU_OK;
        vgpu_ctx* c = m->ctx[i];
        if (hipSetDevice(m->device[i]) != hipSuccess) return VGPU_ERR_HIP;
        float *q = nullptr, *ro = nullptr;
        uint8_t* v = nullptr;
        uint32_t* ix = nullptr;
        int e = VGPU_OK;
        if (hipMalloc(&q, cnt * dim * sizeof(float)) != hipSuccess || hipMalloc(&ro, cnt * dim * sizeof(float)) ||
            hipMalloc(&v, cnt) != hipSuccess || hipMalloc(&ix, cnt * sizeof(uint32_t)) != hipSuccess)
            e = VGPU_ERR_OOM;
        if (e == VGPU_OK) e = vgpu_sample_fkcc(c, r, envs[i], first + lo, cnt, q, v);
        if (e == VGPU_OK) e = vgpu_compact(c, q, v, cnt, dim, ro, ix, &got[i]);
        if (e == VGPU_OK) {
            rows[i].resize(got[i] * dim);
            idx[i].resize(got[i]);
            if (got[i] && (hipMemcpy(rows[i].data(), ro, got[i] * dim * sizeof(float), hipMemcpyDeviceToHost) ||
                           hipMemcpy(idx[i].data(), ix, got[i] * sizeof(uint32_t), hipMemcpyDeviceToHost)))
                e = VGPU_ERR_HIP;
        }
        for (void* p : {(void*)q, (void*)ro, (void*)v, (void*)ix})
            if (p) (void)hipFree(p);
        return e;
    });
    if (rc != VGPU_OK) return rc;
    size_t at = 0;
    for (int i = 0; i < w; ++i) {
        size_t lo, cnt;
        vgpu_shard_range(n_draws, i, w, &lo, &cnt);
        std::memcpy(rows_out + at * dim, rows[i].data(), got[i] * dim * sizeof(float));
        for (size_t j = 0; j < got[i]; ++j) draws_out[at + j] = first + lo + idx[i][j];
        at += got[i];
    }
    *count = at;
    return VGPU_OK;
}

// ---- one process per GPU: RCCL, loaded at run time ----------------------------------------------------
namespace {
struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) allgather = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
    bool ok = false;
};
Rccl& rccl()
{
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            R.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (R.h) break;
        }
        if (!R.h) return;
        R.get_id = (decltype(R.get_id))dlsym(R.h, "ncclGetUniqueId");
        R.init = (decltype(R.init))dlsym(R.h, "ncclCommInitRank");
        R.destroy = (decltype(R.destroy))dlsym(R.h, "ncclCommDestroy");
        R.allgather = (decltype(R.allgather))dlsym(R.h, "ncclAllGather");
        R.errstr = (decltype(R.errstr))dlsym(R.h, "ncclGetErrorString");
        R.ok = R.get_id && R.init && R.destroy && R.allgather && R.errstr;
    });
    return R;
}
}  // namespace

struct vgpu_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1, device = 0;
};

static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");

extern "C" int vgpu_comm_unique_id(uint8_t id[128])
{
    if (!id) return VGPU_ERR_INVALID_ARG;
    Rccl& R = rccl();
    if (!R.ok) return VGPU_ERR_UNSUPPORTED;
    ncclUniqueId u;
    if (R.get_id(&u) != ncclSuccess) return VGPU_ERR_HIP;
    std::memcpy(id, &u, 128);
    return VGPU_OK;
}

extern "C" int vgpu_comm_init(vgpu_ctx* ctx, int rank, int world, const uint8_t id[128], vgpu_comm** out)
{
    if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world) return VGPU_ERR_INVALID_ARG;
    *out = nullptr;
    Rccl& R = rccl();
    if (!R.ok) return VGPU_ERR_UNSUPPORTED;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return VGPU_ERR_HIP;
    auto* c = new (std::nothrow) vgpu_comm();
    if (!c) return VGPU_ERR_OOM;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    if (R.init(&c->comm, world, u, rank) != ncclSuccess) {
        delete c;
        return VGPU_ERR_HIP;
    }
    c->rank = rank;
    c->world = world;
    c->device = dev;
    *out = c;
    return VGPU_OK;
}

extern "C" void vgpu_comm_destroy(vgpu_comm* c)
{
    if (!c) return;
    if (c->comm && rccl().ok) rccl().destroy(c->comm);
    delete c;
}

// PRM vertex stage of the whole job on this rank's device: draws first .. first + n_draws_total - 1, this
// rank's contiguous share sampled here, then the all-gather.  rows[cap][dim], draws[cap] (device) receive
// every rank's valid vertices in rank order = draw order; *count = their number (all ranks alike).  ctx
// must be the rank's context, on the device the communicator was created on.
extern "C" int vgpu_prm_vertices_allgather(vgpu_ctx* ctx, vgpu_comm* comm, const vgpu_robot* r, vgpu_env* e,
                                           uint64_t first, size_t n_draws_total, float* rows, uint64_t* draws,
                                           size_t cap, size_t* count)
{
    if (!ctx || !comm || !count || !rows || !draws || first == 0) return VGPU_ERR_INVALID_ARG;
    *count = 0;
    const int dim = robot_dim(r);
    if (dim < 1) return VGPU_ERR_INVALID_ARG;
    Rccl& R = rccl();
    if (!R.ok) return VGPU_ERR_UNSUPPORTED;
    size_t lo, n;
    vgpu_shard_range(n_draws_total, comm->rank, comm->world, &lo, &n);
    const int W = comm->world;
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return VGPU_ERR_HIP;
    float *q = nullptr, *mine = nullptr, *all_rows = nullptr;
    uint8_t* v = nullptr;
    uint32_t* ix = nullptr;
    uint64_t *cnt_d = nullptr, *mine_d = nullptr, *all_d = nullptr;
    int rc = VGPU_OK;
    size_t got = 0;
    std::vector<uint64_t> cnts(W, 0);
    auto bail = [&](int code) { rc = code; };
    const size_t nn = std::max<size_t>(n, 1);
    if (hipMalloc(&q, nn * dim * 4) || hipMalloc(&mine, nn * dim * 4) || hipMalloc(&v, nn) ||
        hipMalloc(&ix, nn * 4) || hipMalloc(&cnt_d, (W + 1) * 8) || hipMalloc(&mine_d, nn * 8))
        bail(VGPU_ERR_OOM);
    // this rank's share, compacted on the device (the context's stream; joined before the collectives)
    if (rc == VGPU_OK && n) rc = vgpu_sample_fkcc(ctx, r, e, first + lo, n, q, v);
    if (rc == VGPU_OK && n) rc = vgpu_compact(ctx, q, v, n, dim, mine, ix, &got);
    if (rc == VGPU_OK) rc = vgpu_sync(ctx);
    if (rc == VGPU_OK) {
        // draw indices (1-based) of the kept rows, as uint64
        std::vector<uint32_t> hi(got);
        std::vector<uint64_t> hd(got);
        if (got && hipMemcpy(hi.data(), ix, got * 4, hipMemcpyDeviceToHost)) bail(VGPU_ERR_HIP);
        for (size_t j = 0; j < got; ++j) hd[j] = first + lo + hi[j];
        if (rc == VGPU_OK && got && hipMemcpy(mine_d, hd.data(), got * 8, hipMemcpyHostToDevice)) bail(VGPU_ERR_HIP);
        const uint64_t g64 = got;
        if (rc == VGPU_OK && hipMemcpy(cnt_d + W, &g64, 8, hipMemcpyHostToDevice)) bail(VGPU_ERR_HIP);
    }
    // exchange 1: the counts
    if (rc == VGPU_OK && R.allgather(cnt_d + W, cnt_d, 1, ncclUint64, comm->comm, st) != ncclSuccess) bail(VGPU_ERR_HIP);
    if (rc == VGPU_OK && (hipStreamSynchronize(st) || hipMemcpy(cnts.data(), cnt_d, W * 8, hipMemcpyDeviceToHost)))
        bail(VGPU_ERR_HIP);
    uint64_t mx = 0, total = 0;
    for (uint64_t c : cnts) mx = std::max(mx, c), total += c;
    if (rc == VGPU_OK && total > cap) rc = VGPU_ERR_INVALID_ARG;
    // exchange 2: the count-padded rows and draw indices
    if (rc == VGPU_OK && mx) {
        float* pad_rows = nullptr;
        uint64_t* pad_draws = nullptr;
        if (hipMalloc(&pad_rows, mx * dim * 4) || hipMalloc(&pad_draws, mx * 8) ||
            hipMalloc(&all_rows, W * mx * dim * 4) || hipMalloc(&all_d, W * mx * 8))
            bail(VGPU_ERR_OOM);
        if (rc == VGPU_OK && got &&
            (hipMemcpyAsync(pad_rows, mine, got * dim * 4, hipMemcpyDeviceToDevice, st) ||
             hipMemcpyAsync(pad_draws, mine_d, got * 8, hipMemcpyDeviceToDevice, st)))
            bail(VGPU_ERR_HIP);
        if (rc == VGPU_OK &&
            (R.allgather(pad_rows, all_rows, mx * dim, ncclFloat32, comm->comm, st) != ncclSuccess ||
             R.allgather(pad_draws, all_d, mx, ncclUint64, comm->comm, st) != ncclSuccess))
            bail(VGPU_ERR_HIP);
        size_t at = 0;  // concatenate in rank order
        for (int k = 0; rc == VGPU_OK && k < W; ++k) {
            if (cnts[k] && (hipMemcpyAsync(rows + at * dim, all_rows + (size_t)k * mx * dim, cnts[k] * dim * 4,
                                           hipMemcpyDeviceToDevice, st) ||
                            hipMemcpyAsync(draws + at, all_d + (size_t)k * mx, cnts[k] * 8, hipMemcpyDeviceToDevice,
                                           st)))
                bail(VGPU_ERR_HIP);
            at += cnts[k];
        }
        if (rc == VGPU_OK && hipStreamSynchronize(st)) bail(VGPU_ERR_HIP);
        (void)hipStreamSynchronize(st);
        for (void* p : {(void*)pad_rows, (void*)pad_draws})
            if (p) (void)hipFree(p);
    }
    (void)hipStreamSynchronize(st);
    for (void* p : {(void*)q, (void*)mine, (void*)v, (void*)ix, (void*)cnt_d, (void*)mine_d, (void*)all_rows,
                    (void*)all_d})
        if (p) (void)hipFree(p);
    (void)hipStreamDestroy(st);
    if (rc == VGPU_OK) *count = (size_t)total;
    return rc;
}
