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
//     and draw indices, concatenated in rank order = build_roadmap's vertex sequence (prm.hh:235-254);
//     vgpu_prm_edges_allgather is its edge stage (prm.hh:255-299) -- query ranges of equal prefix work, the
//     valid pairs all-gathered, the roadmap assembled on every rank's device.
//     Every rank-local failure (argument, allocation, kernel) still enters exchange 1 with a failure word in
//     place of its count, so all ranks return the same error and none is left inside an all-gather.
#include <dlfcn.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vamp_gpu.h"
#include "vgpu_abi.hh"

extern "C" int vgpu_env_clone(const vgpu_env* src, vgpu_ctx* c, vgpu_env** out);

// ---- shard ranges ---------------------------------------------------------------------------------
extern "C" int vgpu_shard_range(size_t n, int rank, int world, size_t* first, size_t* count)
try {
    if (world < 1 || rank < 0 || rank >= world || !first || !count) return VGPU_ERR_INVALID_ARG;
    const unsigned __int128 lo = (unsigned __int128)n * (unsigned)rank / (unsigned)world;
    const unsigned __int128 hi = (unsigned __int128)n * (unsigned)(rank + 1) / (unsigned)world;
    *first = (size_t)lo;
    *count = (size_t)(hi - lo);
    return VGPU_OK;
} VGPU_ABI_CATCH

// ---- one process, several devices -------------------------------------------------------------------
struct vgpu_multi {
    std::vector<vgpu_ctx*> ctx;
    std::vector<int> device;
    std::string err;
};

extern "C" int vgpu_multi_create(const int* devices, int n, vgpu_multi** out)
try {
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
} VGPU_ABI_CATCH

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
try {
    if (!m || !src || !envs) return VGPU_ERR_INVALID_ARG;
    for (size_t i = 0; i < m->ctx.size(); ++i) {
        const int rc = vgpu_env_clone(src, m->ctx[i], &envs[i]);
        if (rc != VGPU_OK) {
            for (size_t j = 0; j < i; ++j) vgpu_env_destroy(envs[j]);
            return rc;
        }
    }
    return VGPU_OK;
} VGPU_ABI_CATCH

// Runs fn(i) on one host thread per device; the first failure's code and message are returned.
template <class Fn>
static int per_device(vgpu_multi* m, Fn fn)
{
    std::vector<int> rc(m->ctx.size(), VGPU_OK);
    std::vector<std::thread> th;
    th.reserve(m->ctx.size());
    // HIP's current device is per thread and a new thread starts on device 0: select the context's device
    // before fn allocates or launches anything.  No exception leaves a worker (it would terminate the process),
    // and a device whose thread cannot be started runs on this thread after the others have been started
    auto body = [&](size_t i) {
        try {
            rc[i] = hipSetDevice(m->device[i]) != hipSuccess ? VGPU_ERR_HIP : fn((int)i);
        } catch (const std::bad_alloc&) {
            rc[i] = VGPU_ERR_OOM;
        } catch (...) {
            rc[i] = VGPU_ERR_INTERNAL;
        }
    };
    size_t started = 0;
    try {
        for (; started < m->ctx.size(); ++started) th.emplace_back(body, started);
    } catch (...) {
    }
    for (size_t i = started; i < m->ctx.size(); ++i) body(i);
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
try {
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
} VGPU_ABI_CATCH

// The PRM vertex stage over the devices: draws first .. first + n_draws - 1 split into contiguous ranges,
// each device's valid rows compacted on the device and copied back; rows_out[*count][dim] and draws_out
// (1-based draw indices) in draw order (capacity n_draws each).
extern "C" int vgpu_multi_sample_fkcc_host(vgpu_multi* m, const vgpu_robot* r, vgpu_env* const* envs, uint64_t first,
                                           size_t n_draws, float* rows_out, uint64_t* draws_out, size_t* count)
try {
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
        float *q = nullptr, *ro = nullptr;
        uint8_t* v = nullptr;
        uint32_t* ix = nullptr;
        int e = VGPU_OK;
        if (hipMalloc(&q, cnt * dim * sizeof(float)) != hipSuccess ||
            hipMalloc(&ro, cnt * dim * sizeof(float)) != hipSuccess ||
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
} VGPU_ABI_CATCH

// ---- one process per GPU: the exchange a communicator runs its all-gathers over -----------------------
// The sharded stages below need exactly one collective: an all-gather of equal-sized device blocks in rank
// order.  Two implementations sit behind it:
//   * RCCL (librccl.so.1 loaded at run time, no torch): ncclAllGather over xGMI -- the product path;
//   * a loopback hub: the ranks are host threads of ONE process (each with its own context, on one device
//     or several), the all-gather is a barrier plus device copies from every peer's send block.  It runs the
//     stages' multi-rank logic -- rank-order concatenation, count padding, failure words -- at world sizes
//     above one on a single GPU (an in-process loopback communicator for tests).
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

// every rank's `bytes` of send (device) into recv[k * bytes] (device), in rank order; enqueued on st or
// completed before returning -- the caller synchronises st before reading recv
struct Exchange {
    virtual ~Exchange() = default;
    virtual bool allgather(const void* send, void* recv, size_t bytes, hipStream_t st) = 0;
};

struct RcclExchange final : Exchange {
    ncclComm_t comm = nullptr;
    ~RcclExchange() override
    {
        if (comm && rccl().ok) rccl().destroy(comm);
    }
    bool allgather(const void* send, void* recv, size_t bytes, hipStream_t st) override
    {
        return rccl().allgather(send, recv, bytes, ncclUint8, comm, st) == ncclSuccess;
    }
};
}  // namespace

// The loopback hub: `world` ranks as threads of this process.  A generation barrier with a timeout (a rank
// that never arrives makes the others fail instead of hang).
struct vgpu_loopback {
    int world = 1;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0;
    std::vector<const void*> send;
    std::vector<size_t> bytes;
    int members = 0;  // communicators created on the hub and not yet destroyed
    int timeout_s = 120;
    // set for good by the first barrier that times out: a late rank arriving afterwards must not pair up with
    // its peers' NEXT exchange (same sizes, other data), so every later barrier fails at once
    bool failed = false;

    bool barrier()
    {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) return false;
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(timeout_s), [&] { return gen != g || failed; }) || gen == g) {
            failed = true;  // the hub is unusable from here on; wake the peers still waiting
            cv.notify_all();
            return false;
        }
        return true;
    }
};

namespace {
struct LoopbackExchange final : Exchange {
    vgpu_loopback* hub = nullptr;
    int rank = 0;
    ~LoopbackExchange() override
    {
        std::lock_guard<std::mutex> lk(hub->mu);
        --hub->members;
    }
    bool allgather(const void* send, void* recv, size_t bytes, hipStream_t st) override
    {
        // the send block must be complete before a peer copies it
        bool ok = hipStreamSynchronize(st) == hipSuccess;
        {
            std::lock_guard<std::mutex> lk(hub->mu);
            hub->send[rank] = ok ? send : nullptr;
            hub->bytes[rank] = bytes;
        }
        if (!hub->barrier()) return false;
        for (int k = 0; k < hub->world; ++k) {
            const void* src;
            size_t b;
            {
                std::lock_guard<std::mutex> lk(hub->mu);
                src = hub->send[k];
                b = hub->bytes[k];
            }
            if (b != bytes || (bytes && !src)) ok = false;  // mismatched sizes or a peer's failed sync
            if (ok && bytes &&
                hipMemcpyAsync((char*)recv + (size_t)k * bytes, src, bytes, hipMemcpyDefault, st) != hipSuccess)
                ok = false;
        }
        if (hipStreamSynchronize(st) != hipSuccess) ok = false;
        // the peers' send blocks stay untouched until every rank has copied them
        if (!hub->barrier()) return false;
        return ok;
    }
};

// grow-only device buffers of a communicator, one per slot (the stages below name their slots)
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};
constexpr int kSlots = 16;
}  // namespace

struct vgpu_comm {
    std::unique_ptr<Exchange> x;
    int rank = 0, world = 1, device = 0;
    hipStream_t st = nullptr;  // the exchanges' stream (the kernels run on the context's)
    // exchange 1's word buffer (2 * world + 2 u64: the gathered words, this rank's word, the selection
    // count), allocated with the communicator: a stage whose own allocations or arguments fail still has
    // it, so it always enters exchange 1
    uint64_t* words = nullptr;
    DevBuf buf[kSlots];
    std::string err;
};

static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");

extern "C" int vgpu_comm_unique_id(uint8_t id[128])
try {
    if (!id) return VGPU_ERR_INVALID_ARG;
    Rccl& R = rccl();
    if (!R.ok) return VGPU_ERR_UNSUPPORTED;
    ncclUniqueId u;
    if (R.get_id(&u) != ncclSuccess) return VGPU_ERR_HIP;
    std::memcpy(id, &u, 128);
    return VGPU_OK;
} VGPU_ABI_CATCH

// RCCL may print a version banner on stdout while a communicator is created.  With VGPU_RCCL_QUIET=1 the
// caller's stdout (bench.py's one JSON line) stays clean: fd 1 is pointed at stderr for the duration of
// ncclCommInitRank.  The redirect is process-global (other threads' stdout writes in that window go to
// stderr too), hence opt-in.
namespace {
struct StdoutToStderr {
    int saved = -1;
    StdoutToStderr()
    {
        const char* q = std::getenv("VGPU_RCCL_QUIET");
        if (!q || std::strcmp(q, "1") != 0) return;
        std::fflush(stdout);
        saved = dup(1);
        if (saved >= 0) dup2(2, 1);
    }
    ~StdoutToStderr()
    {
        if (saved < 0) return;
        std::fflush(stdout);
        dup2(saved, 1);
        close(saved);
    }
};

// exchange 1's word buffer layout: [0, W) the gathered words, [W] this rank's word, [W + 1] the selection
// count, [W + 2] a pre-set failure word (kFailTag | -VGPU_ERR_HIP): the word a rank sends when even the copy of
// its own word to the device fails, so it still enters the all-gather
constexpr uint64_t kFailTagC = 0xFFFFFFFF00000000ull;
size_t words_len(int world) { return 2 * (size_t)world + 3; }

// the communicator's word buffer (first: the status exchange below needs it) and stream on its device, before
// the exchange itself exists.  Returns the first failure; c->words is non-null whenever that allocation worked
int comm_alloc(vgpu_comm* c, int dev, int world)
{
    c->device = dev;
    c->world = world;
    if (hipMalloc(&c->words, words_len(world) * sizeof(uint64_t)) != hipSuccess) {
        c->words = nullptr;
        return VGPU_ERR_OOM;
    }
    const uint64_t fail = kFailTagC | (uint32_t)(-VGPU_ERR_HIP);
    if (hipMemcpy(c->words + world + 2, &fail, 8, hipMemcpyHostToDevice) != hipSuccess) return VGPU_ERR_HIP;
    if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) {
        c->st = nullptr;
        return VGPU_ERR_HIP;
    }
    return VGPU_OK;
}
}  // namespace

extern "C" void vgpu_comm_destroy(vgpu_comm* c);
static bool injected(const vgpu_comm* c, const char* site);

// The last step of communicator creation, on every rank alike: one all-gather of each rank's creation status
// (0, or kFailTag | -code), so that when ANY rank failed -- an allocation, the exchange, an injected fault --
// EVERY rank destroys its communicator and returns the same code (the lowest failing rank's) instead of leaving
// its peers to block in their first stage's all-gather.  A rank without a word buffer (its 24-byte allocation
// failed) cannot take part: it returns at once, and its peers' status all-gather fails in RCCL (or times out on
// the loopback hub) -- the one case this cannot turn into a clean error.
static int comm_status_exchange(vgpu_comm* c, int local_rc, vgpu_comm** out)
{
    if (local_rc == VGPU_OK && injected(c, "comm_init")) local_rc = VGPU_ERR_HIP, c->err = "injected failure";
    if (!c->words) {
        vgpu_comm_destroy(c);
        return local_rc != VGPU_OK ? local_rc : VGPU_ERR_OOM;
    }
    const int W = c->world;
    const uint64_t mine = local_rc != VGPU_OK ? (kFailTagC | (uint32_t)(-local_rc)) : 0;
    std::vector<uint64_t> all(W, kFailTagC | (uint32_t)(-VGPU_ERR_HIP));
    const hipStream_t st = c->st;  // null stream when the stream could not be created
    const bool put = hipMemcpy(c->words + W, &mine, 8, hipMemcpyHostToDevice) == hipSuccess;
    bool ok = c->x && c->x->allgather(c->words + (put ? W : W + 2), c->words, 8, st);
    ok = ok && hipMemcpyAsync(all.data(), c->words, W * 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
    int rc = ok ? VGPU_OK : VGPU_ERR_HIP;
    for (int k = 0; ok && k < W; ++k)
        if (all[k] >= kFailTagC) {
            rc = -(int)(uint32_t)(all[k] & 0xFFFFFFFFu);
            break;
        }
    if (rc == VGPU_OK && !put) rc = VGPU_ERR_HIP;  // (the pre-set word already told the peers)
    if (rc != VGPU_OK) {
        vgpu_comm_destroy(c);
        return rc;
    }
    *out = c;
    return VGPU_OK;
}

extern "C" int vgpu_comm_init(vgpu_ctx* ctx, int rank, int world, const uint8_t id[128], vgpu_comm** out)
try {
    if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world) return VGPU_ERR_INVALID_ARG;
    *out = nullptr;
    Rccl& R = rccl();
    if (!R.ok) return VGPU_ERR_UNSUPPORTED;
    int dev = 0;
    if (vgpu_ctx_device(ctx, &dev) != VGPU_OK || hipSetDevice(dev) != hipSuccess) return VGPU_ERR_HIP;
    auto* c = new (std::nothrow) vgpu_comm();
    if (!c) return VGPU_ERR_OOM;
    c->rank = rank;
    // the word buffer comes first; a later local failure (the stream, the exchange object, an injected
    // "comm_init:alloc") still joins ncclCommInitRank -- itself collective, into a stack handle that needs no
    // allocation -- and then reports through the status exchange
    int lrc = comm_alloc(c, dev, world);
    if (lrc == VGPU_OK && injected(c, "comm_init:alloc")) lrc = VGPU_ERR_OOM, c->err = "injected failure";
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclComm_t comm = nullptr;
    ncclResult_t ir;
    {
        StdoutToStderr quiet;
        ir = R.init(&comm, world, u, rank);
    }
    (void)hipGetLastError();  // RCCL's device probing may leave a handled error as this thread's last one
    if (ir != ncclSuccess) {  // no communicator to exchange over: RCCL reports its own failure per rank
        vgpu_comm_destroy(c);
        return VGPU_ERR_HIP;
    }
    auto* x = new (std::nothrow) RcclExchange();
    if (!x) {
        // nothing to run the status exchange through but the raw handle: a throwaway exchange on the stack
        RcclExchange tmp;
        tmp.comm = comm;
        c->x.reset();
        if (c->words) {
            const uint64_t* src = c->words + world + 2;  // the pre-set failure word
            (void)tmp.allgather(src, c->words, 8, c->st);
            (void)hipStreamSynchronize(c->st);
        }
        vgpu_comm_destroy(c);
        return VGPU_ERR_OOM;  // tmp's destructor destroys the RCCL communicator
    }
    x->comm = comm;
    c->x.reset(x);
    return comm_status_exchange(c, lrc, out);
} VGPU_ABI_CATCH

extern "C" int vgpu_loopback_create(int world, vgpu_loopback** out)
try {
    if (!out || world < 1) return VGPU_ERR_INVALID_ARG;
    *out = nullptr;
    auto* h = new (std::nothrow) vgpu_loopback();
    if (!h) return VGPU_ERR_OOM;
    h->world = world;
    h->send.assign(world, nullptr);
    h->bytes.assign(world, 0);
    if (const char* t = std::getenv("VGPU_LOOPBACK_TIMEOUT_S")) h->timeout_s = std::max(1, std::atoi(t));
    *out = h;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_loopback_destroy(vgpu_loopback* h)
try {
    if (!h) return VGPU_OK;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        if (h->members) return VGPU_ERR_INVALID_ARG;  // communicators still use it
    }
    delete h;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_comm_init_loopback(vgpu_ctx* ctx, int rank, vgpu_loopback* hub, vgpu_comm** out)
try {
    if (!ctx || !hub || !out || rank < 0 || rank >= hub->world) return VGPU_ERR_INVALID_ARG;
    *out = nullptr;
    int dev = 0;
    if (vgpu_ctx_device(ctx, &dev) != VGPU_OK || hipSetDevice(dev) != hipSuccess) return VGPU_ERR_HIP;
    auto* c = new (std::nothrow) vgpu_comm();
    auto* x = new (std::nothrow) LoopbackExchange();
    if (!c || !x) {
        delete c;
        delete x;
        return VGPU_ERR_OOM;
    }
    x->hub = hub;
    x->rank = rank;
    {
        std::lock_guard<std::mutex> lk(hub->mu);
        ++hub->members;
    }
    c->x.reset(x);
    c->rank = rank;
    // the same status exchange as vgpu_comm_init: a failing rank fails every rank's creation
    int lrc = comm_alloc(c, dev, hub->world);
    if (lrc == VGPU_OK && injected(c, "comm_init:alloc")) lrc = VGPU_ERR_OOM, c->err = "injected failure";
    return comm_status_exchange(c, lrc, out);
} VGPU_ABI_CATCH

extern "C" void vgpu_comm_destroy(vgpu_comm* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->st) (void)hipStreamSynchronize(c->st);
    for (DevBuf& b : c->buf)
        if (b.p) (void)hipFree(b.p);
    if (c->words) (void)hipFree(c->words);
    if (c->st) (void)hipStreamDestroy(c->st);
    c->x.reset();
    delete c;
}

extern "C" const char* vgpu_comm_last_error(const vgpu_comm* c) { return c ? c->err.c_str() : "null comm"; }

template <class T>
static bool comm_buf(vgpu_comm* c, int slot, size_t count, T** out)
{
    DevBuf& b = c->buf[slot];
    const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    if (bytes > b.cap) {
        if (b.p) {
            (void)hipStreamSynchronize(c->st);
            (void)hipFree(b.p);
            b.p = nullptr;
            b.cap = 0;
        }
        if (hipMalloc(&b.p, bytes) != hipSuccess) {
            b.p = nullptr;
            return false;
        }
        b.cap = bytes;
    }
    *out = (T*)b.p;
    return true;
}

// Rank-local fault injection for the failure-path tests: VGPU_FAULT_INJECT=<site>[@rank] makes that rank
// (every rank without @) fail at <site>.  Sites per stage: "<stage>:args" (an argument error, before
// anything else), "<stage>:alloc" (the stage's first allocation fails), "<stage>" (after every allocation),
// with <stage> = prm_vertices | prm_edges.
static bool injected(const vgpu_comm* c, const char* site)
{
    const char* v = std::getenv("VGPU_FAULT_INJECT");
    if (!v) return false;
    const std::string s(v);
    const size_t at = s.find('@');
    if (s.substr(0, at) != site) return false;
    return at == std::string::npos || std::atoi(s.c_str() + at + 1) == c->rank;
}

// A failing rank still enters every collective its peers enter: exchange 1 carries each rank's count, or
// kFailTag | -code, so every rank sees the same failure and returns the same error (the lowest failing
// rank's) instead of leaving its peers blocked in the next all-gather.
static constexpr uint64_t kFailTag = 0xFFFFFFFF00000000ull;

static int exchange_counts(vgpu_comm* c, int local_rc, uint64_t count, std::vector<uint64_t>& all)
{
    const int W = c->world;
    uint64_t* dev_words = c->words;
    const uint64_t mine = local_rc != VGPU_OK ? (kFailTag | (uint32_t)(-local_rc)) : count;
    all.assign(W, 0);
    // the all-gather is entered whatever happens to this rank's word: when its copy to the device fails, the
    // pre-set failure word (comm_alloc) is sent instead, so the peers fail with this rank instead of waiting
    const bool put = hipMemcpyAsync(dev_words + W, &mine, 8, hipMemcpyHostToDevice, c->st) == hipSuccess;
    if (!c->x->allgather(dev_words + (put ? W : W + 2), dev_words, 8, c->st) || !put ||
        hipMemcpyAsync(all.data(), dev_words, W * 8, hipMemcpyDeviceToHost, c->st) != hipSuccess ||
        hipStreamSynchronize(c->st) != hipSuccess) {
        c->err = "count exchange (all-gather) failed";
        return VGPU_ERR_HIP;
    }
    for (int k = 0; k < W; ++k)
        if (all[k] >= kFailTag) {
            const int code = -(int)(uint32_t)(all[k] & 0xFFFFFFFFu);
            if (local_rc == VGPU_OK) c->err = "rank " + std::to_string(k) + " failed (code " + std::to_string(code) + ")";
            return code;
        }
    return VGPU_OK;
}

static int rank_fail(vgpu_comm* c, vgpu_ctx* ctx, int rc, const char* what)
{
    if (rc != VGPU_OK && c->err.empty()) c->err = std::string(what) + (ctx ? std::string(": ") + vgpu_last_error(ctx) : "");
    return rc;
}

// exchange 2: every rank's first cnts[k] items of `send` (padded to max cnts) gathered and concatenated in
// rank order into out; items are `item_bytes` each
static int gather_padded(vgpu_comm* c, const void* send, void* recv, const std::vector<uint64_t>& cnts,
                         size_t item_bytes, void* out)
{
    uint64_t mx = 0;
    for (uint64_t k : cnts) mx = std::max(mx, k);
    if (!mx) return VGPU_OK;
    if (!c->x->allgather(send, recv, mx * item_bytes, c->st)) {
        c->err = "all-gather failed";
        return VGPU_ERR_HIP;
    }
    size_t at = 0;
    for (size_t k = 0; k < cnts.size(); ++k) {
        if (cnts[k] && hipMemcpyAsync((char*)out + at * item_bytes, (const char*)recv + k * mx * item_bytes,
                                      cnts[k] * item_bytes, hipMemcpyDeviceToDevice, c->st) != hipSuccess) {
            c->err = "device copy failed";
            return VGPU_ERR_HIP;
        }
        at += cnts[k];
    }
    if (hipStreamSynchronize(c->st) != hipSuccess) {
        c->err = "exchange stream failed";
        return VGPU_ERR_HIP;
    }
    return VGPU_OK;
}

// The communicator's device becomes current whatever the arguments (exchange 1 runs there); a context on
// another device is a rank-local argument error like any other, reported to every rank through exchange 1.
static int comm_enter(vgpu_ctx* ctx, vgpu_comm* comm)
{
    if (hipSetDevice(comm->device) != hipSuccess) {
        comm->err = "hipSetDevice failed";
        return VGPU_ERR_HIP;
    }
    int dev = -1;
    if (!ctx || vgpu_ctx_device(ctx, &dev) != VGPU_OK) {
        comm->err = "null or invalid context";
        return VGPU_ERR_INVALID_ARG;
    }
    if (dev != comm->device) {
        comm->err = "context device differs from the communicator's";
        return VGPU_ERR_INVALID_ARG;
    }
    return VGPU_OK;
}

// PRM vertex stage of the whole job on this rank's device: draws first .. first + n_draws_total - 1, this
// rank's contiguous share sampled here, then the all-gather.  rows[cap][dim], draws[cap] (device) receive
// every rank's valid vertices in rank order = draw order; *count = their number (all ranks alike).  ctx
// must be the rank's context, on the device the communicator was created on.
extern "C" int vgpu_prm_vertices_allgather(vgpu_ctx* ctx, vgpu_comm* comm, const vgpu_robot* r, vgpu_env* e,
                                           uint64_t first, size_t n_draws_total, float* rows, uint64_t* draws,
                                           size_t cap, size_t* count)
try {
    if (!comm) return VGPU_ERR_INVALID_ARG;  // no communicator: nothing to enter (a caller bug on this rank)
    comm->err.clear();
    if (count) *count = 0;
    const int W = comm->world;
    const int dim = robot_dim(r);
    int rc = comm_enter(ctx, comm);
    if (rc == VGPU_OK && (!count || !rows || !draws || first == 0 || dim < 1))
        rc = VGPU_ERR_INVALID_ARG, comm->err = "invalid argument";
    if (rc == VGPU_OK && injected(comm, "prm_vertices:args")) rc = VGPU_ERR_INVALID_ARG, comm->err = "injected failure";
    size_t lo = 0, n = 0, share_max = (n_draws_total + W - 1) / W;
    vgpu_shard_range(n_draws_total, comm->rank, W, &lo, &n);
    float *q = nullptr, *pad_rows = nullptr, *all_rows = nullptr;
    uint8_t* v = nullptr;
    uint32_t* ix = nullptr;
    uint64_t *pad_draws = nullptr, *all_d = nullptr;
    // every buffer (both exchanges') up front, sized by the largest share: an allocation failure is known
    // before exchange 1 and reported through it
    if (rc == VGPU_OK && injected(comm, "prm_vertices:alloc")) rc = VGPU_ERR_OOM, comm->err = "injected failure";
    if (rc == VGPU_OK && dim > 0 &&
        !(comm_buf(comm, 0, share_max * dim, &q) && comm_buf(comm, 1, share_max, &v) && comm_buf(comm, 2, share_max, &ix) &&
          comm_buf(comm, 4, share_max * dim, &pad_rows) && comm_buf(comm, 5, share_max, &pad_draws) &&
          comm_buf(comm, 6, W * share_max * dim, &all_rows) && comm_buf(comm, 7, W * share_max, &all_d)))
        rc = VGPU_ERR_OOM, comm->err = "device allocation failed";
    if (rc == VGPU_OK && injected(comm, "prm_vertices")) rc = VGPU_ERR_OOM, comm->err = "injected failure";
    size_t got = 0;
    // this rank's share, compacted on the device straight into the exchange's send buffer
    if (rc == VGPU_OK && n) rc = rank_fail(comm, ctx, vgpu_sample_fkcc(ctx, r, e, first + lo, n, q, v), "sample_fkcc");
    if (rc == VGPU_OK && n) rc = rank_fail(comm, ctx, vgpu_compact(ctx, q, v, n, dim, pad_rows, ix, &got), "compact");
    if (rc == VGPU_OK) rc = rank_fail(comm, ctx, vgpu_sync(ctx), "sync");
    if (rc == VGPU_OK && got) {  // draw indices (1-based) of the kept rows, as uint64
        std::vector<uint32_t> hi(got);
        std::vector<uint64_t> hd(got);
        if (hipMemcpy(hi.data(), ix, got * 4, hipMemcpyDeviceToHost) != hipSuccess) rc = VGPU_ERR_HIP;
        for (size_t j = 0; j < got; ++j) hd[j] = first + lo + hi[j];
        if (rc == VGPU_OK && hipMemcpy(pad_draws, hd.data(), got * 8, hipMemcpyHostToDevice) != hipSuccess)
            rc = VGPU_ERR_HIP;
        if (rc != VGPU_OK) comm->err = "draw index copy failed";
    }
    std::vector<uint64_t> cnts;
    rc = exchange_counts(comm, rc, got, cnts);  // exchange 1, always entered
    if (rc != VGPU_OK) return rc;
    uint64_t total = 0;
    for (uint64_t c : cnts) total += c;
    if (total > cap) {  // every rank sees the same total
        comm->err = "vertex capacity too small";
        return VGPU_ERR_INVALID_ARG;
    }
    // exchange 2: the count-padded rows, then the draw indices
    if ((rc = gather_padded(comm, pad_rows, all_rows, cnts, (size_t)dim * sizeof(float), rows)) != VGPU_OK) return rc;
    if ((rc = gather_padded(comm, pad_draws, all_d, cnts, sizeof(uint64_t), draws)) != VGPU_OK) return rc;
    *count = (size_t)total;
    return VGPU_OK;
} VGPU_ABI_CATCH

// Query ranges of equal prefix work: query i scans i candidates, so rank k takes [n sqrt(k/W), n sqrt((k+1)/W))
// rounded half up (vamp_amd.roadmap.query_split is the same expression).
extern "C" int vgpu_query_split(size_t n, int rank, int world, size_t* first, size_t* count)
try {
    if (world < 1 || rank < 0 || rank >= world || !first || !count) return VGPU_ERR_INVALID_ARG;
    auto bound = [&](int k) -> size_t {
        if (k <= 0) return 0;
        if (k >= world) return n;
        const double b = std::floor((double)n * std::sqrt((double)k / (double)world) + 0.5);
        return std::min(n, (size_t)b);
    };
    *first = bound(rank);
    *count = bound(rank + 1) - *first;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" hipError_t vgpu_launch_valid_pairs(uint32_t q_first, uint32_t q_count, const uint32_t* nbr, uint32_t kmax,
                                              const uint32_t* cnt, const uint32_t* off, const uint8_t* ok, size_t E,
                                              unsigned long long* all, unsigned long long* out, uint32_t* count,
                                              void* tmp, size_t* tmp_bytes, hipStream_t st);

// PRM edge stage of the whole job (prm.hh:255-299): this rank's queries (vgpu_query_split) -- neighbour
// query, candidate gather, validate_motion(neighbor, vertex) of every candidate, the valid pairs selected on
// the device in query order -- then ONE exchange (counts, then the count-padded pairs), and the roadmap
// assembled on the device from all ranks' pairs in rank order = query order.  V[n][dim] (device, identical on
// every rank); offsets[n+1] (u64), adj[adj_cap], component[n] (optional) are device memory on ctx and come
// out equal on every rank.  *n_adj = 2 x the valid pairs; adj_cap < *n_adj fails with VGPU_ERR_INVALID_ARG
// on every rank (with *n_adj set).
extern "C" int vgpu_prm_edges_allgather(vgpu_ctx* ctx, vgpu_comm* comm, const vgpu_robot* r, vgpu_env* e,
                                        const float* V, size_t n, double space_measure, double gamma_scale,
                                        uint64_t* offsets, uint32_t* adj, size_t adj_cap, size_t* n_adj,
                                        uint32_t* component)
try {
    if (!comm) return VGPU_ERR_INVALID_ARG;  // no communicator: nothing to enter (a caller bug on this rank)
    comm->err.clear();
    if (n_adj) *n_adj = 0;
    const int W = comm->world;
    const int dim = robot_dim(r);
    int rc = comm_enter(ctx, comm);
    if (rc == VGPU_OK && (!n_adj || !offsets || (n && !V) || dim < 1 || n >= ((size_t)1 << 31)))
        rc = VGPU_ERR_INVALID_ARG, comm->err = "invalid argument";
    if (rc == VGPU_OK && injected(comm, "prm_edges:args")) rc = VGPU_ERR_INVALID_ARG, comm->err = "injected failure";
    // the neighbour parameters and every rank's candidate bound (query i returns at most min(k_i, i)): the
    // same on every rank, so buffer sizes and the cap check agree everywhere
    if (rc != VGPU_OK) n = 0;  // no per-query work sized from arguments that failed
    std::vector<uint32_t> k(std::max<size_t>(n, 1));
    std::vector<float> rad(std::max<size_t>(n, 1));
    if (rc == VGPU_OK && vgpu_prm_neighbor_params(dim, space_measure, gamma_scale, n, k.data(), rad.data()) != VGPU_OK)
        rc = VGPU_ERR_INVALID_ARG, comm->err = "neighbour parameters";
    uint32_t kmax = 1;
    for (size_t i = 0; i < n; ++i) kmax = std::max(kmax, k[i]);
    kmax = (uint32_t)std::min<size_t>(kmax, std::max<size_t>(n, 1));
    if (rc == VGPU_OK && kmax > 64) rc = VGPU_ERR_UNSUPPORTED, comm->err = "more than 64 neighbours per query";
    size_t qf = 0, qc = 0;
    vgpu_query_split(n, comm->rank, W, &qf, &qc);
    size_t e_mine = 0, e_max = 0;
    for (int w = 0; w < W; ++w) {
        size_t f, c, b = 0;
        vgpu_query_split(n, w, W, &f, &c);
        for (size_t i = f; i < f + c; ++i) b += std::min<size_t>(k[i], i);
        if (w == comm->rank) e_mine = b;
        e_max = std::max(e_max, b);
    }
    if (rc == VGPU_OK && (e_max >= ((size_t)1 << 31) || (size_t)W * e_max >= ((size_t)1 << 30)))
        rc = VGPU_ERR_UNSUPPORTED, comm->err = "too many candidate edges";
    uint32_t *dk = nullptr, *nbr = nullptr, *cnt = nullptr, *off = nullptr, *selc = nullptr;
    float *dr = nullptr, *dist = nullptr, *starts = nullptr, *goals = nullptr;
    uint8_t* ok = nullptr;
    unsigned long long *cand = nullptr, *sel = nullptr;
    uint64_t *recv = nullptr, *pairs = nullptr;
    char* tmp = nullptr;
    size_t tmp_bytes = 0;
    if (rc == VGPU_OK &&
        vgpu_launch_valid_pairs(0, 0, nullptr, 1, nullptr, nullptr, nullptr, e_mine, nullptr, nullptr, nullptr, nullptr,
                                &tmp_bytes, nullptr) != hipSuccess)
        rc = VGPU_ERR_HIP, comm->err = "selection scratch size";
    if (rc == VGPU_OK && injected(comm, "prm_edges:alloc")) rc = VGPU_ERR_OOM, comm->err = "injected failure";
    if (rc == VGPU_OK &&
        !(comm_buf(comm, 0, n, &dk) && comm_buf(comm, 1, n, &dr) && comm_buf(comm, 2, qc * kmax, &nbr) &&
          comm_buf(comm, 3, qc * kmax, &dist) && comm_buf(comm, 4, qc + 1, &cnt) && comm_buf(comm, 5, qc + 1, &off) &&
          comm_buf(comm, 6, e_mine * dim, &starts) && comm_buf(comm, 7, e_mine * dim, &goals) &&
          comm_buf(comm, 8, e_mine, &ok) && comm_buf(comm, 9, e_mine, &cand) && comm_buf(comm, 10, e_max, &sel) &&
          comm_buf(comm, 12, (size_t)W * e_max, &recv) && comm_buf(comm, 13, (size_t)W * e_max, &pairs) &&
          comm_buf(comm, 14, tmp_bytes, &tmp)))
        rc = VGPU_ERR_OOM, comm->err = "device allocation failed";
    if (rc == VGPU_OK && injected(comm, "prm_edges")) rc = VGPU_ERR_OOM, comm->err = "injected failure";
    selc = (uint32_t*)(comm->words + W + 1);  // the selection count: the communicator's own word buffer
    size_t got = 0;
    if (rc == VGPU_OK && n) {
        if (hipMemcpy(dk, k.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(dr, rad.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess)
            rc = VGPU_ERR_HIP, comm->err = "parameter upload failed";
    }
    if (rc == VGPU_OK && qc)
        rc = rank_fail(comm, ctx, vgpu_roadmap_knn_range(ctx, dim, V, n, qf, qc, dk, dr, kmax, nbr, dist, cnt), "knn");
    size_t E = 0;
    if (rc == VGPU_OK && qc) {  // candidate offsets (one host read: E sizes the validation)
        std::vector<uint32_t> hc(qc), ho(qc + 1);
        if (vgpu_sync(ctx) != VGPU_OK || hipMemcpy(hc.data(), cnt, qc * 4, hipMemcpyDeviceToHost) != hipSuccess)
            rc = VGPU_ERR_HIP, comm->err = "candidate count read-back failed";
        size_t acc = 0;
        for (size_t i = 0; i < qc; ++i) ho[i] = (uint32_t)acc, acc += hc[i];
        ho[qc] = (uint32_t)acc;
        E = acc;
        if (rc == VGPU_OK && E > e_mine) rc = VGPU_ERR_HIP, comm->err = "candidate count above its bound";
        if (rc == VGPU_OK && hipMemcpy(off, ho.data(), (qc + 1) * 4, hipMemcpyHostToDevice) != hipSuccess)
            rc = VGPU_ERR_HIP, comm->err = "offset upload failed";
    }
    if (rc == VGPU_OK && E)
        rc = rank_fail(comm, ctx,
                       vgpu_roadmap_edge_gather(ctx, dim, V, qf, qc, nbr, kmax, cnt, off, starts, goals), "edge gather");
    if (rc == VGPU_OK && E)  // validate_motion(neighbor, vertex) of every candidate (prm.hh:267-276)
        rc = rank_fail(comm, ctx, vgpu_validate_motions(ctx, r, e, starts, goals, E, ok, nullptr), "validate");
    if (rc == VGPU_OK) rc = rank_fail(comm, ctx, vgpu_sync(ctx), "sync");
    if (rc == VGPU_OK && E) {  // the valid pairs in query order, on the exchange stream
        uint32_t hgot = 0;
        if (vgpu_launch_valid_pairs((uint32_t)qf, (uint32_t)qc, nbr, kmax, cnt, off, ok, E, cand, sel, selc, tmp,
                                    &tmp_bytes, comm->st) != hipSuccess ||
            hipMemcpyAsync(&hgot, selc, 4, hipMemcpyDeviceToHost, comm->st) != hipSuccess ||
            hipStreamSynchronize(comm->st) != hipSuccess)
            rc = VGPU_ERR_HIP, comm->err = "pair selection failed";
        got = hgot;
    }
    std::vector<uint64_t> cnts;
    rc = exchange_counts(comm, rc, got, cnts);  // exchange 1, always entered
    if (rc != VGPU_OK) return rc;
    uint64_t m = 0;
    for (uint64_t c : cnts) m += c;
    *n_adj = (size_t)(2 * m);
    if (2 * m > adj_cap || (m && !adj)) {
        comm->err = "adjacency capacity too small (*n_adj = required entries)";
        return VGPU_ERR_INVALID_ARG;
    }
    if ((rc = gather_padded(comm, sel, recv, cnts, sizeof(uint64_t), pairs)) != VGPU_OK) return rc;  // exchange 2
    return rank_fail(comm, ctx,
                     vgpu_roadmap_assemble_device(ctx, n, (const uint32_t*)pairs, (size_t)m, offsets, adj, component),
                     "roadmap assembly");
} VGPU_ABI_CATCH
