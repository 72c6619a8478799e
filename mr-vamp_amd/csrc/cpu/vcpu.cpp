// vcpu.cpp -- the CPU rake: validate_motion / fkcc / sphere_fk on the host, one reference
// ConfigurationBlock<8> per AVX2 register (vcpu_simd.hh).
//
// Role: the reference's single-edge entry points -- Robot::fkcc<8>(env, block),
// validate_motion<Robot, 8, res>(start, goal, env) -- stay on the CPU, because a GPU launch costs
// far more than one ~2 us edge; planners call these (the C++ mirror include/vamp_gpu.hpp routes
// its Robot concept here).  The batch forms, threaded over the host cores with static contiguous
// chunks, are the CPU reference timing of bench.py (§8(d): "the build's own AVX2 restatement").
// Both are bit-identical to the oracle and to the GPU kernels: the same generated op sequence
// (tools/gen_kernels.py), the host's own _mm256_rsqrt_ps cull, the reference rake arithmetic.
#include <algorithm>
#include <cmath>
#include <limits>
#include <thread>
#include <vector>

#include "../vgpu_host_env.hh"
#include "../vgpu_abi.hh"
#include "vcpu_robot.hh"

namespace vcpu {

// vgpu_api.cpp:check_robot, without a context: PandaBase<X100, Y100, Z100> bases (panda/fk.hh:
// 109-111, static_cast<float>(x100) / 100.0f); Fetch / UR5 / Baxter have none
int bind(const vgpu_robot* r, Bound& b)
{
    if (!r) return VGPU_ERR_INVALID_ARG;
    switch (r->kind) {
        case VGPU_ROBOT_PANDA: b.R = robot_panda(); break;
        case VGPU_ROBOT_PANDA_PAIR: b.R = robot_panda_pair(); break;
        case VGPU_ROBOT_FETCH: b.R = robot_fetch(); break;
        case VGPU_ROBOT_UR5: b.R = robot_ur5(); break;
        case VGPU_ROBOT_BAXTER: b.R = robot_baxter(); break;
        default: return VGPU_ERR_UNSUPPORTED;
    }
    const bool panda = r->kind == VGPU_ROBOT_PANDA || r->kind == VGPU_ROBOT_PANDA_PAIR;
    if (!panda && (r->base_x100 || r->base_y100 || r->base_z100)) return VGPU_ERR_INVALID_ARG;
    b.base[0] = (float)r->base_x100 / 100.0f;
    b.base[1] = (float)r->base_y100 / 100.0f;
    b.base[2] = (float)r->base_z100 / 100.0f;
    b.base[3] = (float)r->base2_x100 / 100.0f;
    b.base[4] = (float)r->base2_y100 / 100.0f;
    b.base[5] = (float)r->base2_z100 / 100.0f;
    return VGPU_OK;
}

int view(vgpu_env* e, Env& out)
{
    if (!e) return VGPU_ERR_INVALID_ARG;
    vgpu::HostEnvView h;
    if (int rc = vgpu_env_host_view(e, &h)) return rc;
    for (int t = 0; t < OBS_TYPES; ++t) {
        out.v.obs[t] = h.obs[t];
        out.v.n[t] = h.n[t];
    }
    out.v.hf = h.hf;
    out.v.pc = h.pc;
    out.v.base = h.base;
    out.v.n_hf = h.n_hf;
    out.v.n_pc = h.n_pc;
    out.v.att = h.att;
    out.v.n_att = h.n_att;
    out.ext = h.n_hf > 0 || h.n_pc > 0;
    out.attached = h.attached;
    return VGPU_OK;
}

// FloatVector<dim>::l2_norm in the reference's lane order (vector/avx.hh:441-452 hsum; two
// registers fma(lo, lo, hi * hi) first for dim > 8), then std::sqrt -- as oracle vo_l2_norm
float l2_norm(const float* v, int dim)
{
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (dim <= 8) {
        for (int i = 0; i < dim; ++i) s[i] = v[i] * v[i];
    } else {
        for (int i = 0; i < 8; ++i) {
            const float hi = i + 8 < dim ? v[i + 8] : 0.0f;
            s[i] = std::fma(v[i], v[i], hi * hi);
        }
    }
    const float a = (s[0] + s[4]) + (s[2] + s[6]);
    const float b = (s[1] + s[5]) + (s[3] + s[7]);
    return std::sqrt(a + b);
}

// validate_vector<Robot, 8, Robot::resolution>(start, v, distance) (planning/validate.hh:23-65).
// Returns validity; *n = n_e (validate.hh:41), *evaluated = rake blocks evaluated before the
// result was known (the reference's early exit: the first invalid block ends the edge).
bool validate_vector_one(const Bound& b, const Env& env, const float* start, const float* v, float distance,
                         int32_t* n, int32_t* evaluated)
{
    const RobotCpu& R = *b.R;
    const int D = R.dim;
    const V pct = _mm256_setr_ps(1.0f / 8, 2.0f / 8, 3.0f / 8, 4.0f / 8, 5.0f / 8, 6.0f / 8, 7.0f / 8, 1.0f);
    V block[kMaxDim];
    for (int j = 0; j < D; ++j) block[j] = fma(V(v[j]), pct, V(start[j]));  // validate.hh:37 (contracted)
    float nf = std::ceil(distance / 8.0f * (float)R.resolution);            // validate.hh:41
    if (!(nf > 1.0f)) nf = 1.0f;
    const int32_t ne = nf < 2147483520.0f ? (int32_t)nf : 2147483520;
    if (n) *n = ne;
    // validate.hh:43: the first block through fkcc_attach when the environment has an attachment
    bool valid = (env.attached && R.fkcc_attach) ? R.fkcc_attach(block, env.v, b.base, env.ext)
                                                 : R.fkcc(block, env.v, b.base, env.ext);
    int32_t done = 1;
    if (valid && ne > 1) {
        V back[kMaxDim];
        for (int j = 0; j < D; ++j) back[j] = V(v[j] / (float)(8 * (int64_t)ne));  // validate.hh:50
        for (int32_t i = 1; i < ne; ++i) {
            for (int j = 0; j < D; ++j) block[j] = block[j] - back[j];  // validate.hh:52-56
            ++done;
            if (!R.fkcc(block, env.v, b.base, env.ext)) {
                valid = false;
                break;
            }
        }
    }
    if (evaluated) *evaluated = done;
    return valid;
}

// full-mask mode: every block of the edge evaluated (no early exit), block_ok[0 .. n_e - 1]
bool validate_all_blocks(const Bound& b, const Env& env, const float* start, const float* goal, uint8_t* block_ok)
{
    const RobotCpu& R = *b.R;
    const int D = R.dim;
    float v[kMaxDim];
    for (int j = 0; j < D; ++j) v[j] = goal[j] - start[j];
    const float distance = l2_norm(v, D);
    const V pct = _mm256_setr_ps(1.0f / 8, 2.0f / 8, 3.0f / 8, 4.0f / 8, 5.0f / 8, 6.0f / 8, 7.0f / 8, 1.0f);
    V block[kMaxDim];
    for (int j = 0; j < D; ++j) block[j] = fma(V(v[j]), pct, V(start[j]));
    float nf = std::ceil(distance / 8.0f * (float)R.resolution);
    if (!(nf > 1.0f)) nf = 1.0f;
    const int32_t ne = nf < 2147483520.0f ? (int32_t)nf : 2147483520;
    bool all = block_ok[0] = (env.attached && R.fkcc_attach) ? R.fkcc_attach(block, env.v, b.base, env.ext)
                                                              : R.fkcc(block, env.v, b.base, env.ext);
    V back[kMaxDim];
    for (int j = 0; j < D; ++j) back[j] = V(v[j] / (float)(8 * (int64_t)ne));
    for (int32_t i = 1; i < ne; ++i) {
        for (int j = 0; j < D; ++j) block[j] = block[j] - back[j];
        block_ok[i] = R.fkcc(block, env.v, b.base, env.ext) ? 1 : 0;
        all = all && block_ok[i];
    }
    return all;
}

// validate_motion<Robot, 8, Robot::resolution> (planning/validate.hh:67-75)
bool validate_one(const Bound& b, const Env& env, const float* start, const float* goal, int32_t* n,
                  int32_t* evaluated)
{
    float v[kMaxDim];
    for (int j = 0; j < b.R->dim; ++j) v[j] = goal[j] - start[j];                   // validate.hh:72
    return validate_vector_one(b, env, start, v, l2_norm(v, b.R->dim), n, evaluated);  // validate.hh:73
}

// static contiguous chunks, one std::thread each (SURVEY §8(d) CPU reference timing)
template <class Fn>
void parallel_for(size_t n, int threads, Fn fn)
{
    const size_t T = (size_t)std::max(1, std::min<int>(threads, (int)std::max<size_t>(1, n)));
    if (T == 1) {
        fn(0, n);
        return;
    }
    // a chunk whose thread cannot be started (std::system_error) runs on the calling thread: the started
    // threads are always joined, so no exception leaves through a joinable std::thread
    std::vector<std::thread> pool;
    pool.reserve(T);
    size_t t = 0;
    try {
        for (; t < T; ++t) {
            const size_t lo = n * t / T, hi = n * (t + 1) / T;
            pool.emplace_back([=] { fn(lo, hi); });
        }
    } catch (...) {
    }
    if (t < T) fn(n * t / T, n);
    for (auto& th : pool) th.join();
}

int resolve_threads(int threads)
{
    if (threads > 0) return threads;
    const unsigned hw = std::thread::hardware_concurrency();
    return hw ? (int)hw : 1;
}

// Robot::eefk (panda/fk.hh:11399-11650, fetch/fk.hh:30993, ur5/fk.hh:5868): the end-effector
// frame's pose in the robot frame (no base offset: PandaBase<...>::eefk = panda::eefk).  The
// reference's generated eefk computes in double (its temporaries are float * double literals,
// std::sin / std::cos of the half angles) and narrows the result to float; this walks the same
// chain in double from the model data (csrc/gen/cpu/eefk_tables.inc).
struct EeFrame {
    int parent;
    double qf[4];  // w x y z
    double t[3];
    int dof, prismatic;
    double axis[3];
};
#include "../gen/cpu/eefk_tables.inc"

static void qmul_d(const double* a, const double* b, double* o)
{
    o[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    o[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    o[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    o[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}
static void rot_d(const double* q, const double* v, double* o)  // R(q) v
{
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    o[0] = (1 - 2 * (y * y + z * z)) * v[0] + 2 * (x * y - w * z) * v[1] + 2 * (x * z + w * y) * v[2];
    o[1] = 2 * (x * y + w * z) * v[0] + (1 - 2 * (x * x + z * z)) * v[1] + 2 * (y * z - w * x) * v[2];
    o[2] = 2 * (x * z - w * y) * v[0] + 2 * (y * z + w * x) * v[1] + (1 - 2 * (x * x + y * y)) * v[2];
}

}  // namespace vcpu

using namespace vcpu;

extern "C" float vgpu_l2_norm(const float* v, int dim)
{
    if (!v || dim < 1 || dim > 16) return std::numeric_limits<float>::quiet_NaN();
    return l2_norm(v, dim);
}

extern "C" int vgpu_robot_scale_params(const vgpu_robot* robot, float* s_m, float* s_a, float* d_m)
try {
    Bound b;
    if (int rc = bind(robot, b)) return rc;
    for (int j = 0; j < b.R->dim; ++j) {
        if (s_m) s_m[j] = b.R->s_m[j];
        if (s_a) s_a[j] = b.R->s_a[j];
        if (d_m) d_m[j] = b.R->d_m[j];
    }
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_eefk(const vgpu_robot* robot, const float* q, size_t n, float* pose)
try {
    if (!robot || (n && (!q || !pose))) return VGPU_ERR_INVALID_ARG;
    Bound b;
    if (int rc = bind(robot, b)) return rc;
    int len = 0;
    const EeFrame* chain = ee_chain(robot->kind, &len);
    if (!chain) return VGPU_ERR_UNSUPPORTED;  // the composite has none; Baxter's eefk is empty (baxter/fk.hh)
    const int D = b.R->dim;
    std::vector<double> Q(4 * (size_t)len), P(3 * (size_t)len);
    for (size_t i = 0; i < n; ++i) {
        const float* qi = q + (size_t)D * i;
        for (int f = 0; f < len; ++f) {
            const EeFrame& fr = chain[f];
            double* qc = &Q[4 * (size_t)f];
            double* pc = &P[3 * (size_t)f];
            if (fr.parent < 0) {
                qc[0] = 1, qc[1] = qc[2] = qc[3] = 0;
                pc[0] = pc[1] = pc[2] = 0;
                continue;
            }
            const double* qp = &Q[4 * (size_t)fr.parent];
            const double* pp = &P[3 * (size_t)fr.parent];
            double a[4], tv[3];
            qmul_d(qp, fr.qf, a);
            rot_d(qp, fr.t, tv);
            for (int k = 0; k < 3; ++k) pc[k] = pp[k] + tv[k];
            if (fr.dof >= 0 && fr.prismatic) {
                const double d[3] = {(double)qi[fr.dof] * fr.axis[0], (double)qi[fr.dof] * fr.axis[1],
                                     (double)qi[fr.dof] * fr.axis[2]};
                double dv[3];
                rot_d(a, d, dv);
                for (int k = 0; k < 3; ++k) pc[k] += dv[k];
                std::copy(a, a + 4, qc);
            } else if (fr.dof >= 0) {
                const double h = (double)qi[fr.dof] * 0.5;
                const double s = std::sin(h);
                const double j[4] = {std::cos(h), s * fr.axis[0], s * fr.axis[1], s * fr.axis[2]};
                qmul_d(a, j, qc);
            } else {
                std::copy(a, a + 4, qc);
            }
        }
        const double* qe = &Q[4 * (size_t)(len - 1)];
        const double* pe = &P[3 * (size_t)(len - 1)];
        float* o = pose + 7 * i;  // x y z, quaternion x y z w (bindings/common.hh:342-352)
        o[0] = (float)pe[0], o[1] = (float)pe[1], o[2] = (float)pe[2];
        o[3] = (float)qe[1], o[4] = (float)qe[2], o[5] = (float)qe[3], o[6] = (float)qe[0];
    }
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_fkcc_block(const vgpu_robot* robot, vgpu_env* env, const float* block, int* valid)
try {
    Bound b;
    Env e;
    if (!block || !valid) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (int rc = view(env, e)) return rc;
    V q[kMaxDim];
    for (int j = 0; j < b.R->dim; ++j) q[j] = V(_mm256_loadu_ps(block + 8 * j));
    *valid = b.R->fkcc(q, e.v, b.base, e.ext) ? 1 : 0;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_fkcc_attach_block(const vgpu_robot* robot, vgpu_env* env, const float* block, int* valid)
try {
    Bound b;
    Env e;
    if (!block || !valid) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (!b.R->fkcc_attach) return VGPU_ERR_UNSUPPORTED;
    if (int rc = view(env, e)) return rc;
    if (!e.attached) return VGPU_ERR_INVALID_ARG;
    V q[kMaxDim];
    for (int j = 0; j < b.R->dim; ++j) q[j] = V(_mm256_loadu_ps(block + 8 * j));
    *valid = b.R->fkcc_attach(q, e.v, b.base, e.ext) ? 1 : 0;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_sphere_fk_block(const vgpu_robot* robot, const float* block, float* out)
try {
    Bound b;
    if (!block || !out) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    V q[kMaxDim];
    for (int j = 0; j < b.R->dim; ++j) q[j] = V(_mm256_loadu_ps(block + 8 * j));
    std::vector<V> o((size_t)3 * b.R->n_spheres);
    b.R->sphere_fk(q, b.base, o.data());
    for (size_t i = 0; i < o.size(); ++i) _mm256_storeu_ps(out + 8 * i, o[i].v);
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_validate_motion(const vgpu_robot* robot, vgpu_env* env, const float* start,
                                        const float* goal, int* valid)
try {
    Bound b;
    Env e;
    if (!start || !goal || !valid) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (int rc = view(env, e)) return rc;
    if (e.attached && !b.R->fkcc_attach) return VGPU_ERR_UNSUPPORTED;
    *valid = validate_one(b, e, start, goal, nullptr, nullptr) ? 1 : 0;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_validate_vector(const vgpu_robot* robot, vgpu_env* env, const float* start,
                                        const float* vector, float distance, int* valid)
try {
    Bound b;
    Env e;
    if (!start || !vector || !valid) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (int rc = view(env, e)) return rc;
    if (e.attached && !b.R->fkcc_attach) return VGPU_ERR_UNSUPPORTED;
    *valid = validate_vector_one(b, e, start, vector, distance, nullptr, nullptr) ? 1 : 0;
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_fkcc(const vgpu_robot* robot, vgpu_env* env, const float* q, size_t n, uint8_t* valid,
                             int threads)
try {
    Bound b;
    Env e;
    if ((n && (!q || !valid))) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (int rc = view(env, e)) return rc;
    const int D = b.R->dim;
    parallel_for(n, resolve_threads(threads), [&](size_t lo, size_t hi) {
        V blk[kMaxDim];
        for (size_t i = lo; i < hi; ++i) {
            for (int j = 0; j < D; ++j) blk[j] = V(q[(size_t)D * i + j]);  // the broadcast block of validate(q)
            valid[i] = b.R->fkcc(blk, e.v, b.base, e.ext) ? 1 : 0;
        }
    });
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_fkcc_attach(const vgpu_robot* robot, vgpu_env* env, const float* q, size_t n,
                                    uint8_t* valid, int threads)
try {
    Bound b;
    Env e;
    if ((n && (!q || !valid))) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (!b.R->fkcc_attach) return VGPU_ERR_UNSUPPORTED;
    if (int rc = view(env, e)) return rc;
    if (!e.attached) return VGPU_ERR_INVALID_ARG;
    const int D = b.R->dim;
    parallel_for(n, resolve_threads(threads), [&](size_t lo, size_t hi) {
        V blk[kMaxDim];
        for (size_t i = lo; i < hi; ++i) {
            for (int j = 0; j < D; ++j) blk[j] = V(q[(size_t)D * i + j]);
            valid[i] = b.R->fkcc_attach(blk, e.v, b.base, e.ext) ? 1 : 0;
        }
    });
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_validate_motions_mask(const vgpu_robot* robot, vgpu_env* env, const float* starts,
                                              const float* goals, size_t n, uint8_t* ok, int32_t* n_blocks,
                                              uint8_t* block_ok, size_t block_cap, size_t* n_total, int threads)
try {
    Bound b;
    Env e;
    if (!n_total || (n && (!starts || !goals || !ok))) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (int rc = view(env, e)) return rc;
    if (e.attached && !b.R->fkcc_attach) return VGPU_ERR_UNSUPPORTED;
    const int D = b.R->dim;
    std::vector<size_t> off(n + 1, 0);  // n_e of every edge first (validate.hh:41), then their offsets
    for (size_t i = 0; i < n; ++i) {
        float v[kMaxDim];
        for (int j = 0; j < D; ++j) v[j] = goals[(size_t)D * i + j] - starts[(size_t)D * i + j];
        float nf = std::ceil(l2_norm(v, D) / 8.0f * (float)b.R->resolution);
        if (!(nf > 1.0f)) nf = 1.0f;
        off[i + 1] = off[i] + (size_t)(nf < 2147483520.0f ? nf : 2147483520.0f);
    }
    *n_total = off[n];
    if (!block_ok || block_cap < off[n]) return VGPU_ERR_INVALID_ARG;
    parallel_for(n, resolve_threads(threads), [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            ok[i] = validate_all_blocks(b, e, starts + (size_t)D * i, goals + (size_t)D * i, block_ok + off[i]) ? 1 : 0;
            if (n_blocks) n_blocks[i] = (int32_t)(off[i + 1] - off[i]);
        }
    });
    return VGPU_OK;
} VGPU_ABI_CATCH

extern "C" int vgpu_cpu_validate_motions(const vgpu_robot* robot, vgpu_env* env, const float* starts,
                                         const float* goals, size_t n, uint8_t* ok, int32_t* n_blocks,
                                         int32_t* n_evaluated, int threads)
try {
    Bound b;
    Env e;
    if (n && (!starts || !goals || !ok)) return VGPU_ERR_INVALID_ARG;
    if (int rc = bind(robot, b)) return rc;
    if (int rc = view(env, e)) return rc;
    if (e.attached && !b.R->fkcc_attach) return VGPU_ERR_UNSUPPORTED;
    const int D = b.R->dim;
    parallel_for(n, resolve_threads(threads), [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            int32_t ne = 0, ev = 0;
            ok[i] = validate_one(b, e, starts + (size_t)D * i, goals + (size_t)D * i, &ne, &ev) ? 1 : 0;
            if (n_blocks) n_blocks[i] = ne;
            if (n_evaluated) n_evaluated[i] = ev;
        }
    });
    return VGPU_OK;
} VGPU_ABI_CATCH
