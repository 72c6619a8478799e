/* vamp_gpu.h -- C ABI of the MI355X (gfx950) motion-validation rake.
 *
 * Drop-in boundary for the reference's hot path (jamesmotes/mr-vamp):
 *   vamp::planning::validate_motion / validate_vector  (src/impl/vamp/planning/validate.hh:23-75)
 *   Robot::fkcc<rake>                                 (src/impl/vamp/robots/panda_base.hh:53-58)
 *   Robot::sphere_fk<rake>                            (src/impl/vamp/robots/panda_base.hh:67-71)
 *   collision::Environment<float> + Environment.add_* (src/impl/vamp/collision/environment.hh:12-66,
 *                                                     src/impl/vamp/bindings/environment.cc:107-146)
 * The reference entry points take one edge / one 8-lane block per call; this ABI takes
 * batches (see INTEGRATION.md for the cgo/ctypes/C++ bindings a maintainer would add).
 *
 * Conventions
 *   - Every function returns int: VGPU_OK (0) or a negative VGPU_ERR_* code; the message
 *     is available from vgpu_last_error(ctx).  No C++ exception crosses this boundary.
 *   - Batch functions take DEVICE pointers and are stream-ordered on the context's stream
 *     (vgpu_ctx_set_stream / vgpu_sync): inputs are read and outputs written by work enqueued
 *     on that stream.  Work sizes that depend on the data are read back with a blocking 4-byte
 *     copy, so these calls are NOT fully asynchronous: a staged pass (fkcc, sample_fkcc, the
 *     head and tail of validate_motions) reads its first round's per-check counts once (the
 *     later rounds' layout is computed on the device), and validate_motions reads its
 *     back-step item count once -- 3 host syncs per staged validate_motions call.  The
 *     monolithic robots (Baxter, the composite) sync once per validate_motions call.
 *     The *_host variants copy in and out and synchronise (convenience; they measure PCIe,
 *     not the kernels).
 *   - Configurations are row-major float32 [n][dim] (reference ConfigurationArray).
 *   - Results use the reference's polarity: 1 = valid (collision-free), 0 = in collision.
 *   - A context is bound to one HIP device and must be used from one host thread at a time.
 */
#ifndef VAMP_GPU_H
#define VAMP_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VGPU_OK 0
#define VGPU_ERR_INVALID_ARG (-1)
#define VGPU_ERR_HIP (-2)
#define VGPU_ERR_OOM (-3)
#define VGPU_ERR_UNSUPPORTED (-4)
#define VGPU_ERR_RSQRT (-5)
#define VGPU_ERR_INTERNAL (-6) /* an unexpected C++ exception inside the library (none crosses this ABI) */

typedef struct vgpu_ctx vgpu_ctx;
typedef struct vgpu_env vgpu_env;

/* Robot selection.  kind = VGPU_ROBOT_PANDA reproduces vamp::robots::PandaBase<X100, Y100, Z100>
 * (robots/panda_base.hh:15-75); the fork's default vamp::robots::Panda is base (200, 200, 0)
 * (robots/panda_grid.hh:39). */
#define VGPU_ROBOT_PANDA 1
/* kind = VGPU_ROBOT_FETCH reproduces vamp::robots::Fetch (robots/fetch.hh:8-48): 8 dof (prismatic
 * torso + 7 revolute), 111 spheres, resolution 32, no base offset (base_*100 must be 0). */
#define VGPU_ROBOT_FETCH 2
/* kind = VGPU_ROBOT_PANDA_PAIR: the two-Panda composite of BASELINE configs[4] (14 dof: arm A =
 * joints 0..6 at base (base_*100), arm B = joints 7..13 at base (base2_*100); resolution 32).
 * The reference has no composite robot; validity = fkcc_A && fkcc_B && no A-B sphere overlap
 * (link-bounding pairs first), composed from the reference primitives. */
#define VGPU_ROBOT_PANDA_PAIR 3
/* kind = VGPU_ROBOT_UR5: vamp::robots::UR5 (robots/ur5.hh: 6 dof, 36 spheres, resolution 32);
 * kind = VGPU_ROBOT_BAXTER: vamp::robots::Baxter (robots/baxter.hh: 14-dof dual arm, 75 spheres,
 * resolution 64).  Neither has a base offset (base_*100 must be 0). */
#define VGPU_ROBOT_UR5 4
#define VGPU_ROBOT_BAXTER 5
typedef struct vgpu_robot {
    int32_t kind;
    int32_t base_x100, base_y100, base_z100;
    int32_t base2_x100, base2_y100, base2_z100; /* second arm (VGPU_ROBOT_PANDA_PAIR only) */
} vgpu_robot;

/* ---- context -------------------------------------------------------------------------- */
/* Creates a context on HIP device `device` and probes the host CPU's rsqrt approximation
 * (the reference culls with v * _mm256_rsqrt_ps(v), vector/avx.hh:411-415), uploading it
 * to the device.  Fails with VGPU_ERR_RSQRT if the host rsqrt is not table-representable. */
int vgpu_ctx_create(int device, vgpu_ctx **out);
void vgpu_ctx_destroy(vgpu_ctx *ctx);
const char *vgpu_last_error(const vgpu_ctx *ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL restores
 * the context's own stream. */
int vgpu_ctx_set_stream(vgpu_ctx *ctx, void *hip_stream);
int vgpu_sync(vgpu_ctx *ctx);
/* the HIP device the context was created on */
int vgpu_ctx_device(const vgpu_ctx *ctx, int *device);
/* Debug builds (make -C mr-vamp_amd DEBUG=1 -> vamp_amd/libvampgpu_debug.so): bounds checks on the
 * data-dependent indices of the staged, CAPT and kNN-index kernels; a failed check is counted (the index
 * clamped, no fault).  vgpu_debug_build() = 1 in such a build.  vgpu_debug_violations reads and resets the
 * counters of the context and (optional) of an environment's device copy: out[0] = violations, out[1] =
 * the first failing site (vgpu_device.hh DBG_*). */
int vgpu_debug_build(void);
int vgpu_debug_violations(vgpu_ctx *ctx, vgpu_env *env, uint32_t out[2]);
/* Per-phase kernel timing of vgpu_validate_motions (HIP events on the context stream; adds
 * one event synchronisation per call while enabled).  vgpu_phase_times returns and resets the
 * accumulated milliseconds: [0] head (first rake block), [1] scan + item count read-back,
 * [2] scatter + tail (back-step blocks), [3] number of calls. */
int vgpu_ctx_set_profiling(vgpu_ctx *ctx, int enable);
int vgpu_phase_times(vgpu_ctx *ctx, float ms[4]);
/* rsqrt table in use: kbits and the 2 << kbits entries (host copy).  Replacing it is for
 * testing cross-host parity only. */
int vgpu_rsqrt_table(const vgpu_ctx *ctx, int *kbits, const uint32_t **table);
int vgpu_rsqrt_table_set(vgpu_ctx *ctx, const uint32_t *table, int kbits);

/* ---- environment (collision::Environment<float>) ---------------------------------------- */
/* ctx may be NULL for a host-only environment (built and inspected, never uploaded). */
int vgpu_env_create(vgpu_ctx *ctx, vgpu_env **out);
void vgpu_env_destroy(vgpu_env *env);
/* Shape constructors of collision/shapes.hh + factory.hh, with the routing of
 * bindings/environment.cc:107-146 (axis_3_z == 1 -> z-aligned cuboid; xv == yv == 0 ->
 * z-aligned capsule) and the min_distance sort of environment.hh:40-66. */
int vgpu_env_add_sphere(vgpu_env *env, const float center[3], float radius);
int vgpu_env_add_cuboid_axes(vgpu_env *env, const float center[3], const float axis_1[3], const float axis_2[3],
                             const float axis_3[3], const float half_extents[3]);
int vgpu_env_add_cuboid_euler(vgpu_env *env, const float center[3], const float euler_xyz[3],
                              const float half_extents[3]);
int vgpu_env_add_capsule_endpoints(vgpu_env *env, const float p1[3], const float p2[3], float radius);
int vgpu_env_add_capsule_euler(vgpu_env *env, const float center[3], const float euler_xyz[3], float radius,
                               float length);
/* obstacle counts: spheres, capsules, z-capsules, cuboids, z-cuboids */
int vgpu_env_counts(const vgpu_env *env, int32_t counts[5]);

/* Environment::add_heightfield(factory::heightfield::array(center, scale, {xd, yd}, data))
 * (bindings/environment.cc:96,144-147; factory.hh:365-423): data row-major xd*yd floats. */
int vgpu_env_add_heightfield(vgpu_env *env, const float center[3], const float scale[3], size_t xd, size_t yd,
                             const float *data);
/* Environment::add_pointcloud(points, r_min, r_max, r_point) (bindings/environment.cc:148-158):
 * builds a CAPT (collision/capt.hh:327-398) on the host; *build_ns (optional) = build time. */
int vgpu_env_add_pointcloud(vgpu_env *env, const float *points, size_t n, float r_min, float r_max,
                            float r_point, int64_t *build_ns);
/* The same CAPT built on the DEVICE (vgpu_capt_build.hip) from device points
 * (n x 3 float32, finite -- not checked), e.g. straight from vgpu_filter_pointcloud's output: the
 * median splits, affordance lists and leaf packing run level by level on ctx's stream, and the
 * arrays (bit-identical to vgpu_env_add_pointcloud's) are appended to env (ctx's environment or a
 * host-only one).  Synchronises the stream (array sizes are data-dependent). */
int vgpu_env_add_pointcloud_device(vgpu_ctx *ctx, vgpu_env *env, const float *points, size_t n, float r_min,
                                   float r_max, float r_point, int64_t *build_ns);
/* Appends a copy of point cloud `index` of src (its built CAPT arrays, host memory) to dst -- e.g.
 * to realise an environment whose cloud was built once (host or device) on another context without
 * rebuilding it or keeping the points alive. */
int vgpu_env_copy_pointcloud(vgpu_env *dst, const vgpu_env *src, int index);
/* counts[0] = heightfields, counts[1] = point clouds */
int vgpu_env_ext_counts(const vgpu_env *env, int32_t counts[2]);
/* the built CAPT of point cloud `index`: 2^nlog2 leaves, n_aff affordance vectors, top box */
int vgpu_env_pointcloud_info(const vgpu_env *env, int index, int32_t *nlog2, size_t *n_aff, float top[6]);
/* copies of its arrays: tests[2^nlog2-1], aabbs[2^nlog2][6], aff_starts[2^nlog2+1],
 * aff[n_aff][3][8] (any pointer may be NULL) */
int vgpu_env_pointcloud_arrays(const vgpu_env *env, int index, float *tests, float *aabbs, uint32_t *aff_starts,
                               float *aff);
/* Environment::attach(Attachment) (bindings/environment.cc:161-162): one attachment, replacing
 * any previous one.  tf = relative frame x y z, quaternion x y z w (Attachment(center,
 * quaternion_xyzw), environment.cc:197-215); spheres[n][4] = x y z r relative to it
 * (Attachment::add_spheres, :226-233).  validate_motions then checks the first rake block
 * through Robot::fkcc_attach (planning/validate.hh:43): Panda, Fetch and UR5 have generated
 * attachment checks; the Baxter's fkcc_attach is its plain fkcc (baxter.hh:44); the composite
 * has none (VGPU_ERR_UNSUPPORTED). */
int vgpu_env_attach(vgpu_env *env, const float tf[7], const float *spheres, size_t n);
/* Environment::detach (environment.cc:163) */
int vgpu_env_detach(vgpu_env *env);
/* Copy the (sorted) environment to the device.  Called implicitly by the batch functions
 * when the environment changed since the last upload.  Incremental: the point clouds (CAPT arrays
 * and their cell grids) form the blob's prefix and are re-sent -- and their grids rebuilt -- only when
 * a cloud was added; obstacles, heightfields and the attachment (add_*, attach, detach) form the tail,
 * rewritten in place (environment.cc:107-163 mutate the reference's environment just as cheaply). */
int vgpu_env_upload(vgpu_env *env);
/* out[0] whole-blob uploads, out[1] tail-only uploads, out[2] cell-grid builds of this environment */
int vgpu_env_upload_stats(const vgpu_env *env, uint64_t out[3]);
/* point cloud `index`'s cell grid as the uploaded device header records it: {nx, ny, nz, cells_off} */
int vgpu_env_pointcloud_grid(vgpu_env *env, int index, uint32_t out[4]);

/* ---- batched hot path (device pointers, asynchronous) ------------------------------------ */
/* Robot::sphere_fk for n configurations q[n][dim] -> xyz[3][n_spheres][ld] (SoA, world frame,
 * base offset added).  ld >= n. */
int vgpu_sphere_fk(vgpu_ctx *ctx, const vgpu_robot *robot, const float *q, size_t n, float *xyz, size_t ld);
/* Robot::fkcc<rake> of each configuration broadcast to the whole rake (the per-configuration
 * mask, as used by validate(q) and the PRM sampler): valid[i] = 1 if q[i] is collision-free. */
int vgpu_fkcc(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *q, size_t n, uint8_t *valid);
/* Robot::fkcc_attach<rake> (robots/panda_base.hh:61-65, fetch.hh:42, ur5.hh:43) of each
 * configuration broadcast to the rake, with the environment's attachment posed at the end
 * effector; requires an attachment (vgpu_env_attach).  Panda, Fetch, UR5 (Baxter: = vgpu_fkcc). */
int vgpu_fkcc_attach(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *q, size_t n,
                     uint8_t *valid);
/* validate_motion<Robot, 8, Robot::resolution>(starts[i], goals[i], env) for every edge:
 * ok[i] = 1 if the whole edge is valid.  n_blocks (optional) receives n_e, the rake
 * back-step count of validate.hh:41 (interpolants = 8 * n_e). */
int vgpu_validate_motions(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *starts,
                          const float *goals, size_t n_edges, uint8_t *ok, int32_t *n_blocks);

/* Full-mask mode: validate_motion's rake blocks ALL evaluated, with no early exit
 * across an edge's blocks, and every block's result kept: block_ok[total] holds edge 0's blocks
 * 0 .. n_0 - 1, then edge 1's, ...; ok[i] = AND of edge i's blocks (== vgpu_validate_motions' ok).
 * *n_total = sum of n_e; fails with VGPU_ERR_INVALID_ARG when block_cap < *n_total (call again with a
 * larger buffer).  Synchronises once (the block count).  Panda only; no attachments. */
int vgpu_validate_motions_mask(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *starts,
                               const float *goals, size_t n_edges, uint8_t *ok, int32_t *n_blocks, uint8_t *block_ok,
                               size_t block_cap, size_t *n_total);

/* ---- host-pointer conveniences (copy + synchronise) ---------------------------------------- */
/* Raw sphere queries against point cloud `index`: simd = 0 -> CAPT::collides(center, r)
 * (capt.hh:403-443); simd = 1 -> one lane of CAPT::collides_simd (capt.hh:457-541).
 * centers[n][3], radii[n] -> out[n] (1 = collision). */
int vgpu_pointcloud_collides(vgpu_ctx *ctx, vgpu_env *env, int index, const float *centers, const float *radii,
                             size_t n, int simd, uint8_t *out);

/* ---- sampling (PRM vertex stage) ---------------------------------------- */
/* rng::Halton<dim>::next (random/halton.hh:73-104): draws first .. first+n-1 of a fresh sampler
 * (first >= 1; the reference resets every 1e6 draws and rotates the bases), out[n][dim]. */
int vgpu_halton(vgpu_ctx *ctx, int dim, uint64_t first, size_t n, float *out);
/* Halton<dimension> draws scaled by Robot::scale_configuration (panda/fk.hh:34-37): q[n][dim] */
int vgpu_sample_configurations(vgpu_ctx *ctx, const vgpu_robot *robot, uint64_t first, size_t n, float *q);
/* the same fused with the per-configuration fkcc (prm.hh:236-251); q may be NULL */
int vgpu_sample_fkcc(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, uint64_t first, size_t n, float *q,
                     uint8_t *valid);
/* stream compaction of the rows whose flag is set: index_out[*count] ascending, rows_out (if not
 * NULL) = the selected rows[dim].  Synchronises to return *count (host). */
int vgpu_compact(vgpu_ctx *ctx, const float *rows, const uint8_t *valid, size_t n, int dim, float *rows_out,
                 uint32_t *index_out, size_t *count);

int vgpu_sphere_fk_host(vgpu_ctx *ctx, const vgpu_robot *robot, const float *q, size_t n, float *xyz);
int vgpu_fkcc_host(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *q, size_t n,
                   uint8_t *valid);
int vgpu_fkcc_attach_host(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *q, size_t n,
                          uint8_t *valid);
int vgpu_validate_motions_host(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *starts,
                               const float *goals, size_t n_edges, uint8_t *ok, int32_t *n_blocks);

/* ---- PRM roadmap edge stage (planning/prm.hh:235-299) ------------------------------------ */
/* PRMStarNeighborParams(dim, space_measure) with gamma_scale (roadmap.hh:42-77, bindings
 * settings.cc:38-44): k[i] = max_neighbors(i), r[i] = neighbor_radius(i) for roadmap sizes
 * i = 0 .. n-1 (k = 0 for i < 2: start and goal are inserted without a query). */
int vgpu_prm_neighbor_params(int dim, double space_measure, double gamma_scale, size_t n, uint32_t *k, float *r);
/* The neighbour query build_roadmap runs for every vertex i (prm.hh:264-266, NN::nearest on
 * the vertices 0 .. i-1): at most k[i] of them within r[i] (distance <= r), nearest first,
 * distance = Space<dim>::distance (nn.hh:53-57).  Device pointers: V[n][dim] -> nbr[n][kmax],
 * dist[n][kmax], cnt[n].  dim in {6, 7, 8, 14}, kmax <= 64. */
int vgpu_roadmap_knn(vgpu_ctx *ctx, int dim, const float *V, size_t n, const uint32_t *k, const float *r,
                     uint32_t kmax, uint32_t *nbr, float *dist, uint32_t *cnt);
/* Neighbour-query method of the context: 0 auto (a spatial index -- Morton-sorted tiles with
 * box culling, vgpu_knn_index.hip -- from 65536 vertices, else the brute-force scan), 1 brute
 * force, 2 index.  Both give the same lists (the k smallest (distance, index) keys within r). */
int vgpu_set_knn_mode(vgpu_ctx *ctx, int mode);
/* The same for the queries q_first .. q_first+q_count-1 only (one rank's share of the edge
 * stage); nbr/dist/cnt are indexed from q_first, V holds all n vertices. */
int vgpu_roadmap_knn_range(vgpu_ctx *ctx, int dim, const float *V, size_t n, size_t q_first, size_t q_count,
                           const uint32_t *k, const float *r, uint32_t kmax, uint32_t *nbr, float *dist,
                           uint32_t *cnt);
/* Candidate edges of queries q_first .. +q_count (device): edge off[i] + m = (nbr[i][m] -> vertex
 * q_first + i) for m < cnt[i], as starts[e][dim] = V[nbr], goals[e][dim] = V[vertex] -- the
 * arguments of validate_motion(neighbor, vertex) (prm.hh:268). */
int vgpu_roadmap_edge_gather(vgpu_ctx *ctx, int dim, const float *V, size_t q_first, size_t q_count,
                             const uint32_t *nbr, uint32_t kmax, const uint32_t *cnt, const uint32_t *off,
                             float *starts, float *goals);
/* Host: the adjacency build_roadmap appends (prm.hh:270-275) from the valid (vertex i, neighbour
 * j) pairs[m][2] listed in query order (i ascending, nearest first): offsets[n+1], adj[2m] (each
 * vertex: its own neighbours, then the later vertices that connected to it, ascending);
 * component (optional) = smallest vertex index of each vertex's connected component. */
int vgpu_roadmap_assemble(size_t n, const uint32_t *pairs, size_t m, size_t *offsets, uint32_t *adj,
                          uint32_t *component);
/* The same on the device (mr-vamp_amd/csrc/vgpu_roadmap_assemble.hip): pairs[m][2], offsets[n+1] (uint64),
 * adj[2m], component[n] (optional) all device memory on ctx; identical output.  2m < 2^31; a pair
 * index >= n fails with VGPU_ERR_INVALID_ARG.  Synchronous (one host read per hooking round). */
int vgpu_roadmap_assemble_device(vgpu_ctx *ctx, size_t n, const uint32_t *pairs, size_t m, uint64_t *offsets,
                                 uint32_t *adj, uint32_t *component);
/* Roadmap::build_roadmap's graph for the vertex sequence V[n][dim] (start, goal, then the valid
 * samples in draw order -- vgpu_sample_fkcc + vgpu_compact): every vertex's neighbour query,
 * validate_motion(neighbor, vertex) of every candidate on the GPU, and the adjacency lists in
 * the reference's append order (prm.hh:270-275, Roadmap::edges): offsets[n+1], adj[*n_adj].
 * If adj_cap < *n_adj the call fails with VGPU_ERR_INVALID_ARG and *n_adj = the required size.
 * component (optional) = smallest vertex index of each vertex's connected component. */
int vgpu_build_roadmap_host(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *V, size_t n,
                            double space_measure, double gamma_scale, size_t *offsets, uint32_t *adj,
                            size_t adj_cap, size_t *n_adj, uint32_t *component);

/* ---- CPU rake (host AVX2; no context, no GPU) --------------------------------------------------- */
/* The reference's single-call entry points stay on the CPU (a GPU launch costs far more than one
 * ~2 us edge): the same generated op sequence as the kernels over one 8-lane AVX2 register per
 * rake block, culling with this host's own _mm256_rsqrt_ps -- bit-identical to the GPU path and to
 * the oracle.  `env` may be a host-only environment (vgpu_env_create(NULL, ...)).  `threads` <= 0
 * uses every hardware thread; batches are split into static contiguous chunks. */
/* Robot::fkcc<8>(env, block) (robots/panda_base.hh:53-58): block = ConfigurationBlock<8>, dim rows
 * of 8 lanes (SoA, lane l = configuration l); *valid = 1 when every lane is collision-free. */
int vgpu_cpu_fkcc_block(const vgpu_robot *robot, vgpu_env *env, const float *block, int *valid);
/* Robot::fkcc_attach<8>(env, block) (robots/panda_base.hh:61-65); requires an attachment. */
int vgpu_cpu_fkcc_attach_block(const vgpu_robot *robot, vgpu_env *env, const float *block, int *valid);
/* Robot::sphere_fk<8>(block, out) (robots/panda_base.hh:67-71): out[3][n_spheres][8] (x, y, z rows). */
int vgpu_cpu_sphere_fk_block(const vgpu_robot *robot, const float *block, float *out);
/* planning::validate_motion<Robot, 8, Robot::resolution>(start, goal, env) (validate.hh:67-75). */
int vgpu_cpu_validate_motion(const vgpu_robot *robot, vgpu_env *env, const float *start, const float *goal,
                             int *valid);
/* Batches (host pointers): fkcc / fkcc_attach of each configuration broadcast to the rake, and
 * validate_motion of each edge; n_blocks (optional) = n_e, n_evaluated (optional) = rake blocks
 * the reference evaluates before the edge's result is known (early exit at the first invalid
 * block: interpolants evaluated = 8 * n_evaluated). */
int vgpu_cpu_fkcc(const vgpu_robot *robot, vgpu_env *env, const float *q, size_t n, uint8_t *valid, int threads);
int vgpu_cpu_fkcc_attach(const vgpu_robot *robot, vgpu_env *env, const float *q, size_t n, uint8_t *valid,
                         int threads);
/* full-mask form (as vgpu_validate_motions_mask): every block evaluated, block_ok[*n_total] edge-major */
int vgpu_cpu_validate_motions_mask(const vgpu_robot *robot, vgpu_env *env, const float *starts, const float *goals,
                                   size_t n_edges, uint8_t *ok, int32_t *n_blocks, uint8_t *block_ok, size_t block_cap,
                                   size_t *n_total, int threads);
int vgpu_cpu_validate_motions(const vgpu_robot *robot, vgpu_env *env, const float *starts, const float *goals,
                              size_t n_edges, uint8_t *ok, int32_t *n_blocks, int32_t *n_evaluated, int threads);

/* Robot::eefk(q) (panda/fk.hh:11399-11650, fetch.hh:47, ur5.hh:48; bindings/common.hh:342-352): the
 * end-effector pose in the robot frame for each q[n][dim]: pose[n][7] = x y z, quaternion x y z w.
 * Double precision internally, as the reference's generated eefk.  Panda, Fetch, UR5 (the Baxter's
 * reference eefk is empty, the composite has none: VGPU_ERR_UNSUPPORTED). */
int vgpu_cpu_eefk(const vgpu_robot *robot, const float *q, size_t n, float *pose);
/* planning::validate_vector<Robot, 8, Robot::resolution>(start, vector, distance, env)
 * (validate.hh:23-65): the caller's distance sets the back-step count (RRT-Connect, rrtc.hh:139). */
int vgpu_cpu_validate_vector(const vgpu_robot *robot, vgpu_env *env, const float *start, const float *vector,
                             float distance, int *valid);

/* ---- RRT-Connect on the CPU rake (BASELINE configs[0]) ------------------------------------------ */
/* vamp::planning::RRTCSettings (planning/rrtc_settings.hh:5-20); defaults: range 2, dynamic_domain 1,
 * radius 4, alpha 1e-4, min_radius 1, balance 1, tree_ratio 1, max_iterations = max_samples =
 * 100000, start_tree_first 1 (the Python layer sets range per robot and 1e6 iterations/samples,
 * src/vamp/__init__.py:80-102). */
typedef struct vgpu_rrtc_settings {
    float range;
    int32_t dynamic_domain;
    float radius, alpha, min_radius;
    int32_t balance;
    float tree_ratio;
    uint64_t max_iterations, max_samples;
    int32_t start_tree_first;
} vgpu_rrtc_settings;
/* vamp::planning::PlanningResult (planning/plan.hh): solved = non-empty path */
typedef struct vgpu_plan_result {
    int32_t solved;
    uint64_t iterations;
    int64_t nanoseconds;
    uint64_t size[2]; /* start tree, goal tree */
    float cost;
    size_t path_len;
} vgpu_plan_result;
/* RRTC<Robot, 8, Robot::resolution>::solve(start, goals, env, settings, rng) (planning/rrtc.hh:33-248)
 * with rng::Halton<dim>: *rng_index is the 1-based index of the sampler's next draw (a fresh sampler:
 * 1; skip(k): +k) and is advanced by the draws taken.  path[path_cap][dim] receives the path; if
 * path_cap < result->path_len the call returns VGPU_ERR_INVALID_ARG with path_len set. */
int vgpu_cpu_rrtc(const vgpu_robot *robot, vgpu_env *env, const float *start, const float *goals, size_t n_goals,
                  const vgpu_rrtc_settings *settings, uint64_t *rng_index, float *path, size_t path_cap,
                  vgpu_plan_result *result);

/* build_roadmap's neighbour queries on the host CPU (the reference's nigh KD-tree role, planning/nn.hh:89-95;
 * mr-vamp_amd/csrc/cpu/vcpu_roadmap.cpp): an exact static k-d tree over V[n][dim] with per-subtree minimum
 * vertex indices, answering the causal query of each listed vertex q = queries[j] (the k[q] nearest of
 * vertices 0 .. q-1 within r[q], Space::distance in the AVX lane order) -- the same lists as
 * vgpu_roadmap_knn.  Rows j of nbr/dist [m][kmax] and cnt[m].  threads <= 0: every hardware thread. */
int vgpu_cpu_roadmap_knn(int dim, const float *V, size_t n, const uint32_t *queries, size_t m, const uint32_t *k,
                         const float *r, uint32_t kmax, uint32_t *nbr, float *dist, uint32_t *cnt, int threads);

/* FloatVector<dim>::l2_norm (vector/interface.hh:402-410): squares summed in the AVX hsum lane order
 * (avx.hh:441-452; above 8 lanes the two registers first as fma(lo, lo, hi * hi), pinned by ref_probe
 * "l2norm"), then std::sqrt.  dim <= 16.  The distance of every planner and NN (nn.hh:53-57). */
float vgpu_l2_norm(const float *v, int dim);

/* ---- robot metadata ------------------------------------------------------------------------ */
/* Robot::scale_configuration / descale_configuration constants (robots/<robot>/fk.hh, e.g. panda/fk.hh:14-
 * 62): q_scaled = fma(q, s_m, s_a), q_unit = (q - s_a) * d_m; dimension floats each (any may be NULL). */
int vgpu_robot_scale_params(const vgpu_robot *robot, float *s_m, float *s_a, float *d_m);
/* dimension, resolution, n_spheres of a robot kind (robots/panda_base.hh:19-23) */
/* Point-cloud filter (replaces vamp::collision::filter_pointcloud, collision/filter.hh:175-268,
 * bound as vamp.filter_pointcloud in bindings/common.hh). pc: n x 3 f32 (device for the first,
 * host for the _host variant). Writes the kept point indices, in the final space-filling-curve
 * order, to out_idx (capacity n) and their number to *count. Equal Morton codes keep their
 * previous order (stable sort; the reference's pdqsort leaves it unspecified). */
int vgpu_filter_pointcloud(vgpu_ctx *ctx, const float *pc, size_t n, float min_dist, float max_range,
                           const float origin[3], const float ws_min[3], const float ws_max[3], int cull,
                           uint32_t *out_idx, size_t *count);
int vgpu_filter_pointcloud_host(vgpu_ctx *ctx, const float *pc, size_t n, float min_dist, float max_range,
                                const float origin[3], const float ws_min[3], const float ws_max[3], int cull,
                                uint32_t *out_idx, size_t *count);

/* vamp.<robot>.filter_from_pointcloud(pointcloud, configuration, environment, point_radius)
 * (replaces binding::filter_robot_from_pointcloud<Robot>, bindings/common.hh:36-87, bound at :713):
 * drops every point (radius point_radius) that overlaps one of the robot's spheres at `configuration`
 * (Robot::sphere_fk<1>, host pointer, dim floats) or collides with the environment.  Device form:
 * pc[n][3] -> keep[n] (1 = kept).  Host form: the kept points, in input order, -> out[*count][3]
 * (capacity n).  Panda (with its base offset), Fetch, UR5, Baxter. */
int vgpu_filter_robot_pointcloud(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, const float *configuration,
                                 const float *pc, size_t n, float point_radius, uint8_t *keep);
int vgpu_filter_robot_pointcloud_host(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env,
                                      const float *configuration, const float *pc, size_t n, float point_radius,
                                      float *out, size_t *count);
int vgpu_pointcloud_collides_host(vgpu_ctx *ctx, vgpu_env *env, int index, const float *centers,
                                  const float *radii, size_t n, int simd, uint8_t *out);
int vgpu_halton_host(vgpu_ctx *ctx, int dim, uint64_t first, size_t n, float *out);
int vgpu_sample_fkcc_host(vgpu_ctx *ctx, const vgpu_robot *robot, vgpu_env *env, uint64_t first, size_t n, float *q,
                          uint8_t *valid);
int vgpu_robot_info(int32_t kind, int32_t *dimension, int32_t *resolution, int32_t *n_spheres);

/* ---- multi-GPU at the C level (mr-vamp_amd/csrc/vgpu_multi.cpp) ----------------------- */
/* Contiguous shard [*first, *first + *count) of n units owned by `rank` of `world` (balanced: sizes differ
 * by at most one).  The split of edges, configurations and Halton draws over devices or ranks. */
int vgpu_shard_range(size_t n, int rank, int world, size_t *first, size_t *count);
/* One process, several devices: one context per device (devices[n]), one host thread per device per call.
 * vgpu_multi_env_create realises a (host-only or any) environment on every device: envs[vgpu_multi_size]
 * (destroy each with vgpu_env_destroy before vgpu_multi_destroy). */
typedef struct vgpu_multi vgpu_multi;
int vgpu_multi_create(const int *devices, int n, vgpu_multi **out);
void vgpu_multi_destroy(vgpu_multi *m);
int vgpu_multi_size(const vgpu_multi *m);
vgpu_ctx *vgpu_multi_context(vgpu_multi *m, int i);
const char *vgpu_multi_last_error(const vgpu_multi *m);
int vgpu_multi_env_create(vgpu_multi *m, const vgpu_env *src, vgpu_env **envs);
/* validate_motion of n edges (host arrays), contiguous ranges per device, results in place */
int vgpu_multi_validate_motions_host(vgpu_multi *m, const vgpu_robot *robot, vgpu_env *const *envs,
                                     const float *starts, const float *goals, size_t n, uint8_t *ok,
                                     int32_t *n_blocks);
/* the PRM vertex stage (prm.hh:235-254) over the devices: the valid draws of first .. first + n_draws - 1
 * in draw order, rows_out[*count][dim] and their 1-based draw indices (capacity n_draws each) */
int vgpu_multi_sample_fkcc_host(vgpu_multi *m, const vgpu_robot *robot, vgpu_env *const *envs, uint64_t first,
                                size_t n_draws, float *rows_out, uint64_t *draws_out, size_t *count);
/* One process per GPU: RCCL communicators (librccl.so.1 loaded at run time; VGPU_ERR_UNSUPPORTED without
 * it).  Rank 0 makes the 128-byte id, the caller ships it to the other ranks (any side channel), every
 * rank calls vgpu_comm_init with its own context current.  Creation is collective and ends in a status
 * all-gather: when any rank fails (its stream or exchange allocation, RCCL, or VGPU_FAULT_INJECT=comm_init
 * [:alloc][@rank]), EVERY rank destroys its communicator and returns the same code (the lowest failing rank's),
 * *comm stays NULL -- no rank is left to block in its first stage's all-gather.  (A rank whose 24-byte word
 * buffer cannot be allocated cannot join that exchange; its peers then fail inside RCCL.) */
typedef struct vgpu_comm vgpu_comm;
int vgpu_comm_unique_id(uint8_t id[128]);
int vgpu_comm_init(vgpu_ctx *ctx, int rank, int world, const uint8_t id[128], vgpu_comm **out);
void vgpu_comm_destroy(vgpu_comm *comm);
/* message of the communicator's last failed call (which rank failed, or what failed here) */
const char *vgpu_comm_last_error(const vgpu_comm *comm);
/* In-process loopback communicators: `world` ranks as host threads of ONE process, each with
 * its own context (on one device or several); the stages' all-gathers become a barrier plus device copies
 * from every peer.  Same stage semantics as RCCL -- it runs the multi-rank logic (rank-order concatenation,
 * count padding, failure words) at world size > 1 without a multi-GPU job.  A rank that does not arrive
 * within VGPU_LOOPBACK_TIMEOUT_S seconds (default 120) makes its peers' exchange fail instead of hang, and
 * the hub stays failed (every later exchange on it fails at once: a late rank never pairs with a later call).
 * vgpu_comm_init_loopback is collective like vgpu_comm_init (one call per rank, from one thread each; the same
 * status exchange).  vgpu_loopback_destroy fails (VGPU_ERR_INVALID_ARG) while communicators still use the hub. */
typedef struct vgpu_loopback vgpu_loopback;
int vgpu_loopback_create(int world, vgpu_loopback **out);
int vgpu_loopback_destroy(vgpu_loopback *hub);
int vgpu_comm_init_loopback(vgpu_ctx *ctx, int rank, vgpu_loopback *hub, vgpu_comm **out);
/* Collective calls below are failure-safe: a rank whose arguments (other than a null comm), allocations or
 * kernels fail still enters the first exchange -- its word buffer is allocated with the communicator --
 * with a failure word in place of its count; then EVERY rank returns the lowest failing rank's error code
 * and nobody blocks in the next all-gather.  Buffers and the exchange stream belong to the communicator
 * (grown on demand, freed by vgpu_comm_destroy); ctx must live on the communicator's device (else
 * VGPU_ERR_INVALID_ARG, reported to every rank).  Fault injection for tests: VGPU_FAULT_INJECT=<site>[@rank]
 * with site prm_vertices|prm_edges followed by ":args" (argument error), ":alloc" (first allocation) or
 * nothing (after every allocation). */
/* The PRM vertex stage of BASELINE configs[3] sharded over the ranks with ONE exchange: this rank's
 * contiguous share of draws first .. first + n_draws_total - 1 through the fused sampler + fkcc +
 * compaction, then an all-gather of the counts and of the count-padded rows and draw indices.  rows[cap][dim]
 * and draws[cap] (device) receive every rank's valid vertices in rank order = draw order, the vertex
 * sequence of build_roadmap after its start and goal; *count alike on every rank. */
int vgpu_prm_vertices_allgather(vgpu_ctx *ctx, vgpu_comm *comm, const vgpu_robot *robot, vgpu_env *env,
                                uint64_t first, size_t n_draws_total, float *rows, uint64_t *draws, size_t cap,
                                size_t *count);
/* Query ranges of the sharded edge stage: equal prefix work (query i scans i vertices), boundaries at
 * floor(n sqrt(k / world) + 0.5). */
int vgpu_query_split(size_t n, int rank, int world, size_t *first, size_t *count);
/* The PRM edge stage of BASELINE configs[3] sharded over the ranks (Roadmap::build_roadmap's graph,
 * prm.hh:255-299, planning/roadmap.hh:49-56): this rank's queries (vgpu_query_split) through the neighbour
 * query, the candidate gather and validate_motion(neighbor, vertex), the valid pairs selected on the device
 * in query order; ONE exchange (counts, then the count-padded pairs); then every rank assembles the whole
 * roadmap on its device in the reference's append order.  V[n][dim] device (identical on all ranks);
 * offsets[n+1] (uint64), adj[adj_cap], component[n] (optional) device; *n_adj = required adjacency
 * entries (2 x valid pairs) -- adj_cap < *n_adj fails with VGPU_ERR_INVALID_ARG on every rank.  Output
 * equals vgpu_build_roadmap_host's for the same vertices. */
int vgpu_prm_edges_allgather(vgpu_ctx *ctx, vgpu_comm *comm, const vgpu_robot *robot, vgpu_env *env, const float *V,
                             size_t n, double space_measure, double gamma_scale, uint64_t *offsets, uint32_t *adj,
                             size_t adj_cap, size_t *n_adj, uint32_t *component);
/* a deep copy of an environment bound to ctx (NULL: host-only) */
int vgpu_env_clone(const vgpu_env *src, vgpu_ctx *ctx, vgpu_env **out);

#ifdef __cplusplus
}
#endif
#endif
