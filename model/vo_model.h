/* vo_model.h -- a robot's kinematic model and collision hierarchy as plain C tables.
 *
 * The generated model/<robot>_model.h files (tools/gen_model_header.py) define one
 * `static const vo_model <robot>_model` each; the oracle (oracle/vamp_oracle.c) walks these
 * tables.  Field meaning follows model/<robot>.json (tools/extract_model.py).
 */
#pragma once

#define VO_JOINT_REVOLUTE 0
#define VO_JOINT_PRISMATIC 1

typedef struct vo_model {
    const char *name;
    int dim, resolution, nframes, nspheres, nbound, nenv, nself;
    const float *s_m, *s_a, *d_m;
    /* frames in topological order; joint dof (-1 fixed) of type jtype along a unit axis */
    const int *frame_parent, *frame_dof, *frame_jtype;
    const float (*frame_t)[3], (*frame_qf)[4], (*frame_axis)[3];
    const int *sphere_frame;
    const float (*sphere_off)[3];
    const float *sphere_r;
    const int *bound_frame;
    const float (*bound_off)[3];
    const float *bound_r;
    const int *bound_base;
    /* env checks: bounding sphere, children [start, end), leaf = the bounding sphere's own hit
     * is the collision (a single-sphere link tested directly, no children) */
    const int *env_bound, *env_child_start, *env_child_sphere, *env_child_base, *env_leaf;
    const int *self_a_kind, *self_a_idx, *self_b_kind, *self_b_idx, *self_child_start;
    const int (*self_child)[2];
    const int *order_kind, *order_idx; /* kind 0 env, 1 self, 2 attachment vs link, 3 attachment vs env */
    /* attachment variant (interleaved_sphere_fk_attachment) only: checks of the attached spheres
     * against a link entity (kind 0 sphere / 1 bounding) with children [start, end), and the
     * end-effector frame the attachment is posed at (-1: no attachment checks) */
    int natt;
    const int *att_ent_kind, *att_ent_idx, *att_child_start, *att_child_sphere, *att_leaf;
    int ee_frame;
} vo_model;
