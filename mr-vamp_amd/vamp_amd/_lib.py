"""ctypes binding of the C ABI (include/vamp_gpu.h) in ``libvampgpu.so``.

The library is built in-tree by ``make -C mr-vamp_amd`` (or ``__graft_entry__.build()``).
There is deliberately no fallback: if the library is missing or no HIP device is present
every entry point raises, so a GPU test can never pass on a silent CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# VAMP_AMD_LIB selects an alternative build of the same ABI (kernel variants for A/B timing)
LIB_PATH = os.environ.get("VAMP_AMD_LIB") or os.path.join(HERE, "libvampgpu.so")

VGPU_OK = 0
VGPU_ROBOT_PANDA = 1
VGPU_ROBOT_FETCH = 2
VGPU_ROBOT_PANDA_PAIR = 3
VGPU_ROBOT_UR5 = 4
VGPU_ROBOT_BAXTER = 5
ERRORS = {-1: "invalid argument", -2: "HIP error", -3: "out of memory", -4: "unsupported", -5: "host rsqrt probe", -6: "internal (C++ exception inside the library)"}

F32P = C.POINTER(C.c_float)
U8P = C.POINTER(C.c_uint8)
I32P = C.POINTER(C.c_int32)
U32P = C.POINTER(C.c_uint32)
VP = C.c_void_p


class VgpuRobot(C.Structure):
    _fields_ = [("kind", C.c_int32), ("base_x100", C.c_int32), ("base_y100", C.c_int32), ("base_z100", C.c_int32),
                ("base2_x100", C.c_int32), ("base2_y100", C.c_int32), ("base2_z100", C.c_int32)]


class VgpuRrtcSettings(C.Structure):
    _fields_ = [("range", C.c_float), ("dynamic_domain", C.c_int32), ("radius", C.c_float), ("alpha", C.c_float),
                ("min_radius", C.c_float), ("balance", C.c_int32), ("tree_ratio", C.c_float),
                ("max_iterations", C.c_uint64), ("max_samples", C.c_uint64), ("start_tree_first", C.c_int32)]


class VgpuPlanResult(C.Structure):
    _fields_ = [("solved", C.c_int32), ("iterations", C.c_uint64), ("nanoseconds", C.c_int64),
                ("size", C.c_uint64 * 2), ("cost", C.c_float), ("path_len", C.c_size_t)]


# every exported symbol of include/vamp_gpu.h with its signature (restype, argtypes)
SIGNATURES = {
    "vgpu_ctx_create": (C.c_int, [C.c_int, C.POINTER(VP)]),
    "vgpu_ctx_destroy": (None, [VP]),
    "vgpu_last_error": (C.c_char_p, [VP]),
    "vgpu_ctx_set_stream": (C.c_int, [VP, VP]),
    "vgpu_sync": (C.c_int, [VP]),
    "vgpu_ctx_set_profiling": (C.c_int, [VP, C.c_int]),
    "vgpu_phase_times": (C.c_int, [VP, F32P]),
    "vgpu_rsqrt_table": (C.c_int, [VP, C.POINTER(C.c_int), C.POINTER(U32P)]),
    "vgpu_rsqrt_table_set": (C.c_int, [VP, U32P, C.c_int]),
    "vgpu_env_create": (C.c_int, [VP, C.POINTER(VP)]),
    "vgpu_env_destroy": (None, [VP]),
    "vgpu_env_add_sphere": (C.c_int, [VP, F32P, C.c_float]),
    "vgpu_env_add_cuboid_axes": (C.c_int, [VP, F32P, F32P, F32P, F32P, F32P]),
    "vgpu_env_add_cuboid_euler": (C.c_int, [VP, F32P, F32P, F32P]),
    "vgpu_env_add_capsule_endpoints": (C.c_int, [VP, F32P, F32P, C.c_float]),
    "vgpu_env_add_capsule_euler": (C.c_int, [VP, F32P, F32P, C.c_float, C.c_float]),
    "vgpu_env_counts": (C.c_int, [VP, I32P]),
    "vgpu_env_add_heightfield": (C.c_int, [VP, F32P, F32P, C.c_size_t, C.c_size_t, F32P]),
    "vgpu_env_add_pointcloud": (C.c_int, [VP, F32P, C.c_size_t, C.c_float, C.c_float, C.c_float,
                                          C.POINTER(C.c_int64)]),
    "vgpu_env_add_pointcloud_device": (C.c_int, [VP, VP, VP, C.c_size_t, C.c_float, C.c_float, C.c_float,
                                                 C.POINTER(C.c_int64)]),
    "vgpu_env_copy_pointcloud": (C.c_int, [VP, VP, C.c_int]),
    "vgpu_env_ext_counts": (C.c_int, [VP, I32P]),
    "vgpu_env_pointcloud_info": (C.c_int, [VP, C.c_int, I32P, C.POINTER(C.c_size_t), F32P]),
    "vgpu_env_pointcloud_arrays": (C.c_int, [VP, C.c_int, F32P, F32P, U32P, F32P]),
    "vgpu_pointcloud_collides": (C.c_int, [VP, VP, C.c_int, VP, VP, C.c_size_t, C.c_int, VP]),
    "vgpu_pointcloud_collides_host": (C.c_int, [VP, VP, C.c_int, F32P, F32P, C.c_size_t, C.c_int, U8P]),
    "vgpu_filter_pointcloud": (C.c_int, [VP, VP, C.c_size_t, C.c_float, C.c_float, F32P, F32P, F32P, C.c_int, VP,
                                         C.POINTER(C.c_size_t)]),
    "vgpu_filter_pointcloud_host": (C.c_int, [VP, F32P, C.c_size_t, C.c_float, C.c_float, F32P, F32P, F32P,
                                              C.c_int, U32P, C.POINTER(C.c_size_t)]),
    "vgpu_filter_robot_pointcloud": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, F32P, VP, C.c_size_t, C.c_float, VP]),
    "vgpu_filter_robot_pointcloud_host": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, F32P, F32P, C.c_size_t, C.c_float,
                                                    F32P, C.POINTER(C.c_size_t)]),
    "vgpu_env_upload": (C.c_int, [VP]),
    "vgpu_env_attach": (C.c_int, [VP, F32P, F32P, C.c_size_t]),
    "vgpu_env_detach": (C.c_int, [VP]),
    "vgpu_fkcc_attach": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, VP, C.c_size_t, VP]),
    "vgpu_fkcc_attach_host": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, F32P, C.c_size_t, U8P]),
    "vgpu_sphere_fk": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, C.c_size_t, VP, C.c_size_t]),
    "vgpu_fkcc": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, VP, C.c_size_t, VP]),
    "vgpu_validate_motions": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, VP, VP, C.c_size_t, VP, VP]),
    "vgpu_validate_motions_mask": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, VP, VP, C.c_size_t, VP, VP, VP, C.c_size_t,
                                             C.POINTER(C.c_size_t)]),
    "vgpu_sphere_fk_host": (C.c_int, [VP, C.POINTER(VgpuRobot), F32P, C.c_size_t, F32P]),
    "vgpu_fkcc_host": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, F32P, C.c_size_t, U8P]),
    "vgpu_validate_motions_host": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, F32P, F32P, C.c_size_t, U8P, I32P]),
    "vgpu_halton": (C.c_int, [VP, C.c_int, C.c_uint64, C.c_size_t, VP]),
    "vgpu_sample_configurations": (C.c_int, [VP, C.POINTER(VgpuRobot), C.c_uint64, C.c_size_t, VP]),
    "vgpu_sample_fkcc": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, C.c_uint64, C.c_size_t, VP, VP]),
    "vgpu_compact": (C.c_int, [VP, VP, VP, C.c_size_t, C.c_int, VP, VP, C.POINTER(C.c_size_t)]),
    "vgpu_halton_host": (C.c_int, [VP, C.c_int, C.c_uint64, C.c_size_t, F32P]),
    "vgpu_sample_fkcc_host": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, C.c_uint64, C.c_size_t, F32P, U8P]),
    "vgpu_robot_info": (C.c_int, [C.c_int32, I32P, I32P, I32P]),
    "vgpu_prm_neighbor_params": (C.c_int, [C.c_int, C.c_double, C.c_double, C.c_size_t, U32P, F32P]),
    "vgpu_set_knn_mode": (C.c_int, [VP, C.c_int]),
    "vgpu_roadmap_knn": (C.c_int, [VP, C.c_int, VP, C.c_size_t, VP, VP, C.c_uint32, VP, VP, VP]),
    "vgpu_roadmap_knn_range": (C.c_int, [VP, C.c_int, VP, C.c_size_t, C.c_size_t, C.c_size_t, VP, VP, C.c_uint32,
                                         VP, VP, VP]),
    "vgpu_roadmap_edge_gather": (C.c_int, [VP, C.c_int, VP, C.c_size_t, C.c_size_t, VP, C.c_uint32, VP, VP, VP,
                                           VP]),
    "vgpu_roadmap_assemble": (C.c_int, [C.c_size_t, U32P, C.c_size_t, C.POINTER(C.c_size_t), U32P, U32P]),
    "vgpu_roadmap_assemble_device": (C.c_int, [VP, C.c_size_t, VP, C.c_size_t, VP, VP, VP]),
    "vgpu_cpu_fkcc_block": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, C.POINTER(C.c_int)]),
    "vgpu_cpu_fkcc_attach_block": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, C.POINTER(C.c_int)]),
    "vgpu_cpu_sphere_fk_block": (C.c_int, [C.POINTER(VgpuRobot), F32P, F32P]),
    "vgpu_cpu_validate_motion": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, F32P, C.POINTER(C.c_int)]),
    "vgpu_cpu_fkcc": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, C.c_size_t, U8P, C.c_int]),
    "vgpu_cpu_fkcc_attach": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, C.c_size_t, U8P, C.c_int]),
    "vgpu_cpu_validate_motions_mask": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, F32P, C.c_size_t, U8P, I32P, U8P,
                                                 C.c_size_t, C.POINTER(C.c_size_t), C.c_int]),
    "vgpu_cpu_validate_motions": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, F32P, C.c_size_t, U8P, I32P, I32P,
                                            C.c_int]),
    "vgpu_l2_norm": (C.c_float, [F32P, C.c_int]),
    "vgpu_shard_range": (C.c_int, [C.c_size_t, C.c_int, C.c_int, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "vgpu_multi_create": (C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(VP)]),
    "vgpu_multi_destroy": (None, [VP]),
    "vgpu_multi_size": (C.c_int, [VP]),
    "vgpu_multi_context": (VP, [VP, C.c_int]),
    "vgpu_multi_last_error": (C.c_char_p, [VP]),
    "vgpu_multi_env_create": (C.c_int, [VP, VP, C.POINTER(VP)]),
    "vgpu_multi_validate_motions_host": (C.c_int, [VP, C.POINTER(VgpuRobot), C.POINTER(VP), F32P, F32P, C.c_size_t,
                                                   U8P, I32P]),
    "vgpu_multi_sample_fkcc_host": (C.c_int, [VP, C.POINTER(VgpuRobot), C.POINTER(VP), C.c_uint64, C.c_size_t, F32P,
                                              C.POINTER(C.c_uint64), C.POINTER(C.c_size_t)]),
    "vgpu_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "vgpu_comm_init": (C.c_int, [VP, C.c_int, C.c_int, C.POINTER(C.c_uint8), C.POINTER(VP)]),
    "vgpu_comm_destroy": (None, [VP]),
    "vgpu_comm_last_error": (C.c_char_p, [VP]),
    "vgpu_loopback_create": (C.c_int, [C.c_int, C.POINTER(VP)]),
    "vgpu_loopback_destroy": (C.c_int, [VP]),
    "vgpu_comm_init_loopback": (C.c_int, [VP, C.c_int, VP, C.POINTER(VP)]),
    "vgpu_env_upload_stats": (C.c_int, [VP, C.POINTER(C.c_uint64)]),
    "vgpu_env_pointcloud_grid": (C.c_int, [VP, C.c_int, C.POINTER(C.c_uint32)]),
    "vgpu_debug_build": (C.c_int, []),
    "vgpu_debug_violations": (C.c_int, [VP, VP, C.POINTER(C.c_uint32)]),
    "vgpu_ctx_device": (C.c_int, [VP, C.POINTER(C.c_int)]),
    "vgpu_query_split": (C.c_int, [C.c_size_t, C.c_int, C.c_int, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "vgpu_prm_edges_allgather": (C.c_int, [VP, VP, C.POINTER(VgpuRobot), VP, VP, C.c_size_t, C.c_double, C.c_double,
                                           VP, VP, C.c_size_t, C.POINTER(C.c_size_t), VP]),
    "vgpu_prm_vertices_allgather": (C.c_int, [VP, VP, C.POINTER(VgpuRobot), VP, C.c_uint64, C.c_size_t, VP, VP,
                                              C.c_size_t, C.POINTER(C.c_size_t)]),
    "vgpu_env_clone": (C.c_int, [VP, VP, C.POINTER(VP)]),
    "vgpu_cpu_roadmap_knn": (C.c_int, [C.c_int, F32P, C.c_size_t, U32P, C.c_size_t, U32P, F32P, C.c_uint32, U32P, F32P,
                                       U32P, C.c_int]),
    "vgpu_robot_scale_params": (C.c_int, [C.POINTER(VgpuRobot), F32P, F32P, F32P]),
    "vgpu_cpu_eefk": (C.c_int, [C.POINTER(VgpuRobot), F32P, C.c_size_t, F32P]),
    "vgpu_cpu_validate_vector": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, F32P, C.c_float, C.POINTER(C.c_int)]),
    "vgpu_cpu_rrtc": (C.c_int, [C.POINTER(VgpuRobot), VP, F32P, F32P, C.c_size_t, C.POINTER(VgpuRrtcSettings),
                                C.POINTER(C.c_uint64), F32P, C.c_size_t, C.POINTER(VgpuPlanResult)]),
    "vgpu_build_roadmap_host": (C.c_int, [VP, C.POINTER(VgpuRobot), VP, F32P, C.c_size_t, C.c_double, C.c_double,
                                          C.POINTER(C.c_size_t), U32P, C.c_size_t, C.POINTER(C.c_size_t), U32P]),
}

_lib = None


def load() -> C.CDLL:
    """Load libvampgpu.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C mr-vamp_amd` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME libamdhip64.so.7) and
    # its libc10_hip asks for it as "libamdhip64.so".  Loaded first, it satisfies this library's
    # libamdhip64.so.7 dependency too; loaded after /opt/rocm's copy, torch would bring in a second
    # runtime, which then finds no GPU.  So torch (when installed) is imported before the CDLL.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class VgpuError(RuntimeError):
    pass


def check(rc: int, ctx=None):
    if rc != VGPU_OK:
        msg = ""
        if ctx is not None:
            m = load().vgpu_last_error(ctx)
            msg = m.decode() if m else ""
        raise VgpuError(f"vamp_gpu: {ERRORS.get(rc, rc)}: {msg}")
