// vgpu_abi.hh -- no C++ exception crosses the C ABI (include/vamp_gpu.h).  Every multi-statement int-returning
// entry point is a function-try-block ending in VGPU_ABI_CATCH: std::bad_alloc becomes VGPU_ERR_OOM, anything
// else VGPU_ERR_INTERNAL (a std::thread that cannot start, a container's length_error), instead of
// std::terminate taking the host process down.  tests/test_c_abi.py checks that every such definition has it.
#pragma once
#include <new>

#define VGPU_ABI_CATCH                                                                                             \
    catch (const std::bad_alloc&) { return VGPU_ERR_OOM; }                                                         \
    catch (...) { return VGPU_ERR_INTERNAL; }
