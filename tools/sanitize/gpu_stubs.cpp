// gpu_stubs.cpp -- CPU sanitizer build only (tools/sanitize): the C-ABI entries whose code lives in the
// HIP translation units (rt_runtime.hip, rt_post.hip, rt_build.hip) as stubs that fail loudly with
// RT_ERR_NO_DEVICE, so the host sources (OBJ/MTL loader, PNG decoder, scene presets, BMP writer, host BVH
// builders) link into one instrumented library the CPU tests can load.  Never part of librt_amd.so.
// (rt_amd.h is not included: the stubs take no arguments, and ctypes / C callers pass theirs regardless)
#include <string>

#include "../../raytracer-group27_amd/csrc/rt_internal.h"

#define RT_ERR_NO_DEVICE (-5)  // rt_amd.h

#define STUB(name)                                                        \
    extern "C" int name() {                                               \
        rt::set_error(#name ": CPU sanitizer build has no GPU path");    \
        return RT_ERR_NO_DEVICE;                                          \
    }

STUB(rt_bitmap) STUB(rt_bitmap_device) STUB(rt_create) STUB(rt_ctx_devices) STUB(rt_ctx_info)
STUB(rt_ctx_set_option) STUB(rt_debug_build_info) STUB(rt_debug_counters) STUB(rt_debug_create_ms)
STUB(rt_debug_job_trace) STUB(rt_debug_records) STUB(rt_debug_wave_trace) STUB(rt_destroy) STUB(rt_device_count)
STUB(rt_device_free) STUB(rt_device_synchronize) STUB(rt_intersect) STUB(rt_ipc_alloc) STUB(rt_ipc_close)
STUB(rt_ipc_open) STUB(rt_memcpy_dtoh) STUB(rt_philox4x32_10) STUB(rt_postprocess) STUB(rt_postprocess_device)
STUB(rt_render) STUB(rt_render_device) STUB(rt_render_views) STUB(rt_render_views_device)
STUB(rt_render_views_image_device) STUB(rt_selftest_math) STUB(rt_set_build_mode) STUB(rt_set_counting)
STUB(rt_shade) STUB(rt_texture_sample) STUB(rt_unpermute_bands_device) STUB(rt_unpermute_views_device)
STUB(rt_update_lights) STUB(rt_update_materials)
