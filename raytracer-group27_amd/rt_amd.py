"""ctypes binding of librt_amd.so (include/rt_amd.h) + the C1..C5 config manifest.

Host-side mirror of the reference interface for the hot path: Scene / loadScene / loadMesh,
BoundingVolumeHierarchy(Scene*) + intersect(), getFinalColor(), renderRayTracing().  The
product path is the HIP library; if it cannot be loaded this module raises -- there is no CPU
fallback.
"""
import ctypes as C
import gzip
import os
import shutil
import sys as _sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
_DEFAULT_LIB = os.path.join(HERE, "librt_amd.so")
LIB_PATH = _DEFAULT_LIB
# tools/sanitize/run.sh only: the CPU-only ASan/UBSan build of the host sources (its GPU entries are stubs
# that fail with RT_ERR_NO_DEVICE, so nothing can pass on it that needs the GPU path)
if os.environ.get("RT_AMD_SANITIZER_LIB"):
    LIB_PATH = os.environ["RT_AMD_SANITIZER_LIB"]
SCENE_DIR = os.path.join(REPO, "tests", "golden", "scenes")

FLT_MAX = float(np.finfo(np.float32).max)


class rt_material(C.Structure):
    _fields_ = [("kd", C.c_float * 3), ("ks", C.c_float * 3), ("shininess", C.c_float),
                ("transparency", C.c_float), ("has_texture", C.c_int), ("texture", C.c_int)]


class rt_texture(C.Structure):
    """Decoded kd texture (stbi_load(..., STBI_rgb) output, src/image.cpp:45)."""
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("channels", C.c_int), ("pad_", C.c_int),
                ("rgb", C.POINTER(C.c_uint8))]


class rt_sphere(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("radius", C.c_float), ("material", rt_material)]


class rt_point_light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("color", C.c_float * 3)]


class rt_spherical_light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("radius", C.c_float), ("color", C.c_float * 3)]


class rt_spot_light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("direction", C.c_float * 3), ("angle", C.c_float),
                ("color", C.c_float * 3)]


class rt_plane_light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("width", C.c_float * 3), ("height", C.c_float * 3),
                ("color", C.c_float * 3)]


class rt_scene_desc(C.Structure):
    _fields_ = [("num_triangles", C.c_int), ("positions", C.POINTER(C.c_float)),
                ("normals", C.POINTER(C.c_float)), ("texcoords", C.POINTER(C.c_float)),
                ("mesh_index", C.POINTER(C.c_int)), ("num_meshes", C.c_int),
                ("materials", C.POINTER(rt_material)), ("num_spheres", C.c_int),
                ("spheres", C.POINTER(rt_sphere)), ("num_point_lights", C.c_int),
                ("point_lights", C.POINTER(rt_point_light)), ("num_spherical_lights", C.c_int),
                ("spherical_lights", C.POINTER(rt_spherical_light)), ("num_spot_lights", C.c_int),
                ("spot_lights", C.POINTER(rt_spot_light)), ("num_plane_lights", C.c_int),
                ("plane_lights", C.POINTER(rt_plane_light)), ("num_textures", C.c_int),
                ("textures", C.POINTER(rt_texture))]


class rt_mesh_view(C.Structure):
    """One mesh as loadMesh returns it (src/mesh.h:14-44): vertices [n][8] = p, n, texCoord."""
    _fields_ = [("num_vertices", C.c_int), ("num_triangles", C.c_int), ("vertices", C.POINTER(C.c_float)),
                ("triangles", C.POINTER(C.c_uint32)), ("material", rt_material), ("texture_path", C.c_char_p)]


class rt_camera(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("quat", C.c_float * 4), ("half_height", C.c_float),
                ("half_width", C.c_float)]


class rt_params(C.Structure):
    _fields_ = [("max_reflection_level", C.c_int), ("sphere_light_ray_count", C.c_int),
                ("plane_light_1D_ray_count", C.c_int), ("glossy_ray_count", C.c_int),
                ("refraction_factor", C.c_float), ("use_bvh", C.c_int), ("anti_aliasing", C.c_int),
                ("multiple_rays", C.c_int), ("sample_size", C.c_int), ("barycentric_mode", C.c_int),
                ("rng_seed", C.c_uint64), ("use_textures", C.c_int), ("texture_filtering", C.c_int),
                ("out_of_bounds_x", C.c_int), ("out_of_bounds_y", C.c_int), ("border_color", C.c_float * 3),
                ("shade_level", C.c_int)]


# TextureFiltering / OutOfBoundsRule (src/image.h:16-29)
TEX_NEAREST, TEX_BILINEAR, TEX_MIP_NEAREST, TEX_MIP_NEAREST_BILINEAR, TEX_TRILINEAR = range(5)
OOB_BORDER, OOB_CLAMP, OOB_REPEAT = range(3)


class rt_ray(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("direction", C.c_float * 3), ("t", C.c_float)]


class rt_hit(C.Structure):
    _fields_ = [("hit", C.c_int), ("t", C.c_float), ("normal", C.c_float * 3), ("hit_point", C.c_float * 3),
                ("uv", C.c_float * 2), ("material_index", C.c_int), ("prim_id", C.c_int),
                ("is_triangle", C.c_int)]


class rt_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64),
                ("hits", C.c_uint64), ("ub_hits", C.c_uint64), ("kernel_ms", C.c_float), ("node_bytes", C.c_uint32),
                ("kernel", C.c_char * 64)]

    @property
    def kernel_name(self):
        """The launched render kernel as rocprofv3 names it (without the argument list)."""
        return self.kernel.decode()


RAY_DTYPE = np.dtype([("origin", "<f4", 3), ("direction", "<f4", 3), ("t", "<f4")])
HIT_DTYPE = np.dtype([("hit", "<i4"), ("t", "<f4"), ("normal", "<f4", 3), ("hit_point", "<f4", 3),
                      ("uv", "<f4", 2), ("material_index", "<i4"), ("prim_id", "<i4"), ("is_triangle", "<i4")])
assert RAY_DTYPE.itemsize == C.sizeof(rt_ray) and HIT_DTYPE.itemsize == C.sizeof(rt_hit)

# Every symbol include/rt_amd.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "rt_abi_version", "rt_device_count", "rt_last_error", "rt_scene_new", "rt_scene_load_obj", "rt_scene_preset",
    "rt_scene_add_sphere", "rt_scene_add_point_light", "rt_scene_add_spherical_light",
    "rt_scene_add_spot_light", "rt_scene_add_plane_light", "rt_scene_clear_lights", "rt_scene_set_material",
    "rt_scene_desc_get", "rt_scene_free", "rt_write_dragon_proxy", "rt_camera_from_trackball", "rt_create",
    "rt_destroy", "rt_render", "rt_render_device", "rt_render_views_device", "rt_render_views", "rt_unpermute_bands_device", "rt_intersect", "rt_shade",
    "rt_set_counting", "rt_debug_counters", "rt_ctx_info", "rt_selftest_math",
    "rt_postprocess_device", "rt_bitmap_device", "rt_postprocess", "rt_bitmap", "rt_encode_bmp", "rt_write_bmp",
    "rt_philox4x32_10", "rt_debug_wave_trace", "rt_debug_job_trace", "rt_debug_phase_trace", "rt_debug_create_ms", "rt_set_build_mode", "rt_debug_build_info", "rt_debug_records", "rt_debug_ref_bvh", "rt_decode_png", "rt_ctx_set_option", "rt_texture_sample",
    "rt_update_lights", "rt_update_materials", "rt_unpermute_views_device", "rt_scene_mesh_count", "rt_scene_mesh_get",
    "rt_ctx_devices", "rt_ctx_peer_stores", "rt_render_views_image_device", "rt_ipc_alloc", "rt_ipc_open", "rt_ipc_close", "rt_device_free",
    "rt_device_synchronize", "rt_memcpy_dtoh", "rt_debug_slab_check", "rt_source_hash",
]
IPC_HANDLE_BYTES = 64

BUILD_AUTO, BUILD_HOST, BUILD_GPU = 0, 1, 2
ASSIMP3_SHININESS_X4, ASSIMP3_NORMALS_DIV = 1, 2  # rt_scene_load_obj / rt_scene_preset compat bits


def set_build_mode(mode):
    """rt_set_build_mode: where later rt_create calls build the acceleration structures."""
    check(lib().rt_set_build_mode(int(mode)))


# rt_ctx_set_option (include/rt_amd.h): test / developer hooks; defaults are the shipped path
OPT_KERNEL, OPT_COOP, OPT_COOP_MAX, OPT_REFILL, OPT_WAVE_TRACE, OPT_VARIANT, OPT_FAN, OPT_INTERLEAVE, OPT_FAN_CAP = \
    1, 2, 3, 4, 5, 6, 7, 8, 9
OPT_DUAL_STEP = 10
OPT_CENTRE_FIRST = 12  # job order: upper-half XCD tile ranges walked bottom-up (-1 by shape, 0 off, 1 on)
OPT_OPAQUE = 11  # opaque-scene kernel: -1 where eligible (default: 4-wave, SPLIT with one light), 0 the general kernels, 1 4-wave without SPLIT, 2 3-wave, 3 re-visit, 4 / 5 SPLIT 4- / 3-wave, 6 / 7 SPLIT without lane groups 5- / 4-wave (A/Bs)
OPT_PEER_STORES = 14  # split renders: -1 peer stores where peer access works (default), 0 band-dense + copy always
OPT_TREE = 13  # recursion-tree kernel (C4 / C5 class): -1 / 2 where eligible (default: 4 waves for batches, 3 for frames), 0 the general kernels, 1 its re-visit group stack build (A/B), 3 a checked 4-wave build, 4 / 5 the 4- / 3-wave build always
OPT_INTERLEAVE_TAIL = 15  # opaque batches: the last n views interleaved over 16 tiles (0 none)
OPT_WF_STREAMS = 18  # wavefront chunks over 1..4 streams (0: default 2)
OPT_PRIO = 19  # opaque kernel: s_setprio 2 after this many iterations of a traversal phase (-1 by shape, 0 never)
OPT_WF_CHUNK = 20  # wavefront path: camera jobs per chunk at most (multiple of 64; 0 the memory budget's)
OPT_WF_BUILD = 17  # wavefront trace kernel build: 0 5 waves (default), 1 6, 2 4 + node prefetch, 3 8
OPT_WAVEFRONT = 16  # opaque-kernel renders, one sample per pixel: -1 (default) / 0 the megakernel, 1 the wavefront path, 2..64 its refill
KERNEL_AUTO, KERNEL_WHOLE_TRAVERSAL, KERNEL_DYNAMIC_FETCH = 0, 1, 2
# compiled kernel variants (rt_megakernel.hip RT_V_*, rt_runtime.hip RT_DF_* / RT_WT_*)
V_CALL, V_NOPF, V_NOCOOP, V_W4 = 1, 2, 4, 16
DF_BATCH, DF_FRAME = V_CALL | V_NOPF | V_NOCOOP | V_W4, 0  # shipped dynamic-fetch variants (by render shape)
DF_ALT = V_CALL | V_NOPF | V_W4  # the one A/B alternate: the batch variant with out-of-line drain lane groups
DF_VARIANTS = [DF_BATCH, DF_FRAME, DF_ALT]
WT_VARIANTS = [0]

class rt_post_params(C.Structure):
    """Screen post-processing settings (src/screen.h:58-111), raw setter values."""
    _fields_ = [("filtering_option", C.c_int), ("kernel", C.c_int), ("repetitions", C.c_int),
                ("filter_size", C.c_int), ("sigma", C.c_float), ("exposure", C.c_float),
                ("gamma_correction", C.c_int), ("gamma", C.c_float), ("bloom_live", C.c_int), ("pad_", C.c_int)]


# FilteringOption / Kernel (src/screen.h:16-30)
BLOOM_NONE, BLOOM, BLOOM_REINHARD, BLOOM_EXPOSURE, BLOOM_ONLY_LIGHT, BLOOM_ONLY_LIGHT_KERNEL = range(6)
KERNEL_BOX, KERNEL_GAUSSIAN = 0, 1


def post_params(filtering_option=BLOOM_NONE, kernel=KERNEL_BOX, repetitions=1, filter_size=5, sigma=2.0,
                exposure=0.5, gamma_correction=False, gamma=2.2, bloom_live=False):
    """Defaults of class Screen and of main.cpp's bloom settings (src/main.cpp:426-435)."""
    return rt_post_params(int(filtering_option), int(kernel), int(repetitions), int(filter_size), float(sigma),
                          float(exposure), int(bool(gamma_correction)), float(gamma), int(bool(bloom_live)), 0)


def postprocess(rgb, W, H, prm):
    """Screen::postprocessImage on a host image (W*H*3 float32, setPixel order); returns a copy."""
    out = np.ascontiguousarray(rgb, np.float32).copy()
    check(lib().rt_postprocess(C.byref(prm), W, H, out.ctypes.data_as(C.POINTER(C.c_float))), "rt_postprocess")
    return out


def bitmap(rgb, W, H, prm):
    """Screen::writeBitmapToFile's pixel path: (bloomed float image, RGBA8 [H*W*4])."""
    out = np.ascontiguousarray(rgb, np.float32).copy()
    rgba = np.zeros(W * H * 4, np.uint8)
    check(lib().rt_bitmap(C.byref(prm), W, H, out.ctypes.data_as(C.POINTER(C.c_float)),
                          rgba.ctypes.data_as(C.POINTER(C.c_uint8))), "rt_bitmap")
    return out, rgba


def encode_bmp(rgba, W, H):
    """stbi_write_bmp bytes of an RGBA8 image (24-bit, bottom-up, alpha dropped)."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    size = 54 + (3 * W + ((-3 * W) & 3)) * H
    buf = np.zeros(size, np.uint8)
    n = lib().rt_encode_bmp(W, H, rgba.ctypes.data_as(C.POINTER(C.c_uint8)), buf.ctypes.data_as(C.POINTER(C.c_uint8)),
                            size)
    check(int(n) if n < 0 else 0, "rt_encode_bmp")
    return buf[:n].tobytes()


_lib = None


def _torch_first():
    """PyTorch wheels bundle their own HIP runtime.  Measured on the MI355X box: if librt_amd.so
    (and /opt/rocm's runtime) is loaded before torch initialises the GPU, one of the two runtimes
    later finds no device; with torch initialised first both work.  The drivers here (tests, bench,
    smoke) use torch for buffers and streams, so initialise it before loading the library."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


def library_source_hash():
    """rt_source_hash: the source hash compiled into the loaded library (build.py source_hash())."""
    buf = C.create_string_buffer(32)
    check(lib().rt_source_hash(buf, 32), "rt_source_hash")
    return buf.value.decode()


def tree_source_hash():
    """The same hash of this tree's sources (csrc/, include/rt_amd.h, build.py)."""
    if HERE not in _sys.path:
        _sys.path.insert(0, HERE)
    import build as _build

    return _build.source_hash()


def provenance(strict=True):
    """Ties the loaded library to the tree it runs from: {library, tree, match}; raises if they differ and
    strict (a stale or foreign library must not be measured or tested as this tree's)."""
    got, want = library_source_hash(), tree_source_hash()
    if strict and got != want:
        raise RuntimeError(f"{LIB_PATH} was built from sources {got}, this tree is {want}: rebuild "
                           "(__graft_entry__.build())")
    return {"library_source_hash": got, "tree_source_hash": want, "match": got == want}


def lib():
    """Load librt_amd.so (raises if it is missing: the product has no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (HIP path has no fallback)")
        _torch_first()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        vp = C.c_void_p
        sigs = {
            "rt_abi_version": ([], C.c_int),
            "rt_source_hash": ([C.c_char_p, C.c_size_t], C.c_int),
            "rt_device_count": ([C.POINTER(C.c_int)], C.c_int),
            "rt_last_error": ([C.c_char_p, C.c_size_t], C.c_int),
            "rt_scene_new": ([P(vp)], C.c_int),
            "rt_scene_load_obj": ([vp, C.c_char_p, C.c_int, C.c_int], C.c_int),
            "rt_scene_preset": ([vp, C.c_int, C.c_char_p, C.c_int], C.c_int),
            "rt_scene_add_sphere": ([vp, P(rt_sphere)], C.c_int),
            "rt_scene_add_point_light": ([vp, P(rt_point_light)], C.c_int),
            "rt_scene_add_spherical_light": ([vp, P(rt_spherical_light)], C.c_int),
            "rt_scene_add_spot_light": ([vp, P(rt_spot_light)], C.c_int),
            "rt_scene_add_plane_light": ([vp, P(rt_plane_light)], C.c_int),
            "rt_scene_clear_lights": ([vp], C.c_int),
            "rt_scene_set_material": ([vp, C.c_int, P(rt_material)], C.c_int),
            "rt_scene_desc_get": ([vp, P(rt_scene_desc)], C.c_int),
            "rt_scene_free": ([vp], C.c_int),
            "rt_write_dragon_proxy": ([C.c_char_p, C.c_int, C.c_int], C.c_int),
            "rt_camera_from_trackball": ([P(C.c_float), P(C.c_float), C.c_float, C.c_float, C.c_float,
                                         P(rt_camera)], C.c_int),
            "rt_create": ([P(rt_scene_desc), P(C.c_int), C.c_int, P(vp)], C.c_int),
            "rt_ctx_devices": ([vp, P(C.c_int), C.c_int], C.c_int),
            "rt_ctx_peer_stores": ([vp, P(C.c_int), C.c_int], C.c_int),
            "rt_render_views_image_device": ([vp, P(rt_camera), C.c_int, P(rt_params), C.c_int, C.c_int, C.c_int,
                                              C.c_int, C.c_int, vp, vp, P(rt_stats)], C.c_int),
            "rt_ipc_alloc": ([C.c_int, C.c_size_t, P(vp), P(C.c_uint8)], C.c_int),
            "rt_ipc_open": ([C.c_int, P(C.c_uint8), P(vp)], C.c_int),
            "rt_ipc_close": ([vp], C.c_int),
            "rt_device_free": ([C.c_int, vp], C.c_int),
            "rt_device_synchronize": ([C.c_int], C.c_int),
            "rt_memcpy_dtoh": ([vp, vp, C.c_size_t], C.c_int),
            "rt_destroy": ([vp], C.c_int),
            "rt_render": ([vp, P(rt_camera), P(rt_params), C.c_int, C.c_int, P(C.c_float), P(rt_stats)], C.c_int),
            "rt_render_device": ([vp, P(rt_camera), P(rt_params), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  vp, vp, P(rt_stats)], C.c_int),
            "rt_render_views_device": ([vp, P(rt_camera), C.c_int, P(rt_params), C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_int, vp, vp, P(rt_stats)], C.c_int),
            "rt_render_views": ([vp, P(rt_camera), C.c_int, P(rt_params), C.c_int, C.c_int, P(C.c_float),
                                 P(rt_stats)], C.c_int),
            "rt_unpermute_bands_device": ([C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp], C.c_int),
            "rt_unpermute_views_device": ([C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp], C.c_int),
            "rt_scene_mesh_count": ([vp, P(C.c_int)], C.c_int),
            "rt_scene_mesh_get": ([vp, C.c_int, P(rt_mesh_view)], C.c_int),
            "rt_intersect": ([vp, vp, C.c_int, C.c_int, vp], C.c_int),
            "rt_shade": ([vp, vp, C.c_int, P(rt_params), P(C.c_float), P(C.c_uint64)], C.c_int),
            "rt_set_counting": ([C.c_int], C.c_int),
            "rt_debug_counters": ([vp, P(C.c_uint64), C.c_int], C.c_int),
            "rt_ctx_info": ([vp, P(C.c_int), P(C.c_int), P(C.c_int), P(C.c_int)], C.c_int),
            "rt_selftest_math": ([vp, P(C.c_float), P(C.c_float), C.c_int, P(C.c_float)], C.c_int),
            "rt_postprocess_device": ([P(rt_post_params), C.c_int, C.c_int, vp, vp, vp], C.c_int),
            "rt_bitmap_device": ([P(rt_post_params), C.c_int, C.c_int, vp, vp, vp, vp], C.c_int),
            "rt_postprocess": ([P(rt_post_params), C.c_int, C.c_int, P(C.c_float)], C.c_int),
            "rt_bitmap": ([P(rt_post_params), C.c_int, C.c_int, P(C.c_float), P(C.c_uint8)], C.c_int),
            "rt_encode_bmp": ([C.c_int, C.c_int, P(C.c_uint8), P(C.c_uint8), C.c_long], C.c_long),
            "rt_write_bmp": ([C.c_char_p, C.c_int, C.c_int, P(C.c_uint8)], C.c_int),
            "rt_philox4x32_10": ([P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)], C.c_int),
            "rt_decode_png": ([P(C.c_uint8), C.c_long, P(C.c_int), P(C.c_int), P(C.c_int), P(C.c_uint8), C.c_long],
                              C.c_int),
            "rt_debug_wave_trace": ([vp, P(C.c_uint64), C.c_int], C.c_int),
            "rt_debug_job_trace": ([vp, P(C.c_uint64), C.c_int], C.c_int),
            "rt_debug_phase_trace": ([vp, P(C.c_uint64), C.c_int], C.c_int),
            "rt_debug_create_ms": ([vp, P(C.c_double), C.c_int], C.c_int),
            "rt_set_build_mode": ([C.c_int], C.c_int),
            "rt_debug_build_info": ([vp, P(C.c_int), C.c_int], C.c_int),
            "rt_debug_records": ([vp, P(C.c_float), C.c_int, C.c_int], C.c_int),
            "rt_debug_ref_bvh": ([vp, P(C.c_float), P(C.c_int), P(C.c_int), P(C.c_int)], C.c_int),
            "rt_debug_slab_check": ([P(C.c_float), P(C.c_float), C.c_int, P(C.c_int)], C.c_int),
            "rt_ctx_set_option": ([vp, C.c_int, C.c_int], C.c_int),
            "rt_texture_sample": ([vp, C.c_int, C.c_int, P(C.c_float), P(rt_params), P(C.c_float)], C.c_int),
            "rt_update_lights": ([vp, P(rt_scene_desc)], C.c_int),
            "rt_update_materials": ([vp, C.c_int, P(rt_material), C.c_int, P(rt_material)], C.c_int),
        }
        for name, (args, res) in sigs.items():
            f = getattr(L, name, None)
            if f is None and LIB_PATH != _DEFAULT_LIB:  # an older A/B build (tools/ab_variants.py --lib)
                continue
            if f is None:
                raise RtError(f"{LIB_PATH} does not export {name} (stale build: run raytracer-group27_amd/build.py)")
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


class RtError(RuntimeError):
    pass


def check(rc, what=""):
    if rc != 0:
        buf = C.create_string_buffer(1024)
        lib().rt_last_error(buf, 1024)
        raise RtError(f"{what} failed ({rc}): {buf.value.decode(errors='replace')}")


def _f3(v):
    return (C.c_float * 3)(*[float(np.float32(x)) for x in v])


def material(kd, ks=(0, 0, 0), shininess=1.0, transparency=1.0):
    """Material{kd, ks{0}, shininess{1}, transparency{1}} (src/mesh.h:23-33)."""
    return rt_material(_f3(kd), _f3(ks), float(np.float32(shininess)), float(np.float32(transparency)), 0, 0)


class Scene:
    """Scene + loadScene/loadMesh (src/scene.cpp:4-150, src/mesh.cpp:58-188)."""

    def __init__(self):
        self.h = C.c_void_p()
        check(lib().rt_scene_new(C.byref(self.h)), "rt_scene_new")

    def __del__(self):
        if getattr(self, "h", None) and self.h.value and callable(lib):  # (module teardown: lib is gone)
            lib().rt_scene_free(self.h)
            self.h = C.c_void_p()

    def load_obj(self, path, normalize=False, shininess_x4=False, normals_div=False):
        """loadMesh; shininess_x4 / normals_div select Assimp 3.x behaviour (RT_ASSIMP3_* in rt_amd.h)."""
        compat = (ASSIMP3_SHININESS_X4 if shininess_x4 else 0) | (ASSIMP3_NORMALS_DIV if normals_div else 0)
        check(lib().rt_scene_load_obj(self.h, str(path).encode(), int(normalize), compat), f"loadMesh({path})")
        return self

    def preset(self, preset, data_dir, shininess_x4=False):
        check(lib().rt_scene_preset(self.h, int(preset), str(data_dir).encode(), int(shininess_x4)),
              f"loadScene({preset})")
        return self

    def add_sphere(self, center, radius, mat):
        s = rt_sphere(_f3(center), float(np.float32(radius)), mat)
        check(lib().rt_scene_add_sphere(self.h, C.byref(s)))

    def add_point_light(self, pos, color):
        check(lib().rt_scene_add_point_light(self.h, C.byref(rt_point_light(_f3(pos), _f3(color)))))

    def add_spherical_light(self, pos, radius, color):
        l = rt_spherical_light(_f3(pos), float(np.float32(radius)), _f3(color))
        check(lib().rt_scene_add_spherical_light(self.h, C.byref(l)))

    def add_spot_light(self, pos, direction, angle, color):
        l = rt_spot_light(_f3(pos), _f3(direction), float(np.float32(angle)), _f3(color))
        check(lib().rt_scene_add_spot_light(self.h, C.byref(l)))

    def add_plane_light(self, pos, width, height, color):
        l = rt_plane_light(_f3(pos), _f3(width), _f3(height), _f3(color))
        check(lib().rt_scene_add_plane_light(self.h, C.byref(l)))

    def clear_lights(self):
        check(lib().rt_scene_clear_lights(self.h))

    def set_material(self, mesh, mat):
        check(lib().rt_scene_set_material(self.h, int(mesh), C.byref(mat)), "set_material")

    def desc(self):
        d = rt_scene_desc()
        check(lib().rt_scene_desc_get(self.h, C.byref(d)), "rt_scene_desc_get")
        return d

    def meshes(self):
        """The meshes as loadMesh returns them: [(vertices [n][8] = p, n, texCoord), triangles [m][3],
        rt_material, texture path)]."""
        n = C.c_int()
        check(lib().rt_scene_mesh_count(self.h, C.byref(n)))
        out = []
        for i in range(n.value):
            v = rt_mesh_view()
            check(lib().rt_scene_mesh_get(self.h, i, C.byref(v)), "rt_scene_mesh_get")
            vert = np.ctypeslib.as_array(v.vertices, shape=(v.num_vertices * 8,)).reshape(-1, 8).copy() \
                if v.num_vertices else np.zeros((0, 8), np.float32)
            tri = np.ctypeslib.as_array(v.triangles, shape=(v.num_triangles * 3,)).reshape(-1, 3).copy() \
                if v.num_triangles else np.zeros((0, 3), np.uint32)
            out.append((vert, tri, rt_material.from_buffer_copy(v.material), v.texture_path.decode()))
        return out

    def arrays(self):
        """numpy copies of the flat scene (positions [T,3,3], normals [T,3,3], mesh [T], materials)."""
        d = self.desc()
        T = d.num_triangles
        pos = np.ctypeslib.as_array(d.positions, shape=(T * 9,)).reshape(T, 3, 3).copy() if T else np.zeros((0, 3, 3), np.float32)
        nrm = np.ctypeslib.as_array(d.normals, shape=(T * 9,)).reshape(T, 3, 3).copy() if T else np.zeros((0, 3, 3), np.float32)
        mesh = np.ctypeslib.as_array(d.mesh_index, shape=(T,)).copy() if T else np.zeros((0,), np.int32)
        mats = [rt_material.from_buffer_copy(d.materials[i]) for i in range(d.num_meshes)]
        return pos, nrm, mesh, mats


def camera_from_trackball(look_at=(0.0, 0.0, 0.0), euler=None, distance=3.0, fovy=None, aspect=1.0):
    """Trackball::position/generateRay constants (framework/src/trackball.cpp:65-98)."""
    if euler is None:
        euler = default_euler()
    if fovy is None:
        fovy = default_fovy()
    cam = rt_camera()
    la = (C.c_float * 3)(*look_at)
    eu = (C.c_float * 3)(*euler)
    check(lib().rt_camera_from_trackball(la, eu, float(np.float32(distance)), float(np.float32(fovy)),
                                         float(np.float32(aspect)), C.byref(cam)), "camera")
    return cam


RADIANS = np.float32(0.01745329251994329576923690768489)


def turntable_eulers(n, step_deg=None):
    """Trackball Euler angles of n views orbiting the default view about the vertical axis
    (Euler y = 20 deg + k * step), e.g. the frames of a turntable animation."""
    step = 360.0 / max(1, n) if step_deg is None else step_deg
    out = []
    for k in range(n):
        e = default_euler()
        e[1] = float(np.float32(np.float32(20.0 + k * step) * RADIANS))
        out.append(e)
    return out


def turntable_cameras(n, aspect, step_deg=None):
    """Cameras of turntable_eulers(n), for one view batch (rt_render_views_device)."""
    return [camera_from_trackball(euler=e, aspect=aspect) for e in turntable_eulers(n, step_deg)]


def default_euler():
    """glm::radians(glm::vec3(20.0f, 20.0f, 0.0f)) (src/main.cpp:414), float32 multiply."""
    return [float(np.float32(20.0) * RADIANS), float(np.float32(20.0) * RADIANS), float(np.float32(0.0) * RADIANS)]


def default_fovy():
    """glm::radians(50.0f) (src/main.cpp:413)."""
    return float(np.float32(50.0) * RADIANS)


def aspect_of(W, H):
    """Window::aspectRatio() = float(w)/float(h) (framework/src/window.cpp:334-337)."""
    return float(np.float32(W) / np.float32(H))


def params(max_reflection_level=5, sphere_light_ray_count=10, plane_light_1D_ray_count=3, glossy_ray_count=10,
           refraction_factor=0.8, use_bvh=False, anti_aliasing=False, multiple_rays=False, sample_size=4, seed=0x5EED,
           use_textures=False, texture_filtering=TEX_NEAREST, out_of_bounds_x=OOB_BORDER, out_of_bounds_y=OOB_BORDER,
           border_color=(0.0, 0.0, 0.0)):
    """Render knobs with the reference defaults (src/main.cpp:54-64,123-127)."""
    return rt_params(max_reflection_level, sphere_light_ray_count, plane_light_1D_ray_count, glossy_ray_count,
                     float(np.float32(refraction_factor)), int(use_bvh), int(anti_aliasing), int(multiple_rays),
                     sample_size, 0, seed, int(use_textures), int(texture_filtering), int(out_of_bounds_x),
                     int(out_of_bounds_y), _f3(border_color), 0)


def decode_png(data):
    """PNG bytes -> (H x W x 3 uint8 array, file channel count), stbi_load(..., STBI_rgb) semantics."""
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    w, h, n = C.c_int(), C.c_int(), C.c_int()
    check(lib().rt_decode_png(buf, len(data), C.byref(w), C.byref(h), C.byref(n), None, 0), "rt_decode_png")
    out = np.zeros((h.value, w.value, 3), np.uint8)
    check(lib().rt_decode_png(buf, len(data), C.byref(w), C.byref(h), C.byref(n),
                              out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size), "rt_decode_png")
    return out, n.value


class Context:
    """Device context = BoundingVolumeHierarchy(Scene*) + uploaded scene: one GPU (`device`), or one scene
    replica per entry of `devices` (renders split their bands over them)."""

    def __init__(self, scene, device=0, devices=None):
        self.scene = scene  # keep the host scene alive (desc points into it)
        self.h = C.c_void_p()
        d = scene.desc()
        devs = [int(device)] if devices is None else [int(x) for x in devices]
        arr = (C.c_int * len(devs))(*devs)
        check(lib().rt_create(C.byref(d), arr, len(devs), C.byref(self.h)), "rt_create")
        self.devices = devs

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().rt_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        # nothing during interpreter shutdown: HIP's own teardown may already have run, and destroying
        # device resources after it can hang or fault the process -- close() contexts explicitly
        # (module-level sys: an import inside __del__ itself fails once shutdown has begun)
        try:
            if _sys.is_finalizing() or not callable(lib):
                return
            self.close()
        except Exception:  # noqa: BLE001 -- a destructor must not raise
            pass

    def create_ms(self):
        """rt_create's cumulative phase clock (ms): device, ref BVH, BVH2/8, records, materials, uploads, total."""
        out = np.zeros(8, np.float64)
        check(lib().rt_debug_create_ms(self.h, out.ctypes.data_as(C.POINTER(C.c_double)), 8))
        return out[:7]

    def peer_stores(self):
        """rt_ctx_peer_stores: per replica, True if it stores pixels straight into devices[0] (peer access),
        False if it renders band-dense and copies."""
        out = (C.c_int * 64)()
        n = lib().rt_ctx_peer_stores(self.h, out, 64)
        if n < 0:
            check(n, "rt_ctx_peer_stores")
        return [bool(out[i]) for i in range(n)]

    def ref_bvh(self):
        """rt_debug_ref_bvh: (node boxes [n, 6], per node its leaf id or -1, per node its stored children: node
        indices for inner nodes -- BFS order, two per inner node -- and for leaves the objects in stored
        order, triangles as scene index, spheres as num_triangles + sphere index)."""
        nref = lib().rt_debug_ref_bvh(self.h, None, None, None, None)
        if nref < 0:
            check(nref, "rt_debug_ref_bvh")
        d = self.scene.desc()
        nobj = d.num_triangles + d.num_spheres
        boxes = np.zeros((max(nref, 1), 6), np.float32)
        node_leaf = np.zeros(max(nref, 1), np.int32)
        obj_leaf = np.zeros(max(nobj, 1), np.int32)
        obj_key = np.zeros(max(nobj, 1), np.int32)
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))  # noqa: E731
        rc = lib().rt_debug_ref_bvh(self.h, boxes.ctypes.data_as(C.POINTER(C.c_float)), ip(node_leaf), ip(obj_leaf),
                                    ip(obj_key))
        if rc < 0:  # (returns the node count)
            check(rc, "rt_debug_ref_bvh")
        boxes, node_leaf, obj_leaf, obj_key = boxes[:nref], node_leaf[:nref], obj_leaf[:nobj], obj_key[:nobj]
        children, nxt = [], 1
        for i in range(nref):
            if node_leaf[i] >= 0:
                objs = np.nonzero(obj_leaf == node_leaf[i])[0]
                children.append(objs[np.argsort(obj_key[objs], kind="stable")].astype(np.int32))
            else:  # BFS: the inner nodes' children were created in order, two each
                children.append(np.array([nxt, nxt + 1], np.int32))
                nxt += 2
        return boxes, node_leaf, children

    def build_info(self):
        """rt_debug_build_info: built on the GPU?, BVH2 nodes, BVH2 depth, BVH8 nodes."""
        out = (C.c_int * 4)()
        check(lib().rt_debug_build_info(self.h, out, 4))
        return {"gpu": bool(out[0]), "bvh2_nodes": out[1], "bvh2_depth": out[2], "bvh8_nodes": out[3]}

    def records(self, first=0, count=None):
        """rt_debug_records: float32 [count, 16] triangle records in BVH8 leaf order."""
        if count is None:
            count = self.info()["tri_records"] - first
        out = np.zeros((count, 16), np.float32)
        check(lib().rt_debug_records(self.h, out.ctypes.data_as(C.POINTER(C.c_float)), first, count))
        return out

    def info(self):
        a, b, c, d = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        check(lib().rt_ctx_info(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return {"bvh_nodes": a.value, "tri_records": b.value, "ref_bvh_nodes": c.value, "ref_bvh_levels": d.value}

    def render(self, cam, prm, W, H):
        """renderRayTracing: returns (float32 [H*W*3] in Screen::m_textureData order, rt_stats)."""
        out = np.empty(W * H * 3, np.float32)
        st = rt_stats()
        check(lib().rt_render(self.h, C.byref(cam), C.byref(prm), W, H,
                              out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)), "rt_render")
        return out, st

    def render_device(self, cam, prm, W, H, band_rows, band_rank, band_count, d_out_ptr, stream_ptr=None):
        st = rt_stats()
        check(lib().rt_render_device(self.h, C.byref(cam), C.byref(prm), W, H, band_rows, band_rank, band_count,
                                     C.c_void_p(d_out_ptr), C.c_void_p(stream_ptr or 0), C.byref(st)),
              "rt_render_device")
        return st

    def render_views(self, cams, prm, W, H):
        """A batch of frames to host memory (rt_render_views): float32 [n_views, W*H*3], stats summed."""
        arr = (rt_camera * len(cams))(*cams)
        out = np.zeros((len(cams), W * H * 3), np.float32)
        st = rt_stats()
        check(lib().rt_render_views(self.h, arr, len(cams), C.byref(prm), W, H,
                                    out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)), "rt_render_views")
        return out, st

    def render_views_device(self, cams, prm, W, H, band_rows, band_rank, band_count, d_out_ptr, stream_ptr=None):
        """A batch of frames, one per camera, in one launch (rt_render_views_device); stats summed."""
        arr = (rt_camera * len(cams))(*cams)
        st = rt_stats()
        check(lib().rt_render_views_device(self.h, arr, len(cams), C.byref(prm), W, H, band_rows, band_rank,
                                           band_count, C.c_void_p(d_out_ptr), C.c_void_p(stream_ptr or 0),
                                           C.byref(st)), "rt_render_views_device")
        return st

    def render_views_image_device(self, cams, prm, W, H, d_images_ptr, stream_ptr=None, band_rows=8, band_rank=0,
                                  band_count=1, stats=True):
        """rt_render_views_image_device: the views' pixels straight into d_images (setPixel layout, view v at
        v*W*H*3), split over the context's devices; this call renders bands b % band_count == band_rank.
        stats=False keeps the call asynchronous on the stream (returns None)."""
        arr = (rt_camera * len(cams))(*cams)
        st = rt_stats() if stats else None
        check(lib().rt_render_views_image_device(self.h, arr, len(cams), C.byref(prm), W, H, band_rows, band_rank,
                                                 band_count, C.c_void_p(d_images_ptr), C.c_void_p(stream_ptr or 0),
                                                 C.byref(st) if stats else None), "rt_render_views_image_device")
        return st

    def intersect(self, rays, use_bvh):
        rays = np.ascontiguousarray(rays, dtype=RAY_DTYPE)
        hits = np.zeros(len(rays), HIT_DTYPE)
        check(lib().rt_intersect(self.h, rays.ctypes.data, len(rays), int(use_bvh), hits.ctypes.data), "rt_intersect")
        return hits

    def shade(self, rays, prm):
        rays = np.ascontiguousarray(rays, dtype=RAY_DTYPE)
        rgb = np.zeros(len(rays) * 3, np.float32)
        cnt = np.zeros(len(rays), np.uint64)
        check(lib().rt_shade(self.h, rays.ctypes.data, len(rays), C.byref(prm),
                             rgb.ctypes.data_as(C.POINTER(C.c_float)),
                             cnt.ctypes.data_as(C.POINTER(C.c_uint64))), "rt_shade")
        return rgb.reshape(-1, 3), cnt

    def set_option(self, option, value):
        """rt_ctx_set_option: test / developer hook (every value renders the same image)."""
        check(lib().rt_ctx_set_option(self.h, int(option), int(value)), "rt_ctx_set_option")

    def texture_sample(self, texture, uv_lod, prm):
        """Image::getPixel(uv, lod) on the device for rows (u, v, lod); returns [n, 3] float32."""
        a = np.ascontiguousarray(uv_lod, np.float32).reshape(-1, 3)
        out = np.zeros((len(a), 3), np.float32)
        check(lib().rt_texture_sample(self.h, int(texture), len(a), a.ctypes.data_as(C.POINTER(C.c_float)),
                                      C.byref(prm), out.ctypes.data_as(C.POINTER(C.c_float))), "rt_texture_sample")
        return out

    def update_lights(self, scene):
        """rt_update_lights: take the scene's current light arrays (ImGui light edits)."""
        d = scene.desc()
        check(lib().rt_update_lights(self.h, C.byref(d)), "rt_update_lights")

    def update_materials(self, mesh_materials, sphere_materials=()):
        """rt_update_materials: replace every mesh and sphere material (counts must match)."""
        mm = (rt_material * max(1, len(mesh_materials)))(*mesh_materials)
        sm = (rt_material * max(1, len(sphere_materials)))(*sphere_materials)
        check(lib().rt_update_materials(self.h, len(mesh_materials), mm, len(sphere_materials), sm),
              "rt_update_materials")

    def debug_counters(self, n=32):
        out = np.zeros(n, np.uint64)
        check(lib().rt_debug_counters(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), n))
        return out

    def selftest_math(self, x, y):
        x = np.ascontiguousarray(x, np.float32)
        y = np.ascontiguousarray(y, np.float32)
        out = np.zeros(len(x) * 4, np.float32)
        check(lib().rt_selftest_math(self.h, x.ctypes.data_as(C.POINTER(C.c_float)),
                                     y.ctypes.data_as(C.POINTER(C.c_float)), len(x),
                                     out.ctypes.data_as(C.POINTER(C.c_float))))
        return out.reshape(-1, 4)


def set_counting(on):
    check(lib().rt_set_counting(int(on)))


def slab_check(boxes, rays):
    """rt_debug_slab_check: per (box [lo, hi], ray [origin, normalised direction]) pair the kernels' slab test
    by IEEE quotients (bit 0) and by quotient bounds (>> 1: 0 miss, 1 hit, 2 left to the quotients)."""
    b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    r = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    assert len(b) == len(r)
    out = np.zeros(len(b), np.int32)
    check(lib().rt_debug_slab_check(b.ctypes.data_as(C.POINTER(C.c_float)), r.ctypes.data_as(C.POINTER(C.c_float)),
                                    len(b), out.ctypes.data_as(C.POINTER(C.c_int))), "rt_debug_slab_check")
    return out


class IpcBuffer:
    """Device memory shared across processes (rt_ipc_alloc / rt_ipc_open): the owner allocates and exports
    a handle (bytes), other processes open it; .ptr is the device address in this process."""

    def __init__(self, device, nbytes=None, handle=None):
        self.device = int(device)
        self.ptr = None
        self.owner = handle is None
        p = C.c_void_p()
        if self.owner:
            h = (C.c_uint8 * IPC_HANDLE_BYTES)()
            check(lib().rt_ipc_alloc(self.device, int(nbytes), C.byref(p), h), "rt_ipc_alloc")
            self.handle = bytes(h)
        else:
            h = (C.c_uint8 * IPC_HANDLE_BYTES).from_buffer_copy(bytes(handle))
            check(lib().rt_ipc_open(self.device, h, C.byref(p)), "rt_ipc_open")
            self.handle = bytes(handle)
        self.ptr = p.value

    def close(self):
        if self.ptr:
            if self.owner:
                lib().rt_device_free(self.device, C.c_void_p(self.ptr))
            else:
                lib().rt_ipc_close(C.c_void_p(self.ptr))
            self.ptr = None


def device_to_host(d_ptr, n):
    """n float32 from device memory (e.g. an IpcBuffer) to a new host array (synchronous)."""
    out = np.empty(int(n), np.float32)
    check(lib().rt_memcpy_dtoh(out.ctypes.data, C.c_void_p(d_ptr), out.nbytes), "rt_memcpy_dtoh")
    return out


def device_synchronize(device):
    check(lib().rt_device_synchronize(int(device)), "rt_device_synchronize")


# --------------------------------------------------------------------------------------------
# Multi-GPU band partition (rt_render_device / rt_unpermute_bands_device contract)
# --------------------------------------------------------------------------------------------
def band_rows_of(H, band_rows, rank, count):
    """Image rows (reference y, 0 = bottom) a rank renders, in its dense output order."""
    nbands = (H + band_rows - 1) // band_rows
    rows = []
    for gb in range(rank, nbands, count):
        rows.extend(range(gb * band_rows, min((gb + 1) * band_rows, H)))
    return rows


def local_band_elems(W, H, band_rows, count):
    """Floats in one rank's (padded) band buffer: max_local_bands * band_rows * W * 3."""
    nbands = (H + band_rows - 1) // band_rows
    return ((nbands + count - 1) // count) * band_rows * W * 3


def unpermute_views_host(gathered, W, H, band_rows, count, n_views):
    """Host statement of unpermute_views_kernel: [count][n_views][max_local][band_rows][W][3] ->
    n_views images in Screen::m_textureData order."""
    nbands = (H + band_rows - 1) // band_rows
    max_local = (nbands + count - 1) // count
    g = np.asarray(gathered, np.float32).reshape(count, n_views, max_local * band_rows * W * 3)
    return np.stack([unpermute_host(g[:, v].reshape(-1), W, H, band_rows, count) for v in range(n_views)])


def unpermute_host(gathered, W, H, band_rows, count):
    """Host statement of unpermute_kernel: gathered [count][max_local][band_rows][W][3] ->
    Screen::m_textureData order (row H-1-y first, src/screen.cpp:32-38)."""
    nbands = (H + band_rows - 1) // band_rows
    max_local = (nbands + count - 1) // count
    g = np.asarray(gathered, np.float32).reshape(count, max_local, band_rows, W, 3)
    out = np.zeros((H, W, 3), np.float32)
    for y in range(H):
        gb, r = divmod(y, band_rows)
        out[H - 1 - y] = g[gb % count, gb // count, r]
    return out.reshape(-1)


# --------------------------------------------------------------------------------------------
# Scene data: the reference's data/*.obj/.mtl inputs ship gzip-compressed under
# tests/golden/scenes/ and are expanded into a cache dir (the GPU box has no /root/reference).
# --------------------------------------------------------------------------------------------
def cache_dir():
    d = os.environ.get("RT_SCENE_CACHE") or os.path.join(tempfile.gettempdir(), f"rt_amd_scenes_{os.getuid()}")
    os.makedirs(d, exist_ok=True)
    return d


def data_dir():
    """Directory holding the expanded reference scene files (tr_def, cube, monkey, Cornell)."""
    out = cache_dir()
    for f in sorted(os.listdir(SCENE_DIR)):
        if not f.endswith(".gz"):
            continue
        dst = os.path.join(out, f[:-3])
        src = os.path.join(SCENE_DIR, f)
        if not os.path.exists(dst) or os.path.getmtime(dst) < os.path.getmtime(src):
            # per-process temporary: ranks of one node expand the same files concurrently
            tmp = f"{dst}.{os.getpid()}.tmp"
            with gzip.open(src, "rb") as fi, open(tmp, "wb") as fo:
                shutil.copyfileobj(fi, fo)
            os.replace(tmp, dst)
    return out


DRAGON_U, DRAGON_V = 1000, 400  # 800 000 triangles


def dragon_proxy_path(u=DRAGON_U, v=DRAGON_V):
    path = os.path.join(cache_dir(), f"dragon_proxy_{u}x{v}.obj")
    if not os.path.exists(path):
        tmp = path + f".{os.getpid()}.obj"
        check(lib().rt_write_dragon_proxy(tmp.encode(), u, v), "rt_write_dragon_proxy")
        mtl_tmp = tmp[:-4] + ".mtl"
        # the .obj names its .mtl by basename: rewrite both to the final names
        with open(tmp) as f:
            text = f.read().replace(os.path.basename(mtl_tmp), os.path.basename(path)[:-4] + ".mtl", 1)
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(mtl_tmp, path[:-4] + ".mtl")
        os.replace(tmp, path)
    return path


# SceneType (src/scene.h:14-34)
PRESETS = {"SingleTriangle": 0, "Bookeshelf": 1, "Cube": 2, "CornellBox": 3, "CornellBoxSphericalLight": 4,
           "CornellBoxPlaneLight": 5, "Monkey": 6, "Teapot": 7, "Dragon": 8, "Spheres": 9, "ChessBoard": 10,
           "Custom": 11, "AndreasScene": 12, "CatalinScene": 13, "MikeScene": 14, "MikeScene2": 15}


def build_config(name, dragon_uv=None):
    """BASELINE.json configs as fixed by SURVEY.md §8d.  Returns (scene, params, W, H, description)."""
    dd = data_dir()
    s = Scene()
    if name == "C1":
        s.load_obj(os.path.join(dd, "cube.obj"), normalize=False)
        s.add_point_light((-1, 1, -1), (1, 1, 1))
        return s, params(max_reflection_level=0, glossy_ray_count=1), 256, 256, \
            "cube.obj 256x256, primary rays, depth 0, 1 point light"
    if name == "C2":
        s.preset(PRESETS["Monkey"], dd)
        return s, params(max_reflection_level=1, glossy_ray_count=1), 1024, 1024, \
            "monkey-rotated.obj 1024x1024, Phong + hard shadows, depth 1"
    if name in ("C3", "C4"):
        u, v = dragon_uv or (DRAGON_U, DRAGON_V)
        s.load_obj(dragon_proxy_path(u, v), normalize=True)
        if name == "C3":
            s.add_point_light((-1, 1, -1), (1, 1, 1))
            return s, params(max_reflection_level=4, glossy_ray_count=1), 1920, 1080, \
                f"dragon-proxy ({2 * u * v} tris) 1920x1080, hard shadows + mirror depth 4"
        s.add_spherical_light((-1, 1, -1), 0.1, (1, 1, 1))
        return s, params(max_reflection_level=0, sphere_light_ray_count=64, glossy_ray_count=1), 1920, 1080, \
            f"dragon-proxy ({2 * u * v} tris) 1920x1080, spherical light 64 samples"
    if name == "C5":
        s.preset(PRESETS["CornellBox"], dd)  # meshes + glass sphere + point light
        s.clear_lights()
        third = float(np.float32(1.0) / np.float32(3.0))
        for dx in (0.0, -0.3, 0.3):
            pos = (float(np.float32(-0.1) + np.float32(dx)), 0.63, -0.1)
            s.add_plane_light(pos, (0.15, -0.05, 0.0), (0.0, 0.0, 0.2), (third, third, third))
        return s, params(max_reflection_level=8, plane_light_1D_ray_count=8, glossy_ray_count=1), 3840, 2160, \
            "CornellBox-Mirror-Rotated 3840x2160, depth 8, 3 plane lights x 64 samples"
    raise ValueError(name)
