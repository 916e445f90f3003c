"""ORACLE ctypes wrapper -- test infrastructure only.

Loads oracle/build/liboracle.so (CPU restatement of the reference hot path, ref_cpu.cpp).
May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker or the timed CPU baseline.  Parity status: pinned to the reference's render.bmp (see ref_cpu.cpp header).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
if os.environ.get("ORACLE_SANITIZER_LIB"):  # tools/sanitize/run.sh: the ASan/UBSan build of the same sources
    LIB = os.environ["ORACLE_SANITIZER_LIB"]

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp = C.c_void_p
        F3 = C.POINTER(C.c_float)
        L.oracle_create.argtypes = [vp]
        L.oracle_create.restype = vp
        L.oracle_destroy.argtypes = [vp]
        L.oracle_bvh_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_bvh_nodes.argtypes = [vp, F3, C.POINTER(C.c_int), C.c_int]
        L.oracle_bvh_children.argtypes = [vp, C.c_int, C.POINTER(C.c_int), C.c_int]
        L.oracle_intersect.argtypes = [vp, vp, C.c_int, C.c_int, vp]
        L.oracle_shade.argtypes = [vp, vp, C.c_int, vp, F3, C.POINTER(C.c_uint64)]
        L.oracle_camera.argtypes = [F3, F3, C.c_float, C.c_float, C.c_float, F3]
        L.oracle_render_pixels.argtypes = [vp, F3, F3, C.c_float, C.c_float, C.c_int, C.c_int, vp,
                                           C.POINTER(C.c_int), C.c_int, F3, C.POINTER(C.c_uint64),
                                           C.POINTER(C.c_uint64)]
        L.oracle_render.argtypes = [vp, F3, F3, C.c_float, C.c_float, C.c_int, C.c_int, vp, F3,
                                    C.POINTER(C.c_uint64)]
        L.oracle_set_threads.argtypes = [C.c_int]
        L.oracle_tex_sample.argtypes = [vp, C.c_int, F3, C.c_int, vp, F3]
        U3 = C.POINTER(C.c_uint32)
        L.oracle_philox.argtypes = [U3, U3, U3]
        L.oracle_postprocess.argtypes = [vp, C.c_int, C.c_int, F3]
        L.oracle_bitmap.argtypes = [vp, C.c_int, C.c_int, F3, C.POINTER(C.c_uint8)]
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Oracle:
    """CPU reference for one scene (takes the product loader's flat rt_scene_desc)."""

    def __init__(self, scene):
        self.scene = scene
        d = scene.desc()
        self._desc = d
        self.h = lib().oracle_create(C.addressof(d))

    def __del__(self):
        import sys as _sys

        if getattr(_sys, "is_finalizing", lambda: False)() or not callable(lib):
            return  # interpreter shutdown: the module's globals may be gone
        if getattr(self, "h", None):
            lib().oracle_destroy(self.h)
            self.h = None

    def bvh_nodes(self):
        n, l = C.c_int(), C.c_int()
        lib().oracle_bvh_info(self.h, C.byref(n), C.byref(l))
        boxes = np.zeros(n.value * 6, np.float32)
        leaf = np.zeros(n.value, np.int32)
        lib().oracle_bvh_nodes(self.h, _fp(boxes), leaf.ctypes.data_as(C.POINTER(C.c_int)), n.value)
        return boxes.reshape(-1, 6), leaf

    def bvh_children(self, node):
        """constructBVH's stored children of `node`: node indices (inner) or, for a leaf, its objects in
        stored order (triangle scene index; spheres as num_triangles + sphere index)."""
        n = lib().oracle_bvh_children(self.h, int(node), None, 0)
        out = np.zeros(max(n, 1), np.int32)
        lib().oracle_bvh_children(self.h, int(node), out.ctypes.data_as(C.POINTER(C.c_int)), n)
        return out[:n]

    def intersect(self, rays, use_bvh, hit_dtype):
        rays = np.ascontiguousarray(rays)
        hits = np.zeros(len(rays), hit_dtype)
        lib().oracle_intersect(self.h, rays.ctypes.data, len(rays), int(use_bvh), hits.ctypes.data)
        return hits

    def shade(self, rays, prm):
        rays = np.ascontiguousarray(rays)
        rgb = np.zeros(len(rays) * 3, np.float32)
        cnt = np.zeros(len(rays), np.uint64)
        lib().oracle_shade(self.h, rays.ctypes.data, len(rays), C.addressof(prm), _fp(rgb),
                           cnt.ctypes.data_as(C.POINTER(C.c_uint64)))
        return rgb.reshape(-1, 3), cnt

    def texture_sample(self, texture, uv_lod, prm):
        """Image::getPixel(uv, lod) for rows (u, v, lod); returns [n, 3] float32."""
        a = np.ascontiguousarray(uv_lod, np.float32).reshape(-1, 3)
        out = np.zeros((len(a), 3), np.float32)
        rc = lib().oracle_tex_sample(self.h, int(texture), _fp(a), len(a), C.addressof(prm), _fp(out))
        if rc != 0:
            raise ValueError(f"no texture {texture}")
        return out

    @staticmethod
    def camera(look_at, euler, dist, fovy, aspect):
        out = np.zeros(9, np.float32)
        la = np.asarray(look_at, np.float32)
        eu = np.asarray(euler, np.float32)
        lib().oracle_camera(_fp(la), _fp(eu), float(dist), float(fovy), float(aspect), _fp(out))
        return out

    def render_pixels(self, prm, W, H, xy, look_at=(0, 0, 0), euler=None, dist=3.0, fovy=None, with_ub=False):
        """Colours and intersect() counts of the listed (x, y) pixels; with_ub adds the per-pixel count
        of shaded hits in the reference's undefined-barycentrics regime."""
        from_rt = _rt()
        euler = from_rt.default_euler() if euler is None else euler
        fovy = from_rt.default_fovy() if fovy is None else fovy
        xy = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
        rgb = np.zeros(len(xy) * 3, np.float32)
        rays = np.zeros(len(xy), np.uint64)
        ub = np.zeros(len(xy), np.uint64)
        la = np.asarray(look_at, np.float32)
        eu = np.asarray(euler, np.float32)
        lib().oracle_render_pixels(self.h, _fp(la), _fp(eu), float(dist), float(fovy), W, H, C.addressof(prm),
                                   xy.ctypes.data_as(C.POINTER(C.c_int)), len(xy), _fp(rgb),
                                   rays.ctypes.data_as(C.POINTER(C.c_uint64)), ub.ctypes.data_as(C.POINTER(C.c_uint64)))
        if with_ub:
            return rgb.reshape(-1, 3), rays, ub
        return rgb.reshape(-1, 3), rays

    def render(self, prm, W, H, look_at=(0, 0, 0), euler=None, dist=3.0, fovy=None):
        from_rt = _rt()
        euler = from_rt.default_euler() if euler is None else euler
        fovy = from_rt.default_fovy() if fovy is None else fovy
        rgb = np.zeros(W * H * 3, np.float32)
        total = C.c_uint64()
        la = np.asarray(look_at, np.float32)
        eu = np.asarray(euler, np.float32)
        lib().oracle_render(self.h, _fp(la), _fp(eu), float(dist), float(fovy), W, H, C.addressof(prm), _fp(rgb),
                            C.byref(total))
        return rgb, total.value


def postprocess(rgb, W, H, prm):
    """Screen::postprocessImage restated on the CPU (ref_post.cpp); prm is an rt_post_params."""
    out = np.ascontiguousarray(rgb, np.float32).copy()
    lib().oracle_postprocess(C.addressof(prm), W, H, _fp(out))
    return out


def bitmap(rgb, W, H, prm):
    """Screen::writeBitmapToFile's pixel path restated on the CPU: (bloomed floats, RGBA8)."""
    out = np.ascontiguousarray(rgb, np.float32).copy()
    rgba = np.zeros(W * H * 4, np.uint8)
    lib().oracle_bitmap(C.addressof(prm), W, H, _fp(out), rgba.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out, rgba


def set_threads(n):
    return lib().oracle_set_threads(int(n))


def _rt():
    import importlib
    import sys
    pkg = os.path.join(os.path.dirname(HERE), "raytracer-group27_amd")
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    return importlib.import_module("rt_amd")
