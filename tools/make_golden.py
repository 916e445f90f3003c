"""Generate tests/golden/*.npz with the CPU oracle (oracle/ref_cpu.cpp).

The reference ships no tests, golden vectors or fixtures for this path and cannot
be built here, so these vectors are produced by the restatement itself: they pin the oracle
(regression) and are what the GPU parity tests compare against.  The oracle itself is pinned to
the reference's render.bmp (tests/test_render_bmp_pin.py).  Re-run after an intentional semantic change:

    python tools/make_golden.py              # images.npz, kats.npz
    python tools/make_golden.py --ref-bvh    # ref_bvh.npz
    python tools/make_golden.py --native800  # native800.npz
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
import rt_amd as R  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")

from golden_cases import IMAGES, NATIVE_800, PRESET_IMAGES, REF_BVH_SCENES, apply  # noqa: E402


def render_case(scene, prm, W, H):
    orc = O.Oracle(scene)
    img, rays = orc.render(prm, W, H)
    return img, rays


def kat_rays(scene, n, seed):
    """Rays for intersect() known-answer tests: random, camera-through-vertex and edge-midpoint rays."""
    rng = np.random.default_rng(seed)
    pos, _, _, _ = scene.arrays()
    lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
    c = (lo + hi) / 2
    ext = float(np.max(hi - lo)) + 1e-3
    rays = np.zeros(n, R.RAY_DTYPE)
    k = n // 3
    # 1) random origins around the scene, random directions
    o = c + (rng.random((k, 3)) - 0.5) * 3 * ext
    d = rng.normal(size=(k, 3))
    rays["origin"][:k] = o
    rays["direction"][:k] = d
    # 2) from the default camera towards vertices and edge midpoints (hits on shared edges: tie-breaks)
    cam = R.camera_from_trackball(aspect=1.0)
    cpos = np.array(list(cam.position), np.float32)
    tri = rng.integers(0, len(pos), size=k)
    a = rng.integers(0, 3, size=k)
    b = (a + rng.integers(1, 3, size=k)) % 3
    tgt = np.where(rng.random(k)[:, None] < 0.5, pos[tri, a], (pos[tri, a] + pos[tri, b]) * np.float32(0.5))
    rays["origin"][k:2 * k] = cpos
    rays["direction"][k:2 * k] = tgt - cpos
    # 3) secondary-like rays starting on the surface (offset along the normal direction)
    m = n - 2 * k
    tri = rng.integers(0, len(pos), size=m)
    w = rng.random((m, 3)).astype(np.float32)
    w /= w.sum(1, keepdims=True)
    p = (pos[tri] * w[:, :, None]).sum(1)
    rays["origin"][2 * k:] = p + rng.normal(size=(m, 3)).astype(np.float32) * np.float32(1e-3)
    rays["direction"][2 * k:] = rng.normal(size=(m, 3))
    rays["t"] = R.FLT_MAX
    # every other ray gets a unit direction (glm::normalize order: v * (1/sqrt(dot)))
    dsel = rays["direction"][::2].astype(np.float32)
    dot = (dsel[:, 0] * dsel[:, 0] + dsel[:, 1] * dsel[:, 1]) + dsel[:, 2] * dsel[:, 2]
    rays["direction"][::2] = dsel * (np.float32(1.0) / np.sqrt(dot))[:, None]
    return rays


def ref_bvh_dumps():
    """tests/golden/ref_bvh.npz: the reference depth-4 BVH (constructBVH, src/bounding_volume_hierarchy.cpp:108-217)
    of each scene as the oracle builds it -- node boxes (BFS creation order), leaf flags and every node's stored
    children (node indices, or a leaf's objects in stored order: triangles by scene index, spheres as
    num_triangles + sphere index), flattened with offsets."""
    out = {}
    for cfg in REF_BVH_SCENES:
        scene, _, _, _, _ = R.build_config(cfg)
        orc = O.Oracle(scene)
        boxes, leaf = orc.bvh_nodes()
        kids = [orc.bvh_children(i) for i in range(len(boxes))]
        off = np.cumsum([0] + [len(k) for k in kids]).astype(np.int32)
        out[f"{cfg}__boxes"] = boxes
        out[f"{cfg}__is_leaf"] = leaf
        out[f"{cfg}__children"] = np.concatenate(kids).astype(np.int32)
        out[f"{cfg}__offsets"] = off
        print(cfg, "ref BVH nodes", len(boxes), "leaves", int(leaf.sum()))
    np.savez_compressed(os.path.join(OUT, "ref_bvh.npz"), **out)


def native_800():
    """tests/golden/native800.npz: C1, C2 and C5 at renderRayTracing's native 800x800 (src/main.cpp:33)."""
    out = {}
    O.set_threads(os.cpu_count() or 1)
    for name, cfg in NATIVE_800:
        scene, prm, _, _, _ = R.build_config(cfg)
        img, rays = render_case(scene, prm, 800, 800)
        out[f"{name}__img"] = img
        out[f"{name}__rays"] = np.uint64(rays)
        print(name, rays, float(img.max()))
    np.savez_compressed(os.path.join(OUT, "native800.npz"), **out)


def main():
    if "--ref-bvh" in sys.argv:
        return ref_bvh_dumps()
    if "--native800" in sys.argv:
        return native_800()
    os.makedirs(OUT, exist_ok=True)
    images = {}
    for name, cfg, W, H, uv, over in IMAGES:
        scene, prm, _, _, desc = R.build_config(cfg, dragon_uv=uv)
        apply(prm, over)
        img, rays = render_case(scene, prm, W, H)
        images[name] = dict(img=img, rays=np.uint64(rays), W=W, H=H, config=cfg, uv=np.array(uv or (0, 0)),
                            over=repr(over))
        print(name, W, H, rays, float(img.max()))
    for name, preset, W, H, over in PRESET_IMAGES:
        scene = R.Scene().preset(R.PRESETS[preset], R.data_dir())
        prm = apply(R.params(), over)
        img, rays = render_case(scene, prm, W, H)
        images[name] = dict(img=img, rays=np.uint64(rays), W=W, H=H, config="preset:" + preset,
                            uv=np.array((0, 0)), over=repr(over))
        print(name, W, H, rays, float(img.max()))
    np.savez_compressed(os.path.join(OUT, "images.npz"),
                        **{f"{k}__{f}": v[f] for k, v in images.items() for f in v})

    kats = {}
    for cfg, n, seed in [("C1", 3000, 1), ("C2", 3000, 2), ("C5", 3000, 3)]:
        scene, _, _, _, _ = R.build_config(cfg)
        rays = kat_rays(scene, n, seed)
        orc = O.Oracle(scene)
        for ub in (0, 1):
            hits = orc.intersect(rays, ub, R.HIT_DTYPE)
            kats[f"{cfg}_bvh{ub}__hits"] = hits
            print(cfg, "use_bvh", ub, "hits", int(hits["hit"].sum()), "/", n)
        kats[f"{cfg}__rays"] = rays
    np.savez_compressed(os.path.join(OUT, "kats.npz"), **kats)


if __name__ == "__main__":
    main()
