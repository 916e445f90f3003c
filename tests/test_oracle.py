"""The CPU oracle (oracle/ref_cpu.cpp) against the committed golden vectors and against
properties the reference's algorithm guarantees.  These vectors were produced by
tools/make_golden.py and pin the restatement against regressions; the pin to a reference-held
output (render.bmp) is tests/test_render_bmp_pin.py."""
import numpy as np
import pytest

from golden_cases import IMAGES, NATIVE_800, PRESET_IMAGES, REF_BVH_SCENES, apply


def golden_images(golden_dir):
    z = np.load(f"{golden_dir}/images.npz")
    out = {}
    for k in z.files:
        name, field = k.split("__")
        out.setdefault(name, {})[field] = z[k]
    return out


def scene_for(R, case):
    name, cfg, W, H, uv, over = case
    scene, prm, _, _, _ = R.build_config(cfg, dragon_uv=uv)
    return scene, apply(prm, over), W, H


@pytest.mark.parametrize("case", IMAGES, ids=[c[0] for c in IMAGES])
def test_oracle_reproduces_golden_images(R, O, golden_dir, case):
    g = golden_images(golden_dir)[case[0]]
    scene, prm, W, H = scene_for(R, case)
    img, rays = O.Oracle(scene).render(prm, W, H)
    assert rays == int(g["rays"])
    assert img.tobytes() == g["img"].tobytes()


@pytest.mark.parametrize("case", PRESET_IMAGES, ids=[c[0] for c in PRESET_IMAGES])
def test_oracle_reproduces_preset_images(R, O, golden_dir, case):
    name, preset, W, H, over = case
    g = golden_images(golden_dir)[name]
    scene = R.Scene().preset(R.PRESETS[preset], R.data_dir())
    prm = apply(R.params(), over)
    img, rays = O.Oracle(scene).render(prm, W, H)
    assert rays == int(g["rays"])
    assert img.tobytes() == g["img"].tobytes()


def test_single_triangle_red_equals_blue(golden_dir):
    # white point light + magenta spherical light on a kd = 1 surface: R == B everywhere
    # (the same invariant render.bmp shows for this scene)
    img = golden_images(golden_dir)["single_triangle_64"]["img"].reshape(-1, 3)
    assert np.array_equal(img[:, 0], img[:, 2])
    assert (img[:, 0] > img[:, 1]).any()


@pytest.mark.parametrize("cfg", ["C1", "C2", "C5"])
def test_oracle_kats(R, O, golden_dir, cfg):
    z = np.load(f"{golden_dir}/kats.npz")
    scene, _, _, _, _ = R.build_config(cfg)
    orc = O.Oracle(scene)
    rays = z[f"{cfg}__rays"]
    for ub in (0, 1):
        hits = orc.intersect(rays, ub, R.HIT_DTYPE)
        assert hits.tobytes() == z[f"{cfg}_bvh{ub}__hits"].tobytes()


@pytest.mark.parametrize("cfg", ["C1", "C2", "C5"])
def test_bvh_hits_are_brute_force_hits(R, golden_dir, cfg):
    """useBVH=true tests a subset of the candidates of useBVH=false: for unit directions a BVH hit
    implies a brute-force hit at t_brute <= t_bvh."""
    z = np.load(f"{golden_dir}/kats.npz")
    rays = z[f"{cfg}__rays"]
    h0, h1 = z[f"{cfg}_bvh0__hits"], z[f"{cfg}_bvh1__hits"]
    unit = np.abs((rays["direction"].astype(np.float64) ** 2).sum(1) - 1) < 1e-6
    sel = unit & (h1["hit"] == 1)
    assert sel.sum() > 100
    assert np.all(h0["hit"][sel] == 1)
    assert np.all(h0["t"][sel] <= h1["t"][sel])


def test_ray_counts_split(R, O):
    """Shading one camera ray through rt_shade's semantics == one pixel of the render loop."""
    scene, prm, _, _, _ = R.build_config("C2")
    orc = O.Oracle(scene)
    W, H = 16, 16
    img, total = orc.render(prm, W, H)
    xy = np.array([(x, y) for y in range(H) for x in range(W)], np.int32)
    rgb, rays = orc.render_pixels(prm, W, H, xy)
    assert int(rays.sum()) == total
    flipped = img.reshape(H, W, 3)[::-1].reshape(-1, 3)
    assert rgb.tobytes() == flipped.tobytes()


def ref_bvh_fixture(golden_dir, cfg):
    z = np.load(f"{golden_dir}/ref_bvh.npz")
    off = z[f"{cfg}__offsets"]
    ch = z[f"{cfg}__children"]
    kids = [ch[off[i]:off[i + 1]] for i in range(len(off) - 1)]
    return z[f"{cfg}__boxes"], z[f"{cfg}__is_leaf"], kids


@pytest.mark.parametrize("cfg", REF_BVH_SCENES)
def test_oracle_ref_bvh_matches_fixture(R, O, golden_dir, cfg):
    """constructBVH's depth-4 median BVH (src/bounding_volume_hierarchy.cpp:108-217) of cube, monkey and
    Cornell: node boxes bit for bit, leaf flags and every node's stored children (BFS node indices, a leaf's
    objects in stored order) -- the dump tests/test_gpu_build.py holds the host and GPU builders to."""
    boxes, leaf, kids = ref_bvh_fixture(golden_dir, cfg)
    scene, _, _, _, _ = R.build_config(cfg)
    orc = O.Oracle(scene)
    b, l = orc.bvh_nodes()
    assert b.tobytes() == boxes.tobytes()
    assert np.array_equal(l, leaf)
    for i in range(len(b)):
        assert np.array_equal(orc.bvh_children(i), kids[i]), i
    # structure: BFS creation order, <= 16 leaves at depth <= 4, every object in exactly one leaf
    objs = np.concatenate([kids[i] for i in range(len(b)) if leaf[i]])
    d = scene.desc()
    assert np.array_equal(np.sort(objs), np.arange(d.num_triangles + d.num_spheres))
    assert int(leaf.sum()) <= 16


def native_fixture(golden_dir):
    z = np.load(f"{golden_dir}/native800.npz")
    return {n: (z[f"{n}__img"], int(z[f"{n}__rays"])) for n, _ in NATIVE_800}


@pytest.mark.parametrize("name,cfg", NATIVE_800, ids=[n for n, _ in NATIVE_800])
def test_oracle_native_800_sampled(R, O, golden_dir, name, cfg):
    """renderRayTracing's native 800x800 frames (src/main.cpp:33): 2 048 pixels of each re-rendered by the
    oracle bit for bit (the GPU renders the whole frame in test_gpu_parity.py)."""
    img, _ = native_fixture(golden_dir)[name]
    scene, prm, _, _, _ = R.build_config(cfg)
    sel = np.random.default_rng(800).permutation(800 * 800)[:2048]
    xy = np.stack([sel % 800, sel // 800], axis=1).astype(np.int32)
    got, _ = O.Oracle(scene).render_pixels(prm, 800, 800, xy)
    ref = img.reshape(800, 800, 3)[::-1].reshape(-1, 3)[sel]  # setPixel rows are top-first
    assert got.reshape(-1, 3).tobytes() == ref.tobytes()
