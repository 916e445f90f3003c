"""The C++ facade (include/rt_facade.hpp) keeps the reference's data model and signatures
(src/scene.h:48-94, src/mesh.h:14-46, src/ray_tracing.h:6-35, src/main.cpp:129,340-341) and drives the
C-ABI the way the reference's main.cpp drives BoundingVolumeHierarchy / getFinalColor /
renderRayTracing.  tests/cpp/facade_example.cpp is written like main.cpp; its intersect / getFinalColor /
frame outputs (including light and material edits made through the Scene's public vectors after the
BVH exists) are compared here with the oracle."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_example(tmp_path):
    exe = str(tmp_path / "facade_example")
    lib_dir = os.path.join(REPO, "raytracer-group27_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "facade_example.cpp"), "-L", lib_dir, "-lrt_amd",
                    f"-Wl,-rpath,{lib_dir}", "-o", exe], check=True)
    return exe


def test_facade_builds_and_fails_loudly_without_gpu(R, tmp_path):
    import torch

    exe = build_example(tmp_path)
    if torch.cuda.is_available():
        pytest.skip("GPU present: see test_facade_matches_oracle_on_gpu")
    r = subprocess.run([exe, R.data_dir(), str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "no HIP device" in r.stdout
    assert "meshes=1 triangles=968 vertices=1968 pointLights=2" in r.stdout  # loadScene's data model


@pytest.mark.gpu
def test_facade_matches_oracle_on_gpu(R, O, tmp_path):
    exe = build_example(tmp_path)
    r = subprocess.run([exe, R.data_dir(), str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "views_identical=3/3" in r.stdout, r.stdout
    assert "autosync stale_same=1 fresh_differs=1 restored=1" in r.stdout, r.stdout

    def load(name, cols):
        return np.fromfile(str(tmp_path / f"{name}.bin"), np.float32).reshape(-1, cols)

    scene = R.Scene().preset(R.PRESETS["Monkey"], R.data_dir())
    prm = R.params(max_reflection_level=1, glossy_ray_count=1)
    o = O.Oracle(scene)
    raw = load("rays", 7)
    rays = np.zeros(len(raw), R.RAY_DTYPE)
    rays["origin"], rays["direction"], rays["t"] = raw[:, 0:3], raw[:, 3:6], raw[:, 6]
    # the facade's Trackball::generateRay = the oracle's camera rays, bit for bit
    cam = O.Oracle.camera((0, 0, 0), R.default_euler(), 3.0, R.default_fovy(), R.aspect_of(64, 48))
    assert raw[:, 0:3].tobytes() == np.tile(cam[0:3], (len(raw), 1)).astype(np.float32).tobytes()
    kd = np.array([m.kd[0] for m in scene.arrays()[3]], np.float32)
    for b in (0, 1):
        got = load(f"hits_bvh{b}", 11)
        ref = o.intersect(rays, b, R.HIT_DTYPE)
        assert np.array_equal(got[:, 0].astype(int), ref["hit"]), b
        h = ref["hit"] == 1
        assert got[h, 1].tobytes() == ref["t"][h].tobytes(), b
        assert got[h, 2:5].tobytes() == ref["normal"][h].tobytes(), b
        assert got[h, 5:8].tobytes() == ref["hit_point"][h].tobytes(), b
        assert np.array_equal(got[h, 8].astype(int), ref["material_index"][h]), b
        assert np.array_equal(got[h, 10], kd[ref["material_index"][h]])  # HitInfo::getMaterial(scene)
    col, _ = o.shade(rays, prm)
    assert float(np.abs(load("colors", 3) - col).max()) <= 1e-5
    p1 = R.rt_params.from_buffer_copy(prm)
    p1.shade_level = 1  # getFinalColor(scene, bvh, ray, 1): no recursion below max_reflection_level 1
    col1, _ = o.shade(rays, p1)
    assert float(np.abs(load("colors_l1", 3) - col1).max()) <= 1e-5
    assert not np.array_equal(col, col1)
    # frames: as loaded, after the light edits, after the material edit
    f0, _ = o.render(prm, 64, 48)
    assert float(np.abs(load("frame0", 3).reshape(-1) - f0).max()) <= 1e-5
    scene.clear_lights()
    scene.add_point_light((0.5, 1.5, -1.0), (1.0, 1.0, 1.0))
    scene.add_point_light((1.0, -1.0, -1.0), (1.0, 1.0, 1.0))  # the preset's second light, unchanged
    scene.add_spherical_light((-1.0, 1.0, -1.0), 0.1, (0.5, 0.25, 1.0))
    p16 = R.rt_params.from_buffer_copy(prm)
    p16.sphere_light_ray_count = 16
    f1, _ = O.Oracle(scene).render(p16, 64, 48)
    assert float(np.abs(load("frame1", 3).reshape(-1) - f1).max()) <= 1e-5
    m = scene.arrays()[3][0]
    scene.set_material(0, R.material(kd=(0.2, 0.9, 0.3), ks=(0.0, 0.0, 0.0), shininess=m.shininess,
                                     transparency=m.transparency))
    f2, _ = O.Oracle(scene).render(p16, 64, 48)
    assert float(np.abs(load("frame2", 3).reshape(-1) - f2).max()) <= 1e-5
    data = open(tmp_path / "render.bmp", "rb").read()
    assert data[:2] == b"BM" and len(data) == 54 + 32 * 3 * 24
