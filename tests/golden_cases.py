"""Golden-fixture cases shared by tools/make_golden.py and the tests."""


# (name, config, W, H, dragon_uv, param overrides)
IMAGES = [
    ("c1_64", "C1", 64, 64, None, {}),
    ("c2_64x48", "C2", 64, 48, None, {}),
    ("c2_aa_32", "C2", 32, 32, None, {"anti_aliasing": 1}),
    ("c2_ms16_24", "C2", 24, 24, None, {"multiple_rays": 1, "sample_size": 16}),
    ("c2_ms4_32", "C2", 32, 32, None, {"multiple_rays": 1, "sample_size": 4}),    # getPixelRays 4 (src/main.cpp:309-335)
    ("c2_ms64_16", "C2", 16, 16, None, {"multiple_rays": 1, "sample_size": 64}),  # ... and 64 (the 6-bit sample field)
    ("c2_bvh_48", "C2", 48, 48, None, {"use_bvh": 1}),
    ("c3s_96x54", "C3", 96, 54, (200, 80), {}),
    ("c4s_64x36", "C4", 64, 36, (200, 80), {}),
    ("c5_96x54", "C5", 96, 54, None, {}),
    ("c5_depth3_bvh_64x36", "C5", 64, 36, None, {"max_reflection_level": 3, "use_bvh": 1}),
]
# native 800x800 frames (renderRayTracing's constexpr windowResolution, src/main.cpp:33) of C1, C2 and C5
# at their BASELINE knobs: tests/golden/native800.npz
NATIVE_800 = [("c1_800", "C1"), ("c2_800", "C2"), ("c5_800", "C5")]
# scenes whose reference depth-4 BVH (constructBVH) is dumped to tests/golden/ref_bvh.npz
REF_BVH_SCENES = ["C1", "C2", "C5"]
PRESET_IMAGES = [
    # loadScene presets with the reference's default knobs (glossy_ray_count forced to 1: no rand())
    ("single_triangle_64", "SingleTriangle", 64, 64, {"glossy_ray_count": 1}),
    ("cube_preset_64", "Cube", 64, 64, {"glossy_ray_count": 1}),
    ("cornell_spherical_48", "CornellBoxSphericalLight", 48, 48, {"glossy_ray_count": 1, "max_reflection_level": 3}),
    ("cornell_plane_48", "CornellBoxPlaneLight", 48, 48, {"glossy_ray_count": 1, "max_reflection_level": 3}),
]


def apply(prm, over):
    for k, v in over.items():
        setattr(prm, k, v)
    return prm
