"""Golden-fixture cases shared by tools/make_golden.py and the tests."""


# (name, config, W, H, dragon_uv, param overrides)
IMAGES = [
    ("c1_64", "C1", 64, 64, None, {}),
    ("c2_64x48", "C2", 64, 48, None, {}),
    ("c2_aa_32", "C2", 32, 32, None, {"anti_aliasing": 1}),
    ("c2_ms16_24", "C2", 24, 24, None, {"multiple_rays": 1, "sample_size": 16}),
    ("c2_bvh_48", "C2", 48, 48, None, {"use_bvh": 1}),
    ("c3s_96x54", "C3", 96, 54, (200, 80), {}),
    ("c4s_64x36", "C4", 64, 36, (200, 80), {}),
    ("c5_96x54", "C5", 96, 54, None, {}),
    ("c5_depth3_bvh_64x36", "C5", 64, 36, None, {"max_reflection_level": 3, "use_bvh": 1}),
]
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
