"""loadMesh / loadScene restatement (src/mesh.cpp:58-188, src/scene.cpp:4-150) with the Assimp 5.0.1
OBJ importer semantics of SURVEY.md Appendix B.  Facts checked here come from the reference's
own data files (tests/golden/scenes/*.gz) and from Assimp's published parser behaviour."""
import os

import numpy as np
import pytest


def load(R, name, normalize=False, x4=False):
    s = R.Scene()
    s.load_obj(os.path.join(R.data_dir(), name), normalize=normalize, shininess_x4=x4)
    return s


def fast_atof(tok):
    """Assimp fast_atoreal_move<float>: float(int) + float(double(frac) * 10^-n), then sign."""
    neg = tok.startswith("-")
    t = tok.lstrip("+-")
    ip, _, fp = t.partition(".")
    f = np.float32(int(ip)) if ip else np.float32(0)
    if fp:
        fp = fp[:15]
        table = [0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001,
                 0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001,
                 0.000000000000001]
        f = np.float32(f + np.float32(float(int(fp)) * table[len(fp)]))
    return np.float32(-f) if neg else f


@pytest.mark.parametrize("name,meshes,tris", [
    ("cube.obj", 6, 12), ("monkey-rotated.obj", 1, 968), ("CornellBox-Mirror-Rotated.obj", 8, 32),
    ("teapot.obj", 2, 15704), ("tr_def.obj", 1, 2)])
def test_mesh_and_triangle_counts(R, name, meshes, tris):
    pos, nrm, mesh, mats = load(R, name).arrays()
    assert len(pos) == tris
    assert len(mats) == meshes
    assert mesh.min() == 0 and mesh.max() == meshes - 1
    assert np.all(np.diff(mesh) >= 0)  # mesh-major scene order


def test_cube_groups_visited_in_reverse(R):
    # 6 'g' groups -> 6 root children; the reference's std::stack pops them last-first.
    _, _, mesh, mats = load(R, "cube.obj").arrays()
    kd = [tuple(np.round(list(m.kd), 2)) for m in mats]
    # file order: back(gray) left(blue) top(red) right(green) bottom(red) front(gray)
    assert kd == [(0.5, 0.5, 0.5), (0.8, 0.0, 0.0), (0.0, 0.8, 0.0), (0.8, 0.0, 0.0), (0.0, 0.0, 0.8), (0.5, 0.5, 0.5)]
    for m in mats:
        assert m.transparency == fast_atof("0.452632")  # 'd' -> opacity
        assert m.shininess == 0.0  # no Ns: ObjFile::Material default
        assert list(m.ks) == [0.0, 0.0, 0.0]


def test_positions_parse_like_fast_atof(R):
    path = os.path.join(R.data_dir(), "CornellBox-Mirror-Rotated.obj")
    verts = [l.split()[1:4] for l in open(path) if l.startswith("v ")]
    pos, _, _, _ = load(R, "CornellBox-Mirror-Rotated.obj").arrays()
    # Cornell: one object, usemtl order floor, ceiling, backWall, rightWall, leftWall, shortBox, tallBox, light;
    # quads fan (0,1,2),(0,2,3).  First triangle = file vertices 1,2,3; second = 1,3,4.
    expect0 = np.array([[fast_atof(t) for t in verts[i]] for i in (0, 1, 2)], np.float32)
    expect1 = np.array([[fast_atof(t) for t in verts[i]] for i in (0, 2, 3)], np.float32)
    assert np.array_equal(pos[0], expect0)
    assert np.array_equal(pos[1], expect1)
    # negative zero in the file ("-0.000000") becomes +0 through glm's identity mat4 * vec4
    flat = pos.reshape(-1)
    assert not np.any((flat == 0) & np.signbit(flat))


def test_fast_atof_is_not_strtof(R, tmp_path):
    # values where float(int) + float(double(frac)*10^-n) differs from correctly rounded strtof
    toks = []
    rng = np.random.default_rng(7)
    for _ in range(400):
        toks.append(f"{rng.uniform(-3, 3):.6f}")
    p = tmp_path / "v.obj"
    with open(p, "w") as f:
        for i in range(0, len(toks) - 2, 3):
            f.write(f"v {toks[i]} {toks[i + 1]} {toks[i + 2]}\n")
        n = (len(toks) - 2) // 3 if (len(toks) - 2) % 3 else (len(toks) - 2) // 3
        for i in range(1, n - 1, 3):
            f.write(f"f {i} {i + 1} {i + 2}\n")
    s = R.Scene()
    s.load_obj(str(p))
    pos, _, _, _ = s.arrays()
    vals = pos.reshape(-1, 3)
    k = 0
    differs = 0
    for i in range(1, n - 1, 3):
        for c in range(3):
            toks3 = toks[(i - 1 + c) * 3:(i - 1 + c) * 3 + 3]
            exp = np.array([fast_atof(t) for t in toks3], np.float32)
            assert np.array_equal(vals[k], exp), (toks3, vals[k], exp)
            differs += int(np.any(exp != np.array([np.float32(t) for t in toks3])))
            k += 1
    assert differs > 0  # the emulation matters


def test_normalize_centres_and_scales(R):
    # centerAndScaleToUnitMesh (src/mesh.cpp:164-188) over Assimp's per-corner vertex list:
    # sequential float accumulation, / float(count), maxD = max glm::length(p - c), p' = (p - c) / maxD
    path = os.path.join(R.data_dir(), "monkey-rotated.obj")
    lines = open(path).read().splitlines()
    verts = [np.array([fast_atof(t) for t in l.split()[1:4]], np.float32) for l in lines if l.startswith("v ")]
    faces = [[int(c.split("/")[0]) - 1 for c in l.split()[1:]] for l in lines if l.startswith("f ")]
    corners = [verts[i] for f in faces for i in f]
    acc = np.zeros(3, np.float32)
    for p in corners:
        acc = (acc + p).astype(np.float32)
    center = (acc / np.float32(len(corners))).astype(np.float32)

    def glm_length(v):
        return np.sqrt(np.float32(np.float32(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]))

    maxd = np.float32(0)
    for p in corners:
        d = glm_length((p - center).astype(np.float32))
        maxd = maxd if d < maxd else d
    pos, _, _, _ = load(R, "monkey-rotated.obj", normalize=True).arrays()
    f0 = faces[0]  # quad -> first triangle (0,1,2)
    expect = np.array([((verts[f0[k]] - center) / maxd).astype(np.float32) for k in (0, 1, 2)])
    assert np.array_equal(pos[0], expect)
    v = pos.reshape(-1, 3).astype(np.float64)
    assert abs(np.sqrt((v ** 2).sum(1)).max() - 1.0) < 1e-6


def test_generated_normals_for_obj_without_vn(R):
    # teapot.obj has no 'vn': GenFaceNormals after Triangulate -> unit per-triangle normals
    pos, nrm, _, _ = load(R, "teapot.obj").arrays()
    n = nrm.astype(np.float64)
    ln = np.sqrt((n ** 2).sum(2))
    ok = ln > 0
    assert np.all(np.abs(ln[ok] - 1) < 1e-5)
    face = np.cross(pos[:, 1] - pos[:, 0], pos[:, 2] - pos[:, 0]).astype(np.float64)
    face /= np.maximum(np.linalg.norm(face, axis=1, keepdims=True), 1e-30)
    # corners shared by the two triangles of a quad carry the last triangle's normal; the third
    # corner of the last triangle of each face always carries its own
    dots = (nrm[:, 2] * face).sum(1)
    assert np.mean(dots > 0.99) > 0.45


def test_shininess_switch(R):
    _, _, _, m5 = load(R, "monkey-rotated.obj").arrays()
    _, _, _, m3 = load(R, "monkey-rotated.obj", x4=True).arrays()
    assert m5[0].shininess == 225.0
    assert m3[0].shininess == 900.0


def test_presets(R):
    dd = R.data_dir()
    s = R.Scene().preset(R.PRESETS["SingleTriangle"], dd)
    pos, _, _, mats = s.arrays()
    assert len(pos) == 2 and list(mats[0].kd) == [1.0, 1.0, 1.0]  # subMeshes[0].material.kd = 1
    d = s.desc()
    assert d.num_point_lights == 1 and d.num_spherical_lights == 1
    s = R.Scene().preset(R.PRESETS["CornellBox"], dd)
    d = s.desc()
    assert d.num_spheres == 1 and d.spheres[0].material.transparency == 0.0
    s = R.Scene().preset(R.PRESETS["Cube"], dd)
    d = s.desc()
    assert d.num_spot_lights == 1 and d.spot_lights[0].angle == 10.0
    s = R.Scene().preset(R.PRESETS["Spheres"], dd)
    assert s.desc().num_spheres == 3
    with pytest.raises(R.RtError):
        R.Scene().preset(R.PRESETS["Dragon"], dd)  # data/dragon.obj is missing in the reference too


def test_dragon_proxy_deterministic(R, tmp_path):
    a, b = str(tmp_path / "a.obj"), str(tmp_path / "b.obj")
    R.check(R.lib().rt_write_dragon_proxy(a.encode(), 40, 16))
    R.check(R.lib().rt_write_dragon_proxy(b.encode(), 40, 16))
    assert open(a).read().replace("a.mtl", "") == open(b).read().replace("b.mtl", "")
    s = R.Scene()
    s.load_obj(a, normalize=True)
    pos, nrm, _, mats = s.arrays()
    assert len(pos) == 2 * 40 * 16
    assert mats[0].shininess == 0.0 and list(mats[0].ks) == [0.5, 0.5, 0.5]


@pytest.mark.parametrize("name,normalize", [("cube.obj", False), ("monkey-rotated.obj", True),
                                            ("CornellBox-Mirror-Rotated.obj", True), ("tr_def.obj", False)])
def test_mesh_view_matches_flat_scene(R, name, normalize):
    """rt_scene_mesh_get (the facade's loadMesh data model: vertices + index triplets per mesh) flattens
    mesh-major to exactly the scene-order triangles rt_create receives (loadObjectsFromScene,
    src/bounding_volume_hierarchy.cpp:80-99)."""
    s = R.Scene().load_obj(os.path.join(R.data_dir(), name), normalize=normalize)
    pos, nrm, mesh, mats = s.arrays()
    flat_p, flat_n, flat_m = [], [], []
    for mi, (vert, tri, mat, _) in enumerate(s.meshes()):
        assert mat.kd[:] == mats[mi].kd[:] and mat.shininess == mats[mi].shininess
        flat_p.append(vert[tri][:, :, 0:3])
        flat_n.append(vert[tri][:, :, 3:6])
        flat_m.append(np.full(len(tri), mi))
    assert np.concatenate(flat_p).astype(np.float32).tobytes() == pos.tobytes()
    assert np.concatenate(flat_n).astype(np.float32).tobytes() == nrm.tobytes()
    assert np.array_equal(np.concatenate(flat_m), mesh)
