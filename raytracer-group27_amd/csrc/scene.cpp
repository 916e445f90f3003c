// scene.cpp -- loadScene presets (reference src/scene.cpp:4-150), the flat scene-order view
// (BoundingVolumeHierarchy::loadObjectsFromScene, src/bounding_volume_hierarchy.cpp:80-99) and the
// deterministic dragon stand-in (data/dragon.obj is absent: .MISSING_LARGE_BLOBS:1).
#include <iterator>
#include <fstream>
#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "host_scene.h"

namespace rt {

void HostScene::flatten() {
    size_t ntri = 0;
    for (const Mesh& m : meshes) ntri += m.triangles.size();
    flat_pos.assign(ntri * 9, 0.0f);
    flat_nrm.assign(ntri * 9, 0.0f);
    flat_uv.assign(ntri * 6, 0.0f);
    flat_mesh.assign(ntri, 0);
    flat_mat.clear();
    size_t t = 0;
    for (size_t mi = 0; mi < meshes.size(); ++mi) {
        const Mesh& m = meshes[mi];
        for (const auto& tri : m.triangles) {
            for (int c = 0; c < 3; ++c) {
                const Vertex& v = m.vertices.at(tri[c]);
                flat_pos[t * 9 + c * 3 + 0] = v.p.x;
                flat_pos[t * 9 + c * 3 + 1] = v.p.y;
                flat_pos[t * 9 + c * 3 + 2] = v.p.z;
                flat_nrm[t * 9 + c * 3 + 0] = v.n.x;
                flat_nrm[t * 9 + c * 3 + 1] = v.n.y;
                flat_nrm[t * 9 + c * 3 + 2] = v.n.z;
                flat_uv[t * 6 + c * 2 + 0] = v.uv.x;
                flat_uv[t * 6 + c * 2 + 1] = v.uv.y;
            }
            flat_mesh[t] = (int)mi;
            ++t;
        }
        rt_material rm{};
        rm.kd[0] = m.material.kd.x;
        rm.kd[1] = m.material.kd.y;
        rm.kd[2] = m.material.kd.z;
        rm.ks[0] = m.material.ks.x;
        rm.ks[1] = m.material.ks.y;
        rm.ks[2] = m.material.ks.z;
        rm.shininess = m.material.shininess;
        rm.transparency = m.material.transparency;
        rm.has_texture = m.material.has_texture ? 1 : 0;
        rm.texture = m.material.texture;
        flat_mat.push_back(rm);
    }
    flat_tex.clear();
    for (const HostTexture& t : textures) {
        rt_texture rt{};
        rt.width = t.width;
        rt.height = t.height;
        rt.channels = t.channels;
        rt.rgb = t.rgb.data();
        flat_tex.push_back(rt);
    }
}

void HostScene::load_textures() {
    for (Mesh& m : meshes) {
        Material& mat = m.material;
        if (!mat.has_texture || mat.texture >= 0 || mat.texture_path.empty()) continue;
        for (size_t i = 0; i < textures.size(); ++i)
            if (textures[i].path == mat.texture_path) mat.texture = (int)i;
        if (mat.texture >= 0) continue;
        std::ifstream f(mat.texture_path, std::ios::binary);
        if (!f) throw std::runtime_error("Texture file " + mat.texture_path + " does not exists!");
        std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        HostTexture t;
        t.path = mat.texture_path;
        if (rt_decode_png(bytes.data(), (long)bytes.size(), &t.width, &t.height, &t.channels, nullptr, 0) != RT_OK)
            throw std::runtime_error("Failed to read texture " + mat.texture_path + " (PNG only)");
        if (t.channels < 3)
            throw std::runtime_error("Only textures with 3 or more color channels are supported. " + mat.texture_path +
                                     " has " + std::to_string(t.channels) + " channels");
        t.rgb.resize((size_t)t.width * t.height * 3);
        if (rt_decode_png(bytes.data(), (long)bytes.size(), &t.width, &t.height, &t.channels, t.rgb.data(),
                          (long)t.rgb.size()) != RT_OK)
            throw std::runtime_error("Failed to read texture " + mat.texture_path);
        mat.texture = (int)textures.size();
        textures.push_back(std::move(t));
    }
}

void HostScene::fill_desc(rt_scene_desc* d) const {
    d->num_triangles = (int)flat_mesh.size();
    d->positions = flat_pos.empty() ? nullptr : flat_pos.data();
    d->normals = flat_nrm.empty() ? nullptr : flat_nrm.data();
    d->texcoords = flat_uv.empty() ? nullptr : flat_uv.data();
    d->mesh_index = flat_mesh.empty() ? nullptr : flat_mesh.data();
    d->num_meshes = (int)flat_mat.size();
    d->materials = flat_mat.empty() ? nullptr : flat_mat.data();
    d->num_spheres = (int)spheres.size();
    d->spheres = spheres.empty() ? nullptr : spheres.data();
    d->num_point_lights = (int)point_lights.size();
    d->point_lights = point_lights.empty() ? nullptr : point_lights.data();
    d->num_spherical_lights = (int)spherical_lights.size();
    d->spherical_lights = spherical_lights.empty() ? nullptr : spherical_lights.data();
    d->num_spot_lights = (int)spot_lights.size();
    d->spot_lights = spot_lights.empty() ? nullptr : spot_lights.data();
    d->num_plane_lights = (int)plane_lights.size();
    d->plane_lights = plane_lights.empty() ? nullptr : plane_lights.data();
    d->num_textures = (int)flat_tex.size();
    d->textures = flat_tex.empty() ? nullptr : flat_tex.data();
}

static void add_meshes(HostScene& s, std::vector<Mesh>&& sub) {
    for (auto& m : sub) s.meshes.push_back(std::move(m));
}

static rt_point_light pl(float x, float y, float z, float c) {
    return rt_point_light{{x, y, z}, {c, c, c}};
}

static rt_material mat(float kdr, float kdg, float kdb, float ksr, float ksg, float ksb, float shin,
                       float transp) {
    rt_material m{};
    m.kd[0] = kdr;
    m.kd[1] = kdg;
    m.kd[2] = kdb;
    m.ks[0] = ksr;
    m.ks[1] = ksg;
    m.ks[2] = ksb;
    m.shininess = shin;
    m.transparency = transp;
    return m;
}

// SceneType enum order, src/scene.h:14-34
enum Preset {
    SingleTriangle = 0,
    Bookeshelf,
    Cube,
    CornellBox,
    CornellBoxSphericalLight,
    CornellBoxPlaneLight,
    Monkey,
    Teapot,
    Dragon,
    Spheres,
    ChessBoard,
    Custom,
    AndreasScene,
    CatalinScene,
    MikeScene,
    MikeScene2
};

void load_preset(HostScene& scene, int preset, const std::string& data_dir, int x4) {
    const std::string d = data_dir.empty() || data_dir.back() == '/' ? data_dir : data_dir + "/";
    switch (preset) {
        case SingleTriangle: {  // src/scene.cpp:9-18
            auto sub = load_obj(d + "tr_def.obj", false, x4);
            sub.at(0).material.kd = splat(1.0f);
            add_meshes(scene, std::move(sub));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
            scene.spherical_lights.push_back(rt_spherical_light{{-2.1f, 1.24f, -0.51f}, 0.5f, {1.0f, 0.0f, 1.0f}});
        } break;
        case Cube: {  // :19-27
            add_meshes(scene, load_obj(d + "cube.obj", false, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
            scene.spot_lights.push_back(rt_spot_light{{(float)-1.2, -1, -1}, {1, (float)1.2, 1}, 10, {1, 1, 1}});
        } break;
        case CornellBox: {  // :28-35
            add_meshes(scene, load_obj(d + "CornellBox-Mirror-Rotated.obj", true, x4));
            scene.spheres.push_back(rt_sphere{{-0.2f, 0.15f, -0.25f}, 0.2f, mat(0, 0, 0, 0, 0, 0, 1, 0)});
            scene.point_lights.push_back(pl(0, 0.58f, 0, 1));
        } break;
        case CornellBoxSphericalLight: {  // :36-43
            add_meshes(scene, load_obj(d + "CornellBox-Mirror-Rotated.obj", true, x4));
            scene.spheres.push_back(rt_sphere{{-0.2f, 0.15f, -0.25f}, 0.2f, mat(0, 0, 0, 0, 0, 0, 1, 0)});
            scene.spherical_lights.push_back(rt_spherical_light{{0, 0.45f, 0}, 0.1f, {1, 1, 1}});
        } break;
        case CornellBoxPlaneLight: {  // :44-50
            add_meshes(scene, load_obj(d + "CornellBox-Mirror-Rotated.obj", true, x4));
            scene.plane_lights.push_back(rt_plane_light{
                {-0.1f, 0.63f, -0.1f}, {(float)0.15, (float)-0.05, 0}, {0, 0, (float)0.2}, {1, 1, 1}});
        } break;
        case Monkey: {  // :51-58
            add_meshes(scene, load_obj(d + "monkey-rotated.obj", true, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
            scene.point_lights.push_back(pl(1, -1, -1, 1));
        } break;
        case Teapot: {  // :59-66
            add_meshes(scene, load_obj(d + "teapot.obj", true, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
        } break;
        case Dragon: {  // :67-74
            add_meshes(scene, load_obj(d + "dragon.obj", true, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
        } break;
        case Spheres: {  // :80-87
            scene.spheres.push_back(rt_sphere{{3.0f, -2.0f, 10.2f}, 1.0f, mat(0.8f, 0.2f, 0.2f, 0, 0, 0, 1, 1)});
            scene.spheres.push_back(rt_sphere{{-2.0f, 2.0f, 4.0f}, 2.0f, mat(0.6f, 0.8f, 0.2f, 0, 0, 0, 1, 1)});
            scene.spheres.push_back(rt_sphere{{0.0f, 0.0f, 6.0f}, 0.75f, mat(0.2f, 0.2f, 0.8f, 0, 0, 0, 1, 1)});
            scene.point_lights.push_back(pl(3, 0, 3, 15));
        } break;
        case Custom: {  // :88-98
            add_meshes(scene, load_obj(d + "custom.obj", false, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
        } break;
        case ChessBoard: {  // :99-116
            auto sub = load_obj(d + "checker.obj", false, x4);
            sub.at(0).material.kd = splat(1.0f);
            add_meshes(scene, std::move(sub));
            scene.spherical_lights.push_back(rt_spherical_light{{-1, 100, -25}, 10, {1, 1, 1}});
        } break;
        case AndreasScene:
            add_meshes(scene, load_obj(d + "AndreasScene.obj", true, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
            break;
        case CatalinScene:
            add_meshes(scene, load_obj(d + "CatalinScene.obj", true, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
            break;
        case MikeScene:
            add_meshes(scene, load_obj(d + "MikeScene.obj", true, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
            break;
        case MikeScene2:
            add_meshes(scene, load_obj(d + "MikeScene2.obj", true, x4));
            scene.point_lights.push_back(pl(-2, 1, -2, 1));
            break;
        case Bookeshelf:
            add_meshes(scene, load_obj(d + "bookshelf.obj", true, x4));
            scene.point_lights.push_back(pl(-1, 1, -1, 1));
            break;
        default:
            throw std::runtime_error("unknown scene preset");
    }
}

// (2,3) torus-knot tube, u_segments x v_segments quads -> 2*u*v triangles, analytic normals,
// "%.6f" text like a Blender export.  Material: Kd .8 .6 .3, Ks .5, Ns 0, d 1 (perfect mirror,
// deterministic, immune to the Ns scaling question -- SURVEY.md §8d C3).
void write_dragon_proxy(const std::string& obj_path, int U, int V) {
    if (U < 3 || V < 3) throw std::runtime_error("dragon proxy needs at least 3x3 segments");
    const std::string mtl_path = obj_path.substr(0, obj_path.find_last_of('.')) + ".mtl";
    const std::string mtl_name = mtl_path.substr(mtl_path.find_last_of("/\\") + 1);
    FILE* fm = std::fopen(mtl_path.c_str(), "w");
    if (!fm) throw std::runtime_error("cannot write " + mtl_path);
    std::fprintf(fm, "newmtl dragon_proxy\nNs 0.000000\nKd 0.800000 0.600000 0.300000\nKs 0.500000 0.500000 0.500000\nd 1.000000\nillum 3\n");
    std::fclose(fm);
    FILE* f = std::fopen(obj_path.c_str(), "w");
    if (!f) throw std::runtime_error("cannot write " + obj_path);
    std::fprintf(f, "# dragon proxy: (2,3) torus knot tube %d x %d quads\nmtllib %s\no DragonProxy\n", U, V,
                 mtl_name.c_str());
    const double R = 0.42;  // tube radius
    const double two_pi = 6.283185307179586;
    for (int i = 0; i < U; ++i) {
        const double u = two_pi * i / U;
        // centre curve c(u) = ((2+cos3u)cos2u, (2+cos3u)sin2u, sin3u)
        const double cx = (2 + std::cos(3 * u)) * std::cos(2 * u), cy = (2 + std::cos(3 * u)) * std::sin(2 * u),
                     cz = std::sin(3 * u);
        double tx = -3 * std::sin(3 * u) * std::cos(2 * u) - 2 * (2 + std::cos(3 * u)) * std::sin(2 * u);
        double ty = -3 * std::sin(3 * u) * std::sin(2 * u) + 2 * (2 + std::cos(3 * u)) * std::cos(2 * u);
        double tz = 3 * std::cos(3 * u);
        const double tl = std::sqrt(tx * tx + ty * ty + tz * tz);
        tx /= tl;
        ty /= tl;
        tz /= tl;
        // N = normalize(T x z), B = N x T  (T is never parallel to z: |T_xy| >= 2)
        double nx = ty, ny = -tx, nz = 0.0;
        const double nl = std::sqrt(nx * nx + ny * ny);
        nx /= nl;
        ny /= nl;
        const double bx = ny * tz - nz * ty, by = nz * tx - nx * tz, bz = nx * ty - ny * tx;
        for (int j = 0; j < V; ++j) {
            const double v = two_pi * j / V;
            const double ox = std::cos(v) * nx + std::sin(v) * bx, oy = std::cos(v) * ny + std::sin(v) * by,
                         oz = std::cos(v) * nz + std::sin(v) * bz;
            std::fprintf(f, "v %.6f %.6f %.6f\n", cx + R * ox, cy + R * oy, cz + R * oz);
            std::fprintf(f, "vn %.4f %.4f %.4f\n", ox, oy, oz);
        }
    }
    std::fprintf(f, "usemtl dragon_proxy\ns 1\n");
    for (int i = 0; i < U; ++i) {
        const int i1 = (i + 1) % U;
        for (int j = 0; j < V; ++j) {
            const int j1 = (j + 1) % V;
            const int a = i * V + j + 1, b = i1 * V + j + 1, c = i1 * V + j1 + 1, e = i * V + j1 + 1;
            std::fprintf(f, "f %d//%d %d//%d %d//%d %d//%d\n", a, a, b, b, c, c, e, e);
        }
    }
    std::fclose(f);
}

}  // namespace rt
