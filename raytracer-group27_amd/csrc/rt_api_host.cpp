// rt_api_host.cpp -- host half of the C-ABI: errors, scene ingest, camera.
//   rt_scene_load_obj  <- loadMesh (src/mesh.cpp:58-188)
//   rt_scene_preset    <- loadScene (src/scene.cpp:4-150)
//   rt_camera_from_trackball <- Trackball::position / generateRay constants (framework/src/trackball.cpp:65-98)
#include <cmath>
#include <cstring>
#include <exception>
#include <string>

#include "../../include/rt_amd.h"
#include "host_scene.h"
#include "rt_internal.h"

struct rt_scene {
    rt::HostScene s;
    bool dirty = true;
    std::vector<std::vector<float>> mesh_vertices;  // rt_scene_mesh_get views ([n][8] per mesh)
};

namespace rt {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace rt

using namespace rt;

#define CATCH_ALL(ret)                           \
    catch (const std::exception& e) {            \
        set_error(e.what());                     \
        return ret;                              \
    }                                            \
    catch (...) {                                \
        set_error("unknown C++ exception");      \
        return ret;                              \
    }

extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

extern "C" int rt_last_error(char* buf, size_t len) {
    if (!buf || len == 0) return (int)g_err.size();
    std::strncpy(buf, g_err.c_str(), len - 1);
    buf[len - 1] = 0;
    return (int)g_err.size();
}

extern "C" int rt_scene_new(rt_scene** out) {
    if (!out) return RT_ERR_INVALID;
    *out = new rt_scene();
    return RT_OK;
}

extern "C" int rt_scene_free(rt_scene* s) {
    delete s;
    return RT_OK;
}

extern "C" int rt_scene_load_obj(rt_scene* sc, const char* path, int normalize, int x4) {
    if (!sc || !path) {
        set_error("rt_scene_load_obj: null argument");
        return RT_ERR_INVALID;
    }
    try {
        auto meshes = load_obj(path, normalize != 0, x4);
        for (auto& m : meshes) sc->s.meshes.push_back(std::move(m));
        sc->dirty = true;
        sc->s.load_textures();
        return RT_OK;
    }
    CATCH_ALL(RT_ERR_IO)
}

extern "C" int rt_scene_preset(rt_scene* sc, int preset, const char* data_dir, int x4) {
    if (!sc || !data_dir) {
        set_error("rt_scene_preset: null argument");
        return RT_ERR_INVALID;
    }
    try {
        load_preset(sc->s, preset, data_dir, x4);
        sc->dirty = true;
        sc->s.load_textures();
        return RT_OK;
    }
    CATCH_ALL(RT_ERR_IO)
}

extern "C" int rt_scene_add_sphere(rt_scene* sc, const rt_sphere* s) {
    if (!sc || !s) return RT_ERR_INVALID;
    sc->s.spheres.push_back(*s);
    return RT_OK;
}
extern "C" int rt_scene_add_point_light(rt_scene* sc, const rt_point_light* l) {
    if (!sc || !l) return RT_ERR_INVALID;
    sc->s.point_lights.push_back(*l);
    return RT_OK;
}
extern "C" int rt_scene_add_spherical_light(rt_scene* sc, const rt_spherical_light* l) {
    if (!sc || !l) return RT_ERR_INVALID;
    sc->s.spherical_lights.push_back(*l);
    return RT_OK;
}
extern "C" int rt_scene_add_spot_light(rt_scene* sc, const rt_spot_light* l) {
    if (!sc || !l) return RT_ERR_INVALID;
    sc->s.spot_lights.push_back(*l);
    return RT_OK;
}
extern "C" int rt_scene_add_plane_light(rt_scene* sc, const rt_plane_light* l) {
    if (!sc || !l) return RT_ERR_INVALID;
    sc->s.plane_lights.push_back(*l);
    return RT_OK;
}
extern "C" int rt_scene_clear_lights(rt_scene* sc) {
    if (!sc) return RT_ERR_INVALID;
    sc->s.point_lights.clear();
    sc->s.spherical_lights.clear();
    sc->s.spot_lights.clear();
    sc->s.plane_lights.clear();
    return RT_OK;
}
extern "C" int rt_scene_set_material(rt_scene* sc, int mesh, const rt_material* m) {
    if (!sc || !m || mesh < 0 || mesh >= (int)sc->s.meshes.size()) {
        set_error("rt_scene_set_material: invalid argument");
        return RT_ERR_INVALID;
    }
    Material& d = sc->s.meshes[mesh].material;
    d.kd = v3{m->kd[0], m->kd[1], m->kd[2]};
    d.ks = v3{m->ks[0], m->ks[1], m->ks[2]};
    d.shininess = m->shininess;
    d.transparency = m->transparency;
    d.has_texture = m->has_texture != 0;
    d.texture = m->has_texture ? m->texture : -1;
    sc->dirty = true;
    return RT_OK;
}

extern "C" int rt_scene_mesh_count(const rt_scene* sc, int* n) {
    if (!sc || !n) return RT_ERR_INVALID;
    *n = (int)sc->s.meshes.size();
    return RT_OK;
}

extern "C" int rt_scene_mesh_get(const rt_scene* csc, int mesh, rt_mesh_view* out) {
    if (!csc || !out || mesh < 0 || mesh >= (int)csc->s.meshes.size()) {
        set_error("rt_scene_mesh_get: invalid argument");
        return RT_ERR_INVALID;
    }
    rt_scene* sc = const_cast<rt_scene*>(csc);
    if (sc->mesh_vertices.size() != sc->s.meshes.size()) sc->mesh_vertices.assign(sc->s.meshes.size(), {});
    const Mesh& m = sc->s.meshes[mesh];
    std::vector<float>& v = sc->mesh_vertices[mesh];
    v.resize(m.vertices.size() * 8);
    for (size_t i = 0; i < m.vertices.size(); ++i) {
        const Vertex& x = m.vertices[i];
        const float f[8] = {x.p.x, x.p.y, x.p.z, x.n.x, x.n.y, x.n.z, x.uv.x, x.uv.y};
        std::memcpy(&v[i * 8], f, sizeof(f));
    }
    out->num_vertices = (int)m.vertices.size();
    out->num_triangles = (int)m.triangles.size();
    out->vertices = v.data();
    out->triangles = m.triangles.empty() ? nullptr : m.triangles[0].data();
    rt_material& r = out->material;
    r = rt_material{};
    r.kd[0] = m.material.kd.x;
    r.kd[1] = m.material.kd.y;
    r.kd[2] = m.material.kd.z;
    r.ks[0] = m.material.ks.x;
    r.ks[1] = m.material.ks.y;
    r.ks[2] = m.material.ks.z;
    r.shininess = m.material.shininess;
    r.transparency = m.material.transparency;
    r.has_texture = m.material.has_texture ? 1 : 0;
    r.texture = m.material.texture;
    out->texture_path = m.material.texture_path.c_str();
    return RT_OK;
}

extern "C" int rt_scene_desc_get(const rt_scene* csc, rt_scene_desc* out) {
    if (!csc || !out) return RT_ERR_INVALID;
    rt_scene* sc = const_cast<rt_scene*>(csc);
    if (sc->dirty) {
        sc->s.flatten();
        sc->dirty = false;
    }
    sc->s.fill_desc(out);
    return RT_OK;
}

extern "C" int rt_write_dragon_proxy(const char* path, int u, int v) {
    if (!path) return RT_ERR_INVALID;
    try {
        write_dragon_proxy(path, u, v);
        return RT_OK;
    }
    CATCH_ALL(RT_ERR_IO)
}

// Trackball (framework/src/trackball.cpp): glm::quat(euler) (c = cos(e*0.5), s = sin(e*0.5)),
// position() = lookAt + quat * vec3(0,0,-dist), halfScreenPlaceHeight = tan(fovy/2).
extern "C" int rt_camera_from_trackball(const float look_at[3], const float e[3], float dist, float fovy, float aspect,
                                        rt_camera* out) {
    if (!look_at || !e || !out) return RT_ERR_INVALID;
    const float cx = std::cos(e[0] * 0.5f), cy = std::cos(e[1] * 0.5f), cz = std::cos(e[2] * 0.5f);
    const float sx = std::sin(e[0] * 0.5f), sy = std::sin(e[1] * 0.5f), sz = std::sin(e[2] * 0.5f);
    const float w = cx * cy * cz + sx * sy * sz;
    const float x = sx * cy * cz - cx * sy * sz;
    const float y = cx * sy * cz + sx * cy * sz;
    const float z = cx * cy * sz - sx * sy * cz;
    const v3 off = quat_rotate(x, y, z, w, v3{0.0f, 0.0f, -dist});
    const v3 pos = v3{look_at[0], look_at[1], look_at[2]} + off;
    out->position[0] = pos.x;
    out->position[1] = pos.y;
    out->position[2] = pos.z;
    out->quat[0] = x;
    out->quat[1] = y;
    out->quat[2] = z;
    out->quat[3] = w;
    out->half_height = std::tan(fovy / 2.0f);
    out->half_width = aspect * out->half_height;
    return RT_OK;
}
