// rt_facade.hpp -- C++ facade over the C-ABI with the reference's data model and signatures, so the
// reference's main.cpp render path switches to the MI355X implementation by swapping includes
// (glm::vec3 -> rt::facade::vec3; the GUI, GL and ImGui code stay out of scope).
//
//   reference                                                  facade (namespace rt::facade)
//   struct Vertex / Material / Mesh, Triangle (src/mesh.h:14-44) Vertex / Material / Mesh, Triangle
//   std::vector<Mesh> loadMesh(path, bool normalize) (:46)      loadMesh
//   struct Sphere / PointLight / SphericalLight / SpotLight /    the same structs, same fields and
//     PlaneLight / Scene (src/scene.h:48-94)                      defaults; Scene has the public vectors
//   Scene loadScene(SceneType, dataDir) (src/scene.h:97)        loadScene
//   struct Ray (framework/include/ray.h:11-29)                   Ray (origin, direction, t)
//   struct HitInfo + getMaterial (src/ray_tracing.h:6-35)        HitInfo (+ prim_id)
//   class BoundingVolumeHierarchy (src/bounding_volume_hierarchy.h:22-81)
//     BoundingVolumeHierarchy(Scene*), intersect(Ray&, HitInfo&, bool useBVH) const, numLevels()
//   class Trackball (framework/include/trackball.h:14-54)        Trackball (setCamera, position,
//                                                                 lookAt, generateRay)
//   getFinalColor(Scene&, const BVH&, Ray, int level = 0)        getFinalColor (src/main.cpp:129)
//   renderRayTracing(Scene&, const Trackball&, const BVH&, Screen&, bool textureDebugging,
//                    bool anti_aliasing, bool multipleRays, int sampleSize)  (src/main.cpp:340-341)
//   class Screen (src/screen.h:32-161)                           Screen (setPixel, postprocessImage,
//                                                                 writeBitmapToFile, bloom setters)
//   render knobs (src/main.cpp:54-64, 123-127)                   the same global names, inline
//
// Scene edits after the BVH exists -- the ImGui light editors (src/main.cpp:511-613) and material
// edits -- are picked up like the reference picks them up (it reads scene.* on every call):
// getFinalColor / renderRayTracing compare the Scene's lights and materials with what the device
// holds and push changes (rt_update_lights / rt_update_materials).  Geometry edits need a new
// BoundingVolumeHierarchy, as in the reference (its BVH is built once in the constructor).
//
// Errors: loadMesh / loadScene throw std::runtime_error like the reference's loadMesh
// (src/mesh.cpp:60-73); intersect() never throws and returns false on a miss.  A device error (no
// GPU) throws from the BoundingVolumeHierarchy constructor -- there is no CPU fallback.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_amd.h"

namespace rt {
namespace facade {

// ---- vector types (glm 0.9.9.8 operation order where the render path computes on the host) ----
struct vec3 {
    float x = 0, y = 0, z = 0;
    vec3() = default;
    constexpr vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    constexpr explicit vec3(float s) : x(s), y(s), z(s) {}
    bool operator==(const vec3& o) const { return x == o.x && y == o.y && z == o.z; }
    bool operator!=(const vec3& o) const { return !(*this == o); }
};
inline vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline float dot(vec3 a, vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline vec3 cross(vec3 a, vec3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
inline vec3 normalize(vec3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
struct vec2 {
    float x = 0, y = 0;
};
struct uvec3 {
    uint32_t x = 0, y = 0, z = 0;
    uint32_t operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline float radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }
inline vec3 radians(vec3 d) { return {radians(d.x), radians(d.y), radians(d.z)}; }

inline std::string last_error() {
    char buf[1024];
    rt_last_error(buf, sizeof(buf));
    return buf;
}
inline void check(int rc, const char* what) {
    if (rc != RT_OK) throw std::runtime_error(std::string(what) + ": " + last_error());
}

// ---- render knobs: the reference's globals (src/main.cpp:54-64, 123-127), same names/defaults ----
enum class TextureFiltering {
    NearestNeighbor = RT_TEX_NEAREST,
    Bilinear = RT_TEX_BILINEAR,
    MipMappingNearestLevelNearestNeighbor = RT_TEX_MIP_NEAREST,
    MipMappingNearestLevelBilinear = RT_TEX_MIP_NEAREST_BILINEAR,
    Trilinear = RT_TEX_TRILINEAR
};
enum class OutOfBoundsRule { Border = RT_OOB_BORDER, Clamp = RT_OOB_CLAMP, Repeat = RT_OOB_REPEAT };
inline TextureFiltering textureFiltering{TextureFiltering::NearestNeighbor};
inline OutOfBoundsRule outOfBoundsRuleX{OutOfBoundsRule::Border};
inline OutOfBoundsRule outOfBoundsRuleY{OutOfBoundsRule::Border};
inline vec3 textureBorderColor{0.0f};
inline bool useTextures = false;
inline bool useBVH = false;
inline int max_reflection_level = 5;
inline int sphere_light_ray_count = 10;
inline int plane_light_1D_ray_count = 3;
inline int glossy_ray_count = 10;  // > 1 draws the glossy lobe from a Philox stream in place of rand()
inline float refraction_factor = 0.8f;
inline uint64_t glossy_seed = 0x5EED;  // the Philox key that replaces rand()'s state

inline rt_params current_params(int shade_level = 0) {
    rt_params p{};
    p.max_reflection_level = max_reflection_level;
    p.sphere_light_ray_count = sphere_light_ray_count;
    p.plane_light_1D_ray_count = plane_light_1D_ray_count;
    p.glossy_ray_count = glossy_ray_count;
    p.refraction_factor = refraction_factor;
    p.use_bvh = useBVH ? 1 : 0;
    p.sample_size = 4;
    p.rng_seed = glossy_seed;
    p.use_textures = useTextures ? 1 : 0;
    p.texture_filtering = (int)textureFiltering;
    p.out_of_bounds_x = (int)outOfBoundsRuleX;
    p.out_of_bounds_y = (int)outOfBoundsRuleY;
    p.border_color[0] = textureBorderColor.x;
    p.border_color[1] = textureBorderColor.y;
    p.border_color[2] = textureBorderColor.z;
    p.shade_level = shade_level;
    return p;
}

// ---- data model (src/mesh.h, src/scene.h) ----
// Image: the decoded kd texture as stbi_load(path, ..., STBI_rgb) returns it (src/image.cpp:37-73);
// getPixel runs on the device.
struct Image {
    std::string path;
    int width = 0, height = 0, channels = 0;
    std::vector<uint8_t> rgb;  // width * height * 3
};

struct Vertex {
    vec3 p;  // Position.
    vec3 n;  // Normal.
    vec2 texCoord;
};

struct Material {
    vec3 kd;  // Diffuse color.
    vec3 ks{0.0f};
    float shininess{1.0f};
    float transparency{1.0f};
    std::optional<Image> kdTexture;
};

using Triangle = uvec3;

struct Mesh {
    std::vector<Vertex> vertices;
    std::vector<Triangle> triangles;
    Material material;
};

struct Sphere {
    vec3 center{0.0f};
    float radius = 1.0f;
    Material material;
};
struct PointLight {
    vec3 position;
    vec3 color;
};
struct SphericalLight {
    vec3 position;
    float radius;
    vec3 color;
};
struct SpotLight {
    vec3 position;
    vec3 direction;
    float angle;
    vec3 color;
};
struct PlaneLight {
    vec3 position;
    vec3 width;
    vec3 height;
    vec3 color;
    vec3 center() const { return position + 0.5f * (width + height); }
};

struct Scene {
    std::vector<Mesh> meshes;
    std::vector<Sphere> spheres;
    std::vector<PointLight> pointLights;
    std::vector<SphericalLight> sphericalLight;
    std::vector<PlaneLight> planeLight;
    std::vector<SpotLight> spotLight;
};

// SceneType (src/scene.h:14-34)
enum SceneType {
    SingleTriangle, Bookeshelf, Cube, CornellBox, CornellBoxSphericalLight, CornellBoxPlaneLight, Monkey, Teapot,
    Dragon, Spheres, ChessBoard, Custom, AndreasScene, CatalinScene, MikeScene, MikeScene2
};

namespace detail {
inline vec3 v3(const float* p) { return {p[0], p[1], p[2]}; }
inline void put(float* d, vec3 v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
}
struct HostScene {  // RAII over rt_scene
    rt_scene* h = nullptr;
    HostScene() { check(rt_scene_new(&h), "rt_scene_new"); }
    ~HostScene() { rt_scene_free(h); }
    HostScene(const HostScene&) = delete;
    HostScene& operator=(const HostScene&) = delete;
};
inline Material material_of(const rt_material& m) {
    Material r;
    r.kd = v3(m.kd);
    r.ks = v3(m.ks);
    r.shininess = m.shininess;
    r.transparency = m.transparency;
    return r;
}
// the scene's meshes (+ decoded kd textures) as loadMesh returns them
inline std::vector<Mesh> meshes_of(const rt_scene* s) {
    rt_scene_desc d;
    check(rt_scene_desc_get(s, &d), "rt_scene_desc_get");
    int n = 0;
    check(rt_scene_mesh_count(s, &n), "rt_scene_mesh_count");
    std::vector<Mesh> out(n);
    for (int i = 0; i < n; ++i) {
        rt_mesh_view v;
        check(rt_scene_mesh_get(s, i, &v), "rt_scene_mesh_get");
        Mesh& m = out[i];
        m.vertices.resize(v.num_vertices);
        for (int k = 0; k < v.num_vertices; ++k) {
            const float* f = v.vertices + 8 * k;
            m.vertices[k] = Vertex{v3(f), v3(f + 3), vec2{f[6], f[7]}};
        }
        m.triangles.resize(v.num_triangles);
        for (int k = 0; k < v.num_triangles; ++k)
            m.triangles[k] = uvec3{v.triangles[3 * k], v.triangles[3 * k + 1], v.triangles[3 * k + 2]};
        m.material = material_of(v.material);
        if (v.material.has_texture && v.material.texture >= 0 && v.material.texture < d.num_textures) {
            const rt_texture& t = d.textures[v.material.texture];
            Image img;
            img.path = v.texture_path;
            img.width = t.width;
            img.height = t.height;
            img.channels = t.channels;
            img.rgb.assign(t.rgb, t.rgb + (size_t)t.width * t.height * 3);
            m.material.kdTexture = std::move(img);
        }
    }
    return out;
}
inline rt_material c_material(const Material& m, int texture) {
    rt_material r{};
    put(r.kd, m.kd);
    put(r.ks, m.ks);
    r.shininess = m.shininess;
    r.transparency = m.transparency;
    r.has_texture = texture >= 0 ? 1 : 0;
    r.texture = texture;
    return r;
}
}  // namespace detail

// loadMesh (src/mesh.cpp:58-188): Assimp 5.0.1 OBJ/MTL semantics, centerAndScaleToUnitMesh
inline std::vector<Mesh> loadMesh(const std::string& file, bool normalize = false) {
    detail::HostScene s;
    check(rt_scene_load_obj(s.h, file.c_str(), normalize ? 1 : 0, 0), "loadMesh");
    return detail::meshes_of(s.h);
}

// loadScene (src/scene.cpp:4-150)
inline Scene loadScene(SceneType type, const std::string& dataDir) {
    detail::HostScene s;
    check(rt_scene_preset(s.h, (int)type, dataDir.c_str(), 0), "loadScene");
    Scene out;
    out.meshes = detail::meshes_of(s.h);
    rt_scene_desc d;
    check(rt_scene_desc_get(s.h, &d), "rt_scene_desc_get");
    for (int i = 0; i < d.num_spheres; ++i) {
        const rt_sphere& x = d.spheres[i];
        out.spheres.push_back(Sphere{detail::v3(x.center), x.radius, detail::material_of(x.material)});
    }
    for (int i = 0; i < d.num_point_lights; ++i)
        out.pointLights.push_back({detail::v3(d.point_lights[i].position), detail::v3(d.point_lights[i].color)});
    for (int i = 0; i < d.num_spherical_lights; ++i) {
        const rt_spherical_light& l = d.spherical_lights[i];
        out.sphericalLight.push_back({detail::v3(l.position), l.radius, detail::v3(l.color)});
    }
    for (int i = 0; i < d.num_plane_lights; ++i) {
        const rt_plane_light& l = d.plane_lights[i];
        out.planeLight.push_back({detail::v3(l.position), detail::v3(l.width), detail::v3(l.height), detail::v3(l.color)});
    }
    for (int i = 0; i < d.num_spot_lights; ++i) {
        const rt_spot_light& l = d.spot_lights[i];
        out.spotLight.push_back({detail::v3(l.position), detail::v3(l.direction), l.angle, detail::v3(l.color)});
    }
    return out;
}

// ---- rays and hits ----
struct Ray {
    vec3 origin{0.0f};
    vec3 direction{0.0f, 0.0f, -1.0f};
    float t{FLT_MAX};
};

struct HitInfo {
    vec3 normal;
    vec3 hitPoint;
    int material_index = 0;  // the mesh that contains the hit triangle
    Material sphere_material;
    vec2 texCoord;
    bool is_triangle = false;
    int prim_id = -1;  // scene-order triangle index, or num_triangles + sphere index
    Material& getMaterial(Scene& scene) {
        if (is_triangle) return scene.meshes[material_index].material;
        return sphere_material;
    }
    Material getMaterialCopy(Scene& scene) { return getMaterial(scene); }
};

// ---- the acceleration structure = the device context ----
class BoundingVolumeHierarchy {
public:
    // Flattens the scene mesh-major exactly as loadObjectsFromScene does
    // (src/bounding_volume_hierarchy.cpp:80-99) and uploads it once.
    // Every visible GPU by default (renderRayTracing splits the frame's bands over them, as the reference's
    // OpenMP row loop uses every core), or the given device list.
    explicit BoundingVolumeHierarchy(Scene* pScene, std::vector<int> devices = {}) : scene_(pScene) {
        if (devices.empty()) {
            int n = 0;
            check(rt_device_count(&n), "BoundingVolumeHierarchy");
            for (int i = 0; i < n; ++i) devices.push_back(i);
        }
        const Scene& sc = *pScene;
        size_t ntri = 0;
        for (const Mesh& m : sc.meshes) ntri += m.triangles.size();
        std::vector<float> pos(ntri * 9), nrm(ntri * 9), uv(ntri * 6);
        std::vector<int> mesh_of(ntri);
        std::vector<rt_material> mats;
        std::vector<rt_texture> texs;
        std::map<const Image*, int> tex_id;
        size_t t = 0;
        for (size_t mi = 0; mi < sc.meshes.size(); ++mi) {
            const Mesh& m = sc.meshes[mi];
            for (const Triangle& tr : m.triangles) {
                for (int c = 0; c < 3; ++c) {
                    const Vertex& v = m.vertices.at(tr[c]);
                    detail::put(&pos[t * 9 + c * 3], v.p);
                    detail::put(&nrm[t * 9 + c * 3], v.n);
                    uv[t * 6 + c * 2] = v.texCoord.x;
                    uv[t * 6 + c * 2 + 1] = v.texCoord.y;
                }
                mesh_of[t++] = (int)mi;
            }
            int tex = -1;
            if (m.material.kdTexture) {
                const Image& img = *m.material.kdTexture;
                auto it = tex_id.find(&img);
                if (it == tex_id.end()) {
                    tex = (int)texs.size();
                    tex_id[&img] = tex;
                    texs.push_back(rt_texture{img.width, img.height, img.channels, 0, img.rgb.data()});
                } else {
                    tex = it->second;
                }
            }
            mats.push_back(detail::c_material(m.material, tex));
        }
        std::vector<rt_sphere> sph;
        for (const Sphere& s : sc.spheres) {
            rt_sphere x{};
            detail::put(x.center, s.center);
            x.radius = s.radius;
            x.material = detail::c_material(s.material, -1);
            sph.push_back(x);
        }
        rt_scene_desc d{};
        d.num_triangles = (int)ntri;
        d.positions = pos.data();
        d.normals = nrm.data();
        d.texcoords = uv.data();
        d.mesh_index = mesh_of.data();
        d.num_meshes = (int)mats.size();
        d.materials = mats.data();
        d.num_spheres = (int)sph.size();
        d.spheres = sph.data();
        d.num_textures = (int)texs.size();
        d.textures = texs.data();
        lights_of(sc, lights_, d);
        check(rt_create(&d, devices.data(), (int)devices.size(), &ctx_), "BoundingVolumeHierarchy");
        mesh_tex_.clear();
        for (const rt_material& m : mats) mesh_tex_.push_back(m.texture);
        synced_mats_ = mats;
        synced_sph_.clear();
        for (const rt_sphere& s : sph) synced_sph_.push_back(s.material);
    }
    ~BoundingVolumeHierarchy() { rt_destroy(ctx_); }
    BoundingVolumeHierarchy(const BoundingVolumeHierarchy&) = delete;
    BoundingVolumeHierarchy& operator=(const BoundingVolumeHierarchy&) = delete;

    // bool intersect(Ray&, HitInfo&, bool useBVH) const (src/bounding_volume_hierarchy.h:33)
    bool intersect(Ray& ray, HitInfo& hitInfo, bool useBVH_) const {
        rt_ray r{{ray.origin.x, ray.origin.y, ray.origin.z}, {ray.direction.x, ray.direction.y, ray.direction.z}, ray.t};
        rt_hit h{};
        if (rt_intersect(ctx_, &r, 1, useBVH_ ? 1 : 0, &h) != RT_OK) return false;
        if (!h.hit) return false;
        ray.t = h.t;
        hitInfo.normal = detail::v3(h.normal);
        hitInfo.hitPoint = detail::v3(h.hit_point);
        hitInfo.material_index = h.is_triangle ? h.material_index : hitInfo.material_index;
        hitInfo.texCoord = vec2{h.uv[0], h.uv[1]};
        hitInfo.is_triangle = h.is_triangle != 0;
        hitInfo.prim_id = h.prim_id;
        if (!hitInfo.is_triangle && scene_) {
            const int s = h.prim_id - num_triangles();
            if (s >= 0 && s < (int)scene_->spheres.size()) hitInfo.sphere_material = scene_->spheres[s].material;
        }
        return true;
    }
    int numLevels() const {
        int nodes = 0, recs = 0, refn = 0, levels = 0;
        rt_ctx_info(ctx_, &nodes, &recs, &refn, &levels);
        return levels;
    }
    int num_triangles() const {
        int nodes = 0, recs = 0, refn = 0, levels = 0;
        rt_ctx_info(ctx_, &nodes, &recs, &refn, &levels);
        return recs;
    }
    rt_ctx* handle() const { return ctx_; }

    // Push the scene's current lights and materials to the device when they changed (the reference
    // reads scene.pointLights & co. and scene.meshes[i].material on every getFinalColor call).  The
    // comparison walks the scene in place against the last pushed copy -- no allocation, no device call
    // when nothing changed; per-ray loops that edit nothing between frames can sync once per frame and
    // turn the per-call check off with autoSync(false).
    void sync(const Scene& sc) const {
        if (sc.meshes.size() != synced_mats_.size() || sc.spheres.size() != synced_sph_.size())
            throw std::runtime_error("BoundingVolumeHierarchy: the scene's geometry changed; build a new one");
        // the new arrays are built aside and become the pushed copies only once the device has them: a
        // failed update throws and leaves the copies as they were, so the next sync() retries it
        if (lights_changed(sc)) {
            rt_scene_desc d{};
            Lights fresh;
            lights_of(sc, fresh, d);
            check(rt_update_lights(ctx_, &d), "rt_update_lights");
            lights_ = std::move(fresh);
        }
        if (materials_changed(sc)) {
            std::vector<rt_material> mats(sc.meshes.size()), sph(sc.spheres.size());
            for (size_t i = 0; i < sc.meshes.size(); ++i) mats[i] = detail::c_material(sc.meshes[i].material, mesh_tex_[i]);
            for (size_t i = 0; i < sc.spheres.size(); ++i) sph[i] = detail::c_material(sc.spheres[i].material, -1);
            check(rt_update_materials(ctx_, (int)mats.size(), mats.data(), (int)sph.size(), sph.data()),
                  "rt_update_materials");
            synced_mats_ = std::move(mats);
            synced_sph_ = std::move(sph);
        }
    }
    // getFinalColor's per-call sync (default on, the reference's semantics); off: the caller syncs
    void autoSync(bool on) { auto_sync_ = on; }
    bool autoSync() const { return auto_sync_; }

private:
    static rt_point_light conv(const PointLight& l) {
        rt_point_light x{};
        detail::put(x.position, l.position);
        detail::put(x.color, l.color);
        return x;
    }
    static rt_spherical_light conv(const SphericalLight& l) {
        rt_spherical_light x{};
        detail::put(x.position, l.position);
        x.radius = l.radius;
        detail::put(x.color, l.color);
        return x;
    }
    static rt_spot_light conv(const SpotLight& l) {
        rt_spot_light x{};
        detail::put(x.position, l.position);
        detail::put(x.direction, l.direction);
        x.angle = l.angle;
        detail::put(x.color, l.color);
        return x;
    }
    static rt_plane_light conv(const PlaneLight& l) {
        rt_plane_light x{};
        detail::put(x.position, l.position);
        detail::put(x.width, l.width);
        detail::put(x.height, l.height);
        detail::put(x.color, l.color);
        return x;
    }
    template <class L, class T>
    static bool differs(const std::vector<L>& src, const std::vector<T>& pushed) {
        if (src.size() != pushed.size()) return true;
        for (size_t i = 0; i < src.size(); ++i) {
            const T x = conv(src[i]);
            if (std::memcmp(&x, &pushed[i], sizeof(T)) != 0) return true;
        }
        return false;
    }
    // the lights last pushed to the device, in the C-ABI's structs
    struct Lights {
        std::vector<rt_point_light> pl;
        std::vector<rt_spherical_light> sl;
        std::vector<rt_spot_light> sp;
        std::vector<rt_plane_light> pn;
    };
    bool lights_changed(const Scene& sc) const {
        return differs(sc.pointLights, lights_.pl) || differs(sc.sphericalLight, lights_.sl) ||
               differs(sc.spotLight, lights_.sp) || differs(sc.planeLight, lights_.pn);
    }
    bool materials_changed(const Scene& sc) const {
        for (size_t i = 0; i < sc.meshes.size(); ++i) {
            const rt_material m = detail::c_material(sc.meshes[i].material, mesh_tex_[i]);
            if (std::memcmp(&m, &synced_mats_[i], sizeof m) != 0) return true;
        }
        for (size_t i = 0; i < sc.spheres.size(); ++i) {
            const rt_material m = detail::c_material(sc.spheres[i].material, -1);
            if (std::memcmp(&m, &synced_sph_[i], sizeof m) != 0) return true;
        }
        return false;
    }
    // the scene's lights into `out` and d's pointers to them
    static void lights_of(const Scene& sc, Lights& out, rt_scene_desc& d) {
        out = Lights{};
        for (const PointLight& l : sc.pointLights) out.pl.push_back(conv(l));
        for (const SphericalLight& l : sc.sphericalLight) out.sl.push_back(conv(l));
        for (const SpotLight& l : sc.spotLight) out.sp.push_back(conv(l));
        for (const PlaneLight& l : sc.planeLight) out.pn.push_back(conv(l));
        d.num_point_lights = (int)out.pl.size();
        d.point_lights = out.pl.data();
        d.num_spherical_lights = (int)out.sl.size();
        d.spherical_lights = out.sl.data();
        d.num_spot_lights = (int)out.sp.size();
        d.spot_lights = out.sp.data();
        d.num_plane_lights = (int)out.pn.size();
        d.plane_lights = out.pn.data();
    }

    Scene* scene_ = nullptr;
    rt_ctx* ctx_ = nullptr;
    std::vector<int> mesh_tex_;
    mutable std::vector<rt_material> synced_mats_, synced_sph_;
    mutable Lights lights_;
    bool auto_sync_ = true;
};

// ---- camera (framework/src/trackball.cpp:15-98; mouse handling out of scope) ----
struct Window {  // what Trackball reads from framework/src/window.cpp: aspectRatio() = w / h
    int width = 800, height = 800;
    float aspectRatio() const { return float(width) / float(height); }
};

class Trackball {
public:
    Trackball(const Window* pWindow, float fovy, float distanceFromLookAt = 4.0f, float rotationX = 0.0f,
              float rotationY = 0.0f)
        : Trackball(pWindow, fovy, vec3(0.0f), distanceFromLookAt, rotationX, rotationY) {}
    Trackball(const Window* pWindow, float fovy, const vec3& lookAt, float distanceFromLookAt = 4.0f,
              float rotationX = 0.0f, float rotationY = 0.0f)
        : window_(pWindow), fovy_(fovy), lookAt_(lookAt), dist_(distanceFromLookAt), rot_(rotationX, rotationY, 0.0f) {}
    void setCamera(const vec3 lookAt, const vec3 rotations, const float dist) {
        lookAt_ = lookAt;
        rot_ = rotations;
        dist_ = dist;
    }
    vec3 lookAt() const { return lookAt_; }
    vec3 position() const { return detail::v3(camera().position); }
    float aspectRatio() const { return window_ ? window_->aspectRatio() : 1.0f; }
    // Trackball::position / generateRay constants (framework/src/trackball.cpp:65-98)
    rt_camera camera(float aspect) const {
        rt_camera c;
        const float la[3] = {lookAt_.x, lookAt_.y, lookAt_.z};
        const float eu[3] = {rot_.x, rot_.y, rot_.z};
        check(rt_camera_from_trackball(la, eu, dist_, fovy_, aspect, &c), "Trackball");
        return c;
    }
    rt_camera camera() const { return camera(aspectRatio()); }
    // generateRay(pixel in NDC), glm::quat * vec3 in glm's order
    Ray generateRay(const vec2& pixel) const {
        const rt_camera c = camera();
        const vec3 csd = normalize(vec3(-pixel.x * c.half_width, pixel.y * c.half_height, 1.0f));
        const vec3 q(c.quat[0], c.quat[1], c.quat[2]);
        const vec3 uv = cross(q, csd), uuv = cross(q, uv);
        Ray r;
        r.origin = detail::v3(c.position);
        r.direction = csd + ((uv * c.quat[3]) + uuv) * 2.0f;
        r.t = FLT_MAX;
        return r;
    }

private:
    const Window* window_;
    float fovy_;
    vec3 lookAt_;
    float dist_;
    vec3 rot_;
};

// ---- framebuffer (src/screen.h:32-161) ----
enum class FilteringOption { None, Bloom, BloomWithReinhardHdr, BloomWithExposureHdr, OnlyLight, OnlyLightWithKernel };
enum class Kernel { BoxKernel, GaussianKernel };

class Screen {
public:
    explicit Screen(int width, int height) : W_(width), H_(height), data_((size_t)width * height * 3, 0.0f) {}
    void clear(const vec3& c) {
        for (size_t k = 0; k < data_.size(); k += 3) detail::put(&data_[k], c);
    }
    void setPixel(int x, int y, const vec3& c) {  // (0,0) bottom left, stored top row first (src/screen.cpp:32-38)
        detail::put(&data_[((size_t)(H_ - 1 - y) * W_ + x) * 3], c);
    }
    void postprocessImage() { check(rt_postprocess(&p_, W_, H_, data_.data()), "postprocessImage"); }
    void writeBitmapToFile(const std::string& path) {
        std::vector<uint8_t> rgba((size_t)W_ * H_ * 4);
        check(rt_bitmap(&p_, W_, H_, data_.data(), rgba.data()), "writeBitmapToFile");
        check(rt_write_bmp(path.c_str(), W_, H_, rgba.data()), "writeBitmapToFile");
    }
    void setBloomFilterLive(bool v) { p_.bloom_live = v ? 1 : 0; }
    void setBloomFilter(FilteringOption o) { p_.filtering_option = (int)o; }
    void setKernel(Kernel k) { p_.kernel = (int)k; }
    void setKernelNumRepetitions(int r) { p_.repetitions = r; }
    void setGammaValue(float g) { p_.gamma = g; }
    void enableGammaCorrection(float on) { p_.gamma_correction = on != 0.0f ? 1 : 0; }
    void setSigma(float s) { p_.sigma = s; }
    void setExposure(float e) { p_.exposure = e; }
    void setFilterSize(int f) { p_.filter_size = f; }
    std::vector<float>& textureData() { return data_; }
    int width() const { return W_; }
    int height() const { return H_; }

private:
    int W_, H_;
    std::vector<float> data_;
    rt_post_params p_{0, 0, 1, 5, 2.0f, 0.5f, 0, 2.2f, 0, 0};  // Screen's member defaults
};

// ---- the render path (src/main.cpp:129-400) ----
// getFinalColor(scene, bvh, ray, level) (src/main.cpp:129): one ray through rt_shade; `level` starts
// the recursion at that depth (the reference's `level >= max_reflection_level` stop).
inline vec3 getFinalColor(Scene& scene, const BoundingVolumeHierarchy& bvh, Ray ray, int level = 0) {
    if (bvh.autoSync()) bvh.sync(scene);
    rt_ray r{{ray.origin.x, ray.origin.y, ray.origin.z}, {ray.direction.x, ray.direction.y, ray.direction.z}, ray.t};
    const rt_params p = current_params(level);
    float rgb[3] = {0, 0, 0};
    check(rt_shade(bvh.handle(), &r, 1, &p, rgb, nullptr), "getFinalColor");
    return vec3{rgb[0], rgb[1], rgb[2]};
}

// renderRayTracing(scene, camera, bvh, screen, textureDebugging, anti_aliasing, multipleRays,
// sampleSize) (src/main.cpp:340-400): the whole frame in one launch, then postprocessImage.  The
// camera's aspect is its window's, the resolution the screen's, as in the reference.
inline void renderRayTracing(Scene& scene, const Trackball& camera, const BoundingVolumeHierarchy& bvh, Screen& screen,
                             bool textureDebugging = false, bool anti_aliasing = false, bool multipleRays = false,
                             int sampleSize = 4) {
    if (textureDebugging)  // getFinalColorNoRayTracingJustTextures (src/main.cpp:76-109): out of scope
        throw std::runtime_error("renderRayTracing: the texture-debug view is not part of the GPU path");
    bvh.sync(scene);
    const rt_camera c = camera.camera();
    rt_params p = current_params();
    p.anti_aliasing = anti_aliasing ? 1 : 0;
    p.multiple_rays = multipleRays ? 1 : 0;
    p.sample_size = sampleSize;
    check(rt_render(bvh.handle(), &c, &p, screen.width(), screen.height(), screen.textureData().data(), nullptr),
          "renderRayTracing");
    screen.postprocessImage();
}

// A batch of renderRayTracing calls, one per camera (a turntable, an animation's camera path), in ONE
// launch of the persistent kernel (rt_render_views): screens[v] = the frame of cameras[v], bit-identical
// to renderRayTracing with that camera (before post-processing).
inline void renderRayTracingViews(Scene& scene, const std::vector<Trackball>& cameras, const BoundingVolumeHierarchy& bvh,
                                  int W, int H, std::vector<std::vector<float>>& screens, bool anti_aliasing = false,
                                  bool multipleRays = false, int sampleSize = 4) {
    bvh.sync(scene);
    std::vector<rt_camera> c;
    for (const Trackball& t : cameras) c.push_back(t.camera());
    rt_params p = current_params();
    p.anti_aliasing = anti_aliasing ? 1 : 0;
    p.multiple_rays = multipleRays ? 1 : 0;
    p.sample_size = sampleSize;
    const size_t frame = (size_t)W * H * 3;
    std::vector<float> all(frame * cameras.size());
    check(rt_render_views(bvh.handle(), c.data(), (int)c.size(), &p, W, H, all.data(), nullptr),
          "renderRayTracingViews");
    screens.assign(cameras.size(), {});
    for (size_t v = 0; v < cameras.size(); ++v) screens[v].assign(all.begin() + v * frame, all.begin() + (v + 1) * frame);
}

}  // namespace facade
}  // namespace rt
