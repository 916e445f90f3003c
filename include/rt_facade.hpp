// rt_facade.hpp -- C++ facade over the C-ABI that keeps the reference's names and semantics, so
// main.cpp's render path can switch to the MI355X implementation by swapping includes.
//
//   reference                                           facade
//   struct Vertex/Material/Mesh (src/mesh.h:14-44)      rt::facade::{Vertex,Material,Mesh}
//   struct Scene + lights (src/scene.h:36-94)           rt::facade::Scene (+ loadScene / loadMesh)
//   struct Ray (framework/include/ray.h:11-29)          rt::facade::Ray
//   struct HitInfo (src/ray_tracing.h:6-37)             rt::facade::HitInfo
//   class BoundingVolumeHierarchy (src/bounding_volume_hierarchy.h:22-81)
//                                                       rt::facade::BoundingVolumeHierarchy
//   getFinalColor (src/main.cpp:129)                    rt::facade::getFinalColor
//   renderRayTracing (src/main.cpp:340)                 rt::facade::renderRayTracing
//   one renderRayTracing per camera, batched             rt::facade::renderRayTracingViews
//
// Errors: loadMesh/loadScene throw std::runtime_error like the reference's loadMesh throws
// (src/mesh.cpp:60-73); intersect() never throws and returns false on a miss.  A device error
// (e.g. no GPU) throws from the BoundingVolumeHierarchy constructor -- there is no CPU fallback.
#pragma once
#include <array>
#include <cfloat>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_amd.h"

namespace rt {
namespace facade {

struct vec3 {
    float x = 0, y = 0, z = 0;
};
struct vec2 {
    float x = 0, y = 0;
};

struct Ray {
    vec3 origin{0, 0, 0};
    vec3 direction{0, 0, -1};
    float t = FLT_MAX;
};

struct Material {
    vec3 kd;
    vec3 ks{0, 0, 0};
    float shininess = 1.0f;
    float transparency = 1.0f;
};

struct HitInfo {
    vec3 normal;
    vec3 hitPoint;
    int material_index = 0;
    vec2 texCoord;
    bool is_triangle = false;
    int prim_id = -1;
};

inline std::string last_error() {
    char buf[1024];
    rt_last_error(buf, sizeof(buf));
    return buf;
}
inline void check(int rc, const char* what) {
    if (rc != RT_OK) throw std::runtime_error(std::string(what) + ": " + last_error());
}

// SceneType (src/scene.h:14-34)
enum SceneType {
    SingleTriangle, Bookeshelf, Cube, CornellBox, CornellBoxSphericalLight, CornellBoxPlaneLight, Monkey, Teapot,
    Dragon, Spheres, ChessBoard, Custom, AndreasScene, CatalinScene, MikeScene, MikeScene2
};

class Scene {
public:
    Scene() { check(rt_scene_new(&h_), "rt_scene_new"); }
    ~Scene() { rt_scene_free(h_); }
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;
    Scene(Scene&& o) noexcept : h_(o.h_) { o.h_ = nullptr; }

    void addPointLight(vec3 p, vec3 c) {
        rt_point_light l{{p.x, p.y, p.z}, {c.x, c.y, c.z}};
        check(rt_scene_add_point_light(h_, &l), "addPointLight");
    }
    void addSphericalLight(vec3 p, float r, vec3 c) {
        rt_spherical_light l{{p.x, p.y, p.z}, r, {c.x, c.y, c.z}};
        check(rt_scene_add_spherical_light(h_, &l), "addSphericalLight");
    }
    void addSpotLight(vec3 p, vec3 d, float angle, vec3 c) {
        rt_spot_light l{{p.x, p.y, p.z}, {d.x, d.y, d.z}, angle, {c.x, c.y, c.z}};
        check(rt_scene_add_spot_light(h_, &l), "addSpotLight");
    }
    void addPlaneLight(vec3 p, vec3 w, vec3 hgt, vec3 c) {
        rt_plane_light l{{p.x, p.y, p.z}, {w.x, w.y, w.z}, {hgt.x, hgt.y, hgt.z}, {c.x, c.y, c.z}};
        check(rt_scene_add_plane_light(h_, &l), "addPlaneLight");
    }
    void addSphere(vec3 center, float radius, const Material& m) {
        rt_sphere s{{center.x, center.y, center.z}, radius, to_c(m)};
        check(rt_scene_add_sphere(h_, &s), "addSphere");
    }
    rt_scene* handle() const { return h_; }
    rt_scene_desc desc() const {
        rt_scene_desc d;
        check(rt_scene_desc_get(h_, &d), "rt_scene_desc_get");
        return d;
    }
    static rt_material to_c(const Material& m) {
        rt_material r{};
        r.kd[0] = m.kd.x; r.kd[1] = m.kd.y; r.kd[2] = m.kd.z;
        r.ks[0] = m.ks.x; r.ks[1] = m.ks.y; r.ks[2] = m.ks.z;
        r.shininess = m.shininess;
        r.transparency = m.transparency;
        return r;
    }

private:
    rt_scene* h_ = nullptr;
};

// loadMesh (src/mesh.cpp:58): appends the file's meshes to the scene (Assimp 5.0.1 semantics)
inline void loadMesh(Scene& scene, const std::string& file, bool normalize = false) {
    check(rt_scene_load_obj(scene.handle(), file.c_str(), normalize ? 1 : 0, 0), "loadMesh");
}

// loadScene (src/scene.cpp:4)
inline Scene loadScene(SceneType type, const std::string& dataDir) {
    Scene s;
    check(rt_scene_preset(s.handle(), (int)type, dataDir.c_str(), 0), "loadScene");
    return s;
}

// TextureFiltering / OutOfBoundsRule (src/image.h:16-29)
enum class TextureFiltering {
    NearestNeighbor = RT_TEX_NEAREST,
    Bilinear = RT_TEX_BILINEAR,
    MipMappingNearestLevelNearestNeighbor = RT_TEX_MIP_NEAREST,
    MipMappingNearestLevelBilinear = RT_TEX_MIP_NEAREST_BILINEAR,
    Trilinear = RT_TEX_TRILINEAR
};
enum class OutOfBoundsRule { Border = RT_OOB_BORDER, Clamp = RT_OOB_CLAMP, Repeat = RT_OOB_REPEAT };

// Render knobs = the reference's globals (src/main.cpp:54-64,123-127)
struct RenderSettings {
    int max_reflection_level = 5;
    int sphere_light_ray_count = 10;
    int plane_light_1D_ray_count = 3;
    int glossy_ray_count = 1;  // reference default 10 draws rand(); 1 is deterministic
    float refraction_factor = 0.8f;
    bool useBVH = false;
    bool useTextures = false;
    TextureFiltering textureFiltering = TextureFiltering::NearestNeighbor;
    OutOfBoundsRule outOfBoundsRuleX = OutOfBoundsRule::Border;
    OutOfBoundsRule outOfBoundsRuleY = OutOfBoundsRule::Border;
    vec3 textureBorderColor{0.0f, 0.0f, 0.0f};
    rt_params to_c() const {
        rt_params p{};
        p.max_reflection_level = max_reflection_level;
        p.sphere_light_ray_count = sphere_light_ray_count;
        p.plane_light_1D_ray_count = plane_light_1D_ray_count;
        p.glossy_ray_count = glossy_ray_count;
        p.refraction_factor = refraction_factor;
        p.use_bvh = useBVH ? 1 : 0;
        p.sample_size = 4;
        p.use_textures = useTextures ? 1 : 0;
        p.texture_filtering = (int)textureFiltering;
        p.out_of_bounds_x = (int)outOfBoundsRuleX;
        p.out_of_bounds_y = (int)outOfBoundsRuleY;
        p.border_color[0] = textureBorderColor.x;
        p.border_color[1] = textureBorderColor.y;
        p.border_color[2] = textureBorderColor.z;
        return p;
    }
};

class BoundingVolumeHierarchy {
public:
    explicit BoundingVolumeHierarchy(Scene* pScene, int device = 0) {
        const rt_scene_desc d = pScene->desc();
        check(rt_create(&d, device, &ctx_), "BoundingVolumeHierarchy");
    }
    ~BoundingVolumeHierarchy() { rt_destroy(ctx_); }
    BoundingVolumeHierarchy(const BoundingVolumeHierarchy&) = delete;
    BoundingVolumeHierarchy& operator=(const BoundingVolumeHierarchy&) = delete;

    // bool intersect(Ray&, HitInfo&, bool useBVH) const (src/bounding_volume_hierarchy.h:33)
    bool intersect(Ray& ray, HitInfo& hitInfo, bool useBVH) const {
        rt_ray r{{ray.origin.x, ray.origin.y, ray.origin.z}, {ray.direction.x, ray.direction.y, ray.direction.z}, ray.t};
        rt_hit h{};
        if (rt_intersect(ctx_, &r, 1, useBVH ? 1 : 0, &h) != RT_OK) return false;
        if (!h.hit) return false;
        ray.t = h.t;
        hitInfo.normal = vec3{h.normal[0], h.normal[1], h.normal[2]};
        hitInfo.hitPoint = vec3{h.hit_point[0], h.hit_point[1], h.hit_point[2]};
        hitInfo.material_index = h.material_index;
        hitInfo.texCoord = vec2{h.uv[0], h.uv[1]};
        hitInfo.is_triangle = h.is_triangle != 0;
        hitInfo.prim_id = h.prim_id;
        return true;
    }
    int numLevels() const {
        int nodes = 0, recs = 0, refn = 0, levels = 0;
        rt_ctx_info(ctx_, &nodes, &recs, &refn, &levels);
        return levels;
    }
    rt_ctx* handle() const { return ctx_; }

private:
    rt_ctx* ctx_ = nullptr;
};

// getFinalColor(scene, bvh, ray, level = 0) (src/main.cpp:129)
inline vec3 getFinalColor(const BoundingVolumeHierarchy& bvh, const Ray& ray, const RenderSettings& s = {}) {
    rt_ray r{{ray.origin.x, ray.origin.y, ray.origin.z}, {ray.direction.x, ray.direction.y, ray.direction.z}, ray.t};
    const rt_params p = s.to_c();
    float rgb[3] = {0, 0, 0};
    check(rt_shade(bvh.handle(), &r, 1, &p, rgb, nullptr), "getFinalColor");
    return vec3{rgb[0], rgb[1], rgb[2]};
}

struct Trackball {  // the parts of framework/include/trackball.h the render path reads
    vec3 lookAt{0, 0, 0};
    vec3 rotationEulerAngles{0.34906584f, 0.34906584f, 0.0f};  // glm::radians(vec3(20,20,0))
    float distance = 3.0f;
    float fovy = 0.87266463f;                                  // glm::radians(50.0f)
};

// renderRayTracing(scene, camera, bvh, screen, textureDebugging, anti_aliasing, multipleRays, sampleSize)
// (src/main.cpp:340); `screen` = W*H*3 floats in Screen::m_textureData order.
inline void renderRayTracing(const Trackball& cam, const BoundingVolumeHierarchy& bvh, int W, int H,
                             std::vector<float>& screen, bool anti_aliasing = false, bool multipleRays = false,
                             int sampleSize = 4, const RenderSettings& s = {}) {
    rt_camera c;
    const float la[3] = {cam.lookAt.x, cam.lookAt.y, cam.lookAt.z};
    const float eu[3] = {cam.rotationEulerAngles.x, cam.rotationEulerAngles.y, cam.rotationEulerAngles.z};
    check(rt_camera_from_trackball(la, eu, cam.distance, cam.fovy, float(W) / float(H), &c), "camera");
    rt_params p = s.to_c();
    p.anti_aliasing = anti_aliasing ? 1 : 0;
    p.multiple_rays = multipleRays ? 1 : 0;
    p.sample_size = sampleSize;
    screen.resize((size_t)W * H * 3);
    check(rt_render(bvh.handle(), &c, &p, W, H, screen.data(), nullptr), "renderRayTracing");
}

// A batch of renderRayTracing calls, one per camera (a turntable, an animation's camera path), in ONE
// launch of the persistent kernel (rt_render_views): screens[v] = the frame of cams[v], bit-identical to
// renderRayTracing(cams[v], ...).
inline void renderRayTracingViews(const std::vector<Trackball>& cams, const BoundingVolumeHierarchy& bvh, int W,
                                  int H, std::vector<std::vector<float>>& screens, bool anti_aliasing = false,
                                  bool multipleRays = false, int sampleSize = 4, const RenderSettings& s = {}) {
    std::vector<rt_camera> c(cams.size());
    for (size_t v = 0; v < cams.size(); ++v) {
        const Trackball& t = cams[v];
        const float la[3] = {t.lookAt.x, t.lookAt.y, t.lookAt.z};
        const float eu[3] = {t.rotationEulerAngles.x, t.rotationEulerAngles.y, t.rotationEulerAngles.z};
        check(rt_camera_from_trackball(la, eu, t.distance, t.fovy, float(W) / float(H), &c[v]), "camera");
    }
    rt_params p = s.to_c();
    p.anti_aliasing = anti_aliasing ? 1 : 0;
    p.multiple_rays = multipleRays ? 1 : 0;
    p.sample_size = sampleSize;
    const size_t frame = (size_t)W * H * 3;
    std::vector<float> all(frame * cams.size());
    check(rt_render_views(bvh.handle(), c.data(), (int)c.size(), &p, W, H, all.data(), nullptr),
          "renderRayTracingViews");
    screens.assign(cams.size(), {});
    for (size_t v = 0; v < cams.size(); ++v) screens[v].assign(all.begin() + v * frame, all.begin() + (v + 1) * frame);
}

// class Screen (src/screen.h:32-161): the framebuffer renderRayTracing fills, with the
// reference's post-processing setters; postprocessImage / writeBitmapToFile run on the GPU
// (rt_postprocess / rt_bitmap + rt_write_bmp).  The GL draw() path is out of scope.
enum class FilteringOption { None, Bloom, BloomWithReinhardHdr, BloomWithExposureHdr, OnlyLight, OnlyLightWithKernel };
enum class Kernel { BoxKernel, GaussianKernel };

class Screen {
public:
    Screen(int width, int height) : W_(width), H_(height), data_((size_t)width * height * 3, 0.0f) {}
    void clear(const vec3& c) {
        for (size_t k = 0; k < data_.size(); k += 3) {
            data_[k] = c.x;
            data_[k + 1] = c.y;
            data_[k + 2] = c.z;
        }
    }
    void setPixel(int x, int y, const vec3& c) {  // (0,0) bottom left, stored top row first
        const size_t i = ((size_t)(H_ - 1 - y) * W_ + x) * 3;
        data_[i] = c.x;
        data_[i + 1] = c.y;
        data_[i + 2] = c.z;
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

// renderRayTracing into a Screen, then Screen::postprocessImage (src/main.cpp:398)
inline void renderRayTracing(const Trackball& cam, const BoundingVolumeHierarchy& bvh, Screen& screen,
                             bool anti_aliasing = false, bool multipleRays = false, int sampleSize = 4,
                             const RenderSettings& s = {}) {
    renderRayTracing(cam, bvh, screen.width(), screen.height(), screen.textureData(), anti_aliasing, multipleRays,
                     sampleSize, s);
    screen.postprocessImage();
}

}  // namespace facade
}  // namespace rt
