// host_scene.h -- host-side scene model mirroring the reference's POD types.
//   Vertex/Material/Mesh: src/mesh.h:14-44      Scene + lights + Sphere: src/scene.h:36-94
#pragma once
#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "rt_math.h"
#include "../../include/rt_amd.h"

namespace rt {

struct Vertex {
    v3 p;
    v3 n;
    v2 uv;
};

struct Material {
    v3 kd{0.0f, 0.0f, 0.0f};
    v3 ks{0.0f, 0.0f, 0.0f};
    float shininess = 1.0f;
    float transparency = 1.0f;
    bool has_texture = false;
    std::string texture_path;
    int texture = -1;  // index into HostScene::textures once loaded
};

// Image (src/image.h): the decoded file as stbi_load(..., STBI_rgb) returns it
struct HostTexture {
    std::string path;
    int width = 0, height = 0, channels = 0;
    std::vector<uint8_t> rgb;
};

struct Mesh {
    std::vector<Vertex> vertices;
    std::vector<std::array<uint32_t, 3>> triangles;
    Material material;
};

struct HostScene {
    std::vector<Mesh> meshes;
    std::vector<rt_sphere> spheres;
    std::vector<rt_point_light> point_lights;
    std::vector<rt_spherical_light> spherical_lights;
    std::vector<rt_spot_light> spot_lights;
    std::vector<rt_plane_light> plane_lights;

    std::vector<HostTexture> textures;
    // Image::Image for every mesh with a kd texture not yet loaded (src/mesh.cpp:141): throws
    // std::runtime_error when the file is missing, undecodable or has fewer than 3 channels
    void load_textures();

    // flattened view (rebuilt by flatten())
    std::vector<float> flat_pos, flat_nrm, flat_uv;
    std::vector<int> flat_mesh;
    std::vector<rt_material> flat_mat;
    std::vector<rt_texture> flat_tex;
    void flatten();
    void fill_desc(rt_scene_desc* d) const;
};

// loadMesh (src/mesh.cpp:58-162) + centerAndScaleToUnitMesh (:164-188) with Assimp 5.0.1
// OBJ/MTL importer semantics.  Throws std::runtime_error on failure.
// compat: RT_ASSIMP3_* bits (rt_amd.h)
std::vector<Mesh> load_obj(const std::string& path, bool normalize, int compat);

// loadScene (src/scene.cpp:4-150)
void load_preset(HostScene& scene, int preset, const std::string& data_dir, int compat);

// Deterministic torus-knot stand-in for data/dragon.obj (missing, .MISSING_LARGE_BLOBS:1)
void write_dragon_proxy(const std::string& obj_path, int u_segments, int v_segments);

// Assimp fast_atoreal_move<float> (fast_atof.h), exposed for tests.
const char* fast_atoreal_move(const char* c, float& out, bool check_comma = true);

}  // namespace rt
