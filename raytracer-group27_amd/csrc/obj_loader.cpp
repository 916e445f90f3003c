// obj_loader.cpp -- loadMesh (reference src/mesh.cpp:58-188) restated without Assimp.
//
// The reference imports OBJ through Assimp 5.0.1 (framework/cmake/download_optional_packages.cmake:43-46)
// with aiProcess_GenNormals | aiProcess_Triangulate (src/mesh.cpp:67), then walks the node tree
// LIFO (src/mesh.cpp:77-154) and optionally centres/normalises (src/mesh.cpp:164-188).  Assimp is
// not available here, so this file restates the parts of its published OBJ importer that decide
// the bits the renderer sees:
//   * float parsing = fast_atoreal_move<float>: float(intpart) + float(double(frac) * 10^-n)
//   * one object (node) per 'o' and per changed 'g' name; one mesh per material inside an object
//   * vertices are never shared between faces (one vertex per face corner, face order)
//   * quads: fan from the concave corner (corner 0 for convex quads); n>4: Assimp's ear cutting
//     in the plane of the Newell normal (ear_cut; AndreasScene.obj and CGSceneAdv.obj have 107)
//   * GenFaceNormals after Triangulate: meshes without 'vn' get per-triangle normals, a corner
//     shared by two triangles keeps the last one written
//   * materials: DefaultMaterial{kd .6, ks 0, Ns 0, d 1}; 'mtllib' leaves the last material of
//     the library current (so a new object/group inherits it until 'usemtl')
//   * node walk: root children are visited in reverse (std::stack), meshes of a node in order
//   * transforms: identity matrices applied with glm's op order (-0 positions become +0;
//     normals go through glm::inverseTranspose(mat3(I)), whose off-diagonals carry -0)
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "host_scene.h"

namespace rt {

// Assimp fast_atof.h: table of 10^-n as double literals
static const double kFastAtofTable[16] = {0.0,
                                          0.1,
                                          0.01,
                                          0.001,
                                          0.0001,
                                          0.00001,
                                          0.000001,
                                          0.0000001,
                                          0.00000001,
                                          0.000000001,
                                          0.0000000001,
                                          0.00000000001,
                                          0.000000000001,
                                          0.0000000000001,
                                          0.00000000000001,
                                          0.000000000000001};

static uint64_t strtoul10_64(const char* in, const char** out, unsigned int* max_inout) {
    unsigned int cur = 0;
    uint64_t value = 0;
    if (*in < '0' || *in > '9') throw std::runtime_error("OBJ: cannot convert string to value");
    for (;;) {
        if (*in < '0' || *in > '9') break;
        const uint64_t nv = value * 10u + (uint64_t)(*in - '0');
        if (nv < value) return 0;  // overflow: Assimp warns and returns 0
        value = nv;
        ++in;
        ++cur;
        if (max_inout && *max_inout == cur) {
            if (out) {
                while (*in >= '0' && *in <= '9') ++in;
                *out = in;
            }
            return value;
        }
    }
    if (out) *out = in;
    if (max_inout) *max_inout = cur;
    return value;
}

const char* fast_atoreal_move(const char* c, float& out, bool check_comma) {
    float f = 0.0f;
    const bool inv = (*c == '-');
    if (inv || *c == '+') ++c;
    if ((c[0] == 'N' || c[0] == 'n') && strncasecmp(c, "nan", 3) == 0) {
        out = std::numeric_limits<float>::quiet_NaN();
        c += 3;
        return c;
    }
    if ((c[0] == 'I' || c[0] == 'i') && strncasecmp(c, "inf", 3) == 0) {
        out = std::numeric_limits<float>::infinity();
        if (inv) out = -out;
        c += 3;
        if ((c[0] == 'I' || c[0] == 'i') && strncasecmp(c, "inity", 5) == 0) c += 5;
        return c;
    }
    if (!(c[0] >= '0' && c[0] <= '9') &&
        !((c[0] == '.' || (check_comma && c[0] == ',')) && c[1] >= '0' && c[1] <= '9')) {
        throw std::runtime_error("OBJ: cannot parse string as real number");
    }
    if (*c != '.' && (!check_comma || c[0] != ',')) {
        f = static_cast<float>(strtoul10_64(c, &c, nullptr));
    }
    if ((*c == '.' || (check_comma && c[0] == ',')) && c[1] >= '0' && c[1] <= '9') {
        ++c;
        unsigned int diff = 15;  // AI_FAST_ATOF_RELAVANT_DECIMALS
        double pl = static_cast<double>(strtoul10_64(c, &c, &diff));
        pl *= kFastAtofTable[diff];
        f += static_cast<float>(pl);
    } else if (*c == '.') {
        ++c;
    }
    if (*c == 'e' || *c == 'E') {
        ++c;
        const bool einv = (*c == '-');
        if (einv || *c == '+') ++c;
        float ex = static_cast<float>(strtoul10_64(c, &c, nullptr));
        if (einv) ex = -ex;
        f *= std::pow(10.0f, ex);
    }
    if (inv) f = -f;
    out = f;
    return c;
}

static float fast_atof(const std::string& s) {
    float r = 0.0f;
    fast_atoreal_move(s.c_str(), r, true);
    return r;
}

namespace {

struct ObjMaterial {
    std::string name;
    v3 diffuse{0.6f, 0.6f, 0.6f};
    v3 specular{0.0f, 0.0f, 0.0f};
    float shineness = 0.0f;
    float alpha = 1.0f;
    std::string texture;
};

struct Face {
    std::vector<int> v, vt, vn;
};

struct ObjMesh {
    std::vector<Face> faces;
    int material = -1;  // index into lib order (-1 == NoMaterial)
    bool has_normals = false;
};

struct ObjObject {
    std::string name;
    std::vector<int> meshes;
};

struct ObjModel {
    std::vector<v3> vertices, normals, texcoords;
    std::vector<ObjObject> objects;
    std::vector<ObjMesh> meshes;
    std::vector<ObjMaterial> materials;  // m_MaterialLib order, [0] = DefaultMaterial
    std::map<std::string, int> material_map;
    int current_object = -1;
    int current_mesh = -1;
    int current_material = -1;
    int default_material = 0;
    std::string active_group;
    bool has_active_group = false;
};

static std::vector<std::string> split_ws(const std::string& s) {
    std::vector<std::string> out;
    size_t i = 0, n = s.size();
    while (i < n) {
        while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\r')) ++i;
        if (i >= n) break;
        size_t j = i;
        while (j < n && s[j] != ' ' && s[j] != '\t' && s[j] != '\r') ++j;
        out.push_back(s.substr(i, j - i));
        i = j;
    }
    return out;
}

static std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r')) ++a;
    while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) --b;
    return s.substr(a, b - a);
}

static void read_lines(const std::string& path, std::vector<std::string>& lines) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("File " + path + " does not exist.");
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string data = ss.str();
    lines.clear();
    size_t i = 0;
    std::string cur;
    while (i < data.size()) {
        const char ch = data[i++];
        if (ch == '\n') {
            // Assimp's IOStreamBuffer joins lines ending in a backslash
            if (!cur.empty() && cur.back() == '\\') {
                cur.pop_back();
                continue;
            }
            lines.push_back(cur);
            cur.clear();
        } else {
            cur.push_back(ch);
        }
    }
    if (!cur.empty()) lines.push_back(cur);
}

static int create_material(ObjModel& m, const std::string& name) {
    auto it = m.material_map.find(name);
    if (it != m.material_map.end()) return it->second;
    ObjMaterial mat;
    mat.name = name;
    m.materials.push_back(mat);
    const int idx = (int)m.materials.size() - 1;
    m.material_map[name] = idx;
    return idx;
}

// ObjFileMtlImporter::load
static void load_mtl(ObjModel& m, const std::string& path) {
    std::vector<std::string> lines;
    try {
        read_lines(path, lines);
    } catch (...) {
        return;  // Assimp logs "OBJ: Unable to locate material file" and goes on
    }
    for (const std::string& raw : lines) {
        std::string line = raw;
        size_t s = 0;
        while (s < line.size() && (line[s] == ' ' || line[s] == '\t')) ++s;
        line = line.substr(s);
        if (line.empty()) continue;
        const std::vector<std::string> tok = split_ws(line);
        if (tok.empty()) continue;
        const char c0 = line[0];
        auto color = [&](v3& dst) {
            // getColorRGBA: r, then optional g b (else g = b = r)
            if (tok.size() >= 2) dst.x = fast_atof(tok[1]);
            if (tok.size() >= 4) {
                dst.y = fast_atof(tok[2]);
                dst.z = fast_atof(tok[3]);
            } else {
                dst.y = dst.z = dst.x;
            }
        };
        if (c0 == 'n' || c0 == 'N') {
            if (line.size() > 1 && line[1] == 'e') {  // newmtl
                std::string name;
                if (tok.size() == 1) {
                    name = "DefaultMaterial";
                } else {
                    size_t ws = line.find_first_of(" \t");
                    size_t nws = line.find_first_not_of(" \t", ws);
                    if (nws != std::string::npos) name = line.substr(nws);
                }
                m.current_material = create_material(m, trim(name));
            } else if (line.size() > 1 && line[1] == 's' && m.current_material >= 0) {
                if (tok.size() >= 2) m.materials[m.current_material].shineness = fast_atof(tok[1]);
            }
        } else if ((c0 == 'K' || c0 == 'k') && m.current_material >= 0 && line.size() > 1) {
            ObjMaterial& mt = m.materials[m.current_material];
            if (line[1] == 'd') color(mt.diffuse);
            else if (line[1] == 's') color(mt.specular);
        } else if (c0 == 'd' && m.current_material >= 0) {
            if (line.compare(0, 4, "disp") != 0 && tok.size() >= 2)
                m.materials[m.current_material].alpha = fast_atof(tok[1]);
        } else if ((c0 == 'm') && m.current_material >= 0) {
            if (tok[0] == "map_Kd" && tok.size() >= 2) m.materials[m.current_material].texture = tok.back();
        }
    }
}

static void create_mesh(ObjModel& m) {
    m.meshes.push_back(ObjMesh{});
    m.current_mesh = (int)m.meshes.size() - 1;
    if (m.current_object >= 0) m.objects[m.current_object].meshes.push_back(m.current_mesh);
}

static void create_object(ObjModel& m, const std::string& name) {
    m.objects.push_back(ObjObject{name, {}});
    m.current_object = (int)m.objects.size() - 1;
    create_mesh(m);
    if (m.current_material >= 0) m.meshes[m.current_mesh].material = m.current_material;
}

static int parse_index(const std::string& s, int size) {
    const int v = std::atoi(s.c_str());
    if (v > 0) return v - 1;
    if (v < 0) return size + v;
    throw std::runtime_error("OBJ: Invalid face indice");
}

static void parse_obj(ObjModel& m, const std::string& path) {
    std::vector<std::string> lines;
    read_lines(path, lines);
    const std::string dir = path.substr(0, path.find_last_of("/\\") + 1);
    // ObjFileParser(): DefaultMaterial is entry 0 of the material library
    m.default_material = create_material(m, "DefaultMaterial");
    for (const std::string& raw : lines) {
        size_t s = 0;
        while (s < raw.size() && (raw[s] == ' ' || raw[s] == '\t')) ++s;
        if (s >= raw.size()) continue;
        const std::string line = raw.substr(s);
        const std::vector<std::string> tok = split_ws(line);
        if (tok.empty()) continue;
        const std::string& k = tok[0];
        if (k == "v") {
            const size_t nc = tok.size() - 1;
            if (nc == 3 || nc == 6) {
                m.vertices.push_back(v3{fast_atof(tok[1]), fast_atof(tok[2]), fast_atof(tok[3])});
            } else if (nc == 4) {
                const float x = fast_atof(tok[1]), y = fast_atof(tok[2]), z = fast_atof(tok[3]),
                            w = fast_atof(tok[4]);
                if (w == 0.0f) throw std::runtime_error("OBJ: Invalid component in homogeneous vector (Division by zero)");
                m.vertices.push_back(v3{x / w, y / w, z / w});
            }
        } else if (k == "vn") {
            if (tok.size() < 4) throw std::runtime_error("OBJ: bad normal");
            m.normals.push_back(v3{fast_atof(tok[1]), fast_atof(tok[2]), fast_atof(tok[3])});
        } else if (k == "vt") {
            const size_t nc = tok.size() - 1;
            if (nc == 2) m.texcoords.push_back(v3{fast_atof(tok[1]), fast_atof(tok[2]), 0.0f});
            else if (nc == 3) m.texcoords.push_back(v3{fast_atof(tok[1]), fast_atof(tok[2]), fast_atof(tok[3])});
            else throw std::runtime_error("OBJ: Invalid number of components");
        } else if (k == "f") {
            if (tok.size() < 2) continue;
            Face face;
            const int vs = (int)m.vertices.size(), vts = (int)m.texcoords.size(), vns = (int)m.normals.size();
            const bool has_vt = !m.texcoords.empty(), has_vn = !m.normals.empty();
            bool has_normal = false;
            for (size_t i = 1; i < tok.size(); ++i) {
                std::vector<std::string> parts;
                size_t a = 0;
                const std::string& t = tok[i];
                for (;;) {
                    size_t b = t.find('/', a);
                    parts.push_back(t.substr(a, b == std::string::npos ? std::string::npos : b - a));
                    if (b == std::string::npos) break;
                    a = b + 1;
                }
                face.v.push_back(parse_index(parts[0], vs));
                if (parts.size() >= 2 && !parts[1].empty() && has_vt) face.vt.push_back(parse_index(parts[1], vts));
                if (parts.size() >= 3 && !parts[2].empty() && has_vn) {
                    face.vn.push_back(parse_index(parts[2], vns));
                    has_normal = true;
                } else if (parts.size() == 2 && !has_vt && has_vn && !parts[1].empty()) {
                    // "v/vn" with no texture coordinates: Assimp skips to the normal slot
                    face.vn.push_back(parse_index(parts[1], vns));
                    has_normal = true;
                }
            }
            if (m.current_object < 0) create_object(m, "defaultobject");
            if (m.current_mesh < 0) create_mesh(m);
            ObjMesh& mesh = m.meshes[m.current_mesh];
            mesh.faces.push_back(face);
            if (has_normal) mesh.has_normals = true;
        } else if (k == "o") {
            std::string name = trim(line.substr(1));
            int found = -1;
            for (size_t i = 0; i < m.objects.size(); ++i)
                if (m.objects[i].name == name) found = (int)i;
            if (found >= 0) {
                m.current_object = found;
            } else {
                create_object(m, name);
            }
        } else if (k == "g") {
            std::string name = trim(line.substr(1));
            if (name.empty()) continue;
            if (!m.has_active_group || m.active_group != name) {
                create_object(m, name);
                m.active_group = name;
                m.has_active_group = true;
            }
        } else if (k == "usemtl") {
            std::string name = trim(line.substr(6));
            if (name.empty()) continue;
            if (m.current_material >= 0 && m.materials[m.current_material].name == name) continue;
            auto it = m.material_map.find(name);
            if (it == m.material_map.end()) {
                m.current_material = create_material(m, name);
            } else {
                m.current_material = it->second;
            }
            // needsNewMesh
            bool need = false;
            if (m.current_mesh < 0) {
                need = true;
            } else {
                const ObjMesh& cm = m.meshes[m.current_mesh];
                if (cm.material != -1 && cm.material != m.current_material && !cm.faces.empty()) need = true;
            }
            if (need) create_mesh(m);
            m.meshes[m.current_mesh].material = m.current_material;
        } else if (k == "mtllib") {
            if (tok.size() >= 2) load_mtl(m, dir + trim(line.substr(6)));
        }
        // 's', 'l', 'p', '#', 'mg' and anything else: skipped
    }
}

// Assimp aiVector3t helpers (float)
static float ai_len(v3 v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
static v3 ai_normalize(v3 v) {
    // Normalize(): *this /= Length()  -- operator/= multiplies by the reciprocal (Assimp 4.x/5.x)
    const float l = ai_len(v);
    const float inv = 1.0f / l;
    return v3{v.x * inv, v.y * inv, v.z * inv};
}
// NormalizeSafe(): 5.x's operator/= multiplies by the reciprocal; 3.x divides each component
// (RT_ASSIMP3_NORMALS_DIV: bit-exact with the Assimp 3.3 build of this image)
static v3 ai_normalize_safe(v3 v, bool div = false) {
    const float l = ai_len(v);
    if (l > 0.0f) {
        if (div) return v3{v.x / l, v.y / l, v.z / l};
        const float inv = 1.0f / l;
        return v3{v.x * inv, v.y * inv, v.z * inv};
    }
    return v;
}
static float ai_dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 ai_cross(v3 a, v3 o) { return v3{a.y * o.z - a.z * o.y, a.z * o.x - a.x * o.z, a.x * o.y - a.y * o.x}; }

struct AiMesh {
    std::vector<v3> verts, norms, uvs;
    bool has_normals = false;
    std::vector<std::array<uint32_t, 3>> tris;
    int material = 0;
};

// TriangulateProcess for n > 4 (code/PostProcessing/TriangulateProcess.cpp, Assimp 5.0.1; the same
// code as 3.3's): project onto the plane of the Newell normal (dropping the axis of its largest
// component, axes swapped when that component is negative), then cut ears in polygon order -- an
// ear is a convex corner (GetArea2D > 0 in double) whose triangle contains no other polygon point
// (PointInTriangle2D on float dot products, open test, points equal to a corner skipped) -- and emit
// the last three corners.  A polygon without an ear (not simple) keeps the triangles cut so far, as
// Assimp does.
static double area2d(const float* a, const float* b, const float* c) {  // GetArea2D(v1, v2, v3)
    return 0.5 * (a[0] * ((double)c[1] - b[1]) + b[0] * ((double)a[1] - c[1]) + c[0] * ((double)b[1] - a[1]));
}

static bool point_in_triangle2d(const float* p0, const float* p1, const float* p2, const float* pp) {
    const float v0[2] = {p1[0] - p0[0], p1[1] - p0[1]};
    const float v1[2] = {p2[0] - p0[0], p2[1] - p0[1]};
    const float v2[2] = {pp[0] - p0[0], pp[1] - p0[1]};
    double dot00 = v0[0] * v0[0] + v0[1] * v0[1];  // aiVector2D operator* (float), then double
    const double dot01 = v0[0] * v1[0] + v0[1] * v1[1];
    const double dot02 = v0[0] * v2[0] + v0[1] * v2[1];
    double dot11 = v1[0] * v1[0] + v1[1] * v1[1];
    const double dot12 = v1[0] * v2[0] + v1[1] * v2[1];
    const double inv_denom = 1 / (dot00 * dot11 - dot01 * dot01);
    dot11 = (dot11 * dot02 - dot01 * dot12) * inv_denom;
    dot00 = (dot00 * dot12 - dot01 * dot02) * inv_denom;
    return (dot11 > 0) && (dot00 > 0) && (dot11 + dot00 < 1);
}

static void ear_cut(const std::vector<v3>& verts, const std::vector<uint32_t>& idx,
                    std::vector<std::array<uint32_t, 3>>& tris) {
    const int max = (int)idx.size();
    // NewellNormal<3,3,3> (PolyTools.h): the first two points repeated at the end
    std::vector<v3> p(max + 2);
    for (int k = 0; k < max; ++k) p[k] = verts[idx[k]];
    p[max] = p[0];
    p[max + 1] = p[1];
    float sum_xy = 0.0f, sum_yz = 0.0f, sum_zx = 0.0f;
    for (int k = 0; k < max; ++k) {
        sum_xy += p[k + 1].x * (p[k + 2].y - p[k].y);
        sum_yz += p[k + 1].y * (p[k + 2].z - p[k].z);
        sum_zx += p[k + 1].z * (p[k + 2].x - p[k].x);
    }
    const v3 n{sum_yz, sum_zx, sum_xy};
    const float ax = n.x > 0 ? n.x : -n.x, ay = n.y > 0 ? n.y : -n.y, az = n.z > 0 ? n.z : -n.z;
    int ac = 0, bc = 1;  // no z: project to xy
    float inv = n.z;
    if (ax > ay) {
        if (ax > az) {  // no x: yz
            ac = 1;
            bc = 2;
            inv = n.x;
        }
    } else if (ay > az) {  // no y: zx
        ac = 2;
        bc = 0;
        inv = n.y;
    }
    if (inv < 0.0f) std::swap(ac, bc);
    auto comp = [](const v3& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); };
    std::vector<std::array<float, 2>> t(max);
    std::vector<char> done(max, 0);
    for (int k = 0; k < max; ++k) t[k] = {comp(verts[idx[k]], ac), comp(verts[idx[k]], bc)};
    int num = max, ear = 0, prev = num - 1, next = 0;
    while (num > 3) {
        int num_found = 0;
        for (ear = next;; prev = ear, ear = next) {
            // break after two loops without a positive match
            for (next = ear + 1; done[(next >= max ? next = 0 : next)]; ++next) {
            }
            if (next < ear) {
                if (++num_found == 2) break;
            }
            const float *p1 = t[ear].data(), *p0 = t[prev].data(), *p2 = t[next].data();
            // a convex corner: OnLeftSideOfLine2D(p0, p2, p1) is GetArea2D(p0, p1, p2) > 0
            if (area2d(p0, p1, p2) > 0) continue;
            int k = 0;
            for (; k < max; ++k) {
                const float* v = t[k].data();
                auto same = [](const float* a, const float* b) { return a[0] == b[0] && a[1] == b[1]; };
                if (!same(v, p1) && !same(v, p2) && !same(v, p0) && point_in_triangle2d(p0, p1, p2, v)) break;
            }
            if (k != max) continue;
            break;  // an ear
        }
        if (num_found == 2) {  // no ear: not a simple polygon (Assimp logs and stops)
            num = 0;
            break;
        }
        tris.push_back({idx[prev], idx[ear], idx[next]});
        done[ear] = 1;
        --num;
    }
    if (num > 0) {
        int k = 0;
        while (done[k]) ++k;
        const int a = k++;
        while (done[k]) ++k;
        const int b = k++;
        while (done[k]) ++k;
        tris.push_back({idx[a], idx[b], idx[k]});
    }
}

// createTopology + createVertexArray + TriangulateProcess + GenFaceNormalsProcess
static bool build_ai_mesh(const ObjModel& m, const ObjMesh& om, AiMesh& out, bool normals_div) {
    if (om.faces.empty()) return false;
    out.material = (om.material >= 0) ? om.material : 0;
    out.has_normals = om.has_normals;
    std::vector<std::vector<uint32_t>> polys;
    uint32_t idx = 0;
    for (const Face& f : om.faces) {
        std::vector<uint32_t> poly;
        for (size_t c = 0; c < f.v.size(); ++c) {
            if (f.v[c] < 0 || f.v[c] >= (int)m.vertices.size()) throw std::runtime_error("OBJ: vertex index out of range");
            out.verts.push_back(m.vertices[f.v[c]]);
            v3 n{0.0f, 0.0f, 0.0f};
            if (om.has_normals && !m.normals.empty() && c < f.vn.size() && f.vn[c] >= 0 && f.vn[c] < (int)m.normals.size())
                n = m.normals[f.vn[c]];
            out.norms.push_back(n);
            v3 uv{0.0f, 0.0f, 0.0f};
            if (!m.texcoords.empty() && c < f.vt.size() && f.vt[c] >= 0 && f.vt[c] < (int)m.texcoords.size())
                uv = m.texcoords[f.vt[c]];
            out.uvs.push_back(uv);
            poly.push_back(idx++);
        }
        polys.push_back(poly);
    }
    // TriangulateProcess::TriangulateMesh
    for (const auto& poly : polys) {
        const size_t n = poly.size();
        if (n < 3) continue;  // points/lines carry no triangles
        if (n == 3) {
            out.tris.push_back({poly[0], poly[1], poly[2]});
        } else if (n == 4) {
            unsigned start = 0;
            for (unsigned i = 0; i < 4; ++i) {
                const v3 v0 = out.verts[poly[(i + 3) % 4]];
                const v3 v1 = out.verts[poly[(i + 2) % 4]];
                const v3 v2 = out.verts[poly[(i + 1) % 4]];
                const v3 v = out.verts[poly[i]];
                v3 left = ai_normalize(v0 - v);
                v3 diag = ai_normalize(v1 - v);
                v3 right = ai_normalize(v2 - v);
                const float angle = std::acos(ai_dot(left, diag)) + std::acos(ai_dot(right, diag));
                if (angle > 3.1415926538f) {
                    start = i;
                    break;
                }
            }
            out.tris.push_back({poly[start], poly[(start + 1) % 4], poly[(start + 2) % 4]});
            out.tris.push_back({poly[start], poly[(start + 2) % 4], poly[(start + 3) % 4]});
        } else {
            ear_cut(out.verts, poly, out.tris);
        }
    }
    // GenFaceNormalsProcess (only meshes without normals)
    if (!out.has_normals) {
        for (const auto& t : out.tris) {
            const v3 p1 = out.verts[t[0]], p2 = out.verts[t[1]], p3 = out.verts[t[2]];
            const v3 nor = ai_normalize_safe(ai_cross(p2 - p1, p3 - p1), normals_div);
            for (int c = 0; c < 3; ++c) out.norms[t[c]] = nor;
        }
        out.has_normals = true;
    }
    return true;
}

// glm::mat4 * glm::vec4 (type_mat4x4.inl): (m0*v0 + m1*v1) + (m2*v2 + m3*v3), column-major
struct M4 {
    float m[4][4];
};
static M4 m4_identity() {
    M4 r;
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) r.m[c][w] = (c == w) ? 1.0f : 0.0f;
    return r;
}
static M4 m4_mul(const M4& a, const M4& b) {
    M4 r;
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < 4; ++w) {
            const float mul0 = a.m[0][w] * b.m[c][0];
            const float mul1 = a.m[1][w] * b.m[c][1];
            const float mul2 = a.m[2][w] * b.m[c][2];
            const float mul3 = a.m[3][w] * b.m[c][3];
            r.m[c][w] = (mul0 + mul1) + (mul2 + mul3);
        }
    return r;
}
static v3 m4_point(const M4& a, v3 p) {
    float out[3];
    for (int w = 0; w < 3; ++w) {
        const float mul0 = a.m[0][w] * p.x;
        const float mul1 = a.m[1][w] * p.y;
        const float mul2 = a.m[2][w] * p.z;
        const float mul3 = a.m[3][w] * 1.0f;
        out[w] = (mul0 + mul1) + (mul2 + mul3);
    }
    return v3{out[0], out[1], out[2]};
}
// glm::inverseTranspose(mat3) (gtc/matrix_inverse.inl)
static m3 inverse_transpose(const M4& a) {
    float m[3][3];
    for (int c = 0; c < 3; ++c)
        for (int w = 0; w < 3; ++w) m[c][w] = a.m[c][w];
    const float det = +m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
                      m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                      m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    m3 r;
    r.m[0][0] = +(m[1][1] * m[2][2] - m[2][1] * m[1][2]);
    r.m[0][1] = -(m[1][0] * m[2][2] - m[2][0] * m[1][2]);
    r.m[0][2] = +(m[1][0] * m[2][1] - m[2][0] * m[1][1]);
    r.m[1][0] = -(m[0][1] * m[2][2] - m[2][1] * m[0][2]);
    r.m[1][1] = +(m[0][0] * m[2][2] - m[2][0] * m[0][2]);
    r.m[1][2] = -(m[0][0] * m[2][1] - m[2][0] * m[0][1]);
    r.m[2][0] = +(m[0][1] * m[1][2] - m[1][1] * m[0][2]);
    r.m[2][1] = -(m[0][0] * m[1][2] - m[1][0] * m[0][2]);
    r.m[2][2] = +(m[0][0] * m[1][1] - m[1][0] * m[0][1]);
    for (int c = 0; c < 3; ++c)
        for (int w = 0; w < 3; ++w) r.m[c][w] = r.m[c][w] / det;
    return r;
}

}  // namespace

std::vector<Mesh> load_obj(const std::string& path, bool normalize, int compat) {
    const bool shininess_x4 = (compat & RT_ASSIMP3_SHININESS_X4) != 0, normals_div = (compat & RT_ASSIMP3_NORMALS_DIV) != 0;
    ObjModel model;
    parse_obj(model, path);
    const std::string dir = path.substr(0, path.find_last_of("/\\") + 1);

    // ObjFileImporter::CreateDataFromImport: one root child per object, meshes with faces only
    struct Node {
        std::vector<int> meshes;  // indices into ai_meshes
    };
    std::vector<AiMesh> ai_meshes;
    std::vector<Node> nodes;
    for (const ObjObject& o : model.objects) {
        Node nd;
        for (int mi : o.meshes) {
            AiMesh am;
            if (build_ai_mesh(model, model.meshes[mi], am, normals_div)) {
                ai_meshes.push_back(std::move(am));
                nd.meshes.push_back((int)ai_meshes.size() - 1);
            }
        }
        nodes.push_back(nd);
    }
    if (ai_meshes.empty()) throw std::runtime_error("Assimp failed to load mesh file " + path);

    // reference LIFO walk (src/mesh.cpp:77-154): the root (identity, no meshes) then its children
    // pushed in order and popped in reverse.  matrix = I*I (root), child: matrix *= I.
    const M4 I = m4_identity();
    const M4 root_matrix = m4_mul(I, I);
    const M4 child_matrix = m4_mul(root_matrix, I);
    const m3 normal_matrix = inverse_transpose(child_matrix);

    std::vector<Mesh> out;
    for (int ni = (int)nodes.size() - 1; ni >= 0; --ni) {
        for (int ami : nodes[ni].meshes) {
            const AiMesh& am = ai_meshes[ami];
            Mesh mesh;
            mesh.triangles = am.tris;
            mesh.vertices.reserve(am.verts.size());
            for (size_t j = 0; j < am.verts.size(); ++j) {
                Vertex v;
                v.p = m4_point(child_matrix, am.verts[j]);
                v.n = mul(normal_matrix, am.norms[j]);
                v.uv = v2{am.uvs[j].x, am.uvs[j].y};
                mesh.vertices.push_back(v);
            }
            const ObjMaterial& om = model.materials[am.material];
            mesh.material.kd = om.diffuse;
            mesh.material.ks = om.specular;
            mesh.material.shininess = shininess_x4 ? om.shineness * 4.0f : om.shineness;
            mesh.material.transparency = om.alpha;
            if (!om.texture.empty()) {
                mesh.material.has_texture = true;
                mesh.material.texture_path = dir + om.texture;
            }
            out.push_back(std::move(mesh));
        }
    }

    if (normalize) {
        // centerAndScaleToUnitMesh (src/mesh.cpp:164-188)
        v3 acc{0.0f, 0.0f, 0.0f};
        size_t count = 0;
        for (const Mesh& m : out)
            for (const Vertex& v : m.vertices) {
                acc = acc + v.p;
                ++count;
            }
        const v3 center = acc / static_cast<float>(count);
        float maxD = 0.0f;
        for (const Mesh& m : out)
            for (const Vertex& v : m.vertices) {
                const float d = length(v.p - center);
                maxD = (d < maxD) ? maxD : d;  // std::max(length, maxD)
            }
        for (Mesh& m : out)
            for (Vertex& v : m.vertices) v.p = (v.p - center) / maxD;
    }
    return out;
}

}  // namespace rt
