// bvh_driver.cpp -- CPU sanitizer build only (tools/sanitize): the host acceleration-structure builders
// (bvh_build.cpp: the reference's depth-4 median BVH, binned-SAH BVH2, BVH8 collapse, on the threaded
// host pool) over every reference scene, the dragon proxy at two tessellations and random triangle soups
// (degenerate, duplicated and axis-aligned triangles included), with structural checks: every triangle
// in exactly one leaf / record slot, depths within the traversal stacks.  Then malformed inputs for the
// parsers: every reference PNG truncated at many lengths and with flipped bytes (rt_decode_png), and every
// reference OBJ/MTL truncated and with garbage lines (rt_scene_load_obj) -- each must return a status,
// never read or write out of bounds.  Built and run with -fsanitize=address,undefined by
// tools/sanitize/run.sh.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "../../include/rt_amd.h"
#include "../../raytracer-group27_amd/csrc/bvh_build.h"
#include "../../raytracer-group27_amd/csrc/rt_internal.h"

using namespace rt;

static int fails = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            std::fprintf(stderr, "FAIL %s: ", #c);     \
            std::fprintf(stderr, __VA_ARGS__);         \
            std::fprintf(stderr, "\n");                \
            ++fails;                                   \
        }                                              \
    } while (0)

static void check_structures(const char* what, const float* pos, int ntri, const float* sph, int nsph) {
    const RefBvh ref = build_ref_bvh(pos, ntri, sph, nsph, 4);
    CHECK(ref.nodes.size() <= RT_MAX_REF_NODES, "%s: %zu reference nodes", what, ref.nodes.size());
    std::vector<int> seen(ntri + nsph, 0);
    for (const RefNode& n : ref.nodes)
        if (n.is_leaf)
            for (size_t k = 0; k < n.children.size(); ++k)  // leaf objects: triangle index, or sphere index
                seen[n.is_triangle[k] ? n.children[k] : ntri + n.children[k]]++;
    for (int i = 0; i < ntri + nsph; ++i) CHECK(seen[i] == 1, "%s: object %d in %d reference leaves", what, i, seen[i]);
    CHECK((int)ref.tri_key.size() == ntri && (int)ref.tri_leaf.size() == ntri, "%s: reference keys", what);
    if (ntri == 0) return;
    float m = 8.0f;
    for (size_t i = 0; i < (size_t)ntri * 9; ++i) m = std::fmax(m, std::fabs(pos[i]));
    const Bvh2 b2 = build_bvh2(pos, ntri, std::ldexp(m, -16), 4);
    CHECK(b2.max_depth + 2 < RT_STACK_SIZE, "%s: BVH2 depth %d", what, b2.max_depth);
    std::vector<int> rec(ntri, 0);
    for (int t : b2.order) rec[t]++;
    for (int i = 0; i < ntri; ++i) CHECK(rec[i] == 1, "%s: triangle %d in %d BVH2 records", what, i, rec[i]);
    const Bvh8 b8 = build_bvh8(b2, 8);
    CHECK((int)b8.order.size() == ntri, "%s: %zu BVH8 records", what, b8.order.size());
    std::vector<int> rec8(ntri, 0);
    for (int t : b8.order) rec8[t]++;
    for (int i = 0; i < ntri; ++i) CHECK(rec8[i] == 1, "%s: triangle %d in %d BVH8 records", what, i, rec8[i]);
    CHECK(b8.nodes.size() % 32 == 0, "%s: BVH8 node words", what);
    std::printf("%-34s %8d triangles  ref %2zu nodes  BVH2 %7zu nodes depth %2d  BVH8 %6zu nodes depth %d\n", what,
                ntri, ref.nodes.size(), b2.nodes.size(), b2.max_depth, b8.nodes.size() / 32, b8.max_depth);
}

static void scene_file(const std::string& dir, const char* obj, bool normalize) {
    rt_scene* s = nullptr;
    CHECK(rt_scene_new(&s) == RT_OK, "rt_scene_new");
    const std::string path = dir + "/" + obj;
    if (rt_scene_load_obj(s, path.c_str(), normalize ? 1 : 0, 0) != RT_OK) {
        char e[512];
        rt_last_error(e, sizeof e);
        CHECK(false, "%s: %s", obj, e);
        rt_scene_free(s);
        return;
    }
    rt_scene_desc d{};
    rt_scene_desc_get(s, &d);
    std::vector<float> sph;
    for (int i = 0; i < d.num_spheres; ++i) {
        for (int k = 0; k < 3; ++k) sph.push_back(d.spheres[i].center[k]);
        sph.push_back(d.spheres[i].radius);
    }
    check_structures(obj, d.positions, d.num_triangles, sph.data(), d.num_spheres);
    rt_scene_free(s);
}

static std::vector<uint8_t> read_file(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static int png_try(const std::vector<uint8_t>& d) {
    int w = 0, h = 0, ch = 0;
    int rc = rt_decode_png(d.data(), (long)d.size(), &w, &h, &ch, nullptr, 0);
    if (rc != RT_OK) return rc;
    if ((long long)w * h > (1ll << 26)) return RT_ERR_INVALID;
    std::vector<uint8_t> rgb((size_t)w * h * 3);
    return rt_decode_png(d.data(), (long)d.size(), &w, &h, &ch, rgb.data(), (long)rgb.size());
}

static void fuzz_png(const std::string& dir, std::mt19937& rng) {
    int ok = 0, rejected = 0;
    for (const char* f : {"default.png", "bookshelf.png", "grass_tex.png", "green_wool.png", "stone_bricks.png"}) {
        const std::vector<uint8_t> d = read_file(dir + "/" + f);
        CHECK(!d.empty(), "%s missing", f);
        CHECK(png_try(d) == RT_OK, "%s does not decode", f);
        for (size_t n = 0; n < d.size(); n += 1 + d.size() / 97) {  // truncations
            std::vector<uint8_t> t(d.begin(), d.begin() + n);
            (png_try(t) == RT_OK ? ok : rejected)++;
        }
        for (int k = 0; k < 200; ++k) {  // random byte flips (headers, chunk lengths, zlib stream)
            std::vector<uint8_t> t = d;
            const int nflip = 1 + (int)(rng() % 4);
            for (int j = 0; j < nflip; ++j) t[rng() % t.size()] ^= (uint8_t)(1u << (rng() % 8));
            (png_try(t) == RT_OK ? ok : rejected)++;
        }
    }
    std::printf("PNG fuzz: %d decoded, %d rejected with a status\n", ok, rejected);
}

static void fuzz_obj(const std::string& dir, const std::string& tmp, std::mt19937& rng) {
    int ok = 0, rejected = 0;
    const char* junk[] = {"f 1 2\n", "f 0 0 0\n", "f -99 1 2\n", "v 1e39 nan inf\n", "vn\n", "vt 0.5\n",
                          "f 1/2/3 4//5 6/7\n", "usemtl nowhere\n", "mtllib missing.mtl\n", "f 999999 1 2\n",
                          "o \n", "g\n", "v 1 2\n", "f 1 2 3 4 5 6 7 8 9 10 11 12\n", "\x01\xff\n"};
    for (const char* f : {"cube.obj", "CornellBox-Mirror-Rotated.obj", "monkey-rotated.obj", "tr_def.obj"}) {
        const std::vector<uint8_t> d = read_file(dir + "/" + f);
        for (int k = 0; k < 60; ++k) {
            std::string text(d.begin(), d.begin() + (k < 30 ? (size_t)(rng() % (d.size() + 1)) : d.size()));
            if (k >= 20) {  // garbage lines inserted at random line starts
                for (int j = 0; j < 3; ++j) {
                    size_t at = rng() % (text.size() + 1);
                    at = text.rfind('\n', at);
                    at = at == std::string::npos ? 0 : at + 1;
                    text.insert(at, junk[rng() % (sizeof(junk) / sizeof(junk[0]))]);
                }
            }
            const std::string p = tmp + "/fuzz.obj";
            std::ofstream(p, std::ios::binary) << text;
            // the reference's MTL files next to it (mtllib names are relative)
            for (const char* m : {"cube.mtl", "CornellBox-Mirror-Rotated.mtl", "monkey-rotated.mtl", "tr_def.mtl"}) {
                const std::vector<uint8_t> md = read_file(dir + "/" + m);
                std::ofstream(tmp + "/" + m, std::ios::binary).write((const char*)md.data(), (std::streamsize)md.size());
            }
            rt_scene* s = nullptr;
            rt_scene_new(&s);
            const int rc = rt_scene_load_obj(s, p.c_str(), k % 2, 0);
            if (rc == RT_OK) {
                rt_scene_desc dd{};
                rt_scene_desc_get(s, &dd);
                if (dd.num_triangles > 0 && dd.num_triangles < 200000) {
                    std::vector<float> sph;
                    check_structures("fuzzed obj", dd.positions, dd.num_triangles, sph.data(), 0);
                }
                ++ok;
            } else {
                ++rejected;
            }
            rt_scene_free(s);
        }
    }
    std::printf("OBJ fuzz: %d loaded, %d rejected with a status\n", ok, rejected);
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: bvh_driver <scene dir> <tmp dir>\n");
        return 2;
    }
    const std::string dir = argv[1], tmp = argv[2];
    for (const char* f : {"cube.obj", "monkey-rotated.obj", "CornellBox-Mirror-Rotated.obj", "teapot.obj", "tr_def.obj"})
        scene_file(dir, f, true);
    for (int uv : {0, 1}) {  // the dragon proxy, coarse and a 200x80 tessellation
        const std::string p = tmp + "/san_proxy_" + std::to_string(uv) + ".obj";
        CHECK(rt_write_dragon_proxy(p.c_str(), uv ? 200 : 40, uv ? 80 : 16) == RT_OK, "proxy");
        std::string base = p.substr(p.rfind('/') + 1);
        scene_file(tmp, base.c_str(), true);
    }
    std::mt19937 rng(12345);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    for (int n : {1, 2, 3, 17, 1000, 40000}) {
        std::vector<float> pos((size_t)n * 9);
        for (int t = 0; t < n; ++t) {
            const int kind = t % 7;
            for (int c = 0; c < 3; ++c)
                for (int k = 0; k < 3; ++k) {
                    float v = U(rng);
                    if (kind == 1) v = U(rng) * 1e-6f;                          // tiny
                    if (kind == 2 && c > 0) v = pos[(size_t)t * 9 + k];         // degenerate (3 equal corners)
                    if (kind == 3 && k == 2) v = 0.25f;                         // axis-aligned (flat box)
                    pos[(size_t)t * 9 + c * 3 + k] = v;
                }
            if (kind == 4 && t > 0)  // duplicate of the previous triangle
                for (int i = 0; i < 9; ++i) pos[(size_t)t * 9 + i] = pos[(size_t)(t - 1) * 9 + i];
        }
        const float sph[8] = {0.1f, 0.2f, 0.3f, 0.5f, -0.4f, 0.0f, 0.4f, 0.25f};
        check_structures(("random soup " + std::to_string(n)).c_str(), pos.data(), n, sph, n % 3 == 0 ? 2 : 0);
    }
    fuzz_png(dir, rng);
    fuzz_obj(dir, tmp, rng);
    std::printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
    return fails ? 1 : 0;
}
