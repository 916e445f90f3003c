// ORACLE -- test infrastructure, not product code.
//
// CPU restatement of the reference hot path of catalinlup/RayTracer-Group27 (paths relative to
// the reference root).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
// may load this library, and only as the checker / the timed CPU baseline; the product path
// (raytracer-group27_amd/librt_amd.so) never links or calls it.
//
// It is written independently of the HIP product (own vector type, own BVH, recursion
// instead of an explicit stack) and follows the reference call structure:
//   renderRayTracing            src/main.cpp:340-400 (pixel loop, AA, getPixelRays :309-335)
//   Trackball::generateRay      framework/src/trackball.cpp:65-68, 87-98
//   getFinalColor / calcColor   src/main.cpp:112-301
//   BVH::intersect              src/bounding_volume_hierarchy.cpp:49-78 (brute force)
//   BVH build + intersectBVH    src/bounding_volume_hierarchy.cpp:80-448 (max_level 4, h:67)
//   primitive tests             src/ray_tracing.cpp:15-316
//   cansee + light gathering    src/shadow.cpp:32-321
// Arithmetic follows glm 0.9.9.8's non-SIMD op order (dot = (x+y)+z, normalize = v*(1/sqrt),
// min/max as ternaries) and C++ promotions (std::pow(float,int) -> double).
//
// PARITY STATUS: pinned to the reference's render.bmp (the only reference-held output): with the
// Trackball state tools/fit_render_bmp.py recovers and the bloom the file was written with, this
// restatement + ref_post.cpp reproduce 99.8 % of its pixels byte for byte
// (tests/test_render_bmp_pin.py).  The reference ships no tests, golden vectors or
// fixtures for this path, and it cannot be built here without stand-ins for
// glm, gsl-lite, Assimp, GLFW and ImGui, which the task forbids.
// Where the reference is undefined (uninitialised barycentrics when barycentricCoordinates
// returns false, src/ray_tracing.cpp:147-157) this restatement uses the "unthresholded"
// definition, shared with the GPU path.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>
#include <array>
#include <queue>
#include <utility>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/rt_amd.h"

namespace oracle {

struct V3 {
    float x = 0, y = 0, z = 0;
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit V3(float s) : x(s), y(s), z(s) {}
    static V3 of(const float* p) { return V3(p[0], p[1], p[2]); }
};
static inline V3 operator+(const V3& a, const V3& b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(const V3& a, const V3& b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator-(const V3& a) { return V3(-a.x, -a.y, -a.z); }
static inline V3 operator*(const V3& a, const V3& b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 operator*(const V3& a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline V3 operator*(float s, const V3& a) { return V3(s * a.x, s * a.y, s * a.z); }
static inline V3 operator/(const V3& a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline V3& operator+=(V3& a, const V3& b) { return a = a + b; }
static inline float vdot(const V3& a, const V3& b) {
    V3 m = a * b;
    return m.x + m.y + m.z;
}
static inline V3 vcross(const V3& a, const V3& b) {
    return V3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline float vlength(const V3& v) { return std::sqrt(vdot(v, v)); }
static inline V3 vnormalize(const V3& v) { return v * (1.0f / std::sqrt(vdot(v, v))); }
static inline V3 vreflect(const V3& i, const V3& n) { return i - n * vdot(n, i) * 2.0f; }
static inline float fmin_g(float a, float b) { return (b < a) ? b : a; }  // glm::min / std::min
static inline float fmax_g(float a, float b) { return (a < b) ? b : a; }  // glm::max / std::max

struct Mat {
    V3 kd, ks;
    float shininess = 1.0f;
    float transparency = 1.0f;
    int texture = -1;  // kdTexture: index into Scene::images
};

// ---------------------------------------------------------------- Image (src/image.cpp)
// The reference's texture: pixels from the stb RGB buffer (stepping by the file's channel
// count, :57-59), the mip chain of square power-of-two images (:408-452), getPixel and its
// filters (:77-360), level choice (:500-540).
struct Image {
    int w = 0, h = 0;
    bool mip = false;
    std::vector<std::vector<V3>> levels;  // _mipmap[0] = m_pixels

    Image(const rt_texture& t) : w(t.width), h(t.height) {
        const size_t nbytes = (size_t)w * h * 3;
        std::vector<V3> px;
        for (size_t i = 0; i < (size_t)w * h * t.channels; i += t.channels) {
            auto at = [&](size_t j) { return j < nbytes ? (float)t.rgb[j] : 0.0f; };
            px.emplace_back(at(i) / 255.0f, at(i + 1) / 255.0f, at(i + 2) / 255.0f);
        }
        levels.push_back(px);
        mip = ((h & (h - 1)) == 0) && ((w & (w - 1)) == 0) && (w == h);
        if (!mip) return;
        for (int k = w; k > 1; k /= 2) {
            const int r = k / 2;
            const std::vector<V3>& o = levels.back();
            std::vector<V3> red((size_t)r * r);
            for (int x = 0, rx = 0; x + 1 < k && rx < r; x += 2, rx++)
                for (int y = 0, ry = 0; y + 1 < k && ry < r; y += 2, ry++)
                    red[(size_t)ry * r + rx] = 0.25f * (o[(size_t)y * k + x] + o[(size_t)(y + 1) * k + x] +
                                                        o[(size_t)y * k + x + 1] + o[(size_t)(y + 1) * k + x + 1]);
            levels.push_back(red);
        }
    }
    int lw(int l) const { return w >> l; }
    int lh(int l) const { return h >> l; }
    static bool out(float c) { return c < 0 || c > 1; }
    static float wrap(float c, int rule) {
        if (rule == RT_OOB_CLAMP) return c > 1 ? 1.0f : (c < 0 ? 0.0f : c);
        if (rule == RT_OOB_REPEAT && out(c)) return c - std::floor(c);
        return c;
    }
    void to_image(float u, float v, int l, float& x, float& y) const {
        x = u * (unsigned)(lw(l) - 1);
        y = (1.0f - v) * (unsigned)(lh(l) - 1);
    }
    V3 nearest(float fx, float fy, int l) const {
        unsigned x = (unsigned)std::round(fx), y = (unsigned)std::round(fy);
        if (x >= (unsigned)lw(l)) x = lw(l) - 1;
        if (y >= (unsigned)lh(l)) y = lh(l) - 1;
        return levels[l][(size_t)y * lw(l) + x];
    }
    static V3 lerp(float lo, float hi, const V3& cl, const V3& ch, float p) {
        if (std::fabs(hi - lo) < 1e-6) return cl;
        const float c = (p - lo) / (hi - lo);
        return (1 - c) * cl + c * ch;
    }
    V3 bilinear(float fx, float fy, int l) const {
        const float x0 = std::floor(fx), x1 = std::ceil(fx), y0 = std::floor(fy), y1 = std::ceil(fy);
        auto at = [&](float x, float y) { return levels[l][(size_t)(unsigned)y * lw(l) + (unsigned)x]; };
        const V3 lo = lerp(x0, x1, at(x0, y0), at(x1, y0), fx);
        const V3 hi = lerp(x0, x1, at(x0, y1), at(x1, y1), fx);
        return lerp(y0, y1, lo, hi, fy);
    }
    int nlevels() const { return (int)levels.size(); }
    V3 get_pixel(float u, float v, float lod, const rt_params& P) const {
        const V3 border = V3::of(P.border_color);
        if (P.out_of_bounds_x == RT_OOB_BORDER && out(u)) return border;
        if (P.out_of_bounds_y == RT_OOB_BORDER && out(v)) return border;
        const float iu = wrap(u, P.out_of_bounds_x), iv = wrap(v, P.out_of_bounds_y);
        float x, y;
        if (P.texture_filtering == RT_TEX_NEAREST || P.texture_filtering == RT_TEX_BILINEAR) {
            to_image(iu, iv, 0, x, y);
            return P.texture_filtering == RT_TEX_NEAREST ? nearest(x, y, 0) : bilinear(x, y, 0);
        }
        // getBestLevelMipmap (:495-529): the floor level is not clamped from above; a level at or
        // past the chain fails getWidthHeightForLevel (:478-486), so trilinear returns black
        // (:334-337) and the nearest-level modes white (:270-274, :294-298).  The level is tested
        // as a float first: (int) of a huge or infinite floor(lod) would be undefined.
        if (P.texture_filtering == RT_TEX_TRILINEAR) {
            if (!mip) return V3(0.0f);
            const float flo = fmax_g(0.0f, std::floor(lod));
            if (!(flo < (float)nlevels())) return V3(0.0f);
            const int hi = (int)fmin_g(nlevels() - 1.0f, std::ceil(lod));
            const int lo = (int)flo;
            float xl, yl, xh, yh;
            to_image(iu, iv, lo, xl, yl);
            to_image(iu, iv, hi, xh, yh);
            return lerp((float)lo, (float)hi, bilinear(xl, yl, lo), bilinear(xh, yh, hi), lod);
        }
        if (!mip) return V3(1.0f);
        float fbest;
        if (lod - std::floor(lod) < std::ceil(lod) - lod)
            fbest = fmax_g(0.0f, std::floor(lod));
        else
            fbest = fmin_g(nlevels() - 1.0f, std::ceil(lod));
        if (!(fbest < (float)nlevels())) return V3(1.0f);
        const unsigned best = (unsigned)(int)fbest;
        to_image(iu, iv, (int)best, x, y);
        return P.texture_filtering == RT_TEX_MIP_NEAREST ? nearest(x, y, (int)best) : bilinear(x, y, (int)best);
    }
};
struct Vert {
    V3 p, n;
    float u = 0, v = 0;
};
struct Sph {
    V3 center;
    float radius = 1.0f;
    Mat mat;
};
struct Ray {
    V3 origin;
    V3 direction{0.0f, 0.0f, -1.0f};
    float t = FLT_MAX;
};
struct Hit {
    V3 normal, hitPoint;
    int material_index = 0;
    Mat sphere_material;
    float u = 0, v = 0;
    bool is_triangle = false;
    int prim = -1;
    bool ub = false;  // barycentricCoordinates returned false for this hit (src/ray_tracing.cpp:281-295)
    Mat& material(std::vector<Mat>& mats) { return is_triangle ? mats[material_index] : sphere_material; }
};
struct Light {  // what getPointLights & co. return (src/shadow.h:14-20)
    V3 color;
    float intensity, cosL, cosS;
};

struct Node {
    bool leaf = false;
    std::vector<int> kids;
    std::vector<char> tri;
    V3 lo, hi;
};

struct Scene {
    std::vector<std::array<Vert, 3>> tris;
    std::vector<int> tri_mesh;
    std::vector<Mat> mats;
    std::vector<Sph> spheres;
    std::vector<rt_point_light> pls;
    std::vector<rt_spherical_light> sls;
    std::vector<rt_spot_light> spots;
    std::vector<rt_plane_light> planes;
    std::vector<Node> nodes;
    std::vector<Image> images;
};

// ---------------------------------------------------------------- primitives (ray_tracing.cpp)
// isZero/isEqual (src/ray_tracing.cpp:15-24) only gate barycentricCoordinates' return value,
// which the "unthresholded" definition below does not consult.

static bool point_in_triangle(const V3& a, const V3& b, const V3& c, const V3& n, const V3& p) {
    const bool e0 = vdot(vcross(p - a, c - a), n) >= 0;
    const bool e1 = vdot(vcross(p - c, b - c), n) >= 0;
    const bool e2 = vdot(vcross(p - b, a - b), n) >= 0;
    return (e0 && e1 && e2) || (!e0 && !e1 && !e2);
}

static void plane_of(const V3& a, const V3& b, const V3& c, V3& n, float& D) {
    n = vnormalize(vcross(a - c, b - c));
    D = vdot(n, a);
}

static bool hit_plane(const V3& n, float D, Ray& r) {
    const float nd = vdot(vnormalize(r.direction), n);
    if (nd == 0) return false;
    const float t = (D - vdot(r.origin, n)) / nd;
    if (!(t >= 0)) return false;
    if (!(t < r.t)) return false;
    r.t = t;
    return true;
}

static bool hit_triangle_flat(const V3& a, const V3& b, const V3& c, Ray& r, Hit& h, int mat) {
    const float keep = r.t;
    V3 n;
    float D;
    plane_of(a, b, c, n, D);
    if (!hit_plane(n, D, r)) return false;
    const V3 p = r.origin + r.direction * r.t;
    if (!point_in_triangle(a, b, c, n, p)) {
        r.t = keep;
        return false;
    }
    h.normal = n;
    h.hitPoint = p;
    h.material_index = mat;
    return true;
}

static float par_area(const V3& a, const V3& b, const V3& c) { return vlength(vcross(b - a, c - a)); }

// barycentricCoordinates with the "unthresholded" definition: the thresholds only decide
// whether the reference's result is defined; the coordinates are the same formula either way.
static V3 barycentric(const V3& a, const V3& b, const V3& c, const V3& p) {
    const float A = par_area(a, b, c);
    if (!(A > 0.0f)) return V3(0.0f);
    return V3(par_area(p, b, c) / A, par_area(a, p, c) / A, par_area(a, b, p) / A);
}

static bool hit_triangle(const Vert& a, const Vert& b, const Vert& c, Ray& r, Hit& h, int mat, int prim) {
    const float before = r.t;
    if (!hit_triangle_flat(a.p, b.p, c.p, r, h, mat)) return false;
    if (r.t < before) {
        h.is_triangle = true;
        h.prim = prim;
    }
    const V3 bc = barycentric(a.p, b.p, c.p, h.hitPoint);
    const V3 face = h.normal;
    // the reference's own checks (isZero: |x| < 1e-4 in double, src/ray_tracing.cpp:15-24): off the
    // plane or a parallelogram area below 1e-4 make barycentricCoordinates return false; the
    // pointInTriangle check repeats the test that accepted the hit
    h.ub = !((double)std::fabs(vdot(face, h.hitPoint - a.p)) < 1e-4) || ((double)par_area(a.p, b.p, c.p) < 1e-4);
    h.normal = a.n * bc.x + b.n * bc.y + c.n * bc.z;
    if (vdot(h.normal, face) < 0) h.normal = -h.normal;
    h.u = a.u * bc.x + b.u * bc.y + c.u * bc.z;
    h.v = a.v * bc.x + b.v * bc.y + c.v * bc.z;
    return true;
}

static bool hit_sphere(const Sph& s, Ray& r, Hit& h, int prim) {
    const V3 m = r.origin - s.center;
    const V3& d = r.direction;
    // glm::pow(float, int) == std::pow(double, double): computed in double, stored as float
    const float A = std::pow((double)d.x, 2) + std::pow((double)d.y, 2) + std::pow((double)d.z, 2);
    const float B = 2 * (d.x * m.x + d.y * m.y + d.z * m.z);
    const float C = std::pow((double)m.x, 2) + std::pow((double)m.y, 2) + std::pow((double)m.z, 2) -
                    std::pow((double)s.radius, 2);
    const float disc = std::pow((double)B, 2) - 4 * A * C;
    if (!(disc >= 0)) return false;
    float t0 = (-B + std::sqrt(disc)) / (2 * A);
    float t1 = (-B - std::sqrt(disc)) / (2 * A);
    if (t0 < 0) t0 = t1;
    if (t1 < 0) t1 = t0;
    const float tm = fmin_g(t0, t1);
    if (!(tm > 0 && tm < r.t)) return false;
    r.t = tm;
    h.hitPoint = r.origin + r.t * r.direction;
    h.normal = vnormalize(h.hitPoint - s.center);
    h.sphere_material = s.mat;
    h.is_triangle = false;
    h.prim = prim;
    h.ub = false;
    return true;
}

static bool hit_box(const V3& lo, const V3& hi, Ray& r) {
    if (lo.x == FLT_MAX && lo.y == FLT_MAX && lo.z == FLT_MAX && hi.x == -FLT_MAX && hi.y == -FLT_MAX &&
        hi.z == -FLT_MAX)
        return false;
    const V3 d = vnormalize(r.direction);
    const float ax = (lo.x - r.origin.x) / d.x, bx = (hi.x - r.origin.x) / d.x;
    const float ay = (lo.y - r.origin.y) / d.y, by = (hi.y - r.origin.y) / d.y;
    const float az = (lo.z - r.origin.z) / d.z, bz = (hi.z - r.origin.z) / d.z;
    if (r.origin.x > lo.x && r.origin.y > lo.y && r.origin.z > lo.z && r.origin.x < hi.x && r.origin.y < hi.y &&
        r.origin.z < hi.z) {
        float best = FLT_MAX;
        for (float v : {ax, bx, ay, by, az, bz})
            if (v > 0 && v < best) best = v;
        r.t = best;
        return true;
    }
    const float tin = fmax_g(fmax_g(fmin_g(ax, bx), fmin_g(ay, by)), fmin_g(az, bz));
    const float tout = fmin_g(fmin_g(fmax_g(ax, bx), fmax_g(ay, by)), fmax_g(az, bz));
    if (tin > tout || tout < 0) return false;
    r.t = tin;
    return true;
}

// ---------------------------------------------------------------- BVH (bounding_volume_hierarchy.cpp)
static void node_bounds(const Scene& sc, const std::vector<int>& ids, const std::vector<char>& tri, V3& lo, V3& hi) {
    lo = V3(FLT_MAX);
    hi = V3(-FLT_MAX);
    auto vmin = [](const V3& a, const V3& b) { return V3(fmin_g(a.x, b.x), fmin_g(a.y, b.y), fmin_g(a.z, b.z)); };
    auto vmax = [](const V3& a, const V3& b) { return V3(fmax_g(a.x, b.x), fmax_g(a.y, b.y), fmax_g(a.z, b.z)); };
    for (size_t i = 0; i < ids.size(); ++i) {
        if (tri[i]) {
            const auto& t = sc.tris[ids[i]];
            lo = vmin(vmin(lo, t[0].p), vmin(t[1].p, t[2].p));
            hi = vmax(vmax(hi, t[0].p), vmax(t[1].p, t[2].p));
        } else {
            const Sph& s = sc.spheres[ids[i]];
            const V3 a = s.center - V3(s.radius), b = s.center + V3(s.radius);
            lo = vmin(lo, vmin(a, b));
            hi = vmax(hi, vmax(a, b));
        }
    }
}

static float split_key(const Scene& sc, int id, bool tri, int level) {
    const int axis = level % 3;
    if (tri) {
        const auto& t = sc.tris[id];
        if (axis == 0) return (t[0].p.x + t[1].p.x + t[2].p.x) / 3;
        if (axis == 1) return (t[0].p.y + t[1].p.y + t[2].p.y) / 3;
        return (t[0].p.z + t[1].p.z + t[2].p.z) / 3;
    }
    const V3& c = sc.spheres[id].center;
    return axis == 0 ? c.x : (axis == 1 ? c.y : c.z);
}

static void build_bvh(Scene& sc) {
    const int max_level = 4;
    std::vector<std::vector<int>> ids;
    std::vector<std::vector<char>> kinds;
    auto make = [&](std::vector<int> i, std::vector<char> k, int level) {
        Node n;
        n.leaf = i.size() <= 1 || level >= max_level;
        node_bounds(sc, i, k, n.lo, n.hi);
        sc.nodes.push_back(n);
        ids.push_back(std::move(i));
        kinds.push_back(std::move(k));
        return (int)sc.nodes.size() - 1;
    };
    std::vector<int> all;
    std::vector<char> allk;
    for (size_t i = 0; i < sc.tris.size(); ++i) {
        all.push_back((int)i);
        allk.push_back(1);
    }
    for (size_t i = 0; i < sc.spheres.size(); ++i) {
        all.push_back((int)i);
        allk.push_back(0);
    }
    std::queue<std::pair<int, int>> work;
    work.push({make(all, allk, 0), 0});
    while (!work.empty()) {
        auto [ni, level] = work.front();
        work.pop();
        std::vector<int> cur = ids[ni];
        std::vector<char> curk = kinds[ni];
        if (sc.nodes[ni].leaf) {
            sc.nodes[ni].kids = cur;
            sc.nodes[ni].tri = curk;
            continue;
        }
        ++level;
        std::vector<std::pair<float, int>> keyed;
        for (size_t i = 0; i < cur.size(); ++i) keyed.emplace_back(split_key(sc, cur[i], curk[i] != 0, level), (int)i);
        std::sort(keyed.begin(), keyed.end());
        std::vector<int> li, ri;
        std::vector<char> lk, rk;
        const size_t nl = (cur.size() + 1) / 2;
        for (size_t i = 0; i < keyed.size(); ++i) {
            const int src = keyed[i].second;
            if (i < nl) {
                li.push_back(cur[src]);
                lk.push_back(curk[src]);
            } else {
                ri.push_back(cur[src]);
                rk.push_back(curk[src]);
            }
        }
        if (!li.empty()) {
            const int c = make(li, lk, level);
            work.push({c, level});
            sc.nodes[ni].kids.push_back(c);
        }
        if (!ri.empty()) {
            const int c = make(ri, rk, level);
            work.push({c, level});
            sc.nodes[ni].kids.push_back(c);
        }
    }
}

static bool walk_bvh(const Scene& sc, int ni, Ray& r, Hit& h) {
    const float keep = r.t;
    const bool in = hit_box(sc.nodes[ni].lo, sc.nodes[ni].hi, r);
    r.t = keep;
    if (!in) return false;
    const Node& n = sc.nodes[ni];
    bool any = false;
    if (n.leaf) {
        for (size_t i = 0; i < n.kids.size(); ++i) {
            const int id = n.kids[i];
            if (n.tri[i]) {
                const auto& t = sc.tris[id];
                any |= hit_triangle(t[0], t[1], t[2], r, h, sc.tri_mesh[id], id);
            } else {
                any |= hit_sphere(sc.spheres[id], r, h, (int)sc.tris.size() + id);
            }
        }
        return any;
    }
    for (int c : n.kids) any |= walk_bvh(sc, c, r, h);
    return any;
}

struct Counter {
    uint64_t rays = 0;
    uint64_t ub = 0;  // shaded hits in the reference's undefined-barycentrics regime
    // glossy lobes: rand() replaced by a Philox-4x32-10 stream, counter (draw, pixel, sample, 0)
    uint32_t pix = 0, sample = 0, draws = 0;
};

// Philox-4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11), Random123's round constants and key bumps.
static void philox(uint32_t ctr[4], uint64_t seed) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int round = 0; round < 10; ++round) {
        if (round) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t m0 = (uint64_t)ctr[0] * 0xD2511F53u, m1 = (uint64_t)ctr[2] * 0xCD9E8D57u;
        const uint32_t x0 = (uint32_t)(m1 >> 32) ^ ctr[1] ^ k0, x1 = (uint32_t)m1;
        const uint32_t x2 = (uint32_t)(m0 >> 32) ^ ctr[3] ^ k1, x3 = (uint32_t)m0;
        ctr[0] = x0;
        ctr[1] = x1;
        ctr[2] = x2;
        ctr[3] = x3;
    }
}

// two uniforms in [0,1) (top 24 bits) per draw, in place of rand() / (float)RAND_MAX
static void draw_pair(Counter& cnt, uint64_t seed, float& a, float& b) {
    uint32_t c[4] = {cnt.draws++, cnt.pix, cnt.sample, 0u};
    philox(c, seed);
    a = (float)(c[0] >> 8) / 16777216.0f;
    b = (float)(c[1] >> 8) / 16777216.0f;
}

static bool intersect(const Scene& sc, Ray& r, Hit& h, bool use_bvh, Counter& cnt) {
    cnt.rays++;
    if (!use_bvh) {
        bool any = false;
        for (size_t i = 0; i < sc.tris.size(); ++i) {
            const auto& t = sc.tris[i];
            if (hit_triangle(t[0], t[1], t[2], r, h, sc.tri_mesh[i], (int)i)) any = true;
        }
        for (size_t s = 0; s < sc.spheres.size(); ++s) any |= hit_sphere(sc.spheres[s], r, h, (int)(sc.tris.size() + s));
        return any;
    }
    if (sc.nodes.empty()) return false;
    return walk_bvh(sc, 0, r, h);
}

// ---------------------------------------------------------------- lights (shadow.cpp)
static bool cansee(Scene& sc, const V3& from, const V3& to, float& intensity, Counter& cnt) {
    V3 d = to - from;
    float dist = vlength(d);
    d = vnormalize(d);
    Ray r;
    r.origin = from + 0.0005f * d;
    r.direction = d;
    Hit h;
    while (dist > 0.0005f) {
        const bool hit = intersect(sc, r, h, true, cnt);
        Mat& m = h.material(sc.mats);
        if (!hit || r.t > dist - 2 * 0.0005f) return true;
        if (m.transparency != 1.0f) {
            dist -= r.t;
            r.t = FLT_MAX;
            r.origin = h.hitPoint + 0.0005f * r.direction;
            const float c = std::abs(vdot(r.direction, h.normal));
            const float R0 = m.transparency;
            intensity *= 1 - (R0 + (1 - R0) * std::pow((double)(1 - c), 5.0));
        } else {
            return false;
        }
    }
    return true;
}

struct Rot {  // glm::mat3 column-major m[col][row]
    float m[3][3];
};
static Rot rodrigues(float angle, const V3& ax) {
    Rot C{{{0, ax.z, -ax.y}, {-ax.z, 0, ax.x}, {ax.y, -ax.x, 0}}};
    Rot CC;
    for (int c = 0; c < 3; ++c)
        for (int w = 0; w < 3; ++w) CC.m[c][w] = C.m[0][w] * C.m[c][0] + C.m[1][w] * C.m[c][1] + C.m[2][w] * C.m[c][2];
    const float s = std::sin(angle), omc = 1 - std::cos(angle);
    Rot R;
    for (int c = 0; c < 3; ++c)
        for (int w = 0; w < 3; ++w) R.m[c][w] = ((c == w ? 1.0f : 0.0f) + C.m[c][w] * s) + CC.m[c][w] * omc;
    return R;
}
static V3 rot_apply(const Rot& R, const V3& v) {
    return V3(R.m[0][0] * v.x + R.m[1][0] * v.y + R.m[2][0] * v.z, R.m[0][1] * v.x + R.m[1][1] * v.y + R.m[2][1] * v.z,
              R.m[0][2] * v.x + R.m[1][2] * v.y + R.m[2][2] * v.z);
}

static Light make_light(const V3& color, float intensity, const Hit& h, const V3& refl, const V3& lpos) {
    Light l;
    l.color = color;
    l.intensity = intensity;
    l.cosL = std::abs(vdot(vnormalize(h.normal), vnormalize(lpos - h.hitPoint)));
    l.cosS = fmax_g(0.0f, vdot(vnormalize(refl), vnormalize(lpos - h.hitPoint)));
    return l;
}

static void gather_lights(Scene& sc, const Hit& h, const V3& refl, const rt_params& P, std::vector<Light>& out,
                          Counter& cnt) {
    for (const auto& L : sc.pls) {
        float I = 1.0f;
        if (cansee(sc, h.hitPoint, V3::of(L.position), I, cnt))
            out.push_back(make_light(V3::of(L.color), I, h, refl, V3::of(L.position)));
    }
    for (const auto& L : sc.sls) {
        const V3 pos = V3::of(L.position);
        float I = 1.0f, sum = 1.0f;
        int seen = 0;
        if (cansee(sc, h.hitPoint, pos, sum, cnt)) seen++;
        V3 d = vnormalize(pos - h.hitPoint);
        V3 other = d;
        if (d.x != 0) {
            other.y = -d.x;
            other.x = d.y;
        } else {
            other.y = -d.z;
            other.z = d.y;
        }
        V3 perp = vnormalize(vcross(d, other)) * L.radius;
        int count = P.sphere_light_ray_count;
        const int rings = std::max(1, (int)(count / std::round(std::sqrt(2 * 3.14159365358979f * count))));
        const int spokes = (count - 1) / rings;
        count = rings * spokes + 1;
        const Rot R = rodrigues(2 * 3.14159365358979f / spokes, d);
        for (int i = 0; i < spokes; i++) {
            for (int j = 0; j < rings; j++) {
                I = 1.0f;
                if (cansee(sc, h.hitPoint, pos + ((rings - j) / (float)rings) * perp, I, cnt)) {
                    seen++;
                    sum += I;
                }
            }
            perp = rot_apply(R, perp);
        }
        if (seen > 0) out.push_back(make_light(V3::of(L.color), sum / (float)count, h, refl, pos));
    }
    for (const auto& L : sc.spots) {
        const V3 pos = V3::of(L.position);
        if (vdot(vnormalize(V3::of(L.direction)), vnormalize(h.hitPoint - pos)) >
            std::cos(L.angle * static_cast<float>(0.01745329251994329576923690768489))) {
            float I = 1.0f;
            if (cansee(sc, h.hitPoint, pos, I, cnt)) out.push_back(make_light(V3::of(L.color), I, h, refl, pos));
        }
    }
    for (const auto& L : sc.planes) {
        const int k = P.plane_light_1D_ray_count;
        float acc = 0;
        int nh = 0;
        float best_cos = 0, sumI = 0, I = 1;
        const V3 w = V3::of(L.width), hh = V3::of(L.height), pos = V3::of(L.position);
        const V3 step_x = (1.0f / (k - 1)) * w, step_y = (1.0f / (k - 1)) * hh;
        V3 row = pos;
        const V3 n = vnormalize(vcross(w, hh));
        if (vdot(vnormalize(h.hitPoint - (pos + 0.5f * (w + hh))), n) > 0) {
            for (int i = 0; i < k; i++) {
                V3 q = row;
                for (int j = 0; j < k; j++) {
                    I = 1;
                    if (cansee(sc, h.hitPoint, q, I, cnt)) {
                        sumI += I;
                        acc += fmax_g(vdot(vnormalize(h.hitPoint - q), n), 0.0f) / vlength(h.hitPoint - q);
                        nh++;
                        best_cos = fmax_g(best_cos, vdot(vnormalize(refl), vnormalize(q - h.hitPoint)));
                    }
                    q += step_x;
                }
                row += step_y;
            }
        }
        if (acc > 0) {
            Light l;
            l.color = V3::of(L.color);
            l.intensity = (sumI / nh) * acc / (float)(k * k);
            l.cosL = 1;
            l.cosS = best_cos;
            out.push_back(l);
        }
    }
}

static V3 phong(const Light& l, const Mat& m) {
    const V3 diffuse = m.kd * l.color * l.intensity * l.cosL;
    V3 spec(0.0f);
    if (m.shininess > 0) spec = l.color * m.ks * std::pow(l.cosS, m.shininess);
    return diffuse + spec;
}

// ---------------------------------------------------------------- getFinalColor (main.cpp:129-301)
// Ray differentials (framework/include/ray.h:17-28, src/ray_differentials.cpp) with the values
// the member initialisers intend (right = (1,0,0), up = (0,-1,0); the reference reads them
// before they are initialised): a camera ray is default-constructed (direction (0,0,-1)) and
// set afterwards, a secondary ray is aggregate-initialised with its direction.  Only the
// transferred dP reaches the level of detail.
static float level_of_detail(const Ray& ray, bool camera_ray, const Hit& h, const std::array<Vert, 3>& tv) {
    const V3 right(1.0f, 0.0f, 0.0f), up(0.0f, -1.0f, 0.0f);
    const V3 dir0 = camera_ray ? V3(0.0f, 0.0f, -1.0f) : ray.direction;
    const V3 dD_dx = (vdot(dir0, dir0) * right - vdot(dir0, right) * dir0) / std::pow(vdot(dir0, dir0), 1.5f);
    const V3 dD_dy = (vdot(dir0, dir0) * up - vdot(dir0, up) * dir0) / std::pow(vdot(dir0, dir0), 1.5f);
    V3 dP_dx(0.0f), dP_dy(0.0f);
    // transfer_ray_differentials (:5-15)
    const V3 N = vnormalize(h.normal), D = vnormalize(ray.direction);
    const float dt_dx = -vdot(dP_dx + ray.t * dD_dx, N) / vdot(D, N);
    const float dt_dy = -vdot(dP_dy + ray.t * dD_dy, N) / vdot(D, N);
    dP_dx = (dP_dx + ray.t * dD_dx) + dt_dx * D;
    dP_dy = (dP_dy + ray.t * dD_dy) + dt_dy * D;
    // computeDerivativeOfBarycentricCoordinate (:36-45), computeTexturePartialDerivative... (:66-80)
    auto dbary = [](const V3& a, const V3& b, const V3& p, const V3& pd, float area) {
        const V3 term1 = vcross(pd, p - b) + vcross(p - a, pd);
        const V3 term2 = vcross(a - p, b - p);
        return (vdot(term1, term2) + vdot(term2, term1)) / (2 * area * std::sqrt(vdot(term2, term2)));
    };
    auto dT = [&](const V3& pd, float& du, float& dv) {
        const float area = vlength(vcross(tv[2].p - tv[0].p, tv[1].p - tv[0].p));
        const float a = dbary(tv[2].p, tv[1].p, h.hitPoint, pd, area);
        const float b = dbary(tv[0].p, tv[2].p, h.hitPoint, pd, area);
        const float g = dbary(tv[1].p, tv[0].p, h.hitPoint, pd, area);
        du = (a * tv[0].u + b * tv[1].u) + g * tv[2].u;
        dv = (a * tv[0].v + b * tv[1].v) + g * tv[2].v;
    };
    float ux, vx, uy, vy;
    dT(1.0f * dP_dx, ux, vx);
    dT(1.0f * dP_dy, uy, vy);
    const float lx = std::sqrt(ux * ux + vx * vx), ly = std::sqrt(uy * uy + vy * vy);
    return fmax_g(0.0f, std::log2(fmax_g(lx, ly)));  // computeLevelOfDetails (:112-139)
}

static V3 final_color(Scene& sc, const rt_params& P, Ray ray, int level, Counter& cnt) {
    Hit h;
    if (!intersect(sc, ray, h, P.use_bvh != 0, cnt)) return V3(0.0f);
    if (h.is_triangle && h.ub) cnt.ub++;
    V3 color(0.0f);
    const V3 refl = vreflect(vnormalize(ray.direction), vnormalize(h.normal));
    Mat m = h.material(sc.mats);
    // matForRendering.kd from the texture (src/main.cpp:146-171)
    if (P.use_textures && h.is_triangle && m.texture >= 0) {
        const auto& tv = sc.tris[h.prim];
        const float lod = P.texture_filtering >= RT_TEX_MIP_NEAREST ? level_of_detail(ray, level == 0, h, tv) : 0.0f;
        m.kd = sc.images[m.texture].get_pixel(h.u, h.v, lod, P);
    }
    std::vector<Light> lights;
    gather_lights(sc, h, refl, P, lights, cnt);
    for (const Light& l : lights) color += phong(l, m);
    if (level >= P.max_reflection_level) return color;
    if (m.transparency == 1.0f) {
        if (m.ks.x > 0 || m.ks.y > 0 || m.ks.z > 0) {
            V3 mirror(0.0f);
            Ray rr;
            rr.origin = h.hitPoint + 0.01f * refl;
            rr.direction = refl;
            mirror += m.ks * final_color(sc, P, rr, level + 1, cnt);
            if (m.shininess != 0) {
                // glossy lobe (main.cpp:209-250); rand() pairs come from the Philox stream
                V3 notr = refl;
                if (refl.x != 0) {
                    notr.y = -refl.x;
                    notr.x = refl.y;
                } else {
                    notr.y = -refl.z;
                    notr.z = refl.y;
                }
                const V3 pr1 = vcross(refl, notr);
                const V3 pr2 = vcross(refl, pr1);
                const float s = m.shininess;
                const float d = std::pow(0.5f, -1 / s) * std::sqrt(1 - std::pow(0.5, 2 / s));
                for (int i = 1; i < P.glossy_ray_count; i++) {
                    V3 dir;
                    float a, b;
                    int loops = 0;
                    do {
                        do {
                            draw_pair(cnt, P.rng_seed, a, b);
                        } while (a == 0 && b == 0 && a * a + b * b < 1);
                        a = (2 * a - 1) * d;
                        b = (2 * b - 1) * d;
                        dir = vnormalize(refl + a * pr1 + b * pr2);
                        loops++;
                    } while (vdot(dir, h.normal) <= 0 && loops < P.glossy_ray_count / 4);
                    if (vdot(dir, h.normal) > 0) {
                        Ray g;
                        g.origin = h.hitPoint + 0.01f * dir;
                        g.direction = dir;
                        mirror += final_color(sc, P, g, level + 1, cnt) * fmax_g(std::pow(vdot(refl, dir), s), 0.0f);
                    }
                }
                color += m.ks * mirror / (float)P.glossy_ray_count;
            } else {
                color += m.ks * mirror;
            }
        }
    } else {
        const V3 l = vnormalize(ray.direction);
        const V3 n = vnormalize(h.normal);
        const float r = P.refraction_factor;
        const float c = std::abs(vdot(l, n));
        V3 refr = r * l + (r * c - std::sqrt(1 - r * r * (1 - c * c))) * n;
        refr = vnormalize(refr);
        const float R0 = m.transparency;
        const float reflect_part = R0 + (1 - R0) * std::pow((double)(1 - c), 5.0);
        const float refract_part = 1 - reflect_part;
        Ray a;
        a.origin = h.hitPoint + 0.01f * refl;
        a.direction = refl;
        color += reflect_part * final_color(sc, P, a, level + 1, cnt);
        if (r * r * (1 - c * c) <= 1.0f) {
            Ray b;
            b.origin = h.hitPoint + 0.01f * refr;
            b.direction = refr;
            color += refract_part * final_color(sc, P, b, level + 1, cnt);
        }
    }
    return color;
}

// ---------------------------------------------------------------- camera (trackball.cpp)
struct Cam {
    V3 pos;
    float qx, qy, qz, qw;
    float hh, hw;
};
static V3 qrot(const Cam& c, const V3& v) {
    const V3 q(c.qx, c.qy, c.qz);
    const V3 uv = vcross(q, v);
    const V3 uuv = vcross(q, uv);
    return v + ((uv * c.qw) + uuv) * 2.0f;
}
static Cam make_cam(const float look[3], const float e[3], float dist, float fovy, float aspect) {
    Cam c;
    const V3 half = V3(e[0], e[1], e[2]) * 0.5f;
    const float cx = std::cos(half.x), cy = std::cos(half.y), cz = std::cos(half.z);
    const float sx = std::sin(half.x), sy = std::sin(half.y), sz = std::sin(half.z);
    c.qw = cx * cy * cz + sx * sy * sz;
    c.qx = sx * cy * cz - cx * sy * sz;
    c.qy = cx * sy * cz + sx * cy * sz;
    c.qz = cx * cy * sz - sx * sy * cz;
    c.pos = V3(look[0], look[1], look[2]) + qrot(c, V3(0, 0, -dist));
    c.hh = std::tan(fovy / 2.0f);
    c.hw = aspect * c.hh;
    return c;
}
static Ray camera_ray(const Cam& c, float px, float py) {
    const V3 local = vnormalize(V3(-px * c.hw, py * c.hh, 1.0f));
    Ray r;
    r.origin = c.pos;
    r.direction = qrot(c, local);
    r.t = FLT_MAX;
    return r;
}

// one camera sample of the pixel (restarts the pixel's glossy draw stream for that sample)
static V3 sample_color(Scene& sc, const rt_params& P, const Ray& r, int sample, Counter& cnt) {
    cnt.sample = (uint32_t)sample;
    cnt.draws = 0;
    return final_color(sc, P, r, 0, cnt);
}

static V3 render_pixel(Scene& sc, const Cam& cam, const rt_params& P, int W, int H, int x, int y, Counter& cnt) {
    cnt.pix = (uint32_t)(y * W + x);
    const float nx = float(x) / W * 2.0f - 1.0f;
    const float ny = float(y) / H * 2.0f - 1.0f;
    if (P.anti_aliasing) {
        const float ox = 1.0f / W * 0.25f, oy = 1.0f / H * 0.25f;
        const float qx[4] = {nx - ox, nx + ox, nx - ox, nx + ox};
        const float qy[4] = {ny + oy, ny + oy, ny - oy, ny - oy};
        V3 avg(0.0f);
        for (int i = 0; i < 4; i++) avg += sample_color(sc, P, camera_ray(cam, qx[i], qy[i]), i, cnt);
        avg = avg * (float)0.25;
        return avg;
    }
    if (P.multiple_rays) {
        const float ox = (1.0f / W) * (1.0f / (std::sqrt(P.sample_size) * 2));
        const float oy = (1.0f / H) * (1.0f / (std::sqrt(P.sample_size) * 2));
        const int moves = std::sqrt(P.sample_size) - 1;
        const float sgn[4][2] = {{-1.0f, 1.0f}, {1.0f, 1.0f}, {-1.0f, -1.0f}, {1.0f, -1.0f}};
        V3 avg(0.0f);
        int k = 0;
        for (int i = 0; i < 4; i++)
            for (int a = 1; a <= moves; a += 2)
                for (int b = 1; b <= moves; b += 2)
                    avg += sample_color(
                        sc, P, camera_ray(cam, nx + (ox * sgn[i][0] * a), ny + (oy * sgn[i][1] * b)), k++, cnt);
        return avg * (float)(1.0f / P.sample_size);
    }
    return sample_color(sc, P, camera_ray(cam, nx, ny), 0, cnt);
}

}  // namespace oracle

using namespace oracle;

struct oracle_scene {
    Scene sc;
};

extern "C" {

oracle_scene* oracle_create(const rt_scene_desc* d) {
    oracle_scene* o = new oracle_scene();
    Scene& sc = o->sc;
    for (int m = 0; m < d->num_meshes; ++m) {
        Mat mm;
        mm.kd = V3::of(d->materials[m].kd);
        mm.ks = V3::of(d->materials[m].ks);
        mm.shininess = d->materials[m].shininess;
        mm.transparency = d->materials[m].transparency;
        if (d->materials[m].has_texture && d->materials[m].texture >= 0 && d->materials[m].texture < d->num_textures)
            mm.texture = d->materials[m].texture;
        sc.mats.push_back(mm);
    }
    for (int t = 0; t < d->num_textures; ++t) sc.images.emplace_back(d->textures[t]);
    for (int t = 0; t < d->num_triangles; ++t) {
        std::array<Vert, 3> tri;
        for (int c = 0; c < 3; ++c) {
            tri[c].p = V3::of(d->positions + t * 9 + c * 3);
            tri[c].n = V3::of(d->normals + t * 9 + c * 3);
            if (d->texcoords) {
                tri[c].u = d->texcoords[t * 6 + c * 2];
                tri[c].v = d->texcoords[t * 6 + c * 2 + 1];
            }
        }
        sc.tris.push_back(tri);
        sc.tri_mesh.push_back(d->mesh_index[t]);
    }
    for (int s = 0; s < d->num_spheres; ++s) {
        Sph sp;
        sp.center = V3::of(d->spheres[s].center);
        sp.radius = d->spheres[s].radius;
        sp.mat.kd = V3::of(d->spheres[s].material.kd);
        sp.mat.ks = V3::of(d->spheres[s].material.ks);
        sp.mat.shininess = d->spheres[s].material.shininess;
        sp.mat.transparency = d->spheres[s].material.transparency;
        sc.spheres.push_back(sp);
    }
    sc.pls.assign(d->point_lights, d->point_lights + d->num_point_lights);
    sc.sls.assign(d->spherical_lights, d->spherical_lights + d->num_spherical_lights);
    sc.spots.assign(d->spot_lights, d->spot_lights + d->num_spot_lights);
    sc.planes.assign(d->plane_lights, d->plane_lights + d->num_plane_lights);
    build_bvh(sc);
    return o;
}

void oracle_destroy(oracle_scene* o) { delete o; }

int oracle_bvh_info(oracle_scene* o, int* num_nodes, int* num_leaves) {
    *num_nodes = (int)o->sc.nodes.size();
    int leaves = 0;
    for (const Node& n : o->sc.nodes) leaves += n.leaf ? 1 : 0;
    *num_leaves = leaves;
    return 0;
}

// node boxes (lo, hi) and leaf flag, BFS creation order
int oracle_bvh_nodes(oracle_scene* o, float* boxes, int* is_leaf, int cap) {
    const int n = (int)o->sc.nodes.size();
    for (int i = 0; i < n && i < cap; ++i) {
        const Node& nd = o->sc.nodes[i];
        const float b[6] = {nd.lo.x, nd.lo.y, nd.lo.z, nd.hi.x, nd.hi.y, nd.hi.z};
        std::memcpy(boxes + i * 6, b, sizeof(b));
        is_leaf[i] = nd.leaf ? 1 : 0;
    }
    return n;
}

// node `node`'s children as constructBVH stored them (src/bounding_volume_hierarchy.cpp:108-217): node
// indices for an inner node; for a leaf its objects in stored order, triangles as their scene index and
// spheres as num_triangles + sphere index.  Returns the count (copies at most cap).
int oracle_bvh_children(oracle_scene* o, int node, int* out, int cap) {
    if (node < 0 || node >= (int)o->sc.nodes.size()) return -1;
    const Node& nd = o->sc.nodes[node];
    const int ntri = (int)o->sc.tris.size();
    const int n = (int)nd.kids.size();
    for (int i = 0; i < n && i < cap; ++i) out[i] = (nd.leaf && !nd.tri[i]) ? ntri + nd.kids[i] : nd.kids[i];
    return n;
}

int oracle_intersect(oracle_scene* o, const rt_ray* rays, int n, int use_bvh, rt_hit* out) {
    for (int i = 0; i < n; ++i) {
        Ray r;
        r.origin = V3::of(rays[i].origin);
        r.direction = V3::of(rays[i].direction);
        r.t = rays[i].t;
        Hit h;
        Counter cnt;
        const bool hit = intersect(o->sc, r, h, use_bvh != 0, cnt);
        rt_hit& x = out[i];
        std::memset(&x, 0, sizeof(x));
        x.hit = hit ? 1 : 0;
        x.t = r.t;
        if (hit) {
            const float nn[3] = {h.normal.x, h.normal.y, h.normal.z};
            const float pp[3] = {h.hitPoint.x, h.hitPoint.y, h.hitPoint.z};
            std::memcpy(x.normal, nn, 12);
            std::memcpy(x.hit_point, pp, 12);
            x.uv[0] = h.u;
            x.uv[1] = h.v;
            x.material_index = h.is_triangle ? h.material_index : -1;
            x.prim_id = h.prim;
            x.is_triangle = h.is_triangle ? 1 : 0;
        } else {
            x.material_index = -1;
            x.prim_id = -1;
        }
    }
    return 0;
}

int oracle_shade(oracle_scene* o, const rt_ray* rays, int n, const rt_params* P, float* rgb, uint64_t* counts) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; ++i) {
        Ray r;
        r.origin = V3::of(rays[i].origin);
        r.direction = V3::of(rays[i].direction);
        r.t = rays[i].t;
        Counter cnt;
        cnt.pix = (uint32_t)i;
        const V3 c = final_color(o->sc, *P, r, P->shade_level, cnt);  // getFinalColor(..., level)
        rgb[i * 3] = c.x;
        rgb[i * 3 + 1] = c.y;
        rgb[i * 3 + 2] = c.z;
        if (counts) counts[i] = cnt.rays;
    }
    return 0;
}

int oracle_camera(const float look[3], const float euler[3], float dist, float fovy, float aspect, float out[9]) {
    const Cam c = make_cam(look, euler, dist, fovy, aspect);
    const float v[9] = {c.pos.x, c.pos.y, c.pos.z, c.qx, c.qy, c.qz, c.qw, c.hh, c.hw};
    std::memcpy(out, v, sizeof(v));
    return 0;
}

// Render the listed pixels (x, y pairs in renderRayTracing's y-up convention).  rgb[i] is the
// colour setPixel(x, y, .) would store; rays[i] the intersect() calls it took.
int oracle_render_pixels(oracle_scene* o, const float look[3], const float euler[3], float dist, float fovy,
                         int W, int H, const rt_params* P, const int* xy, int n, float* rgb, uint64_t* rays,
                         uint64_t* ub) {
    const Cam cam = make_cam(look, euler, dist, fovy, float(W) / float(H));
#pragma omp parallel for schedule(dynamic, 4)
    for (int i = 0; i < n; ++i) {
        Counter cnt;
        const V3 c = render_pixel(o->sc, cam, *P, W, H, xy[2 * i], xy[2 * i + 1], cnt);
        rgb[i * 3] = c.x;
        rgb[i * 3 + 1] = c.y;
        rgb[i * 3 + 2] = c.z;
        if (rays) rays[i] = cnt.rays;
        if (ub) ub[i] = cnt.ub;
    }
    return 0;
}

// Whole frame in Screen::m_textureData order (row (H-1-y) first), src/screen.cpp:32-38.
int oracle_render(oracle_scene* o, const float look[3], const float euler[3], float dist, float fovy, int W, int H,
                  const rt_params* P, float* rgb, uint64_t* total_rays) {
    const Cam cam = make_cam(look, euler, dist, fovy, float(W) / float(H));
    uint64_t total = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            Counter cnt;
            const V3 c = render_pixel(o->sc, cam, *P, W, H, x, y, cnt);
            float* dst = rgb + ((size_t)(H - 1 - y) * W + x) * 3;
            dst[0] = c.x;
            dst[1] = c.y;
            dst[2] = c.z;
            total += cnt.rays;
        }
    }
    if (total_rays) *total_rays = total;
    return 0;
}

// Image::getPixel(texCoord, lod) (src/image.cpp:77-110) of image `tex` for n (u, v, lod) triples.
int oracle_tex_sample(oracle_scene* o, int tex, const float* uvl, int n, const rt_params* P, float* rgb) {
    if (tex < 0 || tex >= (int)o->sc.images.size()) return -1;
    for (int i = 0; i < n; ++i) {
        const V3 c = o->sc.images[tex].get_pixel(uvl[3 * i], uvl[3 * i + 1], uvl[3 * i + 2], *P);
        rgb[3 * i] = c.x;
        rgb[3 * i + 1] = c.y;
        rgb[3 * i + 2] = c.z;
    }
    return 0;
}

int oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    philox(c, (uint64_t)key[0] | ((uint64_t)key[1] << 32));
    std::memcpy(out, c, sizeof(c));
    return 0;
}

int oracle_set_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n);
    return n;
#else
    (void)n;
    return 1;
#endif
}
}
