// Reference-style use of the facade: loadScene -> BoundingVolumeHierarchy -> intersect /
// getFinalColor / renderRayTracing, as src/main.cpp:402-522 drives them.  Exit code 0 = ok,
// 3 = no GPU (the constructor threw, as it must without a device).
#include <cstdio>
#include <vector>

#include "rt_facade.hpp"

using namespace rt::facade;

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    Scene scene = loadScene(Monkey, argv[1]);
    if (scene.desc().num_triangles != 968) return 4;
    try {
        BoundingVolumeHierarchy bvh{&scene};
        Ray ray;
        ray.origin = vec3{0, 0, -3};
        ray.direction = vec3{0, 0, 1};
        HitInfo hit;
        const bool h = bvh.intersect(ray, hit, false);
        std::printf("hit=%d t=%.9g levels=%d\n", (int)h, ray.t, bvh.numLevels());
        const vec3 c = getFinalColor(bvh, Ray{vec3{0, 0, -3}, vec3{0, 0, 1}});
        std::printf("color=%.9g %.9g %.9g\n", c.x, c.y, c.z);
        std::vector<float> screen;
        renderRayTracing(Trackball{}, bvh, 32, 32, screen);
        double sum = 0;
        for (float v : screen) sum += v;
        std::printf("frame_sum=%.9g\n", sum);
        // a turntable batch: every view equals its own renderRayTracing call, bit for bit
        std::vector<Trackball> cams(3);
        cams[1].rotationEulerAngles.y += 0.5f;
        cams[2].rotationEulerAngles.y += 1.0f;
        std::vector<std::vector<float>> views;
        renderRayTracingViews(cams, bvh, 32, 32, views);
        int same = 0;
        for (size_t v = 0; v < cams.size(); ++v) {
            std::vector<float> one;
            renderRayTracing(cams[v], bvh, 32, 32, one);
            same += (one == views[v]) ? 1 : 0;
        }
        std::printf("views_identical=%d/%d\n", same, (int)cams.size());
        // Screen + bloom + gamma + BMP, as the "Render to file" button does (src/main.cpp:513-522)
        Screen scr(32, 24);
        scr.setBloomFilter(FilteringOption::BloomWithReinhardHdr);
        scr.setKernel(Kernel::GaussianKernel);
        scr.setFilterSize(2);
        scr.enableGammaCorrection(true);
        renderRayTracing(Trackball{}, bvh, scr);
        const char* out = argc > 2 ? argv[2] : "facade_render.bmp";
        scr.writeBitmapToFile(out);
        std::printf("bmp=%s\n", out);
        return h ? 0 : 5;
    } catch (const std::exception& e) {
        std::printf("no device: %s\n", e.what());
        return 3;
    }
}
