// The reference's render path (src/main.cpp:402-522) written against the facade: loadScene ->
// BoundingVolumeHierarchy(&scene) -> intersect / getFinalColor / renderRayTracing, light and material
// edits through the Scene's public vectors (the ImGui editors, src/main.cpp:511-613), Screen + BMP.
// Writes every result as raw float32 files <out>/<name>.bin for tests/test_facade.py to compare with
// the oracle.  Exit code 0 = ok, 3 = no GPU (the constructor threw, as it must without a device).
#include <cstdio>
#include <string>
#include <vector>

#include "rt_facade.hpp"

using namespace rt::facade;

static void dump(const std::string& path, const std::vector<float>& v) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return;
    std::fwrite(v.data(), sizeof(float), v.size(), f);
    std::fclose(f);
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string dataPath = argv[1], out = argv[2];
    Window window{64, 48};
    Scene scene = loadScene(SceneType::Monkey, dataPath);
    size_t ntri = 0;
    for (const Mesh& m : scene.meshes) ntri += m.triangles.size();
    std::printf("meshes=%zu triangles=%zu vertices=%zu pointLights=%zu\n", scene.meshes.size(), ntri,
                scene.meshes[0].vertices.size(), scene.pointLights.size());
    if (ntri != 968) return 4;
    try {
        BoundingVolumeHierarchy bvh{&scene};
        Trackball camera{&window, radians(50.0f), 3.0f};
        camera.setCamera(vec3(0.0f, 0.0f, 0.0f), radians(vec3(20.0f, 20.0f, 0.0f)), 3.0f);
        max_reflection_level = 1;  // BASELINE.json configs[1]
        glossy_ray_count = 1;      // no rand()
        std::printf("levels=%d\n", bvh.numLevels());

        // 1. camera rays of a 16 x 12 grid: intersect (both useBVH modes), getFinalColor at level 0 and 1
        std::vector<float> rays, hits[2], colors, colors_l1;
        for (int y = 0; y < 12; ++y)
            for (int x = 0; x < 16; ++x) {
                const vec2 ndc{float(x) / 16 * 2.0f - 1.0f, float(y) / 12 * 2.0f - 1.0f};
                const Ray ray = camera.generateRay(ndc);
                rays.insert(rays.end(), {ray.origin.x, ray.origin.y, ray.origin.z, ray.direction.x, ray.direction.y,
                                         ray.direction.z, ray.t});
                for (int b = 0; b < 2; ++b) {
                    Ray r = ray;
                    HitInfo h;
                    const bool hit = bvh.intersect(r, h, b == 1);
                    hits[b].insert(hits[b].end(), {hit ? 1.0f : 0.0f, r.t, h.normal.x, h.normal.y, h.normal.z,
                                                   h.hitPoint.x, h.hitPoint.y, h.hitPoint.z, (float)h.material_index,
                                                   h.is_triangle ? 1.0f : 0.0f,
                                                   hit ? h.getMaterial(scene).kd.x : -1.0f});
                }
                const vec3 c = getFinalColor(scene, bvh, ray);
                colors.insert(colors.end(), {c.x, c.y, c.z});
                const vec3 c1 = getFinalColor(scene, bvh, ray, 1);
                colors_l1.insert(colors_l1.end(), {c1.x, c1.y, c1.z});
            }
        dump(out + "/rays.bin", rays);
        dump(out + "/hits_bvh0.bin", hits[0]);
        dump(out + "/hits_bvh1.bin", hits[1]);
        dump(out + "/colors.bin", colors);
        dump(out + "/colors_l1.bin", colors_l1);

        // 2. "Render to file" (src/main.cpp:513-522)
        Screen screen{64, 48};
        renderRayTracing(scene, camera, bvh, screen, false, false, false, 4);
        dump(out + "/frame0.bin", screen.textureData());

        // 3. light edits after the BVH exists: move the point light, add a spherical light
        scene.pointLights[0].position = vec3(0.5f, 1.5f, -1.0f);
        scene.sphericalLight.push_back(SphericalLight{vec3(-1.0f, 1.0f, -1.0f), 0.1f, vec3(0.5f, 0.25f, 1.0f)});
        sphere_light_ray_count = 16;
        renderRayTracing(scene, camera, bvh, screen, false, false, false, 4);
        dump(out + "/frame1.bin", screen.textureData());

        // 4. a material edit
        scene.meshes[0].material.kd = vec3(0.2f, 0.9f, 0.3f);
        scene.meshes[0].material.ks = vec3(0.0f);
        renderRayTracing(scene, camera, bvh, screen, false, false, false, 4);
        dump(out + "/frame2.bin", screen.textureData());

        // 5. a turntable batch: every view equals its own renderRayTracing call, bit for bit
        std::vector<Trackball> cams(3, camera);
        cams[1].setCamera(vec3(0.0f), vec3(0.34906584f, 0.84906584f, 0.0f), 3.0f);
        cams[2].setCamera(vec3(0.0f), vec3(0.34906584f, 1.34906584f, 0.0f), 3.0f);
        std::vector<std::vector<float>> views;
        renderRayTracingViews(scene, cams, bvh, 64, 48, views);
        int same = 0;
        for (size_t v = 0; v < cams.size(); ++v) {
            Screen one{64, 48};
            renderRayTracing(scene, cams[v], bvh, one);
            same += (one.textureData() == views[v]) ? 1 : 0;
        }
        std::printf("views_identical=%d/%d\n", same, (int)cams.size());

        // 5b. autoSync(false): a per-ray loop that syncs the scene itself, once
        {
            const Ray ray = camera.generateRay(vec2{0.05f, 0.05f});
            const vec3 before = getFinalColor(scene, bvh, ray);
            const vec3 kd = scene.meshes[0].material.kd;
            bvh.autoSync(false);
            scene.meshes[0].material.kd = vec3(0.9f, 0.1f, 0.1f);
            const vec3 stale = getFinalColor(scene, bvh, ray);
            bvh.sync(scene);
            const vec3 fresh = getFinalColor(scene, bvh, ray);
            bvh.autoSync(true);
            scene.meshes[0].material.kd = kd;
            const vec3 back = getFinalColor(scene, bvh, ray);
            auto eq = [](const vec3& a, const vec3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; };
            std::printf("autosync stale_same=%d fresh_differs=%d restored=%d\n", eq(before, stale) ? 1 : 0,
                        eq(before, fresh) ? 0 : 1, eq(before, back) ? 1 : 0);
        }

        // 6. Screen + bloom + gamma + BMP, as the "Render to file" button does
        Screen scr{32, 24};
        scr.setBloomFilter(FilteringOption::BloomWithReinhardHdr);
        scr.setKernel(Kernel::GaussianKernel);
        scr.setFilterSize(2);
        scr.enableGammaCorrection(true);
        Window w2{32, 24};
        Trackball cam2{&w2, radians(50.0f), 3.0f};
        cam2.setCamera(vec3(0.0f), radians(vec3(20.0f, 20.0f, 0.0f)), 3.0f);
        renderRayTracing(scene, cam2, bvh, scr);
        scr.writeBitmapToFile(out + "/render.bmp");
        std::printf("done\n");
        return 0;
    } catch (const std::exception& e) {
        std::printf("no device: %s\n", e.what());
        return 3;
    }
}
