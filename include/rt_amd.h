/*
 * rt_amd.h -- C-ABI drop-in boundary of the MI355X-native per-pixel ray tracer.
 *
 * Every entry point replaces one C++ seam of the reference renderer
 * (catalinlup/RayTracer-Group27, paths relative to the reference root):
 *
 *   rt_create            BoundingVolumeHierarchy::BoundingVolumeHierarchy(Scene*)
 *                        src/bounding_volume_hierarchy.h:24, .cpp:5-9 (+ scene upload), over a device list:
 *                        one scene replica per GPU
 *   rt_intersect         bool BoundingVolumeHierarchy::intersect(Ray&, HitInfo&, bool useBVH) const
 *                        src/bounding_volume_hierarchy.h:33, .cpp:49-78
 *   rt_shade             static glm::vec3 getFinalColor(Scene&, const BVH&, Ray, int level=0)
 *                        src/main.cpp:129-301
 *   rt_render            static void renderRayTracing(Scene&, const Trackball&, const BVH&, Screen&, ...)
 *                        src/main.cpp:340-400 (+ Screen::setPixel src/screen.cpp:32-38)
 *   rt_render_views_image_device  renderRayTracing's pixel loop split over the context's GPUs (the OpenMP
 *                        row split, src/main.cpp:344-347): every GPU stores its bands straight into
 *                        the setPixel layout on the first GPU -- no gather, no un-permute
 *   rt_render_device     same as rt_render, band-partitioned, device-resident output (multi-GPU path)
 *   rt_render_views_device  a batch of rt_render_device frames (one camera each) in one launch
 *   rt_render_views      the same batch, host output in the rt_render layout
 *   rt_camera_from_trackball  Trackball::generateRay / position(), framework/src/trackball.cpp:65-98
 *   rt_scene_load_obj    std::vector<Mesh> loadMesh(path, bool normalize), src/mesh.cpp:58-188
 *   rt_scene_preset      Scene loadScene(SceneType, dataDir), src/scene.cpp:4-150
 *   rt_update_lights     the ImGui light editors after the BVH exists, src/main.cpp:511-613
 *   rt_update_materials  material edits (scene.meshes[i].material), no BVH rebuild
 *   rt_texture_sample    Image::getPixel(texCoord, lod), src/image.cpp:77-110 (parity tests)
 *   rt_destroy           ~BoundingVolumeHierarchy / scene teardown
 *
 * Conventions: plain pointers and sizes, no C++ or torch types.  Every function returns an
 * int status: 0 = ok, < 0 = error (message via rt_last_error).  The caller owns every host
 * buffer it passes; a context owns its device memory.  Calls on one context must not be made
 * concurrently (the reference BVH is shared read-only by OpenMP threads; here the parallelism is
 * inside the GPU launch).  The *_device calls are asynchronous on the caller's stream (NULL = the
 * null stream, so they are ordered after the caller's default-stream work on their buffers) unless
 * `stats` is given; a context keeps ONE set of per-render scratch (camera table, job counters), so
 * its renders must be ordered on one stream (or separated by events) -- two renders of one
 * context in flight on different streams at once would share that scratch.
 *
 * Multi-device contexts (rt_create with ndev > 1): devices[0] is the context's home device; its
 * streams (the caller's, for the *_device calls) order every call.  rt_render, rt_render_views and
 * rt_render_views_image_device split the frame's interleaved 8-row bands over every device (one host
 * thread per extra device); each extra device waits for the caller stream's earlier work and the
 * caller stream waits for it before its later work, so the call keeps single-stream semantics.  The
 * per-ray and band-dense calls (rt_intersect, rt_shade, rt_render_device, rt_render_views_device,
 * rt_texture_sample) run on devices[0] alone.  A device may appear more than once (replicas on one
 * GPU: the parity tests' stand-in for a multi-GPU node).
 *
 * Edits (rt_update_lights, rt_update_materials) first wait for every render in flight on every device
 * of the context (device-wide synchronise), then replace the arrays: renders enqueued after the edit
 * returns see the new values, none sees a mix.
 */
#ifndef RT_AMD_H
#define RT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 5  /* 2: textures; 3: rt_render_views_device; 4: rt_stats.ub_hits / .kernel,
                             rt_ctx_set_option, rt_update_lights / _materials, rt_texture_sample;
                             5: rt_create over a device list, rt_render_views_image_device, rt_ipc_*,
                             rt_ctx_devices */

/* status codes */
#define RT_OK 0
#define RT_ERR_INVALID (-1)
#define RT_ERR_IO (-2)
#define RT_ERR_HIP (-3)
#define RT_ERR_NOMEM (-4)
#define RT_ERR_NO_DEVICE (-5)

/* Material, src/mesh.h:23-33 (kd, ks{0}, shininess{1}, transparency{1}, optional<Image>). */
typedef struct rt_material {
    float kd[3];
    float ks[3];
    float shininess;
    float transparency;
    int has_texture; /* kdTexture.has_value() */
    int texture;     /* index into rt_scene_desc.textures when has_texture, else ignored */
} rt_material;

/* Decoded kd texture, what Image::Image (src/image.cpp:37-73) gets from
 * stbi_load(path, &w, &h, &numChannels, STBI_rgb): `rgb` holds width*height*3 bytes and
 * `channels` is the file's channel count.  rt_create turns it into texels the way the reference
 * does -- texel k = rgb[k*channels + 0..2] / 255.0f (bytes past the buffer, which the reference
 * reads for 4-channel files, are taken as 0) -- and builds the mip chain (src/image.cpp:408-452)
 * for square power-of-two sizes.  channels < 3 is an error, as in the reference. */
typedef struct rt_texture {
    int width, height;
    int channels;
    int pad_;
    const uint8_t* rgb;
} rt_texture;

/* Sphere, src/scene.h:48-53 */
typedef struct rt_sphere {
    float center[3];
    float radius;
    rt_material material;
} rt_sphere;

/* Light PODs, src/scene.h:55-83 */
typedef struct rt_point_light { float position[3]; float color[3]; } rt_point_light;
typedef struct rt_spherical_light { float position[3]; float radius; float color[3]; } rt_spherical_light;
typedef struct rt_spot_light { float position[3]; float direction[3]; float angle; float color[3]; } rt_spot_light;
typedef struct rt_plane_light { float position[3]; float width[3]; float height[3]; float color[3]; } rt_plane_light;

/*
 * Flat scene in scene order.  Triangles are listed mesh-major exactly as
 * BoundingVolumeHierarchy::loadObjectsFromScene flattens them
 * (src/bounding_volume_hierarchy.cpp:80-99): for each mesh, for each of its triangles,
 * the three Vertex records {p, n, texCoord} (src/mesh.h:16-21).
 */
typedef struct rt_scene_desc {
    int num_triangles;
    const float* positions;   /* [num_triangles][3 corners][3] */
    const float* normals;     /* [num_triangles][3 corners][3] */
    const float* texcoords;   /* [num_triangles][3 corners][2] or NULL (zeros) */
    const int* mesh_index;    /* [num_triangles] index into materials (== triangle_materials) */
    int num_meshes;
    const rt_material* materials; /* [num_meshes] */
    int num_spheres;
    const rt_sphere* spheres;
    int num_point_lights;
    const rt_point_light* point_lights;
    int num_spherical_lights;
    const rt_spherical_light* spherical_lights;
    int num_spot_lights;
    const rt_spot_light* spot_lights;
    int num_plane_lights;
    const rt_plane_light* plane_lights;
    int num_textures;
    const rt_texture* textures;
} rt_scene_desc;

/*
 * Camera constants, computed once per frame on the host with the reference Trackball math
 * (framework/src/trackball.cpp:65-68,87-98): ray.origin = position,
 * ray.direction = quat * normalize(vec3(-ndc.x*half_width, ndc.y*half_height, 1)).
 */
typedef struct rt_camera {
    float position[3];
    float quat[4];      /* x, y, z, w  (glm::quat(eulerAngles)) */
    float half_height;  /* tan(fovy/2) */
    float half_width;   /* aspect * half_height */
} rt_camera;

/* Render knobs: the reference's globals, src/main.cpp:54-64,123-127 (defaults in brackets). */
typedef struct rt_params {
    int max_reflection_level;     /* [5] */
    int sphere_light_ray_count;   /* [10] */
    int plane_light_1D_ray_count; /* [3] */
    int glossy_ray_count;         /* [10]; parity configs use 1 (no rand()) */
    float refraction_factor;      /* [0.8] */
    int use_bvh;                  /* [0] useBVH for primary/secondary rays; shadow rays always use the BVH */
    int anti_aliasing;            /* renderRayTracing(..., anti_aliasing) */
    int multiple_rays;            /* renderRayTracing(..., multipleRays, sampleSize) */
    int sample_size;              /* [4]: 4, 16 or 64 */
    int barycentric_mode;         /* 0 = "unthresholded" (defined semantics for the reference's UB) */
    uint64_t rng_seed;            /* glossy_ray_count > 1: Philox-4x32 stream seed (replaces rand()) */
    /* kd textures (src/main.cpp:54-58,155-171; src/image.cpp:77-110) */
    int use_textures;             /* [0] useTextures */
    int texture_filtering;        /* [RT_TEX_NEAREST] textureFiltering (TextureFiltering, src/image.h) */
    int out_of_bounds_x;          /* [RT_OOB_BORDER] outOfBoundsRuleX */
    int out_of_bounds_y;          /* [RT_OOB_BORDER] outOfBoundsRuleY */
    float border_color[3];        /* [0] textureBorderColor */
    int shade_level;              /* rt_shade only: the recursion level of the given rays, getFinalColor's
                                     `level` argument (src/main.cpp:129); renders ignore it (camera rays
                                     are level 0) */
} rt_params;

/* TextureFiltering (src/image.h:22-29) */
#define RT_TEX_NEAREST 0
#define RT_TEX_BILINEAR 1
#define RT_TEX_MIP_NEAREST 2          /* MipMappingNearestLevelNearestNeighbor */
#define RT_TEX_MIP_NEAREST_BILINEAR 3 /* MipMappingNearestLevelBilinear */
#define RT_TEX_TRILINEAR 4
/* OutOfBoundsRule (src/image.h:16-20) */
#define RT_OOB_BORDER 0
#define RT_OOB_CLAMP 1
#define RT_OOB_REPEAT 2

/* Ray, framework/include/ray.h:11-15 (origin, direction, t{FLT_MAX}) */
typedef struct rt_ray {
    float origin[3];
    float direction[3];
    float t; /* initial ray.t (FLT_MAX for a fresh Ray) */
} rt_ray;

/* HitInfo subset, src/ray_tracing.h:6-37 */
typedef struct rt_hit {
    int hit;              /* return value of intersect() */
    float t;              /* ray.t after the call */
    float normal[3];      /* hitInfo.normal (interpolated, not normalized, for triangles) */
    float hit_point[3];   /* hitInfo.hitPoint */
    float uv[2];          /* hitInfo.texCoord */
    int material_index;   /* mesh index (triangles) / -1 (spheres) */
    int prim_id;          /* scene-order triangle index, or num_triangles + sphere index */
    int is_triangle;
} rt_hit;

/* Per-launch counters (rt_render_device / rt_render). */
typedef struct rt_stats {
    uint64_t rays;          /* intersect() calls: primary + secondary + shadow segments */
    uint64_t node_visits;   /* BVH nodes fetched (counting builds only, else 0) */
    uint64_t tri_tests;     /* triangle records fetched (counting builds only, else 0) */
    uint64_t hits;          /* closest hits shaded (counting builds only, else 0) */
    uint64_t ub_hits;       /* counting builds: shaded triangle hits where the reference's
                               barycentricCoordinates returns false (src/ray_tracing.cpp:281-295) and it
                               interpolates from uninitialised coordinates (:147-157) */
    float kernel_ms;        /* device time of the render launch, HIP events */
    uint32_t node_bytes;    /* bytes per node record of the BVH walked: 128 (quantised BVH8) */
    char kernel[64];        /* the render kernel launched, as rocprofv3 names it (without its argument list) */
} rt_stats;

typedef struct rt_ctx rt_ctx;
typedef struct rt_scene rt_scene;

int rt_abi_version(void);
/* Build provenance: the SHA-256 (first 16 hex digits) of the sources this library was compiled from --
 * the csrc/ sources (.hip, .cpp, .h), include/rt_amd.h and build.py (its compiler flags), in sorted path order; the build
 * writes it into the library, and raytracer-group27_amd/build.py source_hash() recomputes it from a tree,
 * so a library can be tied to a commit.  Writes a NUL-terminated string (17 bytes) into buf. */
int rt_source_hash(char* buf, size_t len);
/* PNG decoding with stbi_load(..., STBI_rgb) semantics (the texture loader of Image::Image,
 * src/image.cpp:45): 8-bit RGB out, `channels` = the file's channel count as stb reports it
 * (1 grey, 2 grey+alpha, 3 RGB or palette, 4 RGBA or palette with tRNS).  Call with rgb = NULL to
 * get the size; rgb_size must then be >= width*height*3.  Non-interlaced PNG only. */
int rt_decode_png(const uint8_t* data, long size, int* width, int* height, int* channels, uint8_t* rgb,
                  long rgb_size);
int rt_last_error(char* buf, size_t len);

/* ---- scene ingest (host) ---- */
/* loadMesh (src/mesh.cpp:58-188) with Assimp 5.0.1 OBJ semantics; appends the meshes to scene.
 * assimp3_compat: 0 for 5.0.1 (the reference's pinned version), or bits of Assimp 3.x behaviour that 5.0.1
 * is believed to have dropped: shininess = 4 x Ns, and GenNormals face normals
 * normalised by division (x / |n|) instead of by the reciprocal (x * (1 / |n|)). */
#define RT_ASSIMP3_SHININESS_X4 1
#define RT_ASSIMP3_NORMALS_DIV 2
int rt_scene_new(rt_scene** out);
int rt_scene_load_obj(rt_scene* scene, const char* path, int normalize, int assimp3_compat);
/* loadScene presets (src/scene.cpp:4-150).  preset: SceneType enum value (src/scene.h:14-34). */
int rt_scene_preset(rt_scene* scene, int preset, const char* data_dir, int assimp3_compat);
int rt_scene_add_sphere(rt_scene* scene, const rt_sphere* s);
int rt_scene_add_point_light(rt_scene* scene, const rt_point_light* l);
int rt_scene_add_spherical_light(rt_scene* scene, const rt_spherical_light* l);
int rt_scene_add_spot_light(rt_scene* scene, const rt_spot_light* l);
int rt_scene_add_plane_light(rt_scene* scene, const rt_plane_light* l);
int rt_scene_clear_lights(rt_scene* scene);
int rt_scene_set_material(rt_scene* scene, int mesh, const rt_material* m);
/* The meshes as loadMesh returns them (src/mesh.h:14-44): per mesh its vertices {p, n, texCoord},
 * its triangles (vertex index triplets) and its material; `texture` indexes rt_scene_desc.textures
 * (-1: none) and texture_path names the file.  Pointers stay valid until the scene is modified or
 * freed. */
typedef struct rt_mesh_view {
    int num_vertices;
    int num_triangles;
    const float* vertices;      /* [num_vertices][8]: p.xyz, n.xyz, texCoord.xy */
    const uint32_t* triangles;  /* [num_triangles][3] */
    rt_material material;
    const char* texture_path;   /* "" without a kd texture */
} rt_mesh_view;
int rt_scene_mesh_count(const rt_scene* scene, int* n);
int rt_scene_mesh_get(const rt_scene* scene, int mesh, rt_mesh_view* out);
/* Flat view (pointers stay valid until the scene is modified or freed). */
int rt_scene_desc_get(const rt_scene* scene, rt_scene_desc* out);
int rt_scene_free(rt_scene* scene);
/* Deterministic 800k-triangle (2,3) torus-knot stand-in for the missing data/dragon.obj. */
int rt_write_dragon_proxy(const char* obj_path, int u_segments, int v_segments);

/* ---- camera ---- */
int rt_camera_from_trackball(const float look_at[3], const float euler_radians[3], float distance,
                             float fovy_radians, float aspect, rt_camera* out);

/* ---- device context ---- */
/* Number of visible HIP devices (initialises this library's HIP runtime); RT_ERR_NO_DEVICE (n = 0)
 * without a GPU.  In a process that also hosts PyTorch's bundled copy of the HIP runtime, let
 * torch initialise the GPU before this library is loaded (rt_amd.py does; the other order leaves
 * one of the two runtimes without a device). */
int rt_device_count(int* n);
/* BoundingVolumeHierarchy(Scene*) over devices[0..ndev): a whole scene replica (acceleration structures
 * built on that device) per entry, peer access from every other device to devices[0] where the node has
 * it.  A device without peer access does not fail the create: its part of every split render is rendered
 * band-dense on that device and copied to devices[0] (hipMemcpyPeerAsync + one scatter launch). */
int rt_create(const rt_scene_desc* desc, const int* devices, int ndev, rt_ctx** out);
/* The context's device list into out (up to n entries); returns ndev. */
int rt_ctx_devices(rt_ctx* ctx, int* out, int n);
/* Per replica: 1 if its kernels store pixels straight into devices[0]'s images (peer access), 0 if it
 * renders band-dense and copies (no peer access, or RT_OPT_PEER_STORES 0); returns ndev. */
int rt_ctx_peer_stores(rt_ctx* ctx, int* out, int n);
int rt_destroy(rt_ctx* ctx);

/* Whole frame to host memory: rgb_out = W*H*3 floats in Screen::m_textureData order (every device of
 * the context renders its bands). */
int rt_render(rt_ctx* ctx, const rt_camera* cam, const rt_params* params, int width, int height,
              float* rgb_out, rt_stats* stats);

/*
 * Band-partitioned render into DEVICE memory on a caller stream (hipStream_t or NULL).
 * The image is cut into bands of band_rows rows (from y = 0); this call renders the bands
 * b with b % band_count == band_rank and writes them densely, band after band, into
 * d_rgb_out ([n_local_bands][band_rows][width][3] floats, row r of a band = image row y in
 * reference y order, i.e. before the setPixel flip).  The host gathers and un-permutes.
 */
int rt_render_device(rt_ctx* ctx, const rt_camera* cam, const rt_params* params, int width,
                     int height, int band_rows, int band_rank, int band_count, float* d_rgb_out,
                     void* stream, rt_stats* stats);
/*
 * View batch: n_views frames of the same scene (one camera each, e.g. a turntable or a multi-view
 * capture) in ONE launch -- a sequence of renderRayTracing calls (src/main.cpp:340-400), one per
 * camera change of the trackball (framework/src/trackball.cpp:87-98).  The persistent job queue
 * spans every view, so the drain tail of one frame overlaps the start of the next.  d_rgb_out
 * holds n_views rt_render_device buffers back to back, each padded to the band count of the
 * busiest rank: view v at v * ceil(nbands / band_count) * band_rows * width * 3 floats, so the ranks'
 * buffers gather into one array for rt_unpermute_views_device.  View v's bands are bit-identical to
 * rt_render_device with cams[v].  Stats are summed over the views.  n_views == 1 is
 * rt_render_device.
 */
int rt_render_views_device(rt_ctx* ctx, const rt_camera* cams, int n_views, const rt_params* params,
                           int width, int height, int band_rows, int band_rank, int band_count,
                           float* d_rgb_out, void* stream, rt_stats* stats);
/* View batch to host memory: rgb_out = n_views frames of W*H*3 floats, each in Screen::m_textureData
 * order (the rt_render layout), view v at v*W*H*3.  Same kernel and results as
 * rt_render_views_device; stats summed over the views (and devices). */
int rt_render_views(rt_ctx* ctx, const rt_camera* cams, int n_views, const rt_params* params, int width,
                    int height, float* rgb_out, rt_stats* stats);
/*
 * The frames' pixels straight into their final place: view v's pixel (x, y) at
 * d_images[v*W*H*3 + ((H-1-y)*W + x)*3] (Screen::setPixel, src/screen.cpp:32-38).  Renders the bands
 * b % band_count == band_rank (0, 1: the whole frame) split further over the context's devices
 * (b / band_count % ndev picks the device).  d_images is device memory of devices[0] -- or of another
 * process's GPU opened with rt_ipc_open (one process per GPU: each rank passes its own band_rank and
 * rank 0's images, and the exchange is the kernels' pixel stores over xGMI).  Asynchronous on the
 * caller's stream unless stats is given; bit-identical to rt_render_views.
 */
int rt_render_views_image_device(rt_ctx* ctx, const rt_camera* cams, int n_views, const rt_params* params, int width,
                                 int height, int band_rows, int band_rank, int band_count, float* d_images,
                                 void* stream, rt_stats* stats);

/* Un-permute gathered band buffers ([band_count][max_local_bands][band_rows][W][3]) into the
 * setPixel layout on the device. */
int rt_unpermute_bands_device(int width, int height, int band_rows, int band_count,
                              const float* d_gathered, float* d_image, void* stream);

/* Un-permute a view batch gathered from band_count ranks -- each rank's rt_render_views_device
 * buffer ([n_views][max_local_bands][band_rows][W][3]) back to back, rank after rank -- into n_views
 * images of W*H*3 floats in the setPixel layout (the multi-GPU tile split of a batch; one launch). */
int rt_unpermute_views_device(int width, int height, int band_rows, int band_count, int n_views,
                              const float* d_gathered, float* d_images, void* stream);

/* Per-ray entry points used by the facade and the parity tests (host buffers). */
int rt_intersect(rt_ctx* ctx, const rt_ray* rays, int n, int use_bvh, rt_hit* hits);
int rt_shade(rt_ctx* ctx, const rt_ray* rays, int n, const rt_params* params, float* rgb,
             uint64_t* rays_per_sample);
/* Image::getPixel (src/image.cpp:77-110) of texture `texture` for n (u, v, lod) triples, under the
 * params' texture_filtering / out_of_bounds rules / border colour: rgb = n * 3 floats. */
int rt_texture_sample(rt_ctx* ctx, int texture, int n, const float* uv_lod, const rt_params* params, float* rgb);

/* Edits after upload.  rt_update_lights replaces the context's four light arrays with desc's (only
 * the light fields of desc are read).  rt_update_materials replaces every mesh material and every
 * sphere material (counts must match the scene; texture bindings are fixed at rt_create). */
int rt_update_lights(rt_ctx* ctx, const rt_scene_desc* desc);
int rt_update_materials(rt_ctx* ctx, int num_meshes, const rt_material* materials, int num_spheres,
                        const rt_material* sphere_materials);

/* Counting build of the same kernel (node visits, triangle records, hits, UB-regime hits) for
 * roofline accounting (process-wide switch). */
int rt_set_counting(int on);
/* Developer counters of the last counting launch (up to 32 words; [8..11] state-machine / traversal clocks,
 * [16..18] node re-visits of popped stack groups, their slots, their slots still hit; [19] / [20] the opaque
 * kernel's reference-box tests of candidate culling per lane / per wave step, [21..23] its lane iterations held to a
 * record test with a node to visit, with both a node visit and a record test, and in all; [24] / [25] the first
 * out-of-range index of a checked build (code << 32 | value) and their count; [32..49] the last wavefront render's
 * path-ray hits per recursion level, of its last chunk of camera jobs). */
int rt_debug_counters(rt_ctx* ctx, uint64_t* out, int n);
/* Context options: test and developer hooks (the library reads no environment variables).  The
 * defaults are the shipped path; every setting renders the same image and ray count. */
#define RT_OPT_KERNEL 1      /* RT_KERNEL_AUTO (by scene size), _WHOLE_TRAVERSAL or _DYNAMIC_FETCH */
#define RT_OPT_COOP 2        /* drain lane groups: -1 by render shape, 0 off, 1 drain only, 2 + full-wave stragglers */
#define RT_OPT_COOP_MAX 3    /* most queries handed to lane groups (0: as many as the LDS pool allows) */
#define RT_OPT_REFILL 4      /* dynamic-fetch kernel: waiting lanes that end a traversal phase (0: by shape) */
#define RT_OPT_WAVE_TRACE 5  /* 1: record rt_debug_wave_trace data; 2: also rt_debug_phase_trace */
#define RT_OPT_VARIANT 6     /* developer A/B: compiled kernel variant (rt_megakernel.hip RT_V_*), -1 default */
#define RT_OPT_FAN_CAP 9     /* fan renders: pixels a wave may have waiting on fans before it takes no new ones (0: default 16) */
#define RT_OPT_INTERLEAVE 8  /* job -> pixel order: -1 by render shape, 0 8x8 tiles per wave, 1 one pixel of each of 64 tiles per wave, k = 2..5 64 / 2^k pixels of each of 2^k tiles */
#define RT_OPT_FAN 7         /* dynamic-fetch kernel, opaque scenes: spherical-light samples as wave-shared fans (1, default) or per lane (0) */
#define RT_OPT_DUAL_STEP 10  /* dynamic-fetch kernel: a lane testing leaf records also visits its next node in the same step (-1 default = 1, 0 off) */
#define RT_OPT_CENTRE_FIRST 12 /* job order: the per-XCD tile ranges above the image centre walked bottom-up, so every range starts at its rows nearest the centre: -1 by render shape, 0 off, 1 on */
#define RT_OPT_OPAQUE 11     /* opaque-scene kernel (opaque materials, point / spot lights, no lobes or textures): -1 where eligible (the 4-wave build; with one light, its SPLIT form: shadow segments traced beside the mirror chain), 0 never, 1 the 4-wave build without SPLIT, 2 the 3-wave build, 3 the 4-wave build with the re-visit group stack, 4 / 5 SPLIT at 4 / 3 waves, 6 / 7 SPLIT without drain lane groups at 5 / 4 waves (A/Bs; SPLIT options fall back to 1 on scenes with more lights) */
#define RT_OPT_TREE 13       /* recursion-tree kernel (transparent materials, all four light types with <= 64-sample fans, no lobes or textures): -1 / 2 where eligible (4-wave build for view batches, 3-wave for single frames), 0 never, 1 its build with the re-visit group stack (A/B), 3 a checked 4-wave build (developer diagnosis: out-of-range indices reported in rt_debug_counters [24] / [25] instead of accessed), 4 / 5 the 4- / 3-wave build for every render */
#define RT_OPT_PEER_STORES 14 /* split renders: -1 the replicas with peer access to devices[0] store their pixels straight into its images (default), 0 every replica renders band-dense on its own device and copies (the path of devices without peer access) */
#define RT_OPT_INTERLEAVE_TAIL 15 /* opaque-kernel view batches: the last n views' jobs spread over 16 tiles per wave (the launch's drain), the others in tile order; 0 none (the default: measured slower) */
#define RT_OPT_WAVEFRONT 16   /* opaque-kernel scenes with one camera sample per pixel: -1 (default) and 0 the persistent opaque megakernel (no render shape is faster on the wavefront path), 1 the wavefront path (rt_wavefront.hip: a lean trace kernel per recursion level and an elementwise shade kernel between; bit-identical images), 2..64 the wavefront path with this trace-kernel refill threshold (A/B) */
#define RT_OPT_WF_BUILD 17   /* wavefront trace kernel build (A/B): 0 5 waves per SIMD (default), 1 6 waves, 2 4 waves with the node prefetch, 3 8 waves, 4 5 waves with a dual step's node and record loads in flight together, 5 the same at 4 waves */
#define RT_OPT_WF_STREAMS 18 /* wavefront path: streams its chunks of camera jobs are spread over (0: 2, the default; 1..4), so one chunk's small recursion levels overlap another's busy ones */
#define RT_OPT_PRIO 19       /* opaque-scene kernel: a traversal phase raises its wave's issue priority (s_setprio 2) after this many iterations, so the waves holding the slowest queries issue first (-1 by render shape, 0 never) */
#define RT_OPT_WF_CHUNK 20   /* wavefront path: camera jobs per chunk at most, a multiple of 64 (0: the memory budget's, the default; chunks are also capped below 2^27 jobs, the segment tag's shading-point field) */
#define RT_KERNEL_AUTO 0
#define RT_KERNEL_WHOLE_TRAVERSAL 1
#define RT_KERNEL_DYNAMIC_FETCH 2
int rt_ctx_set_option(rt_ctx* ctx, int option, int value);
/* Developer wave trace of the last persistent-kernel launch made with RT_OPT_WAVE_TRACE = 1: 8 words
 * per wave (start, end, jobs taken, time the job queue ran dry for it, drain iterations, sum of
 * tracing lanes over them, 0, drain state-machine passes); timestamps of
 * the 100 MHz device clock.  Out holds 8 * max_waves words.  Returns the wave count. */
int rt_debug_wave_trace(rt_ctx* ctx, uint64_t* out, int max_waves);
/* ... and per job (pixel) of that launch: 3 words (start, end, queries of the job); out holds
 * 3 * max_jobs words.  Returns the job count. */
int rt_debug_job_trace(rt_ctx* ctx, uint64_t* out, int max_jobs);
/* ... and with RT_OPT_WAVE_TRACE = 2 (the opaque kernel's counting build), the wave's first RT_PHASE_EV traversal
 * phases: 2 words each (start | tracing lanes << 48, end | traversal iterations << 40 | lane groups << 63; start
 * and end relative to the wave's start, rt_debug_wave_trace word 0);
 * out holds 2 * RT_PHASE_EV * max_waves words.  Returns the wave count. */
#define RT_PHASE_EV 512
int rt_debug_phase_trace(rt_ctx* ctx, uint64_t* out, int max_waves);
/* rt_create's phase clock, cumulative ms (device, reference BVH, BVH2/BVH8, records, materials and
 * textures, uploads, total): up to n doubles. */
int rt_debug_create_ms(rt_ctx* ctx, double* out, int n);
/* Where rt_create builds the acceleration structures (replaces BoundingVolumeHierarchy's constructor,
 * src/bounding_volume_hierarchy.cpp:5-9,108-217): 0 (default) on the GPU from 65 536 triangles, on
 * the host below; 1 always on the host; 2 always on the GPU (rt_create fails if the GPU path declines
 * the scene).  Process-wide; applies to later rt_create calls. */
int rt_set_build_mode(int mode);
/* The context's build: out[0] 1 = built on the GPU, out[1] BVH2 nodes, out[2] BVH2 depth,
 * out[3] BVH8 nodes (up to n ints). */
int rt_debug_build_info(rt_ctx* ctx, int* out, int n);
/* Triangle records [first, first + count) as the kernels read them: 16 floats each (v0, n.x, v1, n.y,
 * v2, n.z, D, then scene index / reference-BVH key / reference leaf as int bits). */
int rt_debug_records(rt_ctx* ctx, float* out, int first, int count);
/* The reference depth-4 BVH the kernels use (constructBVH, src/bounding_volume_hierarchy.cpp:108-217),
 * read back from the device: node boxes [nref][6] (lower, upper; BFS creation order), per node its leaf id
 * or -1, per object (triangles in scene order, then spheres) its leaf id and depth-first visit key (a
 * leaf's stored object list = its objects by key).  Null outputs are skipped; returns nref. */
int rt_debug_ref_bvh(rt_ctx* ctx, float* boxes, int* node_leaf, int* obj_leaf, int* obj_key);
/* Self-check of the kernels' reference slab test (src/ray_tracing.cpp:213-264), no context needed: for n
 * (box [lo, hi], ray [origin, normalised direction]) pairs, out[i] = the IEEE-quotient answer (bit 0) |
 * the quotient-bound answer << 1 (0 miss, 1 hit, 2 left to the IEEE quotients); device 0. */
int rt_debug_slab_check(const float* boxes, const float* rays, int n, int* out);

/* Introspection for tests / roofline accounting. */
int rt_ctx_info(rt_ctx* ctx, int* num_nodes, int* num_tri_records, int* ref_bvh_nodes,
                int* ref_bvh_levels);
/* Device math self-test: out[i] = {sqrtf(x), 1/x, x/y, powf(x,y)} bits for parity of the math lib. */
int rt_selftest_math(rt_ctx* ctx, const float* x, const float* y, int n, float* out);

/* Philox-4x32-10 (the glossy-lobe stream that replaces rand(), src/main.cpp:234-235): the same
 * host/device function the kernels call, exported for known-answer tests. */
int rt_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* ---- device memory shared between processes (one process per GPU) --------------------------------
 * rt_ipc_alloc: hipMalloc on `device` + its IPC handle (RT_IPC_HANDLE_BYTES bytes) for other processes;
 * rt_ipc_open: map another process's buffer into this one (peer access from `device`); rt_ipc_close
 * unmaps it; rt_device_free frees an rt_ipc_alloc buffer; rt_device_synchronize waits for every
 * stream of a device.  rt_ipc_alloc refuses (RT_ERR_INVALID) buffers of 2 GiB or more: on this ROCm the
 * importer's hipIpcOpenMemHandle never returns for them. */
#define RT_IPC_HANDLE_BYTES 64
int rt_ipc_alloc(int device, size_t bytes, void** d_ptr, uint8_t handle[RT_IPC_HANDLE_BYTES]);
int rt_ipc_open(int device, const uint8_t handle[RT_IPC_HANDLE_BYTES], void** d_ptr);
int rt_ipc_close(void* d_ptr);
int rt_device_free(int device, void* d_ptr);
int rt_device_synchronize(int device);
/* Synchronous copy of `bytes` from device memory (this library's, e.g. an rt_ipc_alloc buffer) to host. */
int rt_memcpy_dtoh(void* host, const void* d_ptr, size_t bytes);

/* ---- Screen post-processing (src/screen.cpp) ------------------------------------------------
 * Settings of class Screen (src/screen.h:58-111), raw values as the GUI passes them to the
 * setters; the setters' clamps (setKernelNumRepetitions >= 1, setSigma >= 0.001) are applied
 * inside, and setFilterSize keeps the raw value (its clamp hits a local, src/screen.cpp:212-215).
 * Images are W*H*3 floats in Screen::m_textureData order (top row first).                      */
enum { RT_BLOOM_NONE = 0, RT_BLOOM = 1, RT_BLOOM_REINHARD = 2, RT_BLOOM_EXPOSURE = 3, RT_BLOOM_ONLY_LIGHT = 4,
       RT_BLOOM_ONLY_LIGHT_KERNEL = 5 };                  /* enum class FilteringOption */
enum { RT_KERNEL_BOX = 0, RT_KERNEL_GAUSSIAN = 1 };      /* enum class Kernel */
typedef struct rt_post_params {
    int filtering_option;   /* setBloomFilter */
    int kernel;             /* setKernel */
    int repetitions;        /* setKernelNumRepetitions (raw) */
    int filter_size;        /* setFilterSize (raw) */
    float sigma;            /* setSigma (raw) */
    float exposure;         /* setExposure */
    int gamma_correction;   /* enableGammaCorrection */
    float gamma;            /* setGammaValue */
    int bloom_live;         /* setBloomFilterLive */
    int pad_;
} rt_post_params;

/* Screen::postprocessImage (src/screen.cpp:56-69): bloom if bloom_live, then gamma if enabled.
 * d_rgb is read and written in place; d_scratch holds 2*W*H*3 floats (bloom temporaries). */
int rt_postprocess_device(const rt_post_params* p, int width, int height, float* d_rgb, float* d_scratch,
                          void* stream);
/* Screen::writeBitmapToFile's pixel path (src/screen.cpp:40-54): applyBloomEffect on d_rgb (in
 * place, as the reference mutates m_textureData), then clamp to [0,1] and truncate *255 into
 * RGBA8 (alpha 255). */
int rt_bitmap_device(const rt_post_params* p, int width, int height, float* d_rgb, float* d_scratch,
                     uint8_t* d_rgba8, void* stream);
/* Host-buffer forms of the two above (synchronous, device 0 of the caller's current device). */
int rt_postprocess(const rt_post_params* p, int width, int height, float* rgb);
int rt_bitmap(const rt_post_params* p, int width, int height, float* rgb, uint8_t* rgba8);
/* stbi_write_bmp as the reference calls it (comp 4): 24-bit BMP, bottom-up rows, alpha dropped.
 * rt_encode_bmp writes into out (size >= 54 + (3W + pad) * H) and returns the byte count. */
long rt_encode_bmp(int width, int height, const uint8_t* rgba8, uint8_t* out, long out_size);
int rt_write_bmp(const char* path, int width, int height, const uint8_t* rgba8);

#ifdef __cplusplus
}
#endif
#endif /* RT_AMD_H */
