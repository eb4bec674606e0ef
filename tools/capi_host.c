/* A host program in plain C on the C ABI alone (include/octpt.h, liboctpt.so): what a non-Python host --
 * the Rust RenderingBackend shim of INTEGRATION.md §3, through its extern "C" block -- does to render.
 * It builds a small sphere scene with the library's host octree builder (octpt_build_octree), uploads it
 * (octpt_scene_upload, as GPURenderer::set_scene, gpu_renderer.rs:662-669), sets the camera, renders a
 * progressive frame synchronously (octpt_render) and continues it asynchronously (octpt_render_async +
 * octpt_frame_poll / octpt_frame_wait, FrameInFlight, renderer_trait.rs:30-46), runs a closest-hit batch
 * (octpt_intersect, Scene::hit) and reads the statistics.  The frame is written to OUT as raw float32 RGBA
 * (W * H * 4) followed by the per-ray hit records, for tests/test_gpu_capi_host.py to compare with the
 * same scene rendered through the Python bindings and with the CPU oracle.
 * Usage: capi_host OUT (exit 0 on success; 2 = no gfx950 device).  Built by __graft_entry__.build(). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/octpt.h"

enum { W = 96, H = 64, SPP_SYNC = 3, SPP_ASYNC = 2, NSPH = 24, NRAYS = 256 };

#define CHECK(ctx, call)                                                                     \
    do {                                                                                     \
        octpt_status st_ = (call);                                                           \
        if (st_ != OCTPT_OK) {                                                               \
            fprintf(stderr, "%s failed: %d (%s)\n", #call, st_, octpt_last_error(ctx));      \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

/* the scene both sides build (tests/test_gpu_capi_host.py::capi_scene mirrors it, in exact arithmetic):
 * NSPH spheres scattered over the depth-5 world [0, 32)^3, materials = air + a red and a metal one */
static void make_spheres(octpt_sphere *sp) {
    for (int i = 0; i < NSPH; ++i) {
        memset(&sp[i], 0, sizeof sp[i]);
        sp[i].center[0] = 4.0f + (float)((i * 7) % 24) + 0.25f * (float)(i % 3);
        sp[i].center[1] = 6.0f + (float)((i * 5) % 13);
        sp[i].center[2] = 6.0f + (float)((i * 11) % 20) + 0.5f * (float)(i % 2);
        sp[i].radius = 1.0f + 0.125f * (float)(i % 4);
        sp[i].material = 1u + (uint32_t)(i % 2);
    }
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: capi_host OUT\n");
        return 1;
    }
    if (octpt_device_count() <= 0) return 2;
    octpt_sphere spheres[NSPH];
    make_spheres(spheres);
    octpt_octree *tree = NULL;
    if (octpt_build_octree(spheres, NSPH, NULL, 0, 5, &tree) != OCTPT_OK) return 1;
    octpt_octree_view v;
    if (octpt_octree_get_view(tree, &v) != OCTPT_OK) return 1;

    /* Material::AIR, a diffuse red, a metal (MaterialBuilder defaults: ior 1.000293, OPAQUE | SOLID) */
    octpt_material mats[3];
    memset(mats, 0, sizeof mats);
    for (int i = 0; i < 3; ++i) mats[i].ior = 1.000293f;
    mats[0].flags = 0u;
    mats[1].texture_index = 1u;
    mats[1].flags = 0x1u | 0x10u;
    mats[2].texture_index = 2u;
    mats[2].metalness = 1.0f;
    mats[2].roughness = 0.1f;
    mats[2].flags = 0x1u | 0x10u;
    octpt_texture texs[3];
    memset(texs, 0, sizeof texs);
    const uint8_t rgba[3][4] = {{255, 0, 255, 255}, {200, 60, 40, 255}, {230, 230, 235, 255}};
    for (int i = 0; i < 3; ++i) {
        texs[i].kind = OCTPT_TEXTURE_COLOR;
        memcpy(texs[i].rgba, rgba[i], 4);
    }

    octpt_scene_desc d;
    memset(&d, 0, sizeof d);
    d.abi_version = OCTPT_ABI_VERSION;
    d.octants = v.octants;
    d.octant_count = v.octant_count;
    d.root = v.root;
    d.depth = v.depth;
    d.leaf_first = v.leaf_first;
    d.leaf_count = v.leaf_count;
    d.leaf_table_size = v.leaf_table_size;
    d.leaf_prims = v.leaf_prims;
    d.leaf_prim_count = v.leaf_prim_count;
    d.spheres = spheres;
    d.sphere_count = NSPH;
    d.materials = mats;
    d.material_count = 3;
    d.textures = texs;
    d.texture_count = 3;
    /* Sun::default (scene/mod.rs:294-307) with the IMPORTANCE sampling preset (:98-126) */
    const float pi = 3.14159265358979323846f;
    d.sun.azimuth = pi / 2.5f;
    d.sun.altitude = pi / 3.0f;
    d.sun.radius = 0.03f;
    for (int i = 0; i < 4; ++i) d.sun.color[i] = 1.0f;
    for (int i = 0; i < 3; ++i) d.sun.apparent_color[i] = 1.0f;
    d.sun.draw_texture = 1;
    d.sun.texture_modification = 0;
    d.sun.importance_sample_chance = 0.1f;
    d.sun.importance_sample_radius = 1.2f;
    d.sun.luminosity = 100.0f;
    for (int i = 0; i < 4; ++i) d.sun.texture_rgba[i] = 255;
    d.sun.importance_sampling = 1;
    d.sun.diffuse_sun = 1;
    d.sun.sun_sampling = 0;
    d.sun.strict_direct_light = 0;
    d.sun.sun_luminosity = 1;
    d.sun.luminosity_pdf = 1.0f / 100.0f;
    d.emitters_enabled = 1;
    d.f_sub_surface = 0.3f;

    octpt_ctx *ctx = NULL;
    if (octpt_create(0, &ctx) != OCTPT_OK) return 2;
    CHECK(ctx, octpt_scene_upload(ctx, &d));
    octpt_octree_free(tree); /* the upload deep-copied it */
    octpt_camera cam;
    memset(&cam, 0, sizeof cam);
    cam.eye[0] = 16.0f; cam.eye[1] = 22.0f; cam.eye[2] = -6.0f;
    cam.direction[0] = 0.0f; cam.direction[1] = -0.4472136f; cam.direction[2] = 0.8944272f;
    cam.up[0] = 0.0f; cam.up[1] = 0.8944272f; cam.up[2] = 0.4472136f;
    cam.fov = 70.0f * (pi / 180.0f);
    CHECK(ctx, octpt_set_camera(ctx, &cam));

    float *accum = (float *)malloc(sizeof(float) * 4 * W * H);
    uint8_t *rgba8 = (uint8_t *)malloc(4 * W * H);
    for (int i = 0; i < W * H; ++i) {
        accum[4 * i + 0] = accum[4 * i + 1] = accum[4 * i + 2] = 0.0f;
        accum[4 * i + 3] = 1.0f;
    }
    octpt_render_params p;
    memset(&p, 0, sizeof p);
    p.width = W;
    p.height = H;
    p.spp_start = 0;
    p.spp_count = SPP_SYNC;
    p.max_depth = 5;
    p.branch_count = 1;
    p.seed = 1;
    p.shard_index = 0;
    p.shard_count = 1;
    CHECK(ctx, octpt_render(ctx, &p, accum, NULL));
    /* the frame continued asynchronously: passes SPP_SYNC .. SPP_SYNC + SPP_ASYNC */
    p.spp_start = SPP_SYNC;
    p.spp_count = SPP_ASYNC;
    octpt_frame *f = NULL;
    CHECK(ctx, octpt_render_async(ctx, &p, accum, rgba8, &f));
    octpt_status st;
    while ((st = octpt_frame_poll(f)) == OCTPT_NOT_READY) {
    }
    if (st != OCTPT_OK || octpt_frame_wait(f) != OCTPT_OK) {
        fprintf(stderr, "async frame: %d (%s)\n", st, octpt_last_error(ctx));
        return 1;
    }
    octpt_frame_release(f);

    /* Scene::hit on a batch: rays from the eye through a grid of image points */
    float rays[NRAYS * 6];
    for (int i = 0; i < NRAYS; ++i) {
        const float x = -0.6f + 1.2f * (float)(i % 16) / 15.0f, y = -0.4f + 0.8f * (float)(i / 16) / 15.0f;
        float dx = x, dy = cam.direction[1] + y * cam.up[1], dz = cam.direction[2] + y * cam.up[2];
        const float n = sqrtf(dx * dx + dy * dy + dz * dz);
        rays[6 * i + 0] = cam.eye[0];
        rays[6 * i + 1] = cam.eye[1];
        rays[6 * i + 2] = cam.eye[2];
        rays[6 * i + 3] = dx / n;
        rays[6 * i + 4] = dy / n;
        rays[6 * i + 5] = dz / n;
    }
    float t[NRAYS];
    uint32_t prim[NRAYS], steps[NRAYS];
    CHECK(ctx, octpt_intersect(ctx, rays, NULL, NULL, NRAYS, t, prim, NULL, steps));
    octpt_stats s;
    CHECK(ctx, octpt_get_stats(ctx, &s));

    FILE *out = fopen(argv[1], "wb");
    if (!out) return 1;
    fwrite(accum, sizeof(float), 4 * W * H, out);
    fwrite(rgba8, 1, 4 * W * H, out);
    fwrite(rays, sizeof(float), NRAYS * 6, out);
    fwrite(t, sizeof(float), NRAYS, out);
    fwrite(prim, sizeof(uint32_t), NRAYS, out);
    fwrite(steps, sizeof(uint32_t), NRAYS, out);
    const uint64_t counters[3] = {s.paths, s.segments, s.esvo_steps};
    fwrite(counters, sizeof(uint64_t), 3, out);
    fclose(out);
    printf("capi_host OK: %llu paths, %llu segments\n", (unsigned long long)s.paths, (unsigned long long)s.segments);
    free(accum);
    free(rgba8);
    octpt_destroy(ctx);
    return 0;
}
