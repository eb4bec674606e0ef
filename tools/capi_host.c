/* A host program in plain C on the C ABI alone (include/octpt.h, liboctpt.so): what a non-Python host --
 * the Rust RenderingBackend shim of INTEGRATION.md §3, through its extern "C" block -- does to render.
 * It builds a small sphere scene with the library's host octree builder (octpt_build_octree), uploads it
 * (octpt_scene_upload, as GPURenderer::set_scene, gpu_renderer.rs:662-669), sets the camera, renders a
 * progressive frame synchronously (octpt_render) and continues it asynchronously (octpt_render_async +
 * octpt_frame_poll / octpt_frame_wait, FrameInFlight, renderer_trait.rs:30-46), runs a closest-hit batch
 * (octpt_intersect, Scene::hit) and reads the statistics.  The frame is written to OUT as raw float32 RGBA
 * (W * H * 4) followed by the per-ray hit records, for tests/test_gpu_capi_host.py to compare with the
 * same scene rendered through the Python bindings and with the CPU oracle.
 * With a second argument REFOUT it also runs the Rust shim's own set_scene sequence of INTEGRATION.md §3 in C
 * (run_reference below): a block-value world in the reference writer's form (octant children as bit i + 8 alone,
 * children before parents, the root last, LOD leaves where eight equal blocks compact), the reference's Material
 * list with a colour and an image texture, octpt_scene_from_reference -> octpt_scene_upload, a frame through
 * octpt_render_async / poll / wait / release, and the same frame through a two-entry context
 * (octpt_create_multi over [0, 0]).  REFOUT gets the scene it built and both frames.
 * Usage: capi_host OUT [REFOUT] (exit 0 on success; 2 = no gfx950 device).  Built by __graft_entry__.build(). */
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

/* ---- the reference-scene sequence ---------------------------------- */
enum { RDEPTH = 4, RN = 1 << RDEPTH, RW = 96, RH = 64, RSPP = 4, NMAT = 5, NBLK = 4, IMG = 4, MAXOCT = 1024 };

/* cell (x, y, z) of the 16^3 world: 0 = air, else block id + 1 (grass 0, dirt 1, stone 2, glass pane 3) */
static uint32_t world_cell(int x, int y, int z) {
    const int h = 4 + (x * 3 + z * 5) % 6 + ((x >= 8 && z >= 8) ? 3 : 0);
    if (y >= h) return (x == 3 && y == h && z > 2 && z < 12) ? 4u : 0u;
    if (y == h - 1) return 1u;
    if (y >= h - 3) return 2u;
    return 3u;
}

typedef struct {
    octpt_octant o[MAXOCT];
    uint32_t n;
} RefTree;

/* SectionOctantBuilder's form (new_octree.rs:599-710): children pushed before their parent, Octant::set_mask_for's
 * encoding (a leaf = bits i and i + 8, an octant = bit i + 8 alone, :160-178), and Octant::is_compactable's merge
 * (:227-233) of eight leaves holding one value into a leaf of the parent (the root is never merged).
 * Returns 0 empty, 1 leaf (*payload = block), 2 octant (*payload = its index). */
static int build_ref(RefTree *t, int level, int x0, int y0, int z0, uint32_t *payload) {
    if (level == 0) {
        const uint32_t v = world_cell(x0, y0, z0);
        if (!v) return 0;
        *payload = v - 1u;
        return 1;
    }
    const int half = 1 << (level - 1);
    int kind[8];
    uint32_t pay[8];
    int leaves = 0, empty = 0;
    for (int i = 0; i < 8; ++i) {
        kind[i] = build_ref(t, level - 1, x0 + (i & 1) * half, y0 + ((i >> 1) & 1) * half, z0 + ((i >> 2) & 1) * half,
                            &pay[i]);
        leaves += kind[i] == 1;
        empty += kind[i] == 0;
    }
    if (empty == 8) return 0;
    if (leaves == 8 && level < RDEPTH) {
        int same = 1;
        for (int i = 1; i < 8; ++i) same &= pay[i] == pay[0];
        if (same) {
            *payload = pay[0];
            return 1;
        }
    }
    if (t->n >= MAXOCT) return -1;
    octpt_octant *o = &t->o[t->n];
    memset(o, 0, sizeof *o);
    for (int i = 0; i < 8; ++i) {
        if (kind[i] < 0) return -1;
        if (kind[i] == 1) o->child_mask |= (uint16_t)((1u << i) | (1u << (i + 8)));
        if (kind[i] == 2) o->child_mask |= (uint16_t)(1u << (i + 8));
        o->children[i] = kind[i] ? pay[i] : 0u;
    }
    *payload = t->n++;
    return 2;
}

static void put_u32(FILE *f, uint32_t v) { fwrite(&v, 4, 1, f); }

static int run_reference(const char *path, const octpt_sun *sun) {
    static RefTree t;
    uint32_t root = 0;
    if (build_ref(&t, RDEPTH, 0, 0, 0, &root) != 2) return 1;
    /* the reference's Material list (material.rs:91-101): air, grass, dirt, stone, and a glass pane whose image has
     * alpha-0 texels (the traversal passes through them, C23) */
    static uint8_t img[IMG * IMG * 4];
    for (int y = 0; y < IMG; ++y)
        for (int x = 0; x < IMG; ++x) {
            const int edge = x == 0 || y == 0 || x == IMG - 1 || y == IMG - 1;
            uint8_t *px = &img[4 * (y * IMG + x)];
            px[0] = 200; px[1] = 225; px[2] = 235; px[3] = edge ? 255 : 0;
        }
    octpt_reference_material m[NMAT];
    memset(m, 0, sizeof m);
    const uint8_t col[NMAT][4] = {{255, 0, 255, 255}, {90, 160, 60, 255}, {130, 90, 60, 255}, {120, 120, 125, 255},
                                  {0, 0, 0, 0}};
    for (int i = 0; i < NMAT; ++i) {
        m[i].index_of_refraction = 1.000293f;
        m[i].material_flags = i ? (0x1u | 0x10u) : 0u; /* Material::AIR, then MaterialBuilder's OPAQUE | SOLID */
        m[i].texture_kind = OCTPT_TEXTURE_COLOR;
        memcpy(m[i].color, col[i], 4);
    }
    m[4].texture_kind = OCTPT_TEXTURE_IMAGE;
    m[4].image_width = m[4].image_height = IMG;
    m[4].image_rgba = img;
    /* the host's block table: block value -> face materials W, E, Bottom, Top, South, North */
    octpt_block blk[NBLK];
    const uint32_t faces[NBLK][6] = {{1, 1, 2, 1, 1, 1}, {2, 2, 2, 2, 2, 2}, {3, 3, 3, 3, 3, 3}, {4, 4, 4, 4, 4, 4}};
    for (int b = 0; b < NBLK; ++b) {
        memcpy(blk[b].face_material, faces[b], sizeof faces[b]);
        blk[b].model = OCTPT_MODEL_NONE;
        blk[b].reserved = 0;
    }
    octpt_reference_scene rs;
    memset(&rs, 0, sizeof rs);
    rs.octants = t.o;
    rs.octant_count = t.n;
    rs.root = root;
    rs.depth = RDEPTH;
    rs.blocks = blk;
    rs.block_count = NBLK;
    rs.materials = m;
    rs.material_count = NMAT;
    rs.sun = *sun;
    rs.emitters_enabled = 1;
    rs.f_sub_surface = 0.3f;
    octpt_material mo[NMAT];
    octpt_texture to[NMAT];
    octpt_quad qo[1];
    octpt_scene_desc d;
    if (octpt_scene_from_reference(&rs, mo, to, qo, &d) != OCTPT_OK) {
        fprintf(stderr, "octpt_scene_from_reference failed\n");
        return 1;
    }
    /* camera: from above the world's (-x, -z) corner towards its middle */
    const float pi = 3.14159265358979323846f;
    octpt_camera cam;
    memset(&cam, 0, sizeof cam);
    const float eye[3] = {-7.0f, 21.0f, -9.0f}, at[3] = {8.0f, 6.0f, 8.0f};
    float dir[3] = {at[0] - eye[0], at[1] - eye[1], at[2] - eye[2]};
    const float dn = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    for (int i = 0; i < 3; ++i) dir[i] /= dn;
    /* up = the world's +y made orthogonal to dir, normalised */
    float up[3] = {-dir[1] * dir[0], 1.0f - dir[1] * dir[1], -dir[1] * dir[2]};
    const float un = sqrtf(up[0] * up[0] + up[1] * up[1] + up[2] * up[2]);
    for (int i = 0; i < 3; ++i) {
        up[i] /= un;
        cam.eye[i] = eye[i];
        cam.direction[i] = dir[i];
        cam.up[i] = up[i];
    }
    cam.fov = 70.0f * (pi / 180.0f);
    octpt_render_params p;
    memset(&p, 0, sizeof p);
    p.width = RW;
    p.height = RH;
    p.spp_count = RSPP;
    p.max_depth = 5;
    p.branch_count = 1;
    p.seed = 1;
    p.shard_count = 1;
    static float acc1[RW * RH * 4], acc2[RW * RH * 4];
    static uint8_t rgba[RW * RH * 4];
    for (int i = 0; i < RW * RH; ++i) {
        acc1[4 * i] = acc1[4 * i + 1] = acc1[4 * i + 2] = 0.0f;
        acc1[4 * i + 3] = 1.0f;
    }
    memcpy(acc2, acc1, sizeof acc1);
    /* one context: the RenderingBackend's set_scene / set_camera / render_frame + FrameInFlight */
    octpt_ctx *ctx = NULL;
    if (octpt_create(0, &ctx) != OCTPT_OK) return 2;
    CHECK(ctx, octpt_scene_upload(ctx, &d));
    CHECK(ctx, octpt_set_camera(ctx, &cam));
    octpt_frame *f = NULL;
    CHECK(ctx, octpt_render_async(ctx, &p, acc1, rgba, &f));
    octpt_status st;
    while ((st = octpt_frame_poll(f)) == OCTPT_NOT_READY) {
    }
    if (st != OCTPT_OK || octpt_frame_wait(f) != OCTPT_OK) {
        fprintf(stderr, "reference async frame: %d (%s)\n", st, octpt_last_error(ctx));
        return 1;
    }
    octpt_frame_release(f);
    octpt_stats s1;
    CHECK(ctx, octpt_get_stats(ctx, &s1));
    octpt_destroy(ctx);
    /* the node's GPUs as one context (here the one GPU twice): the same scene, the same frame */
    const int32_t devs[2] = {0, 0};
    octpt_ctx *mctx = NULL;
    if (octpt_create_multi(devs, 2, &mctx) != OCTPT_OK) return 1;
    if (octpt_device_entries(mctx) != 2) return 1;
    CHECK(mctx, octpt_scene_upload(mctx, &d));
    CHECK(mctx, octpt_set_camera(mctx, &cam));
    CHECK(mctx, octpt_render(mctx, &p, acc2, NULL));
    octpt_stats s2;
    CHECK(mctx, octpt_get_stats(mctx, &s2));
    octpt_destroy(mctx);

    FILE *out = fopen(path, "wb");
    if (!out) return 1;
    const uint32_t head[8] = {t.n, root, RDEPTH, NBLK, NMAT, IMG, IMG, RSPP};
    fwrite(head, 4, 8, out);
    for (uint32_t i = 0; i < t.n; ++i) put_u32(out, t.o[i].child_mask);
    for (uint32_t i = 0; i < t.n; ++i) fwrite(t.o[i].children, 4, 8, out);
    for (int b = 0; b < NBLK; ++b) fwrite(blk[b].face_material, 4, 6, out);
    for (int i = 0; i < NMAT; ++i) {
        const float fl[5] = {m[i].index_of_refraction, m[i].specular, m[i].emittance, m[i].roughness, m[i].metalness};
        fwrite(fl, 4, 5, out);
        put_u32(out, m[i].material_flags);
        put_u32(out, m[i].texture_kind);
        fwrite(m[i].color, 1, 4, out);
    }
    fwrite(img, 1, sizeof img, out);
    fwrite(cam.eye, 4, 3, out);
    fwrite(cam.direction, 4, 3, out);
    fwrite(cam.up, 4, 3, out);
    fwrite(&cam.fov, 4, 1, out);
    fwrite(acc1, 4, RW * RH * 4, out);
    fwrite(acc2, 4, RW * RH * 4, out);
    fwrite(rgba, 1, sizeof rgba, out);
    const uint64_t c[6] = {s1.paths, s1.segments, s1.block_tests, s2.paths, s2.segments, s2.block_tests};
    fwrite(c, 8, 6, out);
    fclose(out);
    printf("capi_host reference sequence OK: %u octants (root %u), %llu segments, %llu block tests\n", t.n, root,
           (unsigned long long)s1.segments, (unsigned long long)s1.block_tests);
    return 0;
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
    return argc > 2 ? run_reference(argv[2], &d.sun) : 0;
}
