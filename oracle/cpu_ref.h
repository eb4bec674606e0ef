/*
 * oracle/cpu_ref.h -- CPU restatement ("cpu_ref") of the kekley/octree_pathtracing
 * per-pixel hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (octree_pathtracing_amd/,
 * include/octpt.h, liboctpt.so) links, loads or calls this code.  It is imported
 * only by tests/, __graft_entry__.smoke() (as the checker) and bench.py's
 * cpu_baseline leg.
 *
 * Parity status: the reference (Rust, nightly, missing ../mc_utils path dep) cannot
 * be built here and its hot path is stubbed (Scene::hit returns false,
 * Sphere::hit is todo!()).  The only golden vectors the reference's own tests
 * hold are the Morton-code tests (src/octree/new_octree.rs:866-884), which pin
 * ref_morton_*.  Everything else is a restatement of the reference code plus the
 * semantics contract in DESIGN.md §3:  PARITY UNPINNED for the path tracer
 * proper (pinned only by analytic known-answer tests in tests/).
 *
 * All geometry/shading arithmetic is IEEE f32, compiled with -ffp-contract=off;
 * transcendentals use the portable f32 math of DESIGN.md §3.11 (ref_math_*).
 */
#ifndef OCTPT_CPU_REF_H
#define OCTPT_CPU_REF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Camera, reference src/renderer/camera.rs:8-25 (eye, direction, up, fov). */
typedef struct {
    float eye[3];
    float dir[3];
    float up[3];
    float fov; /* radians */
} ref_camera;

/* Material, reference GPUMaterial layout src/gpu_structs/gpu_material.rs:67-76. */
typedef struct {
    float ior, specular, emittance, roughness, metalness;
    uint32_t texture_index, tint_index, flags;
} ref_material;

/* Texture: kind 0 = Texture::Color(U8Color) (rgba), kind 1 = Texture::Image (RGBA8,
 * w x h at pixels + offset).  reference src/textures/texture.rs:15-18. */
typedef struct {
    uint32_t kind;
    uint8_t rgba[4];
    uint32_t width, height;
    uint64_t offset; /* byte offset into the texel pool */
} ref_texture;

/* Block-model quad: geometry::quad::Quad::new arguments (src/geometry/quad.rs:90-114) in
 * voxel-local units; the same 64-byte layout as octpt_quad (include/octpt.h). */
typedef struct {
    float origin[3];
    uint32_t material;
    float u[3];
    float v[3];
    float texture_u_range[2];
    float texture_v_range[2];
    uint32_t reserved[2];
} ref_quad;

/* Sun + sampling strategy, reference src/scene/mod.rs:60-127, 271-383. */
typedef struct {
    float azimuth, altitude, radius;
    float color[4];
    float apparent_color[3];
    int32_t draw_texture, texture_modification;
    float importance_sample_chance, importance_sample_radius;
    float luminosity;
    uint8_t texture_rgba[4]; /* Sun texture is a Texture::Color */
    int32_t importance_sampling, diffuse_sun, sun_sampling;
    /* SunSamplingStrategy::{strict_direct_light, sun_luminosity} (scene/mod.rs:66-67) and
     * Sun::luminosity_pdf (:274, 376) -- the next-event-estimation presets FAST / HIGH_QUALITY */
    int32_t strict_direct_light, sun_luminosity;
    float luminosity_pdf;
} ref_sun;

typedef struct {
    /* octree, reference new_octree::Octant layout (mask: bit i = present, bit i+8 = leaf) */
    const uint16_t *octant_mask;
    const uint32_t *octant_children; /* 8 per octant */
    uint32_t n_octants, root, depth;
    /* leaf payload -> primitive list */
    const uint32_t *leaf_first, *leaf_count, *leaf_prims;
    uint32_t n_leaves;
    const float *spheres; /* cx, cy, cz, r */
    const uint32_t *sphere_material;
    uint32_t n_spheres;
    const float *cuboids; /* minx, miny, minz, maxx, maxy, maxz */
    const uint32_t *cuboid_material; /* 6 per cuboid, Face order W,E,Bottom,Top,South,North */
    uint32_t n_cuboids;
    const ref_material *materials;
    uint32_t n_materials;
    const ref_texture *textures;
    uint32_t n_textures;
    const uint8_t *texels;
    ref_sun sun;
    int32_t emitters_enabled;
    float f_sub_surface; /* Scene::f_sub_surface (scene/mod.rs:152), path_tracer.rs:237-241 */
    /* block models: cuboid_model NULL or one entry per cuboid (0xFFFFFFFF = plain
     * box); model m owns quads[model_quads[2m] .. + model_quads[2m+1]) */
    const uint32_t *cuboid_model;
    const uint32_t *model_quads;
    uint32_t n_models;
    const ref_quad *quads;
    uint32_t n_quads;
    /* block-value leaves: block_mat non-NULL = every leaf payload is a block id, the
     * reference's own leaf form (new_octree.rs:534-537, 586, 669, 727).  Block b has the face materials
     * block_mat[6b .. 6b+5] (Face order W,E,Bottom,Top,South,North) and block_model[b] (NULL or
     * 0xFFFFFFFF: the block fills its leaf cell, the SingleBlock arm of octree_traversal.rs:143-205;
     * else a block model drawn at the cell's corner, the ResourceModel::Quad arm :207-213) */
    const uint32_t *block_mat;
    const uint32_t *block_model;
    uint32_t n_blocks;
} ref_scene;

typedef struct {
    uint32_t width, height;
    uint32_t spp_start, spp_count;
    uint32_t max_depth;     /* reference hard-codes 5 (path_tracer.rs:56) */
    uint32_t branch_count;  /* TileRenderer branch count; contract default 1 */
    uint32_t seed;
    uint32_t threads;       /* CPU worker threads (TileRenderer rayon pool) */
    int32_t forward_accumulation; /* 0: recursive (reference), 1: forward (kernel order) */
    /* optional pixel subset: rows [row_begin, row_end) */
    uint32_t row_begin, row_end;
    /* 1: RendererMode::Preview -- render_tile_replace + preview_render */
    int32_t preview;
} ref_render_params;

typedef struct {
    uint64_t paths, segments, esvo_steps, node_fetches, prim_tests, leaf_visits, shade_events, texel_reads;
    uint64_t max_path_segs;
    uint64_t block_tests; /* block-value leaf tests [C23] */
} ref_stats;

/* --- math --- */
float ref_math_sin(float x);
float ref_math_cos(float x);
float ref_math_asin(float x);
float ref_math_acos(float x);
float ref_math_atan2(float y, float x);
float ref_math_hypot(float x, float y);
uint32_t ref_rng_path_state(uint32_t seed, uint32_t pixel, uint32_t sample);
uint32_t ref_rng_branch_state(uint32_t state, uint32_t b);
uint32_t ref_branch_count(uint32_t current_spp, uint32_t scene_branch_count);
float ref_rng_next(uint32_t *state);

/* --- Morton, reference new_octree.rs:752-835 --- */
uint64_t ref_morton_encode(uint64_t x, uint64_t y, uint64_t z);
uint64_t ref_morton_encode_lut(uint64_t x, uint64_t y, uint64_t z);
void ref_morton_decode(uint64_t code, uint64_t *x, uint64_t *y, uint64_t *z);
/* returns number of mismatches of encode vs encode_lut over [0,n)^3 (reference test n=1024) */
uint64_t ref_morton_lut_selftest(uint32_t n);

/* --- octree builder --- */
typedef struct {
    uint16_t *octant_mask;
    uint32_t *octant_children;
    uint32_t n_octants, root, depth;
    uint32_t *leaf_first, *leaf_count, *leaf_prims;
    uint32_t n_leaves, n_leaf_prims;
} ref_octree;
/* flags: REF_BUILD_COMPACT merges eight sibling leaves holding the same primitive list into one
 * leaf a level up, bottom-up (Octant::is_compactable, new_octree.rs:227-233) */
#define REF_BUILD_COMPACT 0x1u
int ref_build_octree(const float *spheres, uint32_t n_spheres, const float *cuboids, uint32_t n_cuboids,
                     uint32_t depth, uint32_t flags, ref_octree *out);
void ref_free_octree(ref_octree *t);

/* --- closest-hit query (Scene::hit), one ray per entry ---
 * rays: n x 6 (origin, direction). out_t: world distance or +inf; out_prim: prim id (bit31 = cuboid) or
 * 0xFFFFFFFF; out_normal: n x 3; out_steps: ESVO iterations. last_prim: self-intersection prim per ray (or NULL). */
void ref_intersect(const ref_scene *s, const float *rays, const uint32_t *last_prim, const float *last_normal,
                   uint32_t n, float *out_t, uint32_t *out_prim, float *out_normal, uint32_t *out_steps);
/* brute force over all primitives (no octree), same primitive semantics */
void ref_intersect_brute(const ref_scene *s, const float *rays, uint32_t n, float *out_t, uint32_t *out_prim);
/* Quad::hit (quad.rs:172-200) of one quad for n rays (n*6 floats) at voxel position `voxel`, with
 * t_next = +inf: out n*3 floats (t, alpha, beta), hit flags n bytes.  KAT hook for tests. */
void ref_quad_hit(const ref_quad *q, const float *rays, const float voxel[3], uint32_t n, float *out, uint8_t *hit);

/* --- render: progressive running mean (TileRenderer::render_tile_average) ---
 * accum: W*H*4 floats, in/out (initialise to F32Color::BLACK = 0,0,0,1).
 * seg_count (optional, W*H u32): per-pixel ray segments this call. */
int ref_render(const ref_scene *s, const ref_camera *cam, const ref_render_params *p, float *accum,
               uint32_t *seg_count, ref_stats *stats);

/* Octree::get_traversal_data (octree_traversal.rs:537-714): beam-start octant, scale, stacks */
void ref_traversal_data(const ref_scene *s, const float ray[6], float max_dst_w, uint32_t *start, uint32_t *scale,
                        uint32_t index_stack[24], float time_stack[24]);

/* tone map, colors/mod.rs:408-420 (LUT texture.rs:55-62) */
void ref_tonemap(const float *accum, uint32_t n_pixels, uint8_t *out_rgba8);
/* LUT_TABLE_FLOAT (texture.rs:51-54) for tests */
float ref_lut_float(uint32_t i);
uint8_t ref_lut_byte(uint32_t i);

#ifdef __cplusplus
}
#endif
#endif
