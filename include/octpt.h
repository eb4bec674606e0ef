/*
 * octpt.h -- C ABI of the MI355X-native octree path-tracing hot path.
 *
 * This is the drop-in boundary that replaces the reference's GPU backend
 * (kekley/octree_pathtracing, src/renderer/gpu_renderer.rs:151-702, implementing
 * trait RenderingBackend, src/renderer/renderer_trait.rs:19-46).  A Rust host binds
 * these symbols with an `extern "C"` block and keeps its own
 * Scene / Octree / Camera types; every struct below is #[repr(C)]-compatible.
 *
 * Conventions
 *  - Every entry returns octpt_status (int32).  No C++ exception crosses the ABI.
 *  - Input arrays are borrowed for the duration of the call and deep-copied.
 *  - A context is externally synchronised (one host thread at a time); distinct
 *    contexts are independent.  Frames returned by octpt_render_async are owned by
 *    the caller until octpt_frame_release.
 *  - There is no CPU fallback: without a usable gfx950 device octpt_create fails
 *    with OCTPT_ERR_DEVICE.
 *  - "Drop-in": src/octree is used unchanged (the raw octant masks come from Octant's public is_child /
 *    is_leaf / get_child).  A Rust host binding this header adds one accessor to the
 *    reference, Sun::octpt_args in src/scene/mod.rs (Sun's texture, colour and draw flag are private), and
 *    supplies the block table (block value -> face materials / model) that its resource manager resolves and
 *    Scene does not hold.  src/app and the rest of src/scene are untouched.
 */
#ifndef OCTPT_H
#define OCTPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OCTPT_ABI_VERSION 4u

typedef int32_t octpt_status;
#define OCTPT_OK 0
#define OCTPT_ERR_INVALID_ARG 1
#define OCTPT_ERR_OOM 2
#define OCTPT_ERR_DEVICE 3
#define OCTPT_NOT_READY 4     /* FrameInFlightPoll::NotReady (renderer_trait.rs:37-41) */
#define OCTPT_ERR_UNSUPPORTED 5
#define OCTPT_CANCELLED 6     /* FrameInFlightPoll::Cancelled */
#define OCTPT_ERR_INTERNAL 7

typedef struct octpt_ctx octpt_ctx;
typedef struct octpt_frame octpt_frame;
typedef struct octpt_octree octpt_octree;

/* new_octree::Octant (src/octree/new_octree.rs:70-74) in C layout, 36 bytes.
 * Two mask bits per child i, (bit i, bit i+8):
 *   (0,0) empty; (1,1) leaf, children[i] = the leaf payload (leaf table index);
 *   (1,0) octant, children[i] = octant index -- the OctantChildIterator reading
 *         (new_octree.rs:84-100), what octpt_build_octree writes;
 *   (0,1) octant, children[i] = octant index -- the form Octant::set_mask_for writes for
 *         ChildType::Octant (new_octree.rs:160-178), i.e. every tree the reference's
 *         expand_by / RegionOctreeBuilder / SectionOctantBuilder build.
 * Leaves may sit at any level (LOD leaves above the bottom, new_octree.rs:534-536).
 * Child index i = x | y << 1 | z << 2 (the ESVO/Morton child order, octree_traversal.rs:22-24). */
typedef struct octpt_octant {
    uint16_t child_mask;
    uint16_t reserved;
    uint32_t children[8];
} octpt_octant;

/* geometry::sphere::Sphere (src/geometry/sphere.rs:10-14), 32 bytes */
typedef struct octpt_sphere {
    float center[3];
    float radius;
    uint32_t material;
    uint32_t reserved[3];
} octpt_sphere;

/* geometry::cuboid::Cuboid (src/geometry/cuboid.rs:48-52): AABB + one material per face,
 * Face order West(-X), East(+X), Bottom(-Y), Top(+Y), South(+Z), North(-Z).  48 bytes. */
typedef struct octpt_cuboid {
    float min[3];
    float max[3];
    uint32_t face_material[6];
} octpt_cuboid;

/* Block models.  A leaf cuboid whose cuboid_model entry is not
 * OCTPT_MODEL_NONE is a Minecraft block-model instance (the reference's ResourceModel::Quad leaf,
 * octree_traversal.rs:207-213; Scene::quads, scene/mod.rs:153): its box is the voxel [min, min+1)
 * and its surface is the model's quads, tested with Quad::hit (src/geometry/quad.rs:172-200) in
 * voxel-local coordinates, instead of the six faces of the box.
 * geometry::quad::Quad::new arguments (quad.rs:90-114): origin, edge vectors u and v (voxel-local,
 * the block is [0,1]^3), texture u/v ranges (the face's uv rectangle / 16) and the material.
 * The plane, normal and w = n / (n.n) are derived at upload exactly as Quad::new does.  64 bytes. */
typedef struct octpt_quad {
    float origin[3];
    uint32_t material;
    float u[3];
    float v[3];
    float texture_u_range[2];
    float texture_v_range[2];
    uint32_t reserved[2];
} octpt_quad;
/* gpu_structs::model::Model (src/gpu_structs/model.rs:14-21): the model's quads are
 * quads[first_quad .. first_quad + quad_count).  16 bytes. */
typedef struct octpt_block_model {
    uint32_t flags; /* reserved, 0 */
    uint32_t first_quad, quad_count;
    uint32_t reserved;
} octpt_block_model;
#define OCTPT_MODEL_NONE 0xFFFFFFFFu

/* GPUMaterial (src/gpu_structs/gpu_material.rs:67-76), 32 bytes */
typedef struct octpt_material {
    float ior, specular, emittance, roughness, metalness;
    uint32_t texture_index, tint_index, flags; /* flags: MaterialFlags bits (material.rs:99-108) */
} octpt_material;

#define OCTPT_TEXTURE_COLOR 0u /* Texture::Color(U8Color)  (texture.rs:15-18) */
#define OCTPT_TEXTURE_IMAGE 1u /* Texture::Image(RTWImage), RGBA8, row-major, top row first */
typedef struct octpt_texture {
    uint32_t kind;
    uint8_t rgba[4];
    uint32_t width, height;
    const uint8_t *pixels; /* width*height*4 bytes for OCTPT_TEXTURE_IMAGE, else NULL */
} octpt_texture;

/* scene::Sun::new arguments (src/scene/mod.rs:321-330) + SunSamplingStrategy flags (:60-69) */
typedef struct octpt_sun {
    float azimuth, altitude, radius;
    float color[4];
    float apparent_color[3];
    int32_t draw_texture, texture_modification;
    float importance_sample_chance, importance_sample_radius;
    float luminosity;
    uint8_t texture_rgba[4];
    int32_t importance_sampling, diffuse_sun;
    /* next-event estimation toward the sun (do_diffuse_reflection, path_tracer.rs:225-291;
     * get_direct_light_attenuation :458-483): presets FAST / HIGH_QUALITY (scene/mod.rs:98-126) */
    int32_t sun_sampling, strict_direct_light, sun_luminosity;
    float luminosity_pdf; /* Sun::luminosity_pdf, 1/100 in Sun::new (scene/mod.rs:376) */
} octpt_sun;

/* Block-value leaves: the reference's own leaf form.  Every octree the reference
 * builds stores a u32 block value in its leaves -- (ChildType::Leaf, value) (new_octree.rs:669),
 * Lod(section_fill_block) (:727), Lod(data) one or more levels up (:534-537, 586) -- and traverses
 * such a leaf as the cell itself (octree_traversal.rs:143-214).  With octpt_scene_desc.blocks set, a
 * leaf payload is an index into this table, at any level:
 *  - model == OCTPT_MODEL_NONE: the block fills its leaf cell (ResourceModel::SingleBlock, :193-206).
 *    The face is the cell face the ray enters, the texture coordinates its entry point over the cell
 *    (:156-190), the material face_material[face]; a texel with alpha <= EPSILON lets the ray through
 *    (the traversal advances), and a ray that starts inside the cell passes it (t_min == 0, :194);
 *  - else the block model (C19) drawn at the leaf cell's corner in unit-voxel coordinates
 *    (ResourceModel::Quad, :207-213).
 * Face order West(-X), East(+X), Bottom(-Y), Top(+Y), South(+Z), North(-Z) (cuboid.rs:9-29).  32 bytes. */
typedef struct octpt_block {
    uint32_t face_material[6];
    uint32_t model;
    uint32_t reserved;
} octpt_block;

/* Scene (src/scene/mod.rs:146-156) flattened: octree + leaf primitive lists + primitive,
 * material and texture tables.  Leaf payload p indexes leaf_first/leaf_count; the prims
 * leaf_prims[first .. first+count) are sphere indices, or cuboid indices | 0x80000000.
 * With `blocks` set the leaf payloads are block ids instead (C23): leaf_*, spheres and cuboids
 * must then be empty, and block models draw from models / quads. */
typedef struct octpt_scene_desc {
    uint32_t abi_version; /* = OCTPT_ABI_VERSION */
    const octpt_octant *octants;
    uint32_t octant_count, root, depth; /* depth <= 21 (new_octree.rs:14); world = [0, 2^depth)^3 */
    const uint32_t *leaf_first;
    const uint32_t *leaf_count;
    uint32_t leaf_table_size;
    const uint32_t *leaf_prims;
    uint32_t leaf_prim_count;
    const octpt_sphere *spheres;
    uint32_t sphere_count;
    const octpt_cuboid *cuboids;
    uint32_t cuboid_count;
    const octpt_material *materials; /* materials[0] is the outer medium (air) */
    uint32_t material_count;
    const octpt_texture *textures;
    uint32_t texture_count;
    octpt_sun sun;
    int32_t emitters_enabled;
    float f_sub_surface; /* Scene::f_sub_surface (scene/mod.rs:152): subsurface sun-sample chance */
    /* block models (C19): cuboid_model (nullable = no models) holds one entry per cuboid,
     * OCTPT_MODEL_NONE for a plain box or a model index; such a cuboid must be a unit voxel */
    const uint32_t *cuboid_model;
    const octpt_block_model *models;
    uint32_t model_count;
    const octpt_quad *quads;
    uint32_t quad_count;
    /* block-value leaves (C23): NULL = primitive leaves */
    const octpt_block *blocks;
    uint32_t block_count;
} octpt_scene_desc;

/* renderer::camera::Camera (src/renderer/camera.rs:8-25) */
typedef struct octpt_camera {
    float eye[3];
    float direction[3];
    float up[3];
    float fov; /* radians */
    float aperture, focal_distance; /* must be 0: thin lens is unused by the reference path */
} octpt_camera;

/* One progressive render call = spp_count passes of TileRenderer::render_tile_average
 * (tile_renderer.rs:684-734) continuing a running mean that already holds spp_start samples. */
#define OCTPT_RENDER_SHARD_COMPACT 0x1u /* accum holds only this shard's 8x8 tiles, tile-major */
#define OCTPT_RENDER_MEGAKERNEL 0x2u    /* single persistent megakernel instead of the wavefront loop (A/B) */
#define OCTPT_RENDER_KERNEL_TIMING 0x4u /* bracket every extend / shade launch with HIP events (octpt_stats) */
/* RendererMode::Preview (tile_renderer.rs:293, render_tile_replace :648-682; preview_render,
 * path_tracer.rs:137-158): one un-jittered camera ray per pixel, flat-shaded by the sun
 * (Sun::flat_shading, scene/mod.rs:447-452); rgb is replaced, alpha kept; spp/max_depth ignored */
#define OCTPT_RENDER_PREVIEW 0x8u
typedef struct octpt_render_params {
    uint32_t width, height;
    uint32_t spp_start, spp_count;
    uint32_t max_depth;    /* reference: 5 (path_tracer.rs:56) */
    uint32_t branch_count; /* TileRenderer branch count B <= 64: passes of weight
                            * get_current_branch_count(spp, B), the first reflection split into that many
                            * branches; spp_start and spp_start + spp_count must be pass boundaries */
    uint32_t seed;
    uint32_t shard_index, shard_count; /* 8x8 tile t belongs to shard t % shard_count */
    uint32_t flags;
} octpt_render_params;

/* statistics counter order of octpt_stats::drain */
#define OCTPT_STAT_PATHS 0
#define OCTPT_STAT_SEGMENTS 1
#define OCTPT_STAT_ESVO_STEPS 2
#define OCTPT_STAT_SPHERE_TESTS 3
#define OCTPT_STAT_CUBOID_TESTS 4
#define OCTPT_STAT_SHADE_EVENTS 5
#define OCTPT_STAT_TEXEL_READS 6
#define OCTPT_STAT_BLOCK_TESTS 7
#define OCTPT_STAT_ISSUED_BYTES 8
#define OCTPT_STAT_COUNT 9
typedef struct octpt_stats {
    /* esvo_steps: ESVO iterations executed; camera rays start at their tile's beam start, so
       this is the reference walk's count only with OCTPT_BEAM=0 -- every other field is the same either way */
    uint64_t paths, segments, esvo_steps, sphere_tests, cuboid_tests, shade_events, texel_reads;
    uint64_t launches;
    double kernel_ms; /* HIP-event time of the render calls since the last reset */
    /* per-kernel HIP-event time of the wavefront loop, renders flagged OCTPT_RENDER_KERNEL_TIMING only */
    uint64_t extend_launches, shade_launches;
    double extend_ms, shade_ms;
    double build_ms; /* device time (upload excluded) of the last octpt_build_octree_device */
    uint64_t block_tests;  /* block-value leaf tests */
    /* bytes of the loads wf_extend_kernel issues (node slots actually loaded, primitives, quads, alpha
     * texels): counted only by the OCTPT_COUNT_ISSUED diagnostic build of the library, else 0 */
    uint64_t issued_bytes;
    /* the chunk-tail drain kernel's share of the counters above, in OCTPT_STAT_* order (included in
     * the totals; the extend roofline subtracts it) */
    uint64_t drain[OCTPT_STAT_COUNT];
    uint64_t pool_slots;  /* path slots held by the wavefront state (after any out-of-memory fallback) */
    uint64_t chunk_items; /* (pixel, sample) items per chunk held (likewise) */
    uint64_t wave_allocs; /* wavefront-state (re)allocations since the context was created */
    /* camera rays whose beam start reached the reference's step cap and were traced again from the
     * cube entry (their iterations before the restart are in esvo_steps too) */
    uint64_t beam_restarts;
    /* hit records a field of which the path that produced the hit left unwritten: counted only by the
     * OCTPT_CHECK_HITS diagnostic build of the library, else 0 */
    uint64_t hit_check_failures;
} octpt_stats;

/* --- library / context ------------------------------------------------------ */
uint32_t octpt_abi_version(void);
/* number of visible HIP devices (0 when none) */
int32_t octpt_device_count(void);
/* RenderingBackend construction (gpu_renderer.rs:151-200) on HIP device `device` */
octpt_status octpt_create(int32_t device, octpt_ctx **out);
/* A context over several GPUs of one node (SURVEY.md §8(b) device list, §8(e) tile split):
 * devices[0 .. n) are HIP device ids, n <= 64; an id may repeat (two entries on one GPU).  Every entry
 * point takes such a context: the scene is replicated on every entry, a render deals the 8x8 tiles of the
 * call's shard round-robin over the entries (each renders its tiles concurrently, on a host thread of its
 * own) and gathers them with peer copies into the caller's buffers, which live on devices[0]
 * (octpt_render_device's d_accum / d_seg_count and stream).  Results are bit-identical to one device's.
 * octpt_intersect runs on devices[0]; octpt_stats sums the entries' counters, kernel_ms is the render
 * calls' wall time.  n == 1 is octpt_create(devices[0]). */
octpt_status octpt_create_multi(const int32_t *devices, uint32_t n, octpt_ctx **out);
/* device entries of a context (1 for octpt_create; 0 for NULL) */
uint32_t octpt_device_entries(const octpt_ctx *ctx);
void octpt_destroy(octpt_ctx *ctx);
/* last error message of this context (never NULL) */
const char *octpt_last_error(const octpt_ctx *ctx);

/* --- RenderingBackend surface ----------------------------------------------- */
/* set_scene (gpu_renderer.rs:662-669 -> create_pipeline :201-557): validates and uploads */
octpt_status octpt_scene_upload(octpt_ctx *ctx, const octpt_scene_desc *scene);
/* set_scene with the octree built on the device and kept there (the reference's
 * flattener octree_to_gpu_data, gpu_octree.rs:28-76, is todo!()).  The scene's octree fields
 * (octants, octant_count, root, leaf_*) must be NULL / 0; `depth` is the build depth and flags are
 * the builder's (OCTPT_BUILD_COMPACT).  The primitives are uploaded once, voxelised by the GPU
 * builder and its arrays packed into the device node slots in place: the resulting device scene is
 * the one octpt_scene_upload makes from octpt_build_octree_ex's octree, with no round trip through
 * host memory. */
octpt_status octpt_scene_build_device(octpt_ctx *ctx, const octpt_scene_desc *scene, uint32_t flags);
/* set_camera / get_camera (renderer_trait.rs:20-21) */
octpt_status octpt_set_camera(octpt_ctx *ctx, const octpt_camera *camera);
octpt_status octpt_get_camera(const octpt_ctx *ctx, octpt_camera *camera);

/* Synchronous render into host memory.  accum_rgba: width*height*4 floats (or the shard's
 * compact tiles), in/out running mean, initialise to F32Color::BLACK (0,0,0,1).
 * out_rgba8 (nullable): tone-mapped U8Color image (colors/mod.rs:408-420) of accum. */
octpt_status octpt_render(octpt_ctx *ctx, const octpt_render_params *p, float *accum_rgba, uint8_t *out_rgba8);

/* Device-resident render: d_accum is a device pointer (same layout as accum_rgba), the
 * work is enqueued on `hip_stream` (hipStream_t, NULL = default stream).  The wavefront
 * loop is steered from the host (it reads back queue lengths), so the call returns once the
 * last kernel of the render is enqueued, i.e. after the render has essentially finished.
 * d_seg_count (nullable, device, one u32 per accum pixel) receives += ray segments. */
octpt_status octpt_render_device(octpt_ctx *ctx, const octpt_render_params *p, float *d_accum,
                                 uint32_t *d_seg_count, void *hip_stream);

/* render_frame (renderer_trait.rs:30-34) -> FrameInFlight (:42-46) */
octpt_status octpt_render_async(octpt_ctx *ctx, const octpt_render_params *p, float *accum_rgba,
                                uint8_t *out_rgba8, octpt_frame **out_frame);
octpt_status octpt_frame_poll(octpt_frame *frame);   /* OK = Ready, NOT_READY, CANCELLED */
octpt_status octpt_frame_wait(octpt_frame *frame);   /* FrameInFlight::wait_for */
octpt_status octpt_frame_cancel(octpt_frame *frame); /* result buffers are left untouched */
void octpt_frame_release(octpt_frame *frame);

/* Tone map a device accumulation buffer into device RGBA8 (colors/mod.rs:408-420). */
octpt_status octpt_tonemap_device(octpt_ctx *ctx, const float *d_accum, uint8_t *d_rgba8, uint32_t n_pixels,
                                  void *hip_stream);
/* Rank 0 of a sharded render: scatter shard_count compact tile buffers (device, concatenated
 * in shard order, each padded to `shard_stride_pixels`) into a full width*height frame. */
octpt_status octpt_unshard_device(octpt_ctx *ctx, uint32_t width, uint32_t height, uint32_t shard_count,
                                  const float *d_shards, uint32_t shard_stride_pixels, float *d_frame,
                                  void *hip_stream);
/* pixels a shard owns (its compact buffer length in pixels, tile-padded) */
uint32_t octpt_shard_pixels(uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count);

/* The tile deal (round 5).  The reference splits a frame into threads^2 tiles handed to a
 * thread pool (tile_renderer.rs:398-413); here a shard of N owns the 8x8 tiles at dealing positions
 * s = shard_index + u * N (its local tile u).  By default position s is frame tile s (round robin).
 * octpt_set_tile_order sets the frame tile at each position for width x height renders of this context
 * (order: ceil(W/8) * ceil(H/8) entries, a permutation; NULL = round robin again): renders, the async
 * frame, octpt_unshard_device and every entry of a multi-device context follow it, and a render of another
 * size is refused (INVALID_ARG) while it is set.  Per-pixel RNG streams keep the image bit-identical under
 * any order; the order only moves work between shards. */
octpt_status octpt_set_tile_order(octpt_ctx *ctx, uint32_t width, uint32_t height, const uint32_t *order);
/* A balanced order for shard_count shards from a previous render's per-pixel segment counts (seg_count:
 * width * height, image order, e.g. octpt_render's seg_count output): a tile's cost is the sum of its
 * pixels' counts; tiles go, most costly first, to the shard with the least cost so far among those with
 * positions left (each keeps its round-robin number of tiles), then each shard's tiles in image order.
 * Host-only, no context; writes `order` (as octpt_set_tile_order takes it). */
octpt_status octpt_balance_tiles(uint32_t width, uint32_t height, uint32_t shard_count, const uint32_t *seg_count,
                                 uint32_t *order);

/* Batch closest-hit query = Scene::hit (scene/mod.rs:172-187) with the octree traversal
 * (octree_traversal.rs:54-302) restored.  rays: n*6 floats (origin, unit direction), host.  ESVO's
 * 1 / -|d| is exact for direction components up to 2^126 (components below 2^-23 are clamped to it as
 * the reference does); a ray with a non-finite component or a direction component above 2^126 is
 * reported as a miss and the rest of the batch is traced.  For a non-finite ray that is the reference's
 * result; for a finite component above 2^126 it is a deliberate deviation (the reference's walk runs on a
 * subnormal t_coef, octree_traversal.rs:95, and may hit; parity unpinned).
 * last_prim / last_normal (nullable): self-intersection key per ray.
 * Outputs (host): t (world, +inf on miss), prim (0xFFFFFFFF on miss; in a block-value scene, C23, the
 * block id, or 0x40000000 | quad for a block model's quad), normal n*3 (nullable), esvo steps (nullable). */
octpt_status octpt_intersect(octpt_ctx *ctx, const float *rays, const uint32_t *last_prim, const float *last_normal,
                             uint32_t n, float *t, uint32_t *prim, float *normal, uint32_t *steps);

/* Octree::get_traversal_data (octree_traversal.rs:537-714), the beam-start query of
 * GPURenderer::render_frame (gpu_renderer.rs:579-581 -> CameraUniform.traversal_start_idx/scale,
 * index/time stack buffers :35-80).  Walks `ray` (origin xyz, direction xyz, world units) from
 * the root until the first leaf with t_min > 0 and returns the octant it stopped in, its scale
 * and the descent stacks, indexed by scale and zero where unwritten.  Host-only and stateless:
 * no context or device; `octants` is borrowed (the same layout as octpt_scene_desc).
 * max_dst in world units (Scene::hit uses 1024, scene/mod.rs:181). */
octpt_status octpt_traversal_data(const octpt_octant *octants, uint32_t octant_count, uint32_t root, uint32_t depth,
                                  const float ray[6], float max_dst, uint32_t *start_octant, uint32_t *scale,
                                  uint32_t index_stack[24], float time_stack[24]);
octpt_status octpt_get_stats(const octpt_ctx *ctx, octpt_stats *stats);
octpt_status octpt_reset_stats(octpt_ctx *ctx);

/* --- host octree builder (replaces the Rust-side build for primitive scenes) ---
 * Voxelises spheres/cuboids into depth-`depth` leaf cells, Morton-sorts
 * them (new_octree.rs:752-835 code order) and emits octants in pre-order. */
typedef struct octpt_octree_view {
    const octpt_octant *octants;
    uint32_t octant_count, root, depth;
    const uint32_t *leaf_first, *leaf_count;
    uint32_t leaf_table_size;
    const uint32_t *leaf_prims;
    uint32_t leaf_prim_count;
} octpt_octree_view;
octpt_status octpt_build_octree(const octpt_sphere *spheres, uint32_t sphere_count, const octpt_cuboid *cuboids,
                                uint32_t cuboid_count, uint32_t depth, octpt_octree **out);
/* The same builder on the context's device (the reference's flattener
 * octree_to_gpu_data, gpu_octree.rs:28-76, is todo!()): count / scan / emit (cell, primitive) pairs,
 * stable radix sort by Morton code, leaf tables, pre-order octant ids by a scan of the octants each
 * leaf opens.  The result equals octpt_build_octree's array for array.  Inputs are host arrays
 * (borrowed), the result is a host octree as above. */
octpt_status octpt_build_octree_device(octpt_ctx *ctx, const octpt_sphere *spheres, uint32_t sphere_count,
                                       const octpt_cuboid *cuboids, uint32_t cuboid_count, uint32_t depth,
                                       octpt_octree **out);
/* Builder options (the _ex forms; the plain forms pass 0).
 * OCTPT_BUILD_COMPACT: Octant::is_compactable (new_octree.rs:227-233) applied bottom-up at every
 * level, as RegionOctreeBuilder::recursive_build does (:679-690): an octant whose eight children are
 * leaves holding the same primitive list becomes one leaf of its parent with child 0's payload (the
 * other seven leaf table entries stay, unreferenced).  The root is never merged away (a Lod root
 * stays one octant of eight equal leaves, :534-545).  Host and device builds stay equal array for
 * array. */
#define OCTPT_BUILD_COMPACT 0x1u
octpt_status octpt_build_octree_ex(const octpt_sphere *spheres, uint32_t sphere_count, const octpt_cuboid *cuboids,
                                   uint32_t cuboid_count, uint32_t depth, uint32_t flags, octpt_octree **out);
octpt_status octpt_build_octree_device_ex(octpt_ctx *ctx, const octpt_sphere *spheres, uint32_t sphere_count,
                                          const octpt_cuboid *cuboids, uint32_t cuboid_count, uint32_t depth,
                                          uint32_t flags, octpt_octree **out);
/* Block-value octree builder (C23): one block per voxel cell, cells[4k .. 4k+3] = (x, y, z, block id),
 * x, y, z < 2^depth.  Morton-sorted (new_octree.rs:752-835 order) and emitted in pre-order like
 * octpt_build_octree; the leaf payloads are the block ids (the view's leaf tables are empty).
 * OCTPT_BUILD_COMPACT merges eight sibling leaves holding the same block value into one leaf of their
 * parent, bottom-up at every level: Octant::is_compactable's value equality (new_octree.rs:227-233) as
 * SectionOctantBuilder / RegionOctreeBuilder apply it (:675-690, 582-587); the root is never merged
 * away.  Two cells at one position, or a block id >= 2^27, are INVALID_ARG. */
octpt_status octpt_build_block_octree(const uint32_t *cells, uint32_t cell_count, uint32_t depth, uint32_t flags,
                                      octpt_octree **out);
octpt_status octpt_octree_get_view(const octpt_octree *tree, octpt_octree_view *view);
void octpt_octree_free(octpt_octree *tree);

/* --- the reference's Scene, element by element (the host flattener of INTEGRATION.md §3) ---------
 * textures::material::Material (src/textures/material.rs:91-101) with its Texture (texture.rs:15-18):
 * Texture::Color(U8Color) or Texture::Image(RTWImage) as RGBA8 rows (rtw_image.rs:30-36). */
typedef struct octpt_reference_material {
    float index_of_refraction, specular, emittance, roughness, metalness;
    uint32_t material_flags, tint_index;
    uint32_t texture_kind; /* OCTPT_TEXTURE_COLOR / OCTPT_TEXTURE_IMAGE */
    uint8_t color[4];
    uint32_t image_width, image_height;
    const uint8_t *image_rgba; /* image_width * image_height * 4 bytes, top row first */
} octpt_reference_material;
/* geometry::quad::Quad (src/geometry/quad.rs:7-17) field by field: origin, u, v and the texture
 * ranges are Quad::new's arguments; normal, w and d are what Quad::new derived from them (:90-114) */
typedef struct octpt_reference_quad {
    float origin[3], u[3], v[3], w[3], normal[3], d;
    uint32_t material_id;
    float texture_u_range[2], texture_v_range[2];
} octpt_reference_quad;
/* scene::Scene (src/scene/mod.rs:146-156): the octree as new_octree::Octree holds it (octants_slice,
 * root, depth; either mask encoding, C21; block-value leaves), Box<[Quad]>, Box<[Material]>, the Sun::new
 * arguments with the SunSamplingStrategy, emitters_enabled, f_sub_surface -- plus the block table the
 * host's resource manager resolves block values with (block value -> six face materials or a model;
 * resource_manager.rs:126-318, out of scope) and its block models over `quads`. */
typedef struct octpt_reference_scene {
    const octpt_octant *octants;
    uint32_t octant_count, root, depth;
    const octpt_block *blocks;
    uint32_t block_count;
    const octpt_block_model *models;
    uint32_t model_count;
    const octpt_reference_quad *quads;
    uint32_t quad_count;
    const octpt_reference_material *materials;
    uint32_t material_count;
    octpt_sun sun;
    int32_t emitters_enabled;
    float f_sub_surface;
} octpt_reference_scene;
/* Fill an octpt_scene_desc (for octpt_scene_upload) from the reference's Scene.  Material i becomes
 * octpt_material i with its own texture i (the one-texture-per-material layout GPURenderer uploads,
 * gpu_renderer.rs:221-307); quads keep Quad::new's arguments (octpt_scene_upload derives normal, w and d
 * again, in glam's order).  No allocation: the caller provides materials_out / textures_out
 * (material_count each) and quads_out (quad_count); desc_out points into them and into `ref`'s arrays,
 * so all of them must outlive the upload.  Host-only, no context.  A material, model or quad index out
 * of range, an image without pixels, or a quad whose stored normal disagrees with u x v is INVALID_ARG. */
octpt_status octpt_scene_from_reference(const octpt_reference_scene *ref, octpt_material *materials_out,
                                        octpt_texture *textures_out, octpt_quad *quads_out,
                                        octpt_scene_desc *desc_out);

#ifdef __cplusplus
}
#endif
#endif /* OCTPT_H */
