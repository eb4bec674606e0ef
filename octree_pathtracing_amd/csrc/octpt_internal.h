// octpt_internal.h -- device-side scene layout shared by the host API (octpt_api.cpp) and
// the gfx950 kernels (octpt_kernels.hip).  Layout notes live in DESIGN.md §5.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <new>
#include <utility>
#include <vector>

#include "../../include/octpt.h"

namespace octpt {

constexpr uint32_t kPrimNone = 0xFFFFFFFFu;
constexpr uint32_t kPrimCuboidBit = 0x80000000u;
constexpr uint32_t kPrimIndexMask = 0x07FFFFFFu;  // primitive indices < 2^27 (hit records pack flags above)
// camera-ray beam starts (beam_kernel): one per kBeamTile x kBeamTile pixels (A/B knob)
#ifndef OCTPT_BEAM_TILE
#define OCTPT_BEAM_TILE 2
#endif
constexpr uint32_t kBeamTile = OCTPT_BEAM_TILE;
// the seed's camera rays as 16-B records when every chunk item has its pixel (store_cam_ray; A/B knob; the
// seed-ticket A/B build writes store_ray's records)
#ifndef OCTPT_CAM_RECORDS
#ifdef OCTPT_SEED_TICKET
#define OCTPT_CAM_RECORDS 0
#else
#define OCTPT_CAM_RECORDS 1
#endif
#endif
constexpr uint32_t kTile = 8;          // 8x8 pixel tiles = one wave64 of primary rays
constexpr uint32_t kBlock = 256;       // threads per block (4 waves)
constexpr uint32_t kMaxDepth = 21;     // new_octree.rs:14

// GPUMaterial (gpu_material.rs:67-76) + the material's texture kind and, for colour
// textures, the pre-converted F32Color (colors/mod.rs:280-288): 48 B, three float4 loads
struct alignas(16) DevMaterial {
    float ior, specular, emittance, roughness;
    float metalness;
    uint32_t texture_index, flags, texture_kind;
    float color[4];
};

// texture table entry, 16 B
struct alignas(16) DevTexture {
    uint32_t kind;      // 0 colour, 1 image
    uint32_t rgba;      // packed U8Color (r | g<<8 | b<<16 | a<<24) for kind 0
    uint32_t width;     // image only
    uint32_t height;
    uint64_t offset;    // byte offset in the texel pool
    uint64_t pad;
};

// Sun::new derived constants (scene/mod.rs:321-383) + diffuse_reflection importance
// sampling constants (ray/mod.rs:228-259); computed once on the host with libm.
struct DevSun {
    float sw[3], su[3], sv[3];
    float width, width2;
    float tex[4];
    float isect_mul[3];
    float diffuse_mul[3];
    float emit[3];  // Sun::emmittance = color * INTENSITY^GAMMA (scene/mod.rs:352-353), preview shading
    float luminosity;
    float sun_dx, sun_dy, sun_dz;
    float circle_radius, sample_chance;
    int32_t draw_texture, importance_sampling, diffuse_sun;
    // next-event estimation (path_tracer.rs:225-291, 458-483)
    int32_t sun_sampling, strict_direct_light;
    float lum_a;          // sun_luminosity ? luminosity_pdf : 1
    float radius_cos;     // Sun::radius_cos
    float f_sub_surface;  // Scene::f_sub_surface
};

// block-model quad: Quad::new's derived plane, normal and w (quad.rs:90-114), 96 B
struct alignas(16) DevQuad {
    float4 o_d;    // (origin.xyz, d = normal . origin)
    float4 u_mat;  // (u.xyz, material bits)
    float4 v_tu0;  // (v.xyz, texture_u_range.x)
    float4 w_tu1;  // (w.xyz = n / (n . n), texture_u_range.y)
    float4 n_tv0;  // (normal.xyz, texture_v_range.x)
    float4 tv1;    // (texture_v_range.y, 0, 0, 0)
};

// primitive kinds a kernel instance handles (wf_extend_kernel's kPrims); kPrimsBlocks: block-value leaves (C23)
constexpr int kPrimsSpheres = 0, kPrimsBoxes = 1, kPrimsModels = 2, kPrimsBlocks = 3;
// flags of a block leaf's slot (slot.y, set at upload): bit f (f < 6) = face f's texture has a texel with
// alpha 0 (the leaf test reads the texel there), kBlockIsModel = the block is a block model
constexpr uint32_t kBlockFaceAlphaMask = 0x3Fu;
constexpr uint32_t kBlockIsModel = 0x40u;
// self-intersection key of a ray leaving quad q: kQuadKey | q; prim ids are
// sphere indices < 2^27 or kPrimCuboidBit | index, so the keys never collide
constexpr uint32_t kQuadKey = 0x40000000u;

struct DevScene {
    // sparse packed child slots: an octant's present children are contiguous from
    // its base; octant child = (its base, its child_mask), leaf child = (prim id, 1) or
    // (first leaf prim, prim count)
    const uint2 *node_child;
    const float4 *leaf_sph;         // parallel to node_child: the sphere of a single-sphere leaf slot
    uint32_t root, root_mask, depth, n_octants;  // root = the root octant's base
    uint32_t has_cuboids;
    float octree_scale;             // 2^-depth
    float inv_octree_scale;         // 2^depth (x / 2^-depth == x * 2^depth exactly)
    const uint32_t *leaf_prims;
    const float4 *spheres;          // (cx, cy, cz, r)
    const uint32_t *sphere_mat;
    const float4 *cub_a;            // (min.x, min.y, min.z, max.x)
    const float2 *cub_b;            // (max.y, max.z): 24 B per box in two loads, no padding lanes
    const uint32_t *cub_mat;        // 6 per cuboid
    const uint32_t *cub_model;      // per cuboid: OCTPT_MODEL_NONE or a block model (C19); has_models only
    const uint2 *models;            // (first quad, quad count)
    const DevQuad *quads;
    uint32_t has_models;
    // block-value leaves (C23): a leaf slot is (block id, kBlock* flags); blk_mat = 6 face materials per
    // block, blk_model = its model (OCTPT_MODEL_NONE: the block fills its cell)
    uint32_t has_blocks, n_blocks;
    const uint32_t *blk_mat;
    const uint32_t *blk_model;
    const DevMaterial *mats;
    uint32_t n_mats;
    const DevTexture *texs;
    uint32_t n_texs;
    const uint8_t *texels;
    const float *lut_float;         // LUT_TABLE_FLOAT (texture.rs:51-54)
    DevSun sun;
    int32_t emitters;
    uint32_t has_images;  // some texture is an image (shade's colour-only instance when not)
};

struct DevCamera {
    float eye[3], dir[3], right[3], up[3];
    float d_factor;  // 1 / tan(fov / 2)  (camera.rs:79)
};

// n / d for a divisor d fixed per launch (Lemire, Kaser & Kurz 2019, "Faster remainder by direct computation"):
// with c = ceil(2^64 / d), floor(c * n / 2^64) = floor(n / d) for every 32-bit n and 2 <= d < 2^32; c = 0 marks d = 1.
// Two integer multiplies instead of the ~25-instruction runtime division (item -> pixel maps of seed, shade, resolve).
inline uint64_t udiv_magic(uint32_t d) { return d <= 1u ? 0ull : ~0ull / d + 1ull; }
__host__ __device__ inline uint32_t udiv_c(uint32_t n, uint64_t c) {
    if (c == 0ull) return n;
#ifdef __HIP_DEVICE_COMPILE__
    const uint64_t hi = (uint64_t)(uint32_t)(c >> 32) * n + __umulhi((uint32_t)c, n);
#else
    const uint64_t hi = (uint64_t)(uint32_t)(c >> 32) * n + (((uint64_t)(uint32_t)c * n) >> 32);
#endif
    return (uint32_t)(hi >> 32);
}

struct DevRender {
    uint32_t W, H;
    uint32_t spp_start, spp_count;
    uint32_t max_depth;
    uint32_t seed;
    uint32_t shard_index, shard_count;
    uint32_t compact;        // accum holds the shard's tiles only (tile-major)
    uint32_t tiles_x;        // ceil(W / 8)
    uint64_t div_tiles_x, div_items;  // udiv_magic(tiles_x), udiv_magic(total_items)
    uint32_t shard_tiles;    // tiles owned by this shard
    uint32_t total_items;    // shard_tiles * 64 work items
    float dim;               // max(W, H)
    float jlo, jhi;          // -1 / dim, 1 / dim: the jitter range of render_tile_average (tile_renderer.rs:701-702),
                             // divided once on the host (IEEE division, the same bits as the device's)
    uint32_t preview;        // RendererMode::Preview
    // branch schedule, NULL when branch_count == 1: sub-sample k of this call is
    // subs[k] = (pass spp, pass branch count | branch << 16); spp_count then counts sub-samples
    const uint2 *subs;
    // beam starts of the camera rays, one per kBeamTile^2 pixels of the frame (row-major, beam_tx per
    // row), NULL = off (beam_kernel)
    const float *beam;
    uint32_t beam_tx;
    // the tile deal (octpt_set_tile_order): dealing position s -> frame tile, NULL = identity.  Shard k owns
    // positions s = k + u * shard_count (its local tile u), whatever the order
    const uint32_t *tile_order;
};

// frame tile at dealing position s (octpt_set_tile_order's permutation, or s itself)
__host__ __device__ inline uint32_t dealt_tile(const uint32_t *order, uint32_t s) { return order ? order[s] : s; }

// TileRenderer::get_current_branch_count (tile_renderer.rs:196-206)
inline uint32_t current_branch_count(uint32_t current_spp, uint32_t scene_branch_count) {
    if (current_spp < scene_branch_count) {
        if (current_spp <= (uint32_t)sqrtf((float)scene_branch_count)) return 1u;
        return scene_branch_count - current_spp;
    }
    return scene_branch_count;
}

// wavefront path tracer state.
// A single device-scope counter sustains only ~88 M atomicAdd/s on MI355X (tools/atomic_bench.hip),
// so every queue and work counter is split into kSegs shards, each on its own 256-B line:
//   ray queue q = kSegs segments of seg_cap positions; segment k holds count(q,k) rays;
//   extend claims from head(q,k); shade appends a ray to the segment it came from (one input ray
//   yields at most one output ray, so a segment never overflows); chunk items are split into
//   kSegs contiguous shards claimed through item(k), stolen from other shards once a wave's own
//   shard is exhausted.
constexpr uint32_t kSegs = 64;
constexpr uint32_t kCtrStride = 64;  // uint32 words between counters (256 B)
constexpr uint32_t kCtrlWords = 5u * kSegs * kCtrStride;
__host__ __device__ constexpr uint32_t ctr_count(uint32_t q, uint32_t k) { return (q * kSegs + k) * kCtrStride; }
__host__ __device__ constexpr uint32_t ctr_head(uint32_t q, uint32_t k) { return ((2u + q) * kSegs + k) * kCtrStride; }
__host__ __device__ constexpr uint32_t ctr_item(uint32_t k) { return (4u * kSegs + k) * kCtrStride; }

struct WaveBuffers {
    float4 *ray0[2];  // per queue position: (o.xyz, last_prim)
    float4 *ray1[2];  // per queue position: (d.xyz, slot | self_inward << 31)
    float4 *pa;     // (T.xyz, L.x)
    float4 *pb;     // (L.y, L.z, rng, item)
    uint2 *pc;      // (cur_mat, depth | specular << 8 | path_segs << 16)
    uint32_t *item0;  // per slot: the chunk item the seed started there (the first shade rebuilds pa / pb / pc)
    uint2 *hit;     // per queue position: (cuboid bit | flags << 27 | prim index, t) -- hit_record()
    // per queue position, block-value scenes only (C23): the whole hit record, (face << 27 | block or the quad, t, u, v)
    // -- the hit's texture coordinates or a quad's barycentrics beside it -- one 16-B store in extend and one
    // 16-B load in shade (round 6; until then an 8-B `hit` record and an 8-B (u, v) record in two arrays)
    uint4 *hit4;
    float4 *color;  // per chunk item: (L.xyz, path segments)
    // sun-sampling state, 4 planes of `pool` float4:
    // (co.xyz, clast), (cd.xyz, ccur), (cn.xyz, mult), att
    float4 *pd;
    uint32_t pool;
    uint32_t *ctrl;    // kCtrlWords sharded counters (see above)
    uint32_t seg_cap;  // positions per queue segment (multiple of 64)
    // (camera eye.xyz, kPrimNone): the first half of every ray record the seed writes, which the
    // chunk's first shade takes from here instead of re-reading it
    float4 eye;
    // the lean 24-B path state (pa = (T, rng), pc; pb and item0 unused): no emitters, no sun sampling and the
    // pool holding the chunk (item = slot), set per chunk by the host
    uint32_t lean;
};
// the lean path state's chunks exclude branch schedules (C20) as well as emission and sun sampling (A/B knob)
#ifndef OCTPT_LEAN_STRICT
#define OCTPT_LEAN_STRICT 1
#endif
// shade instance: 0 = 40-B path state, 1 = with regeneration (pool smaller than the chunk), 2 = lean
inline int shade_mode(bool regen, bool lean) { return regen ? 1 : (lean ? 2 : 0); }

// per-launch statistics, accumulated with one atomic per wave
enum StatIndex {
    kStatPaths = 0,
    kStatSegments,
    kStatSteps,
    kStatSphereTests,
    kStatCuboidTests,
    kStatShade,
    kStatTexels,
    kStatBlockTests,  // block-value leaf tests (C23)
    kStatIssued,      // extend's issued load bytes (OCTPT_COUNT_ISSUED builds only)
    kStatCount
};
static_assert(kStatCount == OCTPT_STAT_COUNT, "octpt_stats::drain order");
// statistics rows: kSegs rows of kStatRow counters (256 B each), row = blockIdx % kSegs; the host sums.
// The drain kernel counts into a second set of kSegs rows (octpt_stats::drain).
constexpr uint32_t kStatRow = 32;
constexpr uint32_t kStatWords = 2u * kSegs * kStatRow;
constexpr uint32_t kStatDrainRow = kSegs;
// beam-started rays traced again from the cube entry (octpt_stats::beam_restarts): a word of the row
// past the kStatCount counters, counted by one atomic per event
constexpr uint32_t kStatBeamRestartWord = 10;
// hit records with an unwritten field (OCTPT_CHECK_HITS diagnostic builds; octpt_stats::hit_check_failures)
constexpr uint32_t kStatHitCheckWord = 11;
static_assert(kStatBeamRestartWord >= kStatCount && kStatBeamRestartWord < 12, "below the lane-profile words");

// Multi-device renders (octpt_create_multi): item i of a shard's compact tile order (tile
// u = i / 64, pixel k = i % 64 of it) is rendered by device entry u % n_dev as its local tile u / n_dev --
// the entry's own shard of the kernels' tile split, shard_index + (u % n_dev) * shard_count of
// shard_count * n_dev -- whose compact buffer is staged on the first device at (u % n_dev) * stride.
// `caller` is the item's index in the caller's buffer (the shard's compact buffer, or the W x H frame);
// false for a pixel outside the image in a frame layout (never read or written).
__host__ __device__ inline bool multi_slot(uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t shard_index,
                                           uint32_t shard_count, bool compact, uint32_t n_dev, uint32_t stride,
                                           uint32_t i, uint32_t &caller, uint32_t &staged,
                                           const uint32_t *order = nullptr) {
    const uint32_t u = i / 64u, k = i % 64u;
    staged = (u % n_dev) * stride + (u / n_dev) * 64u + k;
    if (compact) {
        caller = i;
        return true;
    }
    const uint32_t t = dealt_tile(order, shard_index + u * shard_count);
    const uint32_t x = (t % tiles_x) * kTile + k % kTile, y = (t / tiles_x) * kTile + k / kTile;
    if (x >= W || y >= H) return false;
    caller = y * W + x;
    return true;
}

// kernel launchers (octpt_kernels.hip)
hipError_t launch_preview(const DevScene &S, const DevCamera &C, const DevRender &R, float4 *accum,
                          uint32_t *segcount, unsigned long long *stats, hipStream_t stream);
hipError_t launch_render(const DevScene &S, const DevCamera &C, const DevRender &R, float4 *accum,
                         uint32_t *segcount, uint32_t *counter, unsigned long long *stats, int grid,
                         hipStream_t stream);
hipError_t launch_wf_seed(const DevCamera &C, const DevRender &R, const WaveBuffers &B, uint32_t n_seed,
                          uint32_t chunk_items, unsigned long long *stats, hipStream_t stream);
hipError_t launch_wf_extend(const DevScene &S, const WaveBuffers &B, uint32_t q, bool cam, uint32_t refill, int grid,
                            unsigned long long *stats, hipStream_t stream);
// first: the chunk's first shade (the seed's rays: path state rebuilt from item0); regen: the pool is
// smaller than the chunk, finished paths regenerate their slots (the instance with regeneration)
hipError_t launch_wf_shade(const DevScene &S, const DevCamera &C, const DevRender &R, const WaveBuffers &B, uint32_t q,
                           uint32_t chunk_items, uint32_t first, bool regen, int grid, unsigned long long *stats,
                           hipStream_t stream);
// blocks per CU of the shade instance (shade_mode; registers bound it, shade uses no dynamic LDS)
int shade_blocks_per_cu(const DevScene &S, int mode);
// whether the scene's shade instance copies the material / texture tables into LDS
bool shade_lds_tables(const DevScene &S);
// the drain of a chunk's last queued rays (every chunk item claimed): one launch, paths finished in-lane
hipError_t launch_wf_drain(const DevScene &S, const DevRender &R, const WaveBuffers &B, uint32_t q, int grid,
                           unsigned long long *stats, hipStream_t stream);
// the host's snapshot of an iteration's counters: queue q's kSegs segment counts, then the kSegs item
// counters, written by one 128-thread block into pinned host memory (enqueue_wavefront's steering)
hipError_t launch_wf_snapshot(const WaveBuffers &B, uint32_t q, uint32_t *host_out, hipStream_t stream);
hipError_t launch_wf_resolve(const DevRender &R, const WaveBuffers &B, uint32_t chunk_spp, float4 *accum,
                             uint32_t *segcount, hipStream_t stream);
int extend_blocks_per_cu(const DevScene &S);
hipError_t launch_intersect(const DevScene &S, const float *rays, const uint32_t *last_prim,
                            const float *last_normal, uint32_t n, float *t, uint32_t *prim, float *normal,
                            uint32_t *steps, hipStream_t stream);
hipError_t launch_beam(const DevScene &S, const DevCamera &C, const DevRender &R, float *beam, hipStream_t stream);
hipError_t launch_tonemap(const float4 *accum, uchar4 *out, uint32_t n, const uint8_t *lut_byte,
                          hipStream_t stream);
hipError_t launch_unshard(uint32_t W, uint32_t H, uint32_t shard_count, const uint32_t *tile_pos, const float4 *shards,
                          uint32_t stride, float4 *frame, hipStream_t stream);
// the caller's buffers (accum, and seg when not NULL) <-> the staged compact buffers of n_dev device
// entries (multi_slot), to_stage = caller -> staging
hipError_t launch_multi_stage(const DevRender &R, uint32_t n_dev, uint32_t stride, float4 *accum, uint32_t *seg,
                              float4 *stage_accum, uint32_t *stage_seg, bool to_stage, hipStream_t stream);
int render_blocks_per_cu(uint32_t depth);
size_t render_lds_bytes(uint32_t depth);

// std::vector allocator that leaves resized elements uninitialised: the builders overwrite every
// element, and zero-filling a C4 octree's 0.2 GB first costs more than the GPU build itself
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
    template <class U>
    void construct(U *p) noexcept {
        ::new (static_cast<void *>(p)) U;
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
    }
};
template <class T>
using RawVec = std::vector<T, NoInitAlloc<T>>;

// host arrays of a built octree (octpt_octree, include/octpt.h)
struct BuiltOctree {
    RawVec<octpt_octant> octants;
    RawVec<uint32_t> leaf_first, leaf_count, leaf_prims;
    uint32_t root = 0, depth = 0;
};

// grow-only device scratch of the GPU octree builder, owned by the context: repeated builds
// (scene edits) reuse it instead of paying hipMalloc / hipFree per buffer
struct BuildScratch {
    static constexpr int kSlots = 32;
    void *dev[kSlots] = {};
    size_t cap[kSlots] = {};
    void release();
};

// a built octree left on the device (pointers into the BuildScratch, valid until the next build):
// the same arrays as BuiltOctree, plus the primitives the builder uploaded
struct DeviceOctree {
    const octpt_octant *octants = nullptr;
    const uint32_t *leaf_first = nullptr, *leaf_count = nullptr, *leaf_prims = nullptr;
    const octpt_sphere *spheres = nullptr;
    const octpt_cuboid *cuboids = nullptr;
    uint32_t n_octants = 0, n_leaves = 0, n_leaf_prims = 0, ns = 0, nc = 0, depth = 0;
};

// the octree builder on the device (octpt_build.hip); too_many: more than max_pairs pairs.
// dev == nullptr: the result is downloaded into `out`; else it stays on the device in *dev.
hipError_t build_octree_gpu(hipStream_t stream, BuildScratch &scratch, const octpt_sphere *spheres, uint32_t ns,
                            const octpt_cuboid *cuboids, uint32_t nc, uint32_t depth, bool compact,
                            uint64_t max_pairs, BuiltOctree &out, bool &too_many, float *ms,
                            DeviceOctree *dev = nullptr);

// Device-resident scene packing (octpt_scene_build_device): the sparse child-slot bases of a
// DeviceOctree (exclusive scan of the present-child counts; *d_base in the scratch, n_octants + 1
// entries, the last = slot count), then the slots, the single-sphere leaf table and the primitive
// tables, written exactly as octpt_scene_upload packs them on the host.
hipError_t slot_bases_gpu(hipStream_t stream, BuildScratch &scratch, const DeviceOctree &t, uint32_t **d_base,
                          uint32_t &n_slots);
struct ScenePrimTables {
    uint2 *node_child;   // n_slots + 8 (the tail zeroed by the caller)
    float4 *leaf_sph;    // sphere-only scenes, else nullptr
    uint32_t *leaf_prims;
    float4 *spheres;
    uint32_t *sphere_mat;
    float4 *cub_a;
    float2 *cub_b;
    uint32_t *cub_mat;
};
hipError_t fill_scene_gpu(hipStream_t stream, const DeviceOctree &t, const uint32_t *d_base,
                          const ScenePrimTables &out);

}  // namespace octpt
