// octpt_api.cpp -- host side of the octpt C ABI (include/octpt.h).
//
// Replaces the reference's wgpu backend (src/renderer/gpu_renderer.rs:151-702): scene
// validation + upload (set_scene / create_pipeline), camera uniform construction
// (render_frame :590-599), progressive render submission, FrameInFlight polling, and the
// host octree builder for primitive scenes.  No CPU rendering path exists here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <thread>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <memory>
#include <vector>

#include "../../include/octpt.h"
#include "octpt_internal.h"
#include "octpt_mask.h"

using namespace octpt;

namespace {

constexpr uint32_t kCounterRing = 256;
constexpr uint64_t kMaxChunkPaths = 1ull << 31;    // colour buffer: up to 32 GiB of float4 per chunk (OCTPT_CHUNK)
constexpr uint64_t kDefaultChunkPaths = 1ull << 29;  // 4K: 64-spp chunks (C5 4634 vs 3882 Mrays/s at 2^30; C3 stays one chunk)
                                                    // (C3 = 530 M paths = one chunk: one drain tail)
#ifndef OCTPT_LOOKAHEAD
#define OCTPT_LOOKAHEAD 3
#endif
constexpr uint32_t kLookahead = OCTPT_LOOKAHEAD;    // host steering: iterations queued ahead of the check
constexpr uint32_t kDefaultPool = 512u << 20;        // path slots in flight (124 B each: queues + path state)
constexpr uint32_t kMaxPool = 1u << 30;              // the sun-sampling planes index 4 * pool slots in uint32
constexpr uint32_t kMinPool = 1u << 20;              // floor of the out-of-memory fallback (halving)
constexpr uint64_t kMaxBuildPairs = 1ull << 31;      // octree builder: (cell, primitive) pair cap
constexpr uint32_t kDefaultRefill = 0;               // extend: idle lanes before a wave refills (0: adaptive)
constexpr uint32_t kDefaultDrainRays = 4096;         // drain the chunk in one launch below this many queued rays

uint32_t env_u32(const char *name, uint32_t dflt) {
    const char *v = std::getenv(name);
    if (!v || !*v) return dflt;
    const long x = std::strtol(v, nullptr, 10);
    return x > 0 ? (uint32_t)x : dflt;
}

struct EventPair {
    hipEvent_t start, stop;
};

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
};

}  // namespace

struct octpt_ctx {
    int device = 0;
    int num_cu = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // scene
    bool has_scene = false;
    DevScene S{};
    std::vector<void *> scene_allocs;
    // camera
    bool has_camera = false;
    octpt_camera cam{};
    DevCamera C{};
    // per-context device state
    uint32_t *d_counters = nullptr;  // ring of work counters, one per launch
    // branch schedule of the current render (C20): host copy + grow-only device table
    std::vector<uint2> h_subs;
    uint2 *d_subs = nullptr;
    size_t subs_cap = 0;
    // beam starts of the camera rays, one per kBeamTile^2 pixels (beam_kernel), grow-only
    float *d_beam = nullptr;
    size_t beam_cap = 0;
    uint32_t launch_seq = 0;
    unsigned long long *d_stats = nullptr;
    uint8_t *d_lut_byte = nullptr;
    float *d_lut_float = nullptr;
    std::vector<EventPair> pending;
    double kernel_ms = 0.0;
    uint64_t launches = 0;
    // per-kernel timing (OCTPT_RENDER_KERNEL_TIMING): kind 0 extend, 1 shade
    bool ktiming = false;
    std::vector<std::pair<int, EventPair>> kpending;
    std::vector<EventPair> ev_pool;
    double kern_ms[2] = {0.0, 0.0};
    uint64_t kern_n[2] = {0, 0};
    float build_ms = 0.0f;  // device time of the last octpt_build_octree_device
    BuildScratch build_scratch;
    int blocks_per_cu_cache[kMaxDepth + 1] = {0};
    int extend_bpc_cache[kMaxDepth + 1][4] = {};  // [depth][kPrims]
    int shade_bpc_cache[2][2][3] = {};            // [sun sampling][LDS tables][shade_mode]
    bool lean_scene = false;  // no emitters, no sun sampling: the lean path state applies when the pool holds the chunk
    bool no_lean = false;     // OCTPT_LEAN=0: always the 40-B path state (A/B, tests)
    // wavefront pool (grown on demand)
    WaveBuffers wb{};
    size_t pool = 0, color_cap = 0, nee_pool = 0;  // nee_pool: slots of the sun-sampling planes (wb.pd)
    void *nee_alloc = nullptr;
    std::vector<void *> wave_allocs;
    void *color_alloc = nullptr;
    // device bytes of the wavefront state (queues, path state, colour records, sun-sampling planes),
    // tracked against mem_limit (OCTPT_DEVICE_MEM_LIMIT, MiB, 0 = none: a test hook that makes the
    // out-of-memory fallback reproducible on an idle GPU)
    size_t wave_bytes = 0, mem_limit = 0;
    std::vector<std::pair<void *, size_t>> wave_sizes;
    uint64_t wave_allocs_n = 0;  // successful (re)allocations of the queues + path state
    bool oom_warned = false;
    uint32_t *h_count = nullptr;  // pinned ring: the segment counters after each iteration's shade
    uint32_t *d_count = nullptr;  // its device address (wf_snapshot_kernel)
    hipEvent_t count_ev[kLookahead + 1] = {};
    uint32_t pool_cap = kDefaultPool, refill = kDefaultRefill;
    bool beam = true;  // camera rays start at their tile's beam (OCTPT_BEAM=0: off)
    uint32_t drain_rays = kDefaultDrainRays;  // queue length at which the drain takes over (OCTPT_DRAIN_RAYS, 0 = off)
    bool drain_models = false;                // the drain in block-model scenes too (OCTPT_DRAIN_MODELS=1, A/B)
    uint64_t chunk_cap = kDefaultChunkPaths;  // (pixel, sample) items per chunk (OCTPT_CHUNK)
    // one asynchronous frame may be in flight; device-touching calls join it first
    octpt_frame *inflight = nullptr;
    // multi-device context (octpt_create_multi): one child context per device entry; this context's own
    // device is the first entry's, where the caller's buffers live.  Empty for octpt_create.
    std::vector<octpt_ctx *> sub;
    // multi-device renders: the staged compact tile buffers (this context: every entry's, side by side on
    // the first device; a child: its own), grow-only
    float4 *m_acc = nullptr;
    uint32_t *m_seg = nullptr;
    size_t m_acc_cap = 0, m_seg_cap = 0;
    // the tile deal (octpt_set_tile_order): for order_w x order_h frames, dealing position -> frame tile and
    // its inverse, on this context's device; empty = the round-robin deal
    std::vector<uint32_t> h_order;
    uint32_t order_w = 0, order_h = 0;
    uint32_t *d_order = nullptr, *d_order_pos = nullptr;
    // what the beam table in d_beam was computed for (round 5): the scene, camera and tile order (their
    // generations) and the frame size and shard.  A render with the same key reuses it -- a progressive
    // renderer calls render_frame again and again with one camera -- and anything else recomputes it.
    uint64_t scene_gen = 0, camera_gen = 0, order_gen = 0;
    struct BeamKey {
        uint64_t scene = 0, camera = 0, order = 0;
        uint32_t w = 0, h = 0, shard_index = 0, shard_count = 0;
        bool valid = false;
        bool operator==(const BeamKey &o) const {
            return valid && o.valid && scene == o.scene && camera == o.camera && order == o.order && w == o.w &&
                   h == o.h && shard_index == o.shard_index && shard_count == o.shard_count;
        }
    } beam_key;
    // recorded on the stream that computed the table: a render on another stream that reuses it waits for it
    hipEvent_t beam_ev = nullptr;
    hipStream_t beam_stream = nullptr;  // the stream the valid table was computed on
    bool beam_shared = false;           // ... and whether a render on another stream has read it since
};

struct octpt_frame {
    octpt_ctx *ctx = nullptr;
    octpt_render_params params{};  // the call's parameters (a multi-device context re-derives each entry's)
    std::thread worker;
    std::atomic<bool> finished{false};
    std::atomic<bool> cancel_requested{false};
    octpt_status status = OCTPT_OK;
    float *user_accum = nullptr;
    uint8_t *user_rgba = nullptr;
    size_t n_pixels = 0;
    float4 *d_accum = nullptr;
    uchar4 *d_rgba = nullptr;
    float *h_accum = nullptr;   // pinned
    uint8_t *h_rgba = nullptr;  // pinned
    bool delivered = false;
};

struct octpt_octree : octpt::BuiltOctree {};

namespace {

octpt_status fail(octpt_ctx *ctx, octpt_status st, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return st;
}

octpt_status hip_fail(octpt_ctx *ctx, hipError_t e, const char *what) {
    return fail(ctx, e == hipErrorOutOfMemory ? OCTPT_ERR_OOM : OCTPT_ERR_DEVICE,
                std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(ctx, expr)                                 \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #expr); \
    } while (0)

// colour LUTs (texture.rs:42-62), computed with the host libm like the reference
void make_luts(float lut_float[256], uint8_t lut_byte[256]) {
    for (int i = 0; i < 256; ++i) {
        lut_float[i] = powf((float)i / 255.0f, 2.2f);
        const float b = powf((float)i / 255.0f, 1.0f / 2.2f) * 255.0f;
        lut_byte[i] = (uint8_t)(b > 0.0f ? (b >= 255.0f ? 255u : (uint32_t)b) : 0u);
    }
}

// glam-order f32 helpers for the host-side uniforms
inline float dot3(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
inline void cross3(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - b[1] * a[2];
    o[1] = a[2] * b[0] - b[2] * a[0];
    o[2] = a[0] * b[1] - b[0] * a[1];
}

// Sun::new (scene/mod.rs:321-383) + diffuse_reflection sun constants (ray/mod.rs:228-259)
void make_sun(const octpt_sun &p, const float lut_float[256], DevSun &k) {
    const float theta = p.azimuth, phi = p.altitude;
    const float r = fabsf(cosf(phi));
    float sw[3] = {cosf(theta) * r, sinf(phi), sinf(theta) * r};
    float su[3] = {0.0f, 0.0f, 0.0f};
    if (fabsf(sw[0]) > 0.1f) su[1] = 1.0f; else su[0] = 1.0f;
    float sv[3];
    cross3(sw, su, sv);
    const float inv = 1.0f / sqrtf(dot3(sv, sv));
    for (float &c : sv) c = c * inv;
    cross3(sv, sw, su);
    std::memcpy(k.sw, sw, sizeof sw);
    std::memcpy(k.su, su, sizeof su);
    std::memcpy(k.sv, sv, sizeof sv);
    k.width = p.radius * 4.0f;
    k.width2 = k.width * 2.0f;
    const float gamma_b = powf(1.25f, 2.2f);
    k.tex[0] = lut_float[p.texture_rgba[0]];
    k.tex[1] = lut_float[p.texture_rgba[1]];
    k.tex[2] = lut_float[p.texture_rgba[2]];
    k.tex[3] = (float)p.texture_rgba[3] / 255.0f;
    for (int i = 0; i < 3; ++i) {
        const float atb = (p.texture_modification ? p.apparent_color[i] : 1.0f) * gamma_b;
        k.isect_mul[i] = atb * 10.0f;
        k.diffuse_mul[i] = p.color[i] * 10.0f;
        k.emit[i] = p.color[i] * gamma_b;
    }
    k.luminosity = p.luminosity;
    const float pi = 3.14159265358979323846f;
    const float az = p.azimuth, alt_fake = p.altitude;
    const float sgn = std::signbit(alt_fake) ? -1.0f : 1.0f;
    const float alt = fabsf(alt_fake) > pi / 2.0f ? sgn * pi - alt_fake : alt_fake;
    k.sun_dx = cosf(az) * cosf(alt);
    k.sun_dz = sinf(az) * cosf(alt);
    k.sun_dy = sinf(alt);
    k.circle_radius = p.radius * p.importance_sample_radius;
    k.sample_chance = p.importance_sample_chance;
    k.draw_texture = p.draw_texture ? 1 : 0;
    k.importance_sampling = p.importance_sampling ? 1 : 0;
    k.diffuse_sun = p.diffuse_sun ? 1 : 0;
    k.sun_sampling = p.sun_sampling ? 1 : 0;
    k.strict_direct_light = p.strict_direct_light ? 1 : 0;
    k.lum_a = p.sun_luminosity ? p.luminosity_pdf : 1.0f;  // path_tracer.rs:250-254
    k.radius_cos = cosf(p.radius);                          // Sun::new (scene/mod.rs:331)
}

void free_scene(octpt_ctx *ctx) {
    for (void *p : ctx->scene_allocs) (void)hipFree(p);
    ctx->scene_allocs.clear();
    ctx->has_scene = false;
}

template <class T>
hipError_t upload(octpt_ctx *ctx, const T *src, size_t n, T **dst) {
    *dst = nullptr;
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return e;
    ctx->scene_allocs.push_back(p);
    if (n && src) {
        e = hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) return e;
    } else {
        e = hipMemset(p, 0, bytes);
        if (e != hipSuccess) return e;
        // hipMemset runs on the null stream, which does not order itself with the context's non-blocking stream:
        // the kernels that fill these tables on ctx->stream (fill_scene_gpu) must not race it
        e = hipStreamSynchronize(nullptr);
        if (e != hipSuccess) return e;
    }
    *dst = static_cast<T *>(p);
    return hipSuccess;
}

// memoised subtree height with cycle detection; returns -1 on a cycle or bad index.
// masks: the octants' child masks in the reader form (normalized_mask, C21)
int subtree_height(const octpt_scene_desc &d, const std::vector<uint16_t> &masks, uint32_t node, std::vector<int8_t> &h,
                   int level) {
    if (level > (int)kMaxDepth + 1) return -1;
    if (h[node] == -2) return -1;  // on the current DFS path: cycle
    if (h[node] >= 0) return h[node];
    h[node] = -2;
    int best = 1;
    const uint32_t m = masks[node];
    for (int i = 0; i < 8; ++i) {
        const bool present = (m >> i) & 1, leaf = (m >> (i + 8)) & 1;
        if (!present || leaf) continue;
        const int ch = subtree_height(d, masks, d.octants[node].children[i], h, level + 1);
        if (ch < 0) return -1;
        best = std::max(best, ch + 1);
    }
    h[node] = (int8_t)best;
    return best;
}

// Quad::new (quad.rs:90-114): n = u x v, normal = n * (1 / |n|), w = n / (n . n), d = normal . origin
DevQuad make_dev_quad(const octpt_quad &x) {
    const float *u = x.u, *v = x.v, *o = x.origin;
    const float n[3] = {u[1] * v[2] - v[1] * u[2], u[2] * v[0] - v[2] * u[0], u[0] * v[1] - v[0] * u[1]};
    const float nn = (n[0] * n[0] + n[1] * n[1]) + n[2] * n[2];
    const float r = 1.0f / sqrtf(nn);
    const float nrm[3] = {n[0] * r, n[1] * r, n[2] * r};
    const float dd = (nrm[0] * o[0] + nrm[1] * o[1]) + nrm[2] * o[2];
    DevQuad q{};
    uint32_t mb;
    std::memcpy(&mb, &x.material, 4);
    float mat;
    std::memcpy(&mat, &mb, 4);
    q.o_d = make_float4(o[0], o[1], o[2], dd);
    q.u_mat = make_float4(u[0], u[1], u[2], mat);
    q.v_tu0 = make_float4(v[0], v[1], v[2], x.texture_u_range[0]);
    q.w_tu1 = make_float4(n[0] / nn, n[1] / nn, n[2] / nn, x.texture_u_range[1]);
    q.n_tv0 = make_float4(nrm[0], nrm[1], nrm[2], x.texture_v_range[0]);
    q.tv1 = make_float4(x.texture_v_range[1], 0.0f, 0.0f, 0.0f);
    return q;
}

octpt_status validate_tables(octpt_ctx *ctx, const octpt_scene_desc *d);

// the checks that precede the octree's: version, depth, non-empty tables, primitive pointers.
// with_octree = false (octpt_scene_build_device): the octree fields must be NULL / 0
octpt_status validate_head(octpt_ctx *ctx, const octpt_scene_desc *d, bool with_octree) {
    if (!d) return fail(ctx, OCTPT_ERR_INVALID_ARG, "scene is NULL");
    if (d->abi_version != OCTPT_ABI_VERSION) return fail(ctx, OCTPT_ERR_INVALID_ARG, "scene abi_version mismatch");
    if (d->depth < 1 || d->depth > kMaxDepth) return fail(ctx, OCTPT_ERR_INVALID_ARG, "octree depth must be in [1, 21]");
    if (with_octree) {
        if (!d->octants || d->octant_count == 0 || d->root >= d->octant_count)
            return fail(ctx, OCTPT_ERR_INVALID_ARG, "octree has no root octant");
    } else if (d->octants || d->octant_count || d->root || d->leaf_first || d->leaf_count || d->leaf_table_size ||
               d->leaf_prims || d->leaf_prim_count) {
        return fail(ctx, OCTPT_ERR_INVALID_ARG, "the device build makes the octree: its scene fields must be NULL / 0");
    }
    if (d->material_count == 0 || !d->materials) return fail(ctx, OCTPT_ERR_INVALID_ARG, "material table is empty");
    if (d->texture_count == 0 || !d->textures) return fail(ctx, OCTPT_ERR_INVALID_ARG, "texture table is empty");
    if (d->leaf_table_size && (!d->leaf_first || !d->leaf_count))
        return fail(ctx, OCTPT_ERR_INVALID_ARG, "leaf table pointers are NULL");
    if (d->leaf_prim_count && !d->leaf_prims) return fail(ctx, OCTPT_ERR_INVALID_ARG, "leaf_prims is NULL");
    if (d->sphere_count > kPrimIndexMask || d->cuboid_count > kPrimIndexMask)
        return fail(ctx, OCTPT_ERR_UNSUPPORTED, "more than 2^27 - 1 spheres or cuboids");
    if (d->sphere_count && !d->spheres) return fail(ctx, OCTPT_ERR_INVALID_ARG, "spheres is NULL");
    if (d->cuboid_count && !d->cuboids) return fail(ctx, OCTPT_ERR_INVALID_ARG, "cuboids is NULL");
    if (d->blocks) {  // block-value leaves (C23): the payloads are block ids, there are no primitives
        if (!with_octree) return fail(ctx, OCTPT_ERR_INVALID_ARG, "a block-value scene is uploaded with its octree");
        if (d->block_count == 0) return fail(ctx, OCTPT_ERR_INVALID_ARG, "block table is empty");
        if (d->block_count > kPrimIndexMask + 1u) return fail(ctx, OCTPT_ERR_UNSUPPORTED, "more than 2^27 blocks");
        if (d->leaf_first || d->leaf_count || d->leaf_table_size || d->leaf_prims || d->leaf_prim_count ||
            d->sphere_count || d->cuboid_count || d->cuboid_model)
            return fail(ctx, OCTPT_ERR_INVALID_ARG,
                        "a block-value scene has no leaf primitive lists, spheres, cuboids or cuboid models");
    } else if (d->block_count) {
        return fail(ctx, OCTPT_ERR_INVALID_ARG, "block_count without blocks");
    }
    return OCTPT_OK;
}

// masks (out): every octant's child mask in the reader form (C21)
octpt_status validate_scene(octpt_ctx *ctx, const octpt_scene_desc *d, std::vector<uint16_t> &masks) {
    octpt_status st = validate_head(ctx, d, true);
    if (st != OCTPT_OK) return st;
    // both octant encodings are accepted (C21): (present, leaf bit) = (1,0) or set_mask_for's (0,1)
    masks.resize(d->octant_count);
    for (uint32_t n = 0; n < d->octant_count; ++n) {
        const octpt_octant &o = d->octants[n];
        const uint32_t m = masks[n] = normalized_mask(o.child_mask);
        for (int i = 0; i < 8; ++i) {
            const bool present = (m >> i) & 1, leaf = (m >> (i + 8)) & 1;
            if (!present) continue;
            if (leaf && o.children[i] >= (d->blocks ? d->block_count : d->leaf_table_size))
                return fail(ctx, OCTPT_ERR_INVALID_ARG, "octant " + std::to_string(n) + " child " + std::to_string(i) +
                                                            (d->blocks ? ": block " : ": leaf payload ") +
                                                            std::to_string(o.children[i]) + " out of range");
            if (!leaf && o.children[i] >= d->octant_count)
                return fail(ctx, OCTPT_ERR_INVALID_ARG, "octant " + std::to_string(n) + " child " + std::to_string(i) +
                                                            ": child octant index " + std::to_string(o.children[i]) +
                                                            " out of range");
        }
    }
    std::vector<int8_t> h(d->octant_count, -1);
    const int height = subtree_height(*d, masks, d->root, h, 0);
    if (height < 0) return fail(ctx, OCTPT_ERR_INVALID_ARG, "octree contains a cycle");
    if ((uint32_t)height > d->depth) return fail(ctx, OCTPT_ERR_INVALID_ARG, "octree is deeper than its declared depth");
    for (uint32_t l = 0; l < d->leaf_table_size; ++l)
        if ((uint64_t)d->leaf_first[l] + d->leaf_count[l] > d->leaf_prim_count)
            return fail(ctx, OCTPT_ERR_INVALID_ARG, "leaf range exceeds leaf_prims");
    for (uint32_t k = 0; k < d->leaf_prim_count; ++k) {
        const uint32_t p = d->leaf_prims[k];
        if (p & kPrimCuboidBit) {
            if ((p & ~kPrimCuboidBit) >= d->cuboid_count) return fail(ctx, OCTPT_ERR_INVALID_ARG, "cuboid index out of range");
        } else if (p >= d->sphere_count) {
            return fail(ctx, OCTPT_ERR_INVALID_ARG, "sphere index out of range");
        }
    }
    return validate_tables(ctx, d);
}

// primitive materials, block models, materials and textures
octpt_status validate_tables(octpt_ctx *ctx, const octpt_scene_desc *d) {
    for (uint32_t s = 0; s < d->sphere_count; ++s)
        if (d->spheres[s].material >= d->material_count) return fail(ctx, OCTPT_ERR_INVALID_ARG, "sphere material out of range");
    for (uint32_t c = 0; c < d->cuboid_count; ++c)
        for (int f = 0; f < 6; ++f)
            if (d->cuboids[c].face_material[f] >= d->material_count)
                return fail(ctx, OCTPT_ERR_INVALID_ARG, "cuboid material out of range");
    // block-value leaves (C23)
    for (uint32_t b = 0; d->blocks && b < d->block_count; ++b) {
        const octpt_block &x = d->blocks[b];
        if (x.model != OCTPT_MODEL_NONE) {
            if (x.model >= d->model_count) return fail(ctx, OCTPT_ERR_INVALID_ARG, "block model index out of range");
        } else {
            for (int f = 0; f < 6; ++f)
                if (x.face_material[f] >= d->material_count)
                    return fail(ctx, OCTPT_ERR_INVALID_ARG, "block face material out of range");
        }
    }
    if (d->blocks && d->quad_count > kPrimIndexMask)  // a quad hit record is kPrimCuboidBit | quad (C23)
        return fail(ctx, OCTPT_ERR_UNSUPPORTED, "more than 2^27 quads in a block-value scene");
    // block models (C19; and of block-value scenes, C23)
    if (d->cuboid_model || d->blocks) {
        if (d->model_count && !d->models) return fail(ctx, OCTPT_ERR_INVALID_ARG, "models is NULL");
        if (d->quad_count && !d->quads) return fail(ctx, OCTPT_ERR_INVALID_ARG, "quads is NULL");
        if (d->quad_count >= kQuadKey) return fail(ctx, OCTPT_ERR_UNSUPPORTED, "more than 2^30 - 1 quads");
        for (uint32_t c = 0; d->cuboid_model && c < d->cuboid_count; ++c) {
            const uint32_t m = d->cuboid_model[c];
            if (m == OCTPT_MODEL_NONE) continue;
            if (m >= d->model_count) return fail(ctx, OCTPT_ERR_INVALID_ARG, "cuboid model index out of range");
            const octpt_cuboid &b = d->cuboids[c];
            for (int a = 0; a < 3; ++a)
                if (b.max[a] != b.min[a] + 1.0f)
                    return fail(ctx, OCTPT_ERR_INVALID_ARG, "a block-model cuboid must be a unit voxel [min, min+1)");
        }
        for (uint32_t m = 0; m < d->model_count; ++m)
            if ((uint64_t)d->models[m].first_quad + d->models[m].quad_count > d->quad_count)
                return fail(ctx, OCTPT_ERR_INVALID_ARG, "model quad range exceeds quads");
        for (uint32_t q = 0; q < d->quad_count; ++q)
            if (d->quads[q].material >= d->material_count)
                return fail(ctx, OCTPT_ERR_INVALID_ARG, "quad material out of range");
    }
    for (uint32_t m = 0; m < d->material_count; ++m)
        if (d->materials[m].texture_index >= d->texture_count)
            return fail(ctx, OCTPT_ERR_INVALID_ARG, "material texture_index out of range");
    for (uint32_t t = 0; t < d->texture_count; ++t) {
        const octpt_texture &x = d->textures[t];
        if (x.kind == OCTPT_TEXTURE_IMAGE) {
            if (x.width == 0 || x.height == 0 || !x.pixels)
                return fail(ctx, OCTPT_ERR_INVALID_ARG, "image texture without pixels");
        } else if (x.kind != OCTPT_TEXTURE_COLOR) {
            return fail(ctx, OCTPT_ERR_INVALID_ARG, "unknown texture kind");
        }
    }
    return OCTPT_OK;
}

// The octree-independent part of a scene upload: primitive tables (host_prims; the device build
// writes them itself), block models (C19), materials, textures, LUTs and the sun.  S's octree
// fields are set by the caller.
octpt_status upload_tables(octpt_ctx *ctx, const octpt_scene_desc *d, bool host_prims, DevScene &S) {
    if (host_prims) {
        std::vector<float4> sph(d->sphere_count);
        std::vector<uint32_t> sph_mat(d->sphere_count);
        for (uint32_t s = 0; s < d->sphere_count; ++s) {
            const octpt_sphere &x = d->spheres[s];
            sph[s] = make_float4(x.center[0], x.center[1], x.center[2], x.radius);
            sph_mat[s] = x.material;
        }
        std::vector<float4> cmin(d->cuboid_count);
        std::vector<float2> cmax(d->cuboid_count);
        std::vector<uint32_t> cmat((size_t)d->cuboid_count * 6);
        for (uint32_t c = 0; c < d->cuboid_count; ++c) {
            const octpt_cuboid &x = d->cuboids[c];
            cmin[c] = make_float4(x.min[0], x.min[1], x.min[2], x.max[0]);
            cmax[c] = make_float2(x.max[1], x.max[2]);
            std::memcpy(&cmat[(size_t)c * 6], x.face_material, 24);
        }
        float4 *d_sph, *d_cmin;
        float2 *d_cmax;
        uint32_t *d_sph_mat, *d_cmat;
        HIP_TRY(ctx, upload(ctx, sph.data(), sph.size(), &d_sph));
        HIP_TRY(ctx, upload(ctx, sph_mat.data(), sph_mat.size(), &d_sph_mat));
        HIP_TRY(ctx, upload(ctx, cmin.data(), cmin.size(), &d_cmin));
        HIP_TRY(ctx, upload(ctx, cmax.data(), cmax.size(), &d_cmax));
        HIP_TRY(ctx, upload(ctx, cmat.data(), cmat.size(), &d_cmat));
        S.spheres = d_sph;
        S.sphere_mat = d_sph_mat;
        S.cub_a = d_cmin;
        S.cub_b = d_cmax;
        S.cub_mat = d_cmat;
    }
    // block models (C19): Quad::new (quad.rs:90-114) in glam's f32 operation order
    bool has_models = false;  // the scene draws block models (from cuboids, C19, or from blocks, C23)
    if (d->cuboid_model)
        for (uint32_t c = 0; c < d->cuboid_count && !has_models; ++c) has_models = d->cuboid_model[c] != OCTPT_MODEL_NONE;
    for (uint32_t b = 0; d->blocks && b < d->block_count && !has_models; ++b)
        has_models = d->blocks[b].model != OCTPT_MODEL_NONE;
    std::vector<DevQuad> quads;
    std::vector<uint2> models;
    if (has_models) {
        quads.resize(d->quad_count);
        for (uint32_t q = 0; q < d->quad_count; ++q) quads[q] = make_dev_quad(d->quads[q]);
        models.resize(d->model_count);
        for (uint32_t m = 0; m < d->model_count; ++m) models[m] = make_uint2(d->models[m].first_quad, d->models[m].quad_count);
    }
    float lf[256];
    uint8_t lb[256];
    make_luts(lf, lb);
    std::vector<DevMaterial> mats(d->material_count);
    for (uint32_t m = 0; m < d->material_count; ++m) {
        const octpt_material &x = d->materials[m];
        const octpt_texture &t = d->textures[x.texture_index];
        DevMaterial dm{};
        dm.ior = x.ior;
        dm.specular = x.specular;
        dm.emittance = x.emittance;
        dm.roughness = x.roughness;
        dm.metalness = x.metalness;
        dm.texture_index = x.texture_index;
        dm.flags = x.flags;
        dm.texture_kind = t.kind;
        if (t.kind == OCTPT_TEXTURE_COLOR) {  // F32Color::from(&U8Color) (colors/mod.rs:280-288)
            dm.color[0] = lf[t.rgba[0]];
            dm.color[1] = lf[t.rgba[1]];
            dm.color[2] = lf[t.rgba[2]];
            dm.color[3] = (float)t.rgba[3] / 255.0f;
        }
        mats[m] = dm;
    }
    std::vector<DevTexture> texs(d->texture_count);
    std::vector<uint8_t> texels;
    for (uint32_t t = 0; t < d->texture_count; ++t) {
        const octpt_texture &x = d->textures[t];
        DevTexture dt{};
        dt.kind = x.kind;
        dt.rgba = (uint32_t)x.rgba[0] | ((uint32_t)x.rgba[1] << 8) | ((uint32_t)x.rgba[2] << 16) | ((uint32_t)x.rgba[3] << 24);
        if (x.kind == OCTPT_TEXTURE_IMAGE) {
            dt.width = x.width;
            dt.height = x.height;
            dt.offset = texels.size();
            texels.insert(texels.end(), x.pixels, x.pixels + (size_t)x.width * x.height * 4);
        }
        texs[t] = dt;
    }
    DevMaterial *d_mats;
    DevTexture *d_texs;
    uint8_t *d_texels;
    HIP_TRY(ctx, upload(ctx, mats.data(), mats.size(), &d_mats));
    HIP_TRY(ctx, upload(ctx, texs.data(), texs.size(), &d_texs));
    HIP_TRY(ctx, upload(ctx, texels.data(), texels.size(), &d_texels));
    uint32_t *d_cmodel = nullptr;
    uint2 *d_models = nullptr;
    DevQuad *d_quads = nullptr;
    if (has_models) {
        if (d->cuboid_model) HIP_TRY(ctx, upload(ctx, d->cuboid_model, d->cuboid_count, &d_cmodel));
        HIP_TRY(ctx, upload(ctx, models.data(), models.size(), &d_models));
        HIP_TRY(ctx, upload(ctx, quads.data(), quads.size(), &d_quads));
    }
    uint32_t *d_blk_mat = nullptr, *d_blk_model = nullptr;
    if (d->blocks) {  // C23: six face materials and the model of every block
        std::vector<uint32_t> bm((size_t)d->block_count * 6), bmod(d->block_count);
        for (uint32_t b = 0; b < d->block_count; ++b) {
            std::memcpy(&bm[(size_t)b * 6], d->blocks[b].face_material, 24);
            bmod[b] = d->blocks[b].model;
        }
        HIP_TRY(ctx, upload(ctx, bm.data(), bm.size(), &d_blk_mat));
        HIP_TRY(ctx, upload(ctx, bmod.data(), bmod.size(), &d_blk_model));
    }
    S.depth = d->depth;
    S.has_cuboids = d->cuboid_count ? 1u : 0u;
    S.octree_scale = ldexpf(1.0f, -(int)d->depth);  // Octree::scale (new_octree.rs:40-42)
    S.inv_octree_scale = ldexpf(1.0f, (int)d->depth);
    S.cub_model = d_cmodel;
    S.models = d_models;
    S.quads = d_quads;
    // the cuboid-model path (C19) of the primitive kernels; block-value scenes draw their models in
    // the block instance (has_blocks)
    S.has_models = (has_models && !d->blocks) ? 1u : 0u;
    S.has_blocks = d->blocks ? 1u : 0u;
    S.n_blocks = d->blocks ? d->block_count : 0u;
    S.blk_mat = d_blk_mat;
    S.blk_model = d_blk_model;
    S.mats = d_mats;
    S.n_mats = d->material_count;
    S.texs = d_texs;
    S.n_texs = d->texture_count;
    S.has_images = 0u;
    for (uint32_t t = 0; t < d->texture_count; ++t)
        if (d->textures[t].kind == OCTPT_TEXTURE_IMAGE) S.has_images = 1u;
    S.texels = d_texels;
    S.lut_float = ctx->d_lut_float;
    make_sun(d->sun, lf, S.sun);
    S.sun.f_sub_surface = d->f_sub_surface;
    S.emitters = d->emitters_enabled ? 1 : 0;
    // the lean path state (WaveBuffers::lean): a continuing path's radiance is 0 when nothing adds light
    // before its end -- no emitting material (shade_segment adds emittance > EPSILON when emitters are on)
    // and no sun sampling (C18 adds the sun's direct light mid-path)
    bool emissive = false;
    for (uint32_t i = 0; i < d->material_count && d->emitters_enabled; ++i)
        emissive = emissive || d->materials[i].emittance > 5e-8f;  // RAY_EPSILON
    ctx->lean_scene = !emissive && !d->sun.sun_sampling;
    return OCTPT_OK;
}

// The slot flags of every block (C23, kBlock* in octpt_internal.h): kBlockIsModel for a block model, else
// bit f for a face whose material's texture holds a texel of alpha byte 0 -- the only texels that
// SingleBlockModel::intersect's alpha test (texel alpha <= EPSILON, C23) rejects -- so that the leaf test
// reads a texel only where it can decide something
std::vector<uint32_t> block_slot_flags(const octpt_scene_desc *d) {
    std::vector<int8_t> tex_zero(d->texture_count, -1);
    auto zero_alpha = [&](uint32_t t) {
        if (tex_zero[t] < 0) {
            const octpt_texture &x = d->textures[t];
            bool z = false;
            if (x.kind == OCTPT_TEXTURE_COLOR) {
                z = x.rgba[3] == 0;
            } else {
                const size_t n = (size_t)x.width * x.height;
                for (size_t k = 0; k < n && !z; ++k) z = x.pixels[4 * k + 3] == 0;
            }
            tex_zero[t] = z ? 1 : 0;
        }
        return tex_zero[t] != 0;
    };
    std::vector<uint32_t> flags(d->block_count, 0u);
    for (uint32_t b = 0; b < d->block_count; ++b) {
        const octpt_block &x = d->blocks[b];
        if (x.model != OCTPT_MODEL_NONE) {
            flags[b] = kBlockIsModel;
            continue;
        }
        for (uint32_t f = 0; f < 6; ++f)
            if (zero_alpha(d->materials[x.face_material[f]].texture_index)) flags[b] |= 1u << f;
    }
    return flags;
}

uint32_t tiles_of_shard(uint32_t n_tiles, uint32_t shard, uint32_t count) {
    return shard < n_tiles ? (n_tiles - shard + count - 1) / count : 0;
}

octpt_status make_render(octpt_ctx *ctx, const octpt_render_params *p, DevRender &R) {
    if (!p) return fail(ctx, OCTPT_ERR_INVALID_ARG, "render params NULL");
    if (!ctx->has_scene) return fail(ctx, OCTPT_ERR_INVALID_ARG, "no scene uploaded (set_scene)");
    if (!ctx->has_camera) return fail(ctx, OCTPT_ERR_INVALID_ARG, "no camera set");
    if (p->width == 0 || p->height == 0 || (uint64_t)p->width * p->height >= (1ull << 31))
        return fail(ctx, OCTPT_ERR_INVALID_ARG, "bad resolution");
    if (p->max_depth == 0) return fail(ctx, OCTPT_ERR_INVALID_ARG, "max_depth must be >= 1");
    const uint32_t B = p->branch_count ? p->branch_count : 1u;
    if (B > 64u) return fail(ctx, OCTPT_ERR_INVALID_ARG, "branch_count must be <= 64");
    if (p->shard_count == 0 || p->shard_index >= p->shard_count) return fail(ctx, OCTPT_ERR_INVALID_ARG, "bad shard");
    if ((uint64_t)p->spp_start + p->spp_count >= (1ull << 24))
        return fail(ctx, OCTPT_ERR_INVALID_ARG, "spp_start + spp_count must stay below 2^24");
    R.W = p->width;
    R.H = p->height;
    R.spp_start = p->spp_start;
    R.spp_count = p->spp_count;
    R.max_depth = p->max_depth;
    R.seed = p->seed;
    R.shard_index = p->shard_index;
    R.shard_count = p->shard_count;
    R.compact = (p->flags & OCTPT_RENDER_SHARD_COMPACT) ? 1u : 0u;
    ctx->ktiming = (p->flags & OCTPT_RENDER_KERNEL_TIMING) != 0;
    R.tiles_x = (p->width + kTile - 1) / kTile;
    const uint32_t tiles_y = (p->height + kTile - 1) / kTile;
    R.shard_tiles = tiles_of_shard(R.tiles_x * tiles_y, p->shard_index, p->shard_count);
    R.total_items = R.shard_tiles * 64u;
    R.div_tiles_x = udiv_magic(R.tiles_x);
    R.div_items = udiv_magic(R.total_items);
    R.dim = (float)std::max(p->width, p->height);
    R.jlo = -1.0f / R.dim;
    R.jhi = 1.0f / R.dim;
    R.subs = nullptr;
    R.beam = nullptr;
    R.beam_tx = (p->width + kBeamTile - 1) / kBeamTile;
    R.tile_order = nullptr;
    if (!ctx->h_order.empty()) {  // a tile order applies to the frame size it was set for
        if (p->width != ctx->order_w || p->height != ctx->order_h)
            return fail(ctx, OCTPT_ERR_INVALID_ARG,
                        "render size differs from the tile order's (octpt_set_tile_order; NULL resets it)");
        R.tile_order = ctx->d_order;
    }
    if (B > 1u && !(p->flags & OCTPT_RENDER_PREVIEW)) {
        // TileRenderer pass schedule (tile_renderer.rs:416-484, C20): the call covers whole passes
        if (p->flags & OCTPT_RENDER_MEGAKERNEL)
            return fail(ctx, OCTPT_ERR_UNSUPPORTED, "branch_count > 1 runs on the wavefront path only");
        uint64_t spp = 0;
        while (spp < p->spp_start) spp += current_branch_count((uint32_t)spp, B);
        if (spp != p->spp_start)
            return fail(ctx, OCTPT_ERR_INVALID_ARG, "spp_start is not a pass boundary of the branch schedule");
        const uint64_t end = (uint64_t)p->spp_start + p->spp_count;
        ctx->h_subs.clear();
        while (spp < end) {
            const uint32_t bc = current_branch_count((uint32_t)spp, B);
            for (uint32_t b = 0; b < bc; ++b) ctx->h_subs.push_back(make_uint2((uint32_t)spp, bc | (b << 16)));
            spp += bc;
        }
        if (spp != end)
            return fail(ctx, OCTPT_ERR_INVALID_ARG, "spp_start + spp_count is not a pass boundary of the branch schedule");
        if (!ctx->h_subs.empty()) {
            HIP_TRY(ctx, hipDeviceSynchronize());  // an earlier render may still read the table
            if (ctx->h_subs.size() > ctx->subs_cap) {
                if (ctx->d_subs) (void)hipFree(ctx->d_subs);
                ctx->d_subs = nullptr;
                ctx->subs_cap = 0;
                HIP_TRY(ctx, hipMalloc(&ctx->d_subs, ctx->h_subs.size() * sizeof(uint2)));
                ctx->subs_cap = ctx->h_subs.size();
            }
            HIP_TRY(ctx, hipMemcpy(ctx->d_subs, ctx->h_subs.data(), ctx->h_subs.size() * sizeof(uint2),
                                   hipMemcpyHostToDevice));
            R.subs = ctx->d_subs;
        }
    }
    // RendererMode::Preview renders one replacing pass; spp and max_depth do not apply (C16)
    R.preview = (p->flags & OCTPT_RENDER_PREVIEW) ? 1u : 0u;
    if (R.preview) R.spp_count = 1u;
    return OCTPT_OK;
}

size_t accum_pixels(const DevRender &R) { return R.compact ? (size_t)R.total_items : (size_t)R.W * R.H; }

// wavefront-state allocations, counted against the optional mem_limit
hipError_t wave_malloc(octpt_ctx *ctx, void **p, size_t bytes) {
    *p = nullptr;
    if (ctx->mem_limit && ctx->wave_bytes + bytes > ctx->mem_limit) return hipErrorOutOfMemory;
    const hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return e;
    ctx->wave_bytes += bytes;
    ctx->wave_sizes.emplace_back(*p, bytes);
    return hipSuccess;
}
void wave_free(octpt_ctx *ctx, void *&p) {
    if (!p) return;
    for (size_t i = 0; i < ctx->wave_sizes.size(); ++i)
        if (ctx->wave_sizes[i].first == p) {
            ctx->wave_bytes -= ctx->wave_sizes[i].second;
            ctx->wave_sizes.erase(ctx->wave_sizes.begin() + (ptrdiff_t)i);
            break;
        }
    (void)hipFree(p);
    p = nullptr;
}
// the queues and path state (ctx->wave_allocs)
void free_queues(octpt_ctx *ctx) {
    for (void *p : ctx->wave_allocs) wave_free(ctx, p);
    ctx->wave_allocs.clear();
    ctx->pool = 0;
    ctx->wb.hit4 = nullptr;  // allocated with the queues (block-value scenes)
}

void free_wave(octpt_ctx *ctx) {
    free_queues(ctx);
    wave_free(ctx, ctx->color_alloc);
    wave_free(ctx, ctx->nee_alloc);
    ctx->pool = ctx->color_cap = ctx->nee_pool = 0;
    ctx->wb = WaveBuffers{};
}

template <class T>
hipError_t wave_alloc(octpt_ctx *ctx, size_t n, T **out) {
    void *p = nullptr;
    const hipError_t e = wave_malloc(ctx, &p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) return e;
    ctx->wave_allocs.push_back(p);
    *out = static_cast<T *>(p);
    return hipSuccess;
}

// host snapshot of the iteration's counters, read kLookahead iterations later: the kSegs segment counts
// of the queue the iteration's shade filled, then the kSegs chunk item claims (two strided copies of one
// word per 256-B counter line, not the whole 80-KB ctrl block)
constexpr uint32_t kCountSpan = 2u * kSegs;

// queue segment capacity: seed wave w fills segment w % kSegs, so ceil(ceil(pool / 64) / kSegs) waves
size_t seg_cap_for(size_t pool) { return ((pool + 63) / 64 + kSegs - 1) / kSegs * 64; }

// which allocation of ensure_wave ran out of device memory
enum OomPart { kOomNone = 0, kOomQueues, kOomColor, kOomNee };

// The wavefront state of a render: `pool` path slots of queues + path state, `color_items` colour
// records, and (nee) the sun-sampling planes of every slot.  Grow-only.  When the queues + path state
// do not fit (another tenant, the host application's own allocations) the pool halves down to kMinPool
// and the pool obtained becomes the context's cap (pool_cap), so later renders neither retry the larger
// pool nor re-allocate.  A colour or sun-sampling allocation that fails returns OOM with *part set; the
// caller shrinks the chunk or the pool and calls again (enqueue_wavefront).
octpt_status ensure_wave(octpt_ctx *ctx, size_t pool, size_t color_items, bool nee, bool blocks, OomPart *part) {
    *part = kOomNone;
    if (!ctx->h_count) {
        // coherent (fine-grained) pinned memory: wf_snapshot_kernel's stores reach the host directly
        HIP_TRY(ctx, hipHostMalloc(reinterpret_cast<void **>(&ctx->h_count), (kLookahead + 1) * kCountSpan * sizeof(uint32_t),
                                   hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(ctx, hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->d_count), ctx->h_count, 0));
        for (auto &ev : ctx->count_ev) HIP_TRY(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    if (pool > ctx->pool) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        free_queues(ctx);
        WaveBuffers &B = ctx->wb;
        // queues + path state: 124 B per slot
        size_t want = pool;
        for (;;) {
            B.seg_cap = (uint32_t)seg_cap_for(want);
            const size_t qlen = (size_t)kSegs * B.seg_cap;  // queue positions
            hipError_t e = wave_alloc(ctx, qlen, &B.ray0[0]);
            if (e == hipSuccess) e = wave_alloc(ctx, qlen, &B.ray0[1]);
            if (e == hipSuccess) e = wave_alloc(ctx, qlen, &B.ray1[0]);
            if (e == hipSuccess) e = wave_alloc(ctx, qlen, &B.ray1[1]);
            // pa, pb: per slot, or (the lean state) per position of queue 0 / 1; pc: per slot, or both queues
            if (e == hipSuccess) e = wave_alloc(ctx, qlen, &B.pa);
            if (e == hipSuccess) e = wave_alloc(ctx, qlen, &B.pb);
            if (e == hipSuccess) e = wave_alloc(ctx, 2 * qlen, &B.pc);
            if (e == hipSuccess) e = wave_alloc(ctx, want, &B.item0);
            if (e == hipSuccess) e = wave_alloc(ctx, qlen, &B.hit);
            if (e == hipSuccess) e = wave_alloc(ctx, kCtrlWords, &B.ctrl);
            if (e == hipSuccess) break;
            free_queues(ctx);
            (void)hipGetLastError();
            if (e != hipErrorOutOfMemory || want <= kMinPool) {
                *part = kOomQueues;
                return hip_fail(ctx, e, "wave buffers");
            }
            want = std::max<size_t>(want / 2, kMinPool);
        }
        if (want < pool) {
            if (!ctx->oom_warned)
                std::fprintf(stderr, "octpt: %zu path slots did not fit in device memory; using %zu\n", pool, want);
            ctx->oom_warned = true;
            ctx->pool_cap = (uint32_t)want;  // sticky: later renders ask for at most what fitted
        }
        B.pool = (uint32_t)want;
        ctx->pool = want;
        ctx->wave_allocs_n++;
    }
    // block-value scenes (C23): their 16-B hit records (t, u, v beside the block), one per queue position
    if (blocks && !ctx->wb.hit4) {
        const hipError_t e = wave_alloc(ctx, (size_t)kSegs * ctx->wb.seg_cap, &ctx->wb.hit4);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            *part = kOomNee;  // a per-slot plane like the sun-sampling ones: the pool shrinks
            return hip_fail(ctx, e, "block hit coordinates");
        }
    }
    // sun-sampling planes (4 x 16 B per slot) only for scenes that sample the sun (C18)
    if (nee && ctx->nee_pool < ctx->pool) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        wave_free(ctx, ctx->nee_alloc);
        ctx->nee_pool = 0;
        const hipError_t e = wave_malloc(ctx, &ctx->nee_alloc, 4 * ctx->pool * sizeof(float4));
        if (e != hipSuccess) {
            (void)hipGetLastError();
            *part = kOomNee;
            return hip_fail(ctx, e, "sun-sampling planes");
        }
        ctx->nee_pool = ctx->pool;
    }
    ctx->wb.pd = static_cast<float4 *>(ctx->nee_alloc);
    if (color_items > ctx->color_cap) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        wave_free(ctx, ctx->color_alloc);
        ctx->color_cap = 0;
        const hipError_t e = wave_malloc(ctx, &ctx->color_alloc, color_items * sizeof(float4));
        if (e != hipSuccess) {
            (void)hipGetLastError();
            *part = kOomColor;
            return hip_fail(ctx, e, "colour records");
        }
        ctx->color_cap = color_items;
    }
    ctx->wb.color = static_cast<float4 *>(ctx->color_alloc);
    ctx->wb.pool = (uint32_t)ctx->pool;
    return OCTPT_OK;
}

// begin / end a timed kernel launch of `kind` on stream s (no-op unless ctx->ktiming)
octpt_status ktimer_begin(octpt_ctx *ctx, hipStream_t s, EventPair &ev) {
    if (!ctx->ktiming) return OCTPT_OK;
    if (ctx->ev_pool.empty()) {
        EventPair e{};
        HIP_TRY(ctx, hipEventCreate(&e.start));
        HIP_TRY(ctx, hipEventCreate(&e.stop));
        ctx->ev_pool.push_back(e);
    }
    ev = ctx->ev_pool.back();
    ctx->ev_pool.pop_back();
    HIP_TRY(ctx, hipEventRecord(ev.start, s));
    return OCTPT_OK;
}
octpt_status ktimer_end(octpt_ctx *ctx, hipStream_t s, int kind, const EventPair &ev) {
    if (!ctx->ktiming) return OCTPT_OK;
    ctx->kpending.emplace_back(kind, ev);
    HIP_TRY(ctx, hipEventRecord(ev.stop, s));
    return OCTPT_OK;
}

// megakernel variant (OCTPT_RENDER_MEGAKERNEL): one persistent launch per call
octpt_status enqueue_megakernel(octpt_ctx *ctx, const DevRender &R, float4 *d_accum, uint32_t *d_seg, hipStream_t s) {
    uint32_t *counter = ctx->d_counters + (ctx->launch_seq++ % kCounterRing);
    HIP_TRY(ctx, hipMemsetAsync(counter, 0, sizeof(uint32_t), s));
    int &bpc = ctx->blocks_per_cu_cache[ctx->S.depth];
    if (bpc == 0) bpc = render_blocks_per_cu(ctx->S.depth);
    const uint64_t needed = ((uint64_t)R.total_items + kBlock - 1) / kBlock;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(needed, (uint64_t)ctx->num_cu * bpc));
    HIP_TRY(ctx, launch_render(ctx->S, ctx->C, R, d_accum, d_seg, counter, ctx->d_stats, grid, s));
    return OCTPT_OK;
}

// wavefront path tracer: per chunk of passes, seed the path pool, then
// alternate extend/shade until the ray queue drains, then resolve the running means.  The
// host steers the loop with a one-iteration lookahead on the queue length.
octpt_status enqueue_wavefront(octpt_ctx *ctx, const DevRender &R, float4 *d_accum, uint32_t *d_seg, hipStream_t s,
                               const std::atomic<bool> *cancel) {
    const uint64_t n_px = R.total_items;
    uint32_t chunk_spp = 1;
    uint64_t chunk_max = 0;
    octpt_status st = OCTPT_OK;
    for (;;) {
        chunk_spp = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(R.spp_count, ctx->chunk_cap / n_px));
        // a branch-schedule chunk holds whole passes (<= 64 sub-samples each, C20)
        if (R.subs) chunk_spp = std::max(chunk_spp, std::min(64u, R.spp_count));
        chunk_max = (uint64_t)chunk_spp * n_px;
        if (chunk_max > kMaxChunkPaths)  // a branch pass of 64 sub-samples over > 2^25 pixels
            return fail(ctx, OCTPT_ERR_UNSUPPORTED, "a branch-schedule pass exceeds the 2^31-item chunk limit");
        OomPart part = kOomNone;
        st = ensure_wave(ctx, (size_t)std::min<uint64_t>(ctx->pool_cap, chunk_max), chunk_max,
                         ctx->S.sun.sun_sampling != 0, ctx->S.has_blocks != 0, &part);
        if (st == OCTPT_OK) break;
        if (st != OCTPT_ERR_OOM) return st;
        // out of device memory past the queues: a smaller chunk (colour records) or pool (planes), kept
        // for later renders; chunks and pools of any size render the same frame
        if (part == kOomColor && chunk_spp > 1 && !R.subs) {
            ctx->chunk_cap = (uint64_t)(chunk_spp / 2) * n_px;
            if (ctx->pool > ctx->chunk_cap) {  // release the queues too: they were sized for the larger chunk
                HIP_TRY(ctx, hipDeviceSynchronize());
                free_queues(ctx);
                ctx->pool_cap = (uint32_t)std::max<uint64_t>(kMinPool, std::min<uint64_t>(ctx->pool_cap, ctx->chunk_cap));
            }
        } else if (part == kOomNee && ctx->pool > kMinPool) {
            HIP_TRY(ctx, hipDeviceSynchronize());
            ctx->pool_cap = (uint32_t)std::max<size_t>(kMinPool, ctx->pool / 2);
            free_queues(ctx);
        } else {
            return st;
        }
        if (!ctx->oom_warned)
            std::fprintf(stderr, "octpt: wavefront state did not fit in device memory; chunk %llu items, pool cap %u\n",
                         (unsigned long long)ctx->chunk_cap, ctx->pool_cap);
        ctx->oom_warned = true;
    }
    // the pool actually held (smaller than asked after an out-of-memory fallback)
    const size_t pool = (size_t)std::min<uint64_t>(std::min<uint64_t>(ctx->pool_cap, chunk_max), ctx->pool);
    int &bpc = ctx->extend_bpc_cache[ctx->S.depth][ctx->S.has_blocks ? 3 : ctx->S.has_models ? 2 : (ctx->S.has_cuboids ? 1 : 0)];
    if (bpc == 0) bpc = extend_blocks_per_cu(ctx->S);
    const int grid_extend = ctx->num_cu * bpc;
    if (std::getenv("OCTPT_DEBUG"))
        std::fprintf(stderr, "octpt: extend %d blocks/CU x %d CUs (depth %u, cuboids %u, models %u), pool %zu\n", bpc,
                     ctx->num_cu, ctx->S.depth, ctx->S.has_cuboids, ctx->S.has_models, pool);
    // shade maps waves to queue segments: a multiple of kSegs waves (kSegs / 4 blocks)
    const int seg_blocks = (int)(kSegs * 64u / kBlock);
    // blocks per CU: what the instance's registers allow (4 with regeneration, 5 without), or OCTPT_SHADE_BPC
    const uint32_t shade_bpc_env = std::min<uint32_t>(env_u32("OCTPT_SHADE_BPC", 0u), 8u);
    auto grid_shade_of = [&](int mode) {
        int &cached = ctx->shade_bpc_cache[ctx->S.sun.sun_sampling ? 1 : 0]
                                          [shade_lds_tables(ctx->S) ? 1 : 0]
                                          [mode];
        if (cached == 0) cached = shade_blocks_per_cu(ctx->S, mode);
        const int bpc = shade_bpc_env ? (int)shade_bpc_env : cached;
        return (ctx->num_cu * bpc + seg_blocks - 1) / seg_blocks * seg_blocks;
    };
    {
        float none;
        std::memcpy(&none, &kPrimNone, sizeof none);
        ctx->wb.eye = make_float4(ctx->C.eye[0], ctx->C.eye[1], ctx->C.eye[2], none);
    }
    const WaveBuffers &B = ctx->wb;
    // the camera rays' beam starts, once per render call: every chunk's camera rays
    // share them (OCTPT_BEAM=0 switches them off; results are identical, ESVO iterations fewer)
    const float *beam = nullptr;
    if (ctx->beam) {
        const size_t n_tiles = (size_t)R.beam_tx * ((R.H + kBeamTile - 1) / kBeamTile);
        octpt_ctx::BeamKey key;
        key.scene = ctx->scene_gen;
        key.camera = ctx->camera_gen;
        key.order = ctx->order_gen;
        key.w = R.W;
        key.h = R.H;
        key.shard_index = R.shard_index;
        key.shard_count = R.shard_count;
        key.valid = true;
        if (n_tiles > ctx->beam_cap) {
            HIP_TRY(ctx, hipDeviceSynchronize());  // an earlier render may still read the table
            if (ctx->d_beam) (void)hipFree(ctx->d_beam);
            ctx->d_beam = nullptr;
            ctx->beam_cap = 0;
            ctx->beam_key.valid = false;
            HIP_TRY(ctx, hipMalloc(&ctx->d_beam, n_tiles * sizeof(float)));
            ctx->beam_cap = n_tiles;
        }
        if (!ctx->beam_ev) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->beam_ev, hipEventDisableTiming));
        if (!(key == ctx->beam_key)) {  // same scene, camera, size, shard and deal: the table is already there
            // overwriting a valid table: renders on other streams may still read it (write-after-read),
            // so the device drains first; a render on the computing stream is ordered by the stream itself
            if (ctx->beam_key.valid && (s != ctx->beam_stream || ctx->beam_shared)) HIP_TRY(ctx, hipDeviceSynchronize());
            ctx->beam_key.valid = false;
            HIP_TRY(ctx, launch_beam(ctx->S, ctx->C, R, ctx->d_beam, s));
            HIP_TRY(ctx, hipEventRecord(ctx->beam_ev, s));
            ctx->beam_key = key;
            ctx->beam_stream = s;
            ctx->beam_shared = false;
        } else {
            HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->beam_ev, 0));  // (a no-op on the stream that computed it)
            ctx->beam_shared |= s != ctx->beam_stream;  // read on another stream: a recompute drains the device
        }
        beam = ctx->d_beam;
    }
    for (uint32_t c0 = 0, c1 = 0; c0 < R.spp_count; c0 = c1) {
        c1 = c0 + std::min(chunk_spp, R.spp_count - c0);
        if (R.subs) {  // a chunk ends on a pass boundary (C20): branches of one pass resolve together
            uint32_t e = c1;
            while (e < R.spp_count && (ctx->h_subs[e].y >> 16) != 0u) --e;
            if (e <= c0) {  // one pass larger than the chunk: take the whole pass
                e = c1;
                while (e < R.spp_count && (ctx->h_subs[e].y >> 16) != 0u) ++e;
            }
            c1 = e;
        }
        DevRender Rc = R;
        Rc.spp_start = R.spp_start + c0;
        Rc.spp_count = c1 - c0;
        if (R.subs) Rc.subs = R.subs + c0;
        Rc.beam = beam;
        const uint32_t chunk_items = (uint32_t)((uint64_t)Rc.spp_count * n_px);
        HIP_TRY(ctx, hipMemsetAsync(B.ctrl, 0, kCtrlWords * sizeof(uint32_t), s));
        const uint32_t n_seed = (uint32_t)std::min<uint64_t>(pool, chunk_items);
        const bool regen = n_seed < chunk_items;  // else the seed claimed every item of the chunk
        // the lean 24-B path state: L stays 0 until the path ends, item = slot
        // (and, OCTPT_LEAN_STRICT, no branch schedule: the lean shade instances carry no first-reflection split)
        ctx->wb.lean = (!regen && ctx->lean_scene && !ctx->no_lean && !(OCTPT_LEAN_STRICT && R.subs)) ? 1u : 0u;
        const int grid_shade = grid_shade_of(shade_mode(regen, ctx->wb.lean != 0u));
        // the seed writes its camera rays as 16-B records (store_cam_ray) when every item has its pixel: the first
        // extend (cam) and shade (first = 2) decode them
        const bool cam_rec = OCTPT_CAM_RECORDS && !regen && ((Rc.W | Rc.H) & (kTile - 1u)) == 0u;
        HIP_TRY(ctx, launch_wf_seed(ctx->C, Rc, B, n_seed, chunk_items, ctx->d_stats, s));
        for (uint32_t it = 0;; ++it) {
            if (cancel && cancel->load()) return fail(ctx, OCTPT_CANCELLED, "render cancelled");
            const uint32_t q = it & 1u;
            EventPair ev{};
            if ((st = ktimer_begin(ctx, s, ev)) != OCTPT_OK) return st;
            HIP_TRY(ctx, launch_wf_extend(ctx->S, B, q, it == 0u && cam_rec, ctx->refill, grid_extend,
                                          ctx->d_stats, s));
            if ((st = ktimer_end(ctx, s, 0, ev)) != OCTPT_OK) return st;
            if ((st = ktimer_begin(ctx, s, ev)) != OCTPT_OK) return st;
            HIP_TRY(ctx, launch_wf_shade(ctx->S, ctx->C, Rc, B, q, chunk_items, it == 0u ? (cam_rec ? 2u : 1u) : 0u,
                                         regen, grid_shade, ctx->d_stats, s));
            if ((st = ktimer_end(ctx, s, 1, ev)) != OCTPT_OK) return st;
            // snapshot of the queue iteration `it` produced; the host checks the snapshot of
            // iteration it - kLookahead, so the GPU always has kLookahead iterations queued (an
            // iteration over an empty queue exits at once).  The queue only empties once every
            // chunk item is claimed: finished paths regenerate in the same shade pass.
            const uint32_t slot = it % (kLookahead + 1);
#ifdef OCTPT_SNAPSHOT_MEMCPY  // (A/B build: the two strided copies the snapshot kernel replaced)
            uint32_t *hs = ctx->h_count + slot * kCountSpan;
            HIP_TRY(ctx, hipMemcpy2DAsync(hs, sizeof(uint32_t), B.ctrl + ctr_count(q ^ 1u, 0), kCtrStride * sizeof(uint32_t),
                                          sizeof(uint32_t), kSegs, hipMemcpyDeviceToHost, s));
            HIP_TRY(ctx, hipMemcpy2DAsync(hs + kSegs, sizeof(uint32_t), B.ctrl + ctr_item(0), kCtrStride * sizeof(uint32_t),
                                          sizeof(uint32_t), kSegs, hipMemcpyDeviceToHost, s));
#else
            HIP_TRY(ctx, launch_wf_snapshot(B, q ^ 1u, ctx->d_count + slot * kCountSpan, s));
#endif
            HIP_TRY(ctx, hipEventRecord(ctx->count_ev[slot], s));
            if (it >= kLookahead) {
                const uint32_t old = (it - kLookahead) % (kLookahead + 1);
                HIP_TRY(ctx, hipEventSynchronize(ctx->count_ev[old]));
                const uint32_t *h = ctx->h_count + old * kCountSpan;  // that iteration's shade's queue, items
                uint64_t queued = 0;
                for (uint32_t k = 0; k < kSegs; ++k) queued += h[k];
                if (queued == 0u) break;  // iteration it - kLookahead + 1 onwards had nothing to do
                // Drain: every chunk item claimed and few rays left, so the queue only shrinks from
                // here (a ray yields at most one ray, and nothing regenerates).  One launch finishes the
                // paths in the queue this iteration's shade filled instead of the launch-latency-bound
                // tail of near-empty iterations.  Not in the extend timer (rocprof reports it as
                // wf_drain_kernel); its statistics (<= 4096 paths) stay in the totals.
                // (not for block-model scenes: their tails are transparent-texel chains, C5 -1 %)
                if (queued <= ctx->drain_rays && (!ctx->S.has_models || ctx->drain_models)) {
                    bool exhausted = true;
                    for (uint32_t k = 0; k < kSegs && exhausted; ++k) {
                        const uint32_t lo = (uint32_t)(((uint64_t)k * chunk_items) / kSegs);
                        const uint32_t hi = (uint32_t)(((uint64_t)(k + 1u) * chunk_items) / kSegs);
                        exhausted = h[kSegs + k] >= hi - lo;
                    }
                    if (exhausted) {
                        // one path per wave (wf_drain_kernel), four waves per block
                        const int grid = (int)std::min<uint64_t>((queued + 3) / 4 + 1, (uint64_t)ctx->num_cu * 16u);
                        HIP_TRY(ctx, launch_wf_drain(ctx->S, Rc, B, q ^ 1u, grid, ctx->d_stats, s));
                        break;
                    }
                }
            }
        }
        HIP_TRY(ctx, launch_wf_resolve(Rc, B, Rc.spp_count, d_accum, d_seg, s));
    }
    return OCTPT_OK;
}

octpt_status enqueue_render(octpt_ctx *ctx, const DevRender &R, float4 *d_accum, uint32_t *d_seg, hipStream_t s,
                            bool megakernel, const std::atomic<bool> *cancel = nullptr) {
    if (R.spp_count == 0 || R.total_items == 0) return OCTPT_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    EventPair ev{};
    HIP_TRY(ctx, hipEventCreate(&ev.start));
    HIP_TRY(ctx, hipEventCreate(&ev.stop));
    ctx->pending.push_back(ev);  // destroyed by get_stats / destroy
    HIP_TRY(ctx, hipEventRecord(ev.start, s));
    octpt_status st = OCTPT_OK;
    if (R.preview) {
        const hipError_t e = launch_preview(ctx->S, ctx->C, R, d_accum, d_seg, ctx->d_stats, s);
        if (e != hipSuccess) st = hip_fail(ctx, e, "preview launch");
    } else {
        st = megakernel ? enqueue_megakernel(ctx, R, d_accum, d_seg, s)
                        : enqueue_wavefront(ctx, R, d_accum, d_seg, s, cancel);
    }
    HIP_TRY(ctx, hipEventRecord(ev.stop, s));
    if (st == OCTPT_OK) ctx->launches++;
    return st;
}

// ---------------- multi-device contexts (octpt_create_multi) ----------------
// A multi-device context forwards every call to one child context per device entry, each a complete
// single-device context (its own scene replica, stream and wavefront state).  A render deals the caller's
// 8x8 tiles round-robin over the entries (multi_slot: the children's own shards of the kernels' tile
// split), runs each child on a host thread of its own (the wavefront loop is host-steered), and moves the
// tiles between the caller's buffers on the first device and the children's compact buffers with peer
// copies (hipMemcpyPeerAsync: xGMI DMA between MI355X devices; a plain device copy when an entry repeats
// a device).  Per-pixel RNG streams make the result bit-identical to one device's.
bool is_multi(const octpt_ctx *ctx) { return !ctx->sub.empty(); }

// fn(i) for every child i, one host thread each; the first failing entry's status and message are returned
template <class F>
octpt_status for_each_sub(octpt_ctx *ctx, F fn) {
    const size_t n = ctx->sub.size();
    std::vector<octpt_status> st(n, OCTPT_OK);
    std::vector<std::thread> th;
    th.reserve(n);
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&st, &fn, ctx, i]() {
            try {
                st[i] = fn(i);
            } catch (...) {
                st[i] = fail(ctx->sub[i], OCTPT_ERR_INTERNAL, "unexpected exception");
            }
        });
    for (auto &t : th) t.join();
    for (size_t i = 0; i < n; ++i)
        if (st[i] != OCTPT_OK)
            return fail(ctx, st[i], "device entry " + std::to_string(i) + " (HIP device " +
                                        std::to_string(ctx->sub[i]->device) + "): " + ctx->sub[i]->err);
    return OCTPT_OK;
}

// grow-only device buffer of n elements on the current device
template <class T>
octpt_status grow_buf(octpt_ctx *ctx, T *&p, size_t &cap, size_t n) {
    if (n <= cap) return OCTPT_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    HIP_TRY(ctx, hipMalloc(&p, n * sizeof(T)));
    cap = n;
    return OCTPT_OK;
}

// One render call over every device entry: scatter the caller's running mean (and segment counts) into the
// entries' compact tile buffers, render each entry's shard, gather back.  R is the call's layout (on the
// first device, stream s); the caller's buffers are read and written on s, the entries work on their own
// streams.  kernel_ms accumulates the call's wall time (the entries run concurrently).
octpt_status multi_render(octpt_ctx *ctx, const octpt_render_params &p, const DevRender &R, float4 *d_accum,
                          uint32_t *d_seg, hipStream_t s, const std::atomic<bool> *cancel) {
    if (R.spp_count == 0 || R.total_items == 0) return OCTPT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t n = (uint32_t)ctx->sub.size();
    const size_t stride = (size_t)((R.shard_tiles + n - 1) / n) * 64u;  // the largest entry's pixels
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    octpt_status st = grow_buf(ctx, ctx->m_acc, ctx->m_acc_cap, stride * n);
    if (st == OCTPT_OK && d_seg) st = grow_buf(ctx, ctx->m_seg, ctx->m_seg_cap, stride * n);
    if (st != OCTPT_OK) return st;
    HIP_TRY(ctx, launch_multi_stage(R, n, (uint32_t)stride, d_accum, d_seg, ctx->m_acc, ctx->m_seg, true, s));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    const bool megakernel = (p.flags & OCTPT_RENDER_MEGAKERNEL) != 0;
    st = for_each_sub(ctx, [&](size_t i) -> octpt_status {
        octpt_ctx *c = ctx->sub[i];
        HIP_TRY(c, hipSetDevice(c->device));
        octpt_render_params pi = p;  // entry i's shard of the caller's shard (multi_slot)
        pi.shard_index = p.shard_index + (uint32_t)i * p.shard_count;
        pi.shard_count = p.shard_count * n;
        pi.flags |= OCTPT_RENDER_SHARD_COMPACT;
        DevRender Ri{};
        octpt_status r = make_render(c, &pi, Ri);
        if (r != OCTPT_OK || Ri.total_items == 0) return r;
        const size_t np = Ri.total_items;
        if ((r = grow_buf(c, c->m_acc, c->m_acc_cap, np)) != OCTPT_OK) return r;
        if (d_seg && (r = grow_buf(c, c->m_seg, c->m_seg_cap, np)) != OCTPT_OK) return r;
        float4 *stage_acc = ctx->m_acc + i * stride;
        uint32_t *stage_seg = d_seg ? ctx->m_seg + i * stride : nullptr;
        HIP_TRY(c, hipMemcpyPeerAsync(c->m_acc, c->device, stage_acc, ctx->device, np * sizeof(float4), c->stream));
        if (d_seg) HIP_TRY(c, hipMemcpyPeerAsync(c->m_seg, c->device, stage_seg, ctx->device, np * 4, c->stream));
        r = enqueue_render(c, Ri, c->m_acc, d_seg ? c->m_seg : nullptr, c->stream, megakernel, cancel);
        if (r != OCTPT_OK) {
            (void)hipStreamSynchronize(c->stream);
            return r;
        }
        HIP_TRY(c, hipMemcpyPeerAsync(stage_acc, ctx->device, c->m_acc, c->device, np * sizeof(float4), c->stream));
        if (d_seg) HIP_TRY(c, hipMemcpyPeerAsync(stage_seg, ctx->device, c->m_seg, c->device, np * 4, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        return OCTPT_OK;
    });
    if (st != OCTPT_OK) return st;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, launch_multi_stage(R, n, (uint32_t)stride, d_accum, d_seg, ctx->m_acc, ctx->m_seg, false, s));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    ctx->kernel_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ctx->launches++;
    return OCTPT_OK;
}

void join_inflight(octpt_ctx *ctx) {
    octpt_frame *f = ctx->inflight;
    if (f && f->worker.joinable()) f->worker.join();
    ctx->inflight = nullptr;
}

void free_frame_buffers(octpt_frame *f) {
    if (f->d_accum) (void)hipFree(f->d_accum);
    if (f->d_rgba) (void)hipFree(f->d_rgba);
    if (f->h_accum) (void)hipHostFree(f->h_accum);
    if (f->h_rgba) (void)hipHostFree(f->h_rgba);
    f->d_accum = nullptr;
    f->d_rgba = nullptr;
    f->h_accum = nullptr;
    f->h_rgba = nullptr;
}

void deliver(octpt_frame *f) {
    if (f->delivered) return;
    std::memcpy(f->user_accum, f->h_accum, f->n_pixels * 16);
    if (f->user_rgba) std::memcpy(f->user_rgba, f->h_rgba, f->n_pixels * 4);
    f->delivered = true;
}

// ---------------- builder ----------------
uint64_t part_by_2(uint64_t v) {  // new_octree.rs:813-822
    uint64_t x = v & 0x1fffff;
    x = (x | x << 32) & 0x1f00000000ffffULL;
    x = (x | x << 16) & 0x1f0000ff0000ffULL;
    x = (x | x << 8) & 0x100f00f00f00f00fULL;
    x = (x | x << 4) & 0x10c30c30c30c30c3ULL;
    x = (x | x << 2) & 0x1249249249249249ULL;
    return x;
}
inline uint64_t morton(uint64_t x, uint64_t y, uint64_t z) { return (part_by_2(z) << 2) + (part_by_2(y) << 1) + part_by_2(x); }

struct CellPrim {
    uint64_t code;
    uint32_t prim;
    bool operator<(const CellPrim &o) const { return code != o.code ? code < o.code : prim < o.prim; }
};

// Pre-order octant emission.  node() returns the child its parent stores: an octant
// id, or with compaction a leaf payload when the octant's eight children are leaves holding the same
// primitive list (Octant::is_compactable, new_octree.rs:227-233, applied bottom-up at every level as
// RegionOctreeBuilder::recursive_build does, :679-690: the octant becomes Lod(get_child(0))).  The
// root is never merged away (a Lod root stays one octant of eight equal leaves, :534-545).
struct Builder {
    octpt_octree *t;
    std::vector<uint64_t> leaf_code;
    uint32_t depth;
    bool compact;
    struct Child {
        bool leaf;
        uint32_t v;
    };
    bool same_leaf(uint32_t a, uint32_t b) const {
        const uint32_t n = t->leaf_count[a];
        return n == t->leaf_count[b] &&
               std::memcmp(&t->leaf_prims[t->leaf_first[a]], &t->leaf_prims[t->leaf_first[b]], n * sizeof(uint32_t)) == 0;
    }
    Child node(uint32_t level, uint32_t lo, uint32_t hi) {
        const uint32_t id = (uint32_t)t->octants.size();
        t->octants.push_back(octpt_octant{0, 0, {0, 0, 0, 0, 0, 0, 0, 0}});
        const uint32_t shift = 3 * (depth - 1 - level);
        uint32_t a = lo;
        for (uint32_t c = 0; c < 8; ++c) {
            uint32_t b = a;
            while (b < hi && ((leaf_code[b] >> shift) & 7u) == c) ++b;
            if (b == a) continue;
            if (level + 1 == depth) {
                t->octants[id].child_mask |= (uint16_t)((1u << c) | (1u << (c + 8)));
                t->octants[id].children[c] = a;
            } else {
                const Child ch = node(level + 1, a, b);
                t->octants[id].child_mask |= (uint16_t)(ch.leaf ? ((1u << c) | (1u << (c + 8))) : (1u << c));
                t->octants[id].children[c] = ch.v;
            }
            a = b;
        }
        if (compact && level > 0 && t->octants[id].child_mask == 0xFFFFu) {
            const uint32_t *ch = t->octants[id].children;
            bool same = true;
            for (int k = 1; k < 8 && same; ++k) same = same_leaf(ch[0], ch[k]);
            if (same) {  // all children are leaves: this octant is the last one emitted
                const uint32_t v = ch[0];
                t->octants.pop_back();
                return Child{true, v};
            }
        }
        return Child{false, id};
    }
};

// Block-value octree (C23): leaf payloads are block ids.  Pre-order emission over the Morton-sorted
// cells as Builder does; with compaction an octant whose eight children are leaves holding the same
// block value becomes one leaf of its parent (Octant::is_compactable, new_octree.rs:227-233: all eight
// leaf bits set and every child value equal -- the reference's rule for leaf children), bottom-up at
// every level as SectionOctantBuilder::insert_child_and_compact / RegionOctreeBuilder::recursive_build
// apply it (:688-709, 582-587).  The root stays an octant.
struct BlockBuilder {
    octpt_octree *t;
    const std::vector<std::pair<uint64_t, uint32_t>> &cells;  // (Morton code, block), sorted
    uint32_t depth;
    bool compact;
    struct Child {
        bool leaf;
        uint32_t v;
    };
    Child node(uint32_t level, size_t lo, size_t hi) {
        const uint32_t id = (uint32_t)t->octants.size();
        t->octants.push_back(octpt_octant{0, 0, {0, 0, 0, 0, 0, 0, 0, 0}});
        const uint32_t shift = 3 * (depth - 1 - level);
        size_t a = lo;
        for (uint32_t c = 0; c < 8; ++c) {
            size_t b = a;
            while (b < hi && ((cells[b].first >> shift) & 7u) == c) ++b;
            if (b == a) continue;
            Child ch{true, cells[a].second};
            if (level + 1 < depth) ch = node(level + 1, a, b);
            t->octants[id].child_mask |= (uint16_t)(ch.leaf ? ((1u << c) | (1u << (c + 8))) : (1u << c));
            t->octants[id].children[c] = ch.v;
            a = b;
        }
        if (compact && level > 0 && t->octants[id].child_mask == 0xFFFFu) {
            const uint32_t *ch = t->octants[id].children;
            bool same = true;
            for (int k = 1; k < 8 && same; ++k) same = ch[k] == ch[0];
            if (same) {  // eight equal leaves: this octant is the last one emitted
                const uint32_t v = ch[0];
                t->octants.pop_back();
                return Child{true, v};
            }
        }
        return Child{false, id};
    }
};

inline int32_t clamp_cell(float f, int32_t hi) {
    if (!(f >= 0.0f)) return 0;  // also NaN
    if (f >= (float)hi) return hi;
    return (int32_t)f;
}

// Upper bound of the (cell, primitive) pairs: the clamped bounding-box cells of every primitive.
// Leaf tables index pairs with uint32, and a scene past 2^31 pairs (>= 32 GiB of pairs) is refused
// up front rather than discovered by allocating until bad_alloc.  Cuboid cells span floor(min) ..
// ceil(max) - 1: a face on an integer plane does not claim the next cell, so a unit block
// [x, x+1) is exactly one cell (the voxel world of C5).
uint64_t pair_bound(const octpt_sphere *spheres, uint32_t ns, const octpt_cuboid *cuboids, uint32_t nc,
                    uint32_t depth) {
    const int32_t N = 1 << depth;
    uint64_t bound = 0;
    auto cub_hi = [](float lo, float hi) { return std::max(floorf(lo), ceilf(hi) - 1.0f); };
    auto add_box = [&](const float *lo_f, const float *hi_f, bool half_open) {
        uint64_t cells = 1;
        for (int a = 0; a < 3; ++a) {
            const float fl = floorf(lo_f[a]), fh = half_open ? cub_hi(lo_f[a], hi_f[a]) : floorf(hi_f[a]);
            if (fh < 0.0f || fl > (float)(N - 1) || hi_f[a] < lo_f[a]) return;
            cells *= (uint64_t)(clamp_cell(fh, N - 1) - clamp_cell(fl, N - 1) + 1);
        }
        bound = std::min<uint64_t>(bound + cells, UINT64_MAX / 2);
    };
    for (uint32_t i = 0; i < ns; ++i) {
        const float *c = spheres[i].center, r = spheres[i].radius;
        if (!(r > 0.0f)) continue;
        const float lo_f[3] = {c[0] - r, c[1] - r, c[2] - r}, hi_f[3] = {c[0] + r, c[1] + r, c[2] + r};
        add_box(lo_f, hi_f, false);
    }
    for (uint32_t i = 0; i < nc; ++i) add_box(cuboids[i].min, cuboids[i].max, true);
    return bound;
}

}  // namespace

extern "C" {

uint32_t octpt_abi_version(void) { return OCTPT_ABI_VERSION; }

int32_t octpt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

octpt_status octpt_create(int32_t device, octpt_ctx **out) {
    if (!out) return OCTPT_ERR_INVALID_ARG;
    *out = nullptr;
    octpt_ctx *ctx = new (std::nothrow) octpt_ctx();
    if (!ctx) return OCTPT_ERR_OOM;
    auto bail = [&](octpt_status st) {
        octpt_destroy(ctx);
        return st;
    };
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return bail(OCTPT_ERR_DEVICE);
    if (device < 0 || device >= n) return bail(OCTPT_ERR_INVALID_ARG);
    hipDeviceProp_t prop{};
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return bail(OCTPT_ERR_DEVICE);
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return bail(OCTPT_ERR_DEVICE);
    ctx->device = device;
    ctx->num_cu = prop.multiProcessorCount;
    ctx->pool_cap = std::max<uint32_t>(std::min<uint32_t>(env_u32("OCTPT_POOL", kDefaultPool), kMaxPool), 64u);
    ctx->chunk_cap = std::min<uint64_t>(env_u32("OCTPT_CHUNK", (uint32_t)kDefaultChunkPaths), kMaxChunkPaths);
    // OCTPT_REFILL=n fixes the threshold (clamped to [1, 64]); unset: adaptive per wave (0)
    const char *refill_env = std::getenv("OCTPT_REFILL");
    ctx->refill = (refill_env && *refill_env)
                      ? std::max<uint32_t>(std::min<uint32_t>(env_u32("OCTPT_REFILL", 16u), 64u), 1u)
                      : kDefaultRefill;
    // OCTPT_DRAIN_RAYS=n: the drain's queue threshold; 0 turns the drain off (A/B)
    const char *drain_env = std::getenv("OCTPT_DRAIN_RAYS");
    if (drain_env && *drain_env) ctx->drain_rays = (uint32_t)std::strtoul(drain_env, nullptr, 10);
    const char *beam_env = std::getenv("OCTPT_BEAM");
    ctx->beam = !(beam_env && beam_env[0] == '0');
    const char *lean_env = std::getenv("OCTPT_LEAN");
    ctx->no_lean = lean_env && lean_env[0] == '0';
    ctx->drain_models = env_u32("OCTPT_DRAIN_MODELS", 0u) != 0u;
    ctx->mem_limit = (size_t)env_u32("OCTPT_DEVICE_MEM_LIMIT", 0u) << 20;  // MiB, test hook (ensure_wave)
    if (hipSetDevice(device) != hipSuccess) return bail(OCTPT_ERR_DEVICE);
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) return bail(OCTPT_ERR_DEVICE);
    if (hipMalloc(&ctx->d_counters, kCounterRing * sizeof(uint32_t)) != hipSuccess) return bail(OCTPT_ERR_OOM);
    if (hipMalloc(&ctx->d_stats, kStatWords * sizeof(unsigned long long)) != hipSuccess) return bail(OCTPT_ERR_OOM);
    if (hipMemset(ctx->d_stats, 0, kStatWords * sizeof(unsigned long long)) != hipSuccess) return bail(OCTPT_ERR_DEVICE);
    float lf[256];
    uint8_t lb[256];
    make_luts(lf, lb);
    if (hipMalloc(&ctx->d_lut_float, sizeof lf) != hipSuccess) return bail(OCTPT_ERR_OOM);
    if (hipMalloc(&ctx->d_lut_byte, sizeof lb) != hipSuccess) return bail(OCTPT_ERR_OOM);
    if (hipMemcpy(ctx->d_lut_float, lf, sizeof lf, hipMemcpyHostToDevice) != hipSuccess) return bail(OCTPT_ERR_DEVICE);
    if (hipMemcpy(ctx->d_lut_byte, lb, sizeof lb, hipMemcpyHostToDevice) != hipSuccess) return bail(OCTPT_ERR_DEVICE);
    *out = ctx;
    return OCTPT_OK;
}

octpt_status octpt_create_multi(const int32_t *devices, uint32_t n, octpt_ctx **out) {
    if (!out) return OCTPT_ERR_INVALID_ARG;
    *out = nullptr;
    if (!devices || n == 0 || n > 64) return OCTPT_ERR_INVALID_ARG;
    if (n == 1) return octpt_create(devices[0], out);
    int caller_device = 0;
    const bool restore = hipGetDevice(&caller_device) == hipSuccess;
    struct Restore {  // the calling thread's current device is left as it was
        bool on;
        int dev;
        ~Restore() {
            if (on) (void)hipSetDevice(dev);
        }
    } restore_device{restore, caller_device};
    try {
        octpt_ctx *ctx = nullptr;
        octpt_status st = octpt_create(devices[0], &ctx);  // the first entry's device holds the caller's buffers
        if (st != OCTPT_OK) return st;
        for (uint32_t i = 0; i < n && st == OCTPT_OK; ++i) {
            octpt_ctx *c = nullptr;
            st = octpt_create(devices[i], &c);
            if (st == OCTPT_OK) ctx->sub.push_back(c);
        }
        if (st != OCTPT_OK) {
            octpt_destroy(ctx);
            return st;
        }
        // direct peer access between the first device and every other one (xGMI); without it the peer
        // copies still work, staged by the runtime.  A pair that cannot be enabled is not an error, but it is
        // recorded: octpt_last_error then reads "note: peer access ..." 
        std::string note;
        auto enable = [&](int from, int to) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, from, to) != hipSuccess || !can) {
                note += " " + std::to_string(from) + "->" + std::to_string(to) + ": no peer path";
                return;
            }
            if (hipSetDevice(from) != hipSuccess) return;
            const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                note += " " + std::to_string(from) + "->" + std::to_string(to) + ": " + hipGetErrorString(e);
            (void)hipGetLastError();
        };
        for (uint32_t i = 1; i < n; ++i) {
            if (devices[i] == devices[0]) continue;
            enable(devices[0], devices[i]);
            enable(devices[i], devices[0]);
        }
        if (!note.empty()) ctx->err = "note: peer access not enabled (copies staged by the runtime):" + note;
        *out = ctx;
        return OCTPT_OK;
    } catch (...) {
        return OCTPT_ERR_INTERNAL;
    }
}

uint32_t octpt_device_entries(const octpt_ctx *ctx) { return !ctx ? 0u : is_multi(ctx) ? (uint32_t)ctx->sub.size() : 1u; }

void octpt_destroy(octpt_ctx *ctx) {
    if (!ctx) return;
    join_inflight(ctx);
    for (octpt_ctx *c : ctx->sub) octpt_destroy(c);
    ctx->sub.clear();
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto &e : ctx->pending) {
        (void)hipEventSynchronize(e.stop);
        (void)hipEventDestroy(e.start);
        (void)hipEventDestroy(e.stop);
    }
    for (auto &ke : ctx->kpending) ctx->ev_pool.push_back(ke.second);
    for (auto &e : ctx->ev_pool) {
        (void)hipEventSynchronize(e.stop);
        (void)hipEventDestroy(e.start);
        (void)hipEventDestroy(e.stop);
    }
    free_scene(ctx);
    free_wave(ctx);
    ctx->build_scratch.release();
    if (ctx->h_count) (void)hipHostFree(ctx->h_count);
    for (auto &ev : ctx->count_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    if (ctx->d_subs) (void)hipFree(ctx->d_subs);
    if (ctx->d_beam) (void)hipFree(ctx->d_beam);
    if (ctx->beam_ev) (void)hipEventDestroy(ctx->beam_ev);
    if (ctx->d_order) (void)hipFree(ctx->d_order);
    if (ctx->d_order_pos) (void)hipFree(ctx->d_order_pos);
    if (ctx->m_acc) (void)hipFree(ctx->m_acc);
    if (ctx->m_seg) (void)hipFree(ctx->m_seg);
    if (ctx->d_stats) (void)hipFree(ctx->d_stats);
    if (ctx->d_lut_float) (void)hipFree(ctx->d_lut_float);
    if (ctx->d_lut_byte) (void)hipFree(ctx->d_lut_byte);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *octpt_last_error(const octpt_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

octpt_status octpt_scene_upload(octpt_ctx *ctx, const octpt_scene_desc *d) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    join_inflight(ctx);
    try {
        if (is_multi(ctx)) {  // a replica on every device entry
            ctx->has_scene = false;
            const octpt_status st = for_each_sub(ctx, [&](size_t i) { return octpt_scene_upload(ctx->sub[i], d); });
            ctx->has_scene = st == OCTPT_OK;
            return st;
        }
        std::vector<uint16_t> masks;  // reader-form child masks (C21)
        octpt_status st = validate_scene(ctx, d, masks);
        if (st != OCTPT_OK) return st;
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        free_scene(ctx);
        DevScene S{};
        // sparse packed child slots: octant n's present children are stored
        // contiguously from base[n] in child order; child i is at base[n] + popcount(mask & (2^i - 1)).
        // One 8-byte load per descend / leaf visit yields the child's own base and mask.
        std::vector<uint32_t> base(d->octant_count);
        size_t n_slots = 0;
        for (uint32_t n = 0; n < d->octant_count; ++n) {
            base[n] = (uint32_t)n_slots;
            n_slots += (size_t)__builtin_popcount(masks[n] & 0xFFu);
        }
        if (n_slots >= 0xFFFFFFFFull) return fail(ctx, OCTPT_ERR_INVALID_ARG, "octree too large");
        // + 8 zero slots: a child index computed for an absent child of the last octant stays in bounds
        std::vector<uint2> child(n_slots + 8, make_uint2(0u, 0u));
        const std::vector<uint32_t> bflags = d->blocks ? block_slot_flags(d) : std::vector<uint32_t>();
        for (uint32_t n = 0; n < d->octant_count; ++n) {
            const octpt_octant &o = d->octants[n];
            uint32_t k = base[n];
            for (int i = 0; i < 8; ++i) {
                const bool present = (masks[n] >> i) & 1, leaf = (masks[n] >> (i + 8)) & 1;
                if (!present) continue;
                const uint32_t v = o.children[i];
                if (!leaf) {
                    child[k++] = make_uint2(base[v], masks[v]);
                } else if (d->blocks) {  // block-value leaf (C23): (block id, its slot flags)
                    child[k++] = make_uint2(v, bflags[v]);
                } else if (d->leaf_count[v] == 1) {  // single-primitive leaf: the prim id itself
                    child[k++] = make_uint2(d->leaf_prims[d->leaf_first[v]], 1u);
                } else {
                    child[k++] = make_uint2(d->leaf_first[v], d->leaf_count[v]);
                }
            }
        }
        // single-sphere leaf slots carry their sphere in a parallel array, so that extend loads it
        // beside the slot instead of after it (sphere-only scenes)
        std::vector<float4> leaf_sph;
        if (!d->cuboid_count && !d->blocks) {
            leaf_sph.assign(child.size(), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
            for (uint32_t n = 0; n < d->octant_count; ++n) {
                const octpt_octant &o = d->octants[n];
                uint32_t k = base[n];
                for (int i = 0; i < 8; ++i) {
                    const bool present = (masks[n] >> i) & 1, leaf = (masks[n] >> (i + 8)) & 1;
                    if (!present) continue;
                    if (leaf && d->leaf_count[o.children[i]] == 1) {
                        const octpt_sphere &x = d->spheres[d->leaf_prims[d->leaf_first[o.children[i]]]];
                        leaf_sph[k] = make_float4(x.center[0], x.center[1], x.center[2], x.radius);
                    }
                    ++k;
                }
            }
        }
        uint2 *d_child;
        HIP_TRY(ctx, upload(ctx, child.data(), child.size(), &d_child));
        float4 *d_leaf_sph = nullptr;
        if (!leaf_sph.empty()) HIP_TRY(ctx, upload(ctx, leaf_sph.data(), leaf_sph.size(), &d_leaf_sph));
        uint32_t *d_prims;
        HIP_TRY(ctx, upload(ctx, d->leaf_prims, d->leaf_prim_count, &d_prims));
        S.node_child = d_child;
        S.leaf_sph = d_leaf_sph;
        S.leaf_prims = d_prims;
        S.root = base[d->root];  // traversal "parent" values are child-array bases
        S.root_mask = masks[d->root];
        S.n_octants = d->octant_count;
        st = upload_tables(ctx, d, true, S);
        if (st != OCTPT_OK) return st;
        ctx->S = S;
        ctx->has_scene = true;
        ++ctx->scene_gen;
        return OCTPT_OK;
    } catch (const std::bad_alloc &) {
        free_scene(ctx);
        return fail(ctx, OCTPT_ERR_OOM, "host allocation failed");
    } catch (...) {
        free_scene(ctx);
        return fail(ctx, OCTPT_ERR_INTERNAL, "unexpected exception in scene upload");
    }
}

octpt_status octpt_scene_build_device(octpt_ctx *ctx, const octpt_scene_desc *d, uint32_t flags) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    join_inflight(ctx);
    if (flags & ~OCTPT_BUILD_COMPACT) return fail(ctx, OCTPT_ERR_INVALID_ARG, "unknown build flags");
    try {
        if (is_multi(ctx)) {  // every device entry builds its own replica
            ctx->has_scene = false;
            const octpt_status st =
                for_each_sub(ctx, [&](size_t i) { return octpt_scene_build_device(ctx->sub[i], d, flags); });
            ctx->has_scene = st == OCTPT_OK;
            return st;
        }
        octpt_status st = validate_head(ctx, d, false);
        if (st != OCTPT_OK) return st;
        if (d->blocks) return fail(ctx, OCTPT_ERR_INVALID_ARG, "a block-value scene is uploaded with its octree");
        st = validate_tables(ctx, d);
        if (st != OCTPT_OK) return st;
        if (pair_bound(d->spheres, d->sphere_count, d->cuboids, d->cuboid_count, d->depth) > kMaxBuildPairs)
            return fail(ctx, OCTPT_ERR_OOM, "more than 2^31 (cell, primitive) pairs");
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        free_scene(ctx);
        // the GPU builder (§4) with its result left in the build scratch
        BuiltOctree unused;
        DeviceOctree t;
        bool too_many = false;
        float ms = 0.0f;
        hipError_t e = build_octree_gpu(ctx->stream, ctx->build_scratch, d->spheres, d->sphere_count, d->cuboids,
                                        d->cuboid_count, d->depth, (flags & OCTPT_BUILD_COMPACT) != 0, kMaxBuildPairs,
                                        unused, too_many, &ms, &t);
        if (too_many) return fail(ctx, OCTPT_ERR_OOM, "octree build: out of memory");
        if (e != hipSuccess) return hip_fail(ctx, e, "octree build");
        ctx->build_ms = ms;
        // sparse child slots packed on the device, exactly as octpt_scene_upload packs them (§5)
        if ((uint64_t)t.n_octants * 8u >= 0xFFFFFFF0ull)  // the u32 slot scan cannot wrap
            return fail(ctx, OCTPT_ERR_UNSUPPORTED, "octree too large for the device build (>= 2^29 octants)");
        uint32_t *d_base = nullptr, n_slots = 0;
        HIP_TRY(ctx, slot_bases_gpu(ctx->stream, ctx->build_scratch, t, &d_base, n_slots));
        ScenePrimTables out{};
        HIP_TRY(ctx, upload<uint2>(ctx, nullptr, (size_t)n_slots + 8, &out.node_child));  // zeroed: + 8 tail slots
        if (!d->cuboid_count) HIP_TRY(ctx, upload<float4>(ctx, nullptr, (size_t)n_slots + 8, &out.leaf_sph));
        HIP_TRY(ctx, upload<uint32_t>(ctx, nullptr, t.n_leaf_prims, &out.leaf_prims));
        HIP_TRY(ctx, upload<float4>(ctx, nullptr, d->sphere_count, &out.spheres));
        HIP_TRY(ctx, upload<uint32_t>(ctx, nullptr, d->sphere_count, &out.sphere_mat));
        HIP_TRY(ctx, upload<float4>(ctx, nullptr, d->cuboid_count, &out.cub_a));
        HIP_TRY(ctx, upload<float2>(ctx, nullptr, d->cuboid_count, &out.cub_b));
        HIP_TRY(ctx, upload<uint32_t>(ctx, nullptr, (size_t)d->cuboid_count * 6, &out.cub_mat));
        HIP_TRY(ctx, fill_scene_gpu(ctx->stream, t, d_base, out));
        uint16_t root_mask = 0;  // the root is octant 0 (pre-order), base 0
        HIP_TRY(ctx, hipMemcpy(&root_mask, &t.octants[0].child_mask, sizeof root_mask, hipMemcpyDeviceToHost));
        DevScene S{};
        S.node_child = out.node_child;
        S.leaf_sph = out.leaf_sph;
        S.leaf_prims = out.leaf_prims;
        S.spheres = out.spheres;
        S.sphere_mat = out.sphere_mat;
        S.cub_a = out.cub_a;
        S.cub_b = out.cub_b;
        S.cub_mat = out.cub_mat;
        S.root = 0u;
        S.root_mask = root_mask;
        S.n_octants = t.n_octants;
        st = upload_tables(ctx, d, false, S);
        if (st != OCTPT_OK) return st;
        ctx->S = S;
        ctx->has_scene = true;
        ++ctx->scene_gen;
        return OCTPT_OK;
    } catch (const std::bad_alloc &) {
        free_scene(ctx);
        return fail(ctx, OCTPT_ERR_OOM, "host allocation failed");
    } catch (...) {
        free_scene(ctx);
        return fail(ctx, OCTPT_ERR_INTERNAL, "unexpected exception in device scene build");
    }
}

octpt_status octpt_set_camera(octpt_ctx *ctx, const octpt_camera *c) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    if (!c) return fail(ctx, OCTPT_ERR_INVALID_ARG, "camera NULL");
    if (!(c->fov > 0.0f && c->fov < 3.14159265f)) return fail(ctx, OCTPT_ERR_INVALID_ARG, "fov must be in (0, pi)");
    if (c->aperture != 0.0f) return fail(ctx, OCTPT_ERR_UNSUPPORTED, "thin-lens aperture is not used by the reference path");
    ctx->cam = *c;
    DevCamera C{};
    std::memcpy(C.eye, c->eye, 12);
    std::memcpy(C.dir, c->direction, 12);
    std::memcpy(C.up, c->up, 12);
    cross3(c->direction, c->up, C.right);            // camera.rs:80
    C.d_factor = 1.0f / tanf(c->fov / 2.0f);         // camera.rs:79
    ctx->C = C;
    ctx->has_camera = true;
    ++ctx->camera_gen;
    for (octpt_ctx *sc : ctx->sub) {
        const octpt_status st = octpt_set_camera(sc, c);
        if (st != OCTPT_OK) return fail(ctx, st, sc->err);
    }
    return OCTPT_OK;
}

octpt_status octpt_get_camera(const octpt_ctx *ctx, octpt_camera *c) {
    if (!ctx || !c) return OCTPT_ERR_INVALID_ARG;
    if (!ctx->has_camera) return OCTPT_ERR_INVALID_ARG;
    *c = ctx->cam;
    return OCTPT_OK;
}

octpt_status octpt_render_device(octpt_ctx *ctx, const octpt_render_params *p, float *d_accum, uint32_t *d_seg,
                                 void *stream) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    if (!d_accum) return fail(ctx, OCTPT_ERR_INVALID_ARG, "d_accum NULL");
    try {
        join_inflight(ctx);
        DevRender R{};
        octpt_status st = make_render(ctx, p, R);
        if (st != OCTPT_OK) return st;
        if (is_multi(ctx))
            return multi_render(ctx, *p, R, reinterpret_cast<float4 *>(d_accum), d_seg, static_cast<hipStream_t>(stream),
                                nullptr);
        return enqueue_render(ctx, R, reinterpret_cast<float4 *>(d_accum), d_seg, static_cast<hipStream_t>(stream),
                              (p->flags & OCTPT_RENDER_MEGAKERNEL) != 0);
    } catch (...) {
        return fail(ctx, OCTPT_ERR_INTERNAL, "unexpected exception in render");
    }
}

namespace {
// FrameInFlight worker: H2D, render, tone map, D2H on the context stream
void frame_worker(octpt_frame *f, DevRender R, bool megakernel) {
    octpt_ctx *ctx = f->ctx;
    octpt_status st = OCTPT_OK;
    auto run = [&]() -> octpt_status {
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        HIP_TRY(ctx, hipMemcpyAsync(f->d_accum, f->h_accum, f->n_pixels * 16, hipMemcpyHostToDevice, ctx->stream));
        octpt_status r = is_multi(ctx) ? multi_render(ctx, f->params, R, f->d_accum, nullptr, ctx->stream, &f->cancel_requested)
                                       : enqueue_render(ctx, R, f->d_accum, nullptr, ctx->stream, megakernel, &f->cancel_requested);
        if (r != OCTPT_OK) return r;
        if (f->d_rgba) {
            HIP_TRY(ctx, launch_tonemap(f->d_accum, f->d_rgba, (uint32_t)f->n_pixels, ctx->d_lut_byte, ctx->stream));
            HIP_TRY(ctx, hipMemcpyAsync(f->h_rgba, f->d_rgba, f->n_pixels * 4, hipMemcpyDeviceToHost, ctx->stream));
        }
        HIP_TRY(ctx, hipMemcpyAsync(f->h_accum, f->d_accum, f->n_pixels * 16, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        return OCTPT_OK;
    };
    try {
        st = run();
    } catch (...) {
        st = fail(ctx, OCTPT_ERR_INTERNAL, "unexpected exception in frame worker");
    }
    if (st != OCTPT_OK) (void)hipStreamSynchronize(ctx->stream);
    f->status = st;
    f->finished.store(true);
}

octpt_status frame_result(octpt_frame *f) {
    if (f->worker.joinable()) f->worker.join();
    if (f->ctx && f->ctx->inflight == f) f->ctx->inflight = nullptr;
    if (f->cancel_requested.load()) return OCTPT_CANCELLED;
    if (f->status != OCTPT_OK) return f->status;
    deliver(f);
    return OCTPT_OK;
}
}  // namespace

octpt_status octpt_render_async(octpt_ctx *ctx, const octpt_render_params *p, float *accum, uint8_t *rgba,
                                octpt_frame **out) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    if (!out || !accum) return fail(ctx, OCTPT_ERR_INVALID_ARG, "NULL output");
    *out = nullptr;
    octpt_frame *f = nullptr;
    try {
        join_inflight(ctx);
        DevRender R{};
        octpt_status st = make_render(ctx, p, R);
        if (st != OCTPT_OK) return st;
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        f = new octpt_frame();
        f->ctx = ctx;
        f->params = *p;
        f->user_accum = accum;
        f->user_rgba = rgba;
        f->n_pixels = accum_pixels(R);
        auto fail_frame = [&](hipError_t e, const char *what) {
            free_frame_buffers(f);
            delete f;
            return hip_fail(ctx, e, what);
        };
        hipError_t e;
        if ((e = hipMalloc(&f->d_accum, f->n_pixels * 16)) != hipSuccess) return fail_frame(e, "hipMalloc accum");
        if ((e = hipHostMalloc(&f->h_accum, f->n_pixels * 16, hipHostMallocDefault)) != hipSuccess)
            return fail_frame(e, "hipHostMalloc accum");
        if (rgba) {
            if ((e = hipMalloc(&f->d_rgba, f->n_pixels * 4)) != hipSuccess) return fail_frame(e, "hipMalloc rgba");
            if ((e = hipHostMalloc(&f->h_rgba, f->n_pixels * 4, hipHostMallocDefault)) != hipSuccess)
                return fail_frame(e, "hipHostMalloc rgba");
        }
        std::memcpy(f->h_accum, accum, f->n_pixels * 16);
        f->worker = std::thread(frame_worker, f, R, (p->flags & OCTPT_RENDER_MEGAKERNEL) != 0);
        ctx->inflight = f;
        *out = f;
        return OCTPT_OK;
    } catch (...) {
        if (f) {
            if (f->worker.joinable()) f->worker.join();
            free_frame_buffers(f);
            delete f;
        }
        return fail(ctx, OCTPT_ERR_INTERNAL, "unexpected exception in render_async");
    }
}

octpt_status octpt_frame_poll(octpt_frame *f) {
    if (!f) return OCTPT_ERR_INVALID_ARG;
    if (!f->finished.load()) return OCTPT_NOT_READY;
    return frame_result(f);
}

octpt_status octpt_frame_wait(octpt_frame *f) {
    if (!f) return OCTPT_ERR_INVALID_ARG;
    return frame_result(f);
}

octpt_status octpt_frame_cancel(octpt_frame *f) {
    if (!f) return OCTPT_ERR_INVALID_ARG;
    if (!f->delivered) f->cancel_requested.store(true);
    return OCTPT_OK;
}

void octpt_frame_release(octpt_frame *f) {
    if (!f) return;
    if (f->worker.joinable()) f->worker.join();
    if (f->ctx && f->ctx->inflight == f) f->ctx->inflight = nullptr;
    free_frame_buffers(f);
    delete f;
}

octpt_status octpt_render(octpt_ctx *ctx, const octpt_render_params *p, float *accum, uint8_t *rgba) {
    octpt_frame *f = nullptr;
    octpt_status st = octpt_render_async(ctx, p, accum, rgba, &f);
    if (st != OCTPT_OK) return st;
    st = octpt_frame_wait(f);
    octpt_frame_release(f);
    return st;
}

octpt_status octpt_tonemap_device(octpt_ctx *ctx, const float *d_accum, uint8_t *d_rgba, uint32_t n, void *stream) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    if (!d_accum || !d_rgba) return fail(ctx, OCTPT_ERR_INVALID_ARG, "NULL buffer");
    if (n == 0) return OCTPT_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, launch_tonemap(reinterpret_cast<const float4 *>(d_accum), reinterpret_cast<uchar4 *>(d_rgba), n,
                                ctx->d_lut_byte, static_cast<hipStream_t>(stream)));
    return OCTPT_OK;
}

uint32_t octpt_shard_pixels(uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count) {
    if (shard_count == 0 || shard_index >= shard_count) return 0;
    const uint32_t tiles = ((width + kTile - 1) / kTile) * ((height + kTile - 1) / kTile);
    return tiles_of_shard(tiles, shard_index, shard_count) * 64u;
}

octpt_status octpt_unshard_device(octpt_ctx *ctx, uint32_t W, uint32_t H, uint32_t N, const float *d_shards,
                                  uint32_t stride, float *d_frame, void *stream) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    if (!d_shards || !d_frame || N == 0 || W == 0 || H == 0) return fail(ctx, OCTPT_ERR_INVALID_ARG, "bad unshard args");
    if (stride < octpt_shard_pixels(W, H, 0, N)) return fail(ctx, OCTPT_ERR_INVALID_ARG, "shard stride too small");
    if (!ctx->h_order.empty() && (W != ctx->order_w || H != ctx->order_h))
        return fail(ctx, OCTPT_ERR_INVALID_ARG, "frame size differs from the tile order's (octpt_set_tile_order)");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, launch_unshard(W, H, N, ctx->h_order.empty() ? nullptr : ctx->d_order_pos,
                                reinterpret_cast<const float4 *>(d_shards), stride, reinterpret_cast<float4 *>(d_frame),
                                static_cast<hipStream_t>(stream)));
    return OCTPT_OK;
}

octpt_status octpt_set_tile_order(octpt_ctx *ctx, uint32_t width, uint32_t height, const uint32_t *order) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    join_inflight(ctx);
    try {
        // validated once, before any entry changes (a failure part-way through a multi-device
        // context's entries must not leave them dealing differently)
        uint32_t T = 0;
        std::vector<uint32_t> pos;
        if (order) {
            if (width == 0 || height == 0 || (uint64_t)width * height >= (1ull << 31))
                return fail(ctx, OCTPT_ERR_INVALID_ARG, "bad resolution");
            T = ((width + kTile - 1) / kTile) * ((height + kTile - 1) / kTile);
            pos.assign(T, 0xFFFFFFFFu);
            for (uint32_t s = 0; s < T; ++s) {
                if (order[s] >= T || pos[order[s]] != 0xFFFFFFFFu)
                    return fail(ctx, OCTPT_ERR_INVALID_ARG, "tile order is not a permutation of the frame's tiles");
                pos[order[s]] = s;
            }
        }
        for (size_t i = 0; i < ctx->sub.size(); ++i) {  // every device entry deals the same way (its sub-shards nest in it)
            const octpt_status st = octpt_set_tile_order(ctx->sub[i], width, height, order);
            if (st != OCTPT_OK) {
                // an entry failed (out of memory): every entry and the parent go back to round robin, so that the
                // parent's staging and the entries' item mappings agree
                const std::string why = ctx->sub[i]->err;
                for (octpt_ctx *c : ctx->sub) (void)octpt_set_tile_order(c, width, height, nullptr);
                ++ctx->order_gen;
                ctx->h_order.clear();
                ctx->order_w = ctx->order_h = 0;
                return fail(ctx, st, why + " (every entry reset to the round-robin deal)");
            }
        }
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        ++ctx->order_gen;
        if (!order) {
            ctx->h_order.clear();
            ctx->order_w = ctx->order_h = 0;
            return OCTPT_OK;
        }
        // the tables are overwritten in place: a render issued on any stream (render_device / unshard_device take
        // the caller's) may still read them, so the whole device drains first
        HIP_TRY(ctx, hipDeviceSynchronize());
        if (ctx->h_order.size() != T) {
            if (ctx->d_order) (void)hipFree(ctx->d_order);
            if (ctx->d_order_pos) (void)hipFree(ctx->d_order_pos);
            ctx->d_order = ctx->d_order_pos = nullptr;
            ctx->h_order.clear();
            HIP_TRY(ctx, hipMalloc(&ctx->d_order, (size_t)T * 4));
            HIP_TRY(ctx, hipMalloc(&ctx->d_order_pos, (size_t)T * 4));
        }
        HIP_TRY(ctx, hipMemcpy(ctx->d_order, order, (size_t)T * 4, hipMemcpyHostToDevice));
        HIP_TRY(ctx, hipMemcpy(ctx->d_order_pos, pos.data(), (size_t)T * 4, hipMemcpyHostToDevice));
        ctx->h_order.assign(order, order + T);
        ctx->order_w = width;
        ctx->order_h = height;
        return OCTPT_OK;
    } catch (const std::bad_alloc &) {
        return fail(ctx, OCTPT_ERR_OOM, "host allocation");
    } catch (...) {
        return fail(ctx, OCTPT_ERR_INTERNAL, "unexpected exception");
    }
}

octpt_status octpt_balance_tiles(uint32_t width, uint32_t height, uint32_t shard_count, const uint32_t *seg_count,
                                 uint32_t *order) {
    if (!seg_count || !order || shard_count == 0 || width == 0 || height == 0 ||
        (uint64_t)width * height >= (1ull << 31))
        return OCTPT_ERR_INVALID_ARG;
    try {
        const uint32_t tx = (width + kTile - 1) / kTile, T = tx * ((height + kTile - 1) / kTile);
        std::vector<uint64_t> cost(T, 0);
        for (uint32_t y = 0; y < height; ++y)
            for (uint32_t x = 0; x < width; ++x) cost[(y / kTile) * tx + x / kTile] += seg_count[(size_t)y * width + x];
        // longest processing time first: tiles by cost (ties by index), each to the shard with the least work
        // so far among those with positions left -- shard k keeps exactly its round-robin count of positions
        std::vector<uint32_t> by(T);
        for (uint32_t t = 0; t < T; ++t) by[t] = t;
        std::stable_sort(by.begin(), by.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
        const uint32_t N = shard_count;
        std::vector<uint64_t> load(N, 0);
        std::vector<std::vector<uint32_t>> mine(N);
        for (uint32_t k = 0; k < N; ++k) mine[k].reserve(tiles_of_shard(T, k, N));
        for (uint32_t t : by) {
            uint32_t best = N;
            for (uint32_t k = 0; k < N; ++k)
                if (mine[k].size() < tiles_of_shard(T, k, N) && (best == N || load[k] < load[best])) best = k;
            mine[best].push_back(t);
            load[best] += cost[t];
        }
        // each shard's tiles in image order (the seed's coherence: neighbouring tiles trace side by side)
        for (uint32_t k = 0; k < N; ++k) {
            std::sort(mine[k].begin(), mine[k].end());
            for (uint32_t u = 0; u < mine[k].size(); ++u) order[k + (size_t)u * N] = mine[k][u];
        }
        return OCTPT_OK;
    } catch (...) {
        return OCTPT_ERR_OOM;
    }
}

octpt_status octpt_intersect(octpt_ctx *ctx, const float *rays, const uint32_t *last_prim, const float *last_normal,
                             uint32_t n, float *t, uint32_t *prim, float *normal, uint32_t *steps) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    join_inflight(ctx);
    if (!ctx->has_scene) return fail(ctx, OCTPT_ERR_INVALID_ARG, "no scene uploaded");
    if (n == 0) return OCTPT_OK;
    if (!rays || !t || !prim) return fail(ctx, OCTPT_ERR_INVALID_ARG, "NULL buffer");
    if (is_multi(ctx)) {  // one batch on the first entry's replica
        const octpt_status st = octpt_intersect(ctx->sub[0], rays, last_prim, last_normal, n, t, prim, normal, steps);
        return st == OCTPT_OK ? st : fail(ctx, st, ctx->sub[0]->err);
    }
    // esvo_begin's t_coef = 1 / -|d| comes from rcp_rn, exact for |d| in [2^-23, 2^126] (smaller
    // components are clamped to 2^-23 first, octree_traversal.rs:86-93): a ray with a non-finite
    // component or a direction component |d| > 2^126 is outside that range.  Such a ray is reported as a
    // miss -- t = +inf, prim = none, normal 0, 0 steps -- and the rest of the batch is traced as usual (the
    // kernel sees a placeholder ray in its place).  For a non-finite ray this is what the reference's
    // comparisons with NaN t-values give.  For a finite direction above 2^126 it is a DELIBERATE DEVIATION:
    // the reference does not normalise directions (Ray::new, ray/mod.rs:32), its t_coef would be subnormal
    // (octree_traversal.rs:95) and its walk could still hit something; no reference fixture covers that
    // case (parity unpinned), and the render kernels never produce such a direction.
    std::vector<uint32_t> unsupported;
    std::vector<float> clean;
    for (size_t i = 0; i < (size_t)n * 6; ++i) {
        const float v = rays[i];
        if (!std::isfinite(v) || (i % 6 >= 3 && std::fabs(v) > 0x1p126f)) {
            if (clean.empty()) clean.assign(rays, rays + (size_t)n * 6);
            const size_t r = i / 6;
            if (unsupported.empty() || unsupported.back() != r) unsupported.push_back((uint32_t)r);
            for (int k = 0; k < 6; ++k) clean[r * 6 + k] = k == 3 ? 1.0f : 0.0f;
        }
    }
    if (!clean.empty()) rays = clean.data();
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    float *d_rays = nullptr, *d_ln = nullptr, *d_t = nullptr, *d_n = nullptr;
    uint32_t *d_lp = nullptr, *d_p = nullptr, *d_s = nullptr;
    auto cleanup = [&]() {
        for (void *q : {(void *)d_rays, (void *)d_ln, (void *)d_t, (void *)d_n, (void *)d_lp, (void *)d_p, (void *)d_s})
            if (q) (void)hipFree(q);
    };
    hipError_t e = hipSuccess;
    do {
        if ((e = hipMalloc(&d_rays, (size_t)n * 24)) != hipSuccess) break;
        if ((e = hipMemcpy(d_rays, rays, (size_t)n * 24, hipMemcpyHostToDevice)) != hipSuccess) break;
        if (last_prim) {
            if ((e = hipMalloc(&d_lp, (size_t)n * 4)) != hipSuccess) break;
            if ((e = hipMemcpy(d_lp, last_prim, (size_t)n * 4, hipMemcpyHostToDevice)) != hipSuccess) break;
        }
        if (last_normal) {
            if ((e = hipMalloc(&d_ln, (size_t)n * 12)) != hipSuccess) break;
            if ((e = hipMemcpy(d_ln, last_normal, (size_t)n * 12, hipMemcpyHostToDevice)) != hipSuccess) break;
        }
        if ((e = hipMalloc(&d_t, (size_t)n * 4)) != hipSuccess) break;
        if ((e = hipMalloc(&d_p, (size_t)n * 4)) != hipSuccess) break;
        if (normal && (e = hipMalloc(&d_n, (size_t)n * 12)) != hipSuccess) break;
        if (steps && (e = hipMalloc(&d_s, (size_t)n * 4)) != hipSuccess) break;
        if ((e = launch_intersect(ctx->S, d_rays, d_lp, d_ln, n, d_t, d_p, d_n, d_s, ctx->stream)) != hipSuccess) break;
        if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) break;
        if ((e = hipMemcpy(t, d_t, (size_t)n * 4, hipMemcpyDeviceToHost)) != hipSuccess) break;
        if ((e = hipMemcpy(prim, d_p, (size_t)n * 4, hipMemcpyDeviceToHost)) != hipSuccess) break;
        if (normal && (e = hipMemcpy(normal, d_n, (size_t)n * 12, hipMemcpyDeviceToHost)) != hipSuccess) break;
        if (steps && (e = hipMemcpy(steps, d_s, (size_t)n * 4, hipMemcpyDeviceToHost)) != hipSuccess) break;
    } while (0);
    cleanup();
    if (e != hipSuccess) return hip_fail(ctx, e, "intersect");
    for (uint32_t r : unsupported) {
        t[r] = INFINITY;
        prim[r] = 0xFFFFFFFFu;
        if (normal) normal[3 * (size_t)r] = normal[3 * (size_t)r + 1] = normal[3 * (size_t)r + 2] = 0.0f;
        if (steps) steps[r] = 0u;
    }
    return OCTPT_OK;
}

octpt_status octpt_get_stats(const octpt_ctx *cctx, octpt_stats *out) {
    if (!cctx || !out) return OCTPT_ERR_INVALID_ARG;
    octpt_ctx *ctx = const_cast<octpt_ctx *>(cctx);
    join_inflight(ctx);
    if (is_multi(ctx)) {  // the entries' counters summed; kernel_ms = the render calls' wall time
        octpt_stats tot{};
        for (octpt_ctx *c : ctx->sub) {
            octpt_stats cs{};
            const octpt_status st = octpt_get_stats(c, &cs);
            if (st != OCTPT_OK) return fail(ctx, st, c->err);
            tot.paths += cs.paths;
            tot.segments += cs.segments;
            tot.esvo_steps += cs.esvo_steps;
            tot.sphere_tests += cs.sphere_tests;
            tot.cuboid_tests += cs.cuboid_tests;
            tot.shade_events += cs.shade_events;
            tot.texel_reads += cs.texel_reads;
            tot.extend_launches += cs.extend_launches;
            tot.shade_launches += cs.shade_launches;
            tot.extend_ms += cs.extend_ms;
            tot.shade_ms += cs.shade_ms;
            tot.build_ms = std::max(tot.build_ms, cs.build_ms);
            tot.block_tests += cs.block_tests;
            tot.issued_bytes += cs.issued_bytes;
            for (int k = 0; k < OCTPT_STAT_COUNT; ++k) tot.drain[k] += cs.drain[k];
            tot.pool_slots = std::max(tot.pool_slots, cs.pool_slots);
            tot.chunk_items = std::max(tot.chunk_items, cs.chunk_items);
            tot.wave_allocs += cs.wave_allocs;
            tot.beam_restarts += cs.beam_restarts;
            tot.hit_check_failures += cs.hit_check_failures;
        }
        tot.build_ms = std::max(tot.build_ms, (double)ctx->build_ms);  // the builder runs on the first device
        tot.launches = ctx->launches;
        tot.kernel_ms = ctx->kernel_ms;
        *out = tot;
        return OCTPT_OK;
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (auto &e : ctx->pending) {
        HIP_TRY(ctx, hipEventSynchronize(e.stop));
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, e.start, e.stop));
        ctx->kernel_ms += ms;
        (void)hipEventDestroy(e.start);
        (void)hipEventDestroy(e.stop);
    }
    ctx->pending.clear();
    for (auto &ke : ctx->kpending) {
        HIP_TRY(ctx, hipEventSynchronize(ke.second.stop));
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ke.second.start, ke.second.stop));
        ctx->kern_ms[ke.first] += ms;
        ctx->kern_n[ke.first]++;
        ctx->ev_pool.push_back(ke.second);
    }
    ctx->kpending.clear();
    std::vector<unsigned long long> rows(kStatWords);
    HIP_TRY(ctx, hipMemcpy(rows.data(), ctx->d_stats, kStatWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // rows [0, kSegs): every kernel but the drain; [kStatDrainRow, +kSegs): the drain (octpt_stats::drain)
    unsigned long long v[kStatCount] = {0}, dr[kStatCount] = {0};
    for (uint32_t r = 0; r < kSegs; ++r)
        for (uint32_t i = 0; i < kStatCount; ++i) {
            v[i] += rows[r * kStatRow + i];
            dr[i] += rows[(kStatDrainRow + r) * kStatRow + i];
        }
    for (uint32_t i = 0; i < kStatCount; ++i) {
        out->drain[i] = dr[i];
        v[i] += dr[i];
    }
    if (std::getenv("OCTPT_PROFILE_LANES")) {  // diagnostic builds (-DOCTPT_PROFILE_LANES) fill words 12..24
        static const char *names[13] = {"iters", "active", "leaf_it", "leaf_ln", "pop_it", "pop_ln", "push_it",
                                        "desc_ln", "exact", "fold_it", "fold_ln", "dfold_it", "dfold_ln"};
        std::fprintf(stderr, "octpt lanes:");
        for (uint32_t i = 0; i < 13; ++i) {
            unsigned long long x = 0;
            for (uint32_t r = 0; r < kSegs; ++r) x += rows[r * kStatRow + 12 + i];
            std::fprintf(stderr, " %s=%llu", names[i], x);
        }
        std::fprintf(stderr, "\n");
    }
    // beam-started rays traced again from the cube entry: extend's retraced ones took a
    // second queue position, which its segment count includes; the drain's restart in place does not
    unsigned long long redo_main = 0, redo_drain = 0;
    for (uint32_t r = 0; r < kSegs; ++r) {
        redo_main += rows[r * kStatRow + kStatBeamRestartWord];
        redo_drain += rows[(kStatDrainRow + r) * kStatRow + kStatBeamRestartWord];
    }
    out->paths = v[kStatPaths];
    out->segments = v[kStatSegments] - redo_main;
    out->esvo_steps = v[kStatSteps];
    out->sphere_tests = v[kStatSphereTests];
    out->cuboid_tests = v[kStatCuboidTests];
    out->shade_events = v[kStatShade];
    out->texel_reads = v[kStatTexels];
    out->block_tests = v[kStatBlockTests];
    out->issued_bytes = v[kStatIssued];
    out->beam_restarts = redo_main + redo_drain;
    out->hit_check_failures = 0;
    for (uint32_t r = 0; r < 2u * kSegs; ++r) out->hit_check_failures += rows[r * kStatRow + kStatHitCheckWord];
    out->pool_slots = ctx->pool;
    out->chunk_items = ctx->color_cap;
    out->wave_allocs = ctx->wave_allocs_n;
    out->launches = ctx->launches;
    out->kernel_ms = ctx->kernel_ms;
    out->extend_launches = ctx->kern_n[0];
    out->shade_launches = ctx->kern_n[1];
    out->extend_ms = ctx->kern_ms[0];
    out->shade_ms = ctx->kern_ms[1];
    out->build_ms = ctx->build_ms;
    return OCTPT_OK;
}

octpt_status octpt_reset_stats(octpt_ctx *ctx) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    join_inflight(ctx);
    if (is_multi(ctx)) {
        for (octpt_ctx *c : ctx->sub) {
            const octpt_status st = octpt_reset_stats(c);
            if (st != OCTPT_OK) return fail(ctx, st, c->err);
        }
        ctx->kernel_ms = 0.0;
        ctx->launches = 0;
        return OCTPT_OK;
    }
    octpt_stats tmp;
    octpt_status st = octpt_get_stats(ctx, &tmp);  // drains pending events
    if (st != OCTPT_OK) return st;
    HIP_TRY(ctx, hipMemset(ctx->d_stats, 0, kStatWords * sizeof(unsigned long long)));
    ctx->kernel_ms = 0.0;
    ctx->launches = 0;
    ctx->kern_ms[0] = ctx->kern_ms[1] = 0.0;
    ctx->kern_n[0] = ctx->kern_n[1] = 0;
    return OCTPT_OK;
}

octpt_status octpt_build_octree_device(octpt_ctx *ctx, const octpt_sphere *spheres, uint32_t ns,
                                       const octpt_cuboid *cuboids, uint32_t nc, uint32_t depth, octpt_octree **out) {
    return octpt_build_octree_device_ex(ctx, spheres, ns, cuboids, nc, depth, 0u, out);
}

octpt_status octpt_build_octree_device_ex(octpt_ctx *ctx, const octpt_sphere *spheres, uint32_t ns,
                                          const octpt_cuboid *cuboids, uint32_t nc, uint32_t depth, uint32_t flags,
                                          octpt_octree **out) {
    if (!ctx) return OCTPT_ERR_INVALID_ARG;
    if (!out) return fail(ctx, OCTPT_ERR_INVALID_ARG, "out NULL");
    if (flags & ~OCTPT_BUILD_COMPACT) return fail(ctx, OCTPT_ERR_INVALID_ARG, "unknown build flags");
    *out = nullptr;
    if (depth < 1 || depth > kMaxDepth) return fail(ctx, OCTPT_ERR_INVALID_ARG, "depth must be in [1, 21]");
    if ((ns && !spheres) || (nc && !cuboids)) return fail(ctx, OCTPT_ERR_INVALID_ARG, "NULL primitive array");
    try {
        join_inflight(ctx);
        if (pair_bound(spheres, ns, cuboids, nc, depth) > kMaxBuildPairs)
            return fail(ctx, OCTPT_ERR_OOM, "more than 2^31 (cell, primitive) pairs");
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        octpt_octree *t = new octpt_octree();
        bool too_many = false;
        float ms = 0.0f;
        const hipError_t e = build_octree_gpu(ctx->stream, ctx->build_scratch, spheres, ns, cuboids, nc, depth,
                                              (flags & OCTPT_BUILD_COMPACT) != 0, kMaxBuildPairs, *t, too_many, &ms);
        if (e != hipSuccess || too_many) {
            delete t;
            if (e == hipErrorOutOfMemory || too_many) return fail(ctx, OCTPT_ERR_OOM, "octree build: out of memory");
            return hip_fail(ctx, e, "octree build");
        }
        ctx->build_ms = ms;
        *out = t;
        return OCTPT_OK;
    } catch (const std::bad_alloc &) {
        return fail(ctx, OCTPT_ERR_OOM, "octree build: host out of memory");
    } catch (...) {
        return fail(ctx, OCTPT_ERR_INTERNAL, "unexpected exception in octree build");
    }
}

octpt_status octpt_build_octree(const octpt_sphere *spheres, uint32_t ns, const octpt_cuboid *cuboids, uint32_t nc,
                                uint32_t depth, octpt_octree **out) {
    return octpt_build_octree_ex(spheres, ns, cuboids, nc, depth, 0u, out);
}

octpt_status octpt_build_octree_ex(const octpt_sphere *spheres, uint32_t ns, const octpt_cuboid *cuboids, uint32_t nc,
                                   uint32_t depth, uint32_t flags, octpt_octree **out) {
    if (!out) return OCTPT_ERR_INVALID_ARG;
    if (flags & ~OCTPT_BUILD_COMPACT) return OCTPT_ERR_INVALID_ARG;
    *out = nullptr;
    if (depth < 1 || depth > kMaxDepth) return OCTPT_ERR_INVALID_ARG;
    if ((ns && !spheres) || (nc && !cuboids)) return OCTPT_ERR_INVALID_ARG;
    try {
        const int32_t N = 1 << depth;
        const uint64_t bound = pair_bound(spheres, ns, cuboids, nc, depth);
        if (bound > kMaxBuildPairs) return OCTPT_ERR_OOM;
        // cuboid cells are half-open at the top (pair_bound)
        auto cub_hi = [](float lo, float hi) { return std::max(floorf(lo), ceilf(hi) - 1.0f); };
        std::vector<CellPrim> cells;
        cells.reserve((size_t)std::min<uint64_t>(bound, 1ull << 24));
        for (uint32_t i = 0; i < ns; ++i) {
            const float *c = spheres[i].center;
            const float r = spheres[i].radius;
            if (!(r > 0.0f)) continue;
            int32_t lo[3], hi[3];
            bool empty = false;
            for (int a = 0; a < 3; ++a) {
                const float fl = floorf(c[a] - r), fh = floorf(c[a] + r);
                if (fh < 0.0f || fl > (float)(N - 1)) empty = true;
                lo[a] = clamp_cell(fl, N - 1);
                hi[a] = clamp_cell(fh, N - 1);
            }
            if (empty) continue;
            const float r2 = r * r;
            for (int32_t z = lo[2]; z <= hi[2]; ++z)
                for (int32_t y = lo[1]; y <= hi[1]; ++y)
                    for (int32_t x = lo[0]; x <= hi[0]; ++x) {
                        const float bl[3] = {(float)x, (float)y, (float)z};
                        float dd[3];
                        for (int a = 0; a < 3; ++a) {
                            const float l = bl[a], h = bl[a] + 1.0f;
                            dd[a] = c[a] < l ? l - c[a] : (c[a] > h ? c[a] - h : 0.0f);
                        }
                        if ((dd[0] * dd[0] + dd[1] * dd[1]) + dd[2] * dd[2] <= r2)
                            cells.push_back(CellPrim{morton((uint64_t)x, (uint64_t)y, (uint64_t)z), i});
                    }
        }
        for (uint32_t i = 0; i < nc; ++i) {
            const octpt_cuboid &b = cuboids[i];
            int32_t lo[3], hi[3];
            bool empty = false;
            for (int a = 0; a < 3; ++a) {
                const float fl = floorf(b.min[a]), fh = cub_hi(b.min[a], b.max[a]);
                if (fh < 0.0f || fl > (float)(N - 1) || b.max[a] < b.min[a]) empty = true;
                lo[a] = clamp_cell(fl, N - 1);
                hi[a] = clamp_cell(fh, N - 1);
            }
            if (empty) continue;
            for (int32_t z = lo[2]; z <= hi[2]; ++z)
                for (int32_t y = lo[1]; y <= hi[1]; ++y)
                    for (int32_t x = lo[0]; x <= hi[0]; ++x)
                        cells.push_back(CellPrim{morton((uint64_t)x, (uint64_t)y, (uint64_t)z), i | kPrimCuboidBit});
        }
        std::sort(cells.begin(), cells.end());
        octpt_octree *t = new octpt_octree();
        t->depth = depth;
        std::vector<uint64_t> codes;
        t->leaf_prims.resize(cells.size());
        for (size_t k = 0; k < cells.size(); ++k) {
            if (k == 0 || cells[k].code != cells[k - 1].code) {
                t->leaf_first.push_back((uint32_t)k);
                t->leaf_count.push_back(0);
                codes.push_back(cells[k].code);
            }
            t->leaf_count.back()++;
            t->leaf_prims[k] = cells[k].prim;
        }
        Builder b{t, std::move(codes), depth, (flags & OCTPT_BUILD_COMPACT) != 0};
        t->root = b.node(0, 0, (uint32_t)b.leaf_code.size()).v;
        *out = t;
        return OCTPT_OK;
    } catch (const std::bad_alloc &) {
        return OCTPT_ERR_OOM;
    } catch (...) {
        return OCTPT_ERR_INTERNAL;
    }
}

octpt_status octpt_build_block_octree(const uint32_t *cells, uint32_t n, uint32_t depth, uint32_t flags,
                                      octpt_octree **out) {
    if (!out) return OCTPT_ERR_INVALID_ARG;
    *out = nullptr;
    if (flags & ~OCTPT_BUILD_COMPACT) return OCTPT_ERR_INVALID_ARG;
    if (depth < 1 || depth > kMaxDepth || (n && !cells)) return OCTPT_ERR_INVALID_ARG;
    try {
        const uint32_t N = 1u << depth;
        std::vector<std::pair<uint64_t, uint32_t>> sorted(n);
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t *c = cells + 4 * (size_t)k;
            if (c[0] >= N || c[1] >= N || c[2] >= N || c[3] > kPrimIndexMask) return OCTPT_ERR_INVALID_ARG;
            sorted[k] = {morton(c[0], c[1], c[2]), c[3]};
        }
        std::sort(sorted.begin(), sorted.end());
        for (size_t k = 1; k < sorted.size(); ++k)
            if (sorted[k].first == sorted[k - 1].first) return OCTPT_ERR_INVALID_ARG;  // two blocks in one cell
        std::unique_ptr<octpt_octree> t(new octpt_octree());
        t->depth = depth;
        BlockBuilder b{t.get(), sorted, depth, (flags & OCTPT_BUILD_COMPACT) != 0};
        t->root = b.node(0, 0, sorted.size()).v;
        *out = t.release();
        return OCTPT_OK;
    } catch (const std::bad_alloc &) {
        return OCTPT_ERR_OOM;
    } catch (...) {
        return OCTPT_ERR_INTERNAL;
    }
}

octpt_status octpt_octree_get_view(const octpt_octree *t, octpt_octree_view *v) {
    if (!t || !v) return OCTPT_ERR_INVALID_ARG;
    v->octants = t->octants.data();
    v->octant_count = (uint32_t)t->octants.size();
    v->root = t->root;
    v->depth = t->depth;
    v->leaf_first = t->leaf_first.data();
    v->leaf_count = t->leaf_count.data();
    v->leaf_table_size = (uint32_t)t->leaf_first.size();
    v->leaf_prims = t->leaf_prims.data();
    v->leaf_prim_count = (uint32_t)t->leaf_prims.size();
    return OCTPT_OK;
}

void octpt_octree_free(octpt_octree *t) { delete t; }

}  // extern "C"
