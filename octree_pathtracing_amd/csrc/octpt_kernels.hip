// octpt_kernels.hip -- gfx950 (CDNA4) kernels of the octree path-tracing hot path.
//
// render_kernel is a persistent wavefront megakernel.  Every lane owns one pixel at a
// time and runs that pixel's progressive passes (TileRenderer::render_tile_average,
// reference src/renderer/tile_renderer.rs:684-734) back to back; a lane is in one of a
// few states (new path / segment setup / ESVO traversal / shading / refill) and the wave
// keeps traversing while at least half of its live lanes are traversing, then shades the
// lanes that finished their segment (wave-level ballot compaction).  Lanes
// that finish a pixel pull the next work item from a device atomic counter (64 work items
// = one 8x8 screen tile per wave).  The ESVO stack lives in LDS (one 8-byte slot per
// octree level per lane, [slot][lane] so a wave's access is one conflict-free row).
//
// Float semantics follow the oracle (oracle/cpu_ref.c) bit for bit: -ffp-contract=off,
// correctly rounded div/sqrt, the portable f32 math below, and the
// reference's operation order.  The only difference is the radiance accumulation order
// (forward throughput instead of the reference's recursion), which the oracle also
// implements as `forward_accumulation`.
#include "octpt_internal.h"
#include "octpt_rcp.h"

#ifndef OCTPT_RCP_FAST
#define OCTPT_RCP_FAST 1  // esvo_begin's t_coef by rcp_rn (A/B: -DOCTPT_RCP_FAST=0, the division: extend +0.2..0.6 %)
#endif

namespace octpt {
namespace {

#define RAY_EPSILON 0.00000005f
#define RAY_OFFSET 0.000001f
#define OCTREE_MAX_STEPS 1000u
#define OCTREE_MAX_SCALE 23u
#define OCTREE_EPSILON 1.1920929e-7f
#define MAX_DST_WORLD 1024.0f
#define PI_F 3.14159265358979323846f
#define CELL_TOL 0.001f
#define SUN_MAX_CHANCE 0.9f
#define MAT_FLAG_REFRACTIVE 0x4u
#define MAT_FLAG_SUBSURFACE 0x2u  // MaterialFlags::SUBSURFACE_SCATTER (material.rs:9)
#define MAX_PATH_SEGMENTS 64u  // [C15] next_intersection calls per path (grazing self-hit loops)
// a beam start carries, in its low mantissa bits, a bound of the reference iterations it skips (beam_kernel)
constexpr uint32_t kBeamIterBits = 10u;
constexpr uint32_t kBeamIterMask = (1u << kBeamIterBits) - 1u;
static_assert(OCTREE_MAX_STEPS <= kBeamIterMask + 1u, "the skipped-iteration bound fits its bits");

// ---------------------------------------------------------------------------
// f32 vector helpers (glam Vec3A operation order, see oracle/cpu_ref.c)
// ---------------------------------------------------------------------------
struct v3 {
    float x, y, z;
};
__device__ __forceinline__ v3 V(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 vscale(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float vdot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ v3 vcross(v3 a, v3 b) {
    return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
__device__ __forceinline__ v3 vnorm(v3 a) {
    float r = 1.0f / sqrtf(vdot(a, a));
    return vscale(a, r);
}
__device__ __forceinline__ float fmn(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float fmx(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float vmin3(v3 a) { return fmn(fmn(a.x, a.y), a.z); }
__device__ __forceinline__ float vmax3(v3 a) { return fmx(fmx(a.x, a.y), a.z); }
// ESVO t-values: t_coef is finite and non-zero, pos in [1, 2), so every t is finite and an exact
// zero difference rounds to +0 -- no NaN and no -0 reach these, and IEEE minNum/maxNum (one
// v_min3/v_max3) agree bit-for-bit with the a < b ? a : b form the oracle uses.
__device__ __forceinline__ float tmn(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float tmx(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ float tmin3(v3 a) { return tmn(tmn(a.x, a.y), a.z); }
// min of two NaN-free t-values one of which the compiler cannot prove canonical (a loop-carried or
// LDS-loaded t_max): one v_min_f32, where the minNum lowering puts a v_max canonicalisation of that
// operand first (the same instruction, so the same bits, for NaN-free operands)
__device__ __forceinline__ float tmn_nc(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float tmax3(v3 a) { return tmx(tmx(a.x, a.y), a.z); }
__device__ __forceinline__ float signum_(float f) { return (__float_as_uint(f) >> 31) ? -1.0f : 1.0f; }

// ---------------------------------------------------------------------------
// portable f32 math -- identical constants and order to the oracle
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dm_sincos(float x, float &s, float &c) {
    const float kf = floorf(x * 0.636619772367581343f + 0.5f);
    const int k = (int)kf;
    const float r = ((x - kf * 1.5703125f) - kf * 4.837512969970703125e-4f) - kf * 7.54978995489188216e-8f;
    const float z = r * r;
    const float sp = r + r * z * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
    const float cp = (1.0f - 0.5f * z) +
                     z * z * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
    switch (k & 3) {
    case 0: s = sp; c = cp; break;
    case 1: s = cp; c = -sp; break;
    case 2: s = -sp; c = -cp; break;
    default: s = -cp; c = sp; break;
    }
}
__device__ __forceinline__ float dm_cos(float x) { float s, c; dm_sincos(x, s, c); return c; }

__device__ inline float dm_asin(float x) {
    const float a = fabsf(x);
    float z, xx;
    bool flag = false;
    if (a > 0.5f) {
        z = 0.5f * (1.0f - a);
        xx = sqrtf(z);
        flag = true;
    } else {
        xx = a;
        z = a * a;
    }
    float r;
    if (a < 1.0e-4f && !flag) {
        r = xx;
    } else {
        r = ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z +
             1.6666752422e-1f) * z * xx + xx;
    }
    if (flag) {
        r = r + r;
        r = 1.5707963267948966f - r;
    }
    return x < 0.0f ? -r : r;
}
__device__ inline float dm_acos(float x) {
    if (x < -0.5f) return PI_F - 2.0f * dm_asin(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * dm_asin(sqrtf(0.5f * (1.0f - x)));
    return 1.5707963267948966f - dm_asin(x);
}
__device__ inline float dm_atan_core(float x) {
    float sgn = 1.0f, y;
    if (x < 0.0f) { sgn = -1.0f; x = -x; }
    if (x > 2.414213562373095f) {
        y = 1.5707963267948966f;
        x = -1.0f / x;
    } else if (x > 0.4142135623730950f) {
        y = 0.7853981633974483f;
        x = (x - 1.0f) / (x + 1.0f);
    } else {
        y = 0.0f;
    }
    const float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x + x);
    return sgn < 0.0f ? -y : y;
}
__device__ inline float dm_atan2(float y, float x) {
    int code = 0;
    if (x < 0.0f) code = 2;
    if (y < 0.0f) code |= 1;
    if (x == 0.0f) {
        if (code & 1) return -1.5707963267948966f;
        if (y == 0.0f) return 0.0f;
        return 1.5707963267948966f;
    }
    if (y == 0.0f) return (code & 2) ? PI_F : 0.0f;
    float w = 0.0f;
    if (code == 2) w = PI_F;
    else if (code == 3) w = -PI_F;
    return w + dm_atan_core(y / x);
}
__device__ __forceinline__ float dm_hypot(float x, float y) { return sqrtf(x * x + y * y); }

// ---------------------------------------------------------------------------
// counter-based RNG
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t path_state(uint32_t seed, uint32_t pixel, uint32_t sample) {
    uint32_t h = lowbias32(seed ^ 0xA511E9B3u);
    h = lowbias32(h ^ pixel);
    return lowbias32(h ^ (sample * 0x9E3779B9u));
}
__device__ __forceinline__ float rng_next(uint32_t &st) {
    const uint32_t s = st * 747796405u + 2891336453u;
    st = s;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    w = (w >> 22u) ^ w;
    return (float)(w >> 8) * (1.0f / 16777216.0f);
}

// RNG stream of branch b > 0 of a split first reflection
__device__ __forceinline__ uint32_t branch_state(uint32_t state, uint32_t b) {
    return lowbias32(state ^ (b * 0x632BE5ABu));
}

// ---------------------------------------------------------------------------
// rays, path state, counters
// ---------------------------------------------------------------------------
// What a closest-hit query needs (Scene::hit): origin, direction and the self-intersection
// key of contract C2 (last primitive + whether the ray points into it).
struct TraceRay {
    v3 o, d;
    uint32_t last_prim;
    bool self_inward;
};

// per-lane ESVO stack in LDS: entry (parent base, t_max) and 16-bit mask per scale, lanes
// interleaved with stride kStride (the threads of the block that traverse).  (A packed 9-B entry for a
// seventh wave of the depth-11 instances lost, round 5: tools/rejected/packed_stack.patch.)
// (Measured and rejected, round 6: the stackless traversal -- ancestors from a per-octant table, t_max in closed
// form -- and entries without t_max, tools/rejected/stackless.patch)
template <uint32_t kStride>
struct StackT {
    uint2 *e;
    uint16_t *m;
    __device__ __forceinline__ void write(uint32_t slot, uint32_t node, float t, uint32_t mask) const {
        e[slot * kStride] = make_uint2(node, __float_as_uint(t));
        m[slot * kStride] = (uint16_t)mask;
    }
    __device__ __forceinline__ void read(uint32_t slot, uint32_t &node, float &t, uint32_t &mask) const {
        const uint2 v = e[slot * kStride];
        node = v.x;
        mask = m[slot * kStride];
        t = __uint_as_float(v.y);
    }
};
using Stack = StackT<kBlock>;

// Path state between segments (Ray + HitRecord of ray/mod.rs:16-23, hittable/mod.rs:53-84,
// plus the forward throughput T / radiance L of the kernel's accumulation order).
struct PathState {
    v3 o, d, n;
    float col[4];
    v3 T, L;
    uint32_t cur, prev, depth, last_prim, path_segs, rng;
    bool specular;
    uint32_t branch;    // branch of a split first reflection (C20), 0 = the path's own stream
    uint32_t seg_base;  // branch > 0: the segments replayed before the split (not reported)
    float beam;         // a camera ray's beam start (octree t, beam_kernel), 0 = none
    // next-event estimation (sun sampling), used by the kNee instances only: while
    // `shadow` is set the ray is a get_direct_light_attenuation segment carrying `att`; the diffuse
    // bounce it interrupts waits in (co, cd, cn, clast, ccur), `mult` = |d_sun . n| * lum_a
    bool shadow;
    float att[4];
    float mult;
    v3 co, cd, cn;
    uint32_t clast, ccur;
};

struct Esvo {
    v3 t_coef, t_bias, pos;
    float t_min, t_max, h, scale_exp2;
    uint32_t parent, pmask, idx, mirror, iter;  // scale = exponent of scale_exp2 + OCTREE_MAX_SCALE - 127
};

// E.iter: the iteration count the reference's cap applies to (OCTREE_MAX_STEPS, octree_traversal.rs:127).
// A beam-started ray's count begins at beam_kernel's bound of the iterations its start skipped (esvo_begin):
// its caller subtracts that bound from the executed-iteration statistic when the ray begins.  A beam-started
// ray that reaches the cap may still have had iterations left in the reference (the bound over-counts the
// skipped ones), so it is traced again from its cube entry (extend's kHitCapped record, shade's retrace).
__device__ __forceinline__ bool esvo_capped(uint32_t it) { return it >= OCTREE_MAX_STEPS; }

struct Counters {
    uint32_t paths, segs, steps, sph, cub, shade, tex;
    uint32_t blk;  // block-value leaf tests (C23)
    uint32_t ib;   // issued load bytes of extend (OCTPT_COUNT_ISSUED builds; see ISSUED below)
    uint32_t redo;  // beam-started rays traced again from the cube entry (the step cap; stat word kStatBeamRestartWord)
#ifdef OCTPT_PROFILE_LANES  // diagnostic builds: per-wave lane occupancy of extend's step (stat words 8..)
    uint32_t p_iters, p_active, p_leaf_it, p_leaf_ln, p_pop_it, p_pop_ln, p_push_it, p_desc_ln, p_exact, p_fold_it,
        p_fold_ln, p_dfold_it, p_dfold_ln;
#endif
};

// Issued-bytes accounting (the honest reading of extend's roofline): a diagnostic build
// with -DOCTPT_COUNT_ISSUED adds the bytes of every load extend issues -- node slots of the lanes that
// load one, primitives, quads, alpha texels -- to Counters::ib; the product build compiles it out.
#ifdef OCTPT_COUNT_ISSUED
#define ISSUED(cnt, bytes) ((cnt).ib += (uint32_t)(bytes))
// named apart, so that a profile of bench.py (whose issued-bytes probe renders through this build)
// lists the counting kernel separately from the timed one
#define wf_extend_kernel wf_issued_extend_kernel
#else
#define ISSUED(cnt, bytes) ((void)0)
#endif

#ifdef OCTPT_PROFILE_LANES
// counted once per wave (by its first active lane): whether any lane has `cond`, and how many
__device__ __forceinline__ void prof_wave(uint32_t &it, uint32_t &ln, bool cond) {
    const uint64_t m = __ballot(cond), e = __ballot(true);
    if ((threadIdx.x & 63u) == (uint32_t)__ffsll((unsigned long long)e) - 1u) {
        it += m != 0ull ? 1u : 0u;
        ln += (uint32_t)__popcll(m);
    }
}
#endif

__device__ __forceinline__ uint32_t f2u32_sat(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967295.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

// the RGBA8 texel of Texture::value (texture.rs:64-93) for Texture::Image at (u, v): uv clamped, v
// flipped, nearest texel, corrected RGBA stride [C9]
__device__ __forceinline__ uint32_t image_texel(const DevScene &S, const DevTexture &t, float u, float v) {
    float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
    float vv = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    vv = 1.0f - vv;
    uint32_t i = f2u32_sat(uu * (float)t.width);
    uint32_t j = f2u32_sat(vv * (float)t.height);
    if (i > t.width - 1u) i = t.width - 1u;
    if (j > t.height - 1u) j = t.height - 1u;
    return *reinterpret_cast<const uint32_t *>(S.texels + t.offset + ((uint64_t)j * t.width + i) * 4u);
}

// Texture::value (texture.rs:64-93) for Texture::Image; colour textures are pre-converted into the
// material record at upload
__device__ inline void texture_image_value(const DevScene &S, uint32_t tex_idx, float u, float v, float out[4],
                                           Counters &cnt) {
    const DevTexture t = S.texs[tex_idx];
    if (t.height == 0u) { out[0] = out[1] = out[2] = out[3] = 1.0f; return; }
    const uint32_t px = image_texel(S, t, u, v);
    cnt.tex++;
    out[0] = S.lut_float[px & 255u];
    out[1] = S.lut_float[(px >> 8) & 255u];
    out[2] = S.lut_float[(px >> 16) & 255u];
    out[3] = (float)(px >> 24) / 255.0f;
}

// a primitive hit: t and the packed face flags inside | axis << 1 | (normal sign < 0) << 3
// (axis and sign describe the cuboid face; spheres leave them 0)
struct PrimHit {
    float t;
    uint32_t f;
    float u, v;  // block-value leaves (C23): the hit's texture coordinates, or a model quad's barycentrics
    __device__ uint32_t inside() const { return f & 1u; }
    __device__ uint32_t axis() const { return (f >> 1) & 3u; }
    __device__ float nsgn() const { return (f & 8u) ? -1.0f : 1.0f; }
};

// 8-B hit record (extend -> shade): x = cuboid bit | (inside | axis << 1 | neg << 3) << 27 | prim index
// (indices < 2^27, validated at upload, so a hit never encodes to kPrimNone), y = t bits
__device__ __forceinline__ uint2 hit_record(uint32_t prim, const PrimHit &h) {
    return make_uint2((prim & kPrimCuboidBit) | ((h.f & 15u) << 27) | (prim & kPrimIndexMask), __float_as_uint(h.t));
}

// OCTPT_CHECK_HITS (the diagnostic build liboctpt_checkhits.so): every step's PrimHit starts with
// sentinel fields, and a hit whose record fields (the ones shade reads) still hold the sentinel is counted
// (octpt_stats.hit_check_failures): a field the path that produced the hit did not write, or a codegen merge
// that let the lane keep the value it entered the step with (the block-leaf defect of round 3).
#ifdef OCTPT_CHECK_HITS
constexpr uint32_t kHitSentinel = 0x7FC0DEADu;  // a NaN payload no hit computation produces
#define HIT_POISON(prim, h) ((prim) = kPrimNone, (h).t = (h).u = (h).v = __uint_as_float(kHitSentinel), (h).f = kHitSentinel)
template <int kPrims>
__device__ __forceinline__ bool hit_unwritten(uint32_t prim, const PrimHit &h) {
    if (prim == kPrimNone) return true;
    if (kPrims == kPrimsBlocks)  // (face << 27 | block or the quad, t) + (u, v)
        return __float_as_uint(h.t) == kHitSentinel || __float_as_uint(h.u) == kHitSentinel ||
               __float_as_uint(h.v) == kHitSentinel;
    if (!(prim & kPrimCuboidBit)) return h.f == kHitSentinel;  // a sphere: its root flag (t is recomputed)
    return h.f == kHitSentinel || __float_as_uint(h.t) == kHitSentinel;  // a cuboid: face flags and t
}
#define HIT_CHECK(kP, rs, prim, h, stats, row_base)                                                                  \
    do {                                                                                                        \
        if ((rs) == kStepHit && hit_unwritten<kP>((prim), (h)))                                                  \
            atomicAdd(&(stats)[((row_base) + blockIdx.x % kSegs) * kStatRow + kStatHitCheckWord], 1ull);           \
    } while (0)
// The step's node slot is poisoned the same way (esvo_step): only the lanes that load a slot (descend, leaf)
// may take its fields, so a sentinel in the traversal state after a step -- the parent octant's slot base or
// its child mask, which every later step and the LDS stack carry on -- is a lane that read a slot it never
// loaded.  No slot base or mask equals the sentinel (slot arrays are < 2^31 entries, masks < 2^16).
// A lane caught with the sentinel is counted and its ray ends (the step cap: its next step loads nothing and
// reports a miss), so that a defect the check exposes never turns into a load from the poisoned base.
#define SLOT_CHECK(E, stats, row_base)                                                                           \
    do {                                                                                                        \
        if ((E).parent == kHitSentinel || (E).pmask == kHitSentinel) {                                           \
            atomicAdd(&(stats)[((row_base) + blockIdx.x % kSegs) * kStatRow + kStatHitCheckWord], 1ull);           \
            (E).parent = 0u;                                                                                    \
            (E).pmask = 0u;                                                                                     \
            (E).iter = OCTREE_MAX_STEPS;                                                                        \
        }                                                                                                       \
    } while (0)
#else
#define HIT_POISON(prim, h) ((void)0)
#define HIT_CHECK(kP, rs, prim, h, stats, row_base) ((void)0)
#define SLOT_CHECK(E, stats, row_base) ((void)0)
#endif

// Sphere::hit restated (sphere.rs:33-57) + root selection [C2].  The square root and divisions
// run only for lanes that can still hit: 48 % of C3's sphere tests have disc < 0 and 28 % are
// self tests, mostly of rays leaving outward, so the wave usually skips that block.
__device__ __forceinline__ bool sphere_test(float4 sp, const TraceRay &r, bool self_prim, PrimHit &h) {
    const v3 oc = vsub(V(sp.x, sp.y, sp.z), r.o);
    const float a = vdot(r.d, r.d);
    const float hh = vdot(r.d, oc);
    const float cc = vdot(oc, oc) - sp.w * sp.w;
    const float disc = hh * hh - a * cc;
    bool ok = false;
    if (disc >= 0.0f && (!self_prim || r.self_inward)) {
        const float sq = sqrtf(disc);
        bool near_ok = false;
        if (!self_prim) {
            const float t0 = (hh - sq) / a;
            near_ok = t0 > RAY_EPSILON;
            h.t = t0;
            h.f = 0u;
        }
        if (!near_ok) {
            const float t1 = (hh + sq) / a;
            h.t = t1;
            h.f = 1u;
        }
        ok = near_ok || h.t > RAY_EPSILON;
    }
    return ok;
}

// The root a sphere hit was accepted with, recomputed exactly (sphere_test's operations for that
// root): the wavefront extend decides sphere hits with sphere_decide's error-bounded estimate and
// its hit records carry that root (inside flag), not t; shade recomputes t here.
__device__ __forceinline__ float sphere_root(float4 sp, v3 o, v3 d, bool far) {
    const v3 oc = vsub(V(sp.x, sp.y, sp.z), o);
    const float a = vdot(d, d);
    const float hh = vdot(d, oc);
    const float cc = vdot(oc, oc) - sp.w * sp.w;
    const float sq = sqrtf(hh * hh - a * cc);
    return far ? (hh + sq) / a : (hh - sq) / a;
}

enum : int { kDecideMiss = 0, kDecideHit = 1, kDecideExact = 2 };

// sphere_test + the leaf's acceptance (t <= t_accept, C1) decided from an estimate: the hardware
// square root and reciprocal (v_sqrt_f32 / v_rcp_f32, 1 ulp each) instead of the correctly rounded
// expansions (~40 instructions, most of a leaf visit).  Every decision of the exact test -- disc >= 0,
// near root > EPSILON, far root > EPSILON, t <= t_accept -- compares a root against a threshold; the
// estimate differs from the exact root by less than m/2 with
//   m = (|hh| + sq) / a * 2^-19
// (|hh +- sq| <= |hh| + sq; sqrt 1.5 ulp, two roundings of the sum, reciprocal and product ~3 ulp,
// i.e. < 2^-20.2 (|hh| + sq) / a, kept with a factor 2 of slack), so a root farther than m from a
// threshold decides exactly as the exact test would.  Closer than m, or a sub-normal-range disc or a
// far from unit a, returns kDecideExact and the caller runs sphere_test.  disc, hh and a are the exact
// test's own values (same operations).  On kDecideHit, h.f = the root (inside flag); h.t is the
// estimate, never used as the hit's t (shade recomputes it with sphere_root).
__device__ __forceinline__ int sphere_decide(float4 sp, const TraceRay &r, bool self_prim, float t_accept, PrimHit &h) {
    const v3 oc = vsub(V(sp.x, sp.y, sp.z), r.o);
    const float a = vdot(r.d, r.d);
    const float hh = vdot(r.d, oc);
    const float cc = vdot(oc, oc) - sp.w * sp.w;
    const float disc = hh * hh - a * cc;
    if (!(disc >= 0.0f) || (self_prim && !r.self_inward)) return kDecideMiss;
    if (disc < 0x1p-100f || !(a > 0x1p-8f && a < 0x1p8f)) return kDecideExact;
    const float sq = __builtin_amdgcn_sqrtf(disc);
    const float ra = __builtin_amdgcn_rcpf(a);
    const float m = ((fabsf(hh) + sq) * ra) * 0x1p-19f;
    bool far = self_prim;
    float t = 0.0f;
    if (!self_prim) {
        t = (hh - sq) * ra;
        if (!(t > RAY_EPSILON + m)) {
            if (!(t <= RAY_EPSILON - m)) return kDecideExact;
            far = true;  // the near root is <= EPSILON exactly too: sphere_test takes the far root
        }
    }
    if (far) {
        t = (hh + sq) * ra;
        if (!(t > RAY_EPSILON + m)) return t <= RAY_EPSILON - m ? kDecideMiss : kDecideExact;
    }
    if (t > t_accept + m) return kDecideMiss;
    if (!(t <= t_accept - m)) return kDecideExact;
    h.t = t;
    h.f = far ? 1u : 0u;
    return kDecideHit;
}

// Ray::set_direction's clamped 1/d (mod.rs:91-112: |d| < 1e-6 -> 1e6) [C12], taken from ESVO's
// t_coef = 1 / -|rd| (esvo_begin, [C13]) with no division: where |d| >= 1e-6 (above both clamps,
// ESVO's 2^-23 and C12's 1e-6) rd = d, and the correctly rounded quotients 1/d and 1/-|d| are equal up
// to sign, d > 0 being ESVO's mirror bit.  Bit-identical to the three divides (the oracle's form).
__device__ __forceinline__ v3 inv_dir_of(v3 d, v3 t_coef, uint32_t mirror) {
    return V(fabsf(d.x) < 1e-6f ? 1.0f / 1e-6f : ((mirror & 1u) ? -t_coef.x : t_coef.x),
             fabsf(d.y) < 1e-6f ? 1.0f / 1e-6f : ((mirror & 2u) ? -t_coef.y : t_coef.y),
             fabsf(d.z) < 1e-6f ? 1.0f / 1e-6f : ((mirror & 4u) ? -t_coef.z : t_coef.z));
}

// AABB::intersects_new (aabb.rs:172-191) [C3]; inv = Ray::inv_dir (inv_dir_of)
__device__ __forceinline__ bool cuboid_test(float4 bmin, float4 bmax, const TraceRay &r, v3 inv, bool self_prim,
                                            PrimHit &h) {
    const v3 tb = vmul(vsub(V(bmin.x, bmin.y, bmin.z), r.o), inv);
    const v3 tt = vmul(vsub(V(bmax.x, bmax.y, bmax.z), r.o), inv);
    // inv is finite (clamped to +-1e6) and so are tb, tt: no NaN reaches these.  A +-0 can differ
    // from the oracle's a < b ? a : b only in sign, and a zero t is never accepted (t > EPSILON)
    // while the axis tests below compare with ==, so v_min3 / v_max3 give identical results.
    const v3 mins = V(tmn(tb.x, tt.x), tmn(tb.y, tt.y), tmn(tb.z, tt.z));
    const v3 maxs = V(tmx(tb.x, tt.x), tmx(tb.y, tt.y), tmx(tb.z, tt.z));
    float t0 = tmax3(mins);
    const float t1 = tmin3(maxs);
    if (!isfinite(t0)) t0 = t1;
    if (t1 < t0) return false;
    uint32_t inside;
    float t;
    if (self_prim) {
        if (!(r.self_inward && t1 > RAY_EPSILON)) return false;
        inside = 1u; t = t1;
    } else if (t0 > RAY_EPSILON) {
        inside = 0u; t = t0;
    } else if (t1 > RAY_EPSILON) {
        inside = 1u; t = t1;
    } else {
        return false;
    }
    uint32_t axis;
    if (!inside) axis = (mins.x == t0) ? 0u : ((mins.y == t0) ? 1u : 2u);
    else axis = (maxs.x == t1) ? 0u : ((maxs.y == t1) ? 1u : 2u);
    const float ia = axis == 0u ? inv.x : (axis == 1u ? inv.y : inv.z);
    const bool neg = inside ? !(ia > 0.0f) : (ia > 0.0f);  // normal sign per intersects_new's face
    h.t = t;
    h.f = inside | (axis << 1) | (neg ? 8u : 0u);
    return true;
}

// Quad::hit (geometry/quad.rs:172-200) in voxel-local coordinates, with the plane, normal and w
// derived at upload as Quad::new does (:90-114).  Accepts 0 < t <= t_next (back faces culled).
__device__ __forceinline__ bool quad_hit(const DevQuad &Q, v3 o_local, v3 d, float t_next, float &t, float &alpha,
                                         float &beta, Counters &cnt) {
    const float4 a = Q.o_d, n4 = Q.n_tv0;
    ISSUED(cnt, 32);
    const v3 nrm = V(n4.x, n4.y, n4.z);
    const float denom = vdot(d, nrm);
    if (denom >= -RAY_EPSILON) return false;
    t = (a.w - vdot(nrm, o_local)) / denom;
    if (t <= 0.0f || t > t_next) return false;
    const float4 u4 = Q.u_mat, v4 = Q.v_tu0, w4 = Q.w_tu1;
    ISSUED(cnt, 48);
    const v3 qu = V(u4.x, u4.y, u4.z), qv = V(v4.x, v4.y, v4.z), qw = V(w4.x, w4.y, w4.z);
    const v3 planar = vsub(vadd(o_local, vscale(d, t)), V(a.x, a.y, a.z));
    alpha = vdot(qw, vcross(planar, qv));
    beta = vdot(qw, vcross(qu, planar));
    return alpha >= 0.0f && alpha <= 1.0f && beta >= 0.0f && beta <= 1.0f;
}

// a block-model leaf (the reference's ResourceModel::Quad arm, octree_traversal.rs:207-213) [C19]:
// the closest of the model's quads with 0 < t <= t_accept, ties to the later quad (Quad::hit's
// `t > t_next` test), skipping the quad the ray leaves (last_prim = kQuadKey | quad)
__device__ inline bool model_test(const DevScene &S, const TraceRay &r, v3 voxel, uint32_t mdl, float t_accept,
                                  float &t_best, uint32_t &q_best, float &al_best, float &be_best, Counters &cnt) {
    const uint2 m = S.models[mdl];
    ISSUED(cnt, 8);
    const v3 ol = vsub(r.o, voxel);
    float t_next = t_accept;
    bool found = false;
    for (uint32_t k = 0; k < m.y; ++k) {
        const uint32_t q = m.x + k;
        if ((kQuadKey | q) == r.last_prim) continue;
        float t, al, be;
        if (quad_hit(S.quads[q], ol, r.d, t_next, t, al, be, cnt)) {
            t_next = t;
            q_best = q;
            al_best = al;
            be_best = be;
            found = true;
        }
    }
    t_best = t_next;
    return found;
}

__device__ __forceinline__ uint32_t face_index(uint32_t axis, float sgn) {
    if (axis == 0u) return sgn < 0.0f ? 0u : 1u;
    if (axis == 1u) return sgn < 0.0f ? 2u : 3u;
    return sgn > 0.0f ? 4u : 5u;
}

// A block-value leaf (C23; oracle block_leaf_test): the leaf payload is a block id and the block's box
// is the leaf cell itself, at any level -- the leaf arm of intersect_octree_path_tracer
// (octree_traversal.rs:143-214) restated from the ESVO state:
//  - a block model (slot flag kBlockIsModel, ResourceModel::Quad :207-213): its quads at the cell's
//    world corner (pos - 1) / octree_scale, closest before the cell exit + tolerance (C1, C19);
//  - a block filling its cell (ResourceModel::SingleBlock :193-206): passed when t_min == 0 (the ray
//    starts inside it, :194); else the face is the axis of the cell's largest entry t at pos + scale_exp2
//    (:156-162), the texture coordinates the entry point's other two coordinates over the cell, flipped
//    where the ray runs negative (:163-190), |u|, |v| (cuboid.rs:73-90); a face whose texture holds
//    alpha-0 texels (slot flag bit `face`) reads the texel and lets the ray through where its alpha is
//    <= EPSILON (SingleBlockModel::intersect, undefined in the reference).  Hit t = t_min / octree_scale.
// On a hit, prim = face << 27 | block (a full block) or kPrimCuboidBit | quad (a model quad), h.u / h.v =
// the texture coordinates or the quad's barycentrics.  x / 2^-depth and x / scale_exp2 are the products
// with the exact power-of-two reciprocals (the oracle divides).
__device__ inline bool block_leaf_test(const DevScene &S, const TraceRay &r, const Esvo &E, uint2 slot, float tc_max,
                                       uint32_t &prim, PrimHit &h, Counters &cnt) {
    cnt.blk++;
    const float se = E.scale_exp2;
    const v3 upos = V((E.mirror & 1u) ? (3.0f - se) - E.pos.x : E.pos.x,  // :149-154
                      (E.mirror & 2u) ? (3.0f - se) - E.pos.y : E.pos.y,
                      (E.mirror & 4u) ? (3.0f - se) - E.pos.z : E.pos.z);
    h.f = 0u;
    if (slot.y & kBlockIsModel) {
        const float inv = S.inv_octree_scale;
        const v3 voxel = V((upos.x - 1.0f) * inv, (upos.y - 1.0f) * inv, (upos.z - 1.0f) * inv);
        const float t_accept = tc_max * inv + CELL_TOL * (se * inv);
        const uint32_t mdl = S.blk_model[slot.x];
        ISSUED(cnt, 4);
        uint32_t q = 0u;
        float al = 0.0f, be = 0.0f;
        const bool found = model_test(S, r, voxel, mdl, t_accept, h.t, q, al, be, cnt);
        // the hit fields are written on both paths, not after a divergent return (fields
        // written only after the alpha test's divergent branch were left stale on passing lanes, round 3)
        prim = kPrimCuboidBit | q;
        h.u = al;
        h.v = be;
        return found;
    }
    if (E.t_min == 0.0f) return false;
    const float inv_se = __uint_as_float(0x7F000000u - __float_as_uint(se));  // 1 / scale_exp2, exact
    const v3 tcn = vsub(vmul(vadd(E.pos, V(se, se, se)), E.t_coef), E.t_bias);  // :156
    const float tc_min = tmax3(tcn);
    // ro and the clamped rd of esvo_begin (:71-93)
    const v3 ro = vadd(vscale(r.o, S.octree_scale), V(1.0f, 1.0f, 1.0f));
    v3 rd = r.d;
    const uint32_t epsb = __float_as_uint(OCTREE_EPSILON) & 0x7FFFFFFFu;
    if (fabsf(rd.x) < OCTREE_EPSILON) rd.x = __uint_as_float(epsb | (__float_as_uint(rd.x) & 0x80000000u));
    if (fabsf(rd.y) < OCTREE_EPSILON) rd.y = __uint_as_float(epsb | (__float_as_uint(rd.y) & 0x80000000u));
    if (fabsf(rd.z) < OCTREE_EPSILON) rd.z = __uint_as_float(epsb | (__float_as_uint(rd.z) & 0x80000000u));
    uint32_t axis;
    float u, v;
    bool neg;
    if (tcn.x == tc_min) {  // :163-171
        axis = 0u;
        u = ((ro.z + rd.z * tcn.x) - upos.z) * inv_se;
        v = ((ro.y + rd.y * tcn.x) - upos.y) * inv_se;
        neg = rd.x < 0.0f;
        if (neg) u = 1.0f - u;
    } else if (tcn.y == tc_min) {  // :172-180
        axis = 1u;
        u = ((ro.x + rd.x * tcn.y) - upos.x) * inv_se;
        v = ((ro.z + rd.z * tcn.y) - upos.z) * inv_se;
        neg = rd.y < 0.0f;
        if (neg) v = 1.0f - v;
    } else {  // :181-189
        axis = 2u;
        u = ((ro.x + rd.x * tcn.z) - upos.x) * inv_se;
        v = ((ro.y + rd.y * tcn.z) - upos.y) * inv_se;
        neg = rd.z < 0.0f;
        if (neg) u = 1.0f - u;
    }
    u = fabsf(u);
    v = fabsf(v);
    const uint32_t face = face_index(axis, neg ? 1.0f : -1.0f);  // the face entered faces against the ray
    prim = (face << 27) | slot.x;
    h.t = E.t_min * S.inv_octree_scale;
    h.u = u;
    h.v = v;
    if ((slot.y >> face) & 1u) {  // a face with alpha-0 texels: SingleBlockModel::intersect's texel
        const uint32_t mat = S.blk_mat[6u * slot.x + face];
        const DevMaterial &m = S.mats[mat];
        ISSUED(cnt, 8);
        float alpha;
        if (m.texture_kind == 0u) {
            alpha = m.color[3];
        } else {
            const DevTexture t = S.texs[m.texture_index];
            ISSUED(cnt, 32 + 4);
            alpha = t.height == 0u ? 1.0f : (float)(image_texel(S, t, u, v) >> 24) / 255.0f;
        }
        if (!(alpha > RAY_EPSILON)) return false;
    }
    return true;
}

// the material's colour at (u, v) into r.col (Texture::value, colour textures pre-converted)
__device__ __forceinline__ void material_color(const DevScene &S, uint32_t mat, float u, float v, PathState &r,
                                               Counters &cnt) {
    const DevMaterial &m = S.mats[mat];
    if (m.texture_kind == 0u) {
        r.col[0] = m.color[0];
        r.col[1] = m.color[1];
        r.col[2] = m.color[2];
        r.col[3] = m.color[3];
    } else {
        texture_image_value(S, m.texture_index, u, v, r.col, cnt);
    }
}

// Commit of a block-value leaf hit (C23, oracle commit_hit's block branches) [C1]: x = face << 27 | block
// (a block filling its cell: the face's normal and material, (hu, hv) its texture coordinates, no
// self-intersection key -- a ray starting in the block's cell passes it) or kPrimCuboidBit | quad (a
// block model's quad: its normal and material, uv from the barycentrics (hu, hv) as quad.rs:194-197, the
// quad's key kQuadKey | q, C19).
__device__ inline void commit_block_hit(const DevScene &S, PathState &r, uint32_t x, float t, float hu, float hv,
                                        Counters &cnt) {
    const v3 p = vadd(r.o, vscale(r.d, t));
    uint32_t mat, key;
    float u, v;
    v3 n;
    if (x & kPrimCuboidBit) {
        const uint32_t q = x & kPrimIndexMask;
        const DevQuad &Q = S.quads[q];
        n = V(Q.n_tv0.x, Q.n_tv0.y, Q.n_tv0.z);
        mat = __float_as_uint(Q.u_mat.w);
        const float tu0 = Q.v_tu0.w, tu1 = Q.w_tu1.w, tv0 = Q.n_tv0.w, tv1 = Q.tv1.x;
        u = tu0 + hu * (tu1 - tu0);
        v = tv0 + hv * (tv1 - tv0);
        key = kQuadKey | q;
    } else {
        const uint32_t face = x >> 27, block = x & kPrimIndexMask;
        mat = S.blk_mat[6u * block + face];
        // Face::to_normal (cuboid.rs:20-29): W -X, E +X, Bottom -Y, Top +Y, South +Z, North -Z
        const float sgn = (face == 1u || face == 3u || face == 4u) ? 1.0f : -1.0f;
        n = V(0.0f, 0.0f, 0.0f);
        if (face < 2u) n.x = sgn; else if (face < 4u) n.y = sgn; else n.z = sgn;
        u = hu;
        v = hv;
        key = kPrimNone;
    }
    r.o = p;
    r.n = n;
    r.last_prim = key;
    r.cur = mat;
    material_color(S, mat, u, v, r, cnt);
}

// Chunky-style commit [C1]: the ray origin moves to the hit point
// kSP: the primitive kinds of the scene a shade instance serves (kPrims*: spheres only; boxes without block models;
// block values only; kPrimsModels = any scene; kShadeSphColour: spheres only and colour textures only), so that a
// scene's instance carries no other kind's code
constexpr int kShadeSphColour = 4;
constexpr bool sph_kind(int k) { return k == kPrimsSpheres || k == kShadeSphColour; }
template <int kSP = kPrimsModels>
__device__ inline void commit_hit(const DevScene &S, PathState &r, uint32_t prim, const PrimHit &h, Counters &cnt) {
    if (kSP == kPrimsBlocks || (kSP == kPrimsModels && S.has_blocks)) {
        commit_block_hit(S, r, prim, h.t, h.u, h.v, cnt);
        return;
    }
    const v3 p = vadd(r.o, vscale(r.d, h.t));
    float u = 0.0f, v = 0.0f;
    uint32_t mat;
    v3 n;
    bool uv_ready;
    if (sph_kind(kSP) || !(prim & kPrimCuboidBit)) {
        const float4 sp = S.spheres[prim];
        n = V((p.x - sp.x) / sp.w, (p.y - sp.y) / sp.w, (p.z - sp.z) / sp.w);
        mat = S.sphere_mat[prim];
        uv_ready = false;  // sphere uv only feeds image textures (computed lazily below)
    } else {
        // the box, its face material (the face is in the hit record) and its model id load together
        const uint32_t ci = prim & ~kPrimCuboidBit;
        const float4 ca = S.cub_a[ci];
        const float2 cb = S.cub_b[ci];
        const uint32_t axis = h.axis();
        const float nsgn = h.nsgn();
        mat = S.cub_mat[6u * ci + face_index(axis, nsgn)];
        const uint32_t mdl = (kSP == kPrimsModels && S.has_models) ? S.cub_model[ci] : OCTPT_MODEL_NONE;
        if (mdl != OCTPT_MODEL_NONE) {
            // block-model hit [C19]: the hit record holds the instance and t; the quad is the one
            // model_test chose, found again by the same computation with t_next = t
            uint32_t q = 0u;
            float al = 0.0f, be = 0.0f, tq;
            TraceRay tr;
            tr.o = r.o;
            tr.d = r.d;
            tr.last_prim = r.last_prim;
            tr.self_inward = false;
            model_test(S, tr, V(ca.x, ca.y, ca.z), mdl, h.t, tq, q, al, be, cnt);
            const DevQuad &Q = S.quads[q];
            n = V(Q.n_tv0.x, Q.n_tv0.y, Q.n_tv0.z);
            mat = __float_as_uint(Q.u_mat.w);
            const float tu0 = Q.v_tu0.w, tu1 = Q.w_tu1.w, tv0 = Q.n_tv0.w, tv1 = Q.tv1.x;
            u = tu0 + al * (tu1 - tu0);  // quad.rs:194-197
            v = tv0 + be * (tv1 - tv0);
            uv_ready = true;
            prim = kQuadKey | q;  // the self-intersection key of the next segment
        } else {
            const float4 bmin = make_float4(ca.x, ca.y, ca.z, 0.0f), bmax = make_float4(ca.w, cb.x, cb.y, 0.0f);
            n = V(0.0f, 0.0f, 0.0f);
            if (axis == 0u) n.x = nsgn; else if (axis == 1u) n.y = nsgn; else n.z = nsgn;
            const float ex = bmax.x - bmin.x, ey = bmax.y - bmin.y, ez = bmax.z - bmin.z;
            if (axis == 0u) {
                u = (p.z - bmin.z) / ez; v = (p.y - bmin.y) / ey;
                if (r.d.x < 0.0f) u = 1.0f - u;
            } else if (axis == 1u) {
                u = (p.x - bmin.x) / ex; v = (p.z - bmin.z) / ez;
                if (r.d.y < 0.0f) v = 1.0f - v;
            } else {
                u = (p.x - bmin.x) / ex; v = (p.y - bmin.y) / ey;
                if (r.d.z < 0.0f) u = 1.0f - u;
            }
            u = fabsf(u);
            v = fabsf(v);
            uv_ready = true;
        }
    }
    r.o = p;
    r.n = n;
    r.last_prim = prim;
    if (h.inside()) {
        r.cur = 0u;
        r.col[0] = r.col[1] = r.col[2] = r.col[3] = 0.0f;
    } else {
        r.cur = mat;
        const DevMaterial &m = S.mats[mat];
        if (kSP == kShadeSphColour || m.texture_kind == 0u) {  // (a colour-only scene's instance has no image path)
            r.col[0] = m.color[0];
            r.col[1] = m.color[1];
            r.col[2] = m.color[2];
            r.col[3] = m.color[3];
        } else {
            if (!uv_ready) {
                const float theta = dm_acos(-n.y);  // Sphere::get_uv (sphere.rs:60-69)
                const float phi = dm_atan2(-n.z, n.x) + PI_F;
                u = phi / (2.0f * PI_F);
                v = theta / PI_F;
            }
            texture_image_value(S, m.texture_index, u, v, r.col, cnt);
        }
    }
}

// ---------------------------------------------------------------------------
// ESVO (octree_traversal.rs:54-302) split into setup + one iteration
// ---------------------------------------------------------------------------
template <uint32_t kS>
__device__ __forceinline__ void stk_write(const StackT<kS> &stk, uint32_t slot, uint32_t node, float t, uint32_t mask) {
    stk.write(slot, node, t, mask);
}

template <uint32_t kS = kBlock>
__device__ __forceinline__ StackT<kS> stack_of(uint2 *lds, uint32_t depth) {
    StackT<kS> s;
    s.e = lds + threadIdx.x;
    s.m = reinterpret_cast<uint16_t *>(lds + (size_t)(depth - 1u) * kS) + threadIdx.x;
    return s;
}

__device__ __forceinline__ TraceRay make_trace_ray(const DevScene &S, v3 o, v3 d, uint32_t last_prim, bool inward) {
    TraceRay t;
    t.o = o;
    t.d = d;
    t.last_prim = last_prim;
    t.self_inward = inward;
    return t;
}

// The cell of the root that ESVO's first iteration processes: the child holding the point at t_min
// (octree_traversal.rs:113-125).
__device__ __forceinline__ void esvo_first_child(Esvo &E) {
    E.idx = 0u;
    E.pos = V(1.0f, 1.0f, 1.0f);
    const v3 upper = vsub(vscale(E.t_coef, 1.5f), E.t_bias);
    if (upper.x > E.t_min) { E.idx ^= 1u; E.pos.x = 1.5f; }
    if (upper.y > E.t_min) { E.idx ^= 2u; E.pos.y = 1.5f; }
    if (upper.z > E.t_min) { E.idx ^= 4u; E.pos.z = 1.5f; }
}

// ESVO's state at the cube entry from the ray's t_coef / t_bias / mirror (octree_traversal.rs:79-112; the
// first child follows, esvo_first_child): the walk of the reference from its first iteration.  Also how a
// beam-started ray that reached the step cap starts again (the drain's restart): its t_coef, t_bias and
// mirror are the ray's own, only the walk restarts.
__device__ __forceinline__ void esvo_root(const DevScene &S, Esvo &E) {
    E.parent = S.root;
    E.pmask = S.root_mask;
    E.scale_exp2 = 0.5f;
    E.t_min = tmx(tmax3(vsub(vscale(E.t_coef, 2.0f), E.t_bias)), 0.0f);
    E.t_max = tmin3(vsub(E.t_coef, E.t_bias));
    E.h = E.t_max;
    E.iter = 0u;
}

// t_start > 0 (a camera ray with a beam start, beam_kernel): no octree leaf lies within the ray's
// tile frustum before t_start, so ESVO starts there instead of at the cube entry (Laine & Karras'
// beam optimisation).  ESVO lands in the cell that holds the point at t_start and walks on from it;
// the cells it skips are empty, so the first leaf it meets, and with it the hit, is the reference's.
// t_start less a bound of ESVO's own rounding of t-values (which grows with |t_coef|, i.e. for
// rays near-parallel to an axis), clamped to the cube exit.  The low kBeamIterBits of t_start's bits
// hold a bound of the reference iterations before the start (beam_kernel), at which the iteration
// count begins, so that the reference's step cap still applies (a ray reaching it is traced again from
// its cube entry, esvo_capped).
template <uint32_t kS>
__device__ inline void esvo_begin(const DevScene &S, const TraceRay &ray, Esvo &E, const StackT<kS> &stk,
                                  float t_start = 0.0f) {
    const float osc = S.octree_scale;
    // The reference zero-initialises the stack (octree_traversal.rs:69-70).  ESVO only pops to a
    // scale it pushed during the same ray (a push is skipped only when the entry already holds the
    // same parent), so stale entries are never read and the zeroing is omitted; the oracle keeps it
    // and the parity tests would expose any violation.
    v3 ro = vscale(ray.o, osc);
    v3 rd = ray.d;
    ro = vadd(ro, V(1.0f, 1.0f, 1.0f));
    const uint32_t epsb = __float_as_uint(OCTREE_EPSILON) & 0x7FFFFFFFu;
    if (fabsf(rd.x) < OCTREE_EPSILON) rd.x = __uint_as_float(epsb | (__float_as_uint(rd.x) & 0x80000000u));
    if (fabsf(rd.y) < OCTREE_EPSILON) rd.y = __uint_as_float(epsb | (__float_as_uint(rd.y) & 0x80000000u));
    if (fabsf(rd.z) < OCTREE_EPSILON) rd.z = __uint_as_float(epsb | (__float_as_uint(rd.z) & 0x80000000u));
#if OCTPT_RCP_FAST
    // the correctly rounded quotients from v_rcp_f32 + one fused Newton step (octpt_rcp.h: compared with
    // the division for every |rd| in [2^-23, 2^126] by tools/rcp_check.hip), 3 instead of ~11 instructions each
    E.t_coef = V(rcp_rn(-fabsf(rd.x)), rcp_rn(-fabsf(rd.y)), rcp_rn(-fabsf(rd.z)));  // [C13]
#else
    E.t_coef = V(1.0f / -fabsf(rd.x), 1.0f / -fabsf(rd.y), 1.0f / -fabsf(rd.z));  // [C13]
#endif
    E.t_bias = vmul(E.t_coef, ro);
    E.mirror = 0u;
    if (rd.x > 0.0f) { E.mirror |= 1u; E.t_bias.x = 3.0f * E.t_coef.x - E.t_bias.x; }
    if (rd.y > 0.0f) { E.mirror |= 2u; E.t_bias.y = 3.0f * E.t_coef.y - E.t_bias.y; }
    if (rd.z > 0.0f) { E.mirror |= 4u; E.t_bias.z = 3.0f * E.t_coef.z - E.t_bias.z; }
    esvo_root(S, E);
    if (t_start > 0.0f) {
        const float ro_m = tmx(tmx(fabsf(ro.x), fabsf(ro.y)), fabsf(ro.z));
        const float tc_m = -tmn(tmn(E.t_coef.x, E.t_coef.y), E.t_coef.z);
        const float margin = 0x1p-16f * (4.0f + ro_m) * tc_m;
        E.t_min = tmx(E.t_min, tmn(t_start - margin, E.t_max));
        // the reference's step cap counts from the cube entry: the count starts at beam_kernel's bound
        // of the iterations skipped (carried in t_start's low mantissa bits, beam_pack)
        E.iter = __float_as_uint(t_start) & kBeamIterMask;
    }
    esvo_first_child(E);
}

enum : int { kStepContinue = 0, kStepHit = 1, kStepMiss = 2 };

// One descend-only ESVO iteration (octree_traversal.rs:216-244, counted in E.iter) into the child
// whose slot is (its base, its mask); tc / tc_max / tv_max are the current cell's t_corner, its
// minimum and min(t_max, tc_max).  The same operations as esvo_step's descend.
template <uint32_t kS>
__device__ __forceinline__ void esvo_descend(Esvo &E, const StackT<kS> &stk, uint32_t depth, v3 tc, float tc_max,
                                             float tv_max, uint2 slot) {
    E.iter += 1u;
    const float half = E.scale_exp2 * 0.5f;
    const v3 X = vadd(vscale(E.t_coef, half), tc);
    const bool dx = X.x > E.t_min, dy = X.y > E.t_min, dz = X.z > E.t_min;
    if (dx) E.pos.x = E.pos.x + half;
    if (dy) E.pos.y = E.pos.y + half;
    if (dz) E.pos.z = E.pos.z + half;
    const uint32_t slot_u = (__float_as_uint(E.scale_exp2) >> 23) - 128u + depth;
    if (tc_max < E.h) stk_write(stk, slot_u, E.parent, E.t_max, E.pmask);
    E.h = tc_max;
    E.parent = slot.x;
    E.pmask = slot.y;
    E.scale_exp2 = half;
    E.t_max = tv_max;
    E.idx = (dx ? 1u : 0u) | (dy ? 2u : 0u) | (dz ? 4u : 0u);
}


#ifndef OCTPT_LEAD_LOOP
#define OCTPT_LEAD_LOOP 0
#endif
// The descends a ray's ESVO takes before its first other iteration, as a loop of exact descend replicas
// (esvo_descend: the same stop tests, t-values, push and child choice as esvo_step's descend), each one
// dependent node-slot load.  A lane leaves the loop at the first iteration that would not descend.
template <class Stk>
__device__ __forceinline__ void lead_descends(const DevScene &S, Esvo &E, const Stk &stk) {
    const float max_dst = MAX_DST_WORLD * S.octree_scale;
    for (;;) {
        const uint32_t cidx = E.idx ^ E.mirror;
        const v3 tc = vsub(vmul(E.pos, E.t_coef), E.t_bias);
        const float tc_max = tmin3(tc);
        const float tv_max = tmn_nc(E.t_max, tc_max);
        const bool d = (((E.pmask >> cidx) & 0x101u) == 0x001u) & !esvo_capped(E.iter) & !(E.t_min > max_dst) &
                       (E.t_min <= tv_max);
        if (!d) break;
        const uint2 slot = S.node_child[E.parent + __popc(E.pmask & ((1u << cidx) - 1u))];
        esvo_descend(E, stk, S.depth, tc, tc_max, tv_max, slot);
    }
}

#ifndef OCTPT_FOLD
#define OCTPT_FOLD 1  // absent-sibling folds per step (A/B: -DOCTPT_FOLD=0)
#endif
#ifndef OCTPT_FOLD_SPHERES
// the sphere instance folds up to 2 (round 5: C3 +0.4 %; the box instance stays at 1: 2 folds there C4 -2.2 %)
#define OCTPT_FOLD_SPHERES 2
#endif
#ifndef OCTPT_FOLD_MODELS
// the block-model instance folds up to 2 (C5, depth-11 voxel terrain: +1.9 %; 2 folds everywhere:
// C3 -2.4 %, C4 -2.9 %, C2 +-0)
#define OCTPT_FOLD_MODELS 2
#endif
#ifndef OCTPT_DFOLD
// descend fold in esvo_step, per instance: measured +4 % extend on C5 (block models, depth 11),
// +-1 % on C3 / C2 / C4 in round 2, so 3 = the block-model instance, plus the block-value and sphere
// instances by their own knobs below (A/B: -DOCTPT_DFOLD=0 / 1 = all)
#define OCTPT_DFOLD 3
#endif
// the sphere instance's descend fold (round 3, after the lane-mask and spill work: C3 extend -1.4..-2.1 %,
// C2 -1 %; the box instance stays without it, C4 +0.4..+0.8 %)
#ifndef OCTPT_DFOLD_SPHERES
#define OCTPT_DFOLD_SPHERES 1
#endif
// descend folds per step where the descend fold is on (A/B knob)
#ifndef OCTPT_DFOLD_N
#define OCTPT_DFOLD_N 1
#endif
// the block-value instance (C23): absent-sibling folds per step and the descend fold (A/B knobs)
#ifndef OCTPT_FOLD_BLOCKS
#define OCTPT_FOLD_BLOCKS 2
#endif
#ifndef OCTPT_DFOLD_BLOCKS
#define OCTPT_DFOLD_BLOCKS 1
#endif


// leaf primitive list test [C1].  Leaf slot = (first list index, count), or (prim id, 1) for the
// common single-primitive leaf (one dependent load fewer).  t_accept = t_exit_w + CELL_TOL * cell_w.
// kPrims: the primitive kinds a scene holds (kPrimsSpheres: the slab test's temporaries never
// reserve registers, 7 waves/SIMD in wf_extend_kernel; kPrimsBoxes adds cuboids, kPrimsModels
// block-model cuboids)
template <int kPrims>
__device__ __forceinline__ bool prim_test(const DevScene &S, const TraceRay &r, const Esvo &E, uint32_t prim,
                                          float t_accept, PrimHit &h, Counters &cnt) {
    const bool self_prim = prim == r.last_prim;
    bool ok;
    if (kPrims == kPrimsSpheres || !(prim & kPrimCuboidBit)) {
        cnt.sph++;
        ISSUED(cnt, 16);
        ok = sphere_test(S.spheres[prim], r, self_prim, h);
    } else {
        cnt.cub++;
        const uint32_t ci = prim & ~kPrimCuboidBit;
        const float4 ca = S.cub_a[ci];
        ISSUED(cnt, 16);
        if (kPrims == kPrimsModels && S.has_models) {
            const uint32_t mdl = S.cub_model[ci];
            ISSUED(cnt, 4);
            if (mdl != OCTPT_MODEL_NONE) {
                uint32_t q;
                float al, be;
                h.f = 0u;
                return model_test(S, r, V(ca.x, ca.y, ca.z), mdl, t_accept, h.t, q, al, be, cnt);
            }
        }
        const float2 cb = S.cub_b[ci];
        ISSUED(cnt, 8);
        // 1/d without the three correctly-rounded divides: ESVO's t_coef holds the same quotients
        const v3 inv = inv_dir_of(r.d, E.t_coef, E.mirror);
        ok = cuboid_test(make_float4(ca.x, ca.y, ca.z, 0.0f), make_float4(ca.w, cb.x, cb.y, 0.0f), r, inv, self_prim, h);
    }
    return ok && h.t <= t_accept;
}

// kCuboids = false: sphere-only scenes; the slab test's temporaries then never reserve
// registers (70 instead of 85 VGPRs in wf_extend_kernel: 7 waves/SIMD instead of 5).
// The first primitive is tested straight-line (leaves hold 1.02 primitives on average); the
// rest of a multi-primitive list in a loop, keeping the closest accepted hit.
// kFast (wavefront extend): a single-sphere leaf is decided by sphere_decide, falling back to the
// exact test only when the estimate lies too close to a threshold; its hit carries the root, not t.
template <int kPrims = kPrimsModels, bool kFast = false>
__device__ inline bool leaf_test(const DevScene &S, const TraceRay &r, const Esvo &E, uint2 lr, float t_accept,
                                 uint32_t &best_prim, PrimHit &best, Counters &cnt, const float4 *pre = nullptr) {
    uint32_t prim = lr.x;
    if (lr.y != 1u) {
        prim = S.leaf_prims[lr.x];
        ISSUED(cnt, 4);
    }
    bool found;
    if (kFast && lr.y == 1u && (kPrims == kPrimsSpheres || !(prim & kPrimCuboidBit))) {
        cnt.sph++;
        if (!(kPrims == kPrimsSpheres && pre)) ISSUED(cnt, 16);
        const float4 sp = (kPrims == kPrimsSpheres && pre) ? *pre : S.spheres[prim];
        const bool self_prim = prim == r.last_prim;
        const int d = sphere_decide(sp, r, self_prim, t_accept, best);
#ifdef OCTPT_PROFILE_LANES
        cnt.p_exact += d == kDecideExact ? 1u : 0u;
#endif
        if (__builtin_expect(d == kDecideExact, 0)) found = sphere_test(sp, r, self_prim, best) && best.t <= t_accept;
        else found = d == kDecideHit;
        if (found) best_prim = prim;
        return found;
    }
    if (kPrims == kPrimsSpheres && pre && lr.y == 1u) {
        // single-sphere leaf: its sphere arrived with the slot (leaf_sph, loaded beside node_child)
        cnt.sph++;
        found = sphere_test(*pre, r, prim == r.last_prim, best) && best.t <= t_accept;
    } else {
        found = prim_test<kPrims>(S, r, E, prim, t_accept, best, cnt);
    }
    if (found) best_prim = prim;
    for (uint32_t k = 1; k < lr.y; ++k) {
        const uint32_t p = S.leaf_prims[lr.x + k];
        ISSUED(cnt, 4);
        PrimHit hk;
        if (prim_test<kPrims>(S, r, E, p, t_accept, hk, cnt) && (!found || hk.t < best.t)) {
            best = hk;
            best_prim = p;
            found = true;
        }
    }
    return found;
}

// one ESVO iteration (octree_traversal.rs:127-300); on kStepHit (prim, h) hold the accepted
// primitive hit.  The step-limit / max_dst miss is taken at the end: a lane past either runs the
// step with no memory side effects (not live) and reports the miss, so the exit costs no exec-mask
// region.  Callers add E.iter to cnt.steps when the ray finishes.
template <int kPrims = kPrimsModels, bool kFast = false, uint32_t kS = kBlock>
__device__ inline int esvo_step(const DevScene &S, const TraceRay &ray, Esvo &E, const StackT<kS> &stk, Counters &cnt,
                                uint32_t &prim, PrimHit &h) {
    // :128-130: max_dst = 1024 * 2^-depth > 0, so the reference's `max_dst >= 0` guard always holds
    const float max_dst = MAX_DST_WORLD * S.octree_scale;  // :75, wave-uniform
#ifndef OCTPT_SETPRIO
#define OCTPT_SETPRIO 1  // round 6: C3 +0.4..0.6 %, C4 +1.0..1.2 %; the block instances mixed (profiles/r06/setprio_ab.txt)
#endif
    // Wave priority around the node-slot load: a wave at the top of its step (about to issue the load its next
    // iteration waits for) issues ahead of the waves in the rest of their step's arithmetic, so the SIMD's loads
    // go out sooner (the sphere and box instances; the block instances measured mixed)
    constexpr int kPrio = (kPrims == kPrimsSpheres || kPrims == kPrimsBoxes) ? OCTPT_SETPRIO : 0;
    if constexpr (kPrio > 0) __builtin_amdgcn_s_setprio(kPrio);
    const bool stopped = esvo_capped(E.iter) | (E.t_min > max_dst);
    E.iter += stopped ? 0u : 1u;
    const v3 t_corner = vsub(vmul(E.pos, E.t_coef), E.t_bias);
    const float tc_max = tmin3(t_corner);
    const uint32_t cidx = E.idx ^ E.mirror;
    // the child's two mask bits in one word: 0x101 leaf, 0x001 octant (bit 0 present, bit 8 leaf)
    const uint32_t kind = (E.pmask >> cidx) & 0x101u;
    // :142-244.  Leaf (t_min >= 0) and descend (t_min <= min(t_max, tc_max)) lanes share one slot
    // load instruction: on CDNA4 a scattered load costs the vector-memory pipe per instruction.
    // (t_min <= tv_max implies the reference's t_min <= t_max for the descend.)
    const float tv_max = tmn_nc(E.t_max, tc_max);
    const bool take_leaf = (kind == 0x101u) & !stopped & (E.t_min <= E.t_max) & (E.t_min >= 0.0f);
    const bool descend = (kind == 0x001u) & !stopped & (E.t_min <= tv_max);
    // (a lane that loads nothing never reads slot: an empty asm hands it whatever its registers hold
    // instead of zeroing them, two v_mov per step; the check build poisons it instead, SLOT_CHECK)
    uint2 slot;
#ifdef OCTPT_CHECK_HITS
    slot = make_uint2(kHitSentinel, kHitSentinel);
#else
    asm("" : "=v"(slot.x), "=v"(slot.y));
#endif
    const uint32_t sidx = E.parent + __popc(E.pmask & ((1u << cidx) - 1u));
    if (take_leaf | descend) {
        slot = S.node_child[sidx];
        ISSUED(cnt, 8);
    }
    // sphere-only scenes: a leaf's first sphere is loaded beside its slot (no dependent second load)
    float4 lsph = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (kPrims == kPrimsSpheres && take_leaf) {
        lsph = S.leaf_sph[sidx];
        ISSUED(cnt, 16);
    }
    if constexpr (kPrio > 0) __builtin_amdgcn_s_setprio(0);
#ifdef OCTPT_PROFILE_LANES
    prof_wave(cnt.p_leaf_it, cnt.p_leaf_ln, take_leaf);
    prof_wave(cnt.p_push_it, cnt.p_desc_ln, descend);
#endif
    bool leaf_hit = false;
    if (take_leaf) {
        // x / 2^-depth == x * 2^depth exactly (the oracle divides)
        const float cell_w = E.scale_exp2 * S.inv_octree_scale;
        const float t_accept = tc_max * S.inv_octree_scale + CELL_TOL * cell_w;
        // a hit lane runs the advance below too (its state is discarded): the descend / advance
        // block then needs no exec-mask region of its own
        if constexpr (kPrims == kPrimsBlocks)
            leaf_hit = block_leaf_test(S, ray, E, slot, tc_max, prim, h, cnt);
        else
            leaf_hit = leaf_test<kPrims, kFast>(S, ray, E, slot, t_accept, prim, h, cnt,
                                                kPrims == kPrimsSpheres ? &lsph : nullptr);
    }
    // Descend (:216-244) and advance (:249-260) as one select-based update: every lane computes
    // X = t_coef * f + t_corner with f = half for descend (X = t_center) and f = 0 otherwise
    // (t_coef * 0 = -0 and x + -0 == x, so X = t_corner exactly), then moves pos by +half where
    // t_center > t_min (descend) or by -scale_exp2 where t_corner <= tc_max (advance).  A wave
    // runs both paths anyway; one shared body avoids the branch bookkeeping and phi copies.
    const float half = E.scale_exp2 * 0.5f;
    const float f = descend ? half : 0.0f;
    const float Y = descend ? E.t_min : tc_max;
    const float delta = descend ? half : -E.scale_exp2;
    const v3 X = vadd(vscale(E.t_coef, f), t_corner);
    // t-values are NaN-free: !(X > Y) == (X <= Y)
    const bool cx = (X.x > Y) == descend, cy = (X.y > Y) == descend, cz = (X.z > Y) == descend;
    if (cx) E.pos.x = E.pos.x + delta;
    if (cy) E.pos.y = E.pos.y + delta;
    if (cz) E.pos.z = E.pos.z + delta;
    uint32_t step_mask = (cx ? 1u : 0u) | (cy ? 2u : 0u) | (cz ? 4u : 0u);
    // push: level = scale - (OCTREE_MAX_SCALE - depth) = exponent(scale_exp2) - 127 + depth is in
    // [1, depth) for a descend: leaf cells (level 0) are never descended from, and a pop always rises
    // at least one level above them, so level 0 is never written or read and LDS holds levels
    // 1..depth-1 (stack slot = level - 1 >= 0; the oracle's level-0 entry stays zero, like the miss
    // below).  One guarded write, so that the selects below stay branch-free.
    const uint32_t slot_u = (__float_as_uint(E.scale_exp2) >> 23) - 128u + S.depth;
    if (descend & (tc_max < E.h)) stk_write(stk, slot_u, E.parent, E.t_max, E.pmask);
    E.h = descend ? tc_max : E.h;
#ifdef OCTPT_SLOT_LEAK_PROBE
    // negative control of SLOT_CHECK (scripts/stale_hit_probe.py slotleak_check): a lane advancing past an
    // absent child takes the slot it never loaded; the check build must count it
    const bool take_slot = descend | ((kind == 0u) & !stopped);
#else
    const bool take_slot = descend;
#endif
    E.parent = take_slot ? slot.x : E.parent;  // (octant, its mask)
    E.pmask = take_slot ? slot.y : E.pmask;
    E.scale_exp2 = descend ? half : E.scale_exp2;
    E.t_max = descend ? tv_max : E.t_max;
    E.t_min = descend ? E.t_min : tc_max;
    E.idx = descend ? step_mask : (E.idx ^ step_mask);
    bool pop = !descend & ((E.idx & step_mask) != 0u);
#if OCTPT_DFOLD
    // Descend fold: a descend whose chosen child is again an octant the ray enters is followed, in
    // the reference, by an iteration that only descends (:216-244); 26 % of C3's iterations are such
    // descend-after-descend pairs (tools/esvo_trace.py).  That iteration is run here as an exact
    // replica (its own stop tests, t_corner, push and child choice, counted in E.iter); its slot
    // load depends on this step's, which the other waves of the SIMD hide.
    constexpr int kDFolds = (OCTPT_DFOLD != 3 || kPrims == kPrimsModels || (kPrims == kPrimsBlocks && OCTPT_DFOLD_BLOCKS) ||
                             (kPrims == kPrimsSpheres && OCTPT_DFOLD_SPHERES)) ? OCTPT_DFOLD_N : 0;
    bool dmore = descend;
#pragma unroll
    for (int k = 0; k < kDFolds; ++k) {  // up to kDFolds descend-only iterations after a descend (A/B: OCTPT_DFOLD_N)
    if (dmore) {
        const uint32_t cidx2 = E.idx ^ E.mirror;
        const v3 tc2 = vsub(vmul(E.pos, E.t_coef), E.t_bias);
        const float tc2_max = tmin3(tc2);
        const float tv2_max = tmn_nc(E.t_max, tc2_max);
        const bool d2 = (((E.pmask >> cidx2) & 0x101u) == 0x001u) & !esvo_capped(E.iter) &
                        !(E.t_min > max_dst) & (E.t_min <= tv2_max);
#ifdef OCTPT_PROFILE_LANES
        prof_wave(cnt.p_dfold_it, cnt.p_dfold_ln, d2);
#endif
        if (d2) {
            const uint2 slot2 = S.node_child[E.parent + __popc(E.pmask & ((1u << cidx2) - 1u))];
            ISSUED(cnt, 8);
            esvo_descend(E, stk, S.depth, tc2, tc2_max, tv2_max, slot2);
        }
        dmore = d2;
    }
    }
#endif
#if OCTPT_FOLD
    // Absent-sibling fold: when the child this step moved to is absent, the reference's next
    // iteration (:127-141, then :249-299) only advances past it.  That iteration is run here, as an
    // exact replica (same t_corner / tc_max / step_mask operations, counted in E.iter, same stop
    // tests), so the wave does not pay a whole loop iteration for it.  44 % of C3's iterations are
    // such advances; folding the first of each run leaves 72 % of the iterations (tools/esvo_trace.py).
    // A fold that leaves the parent pops below, exactly as that iteration would.
    constexpr int kFolds = kPrims == kPrimsModels ? OCTPT_FOLD_MODELS
                           : kPrims == kPrimsBlocks ? OCTPT_FOLD_BLOCKS
                           : kPrims == kPrimsSpheres ? OCTPT_FOLD_SPHERES : OCTPT_FOLD;
#pragma unroll
    for (int k = 0; k < kFolds; ++k) {  // kFolds folds at most per step
    const bool fold = !leaf_hit & !stopped & !pop & (((E.pmask >> (E.idx ^ E.mirror)) & 1u) == 0u) &
                      !esvo_capped(E.iter) & !(E.t_min > max_dst);
#ifdef OCTPT_PROFILE_LANES
    prof_wave(cnt.p_fold_it, cnt.p_fold_ln, fold);
#endif
    if (fold) {
        E.iter += 1u;
        const v3 tf = vsub(vmul(E.pos, E.t_coef), E.t_bias);
        const float tf_max = tmin3(tf);
        const bool fx = tf.x <= tf_max, fy = tf.y <= tf_max, fz = tf.z <= tf_max;
        if (fx) E.pos.x = E.pos.x - E.scale_exp2;
        if (fy) E.pos.y = E.pos.y - E.scale_exp2;
        if (fz) E.pos.z = E.pos.z - E.scale_exp2;
        step_mask = (fx ? 1u : 0u) | (fy ? 2u : 0u) | (fz ? 4u : 0u);
        E.t_min = tf_max;
        E.idx ^= step_mask;
        pop = (E.idx & step_mask) != 0u;
    }
    }
#endif
    bool escaped = false;
#ifdef OCTPT_PROFILE_LANES
    prof_wave(cnt.p_pop_it, cnt.p_pop_ln, pop);
#endif
    if (pop) {  // pop (:262-299)
        // the three axes' differing bits are selected, not branched on (no exec-mask region)
        const uint32_t dx = __float_as_uint(E.pos.x) ^ __float_as_uint(E.pos.x + E.scale_exp2);
        const uint32_t dy = __float_as_uint(E.pos.y) ^ __float_as_uint(E.pos.y + E.scale_exp2);
        const uint32_t dz = __float_as_uint(E.pos.z) ^ __float_as_uint(E.pos.z + E.scale_exp2);
        const uint32_t diff = ((step_mask & 1u) ? dx : 0u) | ((step_mask & 2u) ? dy : 0u) | ((step_mask & 4u) ? dz : 0u);
        // diff != 0: a stepped axis moved by scale_exp2, so its pos differs from pos + scale_exp2
        // (the reference's diff == 0 case, util.rs:121-133, cannot arise here)
        const uint32_t scale_raw = 31u - (uint32_t)__builtin_clz(diff);  // (diff != 0: no zero-input clamp)
        // escaping the root is a miss (:281-283); its lane finishes the block on a clamped scale
        // and reports the miss at the end, so the pop stays one branch level
        const bool esc = scale_raw >= OCTREE_MAX_SCALE;
        const uint32_t scale = min(scale_raw, OCTREE_MAX_SCALE - 1u);
        E.scale_exp2 = __uint_as_float((scale - OCTREE_MAX_SCALE + 127u) << 23);
        // a pop rises above the level it advanced at (the step's own bit, 2^(s-23) in pos's
        // mantissa, always differs, and the pop condition means a higher one does), so
        // scale > base = OCTREE_MAX_SCALE - depth and the entry is in the LDS stack (levels 1..)
        const uint32_t base1 = OCTREE_MAX_SCALE + 1u - S.depth;  // base + 1, wave-uniform
        stk.read(scale - base1, E.parent, E.t_max, E.pmask);
        // pos truncated to the popped scale; idx = pos bits at that scale
        const uint32_t keep = 0xFFFFFFFFu << scale;
        const uint32_t px = __float_as_uint(E.pos.x) & keep, py = __float_as_uint(E.pos.y) & keep,
                       pz = __float_as_uint(E.pos.z) & keep;
        E.pos = V(__uint_as_float(px), __uint_as_float(py), __uint_as_float(pz));
        E.idx = __builtin_amdgcn_ubfe(px, scale, 1u) | (__builtin_amdgcn_ubfe(py, scale, 1u) << 1) |
                (__builtin_amdgcn_ubfe(pz, scale, 1u) << 2);
        // h = 0 after a pop (:298); an escaped lane's h = -1 carries the escape out of the branch, where
        // one compare turns it into a lane mask (a bool assigned in the branch became a VGPR 0/1 and
        // cost a select and an OR at the merge).  The lane finishes here, so its h is never read.
        E.h = esc ? -1.0f : 0.0f;
    }
    escaped = pop & (E.h < 0.0f);
    return leaf_hit ? kStepHit : ((escaped | stopped) ? kStepMiss : kStepContinue);
}

// ---------------------------------------------------------------------------
// sky + sun (scene/mod.rs:216-268, 384-426)
// ---------------------------------------------------------------------------
__device__ inline void sky_color(const DevSun &K, const PathState &r, float out[3]) {
    out[0] = 0.5f; out[1] = 0.7f; out[2] = 1.0f;
    const v3 d = r.d;
    const bool textured = (r.depth == 0u) || r.specular;  // get_sky_color_interp / get_sky_color(true)
    if (textured ? !K.draw_texture : !K.diffuse_sun) return;
    if (vdot(d, V(K.sw[0], K.sw[1], K.sw[2])) < 0.5f) return;
    const float a = PI_F / 2.0f - dm_acos(vdot(d, V(K.su[0], K.su[1], K.su[2]))) + K.width;
    if (!(a >= 0.0f && a < K.width2)) return;
    const float b = PI_F / 2.0f - dm_acos(vdot(d, V(K.sv[0], K.sv[1], K.sv[2]))) + K.width;
    if (!(b >= 0.0f && b < K.width2)) return;
    if (textured) {
        for (int i = 0; i < 3; ++i) out[i] = K.tex[i] * K.isect_mul[i] + out[i];
    } else {
        for (int i = 0; i < 3; ++i) out[i] = (K.tex[i] * K.diffuse_mul[i]) * K.luminosity + out[i];
    }
}

// ---------------------------------------------------------------------------
// scatter kernels (ray/mod.rs:113-373), in place: `r` becomes the next ray
// ---------------------------------------------------------------------------
__device__ inline void specular_reflection(PathState &r, float roughness) {
    const v3 n = r.n, dir = r.d;
    r.col[0] = r.col[1] = r.col[2] = r.col[3] = 0.0f;
    r.cur = r.prev;
    if (roughness > RAY_EPSILON) {
        const float sdot = -2.0f * vdot(dir, n);
        const v3 spec = vadd(vscale(n, sdot), dir);
        const float x1 = rng_next(r.rng), x2 = rng_next(r.rng);
        const float rr = sqrtf(x1), theta = 2.0f * PI_F * x2;
        float sn, cs;
        dm_sincos(theta, sn, cs);
        const float tx = rr * cs, ty = rr * sn, tz = sqrtf(1.0f - x1);
        const v3 tangent = fabsf(n.x) > 0.1f ? V(0.0f, 1.0f, 0.0f) : V(1.0f, 0.0f, 0.0f);
        const v3 u = vnorm(vcross(tangent, n));
        const v3 v = vcross(n, u);
        const v3 nd = vadd(vadd(vscale(u, tx), vscale(v, ty)), vscale(n, tz));
        r.d = vnorm(vadd(vscale(nd, roughness), vscale(spec, 1.0f - roughness)));
    } else {
        r.d = vsub(dir, vscale(n, 2.0f * vdot(dir, n)));
    }
    r.o = vadd(r.o, vscale(r.d, RAY_OFFSET));
    if (signum_(vdot(n, r.d)) == signum_(vdot(n, dir))) {
        const float factor = vdot(n, dir) * -RAY_EPSILON - vdot(r.d, n);
        r.d = vnorm(vadd(r.d, vscale(n, factor)));
    }
}

// returns the factor the importance-sampling branches multiply ray.hit.color by (ray/mod.rs:262,
// 276, 297, 307), 1 when none applies; only the sun-sampling caller uses it [C5]
__device__ inline float diffuse_reflection(const DevSun &K, PathState &r) {
    float w = 1.0f;
    const v3 n = r.n;
    const v3 d_in = r.d;
    r.col[0] = r.col[1] = r.col[2] = r.col[3] = 0.0f;  // new_from_self
    float x1 = rng_next(r.rng), x2 = rng_next(r.rng);
    float rr = sqrtf(x1), theta = 2.0f * PI_F * x2;
    float sn, cs;
    dm_sincos(theta, sn, cs);
    float tx = rr * cs, ty = rr * sn;
    if (K.importance_sampling) {
        const float sdx = K.sun_dx, sdy = K.sun_dy, sdz = K.sun_dz;
        float stx, sty, sq;
        const float stz = (sdx * n.x + sdy * n.y) + sdz * n.z;
        if (fabsf(n.x) > 0.1f) {
            stx = sdx * n.z - sdz * n.x;
            sty = (sdx * n.x * n.y - sdy * (n.x * n.x + n.z * n.z)) + sdz * n.y * n.z;
            sq = dm_hypot(n.x, n.z);
        } else {
            stx = sdz * n.y - sdy * n.z;
            sty = (sdy * n.x * n.y - sdx * (n.y * n.y + n.z * n.z)) + sdz * n.x * n.z;
            sq = dm_hypot(n.z, n.y);
        }
        stx /= sq;
        sty /= sq;
        const float cr = K.circle_radius;
        float chance = K.sample_chance;
        const float alt_rel = dm_asin(stz);
        if (alt_rel + cr > RAY_EPSILON) {
            if ((dm_hypot(stx, sty) + cr) + RAY_EPSILON < 1.0f) {
                if (rng_next(r.rng) < chance) {
                    tx = stx + tx * cr;
                    ty = sty + ty * cr;
                    w = cr * cr / chance;
                } else {
                    while (dm_hypot(tx - stx, ty - sty) < cr) {
                        tx -= stx;
                        ty -= sty;
                        if (tx == 0.0f && ty == 0.0f) break;
                        tx /= cr;
                        ty /= cr;
                    }
                    w = (1.0f - cr * cr) / (1.0f - chance);
                }
            } else {
                const float min_r = dm_cos(alt_rel + cr);
                const float max_r = dm_cos(fmx(alt_rel - cr, 0.0f));
                const float sun_theta = dm_atan2(sty, stx);
                const float seg = ((max_r * max_r - min_r * min_r) * cr) / PI_F;
                chance *= seg / (cr * cr);
                chance = fmn(chance, SUN_MAX_CHANCE);
                if (rng_next(r.rng) < chance) {
                    rr = sqrtf(min_r * min_r * x1 + max_r * max_r * (1.0f - x1));
                    theta = sun_theta + (2.0f * x2 - 1.0f) * cr;
                    w = seg / chance;
                } else {
                    for (;;) {
                        if (!(rr > min_r && rr < max_r)) break;
                        float diff = fabsf(theta - sun_theta);
                        if (diff >= 2.0f * PI_F) diff = diff - 2.0f * PI_F;
                        const float ad = diff > PI_F ? 2.0f * PI_F - diff : diff;
                        if (!(ad < cr)) break;
                        x1 = rng_next(r.rng);
                        x2 = rng_next(r.rng);
                        rr = sqrtf(x1);
                        theta = 2.0f * PI_F * x2;
                    }
                    w = (1.0f - seg) / (1.0f - chance);
                }
                dm_sincos(theta, sn, cs);
                tx = rr * cs;
                ty = rr * sn;
            }
        }
    }
    const float tz = sqrtf((1.0f - tx * tx) - ty * ty);
    float xx, xy, xz;
    if (fabsf(n.x) > 0.1f) { xx = 0.0f; xy = 1.0f; xz = 0.0f; } else { xx = 1.0f; xy = 0.0f; xz = 0.0f; }
    float ux = xy * n.z - xz * n.y, uy = xz * n.x - xx * n.z, uz = xx * n.y - xy * n.x;
    const float inv = 1.0f / sqrtf((ux * ux + uy * uy) + uz * uz);
    ux *= inv; uy *= inv; uz *= inv;
    const float vx = uy * n.z - uz * n.y, vy = uz * n.x - ux * n.z, vz = ux * n.y - uy * n.x;
    r.d = V((ux * tx + vx * ty) + n.x * tz, (uy * tx + vy * ty) + n.y * tz, (uz * tx + vz * ty) + n.z * tz);
    r.o = vadd(r.o, vscale(r.d, RAY_OFFSET));
    r.cur = r.prev;
    r.specular = false;
    if (signum_(vdot(n, r.d)) == signum_(vdot(n, d_in))) {
        const float factor = signum_(vdot(n, d_in)) * -RAY_EPSILON - vdot(r.d, n);
        r.d = vnorm(vadd(r.d, vscale(n, factor)));
    }
    return w;
}

// Sun::get_random_sun_direction (scene/mod.rs:427-445): (u + v) + normalize(w), not normalised
__device__ inline v3 random_sun_direction(const DevSun &K, uint32_t &rng) {
    const float x1 = rng_next(rng), x2 = rng_next(rng);
    const float cos_a = (1.0f - x1) + x1 * K.radius_cos;
    const float sin_a = sqrtf(1.0f - cos_a * cos_a);
    const float phi = 2.0f * PI_F * x2;
    float sn, cs;
    dm_sincos(phi, sn, cs);
    const v3 u = vscale(V(K.su[0], K.su[1], K.su[2]), cs * sin_a);
    const v3 v = vscale(V(K.sv[0], K.sv[1], K.sv[2]), sn * sin_a);
    const v3 w = vscale(V(K.sw[0], K.sw[1], K.sw[2]), cos_a);
    return vadd(vadd(u, v), vnorm(w));
}

// ---------------------------------------------------------------------------
// path logic shared by the megakernel and the wavefront shade kernel
// ---------------------------------------------------------------------------
// camera ray + fresh path (camera.rs:77-86, tile_renderer.rs:695-703)
__device__ inline void new_path(const DevCamera &C, const DevRender &R, uint32_t x, uint32_t y, uint32_t sample,
                                PathState &ps) {
    ps.rng = path_state(R.seed, y * R.W + x, sample);
    const float jlo = R.jlo, jhi = R.jhi;  // -1 / dim, 1 / dim (make_render)
    const float xn = ((float)(2u * x + 1u) - (float)R.W) / R.dim;
    const float yn = ((float)(2u * (R.H - y) - 1u) - (float)R.H) / R.dim;
    const float dx = jlo + (jhi - jlo) * rng_next(ps.rng);
    const float dy = jlo + (jhi - jlo) * rng_next(ps.rng);
    const v3 nd = vadd(vadd(vscale(V(C.dir[0], C.dir[1], C.dir[2]), C.d_factor),
                            vscale(V(C.right[0], C.right[1], C.right[2]), xn + dx)),
                       vscale(V(C.up[0], C.up[1], C.up[2]), yn + dy));
    ps.o = V(C.eye[0], C.eye[1], C.eye[2]);
    ps.d = vnorm(nd);
    ps.n = V(0.0f, 0.0f, 0.0f);
    ps.col[0] = ps.col[1] = ps.col[2] = ps.col[3] = 0.0f;
    ps.T = V(1.0f, 1.0f, 1.0f);
    ps.L = V(0.0f, 0.0f, 0.0f);
    ps.cur = ps.prev = ps.depth = 0u;
    ps.last_prim = kPrimNone;
    ps.path_segs = 0u;
    ps.specular = true;
    ps.shadow = false;
    ps.branch = 0u;
    ps.seg_base = 0u;
    ps.beam = 0.0f;
}

// next_intersection prologue (path_tracer.rs:438-446) + Scene::hit direction guard
// (scene/mod.rs:175-179) + the per-path segment cap [C15]. false = the path ends here.
__device__ __forceinline__ bool begin_segment(PathState &ps) {
    if (ps.path_segs >= MAX_PATH_SEGMENTS) return false;
    ps.path_segs++;
    ps.prev = ps.cur;
    const v3 d = ps.d;
    if ((d.x == 0.0f && d.y == 0.0f && d.z == 0.0f) || isnan(d.x) || isnan(d.y) || isnan(d.z))
        ps.d = V(0.0f, 1.0f, 0.0f);
    return true;
}

__device__ __forceinline__ TraceRay trace_ray_of(const DevScene &S, const PathState &ps) {
    return make_trace_ray(S, ps.o, ps.d, ps.last_prim, vdot(ps.d, ps.n) < 0.0f);
}

// get_direct_light_attenuation (path_tracer.rs:458-483) after one shadow segment: attenuate by the
// hit's colour and alpha; while light passes, the next shadow segment starts `OFFSET` past the hit.
// Once it is blocked or escapes, add the sun's direct light and resume the waiting diffuse bounce.
__device__ inline void shadow_segment_done(const DevScene &S, PathState &ray, bool hit) {
    if (hit) {
        const float m = 1.0f - ray.col[3];
        for (int i = 0; i < 3; ++i) ray.att[i] *= ray.col[i] * ray.col[3] + m;
        ray.att[3] *= m;
        if (S.sun.strict_direct_light && S.mats[ray.prev].ior != S.mats[ray.cur].ior) ray.att[3] = 0.0f;
        if (ray.att[3] > 0.0f) {
            ray.o = vadd(ray.o, vscale(ray.d, RAY_OFFSET));
            return;
        }
    }
    if (ray.att[3] > 0.0f) {
        const float *e = S.sun.emit;
        v3 &L = ray.L;
        const v3 T = ray.T;
        L = V(L.x + T.x * (((ray.att[0] * ray.att[3]) * ray.mult) * e[0]),
              L.y + T.y * (((ray.att[1] * ray.att[3]) * ray.mult) * e[1]),
              L.z + T.z * (((ray.att[2] * ray.att[3]) * ray.mult) * e[2]));
    }
    ray.shadow = false;
    ray.o = ray.co;
    ray.d = ray.cd;
    ray.n = ray.cn;
    ray.last_prim = ray.clast;
    ray.cur = ray.ccur;
}

// path_tracer.rs:15-135 in forward-throughput form, from a finished segment to either the
// next segment's ray (returns true) or the end of the path (returns false).  kNee: the scene may
// sample the sun; shadow segments run between a diffuse hit and its bounce.
// kLean: the lean path state's chunks (no emitting material, no branch schedule: enqueue_wavefront's lean rule), whose
// instances carry neither the emission term nor the first reflection's split
template <bool kNee, bool kLean = false>
__device__ inline bool shade_segment(const DevScene &S, const DevRender &R, PathState &ray, bool hit,
                                     Counters &cnt) {
    if (kNee && ray.shadow) {
        shadow_segment_done(S, ray, hit);
        return true;
    }
    if (!hit) {
        float sky[3];
        sky_color(S.sun, ray, sky);
        ray.L = V(ray.L.x + ray.T.x * sky[0], ray.L.y + ray.T.y * sky[1], ray.L.z + ray.T.z * sky[2]);
        return false;
    }
    const DevMaterial m = S.mats[ray.cur];
    const float ior2 = S.mats[ray.prev].ior;
    const float specular = m.specular, diffuse = ray.col[3], absorb = ray.col[3];
    const float ior1 = m.ior;
    if (ray.col[3] + specular < RAY_EPSILON && ior1 == ior2) {  // [C4]
        ray.o = vadd(ray.o, vscale(ray.d, RAY_OFFSET));
        return true;
    }
    if (ray.depth + 1u >= R.max_depth) return false;
    ray.depth += 1u;
    if (!(OCTPT_LEAN_STRICT && kLean) && ray.depth == 1u && ray.branch != 0u) {  // the first reflection splits [C20]
        ray.rng = branch_state(ray.rng, ray.branch);
        ray.seg_base = ray.path_segs;
    }
    cnt.shade++;
    v3 &T = ray.T;
    const float metal = m.metalness;
    const bool do_metal = metal > RAY_EPSILON && rng_next(ray.rng) < metal;
    if (do_metal || (specular > RAY_EPSILON && rng_next(ray.rng) < specular)) {
        if (do_metal) T = V(T.x * ray.col[0], T.y * ray.col[1], T.z * ray.col[2]);
        specular_reflection(ray, m.roughness);
    } else if (rng_next(ray.rng) < diffuse) {
        if (!(OCTPT_LEAN_STRICT && kLean) && S.emitters && m.emittance > RAY_EPSILON) {
            const v3 e = V(ray.col[0] * ray.col[0] * m.emittance, ray.col[1] * ray.col[1] * m.emittance,
                           ray.col[2] * ray.col[2] * m.emittance);
            ray.L = V(ray.L.x + T.x * e.x, ray.L.y + T.y * e.y, ray.L.z + T.z * e.z);
        }
        if (kNee && S.sun.sun_sampling) {
            // do_diffuse_reflection's sun-sampling branch (path_tracer.rs:225-291).  Draw order:
            // sun direction, subsurface chance, then the bounce; the shadow loop draws nothing,
            // so the bounce is drawn now and waits while its shadow segments run
            const v3 n = ray.n;
            const v3 sd = random_sun_direction(S.sun, ray.rng);
            const bool front = vdot(sd, n) > 0.0f;
            const bool cast = front || ((m.flags & MAT_FLAG_SUBSURFACE) && rng_next(ray.rng) < S.sun.f_sub_surface);
            const v3 so = front ? ray.o : vadd(ray.o, vscale(n, -RAY_OFFSET));
            const uint32_t scur = ray.prev;
            const float mult = fabsf(vdot(sd, n)) * S.sun.lum_a;
            const float c0 = ray.col[0], c1 = ray.col[1], c2 = ray.col[2];
            const float w = diffuse_reflection(S.sun, ray);
            T = V(T.x * (c0 * w), T.y * (c1 * w), T.z * (c2 * w));
            if (cast) {
                ray.co = ray.o;
                ray.cd = ray.d;
                ray.cn = n;
                ray.clast = ray.last_prim;
                ray.ccur = ray.cur;
                ray.mult = mult;
                ray.att[0] = ray.att[1] = ray.att[2] = ray.att[3] = 1.0f;
                ray.shadow = true;
                ray.o = vadd(so, vscale(sd, RAY_OFFSET));
                ray.d = sd;
                ray.n = n;
                ray.cur = scur;
            }
            return true;
        }
        T = V(T.x * ray.col[0], T.y * ray.col[1], T.z * ray.col[2]);
        diffuse_reflection(S.sun, ray);
    } else if (fabsf(ior1 - ior2) >= RAY_EPSILON) {
        // do_refraction (path_tracer.rs:318-401) [C14]
        const bool refr = (m.flags & MAT_FLAG_REFRACTIVE) != 0u;
        const float n1n2 = ior1 / ior2;
        const float cos_theta = -vdot(ray.d, ray.n);
        const float radicand = 1.0f - n1n2 * n1n2 * (1.0f - cos_theta * cos_theta);
        if (refr && radicand < RAY_EPSILON) {
            specular_reflection(ray, m.roughness);
        } else {
            const float a = n1n2 - 1.0f, b = n1n2 + 1.0f;
            const float r0 = a * a / (b * b);
            const float cc = 1.0f - cos_theta;
            const float c5 = ((cc * cc) * (cc * cc)) * cc;
            const float rtheta = r0 + (1.0f - r0) * c5;
            if (rng_next(ray.rng) < rtheta) {
                specular_reflection(ray, m.roughness);
            } else {
                T = V(T.x * (ray.col[0] * absorb), T.y * (ray.col[1] * absorb), T.z * (ray.col[2] * absorb));
                const v3 d_in = ray.d, n = ray.n;
                ray.col[0] = ray.col[1] = ray.col[2] = ray.col[3] = 0.0f;
                if (refr) {
                    const float t2 = sqrtf(radicand);
                    v3 d;
                    if (cos_theta > 0.0f) d = vadd(vscale(d_in, n1n2), vscale(n, n1n2 * cos_theta - t2));
                    else d = vsub(vscale(d_in, n1n2), vscale(n, -n1n2 * cos_theta - t2));
                    ray.d = vnorm(d);
                    if (signum_(vdot(n, ray.d)) != signum_(vdot(n, d_in))) {
                        const float factor = signum_(vdot(n, d_in)) * -RAY_EPSILON - vdot(ray.d, n);
                        ray.d = vnorm(vadd(ray.d, vscale(n, factor)));
                    }
                    ray.o = vadd(ray.o, vscale(ray.d, RAY_OFFSET));
                }
            }
        }
    } else {
        // do_transmission (path_tracer.rs:403-422)
        T = V(T.x * (ray.col[0] * absorb), T.y * (ray.col[1] * absorb), T.z * (ray.col[2] * absorb));
        ray.col[0] = ray.col[1] = ray.col[2] = ray.col[3] = 0.0f;
        ray.o = vadd(ray.o, vscale(ray.d, RAY_OFFSET));
    }
    return true;
}

// running mean of render_tile_average (tile_renderer.rs:707-733): a sample of weight bc
__device__ __forceinline__ void running_mean(float4 &fb, v3 c, uint32_t spp, uint32_t bc) {
    const float s_inv = 1.0f / (float)(bc + spp);
    const float fs = (float)spp, w = (float)bc;
    fb.x = (fb.x * fs + c.x * w) * s_inv;
    fb.y = (fb.y * fs + c.y * w) * s_inv;
    fb.z = (fb.z * fs + c.z * w) * s_inv;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// kFastDiv: the tile row by udiv_c (the seed, resolve and beam kernels); false: the plain division, which the shade
// kernel's first-launch path keeps (its allocation is sensitive to that path's shape: the fast form measured shade +7 %)
template <bool kFastDiv = true>
__device__ __forceinline__ void item_pixel(const DevRender &R, uint32_t item, uint32_t &x, uint32_t &y) {
    const uint32_t lt = item >> 6, w = item & 63u;
    const uint32_t t = dealt_tile(R.tile_order, R.shard_index + lt * R.shard_count);
    const uint32_t ty = kFastDiv ? udiv_c(t, R.div_tiles_x) : t / R.tiles_x;
    x = (t - ty * R.tiles_x) * kTile + (w & 7u);
    y = ty * kTile + (w >> 3);
}

__device__ inline unsigned long long wave_sum(uint32_t v) {
    unsigned long long s = v;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    return s;
}

// row_base: 0, or kStatDrainRow for the drain kernel (its share is reported apart, octpt_stats::drain)
__device__ inline void flush_counters(const Counters &cnt, unsigned long long *stats, uint32_t row_base = 0u) {
#ifdef OCTPT_NO_STATS  // A/B builds only: every counter update becomes dead code
    return;
#endif
#ifdef OCTPT_PROFILE_LANES
    constexpr int kN = 12 + 13;  // profile words from 12 on (octpt_get_stats prints them)
    const uint32_t vals[kN] = {cnt.paths, cnt.segs, cnt.steps, cnt.sph, cnt.cub, cnt.shade, cnt.tex, cnt.blk, cnt.ib,
                               0u, 0u, 0u,
                               cnt.p_iters, cnt.p_active, cnt.p_leaf_it, cnt.p_leaf_ln, cnt.p_pop_it, cnt.p_pop_ln,
                               cnt.p_push_it, cnt.p_desc_ln, cnt.p_exact, cnt.p_fold_it, cnt.p_fold_ln,
                               cnt.p_dfold_it, cnt.p_dfold_ln};
#else
    constexpr int kN = kStatCount;
    const uint32_t vals[kN] = {cnt.paths, cnt.segs, cnt.steps, cnt.sph, cnt.cub, cnt.shade, cnt.tex, cnt.blk, cnt.ib};
#endif
    // a counter no lane of the wave touched costs one ballot, not a 64-lane reduction: the non-persistent kernels
    // (seed, preview) flush once per wave and touch one or two of the counters
#pragma unroll
    for (int i = 0; i < kN; ++i) {
        if (__ballot(vals[i] != 0u) == 0ull) continue;
        const unsigned long long s = wave_sum(vals[i]);
        if ((threadIdx.x & 63u) == 0u && s)
            atomicAdd(&stats[(row_base + blockIdx.x % kSegs) * kStatRow + i], s);
    }
    if (__ballot(cnt.redo != 0u) == 0ull) return;
    const unsigned long long r = wave_sum(cnt.redo);
    if ((threadIdx.x & 63u) == 0u && r) atomicAdd(&stats[(row_base + blockIdx.x % kSegs) * kStatRow + kStatBeamRestartWord], r);
}

// wave-aggregated atomic ticket: each lane with `want` gets a distinct value from *ctr
__device__ __forceinline__ uint32_t wave_ticket(uint32_t *ctr, bool want) {
    const uint64_t m = __ballot(want);
    if (m == 0ull) return 0u;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    uint32_t base = 0u;
    if ((threadIdx.x & 63u) == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    return base + lanes_below(m);
}

// ===========================================================================
// megakernel (kept for A/B: OCTPT_RENDER_MEGAKERNEL)
// ===========================================================================
enum : uint32_t { ST_IDLE = 0, ST_NEWPATH, ST_BEGIN, ST_TRAV, ST_HIT, ST_MISS, ST_FINISH, ST_DONE };

template <bool kNee, int kPrims>
__global__ __launch_bounds__(kBlock) void render_kernel(DevScene S, DevCamera C, DevRender R, float4 *__restrict__ accum,
                                                        uint32_t *__restrict__ segcount, uint32_t *__restrict__ counter,
                                                        unsigned long long *__restrict__ stats) {
    extern __shared__ uint2 lds_stack[];
    const Stack stk = stack_of(lds_stack, S.depth);
    uint32_t state = ST_IDLE;
    uint32_t pix = 0u, k = 0u, pix_segs = 0u, acc_idx = 0u;
    float4 fb = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    PathState ray;
    TraceRay tr;
    Esvo E;
    uint32_t hprim = kPrimNone;
    PrimHit hh;
    Counters cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};

    for (;;) {
        const bool need = state == ST_IDLE;
        if (__ballot(need)) {
            const uint32_t my = wave_ticket(counter, need);
            if (need) {
                if (my >= R.total_items) {
                    state = ST_DONE;
                } else {
                    uint32_t x, y;
                    item_pixel(R, my, x, y);
                    if (x < R.W && y < R.H) {
                        pix = y * R.W + x;
                        acc_idx = R.compact ? my : pix;
                        fb = accum[acc_idx];
                        k = 0u;
                        pix_segs = 0u;
                        state = ST_NEWPATH;
                    }
                }
            }
        }
        if (__ballot(state != ST_DONE) == 0ull) break;
        if (state == ST_NEWPATH) {
            new_path(C, R, pix % R.W, pix / R.W, R.spp_start + k, ray);
            cnt.paths++;
            state = ST_BEGIN;
        }
        if (state == ST_BEGIN) {
            if (begin_segment(ray)) {
                tr = trace_ray_of(S, ray);
                esvo_begin(S, tr, E, stk);
                cnt.segs++;
                pix_segs++;
                state = ST_TRAV;
            } else {
                state = ST_FINISH;
            }
        }
        bool first = true;
        for (;;) {  // keep stepping while at least half of the live lanes traverse
            const uint64_t tm = __ballot(state == ST_TRAV);
            if (tm == 0ull) break;
            if (!first) {
                const uint64_t am = __ballot(state != ST_DONE);
                if (2u * (uint32_t)__popcll(tm) < (uint32_t)__popcll(am)) break;
            }
            first = false;
            if (state == ST_TRAV) {
                const int rs = esvo_step<kPrims>(S, tr, E, stk, cnt, hprim, hh);
                if (rs == kStepHit) state = ST_HIT;
                else if (rs == kStepMiss) state = ST_MISS;
                if (rs != kStepContinue) cnt.steps += E.iter;
            }
        }
        if (state == ST_HIT || state == ST_MISS || state == ST_FINISH) {
            bool cont = false;
            if (state != ST_FINISH) {
                if (state == ST_HIT) commit_hit(S, ray, hprim, hh, cnt);
                cont = shade_segment<kNee>(S, R, ray, state == ST_HIT, cnt);
            }
            if (cont) {
                state = ST_BEGIN;
            } else {
                running_mean(fb, ray.L, R.spp_start + k, 1u);
                k++;
                if (k < R.spp_count) {
                    state = ST_NEWPATH;
                } else {
                    accum[acc_idx] = fb;
                    if (segcount) segcount[acc_idx] += pix_segs;
                    state = ST_IDLE;
                }
            }
        }
    }
    cnt.ib = 0u;  // issued bytes are extend's only
    flush_counters(cnt, stats);
}

// ===========================================================================
// RendererMode::Preview: render_tile_replace (tile_renderer.rs:648-682) +
// preview_render (path_tracer.rs:137-158).  One un-jittered camera ray per pixel, continued
// through material-0 and transparent hits (next_intersection_preview, :447-455), then sky + sun on
// material 0 or Sun::flat_shading (scene/mod.rs:447-452).  Coherent primary rays: one thread per
// pixel in 8x8 tiles (one tile per wave), no queues.
// ===========================================================================
#ifndef OCTPT_PREVIEW_BOUNDS
#define OCTPT_PREVIEW_BOUNDS 1
#endif
// one wave per SIMD above the natural allocation (78 / 86 / 102 VGPRs -> 72 / 80 / 96), as for extend
#define OCTPT_PREVIEW_WAVES_OF(k) \
    (OCTPT_PREVIEW_BOUNDS ? ((k) == kPrimsSpheres ? 7 : ((k) == kPrimsBoxes || (k) == kPrimsBlocks) ? 6 : 5) : 1)
template <int kPrims>
__global__ __launch_bounds__(kBlock, OCTPT_PREVIEW_WAVES_OF(kPrims)) void preview_kernel(DevScene S, DevCamera C, DevRender R,
                                                         float4 *__restrict__ accum, uint32_t *__restrict__ segcount,
                                                         unsigned long long *__restrict__ stats) {
    extern __shared__ uint2 lds_stack[];
    const Stack stk = stack_of(lds_stack, S.depth);
    Counters cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    const uint32_t item = blockIdx.x * kBlock + threadIdx.x;
    uint32_t x = 0u, y = 0u;
    if (item < R.total_items) item_pixel(R, item, x, y);
    if (item < R.total_items && x < R.W && y < R.H) {
        const uint32_t pix = y * R.W + x;
        PathState ps;
        // Camera::get_ray at the pixel centre (camera.rs:77-86), no jitter
        const float xn = ((float)(2u * x + 1u) - (float)R.W) / R.dim;
        const float yn = ((float)(2u * (R.H - y) - 1u) - (float)R.H) / R.dim;
        const v3 nd = vadd(vadd(vscale(V(C.dir[0], C.dir[1], C.dir[2]), C.d_factor),
                                vscale(V(C.right[0], C.right[1], C.right[2]), xn)),
                           vscale(V(C.up[0], C.up[1], C.up[2]), yn));
        ps.o = V(C.eye[0], C.eye[1], C.eye[2]);
        ps.d = vnorm(nd);
        ps.n = V(0.0f, 0.0f, 0.0f);
        ps.col[0] = ps.col[1] = ps.col[2] = ps.col[3] = 0.0f;
        ps.T = V(1.0f, 1.0f, 1.0f);
        ps.L = V(0.0f, 0.0f, 0.0f);
        ps.cur = ps.prev = ps.depth = 0u;
        ps.rng = 0u;
        ps.last_prim = kPrimNone;
        ps.path_segs = 0u;
        ps.specular = true;
        cnt.paths++;
        uint32_t pix_segs = 0u;
        while (begin_segment(ps)) {  // [C15] bounds the pass-through chain
            cnt.segs++;
            pix_segs++;
            const TraceRay tr = trace_ray_of(S, ps);
            Esvo E;
            esvo_begin(S, tr, E, stk);
            uint32_t prim = kPrimNone;
            PrimHit h;
            int rs;
            do {
                rs = esvo_step<kPrims>(S, tr, E, stk, cnt, prim, h);
            } while (rs == kStepContinue);
            cnt.steps += E.iter;
            if (rs != kStepHit) break;  // a miss leaves the last hit record in place
            commit_hit(S, ps, prim, h, cnt);
            if (ps.cur != 0u && ps.col[3] > 0.0f) break;
            ps.o = vadd(ps.o, vscale(ps.d, RAY_OFFSET));
        }
        float out[3];
        if (ps.cur == 0u) {
            sky_color(S.sun, ps, out);  // depth 0: get_sky_color_inner + add_sun_color
        } else {
            const float shading = fmaxf(0.3f, vdot(ps.n, V(S.sun.sw[0], S.sun.sw[1], S.sun.sw[2])));  // AMBIENT
            for (int i = 0; i < 3; ++i) out[i] = ps.col[i] * (S.sun.emit[i] * shading);
        }
        const uint32_t ai = R.compact ? item : pix;
        float4 fb = accum[ai];
        fb.x = out[0];
        fb.y = out[1];
        fb.z = out[2];
        accum[ai] = fb;
        if (segcount) segcount[ai] += pix_segs;
    }
    cnt.ib = 0u;  // issued bytes are extend's only
    flush_counters(cnt, stats);
}

// ===========================================================================
// wavefront path tracer: seed -> (extend -> shade)* -> resolve
// ===========================================================================
// Records (16 bytes each).  Ray records live at their queue position, so extend reads them
// without an indirection; the path state lives at its slot:
//   ray0[q][i] = (o.xyz, last_prim)   ray1[q][i] = (d.xyz, slot | self_inward << 31)
//   hit[i]     = (prim, t, inside | axis<<1 | (nsgn<0)<<3, -)
//   pa[slot]   = (T.xyz, L.x)  pb[slot] = (L.y, L.z, rng, item)  pc[slot] = (cur_mat, depth | spec<<8 | segs<<16)
//   a camera ray with a beam start: ray1 bit 30 set, ray0.w = the start t (its last_prim is kPrimNone)
constexpr uint32_t kRayBeamBit = 0x40000000u;  // slots < 2^30 (the pool cap)
// a miss record's second word for a ray that ended on the reference's step cap: for a beam-started camera
// ray (its record's kRayBeamBit) shade queues the same ray again without its start (the walk from the cube
// entry), no segment counted; any other such ray is the reference's miss
constexpr uint32_t kHitCapped = 1u;
__device__ __forceinline__ void store_ray(const WaveBuffers &B, uint32_t q, uint32_t pos, uint32_t slot,
                                          const PathState &ps) {
    const bool beam = ps.beam > 0.0f && ps.path_segs == 1u;
    B.ray0[q][pos] = make_float4(ps.o.x, ps.o.y, ps.o.z, beam ? ps.beam : __uint_as_float(ps.last_prim));
    B.ray1[q][pos] = make_float4(ps.d.x, ps.d.y, ps.d.z,
                                 __uint_as_float(slot | (vdot(ps.d, ps.n) < 0.0f ? 0x80000000u : 0u) |
                                                 (beam ? kRayBeamBit : 0u)));
}
// The seed's camera rays when every chunk item has its pixel (direct seeding, OCTPT_CAM_RECORDS): 16 B, ray1
// alone as (d, the beam start or 0); the origin is the eye, the last primitive none, and the slot the item, which
// the position gives (shard_lo(segment) + index in it).  8.5 GB less written by the seed and read by the first
// extend per C3 frame.  cam_ray turns one into store_ray's two records in registers.
__device__ __forceinline__ void store_cam_ray(const WaveBuffers &B, uint32_t pos, const PathState &ps) {
    B.ray1[0][pos] = make_float4(ps.d.x, ps.d.y, ps.d.z, ps.beam > 0.0f ? ps.beam : 0.0f);
}
__device__ __forceinline__ void cam_ray(float4 eye, uint32_t slot, float4 &r0, float4 &r1) {
    const float b = r1.w;
    r0 = make_float4(eye.x, eye.y, eye.z, b > 0.0f ? b : eye.w);  // eye.w: kPrimNone (WaveBuffers::eye)
    r1.w = __uint_as_float(slot | (b > 0.0f ? kRayBeamBit : 0u));
}
// a ray record's last primitive and beam start
__device__ __forceinline__ uint32_t ray_last_prim(float4 r0, float4 r1) {
    return (__float_as_uint(r1.w) & kRayBeamBit) ? kPrimNone : __float_as_uint(r0.w);
}
__device__ __forceinline__ float ray_beam(float4 r0, float4 r1) {
    return (__float_as_uint(r1.w) & kRayBeamBit) ? r0.w : 0.0f;
}

__device__ __forceinline__ void pack_path(const PathState &ps, uint32_t item, float4 &a, float4 &b, uint2 &c) {
    a = make_float4(ps.T.x, ps.T.y, ps.T.z, ps.L.x);
    b = make_float4(ps.L.y, ps.L.z, __uint_as_float(ps.rng), __uint_as_float(item));
    c = make_uint2(ps.cur, ps.depth | (ps.specular ? 1u << 8 : 0u) | (ps.shadow ? 1u << 9 : 0u) | (ps.branch << 10) |
                               (ps.path_segs << 16) | (ps.seg_base << 23));
}
// kLean (WaveBuffers::lean): the 24-B path state (T, rng) + (cur, bits).  The radiance L of a
// path that continues is exactly 0 when the scene has no emitters and no sun sampling (it is added only at the
// path's end, sky on a miss), and its item equals its slot when the pool holds the chunk (the direct seeding):
// neither is stored, 16 B less written and read per segment.
template <bool kLean = false>
__device__ __forceinline__ void store_path(const WaveBuffers &B, uint32_t slot, const PathState &ps, uint32_t item) {
    float4 a, b;
    uint2 c;
    pack_path(ps, item, a, b, c);
    if (kLean) {
        B.pa[slot] = make_float4(a.x, a.y, a.z, b.z);  // (T, rng)
        B.pc[slot] = c;
        return;
    }
    B.pa[slot] = a;
    B.pb[slot] = b;
    B.pc[slot] = c;
}

// The lean state travels with its ray (OCTPT_LEAN_POS, round 5): shade stores it at the continuing ray's queue
// position (queue q: (T, rng) in pa for q = 0, pb for q = 1 -- pb is free in the lean state -- and (cur, bits) in
// pc's half q), so the next shade reads it at the position it reads the ray and hit records at, coalesced and
// without waiting for the ray record's slot word.
#ifndef OCTPT_LEAN_POS
#define OCTPT_LEAN_POS 1
#endif
__device__ __forceinline__ void store_lean_at(const WaveBuffers &B, uint32_t q, uint32_t pos, const PathState &ps) {
    float4 a, b;
    uint2 c;
    pack_path(ps, 0u, a, b, c);
    (q ? B.pb : B.pa)[pos] = make_float4(a.x, a.y, a.z, b.z);
    B.pc[(size_t)q * kSegs * B.seg_cap + pos] = c;
}

// sun-sampling state of a slot (kNee): the waiting bounce + mult, and the attenuation
__device__ __forceinline__ void store_nee(const WaveBuffers &B, uint32_t slot, const PathState &ps) {
    B.pd[slot] = make_float4(ps.co.x, ps.co.y, ps.co.z, __uint_as_float(ps.clast));
    B.pd[B.pool + slot] = make_float4(ps.cd.x, ps.cd.y, ps.cd.z, __uint_as_float(ps.ccur));
    B.pd[2u * B.pool + slot] = make_float4(ps.cn.x, ps.cn.y, ps.cn.z, ps.mult);
}
__device__ __forceinline__ void store_att(const WaveBuffers &B, uint32_t slot, const PathState &ps) {
    B.pd[3u * B.pool + slot] = make_float4(ps.att[0], ps.att[1], ps.att[2], ps.att[3]);
}
__device__ __forceinline__ void load_nee(const WaveBuffers &B, uint32_t slot, PathState &ps) {
    const float4 a = B.pd[slot], b = B.pd[B.pool + slot], c = B.pd[2u * B.pool + slot], d = B.pd[3u * B.pool + slot];
    ps.co = V(a.x, a.y, a.z);
    ps.clast = __float_as_uint(a.w);
    ps.cd = V(b.x, b.y, b.z);
    ps.ccur = __float_as_uint(b.w);
    ps.cn = V(c.x, c.y, c.z);
    ps.mult = c.w;
    ps.att[0] = d.x; ps.att[1] = d.y; ps.att[2] = d.z; ps.att[3] = d.w;
}

__device__ __forceinline__ void unpack_path(float4 a, float4 b, uint2 c, float4 r0, float4 r1, PathState &ps,
                                            uint32_t &item) {
    ps.o = V(r0.x, r0.y, r0.z);
    ps.last_prim = ray_last_prim(r0, r1);
    ps.d = V(r1.x, r1.y, r1.z);
    ps.beam = 0.0f;
    ps.T = V(a.x, a.y, a.z);
    ps.L = V(a.w, b.x, b.y);
    ps.rng = __float_as_uint(b.z);
    item = __float_as_uint(b.w);
    ps.cur = c.x;
    ps.prev = c.x;  // begin_segment set prev = cur before this segment was traced
    ps.depth = c.y & 255u;
    ps.specular = (c.y >> 8) & 1u;
    ps.shadow = (c.y >> 9) & 1u;
    ps.branch = (c.y >> 10) & 63u;
    ps.path_segs = (c.y >> 16) & 127u;
    ps.seg_base = c.y >> 23;
}
template <bool kLean = false>
__device__ __forceinline__ void load_path(const WaveBuffers &B, uint32_t slot, float4 r0, float4 r1, PathState &ps,
                                          uint32_t &item) {
    if (kLean) {  // L = +0 as the path started, item = slot (store_path<true>)
        const float4 a = B.pa[slot];
        unpack_path(make_float4(a.x, a.y, a.z, 0.0f), make_float4(0.0f, 0.0f, a.w, __uint_as_float(slot)), B.pc[slot],
                    r0, r1, ps, item);
        return;
    }
    unpack_path(B.pa[slot], B.pb[slot], B.pc[slot], r0, r1, ps, item);
}

// the path of chunk item `item`, its first segment begun; false when the pixel lies outside the image
template <bool kFastDiv = true>
__device__ __forceinline__ bool item_path(const DevCamera &C, const DevRender &R, uint32_t item, PathState &ps,
                                          uint32_t &x, uint32_t &y) {
    const uint32_t s_local = kFastDiv ? udiv_c(item, R.div_items) : item / R.total_items;
    const uint32_t px_item = item - s_local * R.total_items;
    item_pixel<kFastDiv>(R, px_item, x, y);
    if (x >= R.W || y >= R.H) return false;
    uint32_t sample = R.spp_start + s_local, branch = 0u;
    if (R.subs) {  // branch schedule (C20): the pass's sample key and this item's branch
        const uint2 sb = R.subs[s_local];
        sample = sb.x;
        branch = sb.y >> 16;
    }
    new_path(C, R, x, y, sample, ps);
    ps.branch = branch;
    begin_segment(ps);  // first segment: never capped
    return true;
}

// generate the path of chunk item `item` into `slot`; false when the pixel lies outside the image.
// kSeed (wf_seed_kernel): only the item is stored (item0); the chunk's first shade rebuilds the path
// state from it (shade_lane) instead of reading 40 B per slot that the seed would have written.
template <bool kSeed = false>
__device__ inline bool seed_item(const DevCamera &C, const DevRender &R, const WaveBuffers &B, uint32_t slot,
                                 uint32_t item, PathState &ps, Counters &cnt) {
    uint32_t x, y;
    if (!item_path(C, R, item, ps, x, y)) {
        B.color[item] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        return false;
    }
    cnt.paths++;
    if (R.beam)  // the camera ray's beam start (its tile's, beam_kernel)
        ps.beam = R.beam[(y / kBeamTile) * R.beam_tx + x / kBeamTile];
    if (kSeed) {
        if (!B.lean) B.item0[slot] = item;  // lean: the chunk's first shade takes item = slot
    } else {
        store_path(B, slot, ps, item);
    }
    return true;
}

static_assert(kSegs == 64, "segment scans give one wave lane per segment");

__device__ __forceinline__ uint32_t relaxed_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// chunk item shard k = [shard_lo(k), shard_lo(k + 1))
__device__ __forceinline__ uint32_t shard_lo(uint32_t k, uint32_t n) {
    return (uint32_t)(((uint64_t)k * n) / kSegs);
}
// first set bit of m at or after bit `from`, cyclically; m != 0
__device__ __forceinline__ uint32_t first_from(uint64_t m, uint32_t from) {
    const uint64_t r = from ? ((m >> from) | (m << (64u - from))) : m;
    return (from + (uint32_t)__ffsll((unsigned long long)r) - 1u) & 63u;
}

// Item claims of one wave: the shard it is drawing from and whether any shard has items left
// (both wave-uniform).
struct ItemCursor {
    uint32_t k;
    bool left;
};

// lanes with `want` start the next chunk items in their slots.  The wave draws from shard
// cur.k; when that runs dry, one relaxed load per lane (lane j = shard j) finds the next shard
// with items left.  Items whose pixel lies outside the image are consumed (zero colour) and the
// lane draws again, so a slot only goes idle once every shard is exhausted.  Every lane of the
// wave must call this.
template <bool kSeed = false>
__device__ inline bool regen(const DevCamera &C, const DevRender &R, const WaveBuffers &B, uint32_t slot, bool want,
                             uint32_t chunk_items, ItemCursor &cur, PathState &ps, Counters &cnt) {
    bool need = want, ok = false;
    while (cur.left && __ballot(need) != 0ull) {
        const uint32_t lo = shard_lo(cur.k, chunk_items), n = shard_lo(cur.k + 1u, chunk_items) - lo;
        const uint32_t t = wave_ticket(B.ctrl + ctr_item(cur.k), need);
        bool dry = false;
        if (need) {
            if (t >= n) dry = true;
            else if (seed_item<kSeed>(C, R, B, slot, lo + t, ps, cnt)) { ok = true; need = false; }
        }
        if (__ballot(dry) != 0ull) {
            const uint32_t j = threadIdx.x & 63u;
            const bool has = relaxed_load(B.ctrl + ctr_item(j)) < shard_lo(j + 1u, chunk_items) - shard_lo(j, chunk_items);
            const uint64_t m = __ballot(has);
            cur.left = m != 0ull;
            if (cur.left) cur.k = first_from(m, cur.k);
        }
    }
    return ok;
}

// seed: wave w appends to queue 0 segment w % kSegs, which holds at most seg_cap rays
// (seg_cap = ceil(ceil(pool / 64) / kSegs) * 64).  When the pool holds the whole chunk
// (n_seed == chunk_items: C3's frame, every 4K chunk) the waves of segment k take shard k's items
// in order, item = slot (no item-claim atomics; block 0 marks every shard claimed; the grid is
// launch_wf_seed's kSegs * ceil(shard / 64) waves).  Segment k then holds shard k's samples in tile
// order, so the extend waves draining the 64 segments side by side trace the same image tile for
// 64 sample groups (the item-claim path's order, whose L2 locality this keeps).  Otherwise slot i
// claims items from the shards (regen).
__global__ __launch_bounds__(kBlock) void wf_seed_kernel(DevCamera C, DevRender R, WaveBuffers B, uint32_t n_seed,
                                                         uint32_t chunk_items, unsigned long long *__restrict__ stats) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t seg = (i >> 6) % kSegs;
    Counters cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    PathState ps;
    bool ok = false;
    uint32_t slot = i;
    if (n_seed == chunk_items) {
        if (blockIdx.x == 0u && threadIdx.x < kSegs)
            B.ctrl[ctr_item(threadIdx.x)] = shard_lo(threadIdx.x + 1u, chunk_items) - shard_lo(threadIdx.x, chunk_items);
        const uint32_t lo = shard_lo(seg, chunk_items), hi = shard_lo(seg + 1u, chunk_items);
        const uint32_t item = lo + (i >> 6) / kSegs * 64u + (i & 63u);
        slot = item;
        if (item < hi) ok = seed_item<true>(C, R, B, slot, item, ps, cnt);
        // Every tile inside the image (W and H multiples of the 8x8 tile: C3's 1080p, the 4K frames): no
        // item is dropped, so shard k's items fill segment k in item order -- position item - lo, the
        // count set by block 0 -- without a queue ticket per wave (8.3 M atomics per C3 frame on 64
        // counters, ~2 ms at their measured rate, tools/atomic_bench.hip)
#ifndef OCTPT_SEED_TICKET  // (A/B build: every wave takes a queue ticket)
        if (((R.W | R.H) & (kTile - 1u)) == 0u) {
            if (blockIdx.x == 0u && threadIdx.x < kSegs)
                B.ctrl[ctr_count(0u, threadIdx.x)] = shard_lo(threadIdx.x + 1u, chunk_items) - shard_lo(threadIdx.x, chunk_items);
#if OCTPT_CAM_RECORDS
            if (ok) store_cam_ray(B, seg * B.seg_cap + (item - lo), ps);
            if (blockIdx.x == 0u && threadIdx.x == 0u) B.ray0[0][0] = B.eye;  // the camera records' origin record
#else
            if (ok) store_ray(B, 0u, seg * B.seg_cap + (item - lo), slot, ps);
#endif
            // every item has its pixel (no tile overhangs the image), so the chunk starts chunk_items paths: one
            // add by block 0 instead of a counter flush per wave (8.3 M per C3 frame)
            if (blockIdx.x == 0u && threadIdx.x == 0u) atomicAdd(&stats[kStatPaths], (unsigned long long)chunk_items);
            return;
        }
#endif
    } else {
        ItemCursor cur = {seg, true};
        ok = regen<true>(C, R, B, i, i < n_seed, chunk_items, cur, ps, cnt);
    }
    const uint32_t t = wave_ticket(B.ctrl + ctr_count(0u, seg), ok);
    if (ok) store_ray(B, 0u, seg * B.seg_cap + t, slot, ps);
    flush_counters(cnt, stats);
}

// extend: closest-hit queries for every queued ray.  Persistent waves; a lane that finishes
// its ray idles until at least `refill` lanes of the wave are idle, then the wave hands the idle
// lanes the next positions of the chunk it has claimed (Aila & Laine dynamic fetch, with the
// atomic of the next claim already in flight).
#ifndef OCTPT_EXTEND_WAVES
#define OCTPT_EXTEND_WAVES 1
#endif
// minimum waves per SIMD a wf_extend_kernel instance is compiled for (register budget)
// (measured at 64 spp against the unconstrained allocation: the few spilled dwords sit in cold
// code, the extra waves hide the slot loads' latency)
#ifndef OCTPT_SPH_WAVES
#define OCTPT_SPH_WAVES 8  // 71 -> 64 VGPRs, 20 B/lane spilled: C3 +2.0 %
#endif
#ifndef OCTPT_BOX_WAVES
#define OCTPT_BOX_WAVES 7  // 78 -> 72 VGPRs, 20 B/lane spilled: C4 +5.5 % (8 waves: -5 %)
#endif
#ifndef OCTPT_MDL_WAVES
#define OCTPT_MDL_WAVES 6  // 95 -> 80 VGPRs, 36 B/lane spilled: C5 +5.4 %
#endif
#ifndef OCTPT_BLK_WAVES
#define OCTPT_BLK_WAVES 6  // block-value leaves (C23); LDS holds depth-11 worlds (C5b, C5s) at 6 blocks per CU
#endif
#define OCTPT_EXTEND_WAVES_OF(k)                                                                              \
    ((k) == kPrimsSpheres ? OCTPT_SPH_WAVES                                                                   \
                          : (k) == kPrimsBoxes ? OCTPT_BOX_WAVES : (k) == kPrimsBlocks ? OCTPT_BLK_WAVES : OCTPT_MDL_WAVES)
// positions a wave claims from its segment at a time (one atomic per claim)
#ifndef OCTPT_CLAIM
#define OCTPT_CLAIM 64
#endif
constexpr uint32_t kClaim = OCTPT_CLAIM;
#ifndef OCTPT_XCD_SEGS
#define OCTPT_XCD_SEGS 0
#endif
static_assert(kSegs % 8u == 0u, "eight XCDs share the segments evenly");
// refill == 0 (adaptive): rays shorter than this many ESVO steps on average refill 32 at a time
#ifndef OCTPT_THR_LONG
#define OCTPT_THR_LONG 16   // refill threshold of waves with long rays (A/B knob)
#endif
#ifndef OCTPT_THR_SHORT
#define OCTPT_THR_SHORT 32  // ... and with short rays
#endif
#ifndef OCTPT_SHORT_STEPS
#define OCTPT_SHORT_STEPS 48  // mean ESVO steps below which a wave's rays count as short (A/B knob; round 5: 56 -> 48)
#endif
constexpr uint32_t kShortRaySteps = OCTPT_SHORT_STEPS;
template <int kPrims>
__global__ __launch_bounds__(kBlock, OCTPT_EXTEND_WAVES_OF(kPrims)) void wf_extend_kernel(DevScene S, WaveBuffers B, uint32_t q, uint32_t refill,
                                                           unsigned long long *__restrict__ stats) {
    extern __shared__ uint2 lds_stack[];
    const Stack stk = stack_of(lds_stack, S.depth);
    const float4 *ray0 = B.ray0[q], *ray1 = B.ray1[q];
    // refill bit 31 (launch_wf_extend's cam): the queue holds the seed's 16-B camera records (store_cam_ray), whose
    // origin record (eye, kPrimNone) the seed left at ray0[0] (no LDS for it: one more LDS granule per block
    // takes the depth-10 box instance from 7 blocks per CU to 6)
    const bool cam = OCTPT_CAM_RECORDS && (refill >> 31) != 0u;
    refill &= 0x7FFFFFFFu;
    if (blockIdx.x == 0 && threadIdx.x < kSegs) {  // the other queue is refilled by this iteration's shade
        B.ctrl[ctr_count(q ^ 1u, threadIdx.x)] = 0u;
        B.ctrl[ctr_head(q ^ 1u, threadIdx.x)] = 0u;
    }
    // the wave starts on its home segment (seg, seg_n rays: wave-uniform)
#if OCTPT_XCD_SEGS
    // XCD-aware home segments (A/B knob): blocks are dealt round robin over the 8 XCDs (block b on XCD b % 8), so
    // XCD x takes the 8 contiguous segments 8x .. 8x + 7 -- one band of the image per XCD, whose geometry its own L2
    // holds -- instead of the two bands 4x .. 4x + 3 and 4x + 32 .. 4x + 35 the plain modulo gives it
    uint32_t seg = __builtin_amdgcn_readfirstlane(
        (blockIdx.x % 8u) * (kSegs / 8u) + ((blockIdx.x / 8u) * (kBlock / 64u) + (threadIdx.x >> 6)) % (kSegs / 8u));
#else
    uint32_t seg = __builtin_amdgcn_readfirstlane(((blockIdx.x * kBlock + threadIdx.x) >> 6) % kSegs);
#endif
    uint32_t seg_n = B.ctrl[ctr_count(q, seg)];
    // (the block-model instance holds seg_n in an SGPR: in a VGPR it was spilled, C5 extend -1 %)
    if constexpr (kPrims == kPrimsModels) seg_n = __builtin_amdgcn_readfirstlane(seg_n);
    bool rays_left = true;  // wave-uniform: some segment may still hold unclaimed rays
    uint32_t segs_w = 0u;   // segments started by this wave
    Counters cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    // a lane is busy while E.idx holds a child index (0..7); kIdle marks an idle lane, so that the
    // loop's ballot of the idle lanes is one compare, not a lane-mask bool materialised and compared back
    constexpr uint32_t kIdle = 8u;
    uint32_t pos = 0u;
    TraceRay tr;
    Esvo E;
    E.idx = kIdle;
    bool more = true;
    // chunked claims: the wave owns [c_next, c_end) of segment seg and holds one further claim in
    // flight (lane 0's atomic result, read only when the owned chunk runs out), so a refill hands
    // out positions without waiting on an atomic's round trip
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t c_next = 0u, c_end = 0u, claim_v = 0u;
    uint32_t thr = refill ? refill : OCTPT_THR_LONG;  // idle lanes that trigger a refill (wave-uniform)
    if (lane == 0u)
        claim_v = __hip_atomic_fetch_add(B.ctrl + ctr_head(q, seg), kClaim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    do {
        // refill: one scalar test per iteration
        const bool idle = E.idx >= kIdle;
        const uint64_t im = __ballot(idle);
        if (rays_left && (uint32_t)__popcll(im) >= thr) {
            if (c_next >= c_end) {  // the owned chunk ran out: take the claim in flight
                c_next = __builtin_amdgcn_readfirstlane(claim_v);
                c_end = c_next < seg_n ? __builtin_amdgcn_readfirstlane(min(c_next + kClaim, seg_n))
                                       : c_next;
                if (c_next >= c_end) {
                    // segment drained: lane j checks segment j, the wave moves on and claims there
                    // (j passed through an empty asm: the two per-lane counter addresses are formed
                    // here, not hoisted out of the loop into registers that the loop then spills)
                    uint32_t j = lane;
                    if constexpr (kPrims != kPrimsSpheres) asm volatile("" : "+v"(j));
                    const uint64_t m = __ballot(relaxed_load(B.ctrl + ctr_head(q, j)) < B.ctrl[ctr_count(q, j)]);
                    rays_left = m != 0ull;
                    if (rays_left) {
                        seg = __builtin_amdgcn_readfirstlane(first_from(m, seg));
                        seg_n = B.ctrl[ctr_count(q, seg)];
                        if constexpr (kPrims == kPrimsModels) seg_n = __builtin_amdgcn_readfirstlane(seg_n);
                    }
                }
                if (rays_left && lane == 0u)
                    claim_v = __hip_atomic_fetch_add(B.ctrl + ctr_head(q, seg), kClaim,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const uint32_t avail = c_end - c_next;
            if (idle) {
                const uint32_t r = lanes_below(im);
                if (r < avail) {
                    pos = seg * B.seg_cap + c_next + r;
                    const float4 r1 = ray1[pos];
                    // a camera record (cam, wave-uniform): from the eye (its w kPrimNone, so that the last
                    // primitive decodes as none), r1.w the beam start or 0 (sign clear: not inward)
                    const float4 r0 = ray0[cam ? 0u : pos];
                    const float bm = cam ? r1.w : ray_beam(r0, r1);
                    tr = make_trace_ray(S, V(r0.x, r0.y, r0.z), V(r1.x, r1.y, r1.z), ray_last_prim(r0, r1),
                                        (__float_as_uint(r1.w) >> 31) != 0u);
                    esvo_begin(S, tr, E, stk, bm);
                    cnt.steps -= E.iter;  // a beam start's bound of skipped iterations: executed ones are counted
#if OCTPT_LEAD_LOOP
                    // the ray's leading descends (octree_traversal.rs:216-244, exact replicas counted in E.iter) in a
                    // tight loop of the refilled lanes, while the wave refills anyway, instead of one main-loop step
                    // per level (A/B knob)
                    lead_descends(S, E, stk);
#endif
                }
            }
            const uint32_t took = min((uint32_t)__popcll(im), avail);
            segs_w += took;
            c_next += took;
            if (refill == 0u) {
                // adaptive threshold: when most lanes' rays so far averaged fewer
                // than kShortRaySteps ESVO steps, the wave refills 32 at a time, else 16
                // (a lane's rays counted as the wave's average, segs_w / 64: no per-lane counter, which
                // the block instance spilled to scratch at every refill)
                // (signed: a lane's in-flight beam start has been subtracted already)
                const bool short_rays = (int64_t)(int32_t)cnt.steps * 64 < (int64_t)kShortRaySteps * segs_w;
                thr = __popcll(__ballot(short_rays)) > 32 ? OCTPT_THR_SHORT : OCTPT_THR_LONG;
            }
        }
        // inner loop: step until `thr` lanes are idle (every lane, once no ray is left); its only
        // per-iteration bookkeeping is one ballot, a popcount and a scalar branch
        const uint32_t stop_at = __builtin_amdgcn_readfirstlane(rays_left ? thr : 64u);  // keeps the loop scalar
        if ((uint32_t)__popcll(__ballot(E.idx >= kIdle)) < stop_at) do {
#ifdef OCTPT_PROFILE_LANES
            prof_wave(cnt.p_iters, cnt.p_active, E.idx < kIdle);
#endif
            if (E.idx < kIdle) {
                // set by the leaf test on a hit, the only case that reads it: left unspecified (no v_mov per
                // step), except in the block-model instance, whose allocation spills 4 B more without the init
                // (the check build keeps kPrimNone, so that a hit that never wrote its id is counted)
                uint32_t prim = kPrimNone;
#ifndef OCTPT_CHECK_HITS
                if constexpr (kPrims != kPrimsModels) asm("" : "=v"(prim));
#endif
                PrimHit h;
                HIT_POISON(prim, h);
                const int rs = esvo_step<kPrims, true>(S, tr, E, stk, cnt, prim, h);
                SLOT_CHECK(E, stats, 0u);
                if (rs != kStepContinue) {
                    HIT_CHECK(kPrims, rs, prim, h, stats, 0u);
                    // the record's address is formed here from pos (through an empty asm), not kept
                    // from the refill in two more registers that the loop would spill (not in the
                    // sphere instance, whose allocation is better off as it is: C3 -1 % with it)
                    uint32_t p = pos;
                    if constexpr (kPrims != kPrimsSpheres) asm volatile("" : "+v"(p));
                    // a miss: (kPrimNone, 0), or (kPrimNone, kHitCapped) on the step cap (shade retraces a
                    // beam-started camera ray, esvo_capped)
                    const uint2 miss = make_uint2(kPrimNone, esvo_capped(E.iter) ? kHitCapped : 0u);
                    if constexpr (kPrims == kPrimsBlocks) {  // (face << 27 | block or the quad, t, u, v) (C23): one store
                        B.hit4[p] = rs == kStepHit ? make_uint4(prim, __float_as_uint(h.t), __float_as_uint(h.u),
                                                                __float_as_uint(h.v))
                                                   : make_uint4(miss.x, miss.y, 0u, 0u);
                    } else {
                        B.hit[p] = rs == kStepHit ? hit_record(prim, h) : miss;
                    }
                    cnt.steps += E.iter;
                    E.idx = kIdle;
                }
            }
        } while ((uint32_t)__popcll(__ballot(E.idx >= kIdle)) < stop_at);  // at the bottom: no phi copies
        more = rays_left;  // wave-uniform; every lane is idle when it is false
    } while (more);
    cnt.segs = (threadIdx.x & 63u) == 0u ? segs_w : 0u;  // flush_counters sums over the wave's lanes
    flush_counters(cnt, stats);
}

// Shade of one traced segment (a lane of wf_shade_kernel, and of wf_drain_kernel): the path in the ray
// record's slot is loaded, its hit record (hr, extend's output) committed and its shading step taken.
// Returns true when the path continues (its state stored to the slot, the next ray in ps), false when
// it finished (its colour record written).  first (wave-uniform: the chunk's first shade, whose
// rays the seed started): the path state is rebuilt from the slot's item as the seed computed it,
// through the same pack / unpack as a stored path, instead of being read.
// kLean with OCTPT_LEAN_POS: the state is read at (q, pos) and a continuing path's is not stored here: the caller
// stores it at the position its next ray takes (store_lean_at).
template <bool kNee, bool kLean = false, int kSP = kPrimsModels>
__device__ __forceinline__ bool shade_lane(const DevScene &S, const DevCamera &C, const DevRender &R,
                                           const WaveBuffers &B, bool first, float4 r0, float4 r1, const uint2 *hit_rec,
                                           const uint4 *hit4_rec, PathState &ps, uint32_t &slot, uint32_t &item,
                                           Counters &cnt, uint32_t q = 0u, uint32_t pos = 0u) {
    constexpr bool kPos = kLean && OCTPT_LEAN_POS;
    slot = __float_as_uint(r1.w) & (kRayBeamBit - 1u);
    if (first) {
        item = kLean ? slot : B.item0[slot];
        PathState s0;
        uint32_t x, y;
        item_path<false>(C, R, item, s0, x, y);  // the seed only queued items inside the image
        float4 a, b;
        uint2 c;
        pack_path(s0, item, a, b, c);
        unpack_path(a, b, c, B.eye, r1, ps, item);  // a camera ray's ray0 is (eye, kPrimNone): not re-read
    } else if constexpr (kPos) {  // L = +0 as the path started, item = slot (store_lean_at)
        const float4 a = (q ? B.pb : B.pa)[pos];
        unpack_path(make_float4(a.x, a.y, a.z, 0.0f), make_float4(0.0f, 0.0f, a.w, __uint_as_float(slot)),
                    B.pc[(size_t)q * kSegs * B.seg_cap + pos], r0, r1, ps, item);
    } else {
        load_path<kLean>(B, slot, r0, r1, ps, item);
    }
    // the hit record: 8 B, or in block-value scenes (a uniform branch) 16 B with its (u, v) (C23)
    uint2 hr;
    float2 huv = make_float2(0.0f, 0.0f);
    constexpr bool kMayBlocks = kSP == kPrimsBlocks || kSP == kPrimsModels;
    if (kSP == kPrimsBlocks || (kMayBlocks && S.has_blocks)) {
        const uint4 r = *hit4_rec;
        hr = make_uint2(r.x, r.y);
        huv = make_float2(__uint_as_float(r.z), __uint_as_float(r.w));
    } else {
        hr = *hit_rec;
    }
    if (__builtin_expect((hr.x == kPrimNone) & (hr.y == kHitCapped) & ((__float_as_uint(r1.w) & kRayBeamBit) != 0u), 0)) {
        // a beam-started camera ray that reached the reference's step cap (extend's kHitCapped record): the
        // same ray is queued again without its beam start, for the walk from the cube entry.  No segment
        // is counted; the path state is the seed's (stored now when this shade rebuilt it from the item).
        if (first && !kPos) store_path<kLean>(B, slot, ps, item);
        ps.n = V(0.0f, 0.0f, 0.0f);
        ps.beam = 0.0f;
        cnt.redo++;
        return true;
    }
    const bool was_shadow = kNee && ps.shadow;
    if (was_shadow) load_nee(B, slot, ps);
    const bool hit = hr.x != kPrimNone;
    if (hit && (kSP == kPrimsBlocks || (kMayBlocks && S.has_blocks))) {  // block-value leaf (C23): (u, v) beside it
        ps.n = V(0.0f, 0.0f, 0.0f);
        commit_block_hit(S, ps, hr.x, __uint_as_float(hr.y), huv.x, huv.y, cnt);
    } else if (hit) {
        PrimHit h;
        const uint32_t flags = (hr.x >> 27) & 15u;
        h.t = __uint_as_float(hr.y);
        h.f = flags;
        // a sphere hit record carries its root, decided by extend's estimate: t exactly
        if (sph_kind(kSP) || !(hr.x & kPrimCuboidBit))
            h.t = sphere_root(S.spheres[hr.x & kPrimIndexMask], ps.o, ps.d, flags & 1u);
        ps.n = V(0.0f, 0.0f, 0.0f);
        commit_hit<kSP>(S, ps, (hr.x & kPrimCuboidBit) | (hr.x & kPrimIndexMask), h, cnt);
    }
    bool cont = shade_segment<kNee, kLean>(S, R, ps, hit, cnt);
    if (cont) cont = begin_segment(ps);
    if (cont) {
        if (!kPos) store_path<kLean>(B, slot, ps, item);
        if (kNee && ps.shadow) {  // a shadow segment follows: new sun sample or the next one
            if (!was_shadow) store_nee(B, slot, ps);
            store_att(B, slot, ps);
        }
        return true;
    }
    // segments this item reports (a branch > 0 reports none of the replayed prefix) and whether the
    // first reflection split (C20)
    const uint32_t segs = ((OCTPT_LEAN_STRICT && kLean) || ps.branch == 0u) ? ps.path_segs
                                                                             : (ps.depth ? ps.path_segs - ps.seg_base : 0u);
    B.color[item] = make_float4(ps.L.x, ps.L.y, ps.L.z, __uint_as_float(segs | (ps.depth ? 0x80000000u : 0u)));
    return false;
}

// shade: one lane per traced ray (grid-stride, wave-uniform trip count)
#ifndef OCTPT_SHADE_WAVES
#define OCTPT_SHADE_WAVES 1
#endif
#ifndef OCTPT_SHADE_LEAN_WAVES
#define OCTPT_SHADE_LEAN_WAVES 6  // the lean instance (kMode 2): register budget for 6 waves/SIMD (A/B knob)
#endif
// scenes with at most kShadeLdsMats materials and textures shade from LDS copies of the material
// and texture tables and the sRGB LUT: these loads sit at the end of the dependent chain
// ray -> path state / primitive -> face material -> material -> texture -> texel -> LUT
#ifndef OCTPT_SHADE_LDS_MATS
#define OCTPT_SHADE_LDS_MATS 128
#endif
constexpr uint32_t kShadeLdsMats = OCTPT_SHADE_LDS_MATS;
// ... and at most this many blocks (C23) their face-material table
#ifndef OCTPT_SHADE_LDS_BLOCKS
#define OCTPT_SHADE_LDS_BLOCKS 128
#endif
constexpr uint32_t kShadeLdsBlocks = OCTPT_SHADE_LDS_BLOCKS;
// kRegen: finished lanes regenerate their slot with the next chunk items.  Only a pool smaller than
// the chunk needs it (when the pool holds the chunk -- C3's frame, every 4K chunk -- the seed claimed
// every item); the instance without it is 19 VGPRs leaner (96 instead of 115, 5 waves/SIMD instead of 4).
// kMode: 0 = the 40-B path state, no regeneration; 1 = with regeneration; 2 = the lean 24-B path state (no
// regeneration, no sun sampling, kLean above)
// kNoFirst (OCTPT_SHADE_FIRST_SPLIT): an instance for the chunk's later launches, compiled without the first
// launch's path-state rebuild (first is 0)
template <bool kNee, bool kLdsMats, int kMode, bool kNoFirst = false, int kSP = kPrimsModels>
__global__ __launch_bounds__(kBlock, kMode == 2 ? OCTPT_SHADE_LEAN_WAVES : OCTPT_SHADE_WAVES) void wf_shade_kernel(DevScene Sg, DevCamera C, DevRender R, WaveBuffers B,
                                                          uint32_t q, uint32_t chunk_items, uint32_t first_arg,
                                                          unsigned long long *__restrict__ stats) {
    const uint32_t first = kNoFirst ? 0u : first_arg;
    constexpr uint32_t kT = (kLdsMats && kShadeLdsMats) ? kShadeLdsMats : 1u;
    __shared__ DevMaterial smats[kT];
    __shared__ DevTexture stexs[kT];
    __shared__ float slut[kLdsMats ? 256 : 1];
    __shared__ uint32_t sblk[kLdsMats ? 6u * kShadeLdsBlocks : 1];
    DevScene S = Sg;
    if constexpr (kLdsMats) {
        for (uint32_t m = threadIdx.x; m < Sg.n_mats; m += kBlock) smats[m] = Sg.mats[m];
        for (uint32_t t = threadIdx.x; t < Sg.n_texs; t += kBlock) stexs[t] = Sg.texs[t];
        static_assert(kBlock == 256u, "one LUT entry per thread");
        slut[threadIdx.x] = Sg.lut_float[threadIdx.x];
        // block-value scenes: the block -> face material table too (C5b: 10 blocks), so that a block
        // hit's material is an LDS read, not a dependent global load before the texel's
        const bool lds_blk = Sg.has_blocks && Sg.n_blocks <= kShadeLdsBlocks;
        if (lds_blk)
            for (uint32_t k = threadIdx.x; k < 6u * Sg.n_blocks; k += kBlock) sblk[k] = Sg.blk_mat[k];
        __syncthreads();
        S.mats = smats;
        S.texs = stexs;
        S.lut_float = slut;
        if (lds_blk) S.blk_mat = sblk;
    }
    // wave w shades segment w % kSegs of queue q (grid: a multiple of kSegs waves) and appends
    // the continuing / regenerated rays to the same segment of queue q ^ 1
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * kBlock + threadIdx.x) >> 6;
    const uint32_t seg = wave % kSegs;
    const uint32_t seg_waves = ((gridDim.x * kBlock) >> 6) / kSegs;
    const uint32_t count = B.ctrl[ctr_count(q, seg)];
    const uint32_t seg0 = seg * B.seg_cap;
    ItemCursor cur = {seg, true};
    Counters cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    for (uint32_t base = (wave / kSegs) * 64u; base < count; base += seg_waves * 64u) {
        const uint32_t i = seg0 + base + lane;
        const bool valid = base + lane < count;
        uint32_t slot = 0u, item = 0u;
        bool append = false, finished = false;
        PathState ps;
        if (valid) {
            float4 r1 = B.ray1[q][i];
            if (first == 2u) {  // the seed's 16-B camera records: slot = item = shard_lo(seg) + index in the segment
                float4 r0c;
                cam_ray(B.eye, shard_lo(seg, chunk_items) + base + lane, r0c, r1);
            }
            const float4 r0 = first ? B.eye : B.ray0[q][i];  // (the chunk's first shade: the seed's camera rays)
            append = shade_lane<kNee, kMode == 2, kSP>(S, C, R, B, first != 0u, r0, r1, B.hit + i,
                                                  S.has_blocks ? B.hit4 + i : nullptr, ps, slot, item, cnt, q, i);
            finished = !append;
        }
        // regenerate: finished lanes take the next chunk items (path regeneration)
        if constexpr (kMode == 1) {
            if (regen(C, R, B, slot, finished, chunk_items, cur, ps, cnt)) append = true;
        }
        const uint32_t t = wave_ticket(B.ctrl + ctr_count(q ^ 1u, seg), append);
        if (append) {
            store_ray(B, q ^ 1u, seg0 + t, slot, ps);
            if constexpr (kMode == 2 && OCTPT_LEAN_POS) store_lean_at(B, q ^ 1u, seg0 + t, ps);
        }
    }
    cnt.ib = 0u;  // issued bytes are extend's only
    flush_counters(cnt, stats);
}

// Drain: once every chunk item is claimed and the queue holds few rays, one launch
// finishes every queued path in its lane -- trace, shade, trace, ... -- instead of one extend /
// shade pair per remaining segment: the last ~60 iterations of a chunk are the rare long paths, each
// a near-empty launch pair bounded by host launch latency (5 ms of C3's 288 ms frame, 13 % of an
// 8-way shard's).  Every segment goes through the wavefront's own formats and code (extend's
// esvo_step and hit record, shade_lane, the ray record as store_ray writes it), so results and
// statistics equal the extend / shade iterations it replaces.  No regeneration: items are exhausted.
template <int kPrims, bool kNee>
__global__ __launch_bounds__(kBlock) void wf_drain_kernel(DevScene S, DevRender R, WaveBuffers B, uint32_t q,
                                                          unsigned long long *__restrict__ stats) {
    extern __shared__ uint2 lds_stack[];
    const Stack stk = stack_of(lds_stack, S.depth);
    Counters cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    // one path per wave (its lane 0): the paths are at different segments and phases, and one lane
    // each keeps a wave free of divergence; the grid spreads them over every CU
    const uint32_t wid = (blockIdx.x * kBlock + threadIdx.x) >> 6, nw = (gridDim.x * kBlock) >> 6;
    const uint32_t jlim = (threadIdx.x & 63u) == 0u ? 0xFFFFFFFFu : 0u;
    for (uint32_t k = 0; k < kSegs; ++k) {  // queue q, segment after segment, dealt over the waves
        const uint32_t n = min(B.ctrl[ctr_count(q, k)], jlim);
        for (uint32_t j = wid; j < n; j += nw) {
            const uint32_t p = k * B.seg_cap + j;
            float4 r0 = B.ray0[q][p], r1 = B.ray1[q][p];
            for (;;) {
                const TraceRay tr = make_trace_ray(S, V(r0.x, r0.y, r0.z), V(r1.x, r1.y, r1.z), ray_last_prim(r0, r1),
                                                   (__float_as_uint(r1.w) >> 31) != 0u);
                Esvo E;
                esvo_begin(S, tr, E, stk, ray_beam(r0, r1));
                cnt.steps -= E.iter;  // as in wf_extend_kernel
                bool beam_ray = (__float_as_uint(r1.w) & kRayBeamBit) != 0u;
                uint32_t prim = kPrimNone;
                PrimHit h;
                int rs;
                for (;;) {
                    do {
                        HIT_POISON(prim, h);
                        rs = esvo_step<kPrims, true>(S, tr, E, stk, cnt, prim, h);
                        SLOT_CHECK(E, stats, kStatDrainRow);
                    } while (rs == kStepContinue);
                    HIT_CHECK(kPrims, rs, prim, h, stats, kStatDrainRow);
                    cnt.steps += E.iter;
                    if (!((rs == kStepMiss) & esvo_capped(E.iter) & beam_ray)) break;
                    cnt.redo++;  // traced again from the cube entry, in place (shade_lane's retrace, inline)
                    beam_ray = false;
                    esvo_root(S, E);
                    esvo_first_child(E);
                }
                cnt.segs++;
                uint2 hr;
                if constexpr (kPrims == kPrimsBlocks)
                    hr = rs == kStepHit ? make_uint2(prim, __float_as_uint(h.t)) : make_uint2(kPrimNone, 0u);
                else
                    hr = rs == kStepHit ? hit_record(prim, h) : make_uint2(kPrimNone, 0u);
                const uint4 h4 = make_uint4(hr.x, hr.y, __float_as_uint(h.u), __float_as_uint(h.v));  // block scenes
                PathState ps;
                uint32_t slot, item;
                const bool lean = !kNee && B.lean;
                const bool cont = lean ? shade_lane<kNee, true>(S, DevCamera{}, R, B, false, r0, r1, &hr, &h4, ps, slot, item,
                                                                cnt, q, p)
                                       : shade_lane<kNee, false>(S, DevCamera{}, R, B, false, r0, r1, &hr, &h4, ps, slot, item, cnt);
                if (!cont) break;
                // the lean state back at this path's queue position, where its next shade_lane reads it
                if (OCTPT_LEAN_POS && lean) store_lean_at(B, q, p, ps);
                // the next segment's ray record, as store_ray writes it
                r0 = make_float4(ps.o.x, ps.o.y, ps.o.z, __uint_as_float(ps.last_prim));
                r1 = make_float4(ps.d.x, ps.d.y, ps.d.z,
                                 __uint_as_float(slot | (vdot(ps.d, ps.n) < 0.0f ? 0x80000000u : 0u)));
            }
        }
    }
    flush_counters(cnt, stats, kStatDrainRow);
}

// resolve: per pixel, the chunk's samples in sample order into the running mean
__global__ __launch_bounds__(kBlock) void wf_resolve_kernel(DevRender R, WaveBuffers B, uint32_t chunk_spp,
                                                            float4 *__restrict__ accum, uint32_t *__restrict__ segcount) {
    const uint32_t px_item = blockIdx.x * kBlock + threadIdx.x;
    if (px_item >= R.total_items) return;
    uint32_t x, y;
    item_pixel(R, px_item, x, y);
    if (x >= R.W || y >= R.H) return;
    const uint32_t acc_idx = R.compact ? px_item : y * R.W + x;
    float4 fb = accum[acc_idx];
    uint32_t segs = 0u;
    v3 L0 = V(0.0f, 0.0f, 0.0f), sum = L0;
    bool split = false;
    for (uint32_t s = 0; s < chunk_spp; ++s) {
        const float4 c = B.color[(size_t)s * R.total_items + px_item];
        const uint32_t w = __float_as_uint(c.w);
        segs += w & 0x7FFFFFFFu;
        if (!R.subs) {
            running_mean(fb, V(c.x, c.y, c.z), R.spp_start + s, 1u);
            continue;
        }
        // branch schedule (C20): a pass's branches fold into one sample of weight bc; the colour
        // is their mean when the first reflection split, else branch 0's (all branches agree)
        const uint2 sb = R.subs[s];
        const uint32_t b = sb.y >> 16, bc = sb.y & 0xFFFFu;
        if (b == 0u) {
            L0 = V(c.x, c.y, c.z);
            sum = vadd(V(0.0f, 0.0f, 0.0f), L0);
            split = (w >> 31) != 0u;
        } else {
            sum = vadd(sum, V(c.x, c.y, c.z));
        }
        if (b + 1u == bc) {
            const float inv = 1.0f / (float)bc;
            running_mean(fb, split ? vscale(sum, inv) : L0, sb.x, bc);
        }
    }
    accum[acc_idx] = fb;
    if (segcount) segcount[acc_idx] += segs;
}

// one ray per thread closest-hit query (Scene::hit) for octpt_intersect
template <int kPrims>
__global__ __launch_bounds__(kBlock) void intersect_kernel(DevScene S, const float *__restrict__ rays,
                                                           const uint32_t *__restrict__ last_prim,
                                                           const float *__restrict__ last_normal, uint32_t n,
                                                           float *__restrict__ out_t, uint32_t *__restrict__ out_prim,
                                                           float *__restrict__ out_normal, uint32_t *__restrict__ out_steps) {
    extern __shared__ uint2 lds_stack[];
    const Stack stk = stack_of(lds_stack, S.depth);
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    PathState ps;
    ps.o = V(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
    ps.d = V(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    ps.n = last_normal ? V(last_normal[3 * i], last_normal[3 * i + 1], last_normal[3 * i + 2]) : V(0.0f, 0.0f, 0.0f);
    ps.cur = ps.prev = ps.depth = 0u;
    ps.last_prim = last_prim ? last_prim[i] : kPrimNone;
    ps.specular = true;
    const TraceRay tr = trace_ray_of(S, ps);
    Esvo E;
    Counters cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    esvo_begin(S, tr, E, stk);
    uint32_t prim = kPrimNone;
    PrimHit h;
    int rs;
    do {
        rs = esvo_step<kPrims>(S, tr, E, stk, cnt, prim, h);
    } while (rs == kStepContinue);
    if (rs == kStepHit) {
        commit_hit(S, ps, prim, h, cnt);
        out_t[i] = h.t;
        // block-value scenes (C23): the block id of a block filling its cell, kQuadKey | quad of a model quad
        out_prim[i] = kPrims != kPrimsBlocks ? prim : ((prim & kPrimCuboidBit) ? kQuadKey | (prim & kPrimIndexMask)
                                                                                 : prim & kPrimIndexMask);
        if (out_normal) {
            out_normal[3 * i] = ps.n.x;
            out_normal[3 * i + 1] = ps.n.y;
            out_normal[3 * i + 2] = ps.n.z;
        }
    } else {
        out_t[i] = __int_as_float(0x7f800000);
        out_prim[i] = kPrimNone;
        if (out_normal) out_normal[3 * i] = out_normal[3 * i + 1] = out_normal[3 * i + 2] = 0.0f;
    }
    if (out_steps) out_steps[i] = E.iter;
}

// Beam start of the camera rays (Laine & Karras 2010, §5.2 "beam optimization"; the reference's
// own beam-start device is get_traversal_data, octree_traversal.rs:537-714, C17).  One thread per
// kBeamTile x kBeamTile pixel tile: every camera ray of the tile leaves the eye inside the pyramid spanned by the tile's
// screen rectangle (new_path: pixel centre +- one jitter step, padded), so no ray of the tile meets a
// leaf before the Euclidean distance from the eye to the nearest leaf cell that intersects the
// pyramid.  A front-to-back depth-first walk of the octree, pruned by that distance and by the
// pyramid's four side planes, finds it.  The start is in octree units (the ESVO t of a unit direction),
// shrunk by a relative 2^-16 for the float evaluation; esvo_begin subtracts ESVO's own rounding bound.
// No leaf in the pyramid: +inf (the rays start at their cube exit).  Conservative throughout: a test
// that cannot decide keeps the cell, which can only lower the start.
constexpr int kBeamLevels = 24;
static_assert(kTile % kBeamTile == 0, "beam tiles nest in the 8x8 render tiles");
constexpr uint32_t kBeamSub = (kTile / kBeamTile) * (kTile / kBeamTile);  // beam tiles per render tile
// the walk's stack levels: octants lie at levels 0 .. depth - 1
__host__ __device__ constexpr uint32_t beam_levels(uint32_t depth) {
    return depth < 1u ? 1u : depth < (uint32_t)kBeamLevels ? depth : (uint32_t)kBeamLevels;
}
#ifndef OCTPT_BEAM_VISITS
#define OCTPT_BEAM_VISITS (1u << 13)
#endif
constexpr uint32_t kBeamVisits = OCTPT_BEAM_VISITS;  // cells visited per tile; past it the tile gets no beam (0)
#ifndef OCTPT_BEAM_LOD
#define OCTPT_BEAM_LOD 0.0f
#endif
constexpr float kBeamLod = OCTPT_BEAM_LOD;

// A tile's start t with, in its low kBeamIterBits bits, a bound of the reference iterations a ray of the
// tile runs before it (t is rounded down first, so the packed value never exceeds it).  The reference
// walk (octree_traversal.rs:127-300) spends one iteration per child cell it processes -- a descend
// enters the cell, an advance leaves it, and a cell left by a pop is never processed again -- and it
// processes at most 4 children of an octant it enters, since in mirrored coordinates each axis can
// step across the octant's midplane once.  Every octant a ray of the tile enters before t meets the
// pyramid nearer than t, so this walk entered it too (it prunes only by the pyramid and by distances
// >= the final start): 4 * nodes bounds those iterations.  E.iter starts there (esvo_begin); a bound at
// or past the cap (OCTREE_MAX_STEPS) gives no start (0), as does a start too small to carry it.
__device__ __forceinline__ float beam_pack(float t, uint32_t nodes) {
    const uint32_t bound = 4u * nodes;
    const uint32_t b = __float_as_uint(t);
    if (bound >= OCTREE_MAX_STEPS || b < 2u * (kBeamIterMask + 1u)) return 0.0f;
    return __uint_as_float(((b - (kBeamIterMask + 1u)) & ~kBeamIterMask) | bound);
}

#ifndef OCTPT_BEAM_COOP
#define OCTPT_BEAM_COOP 1
#endif
#if OCTPT_BEAM_COOP
// Round 5: kBeamLanes lanes per beam tile, lane j standing for child j of the octant the
// walk is in.  Entering an octant tests its eight children's boxes at once (while its node slot is in flight),
// and each iteration takes the nearest child still nearer than the best leaf so far (a min over the group's
// eight lanes, three DPP moves), so the walk's sequential length is the number of cells it takes, not the
// number of children it tests; eight tiles share a 64-lane wave, and an 8-way shard's 16 K C3 tiles fill
// 2 K waves instead of 253.  The start is the same distance (the minimum over the pyramid's leaf cells, by the
// same box arithmetic), so only the walk's octant count -- the iteration bound it packs -- differs.
constexpr uint32_t kBeamLanes = 8u;
__global__ __launch_bounds__(64) void beam_kernel(DevScene S, DevCamera C, DevRender R, uint32_t n_tiles,
                                                  float *__restrict__ beam) {
    const uint32_t lane = threadIdx.x & (kBeamLanes - 1u), grp = threadIdx.x / kBeamLanes;
    // group g of block b: beam tile i = b * 8 + g, i.e. beam tile i % kBeamSub of the shard's render tile
    // i / kBeamSub (item_pixel's tile order), so a rank of N computes only its own tiles' starts
    const uint32_t i = blockIdx.x * (64u / kBeamLanes) + grp;
    if (i >= n_tiles) return;  // whole groups leave: the shuffles below stay inside a group
    const uint32_t rt = dealt_tile(R.tile_order, R.shard_index + (i / kBeamSub) * R.shard_count), sub = i % kBeamSub;
    const uint32_t rty = udiv_c(rt, R.div_tiles_x);
    const uint32_t x0 = (rt - rty * R.tiles_x) * kTile + (sub % (kTile / kBeamTile)) * kBeamTile,
                   y0 = rty * kTile + (sub / (kTile / kBeamTile)) * kBeamTile;
    if (x0 >= R.W || y0 >= R.H) return;  // no pixel of the image: never read
    const uint32_t tile = (y0 / kBeamTile) * R.beam_tx + x0 / kBeamTile;
    const uint32_t x1 = min(x0 + kBeamTile, R.W), y1 = min(y0 + kBeamTile, R.H);
    // screen coordinates of the tile's rays (new_path: xn + dx, yn + dy), padded by 2 % + 1e-6
    float s0 = ((float)(2u * x0) - (float)R.W) / R.dim, s1 = ((float)(2u * x1) - (float)R.W) / R.dim;
    float t0 = ((float)(2u * (R.H - y1)) - (float)R.H) / R.dim, t1 = ((float)(2u * (R.H - y0)) - (float)R.H) / R.dim;
    const float ps = 0.02f * (s1 - s0) + 1e-6f, pt = 0.02f * (t1 - t0) + 1e-6f;
    s0 -= ps; s1 += ps; t0 -= pt; t1 += pt;
    const v3 F = vscale(V(C.dir[0], C.dir[1], C.dir[2]), C.d_factor);
    const v3 Rt = V(C.right[0], C.right[1], C.right[2]), Up = V(C.up[0], C.up[1], C.up[2]);
    const v3 Ek[4] = {vadd(vadd(F, vscale(Rt, s0)), vscale(Up, t0)), vadd(vadd(F, vscale(Rt, s1)), vscale(Up, t0)),
                      vadd(vadd(F, vscale(Rt, s1)), vscale(Up, t1)), vadd(vadd(F, vscale(Rt, s0)), vscale(Up, t1))};
    const v3 Ec = vadd(vadd(F, vscale(Rt, 0.5f * (s0 + s1))), vscale(Up, 0.5f * (t0 + t1)));
    v3 pn[4];
    for (int k = 0; k < 4; ++k) {
        v3 n = vcross(Ek[k], Ek[(k + 1) & 3]);
        if (vdot(n, Ec) < 0.0f) n = vscale(n, -1.0f);
        pn[k] = n;
    }
    // the eye as esvo_begin places a ray origin in octree space
    const v3 e = vadd(vscale(V(C.eye[0], C.eye[1], C.eye[2]), S.octree_scale), V(1.0f, 1.0f, 1.0f));
    // distance from the eye to the box [lo, lo + h], or -1 when the box lies outside the pyramid
    auto box = [&](v3 lo, float h) -> float {
        const v3 a = vsub(lo, e), b = vsub(vadd(lo, V(h, h, h)), e);
        const float ext = fmaxf(fmaxf(fmaxf(fabsf(a.x), fabsf(b.x)), fmaxf(fabsf(a.y), fabsf(b.y))),
                                fmaxf(fabsf(a.z), fabsf(b.z)));
        for (int k = 0; k < 4; ++k) {
            const v3 n = pn[k];
            const float mx = (fmaxf(n.x * a.x, n.x * b.x) + fmaxf(n.y * a.y, n.y * b.y)) + fmaxf(n.z * a.z, n.z * b.z);
            const float tol = 1e-5f * ((fabsf(n.x) + fabsf(n.y)) + fabsf(n.z)) * ext;
            if (mx < -tol) return -1.0f;
        }
        const float dx = a.x > 0.0f ? a.x : (b.x < 0.0f ? -b.x : 0.0f);
        const float dy = a.y > 0.0f ? a.y : (b.y < 0.0f ? -b.y : 0.0f);
        const float dz = a.z > 0.0f ? a.z : (b.z < 0.0f ? -b.z : 0.0f);
        return sqrtf((dx * dx + dy * dy) + dz * dz);
    };
    const float lod = kBeamLod * fmaxf(s1 - s0, t1 - t0) / sqrtf(vdot(F, F));
    float best = __builtin_inff();
    // The walk's current octant lives in registers -- its slot base, mask and low corner, and dj, this lane's
    // child distance (+inf: absent, outside the pyramid, or taken) -- and its ancestors in LDS, saved when the walk
    // descends and reloaded when it pops (launch_beam sizes it: (64 + 5 x 8) x depth x 4 B, 3.3 KB at depth 8):
    // st_d[level][thread], and per group the slot base, mask and corner (every lane of a group writes the same
    // value: no lane-0 branch).  Taking a leaf touches no memory at all.
    extern __shared__ uint32_t beam_lds[];
    const uint32_t t = threadIdx.x, L = beam_levels(S.depth);
    constexpr uint32_t G = 64u / kBeamLanes;
    float *const st_d = reinterpret_cast<float *>(beam_lds);
    uint32_t *const st_base = beam_lds + L * 64u, *const st_mask = st_base + L * G;
    float *const st_lx = reinterpret_cast<float *>(st_mask + L * G), *const st_ly = st_lx + L * G, *const st_lz = st_ly + L * G;
    // the minimum of a lane value over the group's 8 lanes in three DPP moves: xor 1 and xor 2 inside each quad
    // (quad_perm 1,0,3,2 and 2,3,0,1), then the half-row mirror (lane i <- 7 - i) between the two quads
    auto grp_min = [](uint32_t k) {
        k = min(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0xB1, 0xF, 0xF, false));
        k = min(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x4E, 0xF, 0xF, false));
        k = min(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x141, 0xF, 0xF, false));
        return k;
    };
    // the box distance of child `lane` of the octant at `lo` (children of size hc), or -1 outside the pyramid
    auto child_box = [&](v3 lo, float hc) -> float {
        return box(V(lo.x + ((lane & 1u) ? hc : 0.0f), lo.y + ((lane & 2u) ? hc : 0.0f), lo.z + ((lane & 4u) ? hc : 0.0f)),
                   hc);
    };
    auto present_d = [&](float db, uint32_t m) { return (((m >> lane) & 1u) != 0u && db >= 0.0f) ? db : __builtin_inff(); };
    bool exhausted = S.depth >= (uint32_t)kBeamLevels;
    uint32_t nodes = 1u;  // octants the walk entered (the root included)
    if (!exhausted && box(V(1.0f, 1.0f, 1.0f), 1.0f) >= 0.0f) {
        int lv = 0;
        uint32_t cbase = S.root, cmask = S.root_mask;
        v3 clo = V(1.0f, 1.0f, 1.0f);
        float dj = present_d(child_box(clo, 0.5f), cmask);
        uint32_t visits = 0u;
        for (;;) {  // group-uniform control flow: every decision below is the group's
            // the nearest child still nearer than best: its distance's bits (>= 0, so ordered as unsigned) with the
            // lane in the low 3 bits, minimised over the group
            const uint32_t k = grp_min(dj < best ? ((__float_as_uint(dj) & ~7u) | lane) : 0xFFFFFFFFu);
            if (k == 0xFFFFFFFFu) {  // this octant is done: back to its parent
                if (--lv < 0) break;
                dj = st_d[lv * 64 + t];
                cbase = st_base[lv * G + grp];
                cmask = st_mask[lv * G + grp];
                clo = V(st_lx[lv * G + grp], st_ly[lv * G + grp], st_lz[lv * G + grp]);
                continue;
            }
            if (++visits > kBeamVisits) { exhausted = true; break; }
            const uint32_t ci = k & 7u;
            // its distance with the low 3 bits cleared: at most 7 ulp below it, so best, and the start, can only
            // come out nearer (conservative), and every octant nearer than the final start is still entered
            const float d = __uint_as_float(k & ~7u);
            if (lane == ci) dj = __builtin_inff();
            const uint32_t kind = (cmask >> ci) & 0x101u;
            const float h = __uint_as_float((126u - (uint32_t)lv) << 23);  // 2^-(lv + 1)
            if (kind == 0x101u || lv + 1 >= (int)L || h <= lod * d) { best = d; continue; }  // leaf / small cell
            const uint2 slot = S.node_child[cbase + __popc(cmask & ((1u << ci) - 1u))];
            st_d[lv * 64 + t] = dj;  // this octant's remaining children, for the pop back to it
            st_base[lv * G + grp] = cbase;
            st_mask[lv * G + grp] = cmask;
            st_lx[lv * G + grp] = clo.x;
            st_ly[lv * G + grp] = clo.y;
            st_lz[lv * G + grp] = clo.z;
            clo = V(clo.x + ((ci & 1u) ? h : 0.0f), clo.y + ((ci & 2u) ? h : 0.0f), clo.z + ((ci & 4u) ? h : 0.0f));
            const float db = child_box(clo, h * 0.5f);  // while the slot is in flight
            ++lv;
            ++nodes;
            cbase = slot.x;
            cmask = slot.y;
            dj = present_d(db, cmask);
        }
    }
    if (lane == 0u) beam[tile] = exhausted ? 0.0f : beam_pack(best * (1.0f - 0x1p-16f), nodes);
}
#else
__global__ __launch_bounds__(64) void beam_kernel(DevScene S, DevCamera C, DevRender R, uint32_t n_tiles,
                                                  float *__restrict__ beam) {
    // thread i: beam tile i % kBeamSub of the shard's render tile i / kBeamSub (item_pixel's tile order),
    // so a rank of N computes only its own tiles' starts
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= n_tiles) return;
    const uint32_t rt = dealt_tile(R.tile_order, R.shard_index + (i / kBeamSub) * R.shard_count), sub = i % kBeamSub;
    const uint32_t rty = udiv_c(rt, R.div_tiles_x);
    const uint32_t x0 = (rt - rty * R.tiles_x) * kTile + (sub % (kTile / kBeamTile)) * kBeamTile,
                   y0 = rty * kTile + (sub / (kTile / kBeamTile)) * kBeamTile;
    if (x0 >= R.W || y0 >= R.H) return;  // no pixel of the image: never read
    const uint32_t tile = (y0 / kBeamTile) * R.beam_tx + x0 / kBeamTile;
    const uint32_t x1 = min(x0 + kBeamTile, R.W), y1 = min(y0 + kBeamTile, R.H);
    // screen coordinates of the tile's rays (new_path: xn + dx, yn + dy), padded by 2 % + 1e-6
    float s0 = ((float)(2u * x0) - (float)R.W) / R.dim, s1 = ((float)(2u * x1) - (float)R.W) / R.dim;
    float t0 = ((float)(2u * (R.H - y1)) - (float)R.H) / R.dim, t1 = ((float)(2u * (R.H - y0)) - (float)R.H) / R.dim;
    const float ps = 0.02f * (s1 - s0) + 1e-6f, pt = 0.02f * (t1 - t0) + 1e-6f;
    s0 -= ps; s1 += ps; t0 -= pt; t1 += pt;
    const v3 F = vscale(V(C.dir[0], C.dir[1], C.dir[2]), C.d_factor);
    const v3 Rt = V(C.right[0], C.right[1], C.right[2]), Up = V(C.up[0], C.up[1], C.up[2]);
    const v3 Ek[4] = {vadd(vadd(F, vscale(Rt, s0)), vscale(Up, t0)), vadd(vadd(F, vscale(Rt, s1)), vscale(Up, t0)),
                      vadd(vadd(F, vscale(Rt, s1)), vscale(Up, t1)), vadd(vadd(F, vscale(Rt, s0)), vscale(Up, t1))};
    const v3 Ec = vadd(vadd(F, vscale(Rt, 0.5f * (s0 + s1))), vscale(Up, 0.5f * (t0 + t1)));
    v3 pn[4];
    for (int k = 0; k < 4; ++k) {
        v3 n = vcross(Ek[k], Ek[(k + 1) & 3]);
        if (vdot(n, Ec) < 0.0f) n = vscale(n, -1.0f);
        pn[k] = n;
    }
    // the eye as esvo_begin places a ray origin in octree space
    const v3 e = vadd(vscale(V(C.eye[0], C.eye[1], C.eye[2]), S.octree_scale), V(1.0f, 1.0f, 1.0f));
    const uint32_t om = (Ec.x < 0.0f ? 1u : 0u) | (Ec.y < 0.0f ? 2u : 0u) | (Ec.z < 0.0f ? 4u : 0u);
    // distance from the eye to the box [lo, lo + h], or -1 when the box lies outside the pyramid
    auto box = [&](v3 lo, float h) -> float {
        const v3 a = vsub(lo, e), b = vsub(vadd(lo, V(h, h, h)), e);
        const float ext = fmaxf(fmaxf(fmaxf(fabsf(a.x), fabsf(b.x)), fmaxf(fabsf(a.y), fabsf(b.y))),
                                fmaxf(fabsf(a.z), fabsf(b.z)));
        for (int k = 0; k < 4; ++k) {
            const v3 n = pn[k];
            const float mx = (fmaxf(n.x * a.x, n.x * b.x) + fmaxf(n.y * a.y, n.y * b.y)) + fmaxf(n.z * a.z, n.z * b.z);
            const float tol = 1e-5f * ((fabsf(n.x) + fabsf(n.y)) + fabsf(n.z)) * ext;
            if (mx < -tol) return -1.0f;
        }
        const float dx = a.x > 0.0f ? a.x : (b.x < 0.0f ? -b.x : 0.0f);
        const float dy = a.y > 0.0f ? a.y : (b.y < 0.0f ? -b.y : 0.0f);
        const float dz = a.z > 0.0f ? a.z : (b.z < 0.0f ? -b.z : 0.0f);
        return sqrtf((dx * dx + dy * dy) + dz * dz);
    };
    // an octant whose cell is at most kBeamLod tile footprints wide at its distance counts as a leaf
    // (conservative: it holds all its leaves; 0 = walk down to the leaf cells)
    const float lod = kBeamLod * fmaxf(s1 - s0, t1 - t0) / sqrtf(vdot(F, F));
    float best = __builtin_inff();
    // the walk's stack in LDS, [level][thread], for the scene's depth levels (launch_beam sizes it:
    // 6 x depth x 64 x 4 B, 12 KB at depth 8, so that 10+ blocks share a CU instead of 4 at a fixed 24
    // levels): octant base, mask, children still to visit (in front-to-back order: bit k = child k ^ om)
    // and the cell's low corner
    extern __shared__ uint32_t beam_lds[];
    const uint32_t t = threadIdx.x, L = beam_levels(S.depth);
    uint32_t *const st_base = beam_lds, *const st_mask = beam_lds + L * 64u, *const st_rem = beam_lds + 2u * L * 64u;
    float *const st_lx = reinterpret_cast<float *>(beam_lds + 3u * L * 64u);
    float *const st_ly = reinterpret_cast<float *>(beam_lds + 4u * L * 64u);
    float *const st_lz = reinterpret_cast<float *>(beam_lds + 5u * L * 64u);
    auto order = [&](uint32_t m) {  // present children, permuted so that bit k = child k ^ om
        uint32_t pm = m & 0xFFu;
        if (om & 1u) pm = ((pm & 0x55u) << 1) | ((pm >> 1) & 0x55u);
        if (om & 2u) pm = ((pm & 0x33u) << 2) | ((pm >> 2) & 0x33u);
        if (om & 4u) pm = ((pm & 0x0Fu) << 4) | ((pm >> 4) & 0x0Fu);
        return pm;
    };
    bool exhausted = S.depth >= (uint32_t)kBeamLevels;
    uint32_t nodes = 1u;  // octants the walk entered (the root included)
    if (!exhausted && box(V(1.0f, 1.0f, 1.0f), 1.0f) >= 0.0f) {
        int lv = 0;
        st_base[t] = S.root;
        st_mask[t] = S.root_mask;
        st_rem[t] = order(S.root_mask);
        st_lx[t] = st_ly[t] = st_lz[t] = 1.0f;
        uint32_t visits = 0u;
        while (lv >= 0) {
            const uint32_t rem = st_rem[lv * 64 + t];
            if (rem == 0u) { --lv; continue; }
            if (++visits > kBeamVisits) { exhausted = true; break; }
            st_rem[lv * 64 + t] = rem & (rem - 1u);
            const uint32_t ci = (uint32_t)(__ffs(rem) - 1) ^ om;
            const uint32_t m = st_mask[lv * 64 + t], kind = (m >> ci) & 0x101u;
            const float h = __uint_as_float((126u - (uint32_t)lv) << 23);  // 2^-(lv + 1)
            const v3 lo = V(st_lx[lv * 64 + t] + ((ci & 1u) ? h : 0.0f), st_ly[lv * 64 + t] + ((ci & 2u) ? h : 0.0f),
                            st_lz[lv * 64 + t] + ((ci & 4u) ? h : 0.0f));
            const float d = box(lo, h);
            if (d < 0.0f || d >= best) continue;
            if (kind == 0x101u || lv + 1 >= (int)L || h <= lod * d) { best = d; continue; }  // leaf / small cell
            const uint2 slot = S.node_child[st_base[lv * 64 + t] + __popc(m & ((1u << ci) - 1u))];
            ++lv;
            ++nodes;
            st_base[lv * 64 + t] = slot.x;
            st_mask[lv * 64 + t] = slot.y;
            st_rem[lv * 64 + t] = order(slot.y);
            st_lx[lv * 64 + t] = lo.x;
            st_ly[lv * 64 + t] = lo.y;
            st_lz[lv * 64 + t] = lo.z;
        }
    }
    beam[tile] = exhausted ? 0.0f : beam_pack(best * (1.0f - 0x1p-16f), nodes);
}

#endif

__global__ void tonemap_kernel(const float4 *__restrict__ accum, uchar4 *__restrict__ out, uint32_t n,
                               const uint8_t *__restrict__ lut) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 c = accum[i];
    const float r = fminf(c.x * 255.0f, 255.0f), g = fminf(c.y * 255.0f, 255.0f), b = fminf(c.z * 255.0f, 255.0f),
                a = fminf(c.w * 255.0f, 255.0f);
    out[i] = make_uchar4(lut[f2u32_sat(r)], lut[f2u32_sat(g)], lut[f2u32_sat(b)], (uint8_t)f2u32_sat(a));
}

// tile_pos (nullable): frame tile -> dealing position, the inverse of the tile order (octpt_set_tile_order)
__global__ void unshard_kernel(uint32_t W, uint32_t H, uint32_t N, const uint32_t *__restrict__ tile_pos,
                               const float4 *__restrict__ shards, uint32_t stride, float4 *__restrict__ frame) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W * H) return;
    const uint32_t x = i % W, y = i / W;
    const uint32_t tiles_x = (W + kTile - 1u) / kTile;
    const uint32_t t = dealt_tile(tile_pos, (y / kTile) * tiles_x + x / kTile);
    const uint32_t shard = t % N, lt = t / N;
    frame[i] = shards[(size_t)shard * stride + (size_t)lt * 64u + (y % kTile) * kTile + (x % kTile)];
}

// a multi-device render's scatter (to_stage) / gather of the caller's buffers (multi_slot)
__global__ void multi_stage_kernel(DevRender R, uint32_t n_dev, uint32_t stride, float4 *__restrict__ accum,
                                   uint32_t *__restrict__ seg, float4 *__restrict__ stage_accum,
                                   uint32_t *__restrict__ stage_seg, uint32_t to_stage) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R.total_items) return;
    uint32_t c, st;
    if (!multi_slot(R.W, R.H, R.tiles_x, R.shard_index, R.shard_count, R.compact != 0u, n_dev, stride, i, c, st,
                    R.tile_order))
        return;
    if (to_stage) {
        stage_accum[st] = accum[c];
        if (seg) stage_seg[st] = seg[c];
    } else {
        accum[c] = stage_accum[st];
        if (seg) seg[c] = stage_seg[st];
    }
}

}  // namespace

// ESVO stack levels 1..depth-1 (level 0 is never used, see esvo_step)
size_t render_lds_bytes(uint32_t depth) { return (size_t)(depth - 1u) * kBlock * (sizeof(uint2) + sizeof(uint16_t)); }

int render_blocks_per_cu(uint32_t depth) {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void *>(render_kernel<true, kPrimsModels>),
                                                     kBlock, render_lds_bytes(depth)) != hipSuccess)
        return 1;
    return blocks > 0 ? blocks : 1;
}

// the extend instance a scene launches: the primitive kinds it holds (sphere-only scenes: no slab test)
static const void *extend_instance(const DevScene &S) {
    if (S.has_blocks) return reinterpret_cast<const void *>(wf_extend_kernel<kPrimsBlocks>);
    if (S.has_models) return reinterpret_cast<const void *>(wf_extend_kernel<kPrimsModels>);
    if (S.has_cuboids) return reinterpret_cast<const void *>(wf_extend_kernel<kPrimsBoxes>);
    return reinterpret_cast<const void *>(wf_extend_kernel<kPrimsSpheres>);
}

int extend_blocks_per_cu(const DevScene &S) {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, extend_instance(S), kBlock, render_lds_bytes(S.depth)) !=
        hipSuccess)
        return 1;
    return blocks > 0 ? blocks : 1;
}

hipError_t launch_preview(const DevScene &S0, const DevCamera &C, const DevRender &R, float4 *accum,
                          uint32_t *segcount, unsigned long long *stats, hipStream_t stream) {
    const DevScene &S = S0;
    const uint32_t grid = (R.total_items + kBlock - 1u) / kBlock;
    // the primitive kinds of the scene pick the instance, as for wf_extend_kernel
    const void *fn = S.has_blocks   ? reinterpret_cast<const void *>(preview_kernel<kPrimsBlocks>)
                     : S.has_models ? reinterpret_cast<const void *>(preview_kernel<kPrimsModels>)
                     : S.has_cuboids ? reinterpret_cast<const void *>(preview_kernel<kPrimsBoxes>)
                                     : reinterpret_cast<const void *>(preview_kernel<kPrimsSpheres>);
    void *args[] = {const_cast<DevScene *>(&S), const_cast<DevCamera *>(&C), const_cast<DevRender *>(&R), &accum,
                    &segcount, &stats};
    const hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(kBlock), args,
                                         render_lds_bytes(S.depth), stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_render(const DevScene &S0, const DevCamera &C, const DevRender &R, float4 *accum, uint32_t *segcount,
                         uint32_t *counter, unsigned long long *stats, int grid, hipStream_t stream) {
    const DevScene &S = S0;
    // the general instance (spheres, cuboids, cuboid models) or the block-value one (C23)
    auto kern = S.sun.sun_sampling ? (S.has_blocks ? render_kernel<true, kPrimsBlocks> : render_kernel<true, kPrimsModels>)
                                   : (S.has_blocks ? render_kernel<false, kPrimsBlocks> : render_kernel<false, kPrimsModels>);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), render_lds_bytes(S.depth), stream, S, C, R, accum, segcount,
                       counter, stats);
    return hipGetLastError();
}

hipError_t launch_wf_seed(const DevCamera &C, const DevRender &R, const WaveBuffers &B, uint32_t n_seed,
                          uint32_t chunk_items, unsigned long long *stats, hipStream_t stream) {
    // direct seeding: kSegs segments x ceil(largest shard / 64) waves (each shard <= ceil(n / kSegs))
    const uint64_t threads = n_seed == chunk_items
                                 ? (uint64_t)kSegs * ((((uint64_t)chunk_items + kSegs - 1u) / kSegs + 63u) / 64u) * 64u
                                 : (uint64_t)n_seed;
    hipLaunchKernelGGL(wf_seed_kernel, dim3((uint32_t)((threads + kBlock - 1u) / kBlock)), dim3(kBlock), 0, stream, C, R, B, n_seed,
                       chunk_items, stats);
    return hipGetLastError();
}

hipError_t launch_wf_extend(const DevScene &S, const WaveBuffers &B, uint32_t q, bool cam, uint32_t refill, int grid,
                            unsigned long long *stats, hipStream_t stream) {
    // refill 0: the adaptive threshold; cam: queue q holds the seed's camera records (refill bit 31)
    uint32_t rf = refill | (cam ? 0x80000000u : 0u);
    void *args[] = {const_cast<DevScene *>(&S), const_cast<WaveBuffers *>(&B), &q, &rf, &stats};
    const hipError_t e = hipLaunchKernel(extend_instance(S), dim3(grid), dim3(kBlock), args, render_lds_bytes(S.depth),
                                         stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

#ifndef OCTPT_SHADE_FIRST_SPLIT
#define OCTPT_SHADE_FIRST_SPLIT 1  // round 6: C3 +0.2..0.4 %, C5b +0.2..0.6 %, C4 +0.25 % (profiles/r06/shade_first_split_ab.txt)
#endif
// the shade instance a scene and chunk launch (sun sampling, LDS material tables, regeneration, lean state; with
// OCTPT_SHADE_FIRST_SPLIT the lean state's later launches, first == false, take the instance without the rebuild)
#ifndef OCTPT_SHADE_COLOUR
#define OCTPT_SHADE_COLOUR 1  // sphere scenes with colour textures only get an instance without the image path (A/B knob)
#endif
#ifndef OCTPT_SHADE_PRIMS
#define OCTPT_SHADE_PRIMS 1  // round 6: the lean instance per primitive kind (C3 +0.15..0.35 %, profiles/r06/shade_prims_ab.txt)
#endif
template <bool kLds, int kSP>
static const void *lean_shade_of(bool first) {
    return (OCTPT_SHADE_FIRST_SPLIT && !first) ? reinterpret_cast<const void *>(wf_shade_kernel<false, kLds, 2, true, kSP>)
                                                : reinterpret_cast<const void *>(wf_shade_kernel<false, kLds, 2, false, kSP>);
}
template <bool kNee, bool kLds>
static const void *shade_instance_of(int mode, bool first, int prims) {
    if (!kNee && mode == 2) {  // the lean instances: per primitive kind (OCTPT_SHADE_PRIMS) and by launch (first)
        if (OCTPT_SHADE_PRIMS && prims == kShadeSphColour) return lean_shade_of<kLds, kShadeSphColour>(first);
        if (OCTPT_SHADE_PRIMS && prims == kPrimsSpheres) return lean_shade_of<kLds, kPrimsSpheres>(first);
        if (OCTPT_SHADE_PRIMS && prims == kPrimsBoxes) return lean_shade_of<kLds, kPrimsBoxes>(first);
        if (OCTPT_SHADE_PRIMS && prims == kPrimsBlocks) return lean_shade_of<kLds, kPrimsBlocks>(first);
        return lean_shade_of<kLds, kPrimsModels>(first);
    }
    return mode == 1 ? reinterpret_cast<const void *>(wf_shade_kernel<kNee, kLds, 1>)
                     : reinterpret_cast<const void *>(wf_shade_kernel<kNee, kLds, 0>);
}
bool shade_lds_tables(const DevScene &S) { return S.n_mats <= kShadeLdsMats && S.n_texs <= kShadeLdsMats; }
static const void *shade_instance(const DevScene &S, int mode, bool first = false) {
    const bool lds = shade_lds_tables(S);
    const int prims = S.has_blocks    ? kPrimsBlocks
                      : S.has_models  ? kPrimsModels
                      : S.has_cuboids ? kPrimsBoxes
                      : S.has_images  ? kPrimsSpheres
                                      : (OCTPT_SHADE_COLOUR ? kShadeSphColour : kPrimsSpheres);
    return S.sun.sun_sampling
               ? (lds ? shade_instance_of<true, true>(mode, first, prims) : shade_instance_of<true, false>(mode, first, prims))
               : (lds ? shade_instance_of<false, true>(mode, first, prims) : shade_instance_of<false, false>(mode, first, prims));
}

int shade_blocks_per_cu(const DevScene &S, int mode) {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, shade_instance(S, mode), kBlock, 0) != hipSuccess)
        return 4;
    return blocks > 0 ? blocks : 1;
}

hipError_t launch_wf_shade(const DevScene &S, const DevCamera &C, const DevRender &R, const WaveBuffers &B, uint32_t q,
                           uint32_t chunk_items, uint32_t first, bool regen, int grid, unsigned long long *stats,
                           hipStream_t stream) {
    uint32_t first_u = first;
    void *args[] = {const_cast<DevScene *>(&S), const_cast<DevCamera *>(&C), const_cast<DevRender *>(&R),
                    const_cast<WaveBuffers *>(&B), &q, &chunk_items, &first_u, &stats};
    const hipError_t e = hipLaunchKernel(shade_instance(S, shade_mode(regen, B.lean != 0u), first != 0u), dim3(grid),
                                         dim3(kBlock), args, 0, stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_wf_drain(const DevScene &S, const DevRender &R, const WaveBuffers &B, uint32_t q, int grid,
                           unsigned long long *stats, hipStream_t stream) {
    const bool nee = S.sun.sun_sampling != 0;
    const void *fn = S.has_blocks ? (nee ? reinterpret_cast<const void *>(wf_drain_kernel<kPrimsBlocks, true>)
                                         : reinterpret_cast<const void *>(wf_drain_kernel<kPrimsBlocks, false>))
                     : S.has_models ? (nee ? reinterpret_cast<const void *>(wf_drain_kernel<kPrimsModels, true>)
                                         : reinterpret_cast<const void *>(wf_drain_kernel<kPrimsModels, false>))
                     : S.has_cuboids ? (nee ? reinterpret_cast<const void *>(wf_drain_kernel<kPrimsBoxes, true>)
                                            : reinterpret_cast<const void *>(wf_drain_kernel<kPrimsBoxes, false>))
                                     : (nee ? reinterpret_cast<const void *>(wf_drain_kernel<kPrimsSpheres, true>)
                                            : reinterpret_cast<const void *>(wf_drain_kernel<kPrimsSpheres, false>));
    void *args[] = {const_cast<DevScene *>(&S), const_cast<DevRender *>(&R), const_cast<WaveBuffers *>(&B), &q, &stats};
    const hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(kBlock), args, render_lds_bytes(S.depth), stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

// The host steering's snapshot (enqueue_wavefront): thread t < kSegs copies segment t's count of queue q,
// thread kSegs + t shard t's item counter, into pinned host memory -- one small launch in the stream
// instead of two strided device-to-host copies per iteration.
__global__ __launch_bounds__(2 * kSegs) void wf_snapshot_kernel(const uint32_t *__restrict__ ctrl, uint32_t q,
                                                                uint32_t *__restrict__ host_out) {
    const uint32_t t = threadIdx.x;
    host_out[t] = ctrl[t < kSegs ? ctr_count(q, t) : ctr_item(t - kSegs)];
}

hipError_t launch_wf_snapshot(const WaveBuffers &B, uint32_t q, uint32_t *host_out, hipStream_t stream) {
    hipLaunchKernelGGL(wf_snapshot_kernel, dim3(1), dim3(2 * kSegs), 0, stream, B.ctrl, q, host_out);
    return hipGetLastError();
}

hipError_t launch_wf_resolve(const DevRender &R, const WaveBuffers &B, uint32_t chunk_spp, float4 *accum,
                             uint32_t *segcount, hipStream_t stream) {
    hipLaunchKernelGGL(wf_resolve_kernel, dim3((R.total_items + kBlock - 1u) / kBlock), dim3(kBlock), 0, stream, R, B,
                       chunk_spp, accum, segcount);
    return hipGetLastError();
}

hipError_t launch_intersect(const DevScene &S0, const float *rays, const uint32_t *last_prim, const float *last_normal,
                            uint32_t n, float *t, uint32_t *prim, float *normal, uint32_t *steps, hipStream_t stream) {
    const DevScene &S = S0;
    const uint32_t grid = (n + kBlock - 1u) / kBlock;
    hipLaunchKernelGGL(S.has_blocks ? intersect_kernel<kPrimsBlocks> : intersect_kernel<kPrimsModels>, dim3(grid),
                       dim3(kBlock), render_lds_bytes(S.depth), stream, S, rays, last_prim, last_normal, n, t, prim,
                       normal, steps);
    return hipGetLastError();
}

hipError_t launch_beam(const DevScene &S, const DevCamera &C, const DevRender &R, float *beam, hipStream_t stream) {
    const uint32_t n = R.shard_tiles * kBeamSub;  // the shard's render tiles' beam tiles
#if OCTPT_BEAM_COOP
    const size_t lds = (64u + 5u * (64u / kBeamLanes)) * beam_levels(S.depth) * sizeof(uint32_t);
    const uint32_t per_block = 64u / kBeamLanes;
#else
    const size_t lds = 6u * beam_levels(S.depth) * 64u * sizeof(uint32_t);
    const uint32_t per_block = 64u;
#endif
    hipLaunchKernelGGL(beam_kernel, dim3((n + per_block - 1u) / per_block), dim3(64), lds, stream, S, C, R, n, beam);
    return hipGetLastError();
}

hipError_t launch_tonemap(const float4 *accum, uchar4 *out, uint32_t n, const uint8_t *lut_byte, hipStream_t stream) {
    hipLaunchKernelGGL(tonemap_kernel, dim3((n + 255u) / 256u), dim3(256), 0, stream, accum, out, n, lut_byte);
    return hipGetLastError();
}

hipError_t launch_multi_stage(const DevRender &R, uint32_t n_dev, uint32_t stride, float4 *accum, uint32_t *seg,
                              float4 *stage_accum, uint32_t *stage_seg, bool to_stage, hipStream_t stream) {
    hipLaunchKernelGGL(multi_stage_kernel, dim3((R.total_items + 255u) / 256u), dim3(256), 0, stream, R, n_dev, stride,
                       accum, seg, stage_accum, stage_seg, to_stage ? 1u : 0u);
    return hipGetLastError();
}

hipError_t launch_unshard(uint32_t W, uint32_t H, uint32_t shard_count, const uint32_t *tile_pos, const float4 *shards,
                          uint32_t stride, float4 *frame, hipStream_t stream) {
    hipLaunchKernelGGL(unshard_kernel, dim3((W * H + 255u) / 256u), dim3(256), 0, stream, W, H, shard_count, tile_pos,
                       shards, stride, frame);
    return hipGetLastError();
}

}  // namespace octpt
