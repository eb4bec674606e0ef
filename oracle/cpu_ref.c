/*
 * oracle/cpu_ref.c -- CPU restatement of the kekley/octree_pathtracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see cpu_ref.h).  This is the parity checker and the
 * CPU baseline ("port") -- never part of the product.  PARITY UNPINNED for the path
 * tracer proper: the reference cannot run and holds no golden vectors for it; the
 * Morton functions are pinned by the reference's own tests (new_octree.rs:866-884).
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * reference root).  Where the reference is a stub or buggy, the numbered
 * semantics-contract item of DESIGN.md §3 is cited as [Cn].
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#include "cpu_ref.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* constants                                                                  */
/* ------------------------------------------------------------------------- */
#define RAY_EPSILON 0.00000005f      /* src/ray/mod.rs:26 */
#define RAY_OFFSET 0.000001f         /* src/ray/mod.rs:27 */
#define OCTREE_MAX_STEPS 1000        /* src/octree/octree_traversal.rs:13 */
#define OCTREE_MAX_SCALE 23          /* src/octree/octree_traversal.rs:14 */
#define OCTREE_EPSILON 1.1920929e-7f /* src/octree/octree_traversal.rs:15 */
#define MAX_DST_WORLD 1024.0f        /* src/scene/mod.rs:181 */
#define PI_F 3.14159265358979323846f /* std::f32::consts::PI */
#define SUN_MAX_IMPORTANCE_SAMPLE_CHANCE 0.9f /* src/scene/mod.rs:313 */
#define CELL_TOL 0.001f              /* [C1] leaf span tolerance, in cell sizes */
#define PRIM_NONE 0xFFFFFFFFu
#define PRIM_CUBOID_BIT 0x80000000u
#define MAT_FLAG_REFRACTIVE 0x4u     /* src/textures/material.rs:104 */
#define MAT_FLAG_SUBSURFACE 0x2u     /* MaterialFlags::SUBSURFACE_SCATTER, src/textures/material.rs:9 */
#ifndef MAX_PATH_SEGMENTS
#define MAX_PATH_SEGMENTS 64u        /* [C15] next_intersection calls per path */
#endif

/* ------------------------------------------------------------------------- */
/* small f32 vector helpers -- glam Vec3A semantics with explicit op order     */
/* ------------------------------------------------------------------------- */
typedef struct { float x, y, z; } v3;
static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
/* glam dot3: (x*x + y*y) + z*z */
static inline float vdot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* glam cross: (a.y*b.z - b.y*a.z, a.z*b.x - b.z*a.x, a.x*b.y - b.x*a.y) */
static inline v3 vcross(v3 a, v3 b) {
    return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
/* glam normalize: self * (1.0 / sqrt(dot(self,self))) */
static inline v3 vnorm(v3 a) {
    float r = 1.0f / sqrtf(vdot(a, a));
    return vscale(a, r);
}
static inline float fmin_(float a, float b) { return a < b ? a : b; }
static inline float fmax_(float a, float b) { return a > b ? a : b; }
static inline float vmin3(v3 a) { return fmin_(fmin_(a.x, a.y), a.z); }
static inline float vmax3(v3 a) { return fmax_(fmax_(a.x, a.y), a.z); }
static inline float vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void vset(v3 *a, int i, float f) {
    if (i == 0) a->x = f; else if (i == 1) a->y = f; else a->z = f;
}
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
/* Rust f32::signum: +1 for +0/positive, -1 for -0/negative */
static inline float signum_(float f) { return (f2u(f) >> 31) ? -1.0f : 1.0f; }
/* Rust `f32 as u32`: saturating, NaN -> 0 */
static inline uint32_t f2u32_sat(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 4294967295.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}
static inline int visfinite(v3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }

/* ------------------------------------------------------------------------- */
/* portable f32 math.  Cephes-style single precision          */
/* polynomials; only + - * / sqrt, floor, no contraction.  Replaces glibc/Rust  */
/* libm for the per-bounce transcendentals so device and host agree bitwise.   */
/* ------------------------------------------------------------------------- */
#define PIO2_HI 1.5703125f
#define PIO2_MID 4.837512969970703125e-4f
#define PIO2_LO 7.54978995489188216e-8f
#define TWO_OVER_PI 0.636619772367581343f

static void sincos_core(float x, float *s, float *c) {
    float kf = floorf(x * TWO_OVER_PI + 0.5f);
    int k = (int)kf;
    float r = ((x - kf * PIO2_HI) - kf * PIO2_MID) - kf * PIO2_LO;
    float z = r * r;
    float sp = r + r * z * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
    float cp = (1.0f - 0.5f * z) +
               z * z * (4.166664568298827e-2f + z * (-1.388731625493765e-3f + z * 2.443315711809948e-5f));
    switch (k & 3) {
    case 0: *s = sp; *c = cp; break;
    case 1: *s = cp; *c = -sp; break;
    case 2: *s = -sp; *c = -cp; break;
    default: *s = -cp; *c = sp; break;
    }
}
float ref_math_sin(float x) { float s, c; sincos_core(x, &s, &c); return s; }
float ref_math_cos(float x) { float s, c; sincos_core(x, &s, &c); return c; }

float ref_math_asin(float x) {
    float a = fabsf(x), z, xx;
    int flag = 0;
    if (a > 0.5f) {
        z = 0.5f * (1.0f - a);
        xx = sqrtf(z);
        flag = 1;
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
float ref_math_acos(float x) {
    if (x < -0.5f) return PI_F - 2.0f * ref_math_asin(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * ref_math_asin(sqrtf(0.5f * (1.0f - x)));
    return 1.5707963267948966f - ref_math_asin(x);
}
static float atan_core(float x) {
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
    float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x + x);
    return sgn < 0.0f ? -y : y;
}
float ref_math_atan2(float y, float x) {
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
    return w + atan_core(y / x);
}
/* f32::hypot restated as sqrt(x*x + y*y) in f32 [C11] */
float ref_math_hypot(float x, float y) { return sqrtf(x * x + y * y); }

/* ------------------------------------------------------------------------- */
/* counter-based RNG [C10] (replaces StdRng::from_os_rng, tile_renderer.rs:692) */
/* ------------------------------------------------------------------------- */
static inline uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
uint32_t ref_rng_path_state(uint32_t seed, uint32_t pixel, uint32_t sample) {
    uint32_t h = lowbias32(seed ^ 0xA511E9B3u);
    h = lowbias32(h ^ pixel);
    h = lowbias32(h ^ (sample * 0x9E3779B9u));
    return h;
}
/* random_float (util.rs:14-17): uniform [0,1) from the top 24 bits */
float ref_rng_next(uint32_t *state) {
    uint32_t s = *state * 747796405u + 2891336453u;
    *state = s;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    w = (w >> 22u) ^ w;
    return (float)(w >> 8) * (1.0f / 16777216.0f);
}

/* ------------------------------------------------------------------------- */
/* Morton codes, src/octree/new_octree.rs:752-835                              */
/* ------------------------------------------------------------------------- */
static uint64_t part_by_2(uint64_t v) { /* new_octree.rs:813-822 */
    uint64_t x = v & 0x1fffff;
    x = (x | x << 32) & 0x1f00000000ffffULL;
    x = (x | x << 16) & 0x1f0000ff0000ffULL;
    x = (x | x << 8) & 0x100f00f00f00f00fULL;
    x = (x | x << 4) & 0x10c30c30c30c30c3ULL;
    x = (x | x << 2) & 0x1249249249249249ULL;
    return x;
}
static uint64_t compact_by_2(uint64_t v) { /* new_octree.rs:824-833 */
    uint64_t x = v & 0x1249249249249249ULL;
    x = (x | x >> 2) & 0x10c30c30c30c30c3ULL;
    x = (x | x >> 4) & 0x100f00f00f00f00fULL;
    x = (x | x >> 8) & 0x1f0000ff0000ffULL;
    x = (x | x >> 16) & 0x1f00000000ffffULL;
    x = (x | x >> 32) & 0x1fffffULL;
    return x;
}
uint64_t ref_morton_encode(uint64_t x, uint64_t y, uint64_t z) { /* new_octree.rs:752-755 */
    return (part_by_2(z) << 2) + (part_by_2(y) << 1) + part_by_2(x);
}
static uint32_t MORTON_X[4096], MORTON_Y[4096], MORTON_Z[4096];
static pthread_once_t morton_once = PTHREAD_ONCE_INIT;
static void morton_init(void) { /* new_octree.rs:761-795 */
    for (uint32_t i = 0; i < 4096; i++) {
        MORTON_X[i] = (uint32_t)part_by_2(i);
        MORTON_Y[i] = (uint32_t)(part_by_2(i) << 1);
        MORTON_Z[i] = (uint32_t)(part_by_2(i) << 2);
    }
}
uint64_t ref_morton_encode_lut(uint64_t x, uint64_t y, uint64_t z) { /* new_octree.rs:797-799 */
    pthread_once(&morton_once, morton_init);
    return (uint64_t)(MORTON_Z[z] + MORTON_Y[y] + MORTON_X[x]);
}
void ref_morton_decode(uint64_t code, uint64_t *x, uint64_t *y, uint64_t *z) { /* new_octree.rs:802-808 */
    *x = compact_by_2(code);
    *y = compact_by_2(code >> 1);
    *z = compact_by_2(code >> 2);
}
uint64_t ref_morton_lut_selftest(uint32_t n) { /* new_octree.rs:876-884 */
    pthread_once(&morton_once, morton_init);
    uint64_t bad = 0;
    for (uint64_t x = 0; x < n; x++)
        for (uint64_t y = 0; y < n; y++)
            for (uint64_t z = 0; z < n; z++)
                bad += (ref_morton_encode(x, y, z) != (uint64_t)(MORTON_Z[z] + MORTON_Y[y] + MORTON_X[x]));
    return bad;
}

/* ------------------------------------------------------------------------- */
/* colour LUTs, src/textures/texture.rs:42-62                                   */
/* ------------------------------------------------------------------------- */
static float LUT_FLOAT[256];
static uint8_t LUT_BYTE[256];
static pthread_once_t lut_once = PTHREAD_ONCE_INIT;
static void lut_init(void) {
    for (int i = 0; i < 256; i++) {
        LUT_FLOAT[i] = powf((float)i / 255.0f, 2.2f);                       /* texture.rs:52 */
        LUT_BYTE[i] = (uint8_t)f2u32_sat(powf((float)i / 255.0f, 1.0f / 2.2f) * 255.0f); /* :59 */
    }
}
float ref_lut_float(uint32_t i) { pthread_once(&lut_once, lut_init); return LUT_FLOAT[i & 255]; }
uint8_t ref_lut_byte(uint32_t i) { pthread_once(&lut_once, lut_init); return LUT_BYTE[i & 255]; }

/* TileRenderer::get_current_branch_count (tile_renderer.rs:196-206) [C20] */
uint32_t ref_branch_count(uint32_t current_spp, uint32_t scene_branch_count) {
    if (current_spp < scene_branch_count) {
        if (current_spp <= (uint32_t)sqrtf((float)scene_branch_count)) return 1;
        return scene_branch_count - current_spp;
    }
    return scene_branch_count;
}

/* RNG stream of branch b > 0 of a split path [C20]: a lowbias32 hash of the stream state at the
 * split and the branch index */
uint32_t ref_rng_branch_state(uint32_t state, uint32_t b) { return lowbias32(state ^ (b * 0x632BE5ABu)); }

/* ------------------------------------------------------------------------- */
/* scene-derived constants: Sun::new (scene/mod.rs:321-383)                     */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 sw, su, sv;
    float radius, width, width2;
    float tex[4];                 /* sun Texture::Color value */
    float isect_mul[3];           /* apparent_texture_brightness * 10 */
    float diffuse_mul[3];         /* color * 10 */
    int draw_texture;
    float luminosity;
    float emit[3];                /* Sun::emmittance = color * INTENSITY^GAMMA (scene/mod.rs:352-353) */
    /* diffuse_reflection importance sampling (ray/mod.rs:227-258) */
    float sun_dx, sun_dy, sun_dz, circle_radius, sample_chance;
    int importance_sampling, diffuse_sun;
    /* next-event estimation (path_tracer.rs:225-291, 458-483) */
    int sun_sampling, strict_direct_light;
    float lum_a;      /* sun_luminosity ? luminosity_pdf : 1 (path_tracer.rs:250-254) */
    float radius_cos; /* Sun::radius_cos (scene/mod.rs:331) */
} sun_k;

typedef struct {
    const ref_scene *s;
    sun_k sun;
    float octree_scale;
    uint32_t max_depth, branch_count; /* branch_count: the schedule's ceiling B [C20] */
    uint32_t cur_bc;                  /* this pass's branch count get_current_branch_count(spp, B) */
    int forward;
    uint32_t path_segs; /* next_intersection calls of the current path [C15] */
    ref_stats st;
} ctx_t;

static void tex_value_color(const uint8_t rgba[4], float out[4]) { /* colors/mod.rs:280-288 */
    out[0] = LUT_FLOAT[rgba[0]];
    out[1] = LUT_FLOAT[rgba[1]];
    out[2] = LUT_FLOAT[rgba[2]];
    out[3] = (float)rgba[3] / 255.0f;
}

static void sun_init(const ref_sun *p, sun_k *k) {
    float theta = p->azimuth, phi = p->altitude;
    float r = fabsf(cosf(phi));
    k->sw = V(cosf(theta) * r, sinf(phi), sinf(theta) * r);
    v3 su = fabsf(k->sw.x) > 0.1f ? V(0, 1, 0) : V(1, 0, 0);
    v3 sv = vnorm(vcross(k->sw, su));
    su = vcross(sv, k->sw);
    k->su = su;
    k->sv = sv;
    k->radius = p->radius;
    k->width = p->radius * 4.0f;
    k->width2 = k->width * 2.0f;
    float gamma_b = powf(1.25f, 2.2f); /* INTENSITY.powf(GAMMA), scene/mod.rs:352-360 */
    float atb[3];
    for (int i = 0; i < 3; i++) atb[i] = (p->texture_modification ? p->apparent_color[i] : 1.0f) * gamma_b;
    tex_value_color(p->texture_rgba, k->tex);
    for (int i = 0; i < 3; i++) {
        k->isect_mul[i] = atb[i] * 10.0f;
        k->diffuse_mul[i] = p->color[i] * 10.0f;
        k->emit[i] = p->color[i] * gamma_b;
    }
    k->draw_texture = p->draw_texture;
    k->luminosity = p->luminosity;
    /* ray/mod.rs:228-237 */
    float az = p->azimuth, alt_fake = p->altitude;
    float alt = fabsf(alt_fake) > PI_F / 2.0f ? signum_(alt_fake) * PI_F - alt_fake : alt_fake;
    k->sun_dx = cosf(az) * cosf(alt);
    k->sun_dz = sinf(az) * cosf(alt);
    k->sun_dy = sinf(alt);
    k->circle_radius = p->radius * p->importance_sample_radius; /* :258 */
    k->sample_chance = p->importance_sample_chance;
    k->importance_sampling = p->importance_sampling;
    k->diffuse_sun = p->diffuse_sun;
    k->sun_sampling = p->sun_sampling;
    k->strict_direct_light = p->strict_direct_light;
    k->lum_a = p->sun_luminosity ? p->luminosity_pdf : 1.0f;
    k->radius_cos = cosf(p->radius);
}

/* ------------------------------------------------------------------------- */
/* ray + hit record, src/ray/mod.rs:16-23, src/hittable/mod.rs:53-84            */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 o, d;
    float t, u, v;
    uint32_t cur_mat, prev_mat;
    v3 n;
    float col[4];
    uint32_t depth;
    int specular;
    uint32_t last_prim; /* [C2] self-intersection key */
} ray_t;

static void ray_new(ray_t *r, v3 o, v3 d) { /* ray/mod.rs:32-49 + HitRecord::default */
    memset(r, 0, sizeof(*r));
    r->o = o;
    r->d = d;
    r->t = INFINITY;
    r->specular = 1;
    r->last_prim = PRIM_NONE;
}
static inline v3 ray_at(const ray_t *r, float t) { return vadd(r->o, vscale(r->d, t)); } /* mod.rs:29-31 */
static void new_from_self(const ray_t *src, ray_t *dst) { /* mod.rs:51-70 */
    ray_t r = *src;
    r.t = 0.0f;
    r.col[0] = r.col[1] = r.col[2] = r.col[3] = 0.0f;
    *dst = r;
}
/* inv_dir rule of Ray::set_direction (mod.rs:91-112) [C12: always derived from direction] */
static inline float inv_clamped(float d) { return fabsf(d) < 1e-6f ? 1.0f / 1e-6f : 1.0f / d; }

/* ------------------------------------------------------------------------- */
/* textures, src/textures/texture.rs:64-93 (+ rtw_image.rs:234-237, [C9])       */
/* ------------------------------------------------------------------------- */
static void texture_value_n(ctx_t *c, uint32_t tex_idx, float u, float v, float out[4], int count) {
    const ref_scene *s = c->s;
    const ref_texture *t = &s->textures[tex_idx];
    if (t->kind == 0) { tex_value_color(t->rgba, out); return; }
    if (t->height == 0) { out[0] = out[1] = out[2] = out[3] = 1.0f; return; }
    float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
    float vv = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    vv = 1.0f - vv;
    uint32_t i = f2u32_sat(uu * (float)t->width);
    uint32_t j = f2u32_sat(vv * (float)t->height);
    if (i > t->width - 1) i = t->width - 1;
    if (j > t->height - 1) j = t->height - 1;
    const uint8_t *px = s->texels + t->offset + ((uint64_t)j * t->width + i) * 4u;
    if (count) c->st.texel_reads++;
    out[0] = LUT_FLOAT[px[0]];
    out[1] = LUT_FLOAT[px[1]];
    out[2] = LUT_FLOAT[px[2]];
    out[3] = (float)px[3] / 255.0f;
}
static void texture_value(ctx_t *c, uint32_t tex_idx, float u, float v, float out[4]) {
    texture_value_n(c, tex_idx, u, v, out, 1);
}

/* ------------------------------------------------------------------------- */
/* primitives                                                                  */
/* ------------------------------------------------------------------------- */
typedef struct {
    float t;
    int inside;  /* origin inside the primitive: exit hit */
    int axis;    /* cuboid face axis */
    v3 n;        /* outward normal */
    int64_t quad;        /* block-model hit: the global quad index, else -1 [C19] */
    float alpha, beta;   /* its Quad::hit barycentrics */
    int64_t block;       /* block-value leaf hit [C23]: the block id, else -1 */
    int face;            /* its face (Face enum index) */
    float u, v;          /* its texture coordinates (octree_traversal.rs:159-190, |u|, |v|) */
} prim_hit;

/* Sphere::hit dead code after todo!() (geometry/sphere.rs:33-57) + [C2] root selection */
static int sphere_test(const float *sp, const ray_t *r, int self_prim, prim_hit *h) {
    v3 c = V(sp[0], sp[1], sp[2]);
    float rad = sp[3];
    v3 oc = vsub(c, r->o);
    float a = vdot(r->d, r->d);
    float hh = vdot(r->d, oc);
    float cc = vdot(oc, oc) - rad * rad;
    float disc = hh * hh - a * cc;
    if (disc < 0.0f) return 0;
    float sq = sqrtf(disc);
    float t0 = (hh - sq) / a;
    float t1 = (hh + sq) / a;
    if (self_prim) {
        if (vdot(r->d, r->n) < 0.0f && t1 > RAY_EPSILON) { h->t = t1; h->inside = 1; return 1; }
        return 0;
    }
    if (t0 > RAY_EPSILON) { h->t = t0; h->inside = 0; return 1; }
    if (t1 > RAY_EPSILON) { h->t = t1; h->inside = 1; return 1; }
    return 0;
}

/* AABB::intersects_new slab (geometry/aabb.rs:172-191) [C3] */
static int cuboid_test(const float *bx, const ray_t *r, int self_prim, prim_hit *h) {
    v3 inv = V(inv_clamped(r->d.x), inv_clamped(r->d.y), inv_clamped(r->d.z));
    v3 bmin = V(bx[0], bx[1], bx[2]), bmax = V(bx[3], bx[4], bx[5]);
    v3 tb = vmul(vsub(bmin, r->o), inv);
    v3 tt = vmul(vsub(bmax, r->o), inv);
    v3 mins = V(fmin_(tb.x, tt.x), fmin_(tb.y, tt.y), fmin_(tb.z, tt.z));
    v3 maxs = V(fmax_(tb.x, tt.x), fmax_(tb.y, tt.y), fmax_(tb.z, tt.z));
    float t0 = vmax3(mins), t1 = vmin3(maxs);
    if (!isfinite(t0)) t0 = t1;
    if (t1 < t0) return 0;
    int inside;
    float t;
    if (self_prim) {
        if (!(vdot(r->d, r->n) < 0.0f && t1 > RAY_EPSILON)) return 0;
        inside = 1; t = t1;
    } else if (t0 > RAY_EPSILON) {
        inside = 0; t = t0;
    } else if (t1 > RAY_EPSILON) {
        inside = 1; t = t1;
    } else {
        return 0;
    }
    int axis;
    if (!inside) axis = (mins.x == t0) ? 0 : ((mins.y == t0) ? 1 : 2);
    else axis = (maxs.x == t1) ? 0 : ((maxs.y == t1) ? 1 : 2);
    float ia = vget(inv, axis);
    /* entry through the min face when moving +axis; exit through the max face */
    float sgn = inside ? (ia > 0.0f ? 1.0f : -1.0f) : (ia > 0.0f ? -1.0f : 1.0f);
    h->n = V(0, 0, 0);
    vset(&h->n, axis, sgn);
    h->t = t;
    h->inside = inside;
    h->axis = axis;
    return 1;
}

/* ---- block models [C19] ---- */
#define MODEL_NONE 0xFFFFFFFFu
#define QUAD_KEY 0x40000000u /* last_prim of a ray leaving quad q: QUAD_KEY | q */
typedef struct { v3 o, u, v, w, n; float d; } quad_geo;

/* Quad::new (geometry/quad.rs:90-114): n = u x v, normal = normalize(n), w = n / n.n, d = normal.origin */
static quad_geo quad_geometry(const ref_quad *q) {
    quad_geo g;
    g.o = V(q->origin[0], q->origin[1], q->origin[2]);
    g.u = V(q->u[0], q->u[1], q->u[2]);
    g.v = V(q->v[0], q->v[1], q->v[2]);
    v3 n = vcross(g.u, g.v);
    g.n = vnorm(n);
    float nn = vdot(n, n);
    g.w = V(n.x / nn, n.y / nn, n.z / nn);
    g.d = vdot(g.n, g.o);
    return g;
}

/* Quad::hit (geometry/quad.rs:172-200): voxel-local, back faces culled, 0 < t <= t_next */
static int quad_hit(const quad_geo *g, const ray_t *r, v3 voxel, float t_next, float *t_out, float *alpha,
                    float *beta) {
    v3 tro = vsub(r->o, voxel);
    float denom = vdot(r->d, g->n);
    if (denom >= -RAY_EPSILON) return 0;
    float t = (g->d - vdot(g->n, tro)) / denom;
    if (t <= 0.0f || t > t_next) return 0;
    v3 inter = vadd(tro, vscale(r->d, t));
    v3 planar = vsub(inter, g->o);
    float a = vdot(g->w, vcross(planar, g->v));
    float b = vdot(g->w, vcross(g->u, planar));
    if (!(a >= 0.0f && a <= 1.0f) || !(b >= 0.0f && b <= 1.0f)) return 0;
    *t_out = t;
    *alpha = a;
    *beta = b;
    return 1;
}

/* a block-model leaf (ResourceModel::Quad, octree_traversal.rs:207-213) [C19]: the closest of the
 * model's quads with 0 < t <= t_accept, ties to the later quad (`t > t_next` rejects), skipping
 * the quad the ray leaves */
static int model_test_at(const ref_scene *s, const ray_t *r, v3 voxel, uint32_t mdl, float t_accept, prim_hit *h) {
    uint32_t first = s->model_quads[2 * (size_t)mdl], cnt = s->model_quads[2 * (size_t)mdl + 1];
    float t_next = t_accept;
    int found = 0;
    for (uint32_t k = 0; k < cnt; k++) {
        uint32_t q = first + k;
        if ((QUAD_KEY | q) == r->last_prim) continue;
        quad_geo g = quad_geometry(&s->quads[q]);
        float t, a, b;
        if (quad_hit(&g, r, voxel, t_next, &t, &a, &b)) {
            t_next = t;
            h->quad = q;
            h->alpha = a;
            h->beta = b;
            h->n = g.n;
            found = 1;
        }
    }
    h->t = t_next;
    h->inside = 0;
    h->axis = 0;
    return found;
}
static int model_test(const ref_scene *s, const ray_t *r, uint32_t ci, uint32_t mdl, float t_accept, prim_hit *h) {
    const float *bx = &s->cuboids[6 * (size_t)ci];
    return model_test_at(s, r, V(bx[0], bx[1], bx[2]), mdl, t_accept, h);
}

/* Face enum index from outward normal (geometry/cuboid.rs:9-29) */
static inline int face_index(int axis, float sgn) {
    if (axis == 0) return sgn < 0.0f ? 0 : 1; /* West(-X), East(+X) */
    if (axis == 1) return sgn < 0.0f ? 2 : 3; /* Bottom(-Y), Top(+Y) */
    return sgn > 0.0f ? 4 : 5;                /* South(+Z), North(-Z) */
}

/* Commit a primitive hit into the ray (Chunky semantics, [C1]): origin moves to the hit. */
static void commit_hit(ctx_t *c, ray_t *r, uint32_t prim, const prim_hit *h) {
    const ref_scene *s = c->s;
    v3 p = ray_at(r, h->t);
    float u, v;
    uint32_t mat;
    v3 n;
    if (h->block >= 0 && h->quad < 0) { /* a block filling its leaf cell [C23]: face and uv from ESVO */
        n = h->n;
        u = h->u;
        v = h->v;
        mat = s->block_mat[6 * (size_t)h->block + (size_t)h->face];
        prim = PRIM_NONE; /* no self-intersection key: a ray starting in a block's cell skips it (t_min == 0) */
    } else if (h->quad >= 0) { /* block-model quad [C19]: uv from the barycentrics (quad.rs:194-197) */
        const ref_quad *q = &s->quads[h->quad];
        n = h->n;
        u = q->texture_u_range[0] + h->alpha * (q->texture_u_range[1] - q->texture_u_range[0]);
        v = q->texture_v_range[0] + h->beta * (q->texture_v_range[1] - q->texture_v_range[0]);
        mat = q->material;
        prim = QUAD_KEY | (uint32_t)h->quad;
    } else if (!(prim & PRIM_CUBOID_BIT)) {
        const float *sp = &s->spheres[4 * (size_t)prim];
        v3 cen = V(sp[0], sp[1], sp[2]);
        float rad = sp[3];
        n = V((p.x - cen.x) / rad, (p.y - cen.y) / rad, (p.z - cen.z) / rad); /* sphere.rs:51 */
        float theta = ref_math_acos(-n.y);                                    /* sphere.rs:60-69 */
        float phi = ref_math_atan2(-n.z, n.x) + PI_F;
        u = phi / (2.0f * PI_F);
        v = theta / PI_F;
        mat = s->sphere_material[prim];
    } else {
        uint32_t ci = prim & ~PRIM_CUBOID_BIT;
        const float *bx = &s->cuboids[6 * (size_t)ci];
        n = h->n;
        float sgn = vget(n, h->axis);
        float ex = bx[3] - bx[0], ey = bx[4] - bx[1], ez = bx[5] - bx[2];
        /* per-face UV as the ESVO leaf (octree_traversal.rs:163-190) */
        if (h->axis == 0) {
            u = (p.z - bx[2]) / ez; v = (p.y - bx[1]) / ey;
            if (r->d.x < 0.0f) u = 1.0f - u;
        } else if (h->axis == 1) {
            u = (p.x - bx[0]) / ex; v = (p.z - bx[2]) / ez;
            if (r->d.y < 0.0f) v = 1.0f - v;
        } else {
            u = (p.x - bx[0]) / ex; v = (p.y - bx[1]) / ey;
            if (r->d.z < 0.0f) u = 1.0f - u;
        }
        u = fabsf(u); /* Cuboid::intersect_texture (cuboid.rs:73-90) */
        v = fabsf(v);
        mat = s->cuboid_material[6 * (size_t)ci + face_index(h->axis, sgn)];
    }
    r->o = p;
    r->t = h->t;
    r->n = n;
    r->u = u;
    r->v = v;
    r->last_prim = prim;
    if (h->inside) { /* [C2] leaving the primitive: enter the outer medium (material 0) */
        r->cur_mat = 0;
        r->col[0] = r->col[1] = r->col[2] = r->col[3] = 0.0f;
    } else {
        r->cur_mat = mat;
        texture_value(c, s->materials[mat].texture_index, u, v, r->col);
    }
}

/* child mask of an octant in the reader form [C21]: OctantChildIterator reads bit i = present,
 * bit i+8 = leaf (new_octree.rs:84-100), while Octant::set_mask_for (:160-178), the reference's
 * only writer, stores ChildType::Octant as bit i+8 alone.  (0,1) is therefore an octant child. */
static inline uint16_t octant_mask(const ref_scene *s, uint32_t octant) {
    uint32_t m = s->octant_mask[octant];
    uint32_t present = m & 0xFFu, high = m >> 8;
    return (uint16_t)((present | (high & ~present)) | ((present & high) << 8));
}

/* closest primitive of one leaf list whose hit lies before the cell exit [C1] */
static int leaf_test(ctx_t *c, const ray_t *r, uint32_t leaf, float t_exit_w, float cell_w, uint32_t *best_prim,
                     prim_hit *best) {
    const ref_scene *s = c->s;
    uint32_t first = s->leaf_first[leaf], cnt = s->leaf_count[leaf];
    float t_accept = t_exit_w + CELL_TOL * cell_w;
    int found = 0;
    c->st.leaf_visits++;
    for (uint32_t k = 0; k < cnt; k++) {
        uint32_t prim = s->leaf_prims[first + k];
        prim_hit h;
        int self_prim = (prim == r->last_prim);
        int ok;
        c->st.prim_tests++;
        h.quad = -1;
        h.block = -1;
        uint32_t mdl = (prim & PRIM_CUBOID_BIT) && s->cuboid_model ? s->cuboid_model[prim & ~PRIM_CUBOID_BIT] : MODEL_NONE;
        if (!(prim & PRIM_CUBOID_BIT)) ok = sphere_test(&s->spheres[4 * (size_t)prim], r, self_prim, &h);
        else if (mdl != MODEL_NONE) ok = model_test(s, r, prim & ~PRIM_CUBOID_BIT, mdl, t_accept, &h);
        else ok = cuboid_test(&s->cuboids[6 * (size_t)(prim & ~PRIM_CUBOID_BIT)], r, self_prim, &h);
        if (ok && h.t <= t_accept && (!found || h.t < best->t)) {
            *best = h;
            *best_prim = prim;
            found = 1;
        }
    }
    return found;
}

/* A block-value leaf [C23]: the leaf payload is a block id and the block's box is the leaf cell itself,
 * at any level (the reference's own leaf form: new_octree.rs:534-537, 586, 669, 727).  Restates the
 * leaf arm of intersect_octree_path_tracer (octree_traversal.rs:143-214) from its ESVO state:
 *  - the unmirrored cell corner (:149-154) and the cell's entry t-values at pos + scale_exp2 (:156);
 *  - the face is the axis of their maximum, UV the entry point's other two coordinates over the cell
 *    (:159-190), flipped where the ray runs negative; |u|, |v| as Cuboid::intersect_texture
 *    (cuboid.rs:73-90).  The face id :164 is written 1 << 0 | sign for X, which always names East: the
 *    pattern of :173 / :182 (2 * axis + sign) is taken for all three axes, like the RGBA stride of C9;
 *  - ResourceModel::SingleBlock (:193-206): skipped when t_min == 0 (the ray starts inside the cell: the
 *    next block's face, not this one's, is hit), else SingleBlockModel::intersect -- undefined in the
 *    reference -- is the face material's texel at (u, v): a hit unless its alpha <= EPSILON (a
 *    transparent texel: ESVO advances, :215), hit t = t_min / octree_scale (:197);
 *  - ResourceModel::Quad (:207-213): the block's model (C19) at the cell's world corner
 *    ((pos - 1) / octree_scale, unit-voxel quads), closest quad before the cell exit + tolerance (C1). */
static int block_leaf_test(ctx_t *c, const ray_t *r, uint32_t block, v3 pos, float scale_exp2, v3 ro, v3 rd,
                           v3 t_coef, v3 t_bias, uint32_t mirror, float t_min, float tc_max, prim_hit *h) {
    const ref_scene *s = c->s;
    const float octree_scale = c->octree_scale;
    c->st.leaf_visits++;
    c->st.block_tests++;
    v3 upos = pos; /* :149-154 */
    for (int i = 0; i < 3; i++)
        if (mirror & (1u << i)) vset(&upos, i, (3.0f - scale_exp2) - vget(pos, i));
    h->quad = -1;
    h->block = block;
    const uint32_t mdl = s->block_model ? s->block_model[block] : MODEL_NONE;
    if (mdl != MODEL_NONE) { /* :207-213 */
        v3 voxel = V((upos.x - 1.0f) / octree_scale, (upos.y - 1.0f) / octree_scale, (upos.z - 1.0f) / octree_scale);
        float t_accept = tc_max / octree_scale + CELL_TOL * (scale_exp2 / octree_scale);
        return model_test_at(s, r, voxel, mdl, t_accept, h);
    }
    if (t_min == 0.0f) return 0; /* :194 */
    const float se = scale_exp2;
    v3 tcn = vsub(vmul(vadd(pos, V(se, se, se)), t_coef), t_bias); /* :156 */
    float tc_min = vmax3(tcn);
    int axis;
    float u, v;
    if (tcn.x == tc_min) { /* :163-171 */
        axis = 0;
        u = ((ro.z + rd.z * tcn.x) - upos.z) / se;
        v = ((ro.y + rd.y * tcn.x) - upos.y) / se;
        if (rd.x < 0.0f) u = 1.0f - u;
    } else if (tcn.y == tc_min) { /* :172-180 */
        axis = 1;
        u = ((ro.x + rd.x * tcn.y) - upos.x) / se;
        v = ((ro.z + rd.z * tcn.y) - upos.z) / se;
        if (rd.y < 0.0f) v = 1.0f - v;
    } else { /* :181-189 */
        axis = 2;
        u = ((ro.x + rd.x * tcn.z) - upos.x) / se;
        v = ((ro.y + rd.y * tcn.z) - upos.y) / se;
        if (rd.z < 0.0f) u = 1.0f - u;
    }
    u = fabsf(u);
    v = fabsf(v);
    const float sgn = vget(rd, axis) < 0.0f ? 1.0f : -1.0f; /* the face the ray enters faces against it */
    const int face = face_index(axis, sgn);
    const uint32_t mat = s->block_mat[6 * (size_t)block + (size_t)face];
    float col[4];
    texture_value_n(c, s->materials[mat].texture_index, u, v, col, 0); /* the alpha test reads no counted texel */
    if (!(col[3] > RAY_EPSILON)) return 0;
    h->t = t_min / octree_scale;
    h->inside = 0;
    h->axis = axis;
    h->n = V(0.0f, 0.0f, 0.0f);
    vset(&h->n, axis, sgn);
    h->face = face;
    h->u = u;
    h->v = v;
    return 1;
}

#ifdef REF_ESVO_TRACE
/* diagnostic build only (tools/esvo_trace.py): one byte per ESVO iteration, single-threaded renders.
 * low 3 bits: 0 advance over an absent child, 1 leaf test missed, 2 leaf hit, 3 descend, 4 advance
 * past a present child not entered; 8 = the advance popped; 16 = first iteration of a ray; 32 = the ray
 * leaves a primitive (a bounce / continue ray, last_prim set) */
static uint8_t *g_trace;
static size_t g_trace_n, g_trace_cap;
static int g_trace_first, g_trace_bounce;
static void trace_put(int code) {
    if (g_trace_n < g_trace_cap)
        g_trace[g_trace_n++] = (uint8_t)(code | (g_trace_first ? 16 : 0) | (g_trace_bounce ? 32 : 0));
    g_trace_first = 0;
}
void ref_esvo_trace_set(uint8_t *buf, size_t cap) { g_trace = buf; g_trace_cap = cap; g_trace_n = 0; }
size_t ref_esvo_trace_len(void) { return g_trace_n; }
#define TRACE(c) trace_put(c)
#define TRACE_BEGIN() (g_trace_first = 1, g_trace_bounce = ray->last_prim != PRIM_NONE)
#else
#define TRACE(c) ((void)0)
#define TRACE_BEGIN() ((void)0)
#endif

/* ------------------------------------------------------------------------- */
/* ESVO traversal: Octree::intersect_octree_path_tracer                        */
/* src/octree/octree_traversal.rs:54-302                                        */
/* ------------------------------------------------------------------------- */
static int esvo(ctx_t *c, const ray_t *ray, float max_dst_w, uint32_t *hit_prim, prim_hit *hit, uint32_t *steps_out) {
    const ref_scene *s = c->s;
    float octree_scale = c->octree_scale;
    uint32_t st_node[OCTREE_MAX_SCALE + 1];
    float st_t[OCTREE_MAX_SCALE + 1];
    memset(st_node, 0, sizeof st_node);
    memset(st_t, 0, sizeof st_t);
    uint32_t steps = 0;
    v3 ro = vscale(ray->o, octree_scale);        /* :71 */
    v3 rd = ray->d;                               /* :73 */
    float max_dst = max_dst_w * octree_scale;     /* :75 */
    ro = vadd(ro, V(1.0f, 1.0f, 1.0f));           /* :77 */
    uint32_t parent = s->root;
    uint32_t scale = OCTREE_MAX_SCALE - 1;
    float scale_exp2 = 0.5f;
    for (int i = 0; i < 3; i++) {                 /* :84-93 epsilon clamp */
        float di = vget(rd, i);
        if (fabsf(di) < OCTREE_EPSILON) vset(&rd, i, u2f((f2u(OCTREE_EPSILON) & 0x7FFFFFFFu) | (f2u(di) & 0x80000000u)));
    }
    /* :95 uses the pre-clamp |rd|, which makes the clamp dead and yields NaN for exact-zero
     * components; [C13] takes |rd| after the clamp as ESVO intends. */
    v3 rd_abs = V(fabsf(rd.x), fabsf(rd.y), fabsf(rd.z));
    v3 t_coef = V(1.0f / -rd_abs.x, 1.0f / -rd_abs.y, 1.0f / -rd_abs.z);
    v3 t_bias = vmul(t_coef, ro);                 /* :97 */
    uint32_t mirror = 0;                          /* :99-106 */
    for (int i = 0; i < 3; i++)
        if (vget(rd, i) > 0.0f) {
            mirror |= 1u << i;
            vset(&t_bias, i, 3.0f * vget(t_coef, i) - vget(t_bias, i));
        }
    float t_min = fmax_(vmax3(vsub(vscale(t_coef, 2.0f), t_bias)), 0.0f); /* :107 */
    float t_max = vmin3(vsub(t_coef, t_bias));                          /* :109 */
    float h = t_max;
    uint32_t idx = 0;
    v3 pos = V(1.0f, 1.0f, 1.0f);
    v3 upper = vsub(vscale(t_coef, 1.5f), t_bias);                       /* :116-125 */
    for (int i = 0; i < 3; i++)
        if (vget(upper, i) > t_min) { idx ^= 1u << i; vset(&pos, i, 1.5f); }

    TRACE_BEGIN();
    for (int it = 0; it < OCTREE_MAX_STEPS; it++) {                      /* :127 */
        if (max_dst >= 0.0f && t_min > max_dst) break;
        steps++;
        int tcode = 4;
        v3 t_corner = vsub(vmul(pos, t_coef), t_bias);
        float tc_max = vmin3(t_corner);
        uint32_t cidx = idx ^ mirror;
        uint16_t mask = octant_mask(s, parent);
        uint32_t payload = s->octant_children[8 * (size_t)parent + cidx];
        c->st.node_fetches++;
        int present = (mask >> cidx) & 1, is_leaf = (mask >> (cidx + 8)) & 1;
        if (present && t_min <= t_max) {                                  /* :142 */
            if (is_leaf && t_min >= 0.0f) {                                /* :143 */
                float cell_w = scale_exp2 / octree_scale;
                tcode = 1;
                int found = s->block_mat
                                ? block_leaf_test(c, ray, payload, pos, scale_exp2, ro, rd, t_coef, t_bias, mirror,
                                                  t_min, tc_max, hit)
                                : leaf_test(c, ray, payload, tc_max / octree_scale, cell_w, hit_prim, hit);
                if (found && s->block_mat) *hit_prim = payload;
                if (found) {
                    TRACE(2);
                    *steps_out = steps;
                    return 1;
                }
            } else {
                float half = scale_exp2 * 0.5f;                            /* :217-244 */
                v3 t_center = vadd(vscale(t_coef, half), t_corner);
                float tv_max = fmin_(t_max, tc_max);
                if (t_min <= tv_max && !is_leaf) {
                    if (tc_max < h) { st_node[scale] = parent; st_t[scale] = t_max; }
                    h = tc_max;
                    parent = payload;
                    scale -= 1;
                    scale_exp2 = half;
                    idx = 0;
                    for (int i = 0; i < 3; i++)
                        if (vget(t_center, i) > t_min) { idx ^= 1u << i; vset(&pos, i, vget(pos, i) + scale_exp2); }
                    t_max = tv_max;
                    TRACE(3);
                    continue;
                }
            }
        }
        if (!present) tcode = 0;
        uint32_t step_mask = 0;                                           /* :249-260 advance */
        for (int i = 0; i < 3; i++)
            if (vget(t_corner, i) <= tc_max) { step_mask ^= 1u << i; vset(&pos, i, vget(pos, i) - scale_exp2); }
        t_min = tc_max;
        idx ^= step_mask;
        TRACE(tcode | ((idx & step_mask) != 0 ? 8 : 0));
        (void)tcode;
        if ((idx & step_mask) != 0) {                                     /* :262-299 pop */
            uint32_t diff = 0;
            if (step_mask & 1) diff |= f2u(pos.x) ^ f2u(pos.x + scale_exp2);
            if (step_mask & 2) diff |= f2u(pos.y) ^ f2u(pos.y + scale_exp2);
            if (step_mask & 4) diff |= f2u(pos.z) ^ f2u(pos.z + scale_exp2);
            scale = diff ? 31u - (uint32_t)__builtin_clz(diff) : 0xFFFFFFFFu; /* util.rs:121-133 */
            if (scale >= OCTREE_MAX_SCALE) break;
            scale_exp2 = u2f((scale - OCTREE_MAX_SCALE + 127u) << 23); /* exp2(scale-23), exact */
            parent = st_node[scale];
            t_max = st_t[scale];
            uint32_t shx = f2u(pos.x) >> scale, shy = f2u(pos.y) >> scale, shz = f2u(pos.z) >> scale;
            pos = V(u2f(shx << scale), u2f(shy << scale), u2f(shz << scale));
            idx = (shx & 1) | ((shy & 1) << 1) | ((shz & 1) << 2);
            h = 0.0f;
        }
    }
    *steps_out = steps;
    return 0;
}

/* Scene::hit (scene/mod.rs:172-187) with the octree call restored [C1]; sets the hit record */
static int scene_hit(ctx_t *c, ray_t *r) {
    v3 d = r->d;
    if ((d.x == 0.0f && d.y == 0.0f && d.z == 0.0f) || isnan(d.x) || isnan(d.y) || isnan(d.z))
        r->d = V(0.0f, 1.0f, 0.0f); /* UP, aabb.rs:11 */
    uint32_t prim = PRIM_NONE, steps = 0;
    prim_hit h;
    int hit = esvo(c, r, MAX_DST_WORLD, &prim, &h, &steps);
    c->st.esvo_steps += steps;
    if (hit) commit_hit(c, r, prim, &h);
    return hit;
}

/* next_intersection, path_tracer.rs:438-446 */
static int next_intersection(ctx_t *c, ray_t *r, uint32_t *segs) {
    r->prev_mat = r->cur_mat;
    r->t = INFINITY;
    c->st.segments++;
    c->path_segs++;
    if (c->path_segs > c->st.max_path_segs) c->st.max_path_segs = c->path_segs;
    (*segs)++;
    return scene_hit(c, r);
}

/* ------------------------------------------------------------------------- */
/* sky + sun (scene/mod.rs:216-268, 384-426)                                   */
/* ------------------------------------------------------------------------- */
static const float SKY_COLOR[4] = {0.5f, 0.7f, 1.0f, 1.0f}; /* scene/mod.rs:170 */
static int sun_intersect(const sun_k *k, ray_t *r) { /* :384-405 */
    v3 d = r->d;
    if (!k->draw_texture || vdot(d, k->sw) < 0.5f) return 0;
    float a = PI_F / 2.0f - ref_math_acos(vdot(d, k->su)) + k->width;
    if (a >= 0.0f && a < k->width2) {
        float b = PI_F / 2.0f - ref_math_acos(vdot(d, k->sv)) + k->width;
        if (b >= 0.0f && b < k->width2) {
            for (int i = 0; i < 4; i++) r->col[i] = k->tex[i];
            for (int i = 0; i < 3; i++) r->col[i] *= k->isect_mul[i];
            return 1;
        }
    }
    return 0;
}
static int sun_intersect_diffuse(const sun_k *k, ray_t *r) { /* :406-426 */
    v3 d = r->d;
    if (vdot(d, k->sw) < 0.5f) return 0;
    float a = PI_F / 2.0f - ref_math_acos(vdot(d, k->su)) + k->width;
    if (a >= 0.0f && a < k->width2) {
        float b = PI_F / 2.0f - ref_math_acos(vdot(d, k->sv)) + k->width;
        if (b >= 0.0f && b < k->width2) {
            for (int i = 0; i < 4; i++) r->col[i] = k->tex[i];
            for (int i = 0; i < 3; i++) r->col[i] *= k->diffuse_mul[i];
            return 1;
        }
    }
    return 0;
}
static void add_sun_color(const sun_k *k, ray_t *r) { /* :244-253 */
    float cr = r->col[0], cg = r->col[1], cb = r->col[2];
    if (sun_intersect(k, r)) { r->col[0] += cr; r->col[1] += cg; r->col[2] += cb; }
}
static void add_sun_color_diffuse_sun(const sun_k *k, ray_t *r) { /* :255-265 */
    float cr = r->col[0], cg = r->col[1], cb = r->col[2];
    if (sun_intersect_diffuse(k, r)) {
        float m = k->luminosity;
        r->col[0] = r->col[0] * m + cr;
        r->col[1] = r->col[1] * m + cg;
        r->col[2] = r->col[2] * m + cb;
    }
}
static void sky_set(ray_t *r) { memcpy(r->col, SKY_COLOR, sizeof SKY_COLOR); }
static void get_sky_color_interp(const sun_k *k, ray_t *r) { sky_set(r); add_sun_color(k, r); r->col[3] = 1.0f; }
static void get_sky_color(const sun_k *k, ray_t *r, int draw_sun) {
    sky_set(r);
    if (draw_sun) add_sun_color(k, r);
    r->col[3] = 1.0f;
}
static void get_sky_color_diffuse_sun(const sun_k *k, ray_t *r, int diffuse_sun) {
    sky_set(r);
    if (diffuse_sun) add_sun_color_diffuse_sun(k, r);
    r->col[3] = 1.0f;
}

/* ------------------------------------------------------------------------- */
/* scatter kernels, src/ray/mod.rs:113-373                                     */
/* ------------------------------------------------------------------------- */
static void specular_reflection(const ray_t *self, float roughness, uint32_t *rng, ray_t *tmp) { /* :113-184 */
    *tmp = *self;
    tmp->t = INFINITY;
    tmp->u = tmp->v = 0.0f;
    tmp->col[0] = tmp->col[1] = tmp->col[2] = tmp->col[3] = 0.0f;
    tmp->cur_mat = tmp->prev_mat;
    v3 n = self->n, dir = self->d;
    if (roughness > RAY_EPSILON) {
        float sdot = -2.0f * vdot(dir, n);
        v3 spec = vadd(vscale(n, sdot), dir);
        float x1 = ref_rng_next(rng), x2 = ref_rng_next(rng);
        float r = sqrtf(x1), theta = 2.0f * PI_F * x2;
        float tx = r * ref_math_cos(theta), ty = r * ref_math_sin(theta), tz = sqrtf(1.0f - x1);
        v3 tangent = fabsf(n.x) > 0.1f ? V(0, 1, 0) : V(1, 0, 0);
        v3 u = vnorm(vcross(tangent, n));
        v3 v = vcross(n, u);
        v3 nd = vadd(vadd(vscale(u, tx), vscale(v, ty)), vscale(n, tz)); /* Mat3A * Vec3A */
        tmp->d = vnorm(vadd(vscale(nd, roughness), vscale(spec, 1.0f - roughness)));
        tmp->o = ray_at(tmp, RAY_OFFSET);
    } else {
        tmp->d = vsub(dir, vscale(n, 2.0f * vdot(dir, n)));
        tmp->o = ray_at(tmp, RAY_OFFSET);
    }
    if (signum_(vdot(n, tmp->d)) == signum_(vdot(n, dir))) { /* :175-181 */
        float factor = vdot(n, dir) * -RAY_EPSILON - vdot(tmp->d, n);
        tmp->d = vnorm(vadd(tmp->d, vscale(n, factor)));
    }
}

/* Ray::diffuse_reflection, :211-373 (self = next, ray = parent).  Returns the factor the
 * importance-sampling branches multiply ray.hit.color by (:262, 276, 297, 307; 1 when none
 * applies).  do_diffuse_reflection discards it when the sun is not sampled [C5] and uses it when
 * it is (:292 reads ray.hit.color after the call). */
static float diffuse_reflection(ctx_t *c, ray_t *self, const ray_t *ray, uint32_t *rng) {
    float w = 1.0f;
    const sun_k *k = &c->sun;
    new_from_self(ray, self);
    v3 n = self->n;
    float x1 = ref_rng_next(rng), x2 = ref_rng_next(rng);
    float r = sqrtf(x1), theta = 2.0f * PI_F * x2;
    float tx = r * ref_math_cos(theta), ty = r * ref_math_sin(theta);
    if (k->importance_sampling) {
        float sdx = k->sun_dx, sdy = k->sun_dy, sdz = k->sun_dz;
        float stx, sty, sq;
        float stz = (sdx * n.x + sdy * n.y) + sdz * n.z;
        if (fabsf(n.x) > 0.1f) {
            stx = sdx * n.z - sdz * n.x;
            sty = (sdx * n.x * n.y - sdy * (n.x * n.x + n.z * n.z)) + sdz * n.y * n.z;
            sq = ref_math_hypot(n.x, n.z);
        } else {
            stx = sdz * n.y - sdy * n.z;
            sty = (sdy * n.x * n.y - sdx * (n.y * n.y + n.z * n.z)) + sdz * n.x * n.z;
            sq = ref_math_hypot(n.z, n.y);
        }
        stx /= sq;
        sty /= sq;
        float cr = k->circle_radius, chance = k->sample_chance;
        float alt_rel = ref_math_asin(stz);
        if (alt_rel + cr > RAY_EPSILON) {
            if ((ref_math_hypot(stx, sty) + cr) + RAY_EPSILON < 1.0f) {
                if (ref_rng_next(rng) < chance) {
                    tx = stx + tx * cr;
                    ty = sty + ty * cr;
                    w = cr * cr / chance;
                } else {
                    while (ref_math_hypot(tx - stx, ty - sty) < cr) {
                        tx -= stx;
                        ty -= sty;
                        if (tx == 0.0f && ty == 0.0f) break;
                        tx /= cr;
                        ty /= cr;
                    }
                    w = (1.0f - cr * cr) / (1.0f - chance);
                }
            } else {
                float min_r = ref_math_cos(alt_rel + cr);
                float max_r = ref_math_cos(fmax_(alt_rel - cr, 0.0f));
                float sun_theta = ref_math_atan2(sty, stx);
                float seg = ((max_r * max_r - min_r * min_r) * cr) / PI_F;
                chance *= seg / (cr * cr);
                chance = fmin_(chance, SUN_MAX_IMPORTANCE_SAMPLE_CHANCE);
                if (ref_rng_next(rng) < chance) {
                    r = sqrtf(min_r * min_r * x1 + max_r * max_r * (1.0f - x1));
                    theta = sun_theta + (2.0f * x2 - 1.0f) * cr;
                    tx = r * ref_math_cos(theta);
                    ty = r * ref_math_sin(theta);
                    w = seg / chance;
                } else {
                    for (;;) {
                        if (!(r > min_r && r < max_r)) break;
                        /* angle_distance, util.rs:134-137 (fmod exact for diff < 4*pi) */
                        float diff = fabsf(theta - sun_theta);
                        if (diff >= 2.0f * PI_F) diff = diff - 2.0f * PI_F;
                        float ad = diff > PI_F ? 2.0f * PI_F - diff : diff;
                        if (!(ad < cr)) break;
                        x1 = ref_rng_next(rng);
                        x2 = ref_rng_next(rng);
                        r = sqrtf(x1);
                        theta = 2.0f * PI_F * x2;
                    }
                    tx = r * ref_math_cos(theta);
                    ty = r * ref_math_sin(theta);
                    w = (1.0f - seg) / (1.0f - chance);
                }
            }
        }
    }
    float tz = sqrtf((1.0f - tx * tx) - ty * ty);
    float xx, xy, xz;
    if (fabsf(n.x) > 0.1f) { xx = 0.0f; xy = 1.0f; xz = 0.0f; } else { xx = 1.0f; xy = 0.0f; xz = 0.0f; }
    float ux = xy * n.z - xz * n.y, uy = xz * n.x - xx * n.z, uz = xx * n.y - xy * n.x;
    r = 1.0f / sqrtf((ux * ux + uy * uy) + uz * uz);
    ux *= r; uy *= r; uz *= r;
    float vx = uy * n.z - uz * n.y, vy = uz * n.x - ux * n.z, vz = ux * n.y - uy * n.x;
    v3 dir = V((ux * tx + vx * ty) + n.x * tz, (uy * tx + vy * ty) + n.y * tz, (uz * tx + vz * ty) + n.z * tz);
    self->d = dir;
    self->o = ray_at(self, RAY_OFFSET);
    self->cur_mat = self->prev_mat;
    self->specular = 0;
    if (signum_(vdot(n, self->d)) == signum_(vdot(n, ray->d))) { /* :367-372 */
        float factor = signum_(vdot(n, ray->d)) * -RAY_EPSILON - vdot(self->d, self->n);
        self->d = vnorm(vadd(self->d, vscale(n, factor)));
    }
    return w;
}

/* ------------------------------------------------------------------------- */
/* path tracer, src/ray/path_tracer.rs:15-437                                  */
/* ------------------------------------------------------------------------- */
typedef struct { float T[3], L[3]; } fwd_t; /* forward-order accumulation (kernel order) */

static int path_trace(ctx_t *c, ray_t *ray, int first, uint32_t *rng, fwd_t *fw, uint32_t *segs);

static int do_specular_reflection(ctx_t *c, const ray_t *ray, ray_t *next, float cum[4], int do_metal,
                                  uint32_t *rng, fwd_t *fw, uint32_t *segs) { /* :160-188 */
    int hit = 0;
    specular_reflection(ray, c->s->materials[ray->cur_mat].roughness, rng, next);
    if (fw && do_metal) for (int i = 0; i < 3; i++) fw->T[i] = fw->T[i] * ray->col[i];
    if (path_trace(c, next, 0, rng, fw, segs)) {
        if (do_metal) for (int i = 0; i < 3; i++) cum[i] += ray->col[i] * next->col[i];
        else for (int i = 0; i < 3; i++) cum[i] += next->col[i];
        hit = 1;
    }
    return hit;
}

/* get_direct_light_attenuation (path_tracer.rs:458-483): shadow segments toward the sampled sun
 * direction until a miss or an opaque hit, attenuated by each hit's colour and alpha.  The
 * segments share the path's next_intersection cap [C15]; a shadow ray that reaches it counts as
 * occluded [C18]. */
static void direct_light_attenuation(ctx_t *c, ray_t *r, float att[4], uint32_t *segs) {
    att[0] = att[1] = att[2] = att[3] = 1.0f;
    while (att[3] > 0.0f) {
        if (c->path_segs >= MAX_PATH_SEGMENTS) { att[3] = 0.0f; break; } /* [C18] */
        r->o = ray_at(r, RAY_OFFSET);
        if (!next_intersection(c, r, segs)) break;
        float mult = 1.0f - r->col[3];
        for (int i = 0; i < 3; i++) att[i] *= r->col[i] * r->col[3] + mult;
        att[3] *= mult;
        if (c->sun.strict_direct_light &&
            c->s->materials[r->prev_mat].ior != c->s->materials[r->cur_mat].ior)
            att[3] = 0.0f;
    }
}

/* Sun::get_random_sun_direction (scene/mod.rs:427-445): a cone of half-angle `radius` around sw;
 * the result is (u + v) + normalize(w), not normalised, as written */
static v3 random_sun_direction(const sun_k *k, uint32_t *rng) {
    float x1 = ref_rng_next(rng), x2 = ref_rng_next(rng);
    float cos_a = (1.0f - x1) + x1 * k->radius_cos;
    float sin_a = sqrtf(1.0f - cos_a * cos_a);
    float phi = 2.0f * PI_F * x2;
    v3 u = vscale(k->su, ref_math_cos(phi) * sin_a);
    v3 v = vscale(k->sv, ref_math_sin(phi) * sin_a);
    v3 w = vscale(k->sw, cos_a);
    return vadd(vadd(u, v), vnorm(w));
}

/* do_diffuse_reflection's sun-sampling branch (path_tracer.rs:225-291): next-event estimation
 * toward the sun (presets FAST, HIGH_QUALITY), then the diffuse bounce.  ray.hit.color is read
 * after diffuse_reflection, so its importance weights apply here (contrast [C5]). */
static int diffuse_sun_sampling(ctx_t *c, ray_t *ray, ray_t *next, float cum[4], const ref_material *m,
                                uint32_t *rng, fwd_t *fw, uint32_t *segs, const float emit[3], int hit) {
    const sun_k *k = &c->sun;
    float direct[3] = {0.0f, 0.0f, 0.0f};
    int lit = 0;
    new_from_self(ray, next);
    next->d = random_sun_direction(k, rng);
    int front_light = vdot(next->d, ray->n) > 0.0f;
    if (front_light || ((m->flags & MAT_FLAG_SUBSURFACE) && ref_rng_next(rng) < c->s->f_sub_surface)) {
        if (!front_light) next->o = vadd(next->o, vscale(ray->n, -RAY_OFFSET));
        next->cur_mat = next->prev_mat;
        float att[4];
        direct_light_attenuation(c, next, att, segs);
        if (att[3] > 0.0f) {
            float mult = fabsf(vdot(next->d, ray->n)) * k->lum_a;
            for (int i = 0; i < 3; i++) direct[i] = att[i] * att[3] * mult;
            hit = 1;
            lit = 1;
        }
    }
    float wgt = diffuse_reflection(c, next, ray, rng);
    for (int i = 0; i < 4; i++) ray->col[i] *= wgt;
    if (fw) {
        if (c->s->emitters_enabled && m->emittance > RAY_EPSILON)
            for (int i = 0; i < 3; i++) fw->L[i] = fw->L[i] + fw->T[i] * emit[i];
        for (int i = 0; i < 3; i++) fw->T[i] = fw->T[i] * ray->col[i];
        if (lit) for (int i = 0; i < 3; i++) fw->L[i] = fw->L[i] + fw->T[i] * (direct[i] * k->emit[i]);
    }
    hit = path_trace(c, next, 0, rng, fw, segs) || hit;
    if (hit)
        for (int i = 0; i < 3; i++)
            cum[i] += emit[i] + ray->col[i] * ((direct[i] * k->emit[i] + next->col[i]) + 0.0f);
    return hit;
}

static int do_diffuse_reflection(ctx_t *c, ray_t *ray, ray_t *next, float cum[4], const ref_material *m,
                                 uint32_t *rng, fwd_t *fw, uint32_t *segs) { /* :190-316 */
    int hit = 0;
    float emit[3] = {0.0f, 0.0f, 0.0f};
    /* emitter_sampling_strategy == NONE [C8]: (NONE || depth == 1) is always true */
    if (c->s->emitters_enabled && m->emittance > RAY_EPSILON) {
        for (int i = 0; i < 3; i++) emit[i] = ray->col[i] * ray->col[i] * m->emittance;
        hit = 1;
    }
    if (c->sun.sun_sampling) return diffuse_sun_sampling(c, ray, next, cum, m, rng, fw, segs, emit, hit);
    /* sun_sampling == false (IMPORTANCE preset) -> :292-314 */
    float ray_color[4];
    memcpy(ray_color, ray->col, sizeof ray_color);
    diffuse_reflection(c, next, ray, rng);
    if (fw) {
        if (hit) for (int i = 0; i < 3; i++) fw->L[i] = fw->L[i] + fw->T[i] * emit[i];
        for (int i = 0; i < 3; i++) fw->T[i] = fw->T[i] * ray_color[i];
    }
    hit = path_trace(c, next, 0, rng, fw, segs) || hit;
    if (hit)
        for (int i = 0; i < 3; i++) cum[i] += emit[i] + ray_color[i] * (next->col[i] + 0.0f);
    memcpy(ray->col, ray_color, sizeof ray_color);
    return hit;
}

static void translucent_ray_color(const ray_t *ray, const ray_t *next, float cum[4], float absorption) { /* :424-437 */
    float rt[3] = {ray->col[0] * absorption, ray->col[1] * absorption, ray->col[2] * absorption};
    cum[0] += rt[0] * next->col[0];
    cum[1] += rt[1] * next->col[1];
    cum[2] += rt[2] * next->col[2];
    cum[3] += 1.0f * next->col[3];
}

static int do_refraction(ctx_t *c, const ray_t *ray, ray_t *next, const ref_material *cur, float cum[4],
                         float ior1, float ior2, float absorb, uint32_t *rng, fwd_t *fw, uint32_t *segs) { /* :318-401 */
    int hit = 0;
    int refr = (cur->flags & MAT_FLAG_REFRACTIVE) != 0;
    float n1n2 = ior1 / ior2;
    float cos_theta = -vdot(ray->d, ray->n);
    float radicand = 1.0f - n1n2 * n1n2 * (1.0f - cos_theta * cos_theta);
    if (refr && radicand < RAY_EPSILON) {
        specular_reflection(ray, cur->roughness, rng, next);
        if (path_trace(c, next, 0, rng, fw, segs)) {
            hit = 1;
            for (int i = 0; i < 3; i++) cum[i] += next->col[i];
        }
        return hit;
    }
    new_from_self(ray, next);
    float a = n1n2 - 1.0f, b = n1n2 + 1.0f;
    float r0 = a * a / (b * b);
    float cc = 1.0f - cos_theta;
    float c5 = ((cc * cc) * (cc * cc)) * cc; /* powi(5) [C11] */
    float rtheta = r0 + (1.0f - r0) * c5;
    if (ref_rng_next(rng) < rtheta) {
        specular_reflection(ray, cur->roughness, rng, next);
        if (path_trace(c, next, 0, rng, fw, segs)) {
            hit = 1;
            for (int i = 0; i < 3; i++) cum[i] += next->col[i];
        }
        /* :395 re-traces the already-traced reflected ray; not replicated [C14] */
        return hit;
    }
    if (refr) {
        float t2 = sqrtf(radicand);
        v3 n = ray->n, d;
        if (cos_theta > 0.0f) d = vadd(vscale(ray->d, n1n2), vscale(n, n1n2 * cos_theta - t2));
        else d = vsub(vscale(ray->d, n1n2), vscale(n, -n1n2 * cos_theta - t2));
        next->d = vnorm(d);
        if (signum_(vdot(next->n, next->d)) != signum_(vdot(next->n, ray->d))) {
            float factor = signum_(vdot(next->n, ray->d)) * -RAY_EPSILON - vdot(next->d, next->n);
            next->d = vnorm(vadd(next->d, vscale(next->n, factor)));
        }
        next->o = ray_at(next, RAY_OFFSET);
    }
    if (fw) for (int i = 0; i < 3; i++) fw->T[i] = fw->T[i] * (ray->col[i] * absorb);
    if (path_trace(c, next, 0, rng, fw, segs)) {
        hit = 1;
        translucent_ray_color(ray, next, cum, absorb);
    }
    return hit;
}

static int do_transmission(ctx_t *c, const ray_t *ray, ray_t *next, float cum[4], float absorb, uint32_t *rng,
                           fwd_t *fw, uint32_t *segs) { /* :403-422 */
    int hit = 0;
    new_from_self(ray, next);
    next->o = ray_at(next, RAY_OFFSET);
    if (fw) for (int i = 0; i < 3; i++) fw->T[i] = fw->T[i] * (ray->col[i] * absorb);
    if (path_trace(c, next, 0, rng, fw, segs)) {
        translucent_ray_color(ray, next, cum, absorb);
        hit = 1;
    }
    return hit;
}

static int path_trace(ctx_t *c, ray_t *ray, int first, uint32_t *rng, fwd_t *fw, uint32_t *segs) { /* :15-135 */
    int hit = 0;
    const ref_scene *s = c->s;
    for (;;) {
        if (c->path_segs >= MAX_PATH_SEGMENTS) break; /* [C15] */
        if (!next_intersection(c, ray, segs)) {
            if (ray->depth == 0) get_sky_color_interp(&c->sun, ray);
            else if (ray->specular) get_sky_color(&c->sun, ray, 1);
            else get_sky_color_diffuse_sun(&c->sun, ray, c->sun.diffuse_sun);
            if (fw) for (int i = 0; i < 3; i++) fw->L[i] = fw->L[i] + fw->T[i] * ray->col[i];
            hit = 1;
            break;
        }
        const ref_material *cur = &s->materials[ray->cur_mat];
        const ref_material *prev = &s->materials[ray->prev_mat];
        float specular = cur->specular, diffuse = ray->col[3], absorb = ray->col[3];
        float ior1 = cur->ior, ior2 = prev->ior;
        if (ray->col[3] + specular < RAY_EPSILON && ior1 == ior2) { /* :52-54 [C4] */
            ray->o = ray_at(ray, RAY_OFFSET);
            continue;
        }
        if (ray->depth + 1 >= c->max_depth) break; /* :56-58 */
        ray->depth += 1;
        c->st.shade_events++;
        float cum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        ray_t next;
        memset(&next, 0, sizeof next);
        float metal = cur->metalness;
        /* the first reflection splits into branch_count branches (:66, [C20]): each branch starts
         * from the same hit record, the same path-segment count [C15] and forward state, branch 0
         * continues the path's RNG stream and branch b > 0 draws from branch_state(stream, b) */
        uint32_t count = first ? c->cur_bc : 1;
        uint32_t rng0 = *rng, ps0 = c->path_segs;
        float col0[4], Lsum[3] = {0.0f, 0.0f, 0.0f};
        fwd_t fw0;
        memcpy(col0, ray->col, sizeof col0);
        if (fw) fw0 = *fw;
        for (uint32_t b = 0; b < count; b++) {
            if (first && b > 0) {
                *rng = ref_rng_branch_state(rng0, b);
                c->path_segs = ps0;
                memcpy(ray->col, col0, sizeof col0);
                if (fw) *fw = fw0;
            }
            int do_metal = metal > RAY_EPSILON && ref_rng_next(rng) < metal;
            if (do_metal || (specular > RAY_EPSILON && ref_rng_next(rng) < specular))
                hit |= do_specular_reflection(c, ray, &next, cum, do_metal, rng, fw, segs);
            else if (ref_rng_next(rng) < diffuse)
                hit |= do_diffuse_reflection(c, ray, &next, cum, cur, rng, fw, segs);
            else if (fabsf(ior1 - ior2) >= RAY_EPSILON)
                hit |= do_refraction(c, ray, &next, cur, cum, ior1, ior2, absorb, rng, fw, segs);
            else
                hit |= do_transmission(c, ray, &next, cum, absorb, rng, fw, segs);
            if (first && fw) for (int i = 0; i < 3; i++) Lsum[i] += fw->L[i];
        }
        float inv = 1.0f / (float)count;
        for (int i = 0; i < 4; i++) ray->col[i] = cum[i] * inv;
        if (first && fw) for (int i = 0; i < 3; i++) fw->L[i] = Lsum[i] * inv;
        break;
    }
    if (!hit) {
        ray->col[0] = ray->col[1] = ray->col[2] = 0.0f;
        ray->col[3] = 1.0f;
    }
    return hit;
}

/* ------------------------------------------------------------------------- */
/* camera + render (camera.rs:77-86, tile_renderer.rs:684-734)                 */
/* ------------------------------------------------------------------------- */
typedef struct {
    const ref_scene *s;
    const ref_camera *cam;
    const ref_render_params *p;
    float *accum;
    uint32_t *seg_count;
    sun_k sun;
    float d_factor;
    v3 cdir, cup, cright, ceye;
    uint32_t next_row;
    pthread_mutex_t lock;
    ref_stats total;
} job_t;

/* preview_render (path_tracer.rs:137-158) with next_intersection_preview (:447-455) and
 * Sun::flat_shading (scene/mod.rs:447-452) [C16].  Intersection = Scene::hit [C1]; the loop skips
 * material-0 and transparent (alpha 0) hits from hit + OFFSET*dir, bounded by [C15].  After a miss
 * the last hit's material decides the shading, exactly as written (a miss leaves the record). */
static void preview_pixel(ctx_t *c, ray_t *ray, uint32_t *segs, float col[3]) {
    ray->cur_mat = 0;
    for (;;) {
        if (c->path_segs >= MAX_PATH_SEGMENTS) break; /* [C15] */
        if (!next_intersection(c, ray, segs)) break;
        if (ray->cur_mat != 0 && ray->col[3] > 0.0f) break;
        ray->o = ray_at(ray, RAY_OFFSET);
    }
    if (ray->cur_mat == 0) { /* get_sky_color_inner + add_sun_color */
        sky_set(ray);
        add_sun_color(&c->sun, ray);
        for (int i = 0; i < 3; i++) col[i] = ray->col[i];
    } else {
        float shading = vdot(ray->n, c->sun.sw);
        shading = fmaxf(0.3f, shading); /* Sun::AMBIENT.max(shading), scene/mod.rs:318 */
        for (int i = 0; i < 3; i++) col[i] = ray->col[i] * (c->sun.emit[i] * shading);
    }
}

/* RendererMode::Preview: render_tile_replace (tile_renderer.rs:648-682) -- one un-jittered
 * camera ray per pixel, rgb replaced, alpha untouched */
static void preview_rows(job_t *j, ctx_t *c) {
    const ref_render_params *p = j->p;
    uint32_t W = p->width, H = p->height;
    float dim = (float)(W > H ? W : H);
    for (;;) {
        pthread_mutex_lock(&j->lock);
        uint32_t y = j->next_row++;
        pthread_mutex_unlock(&j->lock);
        if (y >= p->row_end) break;
        for (uint32_t x = 0; x < W; x++) {
            uint32_t pix = y * W + x;
            float *fb = &j->accum[4 * (size_t)pix];
            uint32_t segs = 0;
            float xn = ((float)(2 * x + 1) - (float)W) / dim;
            float yn = ((float)(2 * (H - y) - 1) - (float)H) / dim;
            v3 nd = vadd(vadd(vscale(j->cdir, j->d_factor), vscale(j->cright, xn)), vscale(j->cup, yn));
            ray_t ray;
            ray_new(&ray, j->ceye, vnorm(nd));
            c->st.paths++;
            c->path_segs = 0;
            float col[3];
            preview_pixel(c, &ray, &segs, col);
            for (int i = 0; i < 3; i++) fb[i] = col[i];
            if (j->seg_count) j->seg_count[pix] = segs;
        }
    }
}

static void render_rows(job_t *j, ctx_t *c) {
    const ref_render_params *p = j->p;
    uint32_t W = p->width, H = p->height;
    float dim = (float)(W > H ? W : H);
    for (;;) {
        pthread_mutex_lock(&j->lock);
        uint32_t y = j->next_row++;
        pthread_mutex_unlock(&j->lock);
        if (y >= p->row_end) break;
        for (uint32_t x = 0; x < W; x++) {
            uint32_t pix = y * W + x;
            float *fb = &j->accum[4 * (size_t)pix];
            uint32_t segs = 0;
            /* TileRenderer passes (tile_renderer.rs:416-484) [C20]: pass weight bc from the schedule,
             * the sample keyed by the accumulated spp at the pass start, until spp_start + spp_count */
            for (uint32_t spp = p->spp_start; spp < p->spp_start + p->spp_count;) {
                uint32_t bc = ref_branch_count(spp, c->branch_count);
                c->cur_bc = bc;
                uint32_t rng = ref_rng_path_state(p->seed, pix, spp);
                float xn = ((float)(2 * x + 1) - (float)W) / dim;
                float yn = ((float)(2 * (H - y) - 1) - (float)H) / dim;
                float lo = -1.0f / dim, hi = 1.0f / dim;
                float dx = lo + (hi - lo) * ref_rng_next(&rng);
                float dy = lo + (hi - lo) * ref_rng_next(&rng);
                float X = xn + dx, Y = yn + dy;
                v3 nd = vadd(vadd(vscale(j->cdir, j->d_factor), vscale(j->cright, X)), vscale(j->cup, Y));
                ray_t ray;
                ray_new(&ray, j->ceye, vnorm(nd));
                c->st.paths++;
                c->path_segs = 0;
                float col[3];
                if (c->forward) {
                    fwd_t fw = {{1.0f, 1.0f, 1.0f}, {0.0f, 0.0f, 0.0f}};
                    path_trace(c, &ray, 1, &rng, &fw, &segs);
                    memcpy(col, fw.L, sizeof col);
                } else {
                    path_trace(c, &ray, 1, &rng, NULL, &segs);
                    memcpy(col, ray.col, sizeof col);
                }
                float s_inv = 1.0f / (float)(bc + spp); /* render_tile_average :707-731 */
                for (int i = 0; i < 3; i++) fb[i] = (fb[i] * (float)spp + col[i] * (float)bc) * s_inv;
                spp += bc;
            }
            if (j->seg_count) j->seg_count[pix] = segs;
        }
    }
}

static void *render_worker(void *arg) {
    job_t *j = (job_t *)arg;
    ctx_t c;
    memset(&c, 0, sizeof c);
    c.s = j->s;
    c.sun = j->sun;
    c.octree_scale = ldexpf(1.0f, -(int)j->s->depth);
    c.max_depth = j->p->max_depth;
    c.branch_count = j->p->branch_count ? j->p->branch_count : 1;
    c.forward = j->p->forward_accumulation;
    if (j->p->preview) preview_rows(j, &c);
    else render_rows(j, &c);
    pthread_mutex_lock(&j->lock);
    j->total.paths += c.st.paths;
    j->total.segments += c.st.segments;
    j->total.esvo_steps += c.st.esvo_steps;
    j->total.node_fetches += c.st.node_fetches;
    j->total.prim_tests += c.st.prim_tests;
    j->total.leaf_visits += c.st.leaf_visits;
    j->total.shade_events += c.st.shade_events;
    j->total.texel_reads += c.st.texel_reads;
    j->total.block_tests += c.st.block_tests;
    if (c.st.max_path_segs > j->total.max_path_segs) j->total.max_path_segs = c.st.max_path_segs;
    pthread_mutex_unlock(&j->lock);
    return NULL;
}

int ref_render(const ref_scene *s, const ref_camera *cam, const ref_render_params *p, float *accum,
               uint32_t *seg_count, ref_stats *stats) {
    pthread_once(&lut_once, lut_init);
    if (!s || !cam || !p || !accum || p->width == 0 || p->height == 0 || s->depth < 1 || s->depth > 21) return 1;
    job_t j;
    memset(&j, 0, sizeof j);
    j.s = s;
    j.cam = cam;
    j.p = p;
    j.accum = accum;
    j.seg_count = seg_count;
    sun_init(&s->sun, &j.sun);
    j.d_factor = 1.0f / tanf(cam->fov / 2.0f); /* camera.rs:79 */
    j.cdir = V(cam->dir[0], cam->dir[1], cam->dir[2]);
    j.cup = V(cam->up[0], cam->up[1], cam->up[2]);
    j.ceye = V(cam->eye[0], cam->eye[1], cam->eye[2]);
    j.cright = vcross(j.cdir, j.cup);
    ref_render_params pp = *p;
    if (pp.row_end == 0 || pp.row_end > pp.height) pp.row_end = pp.height;
    j.p = &pp;
    j.next_row = pp.row_begin;
    pthread_mutex_init(&j.lock, NULL);
    uint32_t nt = p->threads ? p->threads : 1;
    if (nt > 256) nt = 256;
    pthread_t th[256];
    for (uint32_t i = 0; i < nt; i++) pthread_create(&th[i], NULL, render_worker, &j);
    for (uint32_t i = 0; i < nt; i++) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&j.lock);
    if (stats) *stats = j.total;
    return 0;
}

/* Octree::get_traversal_data (octree_traversal.rs:537-714): ESVO from the root until the first
 * leaf with t_min > 0 (:623), returning that parent, its scale and the descent stacks (indexed by
 * scale, zero where unwritten, :552).  max_dst exit (:609) and the escaping pop (:690-692, which
 * reports the scale before the pop) return the state reached; |rd| after the clamp [C13]. */
void ref_traversal_data(const ref_scene *s, const float ray[6], float max_dst_w, uint32_t *start, uint32_t *scale_out,
                        uint32_t index_stack[24], float time_stack[24]) {
    float octree_scale = ldexpf(1.0f, -(int)s->depth);
    memset(index_stack, 0, 24 * sizeof(uint32_t));
    memset(time_stack, 0, 24 * sizeof(float));
    v3 ro = vadd(vscale(V(ray[0], ray[1], ray[2]), octree_scale), V(1.0f, 1.0f, 1.0f));
    v3 rd = V(ray[3], ray[4], ray[5]);
    float max_dst = max_dst_w * octree_scale;
    uint32_t parent = s->root, scale = OCTREE_MAX_SCALE - 1;
    float scale_exp2 = 0.5f;
    for (int i = 0; i < 3; i++) {
        float di = vget(rd, i);
        if (fabsf(di) < OCTREE_EPSILON) vset(&rd, i, u2f((f2u(OCTREE_EPSILON) & 0x7FFFFFFFu) | (f2u(di) & 0x80000000u)));
    }
    v3 t_coef = V(1.0f / -fabsf(rd.x), 1.0f / -fabsf(rd.y), 1.0f / -fabsf(rd.z));
    v3 t_bias = vmul(t_coef, ro);
    uint32_t mirror = 0;
    for (int i = 0; i < 3; i++)
        if (vget(rd, i) > 0.0f) {
            mirror |= 1u << i;
            vset(&t_bias, i, 3.0f * vget(t_coef, i) - vget(t_bias, i));
        }
    float t_min = fmax_(vmax3(vsub(vscale(t_coef, 2.0f), t_bias)), 0.0f);
    float t_max = vmin3(vsub(t_coef, t_bias));
    float h = t_max;
    uint32_t idx = 0;
    v3 pos = V(1.0f, 1.0f, 1.0f);
    v3 upper = vsub(vscale(t_coef, 1.5f), t_bias);
    for (int i = 0; i < 3; i++)
        if (vget(upper, i) > t_min) { idx ^= 1u << i; vset(&pos, i, 1.5f); }
    uint32_t out_scale = scale;
    for (int it = 0; it < OCTREE_MAX_STEPS; it++) {
        out_scale = scale;
        if (max_dst >= 0.0f && t_min > max_dst) break;
        v3 t_corner = vsub(vmul(pos, t_coef), t_bias);
        float tc_max = vmin3(t_corner);
        uint32_t cidx = idx ^ mirror;
        uint16_t mask = octant_mask(s, parent);
        int present = (mask >> cidx) & 1, is_leaf = (mask >> (cidx + 8)) & 1;
        if (present && t_min <= t_max) {
            if (is_leaf && t_min > 0.0f) break;
            float half = scale_exp2 * 0.5f;
            v3 t_center = vadd(vscale(t_coef, half), t_corner);
            float tv_max = fmin_(t_max, tc_max);
            if (t_min <= tv_max && !is_leaf) {
                if (tc_max < h) { index_stack[scale] = parent; time_stack[scale] = t_max; }
                h = tc_max;
                parent = s->octant_children[8 * (size_t)parent + cidx];
                scale -= 1;
                scale_exp2 = half;
                idx = 0;
                for (int i = 0; i < 3; i++)
                    if (vget(t_center, i) > t_min) { idx ^= 1u << i; vset(&pos, i, vget(pos, i) + scale_exp2); }
                t_max = tv_max;
                out_scale = scale;
                continue;
            }
        }
        uint32_t step_mask = 0;
        for (int i = 0; i < 3; i++)
            if (vget(t_corner, i) <= tc_max) { step_mask ^= 1u << i; vset(&pos, i, vget(pos, i) - scale_exp2); }
        t_min = tc_max;
        idx ^= step_mask;
        if ((idx & step_mask) != 0) {
            uint32_t diff = 0;
            if (step_mask & 1) diff |= f2u(pos.x) ^ f2u(pos.x + scale_exp2);
            if (step_mask & 2) diff |= f2u(pos.y) ^ f2u(pos.y + scale_exp2);
            if (step_mask & 4) diff |= f2u(pos.z) ^ f2u(pos.z + scale_exp2);
            uint32_t old_scale = scale;
            scale = diff ? 31u - (uint32_t)__builtin_clz(diff) : 0xFFFFFFFFu;
            if (scale >= OCTREE_MAX_SCALE) { out_scale = old_scale; break; }
            scale_exp2 = u2f((scale - OCTREE_MAX_SCALE + 127u) << 23);
            parent = index_stack[scale];
            t_max = time_stack[scale];
            uint32_t shx = f2u(pos.x) >> scale, shy = f2u(pos.y) >> scale, shz = f2u(pos.z) >> scale;
            pos = V(u2f(shx << scale), u2f(shy << scale), u2f(shz << scale));
            idx = (shx & 1) | ((shy & 1) << 1) | ((shz & 1) << 2);
            h = 0.0f;
        }
        out_scale = scale;
    }
    *start = parent;
    *scale_out = out_scale;
}

/* closest-hit query (Scene::hit) for tests */
void ref_intersect(const ref_scene *s, const float *rays, const uint32_t *last_prim, const float *last_normal,
                   uint32_t n, float *out_t, uint32_t *out_prim, float *out_normal, uint32_t *out_steps) {
    pthread_once(&lut_once, lut_init);
    ctx_t c;
    memset(&c, 0, sizeof c);
    c.s = s;
    c.octree_scale = ldexpf(1.0f, -(int)s->depth);
    for (uint32_t i = 0; i < n; i++) {
        ray_t r;
        ray_new(&r, V(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), V(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
        if (last_prim) r.last_prim = last_prim[i];
        if (last_normal) r.n = V(last_normal[3 * i], last_normal[3 * i + 1], last_normal[3 * i + 2]);
        uint32_t prim = PRIM_NONE, steps = 0;
        prim_hit h;
        int hit = esvo(&c, &r, MAX_DST_WORLD, &prim, &h, &steps);
        if (hit) {
            commit_hit(&c, &r, prim, &h);
            out_t[i] = h.t;
            /* block-value scenes [C23]: the block id, or QUAD_KEY | quad for a block model's quad */
            out_prim[i] = (s->block_mat && h.quad >= 0) ? (QUAD_KEY | (uint32_t)h.quad) : prim;
            if (out_normal) { out_normal[3 * i] = r.n.x; out_normal[3 * i + 1] = r.n.y; out_normal[3 * i + 2] = r.n.z; }
        } else {
            out_t[i] = INFINITY;
            out_prim[i] = PRIM_NONE;
            if (out_normal) out_normal[3 * i] = out_normal[3 * i + 1] = out_normal[3 * i + 2] = 0.0f;
        }
        if (out_steps) out_steps[i] = steps;
    }
}

void ref_intersect_brute(const ref_scene *s, const float *rays, uint32_t n, float *out_t, uint32_t *out_prim) {
    for (uint32_t i = 0; i < n; i++) {
        ray_t r;
        ray_new(&r, V(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), V(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
        float best = INFINITY;
        uint32_t bp = PRIM_NONE;
        for (uint32_t k = 0; k < s->n_spheres; k++) {
            prim_hit h;
            if (sphere_test(&s->spheres[4 * (size_t)k], &r, 0, &h) && h.t < best) { best = h.t; bp = k; }
        }
        for (uint32_t k = 0; k < s->n_cuboids; k++) {
            prim_hit h;
            if (cuboid_test(&s->cuboids[6 * (size_t)k], &r, 0, &h) && h.t < best) { best = h.t; bp = k | PRIM_CUBOID_BIT; }
        }
        out_t[i] = best;
        out_prim[i] = bp;
    }
}

void ref_quad_hit(const ref_quad *q, const float *rays, const float voxel[3], uint32_t n, float *out, uint8_t *hit) {
    quad_geo g = quad_geometry(q);
    for (uint32_t i = 0; i < n; i++) {
        ray_t r;
        ray_new(&r, V(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), V(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
        float t = 0.0f, a = 0.0f, b = 0.0f;
        hit[i] = (uint8_t)quad_hit(&g, &r, V(voxel[0], voxel[1], voxel[2]), INFINITY, &t, &a, &b);
        out[3 * i] = t;
        out[3 * i + 1] = a;
        out[3 * i + 2] = b;
    }
}

/* tone map: From<&F32Color> for U8Color (colors/mod.rs:408-420) */
void ref_tonemap(const float *accum, uint32_t n_pixels, uint8_t *out) {
    pthread_once(&lut_once, lut_init);
    for (uint32_t p = 0; p < n_pixels; p++) {
        float res[4];
        for (int i = 0; i < 4; i++) res[i] = fminf(accum[4 * (size_t)p + i] * 255.0f, 255.0f);
        out[4 * (size_t)p + 0] = LUT_BYTE[f2u32_sat(res[0])];
        out[4 * (size_t)p + 1] = LUT_BYTE[f2u32_sat(res[1])];
        out[4 * (size_t)p + 2] = LUT_BYTE[f2u32_sat(res[2])];
        out[4 * (size_t)p + 3] = (uint8_t)f2u32_sat(res[3]);
    }
}

/* ------------------------------------------------------------------------- */
/* octree builder: voxelise primitives into depth-D leaf cells,  */
/* Morton-sort (new_octree.rs:752-835 ordering), then build pre-order.          */
/* ------------------------------------------------------------------------- */
typedef struct { uint64_t code; uint32_t prim; } cell_pair;
static int pair_cmp(const void *a, const void *b) {
    const cell_pair *x = (const cell_pair *)a, *y = (const cell_pair *)b;
    if (x->code != y->code) return x->code < y->code ? -1 : 1;
    return x->prim < y->prim ? -1 : (x->prim > y->prim ? 1 : 0);
}
typedef struct {
    cell_pair *v;
    size_t n, cap;
} pair_vec;
static int pv_push(pair_vec *pv, uint64_t code, uint32_t prim) {
    if (pv->n == pv->cap) {
        size_t nc = pv->cap ? pv->cap * 2 : 4096;
        cell_pair *nv = (cell_pair *)realloc(pv->v, nc * sizeof(cell_pair));
        if (!nv) return 1;
        pv->v = nv;
        pv->cap = nc;
    }
    pv->v[pv->n].code = code;
    pv->v[pv->n].prim = prim;
    pv->n++;
    return 0;
}
static inline int32_t clampi(int64_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : (int32_t)v); }

typedef struct {
    uint16_t *mask;
    uint32_t *child;
    uint32_t n, cap;
    const uint64_t *leaf_code;
    uint32_t depth;
    int compact; /* REF_BUILD_COMPACT: Octant::is_compactable merge (new_octree.rs:227-233) */
    const uint32_t *leaf_first, *leaf_count, *leaf_prims;
} tree_build;

static int tb_alloc(tree_build *tb) {
    if (tb->n == tb->cap) {
        uint32_t nc = tb->cap ? tb->cap * 2 : 1024;
        uint16_t *m = (uint16_t *)realloc(tb->mask, nc * sizeof(uint16_t));
        if (!m) return -1;
        tb->mask = m;
        uint32_t *c = (uint32_t *)realloc(tb->child, (size_t)nc * 8 * sizeof(uint32_t));
        if (!c) return -1;
        tb->child = c;
        tb->cap = nc;
    }
    uint32_t id = tb->n++;
    tb->mask[id] = 0;
    memset(&tb->child[8 * (size_t)id], 0, 8 * sizeof(uint32_t));
    return (int)id;
}
/* two leaves hold the same primitive list (the leaf-value equality of is_compactable) */
static int same_leaf(const tree_build *tb, uint32_t a, uint32_t b) {
    if (tb->leaf_count[a] != tb->leaf_count[b]) return 0;
    return memcmp(&tb->leaf_prims[tb->leaf_first[a]], &tb->leaf_prims[tb->leaf_first[b]],
                  tb->leaf_count[a] * sizeof(uint32_t)) == 0;
}
/* Pre-order octant emission of the leaves [lo, hi) below a level-`level` octant.  Returns the
 * child the parent stores: *is_leaf = 0 with the octant id, or, with compaction, *is_leaf = 1 and
 * a leaf payload when all eight children are leaves holding the same list -- Octant::
 * is_compactable (new_octree.rs:227-233) as RegionOctreeBuilder::recursive_build applies it at
 * every level (:679-690): the octant becomes Lod(get_child(0)) in its parent.  The root is never
 * merged away (a Lod root stays an octant of eight equal leaves, :534-545).  -1 = out of memory. */
static int tb_node(tree_build *tb, uint32_t level, uint32_t lo, uint32_t hi, int *is_leaf, uint32_t *value) {
    int id = tb_alloc(tb);
    if (id < 0) return -1;
    uint32_t shift = 3 * (tb->depth - 1 - level);
    uint32_t a = lo;
    for (uint32_t cidx = 0; cidx < 8; cidx++) {
        uint32_t b = a;
        while (b < hi && ((tb->leaf_code[b] >> shift) & 7u) == cidx) b++;
        if (b == a) continue;
        if (level + 1 == tb->depth) {
            tb->mask[id] |= (uint16_t)((1u << cidx) | (1u << (cidx + 8)));
            tb->child[8 * (size_t)id + cidx] = a; /* leaf payload = leaf index */
        } else {
            int leaf;
            uint32_t v;
            if (tb_node(tb, level + 1, a, b, &leaf, &v) < 0) return -1;
            tb->mask[id] |= (uint16_t)(leaf ? ((1u << cidx) | (1u << (cidx + 8))) : (1u << cidx));
            tb->child[8 * (size_t)id + cidx] = v;
        }
        a = b;
    }
    *is_leaf = 0;
    *value = (uint32_t)id;
    if (tb->compact && level > 0 && tb->mask[id] == 0xFFFFu) {
        const uint32_t *ch = &tb->child[8 * (size_t)id];
        int same = 1;
        for (int k = 1; k < 8 && same; k++) same = same_leaf(tb, ch[0], ch[k]);
        if (same) { /* all children are leaves, so this octant is the last one emitted */
            *is_leaf = 1;
            *value = ch[0];
            tb->n--;
        }
    }
    return 0;
}

int ref_build_octree(const float *spheres, uint32_t ns, const float *cuboids, uint32_t nc, uint32_t depth,
                     uint32_t flags, ref_octree *out) {
    memset(out, 0, sizeof *out);
    if (depth < 1 || depth > 21) return 1;
    int32_t N = 1 << depth;
    pair_vec pv = {0};
    for (uint32_t i = 0; i < ns; i++) {
        float cx = spheres[4 * i], cy = spheres[4 * i + 1], cz = spheres[4 * i + 2], r = spheres[4 * i + 3];
        if (!(r > 0.0f)) continue;
        int32_t lo[3], hi[3];
        float cen[3] = {cx, cy, cz};
        int empty = 0;
        for (int a = 0; a < 3; a++) {
            float fl = floorf(cen[a] - r), fh = floorf(cen[a] + r);
            if (fh < 0.0f || fl > (float)(N - 1)) empty = 1;
            lo[a] = clampi((int64_t)fmaxf(fl, -1.0f), 0, N - 1);
            hi[a] = clampi((int64_t)fminf(fh, (float)N), 0, N - 1);
        }
        if (empty) continue;
        float r2 = r * r;
        for (int32_t z = lo[2]; z <= hi[2]; z++)
            for (int32_t y = lo[1]; y <= hi[1]; y++)
                for (int32_t x = lo[0]; x <= hi[0]; x++) {
                    float bl[3] = {(float)x, (float)y, (float)z};
                    float dd[3];
                    for (int a = 0; a < 3; a++) {
                        float l = bl[a], h = bl[a] + 1.0f;
                        dd[a] = cen[a] < l ? l - cen[a] : (cen[a] > h ? cen[a] - h : 0.0f);
                    }
                    float dist2 = (dd[0] * dd[0] + dd[1] * dd[1]) + dd[2] * dd[2];
                    if (dist2 <= r2)
                        if (pv_push(&pv, ref_morton_encode((uint64_t)x, (uint64_t)y, (uint64_t)z), i)) goto oom;
                }
    }
    for (uint32_t i = 0; i < nc; i++) {
        const float *b = &cuboids[6 * i];
        int32_t lo[3], hi[3];
        int empty = 0;
        for (int a = 0; a < 3; a++) {
            /* half-open upper bound: a face on an integer plane does not claim the next cell
             * (a unit block [x, x+1) is one cell, the voxel world of C5) */
            float fl = floorf(b[a]), fh = fmaxf(fl, ceilf(b[3 + a]) - 1.0f);
            if (fh < 0.0f || fl > (float)(N - 1) || b[3 + a] < b[a]) empty = 1;
            lo[a] = clampi((int64_t)fmaxf(fl, -1.0f), 0, N - 1);
            hi[a] = clampi((int64_t)fminf(fh, (float)N), 0, N - 1);
        }
        if (empty) continue;
        for (int32_t z = lo[2]; z <= hi[2]; z++)
            for (int32_t y = lo[1]; y <= hi[1]; y++)
                for (int32_t x = lo[0]; x <= hi[0]; x++)
                    if (pv_push(&pv, ref_morton_encode((uint64_t)x, (uint64_t)y, (uint64_t)z), i | PRIM_CUBOID_BIT))
                        goto oom;
    }
    qsort(pv.v, pv.n, sizeof(cell_pair), pair_cmp);
    /* leaves */
    uint32_t nleaves = 0;
    for (size_t k = 0; k < pv.n; k++)
        if (k == 0 || pv.v[k].code != pv.v[k - 1].code) nleaves++;
    out->leaf_first = (uint32_t *)malloc((nleaves ? nleaves : 1) * sizeof(uint32_t));
    out->leaf_count = (uint32_t *)malloc((nleaves ? nleaves : 1) * sizeof(uint32_t));
    out->leaf_prims = (uint32_t *)malloc((pv.n ? pv.n : 1) * sizeof(uint32_t));
    uint64_t *codes = (uint64_t *)malloc((nleaves ? nleaves : 1) * sizeof(uint64_t));
    if (!out->leaf_first || !out->leaf_count || !out->leaf_prims || !codes) { free(codes); goto oom; }
    uint32_t li = 0;
    for (size_t k = 0; k < pv.n; k++) {
        if (k == 0 || pv.v[k].code != pv.v[k - 1].code) {
            out->leaf_first[li] = (uint32_t)k;
            out->leaf_count[li] = 0;
            codes[li] = pv.v[k].code;
            li++;
        }
        out->leaf_count[li - 1]++;
        out->leaf_prims[k] = pv.v[k].prim;
    }
    out->n_leaves = nleaves;
    out->n_leaf_prims = (uint32_t)pv.n;
    free(pv.v);
    pv.v = NULL;
    tree_build tb = {0};
    tb.leaf_code = codes;
    tb.depth = depth;
    tb.compact = (flags & REF_BUILD_COMPACT) != 0;
    tb.leaf_first = out->leaf_first;
    tb.leaf_count = out->leaf_count;
    tb.leaf_prims = out->leaf_prims;
    int root_leaf;
    uint32_t root;
    int rc = tb_node(&tb, 0, 0, nleaves, &root_leaf, &root);
    free(codes);
    if (rc < 0) { free(tb.mask); free(tb.child); goto oom; }
    out->octant_mask = tb.mask;
    out->octant_children = tb.child;
    out->n_octants = tb.n;
    out->root = (uint32_t)root;
    out->depth = depth;
    return 0;
oom:
    free(pv.v);
    ref_free_octree(out);
    return 2;
}

void ref_free_octree(ref_octree *t) {
    if (!t) return;
    free(t->octant_mask);
    free(t->octant_children);
    free(t->leaf_first);
    free(t->leaf_count);
    free(t->leaf_prims);
    memset(t, 0, sizeof *t);
}
