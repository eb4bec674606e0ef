// Host-side queries of the C ABI that need no device: Octree::get_traversal_data.
//
// get_traversal_data (octree_traversal.rs:537-714) is the reference's beam-start query: the
// host walks one ray (GPURenderer::render_frame uses the camera's centre ray,
// gpu_renderer.rs:579-581) down the octree to the first leaf and hands the octant it stopped
// in, its scale and the descent stack to the GPU as CameraUniform.traversal_start_idx / scale
// and the index/time stack buffers (gpu_renderer.rs:35-80).  It is one ray per frame, so it
// stays on the host, where the caller's octree already lives; the arithmetic is the ESVO
// setup and step of DESIGN.md §3 (the same float spec as the kernels: no contraction).
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/octpt.h"
#include "octpt_mask.h"

namespace {
constexpr uint32_t kMaxScale = 23u;   // OCTREE_MAX_SCALE, octree_traversal.rs:14
constexpr uint32_t kMaxSteps = 1000u; // OCTREE_MAX_STEPS, :13
constexpr float kEpsilon = 1.1920929e-7f;  // OCTREE_EPSILON = 2^-23, :15

inline uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
// glam min_element / max_element on NaN-free t-values
inline float mn(float a, float b) { return a < b ? a : b; }
inline float mx(float a, float b) { return a > b ? a : b; }
}  // namespace

extern "C" octpt_status octpt_traversal_data(const octpt_octant *octants, uint32_t octant_count, uint32_t root,
                                             uint32_t depth, const float ray[6], float max_dst,
                                             uint32_t *start_octant, uint32_t *scale_out,
                                             uint32_t index_stack[24], float time_stack[24]) {
    if (!octants || !ray || !start_octant || !scale_out || !index_stack || !time_stack) return OCTPT_ERR_INVALID_ARG;
    if (root >= octant_count || depth < 1u || depth > 21u) return OCTPT_ERR_INVALID_ARG;
    for (int i = 0; i < 24; ++i) {  // Default::default() (:552)
        index_stack[i] = 0u;
        time_stack[i] = 0.0f;
    }
    const float octree_scale = std::ldexp(1.0f, -(int)depth);
    float ro[3], rd[3], t_coef[3], t_bias[3], pos[3] = {1.0f, 1.0f, 1.0f};
    for (int i = 0; i < 3; ++i) {
        ro[i] = ray[i] * octree_scale + 1.0f;  // :553, :559
        rd[i] = ray[3 + i];
        // :566-574 epsilon clamp; |rd| is taken after it ([C13], as the kernels)
        if (std::fabs(rd[i]) < kEpsilon) rd[i] = u2f((f2u(kEpsilon) & 0x7FFFFFFFu) | (f2u(rd[i]) & 0x80000000u));
        t_coef[i] = 1.0f / -std::fabs(rd[i]);
        t_bias[i] = t_coef[i] * ro[i];
    }
    const float max_d = max_dst * octree_scale;
    uint32_t mirror = 0u;
    for (int i = 0; i < 3; ++i)
        if (rd[i] > 0.0f) {  // :579-587
            mirror |= 1u << i;
            t_bias[i] = 3.0f * t_coef[i] - t_bias[i];
        }
    float t_min = mx(mx(mx(2.0f * t_coef[0] - t_bias[0], 2.0f * t_coef[1] - t_bias[1]), 2.0f * t_coef[2] - t_bias[2]),
                     0.0f);
    float t_max = mn(mn(t_coef[0] - t_bias[0], t_coef[1] - t_bias[1]), t_coef[2] - t_bias[2]);
    float h = t_max;
    uint32_t idx = 0u, parent = root, scale = kMaxScale - 1u;
    float scale_exp2 = 0.5f;
    for (int i = 0; i < 3; ++i)
        if (1.5f * t_coef[i] - t_bias[i] > t_min) {  // :597-606
            idx ^= 1u << i;
            pos[i] = 1.5f;
        }
    auto done = [&](uint32_t sc) {
        *start_octant = parent;
        *scale_out = sc;
        return OCTPT_OK;
    };
    for (uint32_t it = 0; it < kMaxSteps; ++it) {
        if (max_d >= 0.0f && t_min > max_d) return done(scale);  // :609-611
        float t_corner[3];
        for (int i = 0; i < 3; ++i) t_corner[i] = pos[i] * t_coef[i] - t_bias[i];
        const float tc_max = mn(mn(t_corner[0], t_corner[1]), t_corner[2]);
        const uint32_t cidx = idx ^ mirror;
        const uint32_t mask = octpt::normalized_mask(octants[parent].child_mask);  // C21
        const bool present = (mask >> cidx) & 1u, leaf = (mask >> (cidx + 8u)) & 1u;
        if (present && t_min <= t_max) {  // :622
            if (leaf && t_min > 0.0f) return done(scale);  // :623-625: the first leaf ends the walk
            const float half = scale_exp2 * 0.5f;
            const float tv_max = mn(t_max, tc_max);
            if (t_min <= tv_max && !leaf) {  // :633-651 descend
                const uint32_t child = octants[parent].children[cidx];
                if (child >= octant_count) return OCTPT_ERR_INVALID_ARG;
                if (tc_max < h) {
                    index_stack[scale] = parent;
                    time_stack[scale] = t_max;
                }
                h = tc_max;
                parent = child;
                scale -= 1u;
                scale_exp2 = half;
                idx = 0u;
                for (int i = 0; i < 3; ++i)
                    if (half * t_coef[i] + t_corner[i] > t_min) {
                        idx ^= 1u << i;
                        pos[i] += scale_exp2;
                    }
                t_max = tv_max;
                continue;
            }
        }
        uint32_t step_mask = 0u;  // :655-668 advance
        for (int i = 0; i < 3; ++i)
            if (t_corner[i] <= tc_max) {
                step_mask ^= 1u << i;
                pos[i] -= scale_exp2;
            }
        t_min = tc_max;
        idx ^= step_mask;
        if ((idx & step_mask) != 0u) {  // :670-711 pop
            uint32_t diff = 0u;
            for (int i = 0; i < 3; ++i)
                if (step_mask & (1u << i)) diff |= f2u(pos[i]) ^ f2u(pos[i] + scale_exp2);
            const uint32_t old_scale = scale;
            scale = diff ? 31u - (uint32_t)__builtin_clz(diff) : 0xFFFFFFFFu;  // util::find_msb_u32
            if (scale >= kMaxScale) return done(old_scale);
            scale_exp2 = u2f((scale - kMaxScale + 127u) << 23);
            parent = index_stack[scale];
            t_max = time_stack[scale];
            uint32_t sh[3];
            for (int i = 0; i < 3; ++i) {
                sh[i] = f2u(pos[i]) >> scale;
                pos[i] = u2f(sh[i] << scale);
            }
            idx = (sh[0] & 1u) | ((sh[1] & 1u) << 1) | ((sh[2] & 1u) << 2);
            h = 0.0f;
        }
    }
    return done(scale);
}
