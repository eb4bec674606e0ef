// The host flattener of the drop-in: the reference's scene::Scene, element by
// element, into the octpt_scene_desc that octpt_scene_upload takes.  Host-only, no allocation.
//
// scene::Scene (src/scene/mod.rs:146-156) holds the octree (new_octree::Octree: octants_slice, root,
// depth), Box<[Quad]> and Box<[Material]>; GPURenderer::create_pipeline (gpu_renderer.rs:201-557) is
// the reference's own flattener for its wgpu backend: one texture per material (:221-307), the quads as
// GPUQuad (:309-320), the octree through octree_to_gpu_data (todo!(), gpu_octree.rs:28-76).  This is
// the same step for the HIP backend, without the lossy GPUQuad packing of the texture ranges into u16
// (gpu_quad.rs:31-38): the quads keep Quad::new's f32 arguments.
#include <cmath>
#include <cstring>

#include "../../include/octpt.h"

namespace {

// Quad::new (quad.rs:90-114): normal = normalize(u x v), in glam's f32 order
void quad_normal(const float u[3], const float v[3], float nrm[3]) {
    const float n[3] = {u[1] * v[2] - v[1] * u[2], u[2] * v[0] - v[2] * u[0], u[0] * v[1] - v[0] * u[1]};
    const float r = 1.0f / sqrtf((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]);
    for (int i = 0; i < 3; ++i) nrm[i] = n[i] * r;
}

}  // namespace

extern "C" octpt_status octpt_scene_from_reference(const octpt_reference_scene *ref, octpt_material *materials_out,
                                                   octpt_texture *textures_out, octpt_quad *quads_out,
                                                   octpt_scene_desc *d) {
    if (!ref || !d) return OCTPT_ERR_INVALID_ARG;
    if (ref->material_count && (!ref->materials || !materials_out || !textures_out)) return OCTPT_ERR_INVALID_ARG;
    if (ref->quad_count && (!ref->quads || !quads_out)) return OCTPT_ERR_INVALID_ARG;
    if (ref->model_count && !ref->models) return OCTPT_ERR_INVALID_ARG;
    if (ref->block_count && !ref->blocks) return OCTPT_ERR_INVALID_ARG;
    // Box<[Material]> -> material i with its own texture i (gpu_renderer.rs:221-307)
    for (uint32_t m = 0; m < ref->material_count; ++m) {
        const octpt_reference_material &x = ref->materials[m];
        octpt_texture t{};
        t.kind = x.texture_kind;
        if (x.texture_kind == OCTPT_TEXTURE_COLOR) {
            std::memcpy(t.rgba, x.color, 4);
        } else if (x.texture_kind == OCTPT_TEXTURE_IMAGE) {
            if (!x.image_rgba || x.image_width == 0 || x.image_height == 0) return OCTPT_ERR_INVALID_ARG;
            t.width = x.image_width;
            t.height = x.image_height;
            t.pixels = x.image_rgba;
        } else {
            return OCTPT_ERR_INVALID_ARG;
        }
        textures_out[m] = t;
        octpt_material o{};
        o.ior = x.index_of_refraction;
        o.specular = x.specular;
        o.emittance = x.emittance;
        o.roughness = x.roughness;
        o.metalness = x.metalness;
        o.texture_index = m;
        o.tint_index = x.tint_index;
        o.flags = x.material_flags;  // MaterialFlags bits (material.rs:99-108)
        materials_out[m] = o;
    }
    // Box<[Quad]> -> Quad::new's arguments; the stored normal must be what Quad::new derived from u x v
    // (a mis-ordered or stale record is refused rather than rendered)
    for (uint32_t q = 0; q < ref->quad_count; ++q) {
        const octpt_reference_quad &x = ref->quads[q];
        if (x.material_id >= ref->material_count) return OCTPT_ERR_INVALID_ARG;
        float nrm[3];
        quad_normal(x.u, x.v, nrm);
        for (int i = 0; i < 3; ++i)
            if (!(fabsf(nrm[i] - x.normal[i]) <= 1e-5f)) return OCTPT_ERR_INVALID_ARG;
        octpt_quad o{};
        std::memcpy(o.origin, x.origin, 12);
        std::memcpy(o.u, x.u, 12);
        std::memcpy(o.v, x.v, 12);
        o.material = x.material_id;
        std::memcpy(o.texture_u_range, x.texture_u_range, 8);
        std::memcpy(o.texture_v_range, x.texture_v_range, 8);
        quads_out[q] = o;
    }
    for (uint32_t k = 0; k < ref->model_count; ++k)
        if ((uint64_t)ref->models[k].first_quad + ref->models[k].quad_count > ref->quad_count)
            return OCTPT_ERR_INVALID_ARG;
    for (uint32_t b = 0; b < ref->block_count; ++b) {
        const octpt_block &x = ref->blocks[b];
        if (x.model != OCTPT_MODEL_NONE) {
            if (x.model >= ref->model_count) return OCTPT_ERR_INVALID_ARG;
        } else {
            for (int f = 0; f < 6; ++f)
                if (x.face_material[f] >= ref->material_count) return OCTPT_ERR_INVALID_ARG;
        }
    }
    octpt_scene_desc o{};
    o.abi_version = OCTPT_ABI_VERSION;
    o.octants = ref->octants;  // either mask encoding (C21); leaf payloads are block values (C23)
    o.octant_count = ref->octant_count;
    o.root = ref->root;
    o.depth = ref->depth;
    o.materials = ref->material_count ? materials_out : nullptr;
    o.material_count = ref->material_count;
    o.textures = ref->material_count ? textures_out : nullptr;
    o.texture_count = ref->material_count;
    o.sun = ref->sun;
    o.emitters_enabled = ref->emitters_enabled;
    o.f_sub_surface = ref->f_sub_surface;
    o.models = ref->models;
    o.model_count = ref->model_count;
    o.quads = ref->quad_count ? quads_out : nullptr;
    o.quad_count = ref->quad_count;
    o.blocks = ref->blocks;
    o.block_count = ref->block_count;
    *d = o;
    return OCTPT_OK;
}
