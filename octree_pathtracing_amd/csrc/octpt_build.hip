// octpt_build.hip -- the octree builder on the GPU (the reference's
// flattener octree_to_gpu_data, gpu_octree.rs:28-76, is todo!()).
//
// It produces the octree of the host builder (octpt_build_octree) array for array:
// the same (cell, primitive) pairs, the same Morton order (new_octree.rs:752-835), the same leaf
// tables and the same pre-order octant numbering.  All integer / byte work, HBM-bound:
//
//   count  : one thread per primitive counts its cells (sphere: bounding-box cells passing the
//            closest-point test; cuboid: the half-open box)           -> per-primitive counts
//   scan   : exclusive sum                                            -> pair offsets
//   emit   : one thread per primitive writes (Morton code, primitive) in primitive order
//   sort   : stable LSD radix sort on the code (3*depth bits); equal codes keep primitive order,
//            which is the host's (code, prim) order because spheres precede cuboids (bit 31)
//   leaves : head flags + scan -> leaf_first / leaf_count / leaf codes
//   octants: leaf j opens floor(msb(code_j ^ code_j-1) / 3) new octants (depth for j = 0), one
//            per level from the first level where its path leaves its predecessor's; pre-order
//            numbers them consecutively, so ids = exclusive scan of that count.  Each new octant
//            links itself into its parent (found by binary search over the leaf codes when the
//            parent was opened by an earlier leaf), each leaf into its level depth-1 octant.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "../../include/octpt.h"
#include "octpt_internal.h"

namespace octpt {
namespace {

constexpr uint32_t kBuildBlock = 256;

__device__ __forceinline__ uint64_t part_by_2(uint64_t v) {  // new_octree.rs:813-822
    uint64_t x = v & 0x1fffff;
    x = (x | x << 32) & 0x1f00000000ffffULL;
    x = (x | x << 16) & 0x1f0000ff0000ffULL;
    x = (x | x << 8) & 0x100f00f00f00f00fULL;
    x = (x | x << 4) & 0x10c30c30c30c30c3ULL;
    x = (x | x << 2) & 0x1249249249249249ULL;
    return x;
}
__device__ __forceinline__ uint64_t morton(uint32_t x, uint32_t y, uint32_t z) {
    return (part_by_2(z) << 2) + (part_by_2(y) << 1) + part_by_2(x);
}

__device__ __forceinline__ int32_t clamp_cell(float f, int32_t hi) {
    if (!(f >= 0.0f)) return 0;  // also NaN
    if (f >= (float)hi) return hi;
    return (int32_t)f;
}

// the host builder's per-primitive cell box (octpt_api.cpp octpt_build_octree); false = no cells
__device__ inline bool prim_box(const octpt_sphere *sp, uint32_t ns, const octpt_cuboid *cb, uint32_t i, int32_t N,
                                int32_t lo[3], int32_t hi[3]) {
    if (i < ns) {
        const octpt_sphere s = sp[i];
        const float r = s.radius;
        if (!(r > 0.0f)) return false;
        bool empty = false;
        for (int a = 0; a < 3; ++a) {
            const float fl = floorf(s.center[a] - r), fh = floorf(s.center[a] + r);
            if (fh < 0.0f || fl > (float)(N - 1)) empty = true;
            lo[a] = clamp_cell(fl, N - 1);
            hi[a] = clamp_cell(fh, N - 1);
        }
        return !empty;
    }
    const octpt_cuboid b = cb[i - ns];
    bool empty = false;
    for (int a = 0; a < 3; ++a) {
        const float fl = floorf(b.min[a]), fh = fmaxf(fl, ceilf(b.max[a]) - 1.0f);  // half-open top
        if (fh < 0.0f || fl > (float)(N - 1) || b.max[a] < b.min[a]) empty = true;
        lo[a] = clamp_cell(fl, N - 1);
        hi[a] = clamp_cell(fh, N - 1);
    }
    return !empty;
}

// closest-point test of the host builder: squared distance from the centre to the cell <= r^2
__device__ __forceinline__ bool sphere_keeps(const octpt_sphere &s, int32_t x, int32_t y, int32_t z) {
    const float bl[3] = {(float)x, (float)y, (float)z};
    float dd[3];
    for (int a = 0; a < 3; ++a) {
        const float l = bl[a], h = bl[a] + 1.0f, c = s.center[a];
        dd[a] = c < l ? l - c : (c > h ? c - h : 0.0f);
    }
    return (dd[0] * dd[0] + dd[1] * dd[1]) + dd[2] * dd[2] <= s.radius * s.radius;
}

__global__ __launch_bounds__(kBuildBlock) void count_cells_kernel(const octpt_sphere *__restrict__ sp, uint32_t ns,
                                                                  const octpt_cuboid *__restrict__ cb, uint32_t nc,
                                                                  int32_t N, unsigned long long *__restrict__ counts) {
    const uint32_t i = blockIdx.x * kBuildBlock + threadIdx.x;
    if (i >= ns + nc) return;
    int32_t lo[3], hi[3];
    unsigned long long n = 0;
    if (prim_box(sp, ns, cb, i, N, lo, hi)) {
        if (i < ns) {
            const octpt_sphere s = sp[i];
            for (int32_t z = lo[2]; z <= hi[2]; ++z)
                for (int32_t y = lo[1]; y <= hi[1]; ++y)
                    for (int32_t x = lo[0]; x <= hi[0]; ++x) n += sphere_keeps(s, x, y, z) ? 1u : 0u;
        } else {
            n = (unsigned long long)(hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1);
        }
    }
    counts[i] = n;
}

__global__ __launch_bounds__(kBuildBlock) void emit_pairs_kernel(const octpt_sphere *__restrict__ sp, uint32_t ns,
                                                                 const octpt_cuboid *__restrict__ cb, uint32_t nc,
                                                                 int32_t N, const unsigned long long *__restrict__ offs,
                                                                 uint64_t *__restrict__ codes,
                                                                 uint32_t *__restrict__ prims) {
    const uint32_t i = blockIdx.x * kBuildBlock + threadIdx.x;
    if (i >= ns + nc) return;
    int32_t lo[3], hi[3];
    if (!prim_box(sp, ns, cb, i, N, lo, hi)) return;
    unsigned long long o = offs[i];
    const bool sphere = i < ns;
    const uint32_t prim = sphere ? i : ((i - ns) | kPrimCuboidBit);
    const octpt_sphere s = sphere ? sp[i] : octpt_sphere{};
    for (int32_t z = lo[2]; z <= hi[2]; ++z)
        for (int32_t y = lo[1]; y <= hi[1]; ++y)
            for (int32_t x = lo[0]; x <= hi[0]; ++x) {
                if (sphere && !sphere_keeps(s, x, y, z)) continue;
                codes[o] = morton((uint32_t)x, (uint32_t)y, (uint32_t)z);
                prims[o] = prim;
                ++o;
            }
}

__global__ __launch_bounds__(kBuildBlock) void leaf_heads_kernel(const uint64_t *__restrict__ codes, uint32_t n,
                                                                 uint32_t *__restrict__ head) {
    const uint32_t k = blockIdx.x * kBuildBlock + threadIdx.x;
    if (k >= n) return;
    head[k] = (k == 0u || codes[k] != codes[k - 1]) ? 1u : 0u;
}

// leaf index of pair k = inclusive scan of heads - 1
__global__ __launch_bounds__(kBuildBlock) void leaf_tables_kernel(const uint64_t *__restrict__ codes,
                                                                  const uint32_t *__restrict__ head,
                                                                  const uint32_t *__restrict__ incl, uint32_t n,
                                                                  uint32_t *__restrict__ leaf_first,
                                                                  uint64_t *__restrict__ leaf_code) {
    const uint32_t k = blockIdx.x * kBuildBlock + threadIdx.x;
    if (k >= n || !head[k]) return;
    const uint32_t l = incl[k] - 1u;
    leaf_first[l] = k;
    leaf_code[l] = codes[k];
}

// leaf_count and the number of octants leaf j opens (pre-order ids follow by an exclusive scan)
__global__ __launch_bounds__(kBuildBlock) void leaf_count_kernel(const uint32_t *__restrict__ leaf_first,
                                                                 const uint64_t *__restrict__ leaf_code, uint32_t L,
                                                                 uint32_t n_pairs, uint32_t depth,
                                                                 uint32_t *__restrict__ leaf_count,
                                                                 uint32_t *__restrict__ opens) {
    const uint32_t j = blockIdx.x * kBuildBlock + threadIdx.x;
    if (j >= L) return;
    leaf_count[j] = (j + 1u < L ? leaf_first[j + 1u] : n_pairs) - leaf_first[j];
    if (j == 0u) {
        opens[j] = depth;
    } else {
        const uint64_t d = leaf_code[j] ^ leaf_code[j - 1u];  // != 0: codes are unique
        opens[j] = (63u - (uint32_t)__clzll((long long)d)) / 3u;
    }
}

// id of the level-`level` octant containing leaf code `code`: opened by the first leaf whose
// code shares the level's prefix
__device__ inline uint32_t octant_at(const uint64_t *__restrict__ leaf_code, const uint32_t *__restrict__ base,
                                     const uint32_t *__restrict__ opens, uint32_t L, uint32_t depth, uint32_t level,
                                     uint64_t code) {
    const uint32_t sh = 3u * (depth - level);
    const uint64_t start = sh >= 64u ? 0ull : (code >> sh) << sh;
    uint32_t lo = 0u, hi = L;  // lower_bound(leaf_code, start)
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (leaf_code[mid] < start) lo = mid + 1u; else hi = mid;
    }
    return base[lo] + (level - (depth - opens[lo]));
}

__global__ __launch_bounds__(kBuildBlock) void link_kernel(const uint64_t *__restrict__ leaf_code,
                                                           const uint32_t *__restrict__ base,
                                                           const uint32_t *__restrict__ opens, uint32_t L,
                                                           uint32_t depth, uint32_t *__restrict__ child,
                                                           uint32_t *__restrict__ mask, uint32_t *__restrict__ up,
                                                           uint8_t *__restrict__ lvl) {
    const uint32_t j = blockIdx.x * kBuildBlock + threadIdx.x;
    if (j >= L) return;
    const uint64_t code = leaf_code[j];
    const uint32_t nj = opens[j], first_level = depth - nj;
    for (uint32_t t = 0; t < nj; ++t) {  // octants opened by this leaf, top down
        const uint32_t level = first_level + t, id = base[j] + t;
        if (level == 0u) continue;  // the root has no parent
        const uint32_t parent = t ? id - 1u : octant_at(leaf_code, base, opens, L, depth, level - 1u, code);
        const uint32_t c = (uint32_t)(code >> (3u * (depth - level))) & 7u;
        child[8u * parent + c] = id;
        atomicOr(&mask[parent], 1u << c);
        if (up) {  // compaction: parent slot and level
            up[id] = 8u * parent + c;
            lvl[id] = (uint8_t)level;
        }
    }
    const uint32_t p = nj ? base[j] + nj - 1u : octant_at(leaf_code, base, opens, L, depth, depth - 1u, code);
    const uint32_t c = (uint32_t)code & 7u;
    child[8u * p + c] = j;  // leaf payload = leaf table index
    atomicOr(&mask[p], (1u << c) | (1u << (c + 8u)));
}

// Compaction (OCTPT_BUILD_COMPACT), one launch per level bottom-up: a level-`level` octant whose
// eight children are leaves holding the same primitive list becomes a leaf of its parent with child
// 0's payload (Octant::is_compactable, new_octree.rs:227-233; RegionOctreeBuilder::recursive_build
// :679-690).  Parents are one level up, handled by the next launch; siblings touch distinct slots.
// up[o] = the parent slot (8 * parent + child index), lvl[o] its level; the root (level 0) stays.
__global__ __launch_bounds__(kBuildBlock) void compact_level_kernel(const uint32_t *__restrict__ up,
                                                                    const uint8_t *__restrict__ lvl, uint32_t n_oct,
                                                                    uint32_t level, const uint32_t *__restrict__ leaf_first,
                                                                    const uint32_t *__restrict__ leaf_count,
                                                                    const uint32_t *__restrict__ prims,
                                                                    uint32_t *__restrict__ child,
                                                                    uint32_t *__restrict__ mask,
                                                                    uint32_t *__restrict__ keep) {
    const uint32_t o = blockIdx.x * kBuildBlock + threadIdx.x;
    if (o == 0u || o >= n_oct) return;  // octant 0 is the root
    if (lvl[o] != level || mask[o] != 0xFFFFu) return;
    const uint32_t c0 = child[8u * o];
    const uint32_t f0 = leaf_first[c0], n0 = leaf_count[c0];
    for (int k = 1; k < 8; ++k) {
        const uint32_t ck = child[8u * o + k];
        if (leaf_count[ck] != n0) return;
        const uint32_t fk = leaf_first[ck];
        for (uint32_t e = 0; e < n0; ++e)
            if (prims[fk + e] != prims[f0 + e]) return;
    }
    keep[o] = 0u;
    const uint32_t slot = up[o];
    child[slot] = c0;
    atomicOr(&mask[slot >> 3], 1u << ((slot & 7u) + 8u));
}

// surviving octants in pre-order: new id = exclusive scan of keep; octant children renumbered
__global__ __launch_bounds__(kBuildBlock) void pack_compacted_kernel(const uint32_t *__restrict__ child,
                                                                     const uint32_t *__restrict__ mask,
                                                                     const uint32_t *__restrict__ keep,
                                                                     const uint32_t *__restrict__ new_id, uint32_t n,
                                                                     octpt_octant *__restrict__ out) {
    const uint32_t o = blockIdx.x * kBuildBlock + threadIdx.x;
    if (o >= n || !keep[o]) return;
    octpt_octant v;
    const uint32_t m = mask[o];
    v.child_mask = (uint16_t)m;
    v.reserved = 0;
    for (int c = 0; c < 8; ++c) {
        const uint32_t x = child[8u * o + c];
        v.children[c] = ((m >> c) & 1u) && !((m >> (c + 8)) & 1u) ? new_id[x] : x;
    }
    out[new_id[o]] = v;
}

// keep[i] = 1 for i < n_ones, 0 for the scan's trailing entry
__global__ __launch_bounds__(kBuildBlock) void fill_u32_kernel(uint32_t *__restrict__ a, uint32_t n, uint32_t n_ones) {
    const uint32_t i = blockIdx.x * kBuildBlock + threadIdx.x;
    if (i < n) a[i] = i < n_ones ? 1u : 0u;
}

__global__ __launch_bounds__(kBuildBlock) void pack_octants_kernel(const uint32_t *__restrict__ child,
                                                                   const uint32_t *__restrict__ mask, uint32_t n,
                                                                   octpt_octant *__restrict__ out) {
    const uint32_t o = blockIdx.x * kBuildBlock + threadIdx.x;
    if (o >= n) return;
    octpt_octant v;
    v.child_mask = (uint16_t)mask[o];
    v.reserved = 0;
    for (int c = 0; c < 8; ++c) v.children[c] = child[8u * o + c];
    out[o] = v;
}

inline uint32_t blocks(uint64_t n) { return (uint32_t)((n + kBuildBlock - 1) / kBuildBlock); }

// slots of the context's grow-only scratch, taken in a fixed order per build
struct ScratchCursor {
    BuildScratch &s;
    int next = 0;  // the build takes at most slots 0..25 in a fixed order, slot_bases_gpu 27..29
    template <class T>
    hipError_t get(T **ptr, size_t n) {
        const int k = next++;
        if (k >= BuildScratch::kSlots) return hipErrorInvalidValue;
        const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        if (s.cap[k] < bytes) {
            if (s.dev[k]) (void)hipFree(s.dev[k]);
            s.dev[k] = nullptr;
            s.cap[k] = 0;
            const size_t want = (bytes + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);  // whole MiB
            const hipError_t e = hipMalloc(&s.dev[k], want);
            if (e != hipSuccess) return e;
            s.cap[k] = want;
        }
        *ptr = static_cast<T *>(s.dev[k]);
        return hipSuccess;
    }
};

}  // namespace

#define BTRY(expr)                                 \
    do {                                           \
        const hipError_t _e = (expr);              \
        if (_e != hipSuccess) return _e;           \
    } while (0)

// Builds on `stream` and returns the host arrays of octpt_octree.  too_many = the pair count
// exceeded max_pairs (nothing else is built then).
void BuildScratch::release() {
    for (int k = 0; k < kSlots; ++k) {
        if (dev[k]) (void)hipFree(dev[k]);
        dev[k] = nullptr;
        cap[k] = 0;
    }
}

hipError_t build_octree_gpu(hipStream_t stream, BuildScratch &scratch, const octpt_sphere *spheres, uint32_t ns,
                            const octpt_cuboid *cuboids, uint32_t nc, uint32_t depth, bool compact,
                            uint64_t max_pairs, BuiltOctree &out, bool &too_many, float *ms,
                            DeviceOctree *dev) {
    too_many = false;
    const int32_t N = 1 << depth;
    const uint32_t np = ns + nc;
    ScratchCursor pool{scratch};
    hipEvent_t e0, e1;
    BTRY(hipEventCreate(&e0));
    BTRY(hipEventCreate(&e1));
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
    } evg{e0, e1};
    octpt_sphere *d_sp;
    octpt_cuboid *d_cb;
    unsigned long long *d_cnt, *d_off;
    BTRY(pool.get(&d_sp, ns));
    BTRY(pool.get(&d_cb, nc));
    BTRY(pool.get(&d_cnt, np));
    BTRY(pool.get(&d_off, np + 1));
    if (ns) BTRY(hipMemcpyAsync(d_sp, spheres, ns * sizeof(octpt_sphere), hipMemcpyHostToDevice, stream));
    if (nc) BTRY(hipMemcpyAsync(d_cb, cuboids, nc * sizeof(octpt_cuboid), hipMemcpyHostToDevice, stream));
    BTRY(hipEventRecord(e0, stream));
    unsigned long long total = 0;
    if (np) {
        hipLaunchKernelGGL(count_cells_kernel, dim3(blocks(np)), dim3(kBuildBlock), 0, stream, d_sp, ns, d_cb, nc, N,
                           d_cnt);
        BTRY(hipGetLastError());
        size_t tmp_bytes = 0;
        BTRY(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, d_cnt, d_off + 1, np, stream));
        void *d_tmp;
        BTRY(pool.get(reinterpret_cast<char **>(&d_tmp), tmp_bytes));
        BTRY(hipMemsetAsync(d_off, 0, sizeof(unsigned long long), stream));
        BTRY(hipcub::DeviceScan::InclusiveSum(d_tmp, tmp_bytes, d_cnt, d_off + 1, np, stream));
        BTRY(hipMemcpyAsync(&total, d_off + np, sizeof total, hipMemcpyDeviceToHost, stream));
        BTRY(hipStreamSynchronize(stream));
    }
    if (total > max_pairs) {
        too_many = true;
        return hipSuccess;
    }
    const uint32_t n = (uint32_t)total;
    out.depth = depth;
    out.root = 0u;
    if (dev) {
        *dev = DeviceOctree{};
        dev->spheres = d_sp;
        dev->cuboids = d_cb;
        dev->ns = ns;
        dev->nc = nc;
        dev->depth = depth;
    }
    if (n == 0u) {  // empty world: a childless root, as the host builder emits
        if (ms) *ms = 0.0f;
        if (dev) {
            octpt_octant *d_root;
            BTRY(pool.get(&d_root, 1));
            BTRY(hipMemsetAsync(d_root, 0, sizeof(octpt_octant), stream));
            BTRY(hipStreamSynchronize(stream));
            dev->octants = d_root;
            dev->n_octants = 1u;
            return hipSuccess;
        }
        out.octants.assign(1, octpt_octant{0, 0, {0, 0, 0, 0, 0, 0, 0, 0}});
        out.leaf_first.clear();
        out.leaf_count.clear();
        out.leaf_prims.clear();
        return hipSuccess;
    }
    uint64_t *d_code, *d_code_s;
    uint32_t *d_prim, *d_prim_s, *d_head, *d_incl;
    BTRY(pool.get(&d_code, n));
    BTRY(pool.get(&d_code_s, n));
    BTRY(pool.get(&d_prim, n));
    BTRY(pool.get(&d_prim_s, n));
    BTRY(pool.get(&d_head, n));
    BTRY(pool.get(&d_incl, n));
    hipLaunchKernelGGL(emit_pairs_kernel, dim3(blocks(np)), dim3(kBuildBlock), 0, stream, d_sp, ns, d_cb, nc, N, d_off,
                       d_code, d_prim);
    BTRY(hipGetLastError());
    size_t sort_bytes = 0, scan_bytes = 0;
    BTRY(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, d_code, d_code_s, d_prim, d_prim_s, n, 0,
                                            (int)(3u * depth), stream));
    BTRY(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, d_head, d_incl, n, stream));
    char *d_tmp;
    BTRY(pool.get(&d_tmp, std::max(sort_bytes, scan_bytes)));
    BTRY(hipcub::DeviceRadixSort::SortPairs(d_tmp, sort_bytes, d_code, d_code_s, d_prim, d_prim_s, n, 0,
                                            (int)(3u * depth), stream));
    hipLaunchKernelGGL(leaf_heads_kernel, dim3(blocks(n)), dim3(kBuildBlock), 0, stream, d_code_s, n, d_head);
    BTRY(hipGetLastError());
    BTRY(hipcub::DeviceScan::InclusiveSum(d_tmp, scan_bytes, d_head, d_incl, n, stream));
    uint32_t L = 0;
    BTRY(hipMemcpyAsync(&L, d_incl + (n - 1), sizeof L, hipMemcpyDeviceToHost, stream));
    BTRY(hipStreamSynchronize(stream));
    uint32_t *d_first, *d_count, *d_opens, *d_base;
    uint64_t *d_lcode;
    BTRY(pool.get(&d_first, L));
    BTRY(pool.get(&d_count, L));
    BTRY(pool.get(&d_opens, L + 1));  // entry L = 0: the exclusive scan's last input
    BTRY(pool.get(&d_base, L + 1));
    BTRY(pool.get(&d_lcode, L));
    BTRY(hipMemsetAsync(d_opens + L, 0, sizeof(uint32_t), stream));
    hipLaunchKernelGGL(leaf_tables_kernel, dim3(blocks(n)), dim3(kBuildBlock), 0, stream, d_code_s, d_head, d_incl, n,
                       d_first, d_lcode);
    BTRY(hipGetLastError());
    hipLaunchKernelGGL(leaf_count_kernel, dim3(blocks(L)), dim3(kBuildBlock), 0, stream, d_first, d_lcode, L, n, depth,
                       d_count, d_opens);
    BTRY(hipGetLastError());
    size_t base_bytes = 0;
    BTRY(hipcub::DeviceScan::ExclusiveSum(nullptr, base_bytes, d_opens, d_base, L + 1, stream));
    // exclusive sum over L + 1 entries: d_base[L] = octant count
    char *d_tmp2;
    BTRY(pool.get(&d_tmp2, base_bytes));
    BTRY(hipcub::DeviceScan::ExclusiveSum(d_tmp2, base_bytes, d_opens, d_base, L + 1, stream));
    uint32_t n_oct = 0;
    BTRY(hipMemcpyAsync(&n_oct, d_base + L, sizeof n_oct, hipMemcpyDeviceToHost, stream));
    BTRY(hipStreamSynchronize(stream));
    uint32_t *d_child, *d_mask, *d_up = nullptr, *d_keep = nullptr, *d_newid = nullptr;
    uint8_t *d_lvl = nullptr;
    octpt_octant *d_oct;
    BTRY(pool.get(&d_child, (size_t)n_oct * 8));
    BTRY(pool.get(&d_mask, n_oct));
    BTRY(pool.get(&d_oct, n_oct));
    if (compact) {
        BTRY(pool.get(&d_up, n_oct));
        BTRY(pool.get(&d_lvl, n_oct));
        BTRY(pool.get(&d_keep, n_oct + 1));  // entry n_oct = 0: the exclusive scan's last input
        BTRY(pool.get(&d_newid, n_oct + 1));
    }
    BTRY(hipMemsetAsync(d_child, 0, (size_t)n_oct * 8 * sizeof(uint32_t), stream));
    BTRY(hipMemsetAsync(d_mask, 0, (size_t)n_oct * sizeof(uint32_t), stream));
    hipLaunchKernelGGL(link_kernel, dim3(blocks(L)), dim3(kBuildBlock), 0, stream, d_lcode, d_base, d_opens, L, depth,
                       d_child, d_mask, d_up, d_lvl);
    BTRY(hipGetLastError());
    if (compact) {
        // keep = 1 per octant, then one pass per level, bottom-up
        hipLaunchKernelGGL(fill_u32_kernel, dim3(blocks(n_oct + 1)), dim3(kBuildBlock), 0, stream, d_keep, n_oct + 1,
                           n_oct);
        BTRY(hipGetLastError());
        for (uint32_t level = depth - 1; level >= 1; --level) {
            hipLaunchKernelGGL(compact_level_kernel, dim3(blocks(n_oct)), dim3(kBuildBlock), 0, stream, d_up, d_lvl, n_oct,
                               level, d_first, d_count, d_prim_s, d_child, d_mask, d_keep);
            BTRY(hipGetLastError());
        }
        size_t id_bytes = 0;
        BTRY(hipcub::DeviceScan::ExclusiveSum(nullptr, id_bytes, d_keep, d_newid, n_oct + 1, stream));
        char *d_tmp3;
        BTRY(pool.get(&d_tmp3, id_bytes));
        BTRY(hipcub::DeviceScan::ExclusiveSum(d_tmp3, id_bytes, d_keep, d_newid, n_oct + 1, stream));
        hipLaunchKernelGGL(pack_compacted_kernel, dim3(blocks(n_oct)), dim3(kBuildBlock), 0, stream, d_child, d_mask,
                           d_keep, d_newid, n_oct, d_oct);
        BTRY(hipGetLastError());
        BTRY(hipMemcpyAsync(&n_oct, d_newid + n_oct, sizeof n_oct, hipMemcpyDeviceToHost, stream));
        BTRY(hipStreamSynchronize(stream));
    } else {
        hipLaunchKernelGGL(pack_octants_kernel, dim3(blocks(n_oct)), dim3(kBuildBlock), 0, stream, d_child, d_mask,
                           n_oct, d_oct);
        BTRY(hipGetLastError());
    }
    BTRY(hipEventRecord(e1, stream));
    if (dev) {  // device-resident: the arrays stay in the scratch
        dev->octants = d_oct;
        dev->leaf_first = d_first;
        dev->leaf_count = d_count;
        dev->leaf_prims = d_prim_s;
        dev->n_octants = n_oct;
        dev->n_leaves = L;
        dev->n_leaf_prims = n;
        BTRY(hipStreamSynchronize(stream));
        if (ms) BTRY(hipEventElapsedTime(ms, e0, e1));
        return hipSuccess;
    }
    out.octants.resize(n_oct);
    out.leaf_first.resize(L);
    out.leaf_count.resize(L);
    out.leaf_prims.resize(n);
    BTRY(hipMemcpyAsync(out.octants.data(), d_oct, (size_t)n_oct * sizeof(octpt_octant), hipMemcpyDeviceToHost,
                        stream));
    BTRY(hipMemcpyAsync(out.leaf_first.data(), d_first, (size_t)L * 4, hipMemcpyDeviceToHost, stream));
    BTRY(hipMemcpyAsync(out.leaf_count.data(), d_count, (size_t)L * 4, hipMemcpyDeviceToHost, stream));
    BTRY(hipMemcpyAsync(out.leaf_prims.data(), d_prim_s, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
    BTRY(hipStreamSynchronize(stream));
    if (ms) BTRY(hipEventElapsedTime(ms, e0, e1));
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// device-resident scene packing (octpt_scene_build_device): the slots octpt_scene_upload packs on
// the host (octpt_api.cpp), from a DeviceOctree, with no round trip through host memory
// ---------------------------------------------------------------------------
namespace {

// present children per octant (the exclusive scan's trailing entry n = 0)
__global__ __launch_bounds__(kBuildBlock) void slot_count_kernel(const octpt_octant *__restrict__ oct, uint32_t n,
                                                                 uint32_t *__restrict__ cnt) {
    const uint32_t o = blockIdx.x * kBuildBlock + threadIdx.x;
    if (o > n) return;
    cnt[o] = o < n ? (uint32_t)__popc(oct[o].child_mask & 0xFFu) : 0u;
}

// octant o's present children from base[o] in child order: octant child = (its base, its mask),
// single-primitive leaf = (prim id, 1), else (first list index, count); sphere-only scenes also get
// the single-sphere leaf's sphere beside the slot (leaf_sph, zero elsewhere)
__global__ __launch_bounds__(kBuildBlock) void slot_fill_kernel(const octpt_octant *__restrict__ oct, uint32_t n,
                                                                const uint32_t *__restrict__ base,
                                                                const uint32_t *__restrict__ first,
                                                                const uint32_t *__restrict__ count,
                                                                const uint32_t *__restrict__ prims,
                                                                const octpt_sphere *__restrict__ sp,
                                                                uint2 *__restrict__ child, float4 *__restrict__ leaf_sph) {
    const uint32_t o = blockIdx.x * kBuildBlock + threadIdx.x;
    if (o >= n) return;
    const octpt_octant v = oct[o];
    const uint32_t m = v.child_mask;
    uint32_t k = base[o];
    for (int i = 0; i < 8; ++i) {
        if (!((m >> i) & 1u)) continue;
        const uint32_t c = v.children[i];
        if (!((m >> (i + 8)) & 1u)) {
            child[k] = make_uint2(base[c], oct[c].child_mask);
        } else if (count[c] == 1u) {
            const uint32_t p = prims[first[c]];
            child[k] = make_uint2(p, 1u);
            if (leaf_sph) {
                const octpt_sphere s = sp[p];
                leaf_sph[k] = make_float4(s.center[0], s.center[1], s.center[2], s.radius);
            }
        } else {
            child[k] = make_uint2(first[c], count[c]);
        }
        ++k;
    }
}

__global__ __launch_bounds__(kBuildBlock) void prim_tables_kernel(const octpt_sphere *__restrict__ sp, uint32_t ns,
                                                                  const octpt_cuboid *__restrict__ cb, uint32_t nc,
                                                                  float4 *__restrict__ sph, uint32_t *__restrict__ sph_mat,
                                                                  float4 *__restrict__ cub_a, float2 *__restrict__ cub_b,
                                                                  uint32_t *__restrict__ cub_mat) {
    const uint32_t i = blockIdx.x * kBuildBlock + threadIdx.x;
    if (i < ns) {
        const octpt_sphere s = sp[i];
        sph[i] = make_float4(s.center[0], s.center[1], s.center[2], s.radius);
        sph_mat[i] = s.material;
    } else if (i < ns + nc) {
        const uint32_t c = i - ns;
        const octpt_cuboid b = cb[c];
        cub_a[c] = make_float4(b.min[0], b.min[1], b.min[2], b.max[0]);
        cub_b[c] = make_float2(b.max[1], b.max[2]);
        for (int f = 0; f < 6; ++f) cub_mat[6u * c + f] = b.face_material[f];
    }
}

}  // namespace

hipError_t slot_bases_gpu(hipStream_t stream, BuildScratch &scratch, const DeviceOctree &t, uint32_t **d_base,
                          uint32_t &n_slots) {
    ScratchCursor pool{scratch, 27};  // after the build's own slots (0..25)
    const uint32_t n = t.n_octants;
    uint32_t *d_cnt;
    BTRY(pool.get(&d_cnt, n + 1));
    BTRY(pool.get(d_base, n + 1));
    hipLaunchKernelGGL(slot_count_kernel, dim3(blocks(n + 1)), dim3(kBuildBlock), 0, stream, t.octants, n, d_cnt);
    BTRY(hipGetLastError());
    size_t bytes = 0;
    BTRY(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, d_cnt, *d_base, n + 1, stream));
    char *d_tmp;
    BTRY(pool.get(&d_tmp, bytes));
    BTRY(hipcub::DeviceScan::ExclusiveSum(d_tmp, bytes, d_cnt, *d_base, n + 1, stream));
    BTRY(hipMemcpyAsync(&n_slots, *d_base + n, sizeof n_slots, hipMemcpyDeviceToHost, stream));
    return hipStreamSynchronize(stream);
}

hipError_t fill_scene_gpu(hipStream_t stream, const DeviceOctree &t, const uint32_t *d_base,
                          const ScenePrimTables &out) {
    if (t.n_octants) {
        hipLaunchKernelGGL(slot_fill_kernel, dim3(blocks(t.n_octants)), dim3(kBuildBlock), 0, stream, t.octants,
                           t.n_octants, d_base, t.leaf_first, t.leaf_count, t.leaf_prims, t.spheres, out.node_child,
                           out.leaf_sph);
        BTRY(hipGetLastError());
    }
    if (t.n_leaf_prims)
        BTRY(hipMemcpyAsync(out.leaf_prims, t.leaf_prims, (size_t)t.n_leaf_prims * 4, hipMemcpyDeviceToDevice, stream));
    if (t.ns + t.nc) {
        hipLaunchKernelGGL(prim_tables_kernel, dim3(blocks((uint64_t)t.ns + t.nc)), dim3(kBuildBlock), 0, stream,
                           t.spheres, t.ns, t.cuboids, t.nc, out.spheres, out.sphere_mat, out.cub_a, out.cub_b,
                           out.cub_mat);
        BTRY(hipGetLastError());
    }
    return hipStreamSynchronize(stream);
}

}  // namespace octpt
