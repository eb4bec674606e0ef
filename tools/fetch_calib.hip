// FETCH_SIZE calibration for wf_extend_kernel's access shapes ("Traffic").
//
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16-B/lane coalesced streaming reads (it reports
// half of the bytes).  extend reads 8-B node slots and 16-B leaf spheres at scattered addresses, so
// this tool issues reads of a known footprint in each shape; run it under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/fetch_calib
// and divide each kernel's FETCH_SIZE by the footprint it prints (scripts/fetch_calib.py does this).
//
//   stream16   : 16 B per lane, coalesced, over a 1 GiB buffer (the guide's calibrated case)
//   gather8    : 8 B per lane at hashed addresses in a 2 GiB table (beyond the 256 MiB Infinity
//                Cache): the footprint is the number of distinct 64-B / 128-B lines touched, counted
//                on the host from the same hash
//   gather16   : the same with 16-B reads (extend's leaf-sphere loads)
//   gather8_l3 : 8-B hashed reads, 16 passes over a 6 MiB table (C3's node table is 5.9 MB): shows
//                whether lines served by L2 / the Infinity Cache reach FETCH_SIZE
//
// Built with hipcc --offload-arch=gfx950 -O3 (scripts: tools/Makefile).  Each kernel writes one
// word per wave so that the loads are not dead.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <unordered_set>
#include <vector>

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

__host__ __device__ inline uint32_t mix32(uint32_t x) {  // lowbias32
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void stream16(const uint4 *__restrict__ a, size_t n, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0xFFFFFFFFu) out[blockIdx.x] = acc;
}

// element i of lane g, pass p: hashed index into [0, n_elems)
__host__ __device__ inline uint64_t gather_index(uint32_t g, uint32_t p, uint64_t n_elems) {
    const uint64_t h = ((uint64_t)mix32(g * 2654435761u + p * 0x9E3779B9u) << 32) | mix32(g ^ (p + 0x632BE5ABu));
    return h % n_elems;
}

template <typename T>
__global__ __launch_bounds__(256) void gather(const T *__restrict__ a, uint64_t n_elems, uint32_t n_lanes,
                                              uint32_t passes, uint32_t *__restrict__ out) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;
    if (g >= n_lanes) return;
    uint32_t acc = 0;
    for (uint32_t p = 0; p < passes; ++p) {
        const T v = a[gather_index(g, p, n_elems)];
        acc ^= reinterpret_cast<const uint32_t *>(&v)[0];
    }
    if (acc == 0xFFFFFFFFu) out[g] = acc;
}

static size_t distinct_lines(uint64_t n_elems, uint32_t elem_bytes, uint32_t n_lanes, uint32_t passes, uint32_t line) {
    std::unordered_set<uint64_t> s;
    s.reserve((size_t)n_lanes * passes);
    for (uint32_t p = 0; p < passes; ++p)
        for (uint32_t g = 0; g < n_lanes; ++g) s.insert(gather_index(g, p, n_elems) * elem_bytes / line);
    return s.size();
}

int main() {
    const size_t big = 2ull << 30, stream_bytes = 1ull << 30, small = 6ull << 20;
    void *d_big = nullptr;
    uint32_t *d_out = nullptr;
    CHECK(hipMalloc(&d_big, big));
    CHECK(hipMalloc(&d_out, 64u << 20));
    CHECK(hipMemset(d_big, 0x5A, big));
    CHECK(hipDeviceSynchronize());
    const uint32_t lanes = 4u << 20;  // 4 M scattered reads: ~12 % of them share a 64-B line

    stream16<<<1024 * 8, 256>>>(static_cast<const uint4 *>(d_big), stream_bytes / 16, d_out);
    CHECK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"stream16\", \"footprint_bytes\": %zu}\n", stream_bytes);

    const uint64_t n8 = big / 8;
    gather<uint2><<<lanes / 256, 256>>>(static_cast<const uint2 *>(d_big), n8, lanes, 1, d_out);
    CHECK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"gather8\", \"reads\": %u, \"read_bytes\": %llu, \"lines64\": %zu, \"lines128\": %zu}\n",
                lanes, (unsigned long long)lanes * 8ull, distinct_lines(n8, 8, lanes, 1, 64),
                distinct_lines(n8, 8, lanes, 1, 128));

    const uint64_t n16 = big / 16;
    gather<uint4><<<lanes / 256, 256>>>(static_cast<const uint4 *>(d_big), n16, lanes, 1, d_out);
    CHECK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"gather16\", \"reads\": %u, \"read_bytes\": %llu, \"lines64\": %zu, \"lines128\": %zu}\n",
                lanes, (unsigned long long)lanes * 16ull, distinct_lines(n16, 16, lanes, 1, 64),
                distinct_lines(n16, 16, lanes, 1, 128));

    // resident table: a separate 6 MiB region, touched once before the timed kernel
    const uint64_t ns = small / 8;
    const uint2 *tab = reinterpret_cast<const uint2 *>(static_cast<const char *>(d_big) + big - small);
    gather<uint2><<<lanes / 256, 256>>>(tab, ns, lanes, 1, d_out);
    CHECK(hipDeviceSynchronize());
    const uint32_t passes = 16;
    gather<uint2><<<lanes / 256, 256>>>(tab, ns, lanes, passes, d_out);
    CHECK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"gather8_l3\", \"reads\": %llu, \"read_bytes\": %llu, \"table_bytes\": %zu}\n",
                (unsigned long long)lanes * passes, (unsigned long long)lanes * passes * 8ull, (size_t)small);
    CHECK(hipFree(d_big));
    CHECK(hipFree(d_out));
    return 0;
}
