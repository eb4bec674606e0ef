// Exhaustive check of octpt::rcp_rn (csrc/octpt_rcp.h) against the correctly rounded division 1.0f / a
// (this file is built with -fhip-fp32-correctly-rounded-divide-sqrt, as liboctpt is) for every float a
// with |a| in [2^-23, 2^126], both signs (every quotient a normal float).  Prints the number of values checked and of mismatches, exit 0 iff
// there are none.  Built by __graft_entry__.build(); run by tests/test_gpu_beam.py on the GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../octree_pathtracing_amd/csrc/octpt_rcp.h"

__global__ void check(uint32_t lo, uint32_t n, unsigned long long *bad, uint32_t *first) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float a = __uint_as_float(lo + i);
        const bool ok = __float_as_uint(octpt::rcp_rn(a)) == __float_as_uint(1.0f / a) &&
                        __float_as_uint(octpt::rcp_rn(-a)) == __float_as_uint(1.0f / -a);
        if (!ok) {
            atomicAdd(bad, 1ull);
            atomicCAS(first, 0u, lo + i);
        }
    }
}

int main() {
    const uint32_t lo = 0x34000000u;  // 2^-23
    const uint32_t hi = 0x7E800000u;  // 2^126
    const uint32_t n = hi - lo + 1u;
    unsigned long long *bad;
    uint32_t *first;
    if (hipMalloc(&bad, sizeof *bad) != hipSuccess || hipMalloc(&first, sizeof *first) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, sizeof *bad);
    (void)hipMemset(first, 0, sizeof *first);
    hipLaunchKernelGGL(check, dim3(16384), dim3(256), 0, 0, lo, n, bad, first);
    unsigned long long h_bad = 0;
    uint32_t h_first = 0;
    if (hipMemcpy(&h_bad, bad, sizeof h_bad, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    (void)hipMemcpy(&h_first, first, sizeof h_first, hipMemcpyDeviceToHost);
    std::printf("checked %u values (x2 signs), mismatches %llu, first 0x%08x\n", n, h_bad, h_first);
    return h_bad == 0 ? 0 : 1;
}
