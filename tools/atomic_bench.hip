// Microbenchmark: throughput of one-lane-per-wave atomicAdd-with-return (the wavefront queue
// ticket) on one counter vs counters sharded per XCD / per CU-slot.  Diagnostic tool only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void ticket_kernel(unsigned *ctr, unsigned iters, unsigned shards, unsigned stride, unsigned *sink) {
    const unsigned lane = threadIdx.x & 63u;
    unsigned acc = 0;
    unsigned *c = ctr + (blockIdx.x % shards) * stride;
    for (unsigned k = 0; k < iters; ++k) {
        const unsigned long long m = __ballot(lane < 40u);
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(c, (unsigned)__popcll(m));
        base = __shfl(base, 0);
        acc += base + lane;
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

int main(int argc, char **argv) {
    const unsigned blocks = argc > 1 ? atoi(argv[1]) : 1024, iters = argc > 2 ? atoi(argv[2]) : 12;
    unsigned *ctr, *sink;
    hipMalloc(&ctr, 1 << 20);
    hipMalloc(&sink, 64);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const unsigned cfg[][2] = {{1, 0}, {8, 64}, {64, 64}, {1024, 64}};
    for (auto &c : cfg) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(ctr, 0, 1 << 20);
            hipEventRecord(a);
            hipLaunchKernelGGL(ticket_kernel, dim3(blocks), dim3(256), 0, 0, ctr, iters, c[0], c[1], sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double n = (double)blocks * 4 * iters;
            if (rep == 2)
                printf("shards %5u: %8.1f us  %.3g wave-atomics  %.1f M atomics/s\n", c[0], ms * 1e3, n, n / ms / 1e3);
        }
    }
    return 0;
}
