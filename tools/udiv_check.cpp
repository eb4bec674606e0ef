// Check of octpt_internal.h's fixed-divisor division (udiv_magic / udiv_c, the item -> pixel maps of the kernels)
// against the C division: every divisor 1..4096, the frame sizes' tile and item counts, and divisors up to 2^32 - 1,
// each with the edge numerators (0, multiples of d and their neighbours, 2^32 - 1) and 2^13 random ones.  Host code;
// the device path is the same arithmetic with __umulhi (tests/test_udiv_cpu.py builds and runs this).
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../octree_pathtracing_amd/csrc/octpt_internal.h"

int main() {
    std::vector<uint32_t> ds;
    for (uint32_t d = 1; d <= 4096; ++d) ds.push_back(d);
    for (uint32_t d : {240u, 480u, 160u, 32400u * 64u, 129600u * 64u, 518400u, 2073600u, 8294400u, 530841600u,
                       0x7FFFFFFFu, 0x80000000u, 0x80000001u, 0xFFFFFFFEu, 0xFFFFFFFFu})
        ds.push_back(d);
    std::mt19937_64 rng(12345);
    for (int i = 0; i < 2000; ++i) ds.push_back((uint32_t)(rng() >> 32) | 1u);
    uint64_t checks = 0, bad = 0;
    for (uint32_t d : ds) {
        const uint64_t c = octpt::udiv_magic(d);
        auto check = [&](uint32_t n) {
            ++checks;
            if (octpt::udiv_c(n, c) != n / d) {
                if (++bad < 10) std::printf("mismatch: %u / %u -> %u\n", n, d, octpt::udiv_c(n, c));
            }
        };
        check(0u);
        check(0xFFFFFFFFu);
        check(0xFFFFFFFEu);
        for (uint64_t k = 1; k <= 64; ++k) {
            const uint64_t m = k * d;
            if (m <= 0xFFFFFFFFull) check((uint32_t)m);
            if (m - 1 <= 0xFFFFFFFFull) check((uint32_t)(m - 1));
            if (m + 1 <= 0xFFFFFFFFull) check((uint32_t)(m + 1));
            const uint64_t top = (0xFFFFFFFFull / d) * d;  // the largest multiple and its neighbours
            if (top >= k * d) { check((uint32_t)(top - (k - 1) * d)); check((uint32_t)(top - (k - 1) * d - 1)); }
        }
        for (int i = 0; i < 8192; ++i) check((uint32_t)(rng() >> 32));
    }
    std::printf("udiv_check: %llu divisions, %llu mismatches\n", (unsigned long long)checks, (unsigned long long)bad);
    return bad ? 1 : 0;
}
