// Host check of multi_slot (octpt_internal.h), the tile bookkeeping of a multi-device render
// (octpt_create_multi), against the kernels' own shard rule: tile t of a W x H frame
// (8x8 tiles, row-major) belongs to shard t % count as its local tile t / count.  For every frame size,
// caller shard and entry count below, the caller's items must map one to one onto the entries' compact
// buffers -- entry i rendering shard shard_index + i * shard_count of shard_count * n -- and a frame-layout
// item onto its own pixel.  Round 5: with and without a tile order (octpt_set_tile_order: dealing position s
// holds frame tile order[s]; here a seeded shuffle).  Built and run by tests/test_multi_cpu.py (g++, no GPU).
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../octree_pathtracing_amd/csrc/octpt_internal.h"

using namespace octpt;

static uint32_t tiles_of(uint32_t n_tiles, uint32_t shard, uint32_t count) {
    uint32_t k = 0;
    for (uint32_t t = shard; t < n_tiles; t += count) ++k;
    return k;
}

int main() {
    long checked = 0, bad = 0;
    const uint32_t sizes[][2] = {{1, 1}, {8, 8}, {9, 17}, {70, 45}, {64, 64}, {129, 33}, {200, 120}, {17, 300}};
    for (const auto &wh : sizes) {
        const uint32_t W = wh[0], H = wh[1], tx = (W + 7) / 8, n_tiles = tx * ((H + 7) / 8);
        std::vector<uint32_t> shuffled(n_tiles);
        for (uint32_t t = 0; t < n_tiles; ++t) shuffled[t] = t;
        std::shuffle(shuffled.begin(), shuffled.end(), std::mt19937(W * 131u + H));
        for (int use_order = 0; use_order <= 1; ++use_order)
        for (uint32_t C = 1; C <= 3; ++C)
            for (uint32_t s = 0; s < C; ++s)
                for (uint32_t n = 1; n <= 9; ++n)
                    for (int compact = 0; compact <= 1; ++compact) {
                        const uint32_t U = tiles_of(n_tiles, s, C);
                        const uint32_t stride = (U + n - 1) / n * 64u;
                        std::vector<int> hits((size_t)stride * n + 1, 0);
                        for (uint32_t i = 0; i < U * 64u; ++i) {
                            uint32_t caller = 0, staged = 0;
                            const uint32_t *order = use_order ? shuffled.data() : nullptr;
                            const bool in = multi_slot(W, H, tx, s, C, compact != 0, n, stride, i, caller, staged,
                                                       order);
                            const uint32_t u = i / 64u, k = i % 64u, t = s + u * C;  // t: the dealing position
                            const uint32_t ft = use_order ? shuffled[t] : t;      // the frame tile there
                            const uint32_t x = (ft % tx) * 8 + k % 8, y = (ft / tx) * 8 + k / 8;
                            const bool inside = x < W && y < H;
                            // the entry owning tile t under the kernels' rule, and its local tile
                            const uint32_t e = (t % (C * n) - s) / C, lt = t / (C * n);
                            bool ok = (t % (C * n)) % C == s && e < n && staged == e * stride + lt * 64u + k &&
                                      lt < tiles_of(n_tiles, s + e * C, C * n);
                            if (compact) ok = ok && in && caller == i;
                            else ok = ok && in == inside && (!in || caller == y * W + x);
                            if (ok && in) ok = ++hits[staged] == 1;
                            ++checked;
                            if (!ok && bad++ < 5)
                                std::printf("mismatch W=%u H=%u C=%u s=%u n=%u compact=%d item=%u\n", W, H, C, s, n,
                                            compact, i);
                        }
                        for (uint32_t e = 0; e < n; ++e)  // every pixel of every entry's buffer is covered
                            for (uint32_t lt = 0; lt < tiles_of(n_tiles, s + e * C, C * n); ++lt)
                                for (uint32_t k = 0; k < 64; ++k) {
                                    const uint32_t t = s + e * C + lt * C * n;
                                    const uint32_t ft = use_order ? shuffled[t] : t;
                                    const bool inside = (ft % tx) * 8 + k % 8 < W && (ft / tx) * 8 + k / 8 < H;
                                    if ((compact || inside) && hits[e * stride + lt * 64 + k] != 1 && bad++ < 5)
                                        std::printf("uncovered W=%u H=%u C=%u s=%u n=%u e=%u lt=%u k=%u\n", W, H, C, s,
                                                    n, e, lt, k);
                                }
                    }
    }
    std::printf("checked %ld items, mismatches %ld\n", checked, bad);
    return bad ? 1 : 0;
}
