// shpl_tilesort.h -- one-workgroup stable sort of packed 64-bit words by
// their numeric value, used where a frame's work must be grouped by key in
// the reference's order (voxel cells, MV3D voxels): an LDS histogram over
// key tiles, an exclusive scan, LDS-atomic placement into tile segments and
// an in-tile rank (words are unique, so the rank is the count of smaller
// words of the tile, read from an LDS window of the placed words). Tiles hold
// a few words each, so the quadratic rank is cheaper than a second sort pass.
#pragma once

#include "shpl_common.h"

namespace shpl {

constexpr int TS_BLOCK = 1024;
constexpr int TS_TILES = 16384;
constexpr int TS_WIN = 10240;  // placed words staged in LDS for the rank (80 KiB)

struct TileSortLds {
    int32_t cnt[TS_TILES];
    int32_t wsum[TS_BLOCK / 64];
    uint64_t win[TS_WIN];
};

// Block-wide exclusive scan of the TS_TILES counters in place.
__device__ __forceinline__ void ts_scan(TileSortLds &l) {
    constexpr int PER = TS_TILES / TS_BLOCK;
    int32_t v[PER];
    int32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        v[q] = l.cnt[threadIdx.x * PER + q];
        sum += v[q];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) l.wsum[wid] = x;
    __syncthreads();
    int32_t run = x - sum;
    for (int w = 0; w < wid; ++w) run += l.wsum[w];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        l.cnt[threadIdx.x * PER + q] = run;
        run += v[q];
    }
}

// Sorts the words produced by `each(emit)` (every thread enumerates its share
// and calls emit(word) per word) into srt[0..n), using tmp[0..n) as scratch.
// tile(word) -> tile index in [0, n_tiles). Returns n (same in every thread).
template <typename Each, typename Tile>
__device__ int32_t tile_sort(TileSortLds &l, int n_tiles, uint64_t *tmp, uint64_t *srt, Each &&each, Tile &&tile) {
    for (int t = threadIdx.x; t < TS_TILES; t += TS_BLOCK) l.cnt[t] = 0;
    block_publish();  // the caller's earlier global stores (e.g. zeroed flags) land first
    each([&](uint64_t w) { atomicAdd(&l.cnt[tile(w)], 1); });
    __syncthreads();
    ts_scan(l);
    __syncthreads();
    each([&](uint64_t w) { tmp[atomicAdd(&l.cnt[tile(w)], 1)] = w; });
    block_publish();  // tmp came from other waves through memory
    const int32_t n = l.cnt[n_tiles - 1];
    // rank of each word inside its tile, the tile's words read from an LDS window
    for (int32_t w0 = 0; w0 < n; w0 += TS_WIN) {
        const int32_t w1 = w0 + TS_WIN < n ? w0 + TS_WIN : n;
        for (int32_t s = w0 + threadIdx.x; s < w1; s += TS_BLOCK) l.win[s - w0] = tmp[s];
        __syncthreads();
        for (int32_t s = w0 + threadIdx.x; s < w1; s += TS_BLOCK) {
            const uint64_t me = l.win[s - w0];
            const int t = tile(me);
            const int32_t a = t ? l.cnt[t - 1] : 0, b = l.cnt[t];
            int32_t rank = 0;
            if (a >= w0 && b <= w1) {
                for (int32_t u = a; u < b; ++u) rank += l.win[u - w0] < me ? 1 : 0;
            } else {  // the tile straddles the window edge
                for (int32_t u = a; u < b; ++u) rank += tmp[u] < me ? 1 : 0;
            }
            srt[a + rank] = me;
        }
        __syncthreads();  // the next window overwrites win
    }
    block_publish();
    return n;
}

}  // namespace shpl
