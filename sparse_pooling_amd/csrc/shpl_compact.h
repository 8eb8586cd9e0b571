// shpl_compact.h -- batched, stable per-frame compaction used by the point
// stages (index builder, KITTI velodyne loader): every frame's points are cut
// into chunks of IDX_CHUNK points, one 1024-thread workgroup per chunk.
//   k_count   -- kept points per chunk (Stage::load + Stage::eval)
//   k_compact -- the chunk's kept points land after those of the frame's
//                earlier chunks, in point order; each chunk also writes the
//                sentinels of the unused capacity in its stretch of slots, and
//                the frame's last chunk the frame's count.
// A Stage provides: In/Payload types, load(i, in), eval(ctx, f, i, in, pl) ->
// flag mask, touch(f, i, pl, keep) (every point, write pass), emit(f, i, pos,
// fstart, pl), hole(pos) and HAS_BUCKETS (with bucket_keys, see Bkt).
//
// Column counts. numpy's np.dot over a frame's points evaluates a row product
// in one order for two or more columns (dgemm) and in another for exactly one
// (dgemv; shpl_common.h dot4_gemv). A stage's products therefore depend on
// per-frame counts: ctx.n_live (the frame's points, known up front) and
// ctx.n_aux (how many points pass the stage's first filter -- the columns of
// its second product; -1 = not yet known, in k_count). eval returns
//   KEEP_MULTI -- kept, when the second product has >= 2 columns (or none)
//   KEEP_ONE   -- kept, when it has exactly one (n_aux == 1)
//   AUX        -- the point is one of the second product's columns
// k_count counts all three per chunk; k_compact sums the AUX counts of the
// frame first, then uses the matching KEEP count and passes n_aux to eval.
#pragma once

#include "shpl_common.h"

namespace shpl {
namespace {

constexpr int IDX_BLOCK = 1024;
#ifndef SHPL_IDX_BATCH
#define SHPL_IDX_BATCH 1
#endif
constexpr int IDX_BATCH = SHPL_IDX_BATCH;         // point rows per thread whose loads are in flight together
constexpr int IDX_CHUNK = IDX_BLOCK * IDX_BATCH;  // points per workgroup: one round

constexpr uint32_t KEEP_MULTI = 1u, KEEP_ONE = 2u, AUX = 4u;

struct Ctx {
    int64_t n_live;  // live points of the frame
    int64_t n_aux;   // points of the frame with AUX set; -1 = unknown (k_count)
};

struct Frames {
    const int64_t *pt_off, *pt_count;
    int n_frames, n_chunks;  // chunks of IDX_CHUNK points per frame (grid.x)
    int32_t *chunk_kept;     // [3][n_frames][n_chunks] workspace: KEEP_MULTI, KEEP_ONE, AUX counts
    int64_t *frame_nnz, *frame_out_off;
    uint32_t *err;
};

// Destination buckets of the kept entries (BKT instantiations; shpl_common.h
// BkLayout): k_count adds per-chunk histograms over each key's destination
// ranges, k_compact places every kept entry with valid destinations into its
// (key, range) bucket, stably -- after the frame's earlier ranges and the
// range's entries of earlier chunks, in chunk order inside the chunk.
// A Stage with buckets provides bucket_keys(pl, kc, kp): the entry's
// frame-local destinations (BEV cell, image pixel), false if either is invalid.
// Frames of at most one entry get no bucket (the pull reads that entry from
// the index arrays): only there may the second projection's column count
// (dgemv order) differ from the count k_count assumed.
// A rider of the bucketed launches (optional): extra workgroups of each launch
// copy row bytes [0, row_bytes) of frame f's rows_per_frame rows from src to
// out (16-byte pieces, nontemporal) -- the concat's pass-through halves, which
// need no index: k_count copies cp[0], k_compact cp[1], so the copies ride
// the two latency-bound launches instead of a stream of their own.
struct PassCopy {
    const uint8_t *src;
    uint8_t *out;
    int64_t src_stride, out_stride, row_bytes, rows_per_frame;  // bytes (16-byte multiples), rows
};

struct Bkt {
    int nr[2], nrmax;
    int64_t nnz_cap;
    int32_t *hist;    // [2][F][n_chunks][nrmax]
    int32_t *ext;     // [2][F][nrmax][2]
    uint32_t *words;  // [2][nnz_cap]
    PassCopy cp[2];
    int cp_at[2];     // the launch each copy rides: 0 = k_count, 1 = k_compact
    int cp_blocks;    // rider workgroups per frame in each launch (0: none)
    int32_t *bar;     // [2][F] k_index1's frame barrier words (arrivals, departures): zero between calls
};

#ifndef SHPL_CP_BATCH
#define SHPL_CP_BATCH 8
#endif
constexpr int CP_BATCH = SHPL_CP_BATCH;  // 16-byte pieces per thread in flight

// 32-bit piece arithmetic (a frame's pieces < 2^31, checked on the host; a shift when a row holds a power of
// two of pieces): the 64-bit divisions of an earlier form held the rider path at 111 / 122 VGPRs, and with it
// the whole launch at one 1024-thread workgroup per CU.
__device__ __forceinline__ void pass_copy(const PassCopy &c, int f, int b, int nb) {
    typedef uint32_t u32x4c __attribute__((ext_vector_type(4)));
    const uint32_t per_row = (uint32_t)(c.row_bytes >> 4), total = (uint32_t)c.rows_per_frame * per_row;
    const int sh = per_row & (per_row - 1) ? -1 : __builtin_ctz(per_row);
    const uint8_t *src = c.src + (int64_t)f * c.rows_per_frame * c.src_stride;
    uint8_t *out = c.out + (int64_t)f * c.rows_per_frame * c.out_stride;
    const uint32_t step = (uint32_t)nb * IDX_BLOCK;
    for (uint32_t i0 = (uint32_t)b * IDX_BLOCK + threadIdx.x; i0 < total; i0 += step * CP_BATCH) {
        u32x4c v[CP_BATCH];
#pragma unroll
        for (int u = 0; u < CP_BATCH; ++u) {
            const uint32_t i = i0 + u * step;
            if (i >= total) continue;
            const uint32_t row = sh >= 0 ? i >> sh : i / per_row, pc = i - row * per_row;
            v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4c *>(src + (uint64_t)row * c.src_stride) + pc);
        }
#pragma unroll
        for (int u = 0; u < CP_BATCH; ++u) {
            const uint32_t i = i0 + u * step;
            if (i >= total) continue;
            const uint32_t row = sh >= 0 ? i >> sh : i / per_row, pc = i - row * per_row;
            __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4c *>(out + (uint64_t)row * c.out_stride) + pc);
        }
    }
}

// A caller's shpl_pass_copy (rows_per_frame rows per frame) as a PassCopy: SHPL_OK, or the status its shape
// gets (SHPL_ERR_ARG / SHPL_ERR_BAD_SHAPE); *bytes += its read + write bytes per frame. NULL or 0 channels:
// no copy (row_bytes 0).
inline int make_pass_copy(const shpl_pass_copy *c, int64_t rows_per_frame, PassCopy *pc, int64_t *bytes) {
    *pc = PassCopy{};
    if (!c || c->channels == 0) return SHPL_OK;
    if (c->dtype != SHPL_F32 && c->dtype != SHPL_BF16) return SHPL_ERR_ARG;
    if (!c->src || !c->out || c->channels < 0) return SHPL_ERR_ARG;
    const int64_t esz = c->dtype == SHPL_F32 ? 4 : 2;
    const int64_t rb = c->channels * esz;
    if (rb % 16 || (c->src_stride * esz) % 16 || (c->out_stride * esz) % 16 || ((uintptr_t)c->src & 15) ||
        ((uintptr_t)c->out & 15) || c->src_stride < c->channels || c->out_stride < c->channels ||
        (rb / 16) * rows_per_frame >= ((int64_t)1 << 31))  // a frame's pieces in 32 bits
        return SHPL_ERR_BAD_SHAPE;
    *pc = PassCopy{(const uint8_t *)c->src, (uint8_t *)c->out, c->src_stride * esz, c->out_stride * esz, rb,
                   rows_per_frame};
    *bytes += 2 * rb * rows_per_frame;
    return SHPL_OK;
}

// Rider workgroups per frame for copies of `bytes` per frame: ~240 over the batch (the chip's CUs beside the
// latency-bound workgroups), at most one per 64 KiB of a frame's copy.
inline int rider_blocks(int n_frames, int64_t bytes) {
    if (bytes <= 0) return 0;
    int64_t per = 240 / n_frames;
    const int64_t by_size = bytes / (64 * 1024);
    if (per > by_size) per = by_size;
    return (int)(per < 1 ? 1 : per);
}

__device__ __forceinline__ void frame_range(const Frames &fr, int f, int64_t &p0, int64_t &p1, int64_t &cap_end) {
    p0 = fr.pt_off[f];
    cap_end = fr.pt_off[f + 1];
    // live points of the frame: [p0, p0 + count) when counts are given (capacity layout input)
    p1 = fr.pt_count ? (p0 + fr.pt_count[f] < cap_end ? p0 + fr.pt_count[f] : cap_end) : cap_end;
}

#ifndef SHPL_IDX1_PROBE
#define SHPL_IDX1_PROBE 0  // 1: each chunk workgroup's s_memrealtime stamps into g_idx1_probe (probe builds)
#endif
#if SHPL_IDX1_PROBE
constexpr int IDX1_PROBE_BLOCKS = 4096;
__device__ uint64_t g_idx1_probe[IDX1_PROBE_BLOCKS * 8];
#define SHPL_IDX1_STAMP(k)                                                                          \
    do {                                                                                            \
        if (threadIdx.x == 0 && blockIdx.x < IDX1_PROBE_BLOCKS) {                                            \
            uint64_t t_;                                                                            \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
            g_idx1_probe[blockIdx.x * 8 + (k)] = t_;                                                         \
        }                                                                                           \
    } while (0)
#else
#define SHPL_IDX1_STAMP(k) \
    do {                   \
    } while (0)
#endif
// A block barrier for LDS data only: no wait for the wave's global stores (__syncthreads() drains vmcnt, which
// after the entries' stores held each barrier of the placement for their round trip to memory).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void store_agent(int32_t *p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the frame's aggregates are read with sc1 loads (agent scope, past this CU's L1): k_index1's barrier then
// needs no acquire fence (the guide's hand-off with every handed-off byte stored and loaded sc1)
__device__ __forceinline__ int32_t load_agent(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Pass 1 of chunk j of frame f: KEEP_MULTI / KEEP_ONE / AUX points, and (BKT) the chunk's histograms over
// the destination ranges; leaves the chunk's points in `in`.
template <typename Stage, bool BKT>
__device__ __forceinline__ void count_phase(const Stage &st, const Frames &fr, const Bkt &bk, int f, int j,
                                            typename Stage::In (&in)[IDX_BATCH], uint32_t (&m_out)[IDX_BATCH],
                                            typename Stage::Payload (&pl_out)[IDX_BATCH]) {
    __shared__ int32_t wsum[3][IDX_BLOCK / 64];
    __shared__ int32_t hist[BKT ? 2 * BK_MAX_RANGES : 1];
    if constexpr (BKT) {
        for (int q = threadIdx.x; q < 2 * BK_MAX_RANGES; q += IDX_BLOCK) hist[q] = 0;
    }
    int64_t p0, p1, cap_end;
    frame_range(fr, f, p0, p1, cap_end);
    const int64_t base = p0 + (int64_t)j * IDX_CHUNK;
    if (j == fr.n_chunks - 1 && p1 > base + IDX_CHUNK && threadIdx.x == 0 && fr.err)
        atomicOr(fr.err, SHPL_EBIT_CAPACITY);  // frame larger than max_points_per_frame
    const Ctx ctx{p1 - p0, -1};
#pragma unroll
    for (int u = 0; u < IDX_BATCH; ++u) {
        const int64_t i = base + (int64_t)u * IDX_BLOCK + threadIdx.x;
        if (i < p1) st.load(i, in[u]);
    }
    int32_t n[3] = {0, 0, 0};
    if constexpr (BKT) __syncthreads();  // hist cleared
#pragma unroll
    for (int u = 0; u < IDX_BATCH; ++u) {
        const int64_t i = base + (int64_t)u * IDX_BLOCK + threadIdx.x;
        typename Stage::Payload &pl = pl_out[u];
        const uint32_t m = i < p1 ? st.eval(ctx, f, i, in[u], pl) : 0u;
        m_out[u] = m;
#pragma unroll
        for (int k = 0; k < 3; ++k) n[k] += (m >> k) & 1u;
        if constexpr (BKT) {
            int32_t kc, kp;
            if ((m & KEEP_MULTI) && st.bucket_keys(pl, kc, kp)) {
                atomicAdd(&hist[kc / BK_KEYS], 1);
                atomicAdd(&hist[BK_MAX_RANGES + kp / BK_KEYS], 1);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        n[k] = wave_sum(n[k]);
        if ((threadIdx.x & 63) == 0) wsum[k][threadIdx.x >> 6] = n[k];
    }
    __syncthreads();
    // the chunk's counts and histograms: write-through stores (sc1), which k_index1's frame barrier hands to
    // the frame's other chunks with no release fence (the guide's in-launch counter form)
    if (threadIdx.x < 3) {
        int32_t t = 0;
        for (int w = 0; w < IDX_BLOCK / 64; ++w) t += wsum[threadIdx.x][w];
        store_agent(fr.chunk_kept + ((int64_t)threadIdx.x * fr.n_frames + f) * fr.n_chunks + j, t);
    }
    if constexpr (BKT) {
        for (int i = threadIdx.x; i < 2 * bk.nrmax; i += IDX_BLOCK) {
            const int K = i / bk.nrmax, q = i - K * bk.nrmax;
            store_agent(bk.hist + (((int64_t)K * fr.n_frames + f) * fr.n_chunks + j) * bk.nrmax + q,
                        q < bk.nr[K] ? hist[K * BK_MAX_RANGES + q] : 0);
        }
    }
}

// Pass 1 (grid n_chunks x n_frames).
template <typename Stage, bool BKT = false>
__global__ __launch_bounds__(IDX_BLOCK) void k_count(Stage st, Frames fr, Bkt bk) {
    // rider workgroups: the launch's blocks past n_chunks in x (before the chunks measured slower)
    const int f = blockIdx.y, j = (int)blockIdx.x;
    if constexpr (BKT) {
        if (j >= fr.n_chunks) {  // a rider workgroup (uniform)
            const int rj = j - fr.n_chunks;
            for (int c = 0; c < 2; ++c)
                if (bk.cp_at[c] == 0) pass_copy(bk.cp[c], f, rj, bk.cp_blocks);
            return;
        }
    }
    typename Stage::In in[IDX_BATCH];
    uint32_t m[IDX_BATCH];
    typename Stage::Payload pl[IDX_BATCH];
    count_phase<Stage, BKT>(st, fr, bk, f, j, in, m, pl);
}

// k_compact's bucket placement (BKT), all threads: b_tot / b_bef = thread
// (key bK, range bq)'s entries in the frame / in its earlier chunks; pos = this
// point's entry slot in the frame when `keep`.
template <typename Stage>
__device__ __forceinline__ void bucket_place(const Stage &st, const Frames &fr, const Bkt &bk, int f, int j,
                                             int64_t p0, int64_t cap, int64_t total, bool keep,
                                             const typename Stage::Payload &pl, int64_t pos, int32_t b_tot,
                                             int32_t b_bef, int32_t *s_off, int32_t *s_scan,
                                             int16_t (*s_w)[IDX_BLOCK / 64][BK_MAX_RANGES],
                                             uint64_t (*s_peer)[BK_MAX_RANGES]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int bK = threadIdx.x / BK_MAX_RANGES, bq = threadIdx.x % BK_MAX_RANGES;
    // 1. each range's start in the frame: exclusive scan of the totals, per key
    const int32_t x = wave_incl_scan(b_tot);  // over the wave's 64 (key, range) lanes
    if (lane == 63) s_scan[wid] = x;
    lds_barrier();
    int32_t start = x - b_tot;
    const int w0 = bK * (BK_MAX_RANGES / 64);  // the key's first wave
    for (int w = w0; w < wid; ++w) start += s_scan[w];
    if (bq < bk.nr[bK]) {
        s_off[threadIdx.x] = start + b_bef;
        if (j == 0 && total >= 2) {
            int32_t *x2 = bk.ext + (((int64_t)bK * fr.n_frames + f) * bk.nrmax + bq) * 2;
            x2[0] = start;
            x2[1] = b_tot;
        }
    }
    // 2. stable multisplit of the chunk's entries by range, per key: each lane ORs its bit into its wave's word
    // of its range (s_peer, zero between uses), reads the word back -- the wave's lanes of the same range, its
    // rank among them = the lanes below it -- and the lanes zero it again. One wave's LDS operations run in
    // order, so the reads follow every OR of the wave and the zeroing every read. (Measured: a multisplit of
    // ballots over the range bits spent ~2.4 us of VALU here at config 3.)
    int32_t kk[2] = {0, 0};
    const bool ok = total >= 2 && keep && pos >= 0 && st.bucket_keys(pl, kk[0], kk[1]);
    int32_t rank[2];
#pragma unroll
    for (int K = 0; K < 2; ++K) {
        const int r = ok ? kk[K] / BK_KEYS : 0;
        uint64_t peers = 0;
        if (ok) atomicOr(reinterpret_cast<unsigned long long *>(&s_peer[wid][r]), 1ull << lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ok) peers = s_peer[wid][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ok) s_peer[wid][r] = 0;
        rank[K] = (int32_t)lane_rank(peers);
        if (ok && rank[K] == 0) s_w[K][wid][r] = (int16_t)__popcll(peers);
    }
    lds_barrier();
    SHPL_IDX1_STAMP(5);
    if (bq < bk.nr[bK]) {  // waves' exclusive prefix per (key, range)
        int32_t run = 0;
#pragma unroll
        for (int w = 0; w < IDX_BLOCK / 64; ++w) {
            const int32_t v = s_w[bK][w][bq];
            s_w[bK][w][bq] = (int16_t)run;
            run += v;
        }
    }
    lds_barrier();
    SHPL_IDX1_STAMP(6);
    if (!ok) return;
#pragma unroll
    for (int K = 0; K < 2; ++K) {
        const int r = kk[K] / BK_KEYS;
        const int64_t at = (int64_t)s_off[K * BK_MAX_RANGES + r] + s_w[K][wid][r] + rank[K];  // in the frame
        if (at < 0 || at >= cap) {  // half-written aggregates (a failed barrier): no stray write
            if (fr.err) atomicOr(fr.err, SHPL_EBIT_BARRIER);
            continue;
        }
        const int64_t slot = (int64_t)K * bk.nnz_cap + p0 + at;
        bk.words[slot] = ((uint32_t)(kk[K] % BK_KEYS) << 24) | (uint32_t)pos;
    }
}

// Pass 2 (same grid): the chunk's kept points land after those of the
// frame's earlier chunks, in point order (a stable compaction); rows of the
// chunk are ranked in order by wave ballots + an LDS prefix. Each chunk also
// writes the sentinels of the unused capacity that falls in its stretch of
// slots, and the frame's last chunk the frame's entry count.
// Pass 2 of chunk j of frame f (`loaded`: its points already in `in`, and pass 1's flags and payloads in
// flags1 / pay1, from count_phase in the same launch: they are pass 2's own unless the frame has exactly one AUX point --
// the stage's second product in the other order -- so only then is a point evaluated again).
template <typename Stage, bool BKT>
__device__ __forceinline__ void compact_phase(const Stage &st, const Frames &fr, const Bkt &bk, int f, int j,
                                              typename Stage::In (&in)[IDX_BATCH], bool loaded,
                                              const uint32_t (&flags1)[IDX_BATCH],
                                              const typename Stage::Payload (&pay1)[IDX_BATCH]) {
    static_assert(!BKT || IDX_BATCH == 1, "bucket placement ranks one point per thread");
    __shared__ int32_t wsum[IDX_BATCH][IDX_BLOCK / 64];
    __shared__ int32_t pre[2][IDX_BLOCK / 64], all[2][IDX_BLOCK / 64], naux[IDX_BLOCK / 64];
    __shared__ int32_t s_off[BKT ? 2 * BK_MAX_RANGES : 1], s_scan[IDX_BLOCK / 64];
    // per-wave range counts, then their prefixes over the waves (at most IDX_BLOCK: 16 bits). LDS of the
    // bucketed form, with s_peer's 64 KiB: ~113 KiB per 1024-thread workgroup, one workgroup per CU (two would
    // also need <= 64 VGPRs: amdgpu_waves_per_eu(8) measured 41 vs 17 us for k_index1, docs/HISTORY.md §4)
    __shared__ int16_t s_w[BKT ? 2 : 1][IDX_BLOCK / 64][BKT ? BK_MAX_RANGES : 1];
    __shared__ int32_t s_tb[BKT ? 4 * BK_MAX_RANGES : 1];  // per (key, range): entries in the frame, in earlier chunks
    __shared__ uint64_t s_peer[BKT ? IDX_BLOCK / 64 : 1][BKT ? BK_MAX_RANGES : 1];  // per wave and range: lane bits
    int64_t p0, p1, cap_end;
    frame_range(fr, f, p0, p1, cap_end);
    const int wid = threadIdx.x >> 6;
    // buckets: each (key, range) thread's entries in all of the frame's chunks and in the earlier ones
    // (loads issued first, beside the point loads)
    if constexpr (BKT) {
        // (key K, range q) pairs x S slices of the chunks: S adjacent lanes per pair (S a power of two, at
        // most 64, S x pairs <= the block), each summing every S-th chunk -- all its loads in flight --
        // then a shuffle reduction; s_tb[K][q] / s_tb[2][K][q] = the pair's entries in all / earlier chunks
        static_assert(IDX_BLOCK == 2 * BK_MAX_RANGES, "one thread per (key, range)");
        const int P = 2 * bk.nrmax;
        int S = 1;
        while (S < 64 && 2 * S * P <= IDX_BLOCK) S <<= 1;
        const int pair = threadIdx.x / S, sl = threadIdx.x & (S - 1);
        const int K = pair / bk.nrmax, q = pair - K * bk.nrmax;
        int32_t tot = 0, bef = 0;
        if (pair < P && q < bk.nr[K]) {
            const int32_t *h = bk.hist + ((int64_t)K * fr.n_frames + f) * fr.n_chunks * bk.nrmax + q;
            for (int j0 = sl; j0 < fr.n_chunks; j0 += 8 * S) {  // 8 loads in flight
                int32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    v[u] = j0 + u * S < fr.n_chunks ? load_agent(h + (int64_t)(j0 + u * S) * bk.nrmax) : 0;
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    tot += v[u];
                    bef += j0 + u * S < j ? v[u] : 0;
                }
            }
        }
        for (int o = 1; o < S; o <<= 1) {  // S lanes of one wave (S <= 64, aligned)
            tot += __shfl_xor(tot, o, 64);
            bef += __shfl_xor(bef, o, 64);
        }
        if (pair < P && sl == 0) {
            s_tb[K * BK_MAX_RANGES + q] = tot;
            s_tb[2 * BK_MAX_RANGES + K * BK_MAX_RANGES + q] = bef;
        }
        for (int i = threadIdx.x; i < 2 * (IDX_BLOCK / 64) * bk.nrmax; i += IDX_BLOCK) {  // the ranges in use
            const int kw = i / bk.nrmax;
            s_w[kw / (IDX_BLOCK / 64)][kw % (IDX_BLOCK / 64)][i - kw * bk.nrmax] = 0;
        }
        for (int i = threadIdx.x; i < (IDX_BLOCK / 64) * bk.nrmax; i += IDX_BLOCK)
            s_peer[i / bk.nrmax][i % bk.nrmax] = 0;
    }
    // the frame's AUX count picks the KEEP count (and the stage's product order): the AUX counts and both
    // KEEP counts of every chunk in one round trip, then the frame's and the earlier chunks' sums of each
    const int32_t *aux_c = fr.chunk_kept + ((int64_t)2 * fr.n_frames + f) * fr.n_chunks;
    const int32_t *k0_c = fr.chunk_kept + (int64_t)f * fr.n_chunks;
    const int32_t *k1_c = fr.chunk_kept + ((int64_t)fr.n_frames + f) * fr.n_chunks;
    int32_t na = 0, m0 = 0, e0 = 0, m1 = 0, e1 = 0;
    for (int q = threadIdx.x; q < fr.n_chunks; q += IDX_BLOCK) {
        const int32_t a = load_agent(aux_c + q), c0 = load_agent(k0_c + q), c1 = load_agent(k1_c + q);
        na += a;
        m0 += q < j ? c0 : 0;
        e0 += c0;
        m1 += q < j ? c1 : 0;
        e1 += c1;
    }
    na = wave_sum(na);
    m0 = wave_sum(m0);
    e0 = wave_sum(e0);
    m1 = wave_sum(m1);
    e1 = wave_sum(e1);
    if ((threadIdx.x & 63) == 0) {
        naux[wid] = na;
        pre[0][wid] = m0;
        all[0][wid] = e0;
        pre[1][wid] = m1;
        all[1][wid] = e1;
    }
    __syncthreads();
    int64_t n_aux = 0;
    for (int w = 0; w < IDX_BLOCK / 64; ++w) n_aux += naux[w];
    SHPL_IDX1_STAMP(3);
    const Ctx ctx{p1 - p0, n_aux};
    const int variant = n_aux == 1 ? 1 : 0;
    const uint32_t keep_bit = variant ? KEEP_ONE : KEEP_MULTI;
    const int64_t base = p0 + (int64_t)j * IDX_CHUNK;
    typename Stage::Payload pl[IDX_BATCH];
    bool keep[IDX_BATCH];
    if (!loaded) {
#pragma unroll
        for (int u = 0; u < IDX_BATCH; ++u) {
            const int64_t i = base + (int64_t)u * IDX_BLOCK + threadIdx.x;
            if (i < p1) st.load(i, in[u]);
        }
    }
    uint64_t m[IDX_BATCH];
    int64_t b_pos = 0;  // BKT: this point's entry slot in the frame
#pragma unroll
    for (int u = 0; u < IDX_BATCH; ++u) {
        const int64_t i = base + (int64_t)u * IDX_BLOCK + threadIdx.x;
        keep[u] = false;
        if (i < p1) {
            if (loaded && n_aux != 1) {
                keep[u] = (flags1[u] & keep_bit) != 0;
                pl[u] = pay1[u];
            } else {
                keep[u] = (st.eval(ctx, f, i, in[u], pl[u]) & keep_bit) != 0;
            }
            st.touch(f, i, pl[u], keep[u]);
        }
        m[u] = __ballot(keep[u]);
        if ((threadIdx.x & 63) == 0) wsum[u][wid] = (int32_t)__popcll(m[u]);
    }
    lds_barrier();
    int64_t kept = 0;
    for (int w = 0; w < IDX_BLOCK / 64; ++w) kept += pre[variant][w];
#pragma unroll
    for (int u = 0; u < IDX_BATCH; ++u) {
        int32_t before = 0, tot = 0;
        for (int w = 0; w < IDX_BLOCK / 64; ++w) {
            const int32_t c = wsum[u][w];
            before += w < wid ? c : 0;
            tot += c;
        }
        const int64_t i = base + (int64_t)u * IDX_BLOCK + threadIdx.x;
        const int64_t slot = kept + before + lane_rank(m[u]);  // (entries of the frame before this one)
        // every write the frame's aggregates address stays inside the frame's capacity: aggregates a failed
        // barrier left half-written (SHPL_EBIT_BARRIER is set then) can make a wrong map, never a stray write
        const bool in_cap = slot >= 0 && slot < cap_end - p0;
        if (keep[u] && !in_cap && fr.err) atomicOr(fr.err, SHPL_EBIT_BARRIER);
        if (keep[u] && in_cap) st.emit(f, i, p0 + slot, p0, pl[u]);
        if constexpr (BKT) b_pos = in_cap ? slot : -1;
        kept += tot;
    }
    // sentinels of the unused capacity [p0 + total, cap_end), each chunk its own stretch
    int64_t total = 0;
    for (int w = 0; w < IDX_BLOCK / 64; ++w) total += all[variant][w];
    SHPL_IDX1_STAMP(4);
    if constexpr (BKT) {  // (s_tb written before k_compact's first barrier; entries past nr[K] never)
        const bool live = (int)(threadIdx.x % BK_MAX_RANGES) < bk.nr[threadIdx.x / BK_MAX_RANGES];
        bucket_place(st, fr, bk, f, j, p0, cap_end - p0, total, keep[0], pl[0], b_pos,
                     live ? s_tb[threadIdx.x] : 0,
                     live ? s_tb[2 * BK_MAX_RANGES + threadIdx.x] : 0, s_off, s_scan, s_w, s_peer);
    }
    const int64_t h0 = p0 + total > base ? p0 + total : base;
    const int64_t h1 = j == fr.n_chunks - 1 ? cap_end : (base + IDX_CHUNK < cap_end ? base + IDX_CHUNK : cap_end);
    for (int64_t pos = h0 + threadIdx.x; pos < h1; pos += IDX_BLOCK) st.hole(pos);
    if (j == fr.n_chunks - 1 && threadIdx.x == 0) {
        if (fr.frame_nnz) fr.frame_nnz[f] = total;
        if (fr.frame_out_off) {
            fr.frame_out_off[f] = p0;
            if (f == fr.n_frames - 1) fr.frame_out_off[fr.n_frames] = cap_end;
        }
    }
}

// Pass 2 (same grid as pass 1).
template <typename Stage, bool BKT = false>
__global__ __launch_bounds__(IDX_BLOCK) void k_compact(Stage st, Frames fr, Bkt bk) {
    // rider workgroups: the launch's blocks past n_chunks in x (before the chunks measured slower)
    const int f = blockIdx.y, j = (int)blockIdx.x;
    if constexpr (BKT) {
        if (j >= fr.n_chunks) {  // a rider workgroup (uniform)
            const int rj = j - fr.n_chunks;
            for (int c = 0; c < 2; ++c)
                if (bk.cp_at[c] == 1) pass_copy(bk.cp[c], f, rj, bk.cp_blocks);
            return;
        }
    }
    typename Stage::In in[IDX_BATCH];
    uint32_t m[IDX_BATCH] = {};
    typename Stage::Payload pl[IDX_BATCH];
    compact_phase<Stage, BKT>(st, fr, bk, f, j, in, false, m, pl);
}

// Both passes of the bucketed index in ONE launch (k_index1, small batches): a 1-D grid, every frame's chunk
// workgroups first (f = b / n_chunks, j = b % n_chunks), then the rider workgroups of both copies. Between the
// passes each chunk waits at its frame's barrier -- pass 2 needs the frame's totals (its AUX count, every
// chunk's kept count and range histogram) -- published by the release / acquire hand-off of the guide's
// in-launch counter form: the chunk's write-through (sc1) stores, every wave's vmcnt(0), the block barrier and
// an agent-scope fetch_add on the frame's arrival word (no release fence); one lane polls it (relaxed, agent scope,
// bounded: SHPL_EBIT_BARRIER on give-up), and every load of the aggregates is an sc1 load (no acquire fence). The chunk's points stay
// in registers between the passes (no second load). Each chunk then adds to the frame's departure word, and
// the last to depart zeroes both words for the next call (the words start at zero: the caller's workspace is
// zeroed once; every call leaves them zero, a timed-out one included).
// Dirty words (a workspace never zeroed): the arrivals the chunks of a frame see are n_chunks consecutive
// values from the word's start value, so unless it started at zero some chunk sees one outside [0, n_chunks)
// -- that chunk raises SHPL_EBIT_BARRIER (so does one whose departure count is outside that range): the call
// reports the bad state instead of handing out half-aggregated buckets (shpl_bucket_workspace_reset clears it).
// Residency, independent of the order in which workgroups are dispatched: the host takes this form only when
// the launch's chunk workgroups all fit on the GPU at once (the kernel's occupancy x the CUs) and frames have
// at most IDX1_MAX_CHUNKS chunks. A chunk waits only for its own frame's chunks; riders never wait, so while
// a chunk of the launch is undispatched at most (chunks - 1) slots are held by waiting chunks and one is free
// for it. (A GPU shared with other processes can still starve a frame: then the give-up below.)
constexpr int IDX1_MAX_CHUNKS = 32;
constexpr uint64_t IDX1_SPIN_TICKS = 2000000;  // 20 ms of s_memrealtime (100 MHz): the barrier's give-up
#ifndef SHPL_IDX1_FAULT
#define SHPL_IDX1_FAULT 0  // test builds only (libshpl_fault.so): chunk 0 of frame 0 never arrives -> the give-up
#endif

__device__ __forceinline__ void frame_barrier(const Frames &fr, const Bkt &bk, int f, int j) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its write-through aggregate stores done
    __syncthreads();
    if (threadIdx.x == 0) {
        const bool skip = SHPL_IDX1_FAULT && f == 0 && j == 0;
        const int32_t a = skip ? 0 : __hip_atomic_fetch_add(bk.bar + f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool dirty = a < 0 || a >= fr.n_chunks;  // the word did not start the call at zero
        if (dirty && fr.err) atomicOr(fr.err, SHPL_EBIT_BARRIER);
        const uint64_t t0 = wall_clock64();
        while (!dirty && __hip_atomic_load(bk.bar + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < fr.n_chunks) {
            if (wall_clock64() - t0 > IDX1_SPIN_TICKS) {
                if (fr.err) atomicOr(fr.err, SHPL_EBIT_BARRIER);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();  // (every later load of the frame's aggregates is an sc1 load: no acquire fence)
}

#ifndef SHPL_IDX1_WPE
#define SHPL_IDX1_WPE 0  // waves per SIMD asked of the register allocator (8: two workgroups per CU); 0 = its own
#endif
template <typename Stage>
__global__ __launch_bounds__(IDX_BLOCK)
#if SHPL_IDX1_WPE
__attribute__((amdgpu_waves_per_eu(SHPL_IDX1_WPE, SHPL_IDX1_WPE)))
#endif
void k_index1(Stage st, Frames fr, Bkt bk) {
    const int64_t b = blockIdx.x, n_ch = (int64_t)fr.n_frames * fr.n_chunks;
    if (b >= n_ch) {  // a rider workgroup (uniform): copy c's workgroup r of frame f
        const int64_t rj = b - n_ch;
        const int per = bk.cp_blocks;
        const int f = (int)(rj / (2 * per)), c = (int)((rj / per) & 1), r = (int)(rj % per);
        if (bk.cp[c].row_bytes > 0) pass_copy(bk.cp[c], f, r, per);
        return;
    }
    const int f = (int)(b / fr.n_chunks), j = (int)(b - (int64_t)f * fr.n_chunks);
    SHPL_IDX1_STAMP(0);
    // the frame's projection matrix into LDS, its loads in flight beside the frame offsets' (count_phase's first
    // block barrier precedes every eval): read from global memory inside eval it was one more round trip
    __shared__ double s_P[12];
    if (threadIdx.x < 12) s_P[threadIdx.x] = st.P[12 * (int64_t)f + threadIdx.x];
    Stage sf = st;
    sf.P_frame = s_P;
    typename Stage::In in[IDX_BATCH];
    uint32_t m[IDX_BATCH];
    typename Stage::Payload pl[IDX_BATCH];
    count_phase<Stage, true>(sf, fr, bk, f, j, in, m, pl);
    SHPL_IDX1_STAMP(1);
    frame_barrier(fr, bk, f, j);
    SHPL_IDX1_STAMP(2);
    compact_phase<Stage, true>(sf, fr, bk, f, j, in, true, m, pl);
    lds_barrier();  // every wave is past its reads of the frame's aggregates
    SHPL_IDX1_STAMP(7);
    if (threadIdx.x == 0) {
        const int32_t d = __hip_atomic_fetch_add(bk.bar + fr.n_frames + f, 1, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        if ((d < 0 || d >= fr.n_chunks) && fr.err) atomicOr(fr.err, SHPL_EBIT_BARRIER);  // dirty departure word
        if (d == fr.n_chunks - 1) {  // the last to leave: every chunk of the frame is past its poll
            __hip_atomic_store(bk.bar + f, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bk.bar + fr.n_frames + f, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// k_index1 workgroups the current device holds at once: the kernel's occupancy (its LDS and registers: one per
// CU) x the CUs. 0 when the runtime cannot say (the two-launch form then runs).
template <typename Stage>
int64_t index1_resident() {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_index1<Stage>, IDX_BLOCK, 0) != hipSuccess) {
        (void)hipGetLastError();  // not the caller's launch error
        return 0;
    }
    return (int64_t)cus * per_cu;
}

int n_chunks_for(int64_t max_points) {
    const int64_t c = (max_points + IDX_CHUNK - 1) / IDX_CHUNK;
    return (int)(c < 1 ? 1 : c);
}

constexpr size_t IDX_WS_HEAD = 256;  // single-frame [0, n] offsets

size_t index_ws_bytes(int n_frames, int64_t max_points) {
    return IDX_WS_HEAD + align_up(3 * sizeof(int32_t) * (size_t)n_frames * (size_t)n_chunks_for(max_points), 256);
}

template <typename Stage>
int run_compaction(const Stage &st, int n_frames, int64_t max_points, const int64_t *pt_off,
                   const int64_t *pt_count, int64_t *frame_nnz, int64_t *frame_out_off, uint32_t *err, void *ws,
                   size_t ws_bytes, hipStream_t stream, const Bkt *bk = nullptr) {
    if (ws_bytes < index_ws_bytes(n_frames, max_points)) return SHPL_ERR_WORKSPACE;
    Frames fr{pt_off, pt_count, n_frames, n_chunks_for(max_points),
              (int32_t *)((char *)ws + IDX_WS_HEAD), frame_nnz, frame_out_off, err};
    const dim3 grid(fr.n_chunks, n_frames);
    if constexpr (Stage::HAS_BUCKETS) {
        if (bk) {
#ifndef SHPL_INDEX1
#define SHPL_INDEX1 1
#endif
#ifndef SHPL_IDX1_RIDERS
#define SHPL_IDX1_RIDERS 240
#endif
            // (an error word is needed to report a failed barrier: without one, the two launches)
            if (SHPL_INDEX1 && bk->bar && err && fr.n_chunks <= IDX1_MAX_CHUNKS &&
                (int64_t)n_frames * fr.n_chunks <= index1_resident<Stage>()) {
                // rider workgroups per copy and frame: SHPL_IDX1_RIDERS per copy over the batch, at most one per
                // 64 KiB of a frame's copy (the two-launch form's cp_blocks bound)
                int per = SHPL_IDX1_RIDERS / n_frames;
                if (per > bk->cp_blocks) per = bk->cp_blocks;
                if (per < 1) per = 1;
                Bkt b1 = *bk;
                b1.cp_blocks = per;
                const bool any = bk->cp[0].row_bytes > 0 || bk->cp[1].row_bytes > 0;
                const int64_t blocks = (int64_t)n_frames * fr.n_chunks + (any ? (int64_t)n_frames * 2 * per : 0);
                hipLaunchKernelGGL((k_index1<Stage>), dim3((unsigned)blocks), dim3(IDX_BLOCK), 0, stream, st, fr, b1);
                SHPL_LAUNCH_CHECK();
                return SHPL_OK;
            }
            bool rides[2] = {false, false};
            for (int c = 0; c < 2; ++c)
                if (bk->cp[c].row_bytes > 0) rides[bk->cp_at[c]] = true;
            const dim3 grid0(fr.n_chunks + (rides[0] ? bk->cp_blocks : 0), n_frames);
            const dim3 grid1(fr.n_chunks + (rides[1] ? bk->cp_blocks : 0), n_frames);
            hipLaunchKernelGGL((k_count<Stage, true>), grid0, dim3(IDX_BLOCK), 0, stream, st, fr, *bk);
            SHPL_LAUNCH_CHECK();
            hipLaunchKernelGGL((k_compact<Stage, true>), grid1, dim3(IDX_BLOCK), 0, stream, st, fr, *bk);
            SHPL_LAUNCH_CHECK();
            return SHPL_OK;
        }
    } else {
        if (bk) return SHPL_ERR_ARG;
    }
    hipLaunchKernelGGL((k_count<Stage, false>), grid, dim3(IDX_BLOCK), 0, stream, st, fr, Bkt{});
    SHPL_LAUNCH_CHECK();
    hipLaunchKernelGGL((k_compact<Stage, false>), grid, dim3(IDX_BLOCK), 0, stream, st, fr, Bkt{});
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

}  // namespace
}  // namespace shpl
