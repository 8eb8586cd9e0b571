// shpl_conv_wide.hip -- the bf16 3x3 conv for wide channel counts: RetinaNet's post-fusion conv,
// slim.conv2d(bev_fused, 256, [3, 3]) over 256 BEV + 256 pooled image channels with a bias and ReLU
// (avod/avod/core/models/retinanet_model.py:334-348), on v_mfma_f32_16x16x32_bf16.
//
// Implicit GEMM with the output channels as M and the pixels as N: D[co][px] = sum_k W[co][k] X[k][px],
// K = 9 taps x the input channels. A 16 x 16 output tile of one frame against all 256 output channels per
// 512-thread workgroup (one per CU), so each input row is staged once for every output channel and the
// weights once per 256 pixels. Wave w owns 64 output channels (w >> 1) x 8 tile rows (w & 1): 4 x 8 tiles of
// 16 x 16 (128 accumulator registers: two waves per SIMD within 256 registers each), fed per 32-channel K step
// by 4 weight and 8 pixel fragments for 32 MFMAs.
//
// The K loop walks chunks of 64 input channels (A's, then B's) and, per chunk, the 9 taps. A chunk's 18 x 18
// halo (128 B per pixel) is staged by LDS-DMA into a double buffer, chunk q + 1's DMAs spread over chunk q's
// taps. LDS rows are 128 B (8 pieces of 16 B) with piece c of row r at c ^ (r & 7) -- r the halo column or the
// output channel -- so every 16x16x32 fragment read (16 lanes on consecutive rows, 4 K pieces) is
// conflict-free; the DMA sources carry the swizzle (the destination of an LDS-DMA is lane-linear).
// A tap's 256 x 64 weights (32 KB, pre-swizzled by k_pack_wide) are staged per step by LDS-DMA into a second
// double buffer; one counted vmcnt + barrier per step. (Measured and dropped, profiles/r05_wide_ab.log: each
// wave's weight fragments loaded from L2 straight into registers one K step ahead, a barrier per chunk only;
// register staging of weights and halo; one wave per SIMD with AGPR accumulators; 32x32x16 MFMAs; nontemporal
// halo DMAs.)
//
// Epilogue: act(round(fma(acc, scale, shift - center * scale))) -- shpl.h's contract, the tiled and row
// kernels' arithmetic -- transposed through LDS and stored as whole 512-byte pixel rows.
#include "shpl_conv_wide.h"
#include "shpl_conv_rows.h"

namespace shpl {
namespace wide {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#ifndef SHPL_WIDE_PROBE
// timing probes (wrong results): 1 no staging in the K loop, 3 no MFMAs
#define SHPL_WIDE_PROBE 0
#endif

constexpr int TH = 16, TW = 16;                        // output tile
constexpr int HH = TH + 2, HW = TW + 2, HPIX = HH * HW;  // 18 x 18 halo
constexpr int WAVES = 8, BLOCK = 64 * WAVES;
constexpr int MI = 4, NJ = 8;                          // 16 x 16 tiles per wave: 64 channels x 128 pixels
constexpr int KS = KC / 32;                            // 32-channel K steps per chunk
constexpr int HALO_DMAS = (HPIX * 8 + 63) / 64;        // 41 DMAs of 1 KB (the last one part padding)
constexpr int HALO_BYTES = HALO_DMAS * 1024;
constexpr int W_DMAS = NT * 8 / 64;                    // 32
constexpr int W_BYTES = NT * KC * 2;                   // 32 KB per (chunk, tap)
constexpr int LDS_BYTES = 2 * HALO_BYTES + 2 * W_BYTES;
constexpr int OPITCH = NT * 2 + 16;                    // epilogue transpose: 528 B per pixel
constexpr int LDS_ALLOC = LDS_BYTES > TH * TW * OPITCH ? LDS_BYTES : TH * TW * OPITCH;
constexpr int HW_PER_WAVE = (HALO_DMAS + WAVES - 1) / WAVES;  // halo DMAs a wave issues per chunk (6)
constexpr int WD_PER_WAVE = W_DMAS / WAVES;                     // weight DMAs a wave issues per step (4)
static_assert(HW_PER_WAVE <= 9, "a chunk's halo DMAs spread one per tap step");

__device__ __forceinline__ constexpr int key(int r) { return r & 7; }

__device__ u32x4 g_wide_zero;  // the LDS-DMA source of pieces outside the map

// One LDS-DMA of 16 bytes per lane (lane k's piece lands at dst + 16 k), hidden from the compiler in inline
// asm: seeing an LDS write by DMA it would drain every outstanding DMA (vmcnt(0)) before the next ds_read.
// The kernel orders them itself (counted vmcnt + barriers; no step reads a buffer its own DMAs fill). M0 holds
// the destination (one wait state before the DMA reads it).
__device__ __forceinline__ void dma(const void *src, uint8_t *dst) {
    const uint32_t lds = (uint32_t)(uintptr_t)dst;
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(lds) : "memory");
}
__device__ __forceinline__ void dma_halo(const void *src, uint8_t *dst) { dma(src, dst); }

__device__ __forceinline__ int64_t xcd_tile(int64_t bid, int64_t n) {
    const int64_t q = n >> 3, r = n & 7, xcd = bid & 7, i = bid >> 3;
    return xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
}

// Packed weights, HWIO [3][3][c_a+c_b][c_out] bf16 -> [nb][chunk q][tap t][co 256][64 channels], piece c of
// output channel co at c ^ key(co): the LDS image a step DMAs in as it lies.
__global__ __launch_bounds__(256) void k_pack_wide(const uint16_t *w, int c_in, int c_out, uint16_t *wp) {
    const int64_t n = (int64_t)9 * c_in * c_out;
    const int Q = c_in / KC;
    for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < n; o += (int64_t)gridDim.x * 256) {
        const int e = (int)(o & 7);
        const int slot = (int)((o >> 3) & 7);
        const int64_t r = o >> 6;
        const int co = (int)(r % NT);
        const int64_t r2 = r / NT;
        const int t = (int)(r2 % 9);
        const int64_t r3 = r2 / 9;
        const int q = (int)(r3 % Q);
        const int nb = (int)(r3 / Q);
        const int ci = q * KC + (slot ^ key(co)) * 8 + e;
        wp[o] = w[((int64_t)t * c_in + ci) * c_out + nb * NT + co];
    }
}

__global__ __launch_bounds__(BLOCK, 2) void k_conv_wide(const WideArgs p) {
    __shared__ __attribute__((aligned(1024))) uint8_t s_lds[LDS_ALLOC];
    __shared__ __attribute__((aligned(16))) float s_par[2][NT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;  // tile rows 8 wm .. + 7, output channels 64 wn .. + 63
    const int nb = blockIdx.y;
    const int H = p.h, W = p.w;
    const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
    const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const int f = (int)(tile / ((int64_t)tiles_x * tiles_y));
    const int tr = (int)(tile - (int64_t)f * tiles_x * tiles_y);
    const int ty0 = (tr / tiles_x) * TH, tx0 = (tr % tiles_x) * TW;
    const int64_t frame_row0 = (int64_t)f * H * W;
    const int Q = (p.c_a + p.c_b) / KC, QA = p.c_a / KC, steps = 9 * Q;

    if (tid < NT) {  // epilogue coefficients: scale (1 when absent), shift - center * scale
        const int co = nb * NT + tid;
        const float sc = p.scale ? p.scale[co] : 1.0f;
        const float ce = p.center ? p.center[co] : 0.0f;
        const float sh = p.shift ? p.shift[co] : 0.0f;
        s_par[0][tid] = sc;
        s_par[1][tid] = __fsub_rn(sh, __fmul_rn(ce, sc));
    }

    uint8_t *const hbuf0 = s_lds;
    const uint8_t *const wsrc = reinterpret_cast<const uint8_t *>(p.wp) + (size_t)nb * Q * 9 * W_BYTES;

    // The wave's halo DMAs k = WAVES j + wave (j < HW_PER_WAVE): per lane, once per tile, its LDS slot's pixel
    // (as a byte offset in A's and in B's frame rows, with its logical piece folded in) or -1 outside the map.
    // A chunk's piece then only adds the chunk's channel offset to a wave-uniform base.
    const uint8_t *const fa = reinterpret_cast<const uint8_t *>(p.a + frame_row0 * p.a_stride);
    const uint8_t *const fb = p.cmp ? reinterpret_cast<const uint8_t *>(p.cmp)
                                    : p.c_b ? reinterpret_cast<const uint8_t *>(p.b + frame_row0 * p.b_stride) : fa;
    const int64_t cmp0 = p.cmp ? p.frame_off[f] : 0;
    int32_t hoff_a[HW_PER_WAVE], hoff_b[HW_PER_WAVE];
#pragma unroll
    for (int j = 0; j < HW_PER_WAVE; ++j) {
        const int k = WAVES * j + wave;
        const int slot = k * 64 + lane, hp = slot >> 3, phys = slot & 7;
        const int hy = hp / HW, hx = hp - hy * HW;
        const int y = ty0 + hy - 1, x = tx0 + hx - 1;
        const bool in = k < HALO_DMAS && hp < HPIX && y >= 0 && y < H && x >= 0 && x < W;
        const int pix = y * W + x, piece = (phys ^ key(hx)) << 4;
        hoff_a[j] = in ? (int32_t)(pix * (int32_t)p.a_stride * 2 + piece) : -1;
        if (p.cmp) {  // the pixel's compact pooled row, when a run lands on it
            int32_t off = -1;
            if (in) {
                const int64_t wi = ((int64_t)f * H + y) * p.wpr + (x >> 5);
                const uint32_t bits = p.occ[wi];
                if ((bits >> (x & 31)) & 1u)
                    off = (int32_t)((cmp0 + p.occ_base[wi] + __popc(bits & ((1u << (x & 31)) - 1u))) * p.c_b * 2 +
                                    piece);
            }
            hoff_b[j] = off;
        } else {
            hoff_b[j] = in ? (int32_t)(pix * (int32_t)p.b_stride * 2 + piece) : -1;
        }
    }
    // the global source of this lane's piece of the wave's halo DMA j of chunk q (the zero piece outside the map)
    auto halo_src = [&](int q, int j) -> const u32x4 * {
        const bool from_a = q < QA;
        int32_t off = -1;  // hoff_[j] by selects: a run-time index into a register array would go to scratch
#pragma unroll
        for (int jj = 0; jj < HW_PER_WAVE; ++jj)
            if (jj == j) off = from_a ? hoff_a[jj] : hoff_b[jj];
        const uint8_t *base = from_a ? fa + q * KC * 2 : fb + (q - QA) * KC * 2;
        return off >= 0 ? reinterpret_cast<const u32x4 *>(base + off) : &g_wide_zero;
    };

    // prologue: chunk 0's halo (and, LDS-DMA form, step 0's weights)
#pragma unroll
    for (int j = 0; j < HW_PER_WAVE; ++j)
        if (WAVES * j + wave < HALO_DMAS) dma_halo(halo_src(0, j), hbuf0 + (WAVES * j + wave) * 1024);

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    // fragment reads: B (pixels) -- tile row 8 wm + j, column lane & 15 (+ kx), K piece 4 ks + lane / 16
    const int l16 = lane & 15, kg = lane >> 4;

    uint8_t *const wbuf0 = s_lds + 2 * HALO_BYTES;
    auto issue_w = [&](int s, int k) {  // weight DMA k (0 .. WD_PER_WAVE - 1) of this wave for step s
        const int d = wave * WD_PER_WAVE + k;
        dma(wsrc + (size_t)s * W_BYTES + d * 1024 + lane * 16, wbuf0 + (s & 1) * W_BYTES + d * 1024);
    };
#pragma unroll
    for (int k = 0; k < WD_PER_WAVE; ++k) issue_w(0, k);
    // A fragment reads: output channel wn*64 + 16 i + (lane & 15), K piece 4 ks + lane / 16 (row key lane & 7)
    uint32_t a_off[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
        a_off[ks] = (uint32_t)((wn * 64 + l16) * 128 + (((4 * ks + kg) ^ (lane & 7)) << 4));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < steps; ++s) {
        const int q = s / 9, t = s - 9 * q, ky = t / 3, kx = t - 3 * ky;
        const uint8_t *hb = hbuf0 + (q & 1) * HALO_BYTES;
        const uint8_t *wb = wbuf0 + (s & 1) * W_BYTES;
        const int hx = kx + l16;
        const uint8_t *bbase = hb + ((wm * 8 + ky) * HW + hx) * 128;
        // the next step's DMAs, issued unconditionally (no branch among the MFMAs): past the last step they
        // repeat the last step's weights / chunk into the buffer nobody reads any more (drained below)
        const int s_next = s + 1 < steps ? s + 1 : s;
        const int q_next = q + 1 < Q ? q + 1 : q;
        int jh = t < HW_PER_WAVE ? t : HW_PER_WAVE - 1;  // this wave's halo DMA of the step
        if (WAVES * jh + wave >= HALO_DMAS) jh -= 1;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            bf16x8 av[MI], bv[NJ];
            const int bpiece = ((4 * ks + kg) ^ key(hx)) << 4;
#pragma unroll
            for (int i = 0; i < MI; ++i) av[i] = *reinterpret_cast<const bf16x8 *>(wb + a_off[ks] + i * 16 * 128);
#pragma unroll
            for (int j = 0; j < NJ; ++j) bv[j] = *reinterpret_cast<const bf16x8 *>(bbase + j * HW * 128 + bpiece);
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                // the next step's DMAs among the MFMA groups: the weights first, then the halo
                const int g = ks * MI + i;
                if (SHPL_WIDE_PROBE != 1) {
                    if (g < WD_PER_WAVE) issue_w(s_next, g);
                    if (g == WD_PER_WAVE)
                        dma_halo(halo_src(q_next, jh), hbuf0 + (q_next & 1) * HALO_BYTES + (WAVES * jh + wave) * 1024);
                }
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    if (SHPL_WIDE_PROBE == 3)
                        acc[i][j][0] += (float)av[i][0] * (float)bv[j][0];
                    else
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
                }
            }
        }
        // the step's weight DMAs have landed (the halo DMA issued last may stay in flight, but not past the
        // chunk's last tap), and every wave is done with the buffers the next step's DMAs overwrite
        if (t != 8)
            asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // epilogue: lane (pixel, 4 consecutive channels) -> LDS [pixel][256 channels] bf16, then whole pixel rows out
    uint8_t *const s_out = s_lds;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int co = wn * 64 + 16 * i + 4 * kg;
        const f32x4 sc = *reinterpret_cast<const f32x4 *>(&s_par[0][co]);
        const f32x4 sh = *reinterpret_cast<const f32x4 *>(&s_par[1][co]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            uint16_t o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint16_t v = f32_to_bf16(__builtin_fmaf(acc[i][j][e], sc[e], sh[e]));
                o[e] = (p.act == 1 && (int16_t)v <= 0) ? (uint16_t)0 : v;
            }
            u32x2 pk;
            __builtin_memcpy(&pk, o, 8);
            const int px = (wm * 8 + j) * TW + l16;
            *reinterpret_cast<u32x2 *>(s_out + px * OPITCH + co * 2) = pk;
        }
    }
    __syncthreads();
    const int piece = lane & 31;
#pragma unroll 4
    for (int k = 0; k < TH * TW / (2 * WAVES); ++k) {  // a wave stores two pixels per instruction
        const int px = wave * (TH * TW / WAVES) + 2 * k + (lane >> 5);
        const int y = ty0 + px / TW, x = tx0 + px % TW;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(s_out + px * OPITCH + piece * 16);
        if (y < H && x < W)
            __builtin_nontemporal_store(
                v, reinterpret_cast<u32x4 *>(p.out + (frame_row0 + (int64_t)y * W + x) * p.out_stride + nb * NT + piece * 8));
    }
}

// The pooled vector of every run of the cell-keyed CSR, piece g, into its compact row frame_off[f] + (run rank
// in frame f): one thread per (entry, 16-byte piece); the thread on a run's first entry sums the run in entry
// order with separate multiply and add from 0 and rounds once -- k_sparse's arithmetic, bit for bit.
__global__ __launch_bounds__(256) void k_pool_runs_wide(const int32_t *ent_dst, const int32_t *ent_src,
                                                        const float *ent_val, int64_t nnz_cap, const uint16_t *img,
                                                        int64_t img_stride, int64_t img_off, int c_b, int np, int H,
                                                        int W, int wpr, const uint32_t *occ, const int32_t *occ_base,
                                                        const int64_t *frame_off, uint16_t *cmp) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t e = t / np;
    const int g = (int)(t - e * np);
    if (e >= nnz_cap) return;
    const int32_t d = ent_dst[e];
    const int32_t prev = e > 0 ? ent_dst[e - 1] : -1;
    int32_t dn = e + 1 < nnz_cap ? ent_dst[e + 1] : -1;
    float wv = ent_val[e];
    int32_t src = ent_src[e];
    if (d < 0 || prev == d) return;
    const int64_t cells = (int64_t)H * W;
    const int f = (int)(d / cells);
    const int c = (int)(d - f * cells), y = c / W, x = c - y * W;
    const int64_t wi = ((int64_t)f * H + y) * wpr + (x >> 5);
    const int32_t rid = occ_base[wi] + __popc(occ[wi] & ((1u << (x & 31)) - 1u));
    float sum[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sum[j] = 0.0f;
    // entry i's row piece goes out with entry i+1's index words (one round trip per entry)
    for (int64_t i = e;; ++i) {
        const u32x4 raw = *reinterpret_cast<const u32x4 *>(img + (int64_t)src * img_stride + img_off + g * 8);
        const bool more = dn == d;
        float wn = 0.0f;
        int32_t sn = 0, dnn = -1;
        if (more) {
            wn = ent_val[i + 1];
            sn = ent_src[i + 1];
            dnn = i + 2 < nnz_cap ? ent_dst[i + 2] : -1;
        }
        uint16_t xv[8];
        __builtin_memcpy(xv, &raw, 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) sum[j] = __fadd_rn(sum[j], __fmul_rn(wv, bf16_to_f32(xv[j])));
        if (!more) break;
        wv = wn;
        src = sn;
        dn = dnn;
    }
    uint16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(sum[j]);
    *reinterpret_cast<u32x4 *>(cmp + (frame_off[f] + rid) * (int64_t)c_b + g * 8) = *reinterpret_cast<u32x4 *>(v);
}

// K consecutive entries per thread, one 8-channel piece g of each: their index words in one round trip and
// their K row pieces in flight together (the runs of a cell are mostly one entry long, so a thread per entry
// spent a round trip per index word and per row with little else in flight); each run head sums its run in
// entry order from 0 with separate multiply and add, as k_pool_runs_wide does -- bit for bit -- walking on past
// the group when the run does.
#ifndef SHPL_WIDE_RUNS_K
#define SHPL_WIDE_RUNS_K 4  // 1: k_pool_runs_wide (a thread per entry and piece)
#endif
template <int K>
__global__ __launch_bounds__(256) void k_pool_runs_wide_k(const int32_t *ent_dst, const int32_t *ent_src,
                                                          const float *ent_val, int64_t nnz_cap, const uint16_t *img,
                                                          int64_t img_stride, int64_t img_off, int c_b, int np, int H,
                                                          int W, int wpr, const uint32_t *occ,
                                                          const int32_t *occ_base, const int64_t *frame_off,
                                                          uint16_t *cmp) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t grp = t / np;
    const int g = (int)(t - grp * np);
    const int64_t e0 = grp * K;
    if (e0 >= nnz_cap) return;
    int32_t d[K + 1], src[K];
    float wv[K];
    const int32_t prev0 = e0 > 0 ? ent_dst[e0 - 1] : -1;
#pragma unroll
    for (int k = 0; k <= K; ++k) d[k] = e0 + k < nnz_cap ? ent_dst[e0 + k] : -1;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool in = e0 + k < nnz_cap;
        wv[k] = in ? ent_val[e0 + k] : 0.0f;
        src[k] = in ? ent_src[e0 + k] : 0;
    }
    u32x4 raw[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        raw[k] = d[k] >= 0 ? *reinterpret_cast<const u32x4 *>(img + (int64_t)src[k] * img_stride + img_off + g * 8)
                           : u32x4{0u, 0u, 0u, 0u};
    const int64_t cells = (int64_t)H * W;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (d[k] < 0 || d[k] == (k ? d[k - 1] : prev0)) continue;  // not a run head
        float sum[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sum[j] = 0.0f;
        bool tail = true;  // the run reaches past the group
#pragma unroll
        for (int m = k; m < K; ++m) {
            if (m > k && d[m] != d[k]) {
                tail = false;
                break;
            }
            uint16_t xv[8];
            __builtin_memcpy(xv, &raw[m], 16);
#pragma unroll
            for (int j = 0; j < 8; ++j) sum[j] = __fadd_rn(sum[j], __fmul_rn(wv[m], bf16_to_f32(xv[j])));
        }
        if (tail && d[K] == d[k]) {  // entries e0 + K, ... of the same cell, one round trip each
            int64_t i = e0 + K;
            float w = ent_val[i];
            int32_t sr = ent_src[i];
            int32_t dn = i + 1 < nnz_cap ? ent_dst[i + 1] : -1;
            for (;; ++i) {
                const u32x4 r = *reinterpret_cast<const u32x4 *>(img + (int64_t)sr * img_stride + img_off + g * 8);
                const bool more = dn == d[k];
                float wn = 0.0f;
                int32_t sn = 0, dnn = -1;
                if (more) {
                    wn = ent_val[i + 1];
                    sn = ent_src[i + 1];
                    dnn = i + 2 < nnz_cap ? ent_dst[i + 2] : -1;
                }
                uint16_t xv[8];
                __builtin_memcpy(xv, &r, 16);
#pragma unroll
                for (int j = 0; j < 8; ++j) sum[j] = __fadd_rn(sum[j], __fmul_rn(w, bf16_to_f32(xv[j])));
                if (!more) break;
                w = wn;
                sr = sn;
                dn = dnn;
            }
        }
        const int f = (int)(d[k] / cells);
        const int c = (int)(d[k] - f * cells), y = c / W, x = c - y * W;
        const int64_t wi = ((int64_t)f * H + y) * wpr + (x >> 5);
        const int32_t rid = occ_base[wi] + __popc(occ[wi] & ((1u << (x & 31)) - 1u));
        uint16_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(sum[j]);
        *reinterpret_cast<u32x4 *>(cmp + (frame_off[f] + rid) * (int64_t)c_b + g * 8) = *reinterpret_cast<u32x4 *>(v);
    }
}

}  // namespace

int prep(int n_frames, int h, int w, int wpr, const int32_t *ent_dst, const int32_t *ent_src, const float *ent_val,
         int64_t nnz_cap, const int64_t *frame_off, const uint16_t *img, int64_t img_stride, int64_t img_off, int c_b,
         uint32_t *occ, int32_t *occ_base, uint16_t *cmp, hipStream_t s) {
    // the occupancy words alone (no pooled channels: rows::prep_pooled's k_occ_frame)
    int rc = rows::prep_pooled(n_frames, h, w, wpr, ent_dst, ent_src, ent_val, nnz_cap, frame_off, img, img_stride,
                               img_off, 0, occ, occ_base, cmp, s);
    if (rc) return rc;
    const int np = c_b / 8;
    if (nnz_cap > 0 && np > 0 && SHPL_WIDE_RUNS_K > 1) {
        const int64_t threads = (nnz_cap + SHPL_WIDE_RUNS_K - 1) / SHPL_WIDE_RUNS_K * np;
        hipLaunchKernelGGL(k_pool_runs_wide_k<SHPL_WIDE_RUNS_K>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                           s, ent_dst, ent_src, ent_val, nnz_cap, img, img_stride, img_off, c_b, np, h, w, wpr, occ,
                           occ_base, frame_off, cmp);
        SHPL_LAUNCH_CHECK();
    } else if (nnz_cap > 0 && np > 0) {
        const int64_t threads = nnz_cap * np;
        hipLaunchKernelGGL(k_pool_runs_wide, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, ent_dst,
                           ent_src, ent_val, nnz_cap, img, img_stride, img_off, c_b, np, h, w, wpr, occ, occ_base,
                           frame_off, cmp);
        SHPL_LAUNCH_CHECK();
    }
    return SHPL_OK;
}

bool supported(int64_t c_a, int64_t c_b, int64_t c_out) {
    return c_a > 0 && c_a % KC == 0 && c_b >= 0 && c_b % KC == 0 && c_a + c_b > 64 && c_out > 0 && c_out % NT == 0;
}

size_t packed_bytes(int64_t c_a, int64_t c_b, int64_t c_out) { return (size_t)9 * (c_a + c_b) * c_out * 2; }

int launch(const WideArgs &a, const uint16_t *w_hwio, uint16_t *wp, hipStream_t s) {
    const int64_t n = (int64_t)9 * (a.c_a + a.c_b) * a.c_out;
    hipLaunchKernelGGL(k_pack_wide, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, w_hwio, a.c_a + a.c_b, a.c_out,
                       wp);
    SHPL_LAUNCH_CHECK();
    const int64_t tiles = (int64_t)a.n_frames * ((a.h + TH - 1) / TH) * ((a.w + TW - 1) / TW);
    if (tiles == 0) return SHPL_OK;
    if (tiles >= (1LL << 31)) return SHPL_ERR_BAD_SHAPE;
    WideArgs p = a;
    p.wp = wp;
    hipLaunchKernelGGL(k_conv_wide, dim3((unsigned)tiles, (unsigned)(a.c_out / NT)), dim3(BLOCK), 0, s, p);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

}  // namespace wide
}  // namespace shpl
