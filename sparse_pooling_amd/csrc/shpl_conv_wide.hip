// shpl_conv_wide.hip -- the bf16 3x3 conv for wide channel counts: RetinaNet's post-fusion conv,
// slim.conv2d(bev_fused, 256, [3, 3]) over 256 BEV + 256 pooled image channels with a bias and ReLU
// (avod/avod/core/models/retinanet_model.py:334-348), on v_mfma_f32_16x16x32_bf16.
//
// Implicit GEMM with the output channels as M and the pixels as N: D[co][px] = sum_k W[co][k] X[k][px],
// K = 9 taps x the input channels. A 16 x 16 output tile of one frame against all 256 output channels per
// 512-thread workgroup (one per CU: 148 KB of LDS), so each input row is staged once for every output
// channel and the weights once per 256 pixels. Wave w owns 64 output channels (w >> 1) x 8 tile rows
// (w & 1): 4 x 8 accumulator tiles of 16 x 16 (128 registers; two waves per SIMD within 256 registers each),
// fed per 32-channel K step by 4 weight and 8 pixel fragments (one ds_read_b128 each) for 32 MFMAs.
//
// The K loop walks chunks of 64 input channels (A's, then B's) and, per chunk, the 9 taps. A chunk's 18 x 18
// halo (128 B per pixel) and a tap's 256 x 64 weights (32 KB) are staged by LDS-DMA into double buffers:
// step s (chunk q, tap t) multiplies from its buffers while the waves issue step s + 1's weight DMAs and, spread
// over chunk q's 9 taps, chunk q + 1's halo DMAs; one vmcnt(0) + barrier per step. LDS rows are 128 B (8 pieces
// of 16 B) with piece c of row r stored at c ^ (r & 7) -- r the halo column or the output channel -- so every
// fragment read (16 lanes on 16 consecutive rows, 4 K pieces) is conflict-free; the DMA sources carry the
// swizzle (the destination of an LDS-DMA is lane-linear), and the packed weights come pre-swizzled.
//
// Epilogue: act(round(fma(acc, scale, shift - center * scale))) -- shpl.h's contract, the tiled and row
// kernels' arithmetic -- transposed through LDS and stored as whole 512-byte pixel rows.
#include "shpl_conv_wide.h"

namespace shpl {
namespace wide {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int TH = 16, TW = 16;                        // output tile
constexpr int HH = TH + 2, HW = TW + 2, HPIX = HH * HW;  // 18 x 18 halo
#ifndef SHPL_WIDE_WAVES
// 4: one wave per SIMD, 128 channels x 128 pixels each (256 accumulator registers, in AGPRs by inline-asm
// MFMAs); 8: two per SIMD, 64 x 128 each (128 registers)
#define SHPL_WIDE_WAVES 4
#endif
constexpr int WAVES = SHPL_WIDE_WAVES, BLOCK = 64 * WAVES;
constexpr int MI = NT / (WAVES / 2) / 16;              // 16-channel tiles per wave (8 / 4)
constexpr int HALO_DMAS = (HPIX * 8 + 63) / 64;        // 41 DMAs of 1 KB (the last one part padding)
constexpr int HALO_BYTES = HALO_DMAS * 1024;
constexpr int W_DMAS = NT * 8 / 64;                    // 32
constexpr int W_BYTES = NT * KC * 2;                   // 32 KB per (chunk, tap)
constexpr int LDS_BYTES = 2 * HALO_BYTES + 2 * W_BYTES;
constexpr int OPITCH = NT * 2 + 16;                    // epilogue transpose: 528 B per pixel
static_assert(TH * TW * OPITCH <= LDS_BYTES, "epilogue tile fits the staging buffers");
constexpr int HW_PER_WAVE = (HALO_DMAS + WAVES - 1) / WAVES;  // halo DMAs a wave issues per chunk (11 / 6)
constexpr int HS = (HW_PER_WAVE + 8) / 9;                       // halo DMA slots per step (2 / 1)
constexpr int WD_PER_WAVE = W_DMAS / WAVES;                     // weight DMAs a wave issues per step (8 / 4)
static_assert(WD_PER_WAVE <= MI && HS <= MI, "the DMAs of a step ride the MFMA groups");

#ifndef SHPL_WIDE_PROBE
// timing probes (wrong results): 1 no DMAs in the K loop, 2 no barrier in it, 3 no MFMAs
#define SHPL_WIDE_PROBE 0
#endif
#ifndef SHPL_WIDE_VMCNT
// 1: a step waits for its weight DMAs only (vmcnt(HS)); its halo DMAs may land during the next step, except at
// a chunk's last tap (vmcnt(0))
#define SHPL_WIDE_VMCNT 1
#endif

__device__ u32x4 g_wide_zero;  // the LDS-DMA source of pieces outside the map

// One LDS-DMA of 16 bytes per lane (lane k's piece lands at dst + 16 k), hidden from the compiler in inline
// asm: seeing an LDS write by DMA it would drain every outstanding DMA (vmcnt(0)) before the next ds_read --
// the prefetch of step s + 1 before step s's second K half. The kernel orders them itself: one vmcnt(0) +
// barrier per step, and no step reads a buffer its own DMAs fill. M0 holds the destination (one wait state
// before the DMA reads it).
__device__ __forceinline__ void dma(const void *src, uint8_t *dst) {
    const uint32_t lds = (uint32_t)(uintptr_t)dst;
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(lds) : "memory");
}

// acc += A B on v_mfma_f32_16x16x32_bf16. One wave per SIMD: in inline asm with the accumulator in AGPRs (the
// compiler otherwise keeps the 256 accumulators in VGPRs and spills the operands to AGPRs around every MFMA);
// volatile, so the MFMAs keep their order among the DMAs; the hazard before reading AGPRs back is the
// epilogue's (s_nops after the loop).
__device__ __forceinline__ void mfma(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
    if constexpr (WAVES == 4)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
    else
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}

__device__ __forceinline__ int64_t xcd_tile(int64_t bid, int64_t n) {
    const int64_t q = n >> 3, r = n & 7, xcd = bid & 7, i = bid >> 3;
    return xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
}

// Packed weights: HWIO [3][3][c_a+c_b][c_out] bf16 -> [nb][chunk][tap][co 256][64 channels], piece c of
// output channel co at (c ^ (co & 7)) -- the LDS image one (chunk, tap) step DMAs in as it lies.
__global__ __launch_bounds__(256) void k_pack_wide(const uint16_t *w, int c_in, int c_out, uint16_t *wp) {
    const int64_t n = (int64_t)9 * c_in * c_out;
    const int Q = c_in / KC;
    for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < n; o += (int64_t)gridDim.x * 256) {
        // o indexes the packed array: [nb][q][t][co][slot 8][8]
        const int e = (int)(o & 7);
        const int slot = (int)((o >> 3) & 7);
        const int64_t r = o >> 6;
        const int co = (int)(r % NT);
        const int64_t r2 = r / NT;
        const int t = (int)(r2 % 9);
        const int64_t r3 = r2 / 9;
        const int q = (int)(r3 % Q);
        const int nb = (int)(r3 / Q);
        const int c = slot ^ (co & 7);
        const int ci = q * KC + c * 8 + e;
        wp[o] = w[((int64_t)t * c_in + ci) * c_out + nb * NT + co];
    }
}

__global__ __launch_bounds__(BLOCK, WAVES == 4 ? 1 : 2) void k_conv_wide(const WideArgs p) {
    __shared__ __attribute__((aligned(1024))) uint8_t s_lds[LDS_BYTES];
    __shared__ __attribute__((aligned(16))) float s_par[2][NT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int nb = blockIdx.y;
    const int H = p.h, W = p.w;
    const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
    const int64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const int f = (int)(tile / ((int64_t)tiles_x * tiles_y));
    const int tr = (int)(tile - (int64_t)f * tiles_x * tiles_y);
    const int ty0 = (tr / tiles_x) * TH, tx0 = (tr % tiles_x) * TW;
    const int64_t frame_row0 = (int64_t)f * H * W;
    const int Q = (p.c_a + p.c_b) / KC, steps = 9 * Q;

    if (tid < NT) {  // epilogue coefficients: scale (1 when absent), shift - center * scale
        const int co = nb * NT + tid;
        const float sc = p.scale ? p.scale[co] : 1.0f;
        const float ce = p.center ? p.center[co] : 0.0f;
        const float sh = p.shift ? p.shift[co] : 0.0f;
        s_par[0][tid] = sc;
        s_par[1][tid] = __fsub_rn(sh, __fmul_rn(ce, sc));
    }

    uint8_t *const hbuf0 = s_lds, *const wbuf0 = s_lds + 2 * HALO_BYTES;
    const uint8_t *const wsrc = reinterpret_cast<const uint8_t *>(p.wp) + (size_t)nb * Q * 9 * W_BYTES;

    // halo DMA k (0 .. HALO_DMAS - 1) of chunk q: LDS slot k * 64 + lane = (halo pixel, physical piece).
    // Branch-free (selects): issued between MFMAs, a branch would split the accumulators' live range.
    auto issue_halo = [&](int q, int k) {
        const int slot = k * 64 + lane, hp = slot >> 3, phys = slot & 7;
        const int hy = hp / HW, hx = hp - hy * HW;
        const int y = ty0 + hy - 1, x = tx0 + hx - 1;
        const bool in = hp < HPIX && y >= 0 && y < H && x >= 0 && x < W;
        const int ch = q * KC + ((phys ^ (hx & 7)) << 3);
        const int64_t row = frame_row0 + (int64_t)(in ? y : 0) * W + (in ? x : 0);
        const bool from_a = ch < p.c_a;
        const uint16_t *base = from_a ? p.a : p.b;
        const int64_t off = from_a ? row * p.a_stride + ch : row * p.b_stride + (ch - p.c_a);
        const void *src = in ? static_cast<const void *>(base + off) : static_cast<const void *>(&g_wide_zero);
        dma(src, hbuf0 + (q & 1) * HALO_BYTES + k * 1024);
    };
    // weight DMA k (0 .. WD_PER_WAVE - 1) of this wave for step s
    auto issue_w = [&](int s, int k) {
        const int d = wave * WD_PER_WAVE + k;
        dma(wsrc + (size_t)s * W_BYTES + d * 1024 + lane * 16, wbuf0 + (s & 1) * W_BYTES + d * 1024);
    };

    // prologue: chunk 0's halo and step 0's weights
    for (int k = wave; k < HALO_DMAS; k += WAVES) issue_halo(0, k);
#pragma unroll
    for (int k = 0; k < WD_PER_WAVE; ++k) issue_w(0, k);

    f32x4 acc[MI][8];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    // fragment read offsets: weights -- output channel wn*16*MI + 16 i + (lane & 15), K piece 4 ks + lane / 16
    // (its row key: lane & 7); pixels -- tile row 8 wm + j, column lane & 15 (+ kx), the same K piece
    const int l16 = lane & 15, kp = lane >> 4;
    uint32_t a_off[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
        a_off[ks] = (uint32_t)((wn * 16 * MI + l16) * 128 + (((4 * ks + kp) ^ (lane & 7)) << 4));

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
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 av[MI], bv[8];
            const int bpiece = ((4 * ks + kp) ^ (hx & 7)) << 4;
#pragma unroll
            for (int i = 0; i < MI; ++i) av[i] = *reinterpret_cast<const bf16x8 *>(wb + a_off[ks] + i * 16 * 128);
#pragma unroll
            for (int j = 0; j < 8; ++j) bv[j] = *reinterpret_cast<const bf16x8 *>(bbase + j * HW * 128 + bpiece);
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                // the next step's DMAs among the MFMAs: weights in the first K step, the halo in the second
                if (ks == 0 && i < WD_PER_WAVE && SHPL_WIDE_PROBE != 1) issue_w(s_next, i);
                if (ks == 1 && i < HS) {
                    // this wave's halo DMA WAVES (t + 9 i) + wave (past the wave's list: its last one again)
                    int k = WAVES * (t + 9 * i) + wave;
                    k = k < HALO_DMAS ? k : WAVES * ((HALO_DMAS - 1 - wave) / WAVES) + wave;
                    if (SHPL_WIDE_PROBE != 1) issue_halo(q_next, k);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (SHPL_WIDE_PROBE == 3)
                        acc[i][j][0] += (float)av[i][0] * (float)bv[j][0];
                    else
                        mfma(acc[i][j], av[i], bv[j]);
                }
            }
        }
        if (SHPL_WIDE_VMCNT && t != 8)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HS) : "memory");  // the halo DMAs issued last may stay in flight
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (SHPL_WIDE_PROBE != 2) __syncthreads();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the last MFMAs' results before their AGPRs are read (the hazard the compiler cannot see in the asm)
    if constexpr (WAVES == 4) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    // epilogue: lane (px = tile row 8 wm + j, column l16; channels wn*64 + 16 i + 4 kp .. + 3) -> LDS
    // [pixel][256 channels] bf16, then whole pixel rows out
    uint8_t *const s_out = s_lds;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int co = wn * 16 * MI + 16 * i + 4 * kp;
        const f32x4 sc = *reinterpret_cast<const f32x4 *>(&s_par[0][co]);
        const f32x4 sh = *reinterpret_cast<const f32x4 *>(&s_par[1][co]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint16_t o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                uint16_t v = f32_to_bf16(__builtin_fmaf(acc[i][j][e], sc[e], sh[e]));
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

}  // namespace

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
