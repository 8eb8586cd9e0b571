// shpl_conv_rows.hip -- the row-streaming bf16 3x3 conv (k_conv_rows): the
// forward of shpl_conv3x3 (avod/avod/core/models/
// rpn_model.py:338-346) for bf16 inputs of at most 64 channels, where the
// tiled kernel of shpl_conv.hip is bound by its per-tile chain of staging
// round trips, not by MFMA or HBM.
//
// One wave per workgroup walks a band of output rows of one 32-column strip
// (and one block of 32 output channels). The chunk weights of all 9 taps sit
// in VGPRs for the whole band (9 Q bf16x8 A operands: 144 registers at Q =
// 4), so the LDS holds only pixels. Input row r of the halo contributes to
// output rows r+1, r, r-1 (ky = 0, 1, 2): three f32 accumulators roll over the
// band, and each input row is staged, read and multiplied once: 12
// ds_read_b128 per 36 MFMAs at Q = 4. Rows arrive by LDS-DMA into a per-wave
// ring of RING slots, RING-1 rows ahead of the MFMAs, behind counted
// `s_waitcnt vmcnt` -- no barrier anywhere (one wave). Two waves per SIMD (8
// per CU) each run their own ring.
//
// The loop is vector-issue-bound before it is MFMA-bound (an MFMA holds the
// SIMD's vector issue for 8 of its 32 cycles, a VALU op for 4, an LDS-DMA for
// ~60), so the staging does no per-row address arithmetic for dense sources:
// each row is one uniform buffer descriptor (its base pointer; num_records 0
// for rows outside the map) and every lane's 32-bit offset into it is fixed for
// the band; pieces outside the map or the channels carry an offset past
// num_records and read as zeros.
//
// Slot layout: A pieces (g = 2 chunk + half: channels 16 chunk + 8 half) as
// [g][34 pixels] of 16 bytes from slot 0, B pieces likewise from slot RB (the
// next multiple of 64 slots), so that every DMA (64 consecutive slots) reads
// one tensor. The lanes of a ds_read_b128 read 16 consecutive pixels of one
// piece (16 distinct bank quads), and every pixel-operand read of a row is one
// base register plus an immediate. After a row's MFMAs its slot holds the
// epilogue's transpose until the next DMA into it.
//
// Pooled B channels (CMP): the pooled vectors of the occupied cells, computed
// once by k_pool_runs with shpl_pull's arithmetic into a compact buffer (one
// row per run of the cell-keyed CSR), are gathered by the B DMAs: cell (y, x)
// holds run  occ_base[word] + popc(occ[word] below bit x%32)  of its frame
// (k_occ_frame), unoccupied cells read zeros. The conv of the fused form is
// bitwise the conv of [bev || shpl_pull(...)] through this same kernel.
#include "shpl_conv_rows.h"

namespace shpl {
namespace rows {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

#ifndef SHPL_ROWS_M16
// 1: even chunk counts multiply with v_mfma_f32_16x16x32_bf16 (K = 32 input channels, the block's 32 output
// channels as two halves of 16, the row's 32 pixels as two halves of 16) instead of 32x32x16 -- the same
// cycles per FLOP; under the chip's load-dependent clock the 16x16 shape has measured more FLOP/s
// (MI355X_MICROARCH.md, DVFS item 7)
#define SHPL_ROWS_M16 1
#endif
#ifndef SHPL_ROWS_M16_ST
#define SHPL_ROWS_M16_ST 1  // the statistics forms too (pooled: one operand read ahead of the MFMAs)
#endif
#ifndef SHPL_ROWS_STREG
// 1: the 16x16 statistics forms sum each row straight from the accumulators (a lane's two pixels, then one
// DPP exchange across lane ^ 8) into per-lane band sums in LDS, reduced over the pixel lanes once per band;
// 2: the same with the band sums in 8 registers (training forward 1,287-1,313 -> 1,271-1,278 us,
// profiles/r04_streg2_ab.log); 0: each row's f32 accumulators through a transpose in the ring slot (the
// 32x32 forms always do)
#define SHPL_ROWS_STREG 2
#endif
constexpr int NCO = 32;           // output channels per wave
constexpr int TW = 32;            // strip width (output pixels)
constexpr int HWD = TW + 2;       // halo row (pixels)
constexpr int W_ROWS = 9 * NCO;   // packed weight rows of a chunk
constexpr int RING = 3;           // ring slots per wave = the row loop's unroll (accumulator roles)
constexpr int REPI = NCO * 2 + 16;  // epilogue transpose pitch (bytes per pixel)
#ifndef SHPL_ROWS_XCD
#define SHPL_ROWS_XCD 1  // XCD-contiguous item order (0: blockIdx order)
#endif
#ifndef SHPL_ROWS_EPI8
#define SHPL_ROWS_EPI8 0  // 1: 8-byte stores straight from the accumulators (4 per lane and row), no LDS transpose: correct
                          // with RSTORES = 4, measured 1.2-1.6x slower (profiles/r04_epi_ab.log)
#endif
#ifndef SHPL_ROWS_DEAD3
#define SHPL_ROWS_DEAD3 0  // 1: masked input-gradient waves skip three dead rows' MFMAs (A/B: within noise, profiles/r06_ab/dead3_*)
#endif
#ifndef SHPL_ROWS_NTSTORE
#define SHPL_ROWS_NTSTORE 1  // the epilogue's stores nontemporal (0: plain stores, A/B)
#endif
#ifndef SHPL_ROWS_RSTORES
#define SHPL_ROWS_RSTORES (SHPL_ROWS_EPI8 ? 4 : 2)
#endif
constexpr int RSTORES = SHPL_ROWS_RSTORES;  // output stores per row step, always issued (the vmcnt arithmetic)
constexpr uint32_t OOB = 0x80000000u;  // an offset past every descriptor's num_records: reads zeros
#ifndef SHPL_ROWS_PROBE
// timing probes of k_conv_rows: 1 no epilogue, 2 no in-loop DMAs (wrong results); 3 s_memtime stamps of each
// row step's phases (ring wait, operand reads + MFMA issue, epilogue, staging) summed per wave into g_cprobe
// (shpl_probe_conv_phases reads them; the stamps' lgkmcnt(0) waits cost a few % of the loop)
#define SHPL_ROWS_PROBE 0
#endif
#if SHPL_ROWS_PROBE == 3
constexpr int CPROBE_WAVES = 1 << 17;
__device__ uint64_t g_cprobe[CPROBE_WAVES * 10];
#define SHPL_RSTAMP(t) asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory")
#define SHPL_STAMP(t)                                                                  \
    do {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                             \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");     \
        __builtin_amdgcn_sched_barrier(0);                                             \
    } while (0)
#endif
constexpr int SPF = NCO + 4;      // ST: f32 transpose pitch (floats per pixel; 16-byte rows, conflict-free b64 reads)
#ifndef SHPL_ROWS_WLATE
#define SHPL_ROWS_WLATE 0  // 1: no wait for the weights before the loop (the round-3 form, A/B)
#endif
#ifndef SHPL_ROWS_WPE
#define SHPL_ROWS_WPE 2  // waves per SIMD of the row kernels (tests/test_isa_guard.py forces 4: spills)
#endif

// The 16x16x32 shape: even chunk counts without statistics (the statistics forms keep 32x32x16: at 4 chunks
// pooled they would spill). Independent of the A / B split and of pooling, so that those forms stay bitwise
// equal to each other.
template <int Q, bool ST>
constexpr bool m16() { return SHPL_ROWS_M16 && Q % 2 == 0 && (SHPL_ROWS_M16_ST || !ST); }

// The statistics forms that sum from the accumulators (SHPL_ROWS_STREG): the 16x16 ones but the dense 1 + 3
// chunk form (its registers spill)
template <int Q, int QA, bool CMP, bool ST>
constexpr bool streg() { return SHPL_ROWS_STREG && ST && m16<Q, ST>() && !(Q == 4 && QA == 1 && !CMP); }

// v of lane i ^ 8 inside each row of 16 lanes (DPP row_ror:8, no LDS)
__device__ __forceinline__ float lane_xor8(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false));
}

// An f32x16 accumulator as four 16x16 tiles (16 output channels x 16 pixels each): tile 2h + nb.
__device__ __forceinline__ f32x4 tile4(const f32x16 &a, int t) {
    return f32x4{a[4 * t], a[4 * t + 1], a[4 * t + 2], a[4 * t + 3]};
}
__device__ __forceinline__ void set_tile4(f32x16 &a, int t, const f32x4 &v) {
    a[4 * t] = v[0];
    a[4 * t + 1] = v[1];
    a[4 * t + 2] = v[2];
    a[4 * t + 3] = v[3];
}

// The ring's counted wait: vmcnt(K) leaves the K most recent vector-memory operations -- the DMAs and
// stores of the RING-1 later steps -- in flight. expcnt(6) is a no-op in a compute kernel (no exports)
// that marks the wait as this one, so tests/test_isa_guard.py can find it in the disassembly and
// check that every path between two of them issues exactly K / (RING-1) vector-memory operations.
#ifndef SHPL_ROWS_DRAIN
#define SHPL_ROWS_DRAIN 0  // 1: every ring wait drains (vmcnt(0); probes of the epilogue variants only)
#endif
#if SHPL_ROWS_DRAIN
#define SHPL_RING_WAIT(K) asm volatile("s_waitcnt vmcnt(0) expcnt(6)" ::: "memory")
#else
#define SHPL_RING_WAIT(K) asm volatile("s_waitcnt vmcnt(%0) expcnt(6)" ::"n"(K) : "memory")
#endif

// Forms whose per-lane DMA offsets live in LDS instead of VGPRs (one ds_read_b32 each per row): pooled with
// statistics, and every 4-chunk form (they would otherwise spill to scratch, whose reloads inside the loop
// drain the ring).
template <int Q, int QA, bool CMP, bool ST>
constexpr bool offsets_in_lds() { return (CMP && ST) || (Q == 4 && (CMP || QA == 1)); }

template <int Q, int QA, bool ST = false>
struct Layout {
    static constexpr int QB = Q - QA;
    static constexpr int NA = (2 * QA * HWD + 63) / 64;  // A DMAs (the last one: TA lanes)
    static constexpr int TA = 2 * QA * HWD - 64 * (NA - 1);
    static constexpr int RB = 64 * NA;                   // first B slot
    static constexpr int NB = (2 * QB * HWD + 63) / 64;
    static constexpr int TB = QB ? 2 * QB * HWD - 64 * (NB - 1) : 0;
    static constexpr int NDMA = NA + NB;
    static constexpr int DATA = (QB ? RB + 2 * QB * HWD : 2 * QA * HWD) * 16;  // bytes of pieces
    static constexpr int SLOT0 = DATA > 32 * REPI ? DATA : 32 * REPI;  // also the epilogue's transpose
    static constexpr int SLOT = ST && SLOT0 < 32 * SPF * 4 ? 32 * SPF * 4 : SLOT0;  // ... and ST's f32 one
};

// Occupancy of the cell-keyed CSR per frame: bit x%32 of word (f, y, x/32) is
// set when cell (y, x) of frame f has entries; occ_base[word] counts the
// frame's occupied cells before the word (row-major). One 1024-thread
// workgroup per frame: run heads set bits of an LDS mask; each thread sums
// the popcounts of a contiguous run of words, one block scan, the prefixes
// written back to LDS beside the mask, then both copied out coalesced.
__global__ __launch_bounds__(1024) void k_occ_frame(const int32_t *ent_dst, const int64_t *frame_off, int H, int W,
                                                    int wpr, uint32_t *occ, int32_t *occ_base) {
    __shared__ uint32_t s_mask[OCC_MAX_WORDS];
    __shared__ int32_t s_base[OCC_MAX_WORDS];
    __shared__ int32_t s_tot[17];
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nw = H * wpr;
    for (int i = tid; i < nw; i += 1024) s_mask[i] = 0u;
    __syncthreads();
    const int64_t e0 = frame_off[f], e1 = frame_off[f + 1];
    const int64_t cell0 = (int64_t)f * H * W;
    for (int64_t e = e0 + tid; e < e1; e += 1024) {
        const int32_t d = ent_dst[e];
        if (d < 0) continue;
        if (e == e0 || ent_dst[e - 1] != d) {
            const int c = (int)(d - cell0), y = c / W, x = c - y * W;
            atomicOr(&s_mask[y * wpr + (x >> 5)], 1u << (x & 31));
        }
    }
    __syncthreads();
    const int per = (nw + 1023) / 1024, w0 = tid * per, w1 = min(w0 + per, nw);
    int32_t cnt = 0;
    for (int i = w0; i < w1; ++i) cnt += __popc(s_mask[i]);
    int32_t x = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_tot[wave] = x;
    __syncthreads();
    if (tid == 0) {
        int32_t sum = 0;
        for (int w = 0; w < 16; ++w) {
            const int32_t t = s_tot[w];
            s_tot[w] = sum;
            sum += t;
        }
    }
    __syncthreads();
    int32_t run = s_tot[wave] + x - cnt;
    for (int i = w0; i < w1; ++i) {
        s_base[i] = run;
        run += __popc(s_mask[i]);
    }
    __syncthreads();
    uint32_t *om = occ + (int64_t)f * nw;
    int32_t *ob = occ_base + (int64_t)f * nw;
    for (int i = tid; i < nw; i += 1024) {
        om[i] = s_mask[i];
        ob[i] = s_base[i];
    }
}

// The pooled vector of every run of the cell-keyed CSR into its compact row
// frame_off[f] + (run rank in frame f): one thread per entry; the thread on a
// run's first entry sums the run in entry order with separate multiply and add
// from 0 and rounds once per channel -- shpl_pull's (k_sparse's) arithmetic,
// bit for bit -- all NP 16-byte pieces of each entry's row in flight together.
template <int NP>
__global__ __launch_bounds__(SHPL_BLOCK) void k_pool_runs(const int32_t *ent_dst, const int32_t *ent_src,
                                                          const float *ent_val, int64_t nnz_cap, const uint16_t *img,
                                                          int64_t img_stride, int64_t img_off, int c_b, int H, int W,
                                                          int wpr, const uint32_t *occ, const int32_t *occ_base,
                                                          const int64_t *frame_off, uint16_t *cmp) {
    const int64_t e = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x;
    if (e >= nnz_cap) return;
    // the head test, the first entry's index words and the next entry's destination in one round trip
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
    float sum[NP][8];
#pragma unroll
    for (int g = 0; g < NP; ++g)
#pragma unroll
        for (int j = 0; j < 8; ++j) sum[g][j] = 0.0f;
    // entry i's row loads go out with entry i+1's index words (one round trip per entry, not two)
    for (int64_t i = e;; ++i) {
        const uint16_t *row = img + (int64_t)src * img_stride + img_off;
        u32x4 raw[NP];
#pragma unroll
        for (int g = 0; g < NP; ++g) raw[g] = *reinterpret_cast<const u32x4 *>(row + g * 8);
        const bool more = dn == d;  // entry i+1 is in the run (dn is -1 past the capacity)
        float wn = 0.0f;
        int32_t sn = 0, dnn = -1;
        if (more) {
            wn = ent_val[i + 1];
            sn = ent_src[i + 1];
            dnn = i + 2 < nnz_cap ? ent_dst[i + 2] : -1;
        }
#pragma unroll
        for (int g = 0; g < NP; ++g) {
            uint16_t xv[8];
            __builtin_memcpy(xv, &raw[g], 16);
#pragma unroll
            for (int j = 0; j < 8; ++j) sum[g][j] = __fadd_rn(sum[g][j], __fmul_rn(wv, bf16_to_f32(xv[j])));
        }
        if (!more) break;
        wv = wn;
        src = sn;
        dn = dnn;
    }
    uint16_t *o = cmp + (frame_off[f] + rid) * (int64_t)c_b;
#pragma unroll
    for (int g = 0; g < NP; ++g) {
        uint16_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(sum[g][j]);
        *reinterpret_cast<u32x4 *>(o + g * 8) = *reinterpret_cast<u32x4 *>(v);
    }
}

// A raw buffer descriptor (gfx9: dword 3 = 0x00020000) over `bytes` bytes from
// `base` (wave-uniform; readfirstlane pins it to SGPRs for the asm operand).
__device__ __forceinline__ i32x4 rsrc(const void *base, uint32_t bytes) {
    const uint64_t b = (uint64_t)base;
    return i32x4{__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)b),
                 __builtin_amdgcn_readfirstlane((int32_t)((b >> 32) & 0xffffu)),
                 __builtin_amdgcn_readfirstlane((int32_t)bytes), 0x00020000};
}

// One LDS-DMA of 16 bytes per lane from buffer offset voff (lane k's piece
// lands at wave_dst + 16 k), hidden from the compiler: the kernel waits for
// its ring slots itself (counted vmcnt), while the compiler, seeing an LDS
// write by DMA, would drain every outstanding DMA (vmcnt(0)) before each
// ds_read -- the whole prefetch ring. M0 holds the LDS destination (one wait
// state before the DMA reads it). Measured and not kept: the DMAs nontemporal (`offen nt lds`: the dense conv
// 1.40 -> 2.10 ms, its rows' re-reads by the halo and the other output block then miss L2;
// profiles/r04_ntl_ab.log), and a slot layout of 64-byte pixel quads so that each DMA lane quad reads one
// contiguous segment instead of 4 (dense conv 1.40 -> 1.34 ms, the pooled and training forms 1-2 % slower;
// profiles/r04_quad_ab.log).
__device__ __forceinline__ void dma16(i32x4 rs, uint32_t voff, const uint8_t *wave_dst) {
    const uint32_t lds = (uint32_t)(uintptr_t)wave_dst;
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "{m0}"(lds) : "memory");
}

// Per band, per lane: the byte offset of the lane's piece in each DMA's row
// (dense), or for pooled B pieces pixel << 16 | channel (-1: outside).
template <int Q, int QA, bool CMP>
__device__ __forceinline__ void lane_offsets(const RowArgs &r, int x0, int lane, uint32_t (&offa)[Layout<Q, QA>::NA],
                                             int32_t (&offb)[Layout<Q, QA>::NB > 0 ? Layout<Q, QA>::NB : 1]) {
    typedef Layout<Q, QA> L;
#pragma unroll
    for (int i = 0; i < L::NA; ++i) {
        const int sl = 64 * i + lane, g = sl / HWD, px = sl - g * HWD, x = x0 - 1 + px;
        const int ch = (g >> 1) * 16 + (g & 1) * 8;
        const bool ok = sl < 2 * QA * HWD && x >= 0 && x < r.w && ch < r.c_a;
        offa[i] = ok ? (uint32_t)((px * (int)r.a_stride + ch) * 2) : OOB;
    }
#pragma unroll
    for (int i = 0; i < L::NB; ++i) {
        const int sl = 64 * i + lane, g = sl / HWD, px = sl - g * HWD, x = x0 - 1 + px;
        const int ch = (g >> 1) * 16 + (g & 1) * 8;
        const bool ok = sl < 2 * L::QB * HWD && x >= 0 && x < r.w && ch < r.c_b;
        if constexpr (CMP)
            offb[i] = ok ? (px << 16) | ch : -1;
        else
            offb[i] = ok ? (int32_t)((px * (int)r.b_stride + ch) * 2) : (int32_t)OOB;
    }
}

// Stages input row y (its pixel 0 at global pixel pix0) into a ring slot:
// NDMA LDS-DMAs, always issued (the vmcnt arithmetic counts instructions).
template <int Q, int QA, bool CMP>
__device__ __forceinline__ void stage(const RowArgs &r, int64_t pix0, bool yok, uint64_t occ, int32_t first,
                                      const uint32_t (&offa)[Layout<Q, QA>::NA],
                                      const int32_t (&offb)[Layout<Q, QA>::NB > 0 ? Layout<Q, QA>::NB : 1],
                                      uint8_t *slot, int lane) {
    typedef Layout<Q, QA> L;
    const uint32_t nrec = yok ? OOB : 0u;
    const i32x4 ra = rsrc(r.a + pix0 * r.a_stride, nrec);
#pragma unroll
    for (int i = 0; i < L::NA; ++i)
        if (i < L::NA - 1 || lane < L::TA) dma16(ra, offa[i], slot + i * 1024);
    if constexpr (L::QB > 0) {
        const i32x4 rb = CMP ? rsrc(r.cmp, nrec) : rsrc(r.b + pix0 * r.b_stride, nrec);
#pragma unroll
        for (int i = 0; i < L::NB; ++i) {
            uint32_t o = (uint32_t)offb[i];
            if constexpr (CMP) {
                const int px = (offb[i] >> 16) & 63;
                const bool hit = offb[i] >= 0 && ((occ >> px) & 1);
                const int rank = first + (int)__popcll(occ & ((1ull << px) - 1));
                o = hit ? (uint32_t)((rank * r.c_b + (offb[i] & 0xffff)) * 2) : OOB;
            }
            if (i < L::NB - 1 || lane < L::TB) dma16(rb, o, slot + (L::RB + 64 * i) * 16);
        }
    }
}

// One staged input row j (j % RING == U: its slot and the accumulators'
// roles) of the band: wait for its slot, 3 kx x Q chunks x 3 ky MFMAs, the
// epilogue of output row j-2 of the band (always stored: rows and pixels
// outside the map go to the junk line; its accumulator is cleared), then
// stage input row j + RING into the slot just read.
// The forms whose out2 stores may be limited to occupied cells (RowArgs::occ2): the input gradient's (dense A,
// no ReLU, no statistics) of at most 32 gradient channels (the 4-chunk form has no register for the mask: it
// spills; it writes out2 whole)
template <int Q, bool CMP, bool RELU, bool ST>
constexpr bool occ2_form() { return Q <= 2 && !CMP && !RELU && !ST && !SHPL_ROWS_EPI8; }
static_assert(TW == 32, "occ2: one occupancy word per strip row");

template <int Q, int QA, bool CMP, bool RELU, bool ST, int U>
__device__ __forceinline__ void step(const RowArgs &r, const bf16x8 (&wr)[Q][9], f32x16 (&acc)[3],
                                     const float (*s_par)[NCO], const uint8_t *rd, uint8_t *s_ring,
                                     int64_t frame_row0, int x0, int ya, int n_in, int n_out, uint16_t *obase,
                                     int64_t ostr, f32x4 *s_st, int j,
                                     const uint64_t *s_occ, const int32_t *s_first, uint64_t b_rows,
                                     const uint32_t (&offa)[Layout<Q, QA>::NA],
                                     const int32_t (&offb)[Layout<Q, QA>::NB > 0 ? Layout<Q, QA>::NB : 1],
                                     const uint32_t *s_offs, const uint32_t (&rdq)[2], int lane,
                                     f32x4 (&str)[2], uint64_t (&ph)[5], uint32_t m2row, bool m2, uint64_t m2live) {
    typedef Layout<Q, QA, ST> L;
#if SHPL_ROWS_PROBE == 3
    uint64_t t0, t1, t2, t3, t4;
    SHPL_STAMP(t0);
#endif
    // rows j+1 .. j+RING-1 may still be in flight: per later step RSTORES stores and NDMA DMAs
    SHPL_RING_WAIT((L::NDMA + RSTORES) * (RING - 1));
#if SHPL_ROWS_PROBE == 3
    SHPL_STAMP(t1);
#endif
    f32x16 &a0 = acc[(U + 1) % 3], &a1 = acc[U], &a2 = acc[(U + 2) % 3];
    // m2: output rows j-2 .. j (the three accumulators' rows) all without an occupied cell -- none of them is
    // stored, so their MFMAs are skipped (a uniform branch: no memory operation inside)
    bool dead3 = false;
    if constexpr (occ2_form<Q, CMP, RELU, ST>()) dead3 = SHPL_ROWS_DEAD3 && m2 && (((m2live << 2) >> j) & 7ull) == 0;
    if (!dead3) {
    if constexpr (m16<Q, ST>()) {
        // K-chunk c (32 channels: pieces 4c .. 4c+3, each lane its piece 4c + lane / 16 from A or B), then kx,
        // then the pixel half nb; both output halves h per operand read. A split between A and B and the
        // skipped pooled chunks leave every accumulator's summation order unchanged, as below
#pragma unroll
        for (int c = 0; c < Q / 2; ++c) {
            // a chunk of B pieces only, in a pooled row without an occupied cell in the window: exact zeros
            if (CMP && 4 * c >= 2 * QA && !((b_rows >> j) & 1)) continue;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    const bf16x8 xv =
                        *reinterpret_cast<const bf16x8 *>(s_ring + rdq[c] + (U * L::SLOT + (16 * nb + kx) * 16));
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int t = 2 * h + nb;
                        set_tile4(a0, t, __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[2 * c + h][kx], xv, tile4(a0, t), 0, 0, 0));
                        set_tile4(a1, t,
                                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[2 * c + h][3 + kx], xv, tile4(a1, t), 0, 0, 0));
                        set_tile4(a2, t,
                                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[2 * c + h][6 + kx], xv, tile4(a2, t), 0, 0, 0));
                    }
                    // pooled statistics forms: at most one operand read ahead of the MFMAs (registers)
                    if constexpr (ST && CMP) asm volatile("" ::: "memory");
                }
        }
    } else {
    // chunk-major (q outer): a split of the channels between A and B, and the skipped pooled chunks below,
    // leave every accumulator's summation order unchanged
#pragma unroll
    for (int q = 0; q < QA; ++q) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const bf16x8 xv = *reinterpret_cast<const bf16x8 *>(rd + U * L::SLOT + kx * 16 + 2 * q * HWD * 16);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[q][kx], xv, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[q][3 + kx], xv, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[q][6 + kx], xv, a2, 0, 0, 0);
        }
    }
    // pooled rows without an occupied cell in the window are all zeros: their MFMAs would add exact zeros
    // to accumulators that are never -0, so skipping them is bitwise the same
    if (L::QB > 0 && (!CMP || ((b_rows >> j) & 1))) {
#pragma unroll
        for (int q = QA; q < Q; ++q) {
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const bf16x8 xv = *reinterpret_cast<const bf16x8 *>(rd + U * L::SLOT + kx * 16 +
                                                                    (L::RB + 2 * (q - QA) * HWD) * 16);
                a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[q][kx], xv, a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[q][3 + kx], xv, a1, 0, 0, 0);
                a2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wr[q][6 + kx], xv, a2, 0, 0, 0);
            }
        }
    }
    }
    }
#if SHPL_ROWS_PROBE == 3
    SHPL_STAMP(t2);
#endif
    // epilogue of band output row b: acc * scale + (shift - center * scale), ReLU on the bf16 pairs;
    // the lane's 4 runs of 4 channels to rows of the slot just read, then 2 x 16-byte stores per lane
    // (consecutive lanes, consecutive pieces)
    const int b = j - 2;
    uint8_t *s_o = s_ring + U * L::SLOT;
    if (SHPL_ROWS_PROBE == 1) {  // keep the accumulator alive, skip the epilogue
        if (a2[0] == 12345.0f) r.junk[lane] = 1;
    } else {
        const int pl = lane & 31, hf = lane >> 5;
        const bool row_ok = b >= 0 && b < n_out;
        uint16_t *orow = obase + (frame_row0 + (int64_t)(ya + b) * r.w + x0) * ostr;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the MFMAs' operand reads of the slot are done
#if SHPL_ROWS_EPI8
        // 8-byte stores straight from the accumulators: 4 per lane and row (RSTORES = 4 in the ring's counted
        // wait; with 2 the wait left two of the next row's DMAs unwaited-for -- the round-2 failure)
    #pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int cl = 8 * g + 4 * hf;
            uint32_t pk[2];
    #pragma unroll
            for (int k = 0; k < 4; k += 2) {
                const float v0 = __builtin_fmaf(a2[4 * g + k], s_par[0][cl + k], s_par[1][cl + k]);
                const float v1 = __builtin_fmaf(a2[4 * g + k + 1], s_par[0][cl + k + 1], s_par[1][cl + k + 1]);
                uint32_t w = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
                if (RELU) {
                    s16x2 h;
                    __builtin_memcpy(&h, &w, 4);
                    h = __builtin_elementwise_max(h, s16x2{0, 0});
                    __builtin_memcpy(&w, &h, 4);
                }
                pk[k >> 1] = w;
            }
            uint16_t *dst = row_ok && x0 + pl < r.w ? orow + pl * (int)ostr + cl : r.junk + lane * 16 + 4 * g;
            __builtin_memcpy(dst, pk, sizeof(pk));
        }
#else
        if constexpr (m16<Q, ST>()) {
            // tile t = 2h + nb: the lane's 4 consecutive channels 16h + 4 (lane / 16) .. of pixel 16 nb + lane % 16
    #pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int cl = 16 * (t >> 1) + 4 * (lane >> 4), px = 16 * (t & 1) + (lane & 15);
                uint32_t pk[2];
    #pragma unroll
                for (int k = 0; k < 4; k += 2) {
                    const float v0 = __builtin_fmaf(a2[4 * t + k], s_par[0][cl + k], s_par[1][cl + k]);
                    const float v1 = __builtin_fmaf(a2[4 * t + k + 1], s_par[0][cl + k + 1], s_par[1][cl + k + 1]);
                    uint32_t w = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
                    if (RELU) {
                        s16x2 hh;
                        __builtin_memcpy(&hh, &w, 4);
                        hh = __builtin_elementwise_max(hh, s16x2{0, 0});
                        __builtin_memcpy(&w, &hh, 4);
                    }
                    pk[k >> 1] = w;
                }
                __builtin_memcpy(s_o + px * REPI + cl * 2, pk, sizeof(pk));
            }
        } else {
    #pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int cl = 8 * g + 4 * hf;
            uint32_t pk[2];
    #pragma unroll
            for (int k = 0; k < 4; k += 2) {
                // fma(acc, scale, shift - center * scale) (scale 1 / shift 0 when absent), rounded to bf16,
                // ReLU as max(bits, 0) on the bf16 bit patterns as signed 16-bit integers (negatives, -0
                // and -NaN -> +0, +NaN kept): the tiled kernel's epilogue, bit for bit (shpl.h).
                const float v0 = __builtin_fmaf(a2[4 * g + k], s_par[0][cl + k], s_par[1][cl + k]);
                const float v1 = __builtin_fmaf(a2[4 * g + k + 1], s_par[0][cl + k + 1], s_par[1][cl + k + 1]);
                uint32_t w = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
                if (RELU) {
                    s16x2 h;
                    __builtin_memcpy(&h, &w, 4);
                    h = __builtin_elementwise_max(h, s16x2{0, 0});
                    __builtin_memcpy(&w, &h, 4);
                }
                pk[k >> 1] = w;
            }
            __builtin_memcpy(s_o + pl * REPI + cl * 2, pk, sizeof(pk));
        }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (occ2_form<Q, CMP, RELU, ST>()) {
            // buffer stores, whose masked lanes carry an offset past the row's range that the hardware drops:
            // pixels outside the map, and with m2 the unoccupied cells of out2 (the input gradient's pooled
            // channels: the pixel-keyed pull back to the image reads no other row) -- both stores always
            // issued, on one path (the ring's vmcnt arithmetic; no branch on m2)
            const uint32_t m = m2 ? (uint32_t)__builtin_amdgcn_readlane((int)m2row, b < 0 ? 0 : b) : 0xffffffffu;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(orow, (short)0, (int)((31 * ostr + 32) * 2), 0x00020000);
    #pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int pc = lane + 64 * k, px = pc >> 2, pi = pc & 3;
                const u32x4 v = *reinterpret_cast<const u32x4 *>(s_o + px * REPI + pi * 16);
                const bool ok = row_ok && x0 + px < r.w && ((m >> px) & 1u);
                const int off = ok ? (int)((px * ostr + pi * 8) * 2) : (int)0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, SHPL_ROWS_NTSTORE ? 2 : 0);  // 2: nt
            }
        } else {
    #pragma unroll
        for (int k = 0; k < 2; ++k) {  // 32 pixels x 4 pieces of 8 channels
            const int pc = lane + 64 * k, px = pc >> 2, pi = pc & 3;
            const u32x4 v = *reinterpret_cast<const u32x4 *>(s_o + px * REPI + pi * 16);
            uint16_t *dst = row_ok && x0 + px < r.w ? orow + px * (int)ostr + pi * 8 : r.junk + pc * 8;
#if SHPL_ROWS_NTSTORE
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(dst));
#else
            *reinterpret_cast<u32x4 *>(dst) = v;
#endif
        }
        }
#endif
        if constexpr (streg<Q, QA, CMP, ST>()) {
            // batch statistics of the pre-activation row (f32): the lane's channels 16h + 4 (lane / 16) + k at its
            // pixels lane % 16 and 16 + lane % 16 (tiles 2h, 2h + 1) summed, then halves exchanged across lane ^ 8
            // (bit 3 clear keeps h = 0, set h = 1) and added to the lane's band sums s_st[lane] / s_st[64 + lane]
            if (row_ok) {
                const int nv = r.w - x0, p = lane & 15;
                const bool ok0 = p < nv, ok1 = 16 + p < nv, hi = (lane >> 3) & 1;
                f32x4 ss = SHPL_ROWS_STREG == 2 ? str[0] : s_st[lane], sq = SHPL_ROWS_STREG == 2 ? str[1] : s_st[64 + lane];
    #pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float sv[2], qv[2];
    #pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const float v0 = ok0 ? a2[4 * (2 * h) + k] : 0.0f, v1 = ok1 ? a2[4 * (2 * h + 1) + k] : 0.0f;
                        sv[h] = __fadd_rn(v0, v1);
                        qv[h] = __fadd_rn(__fmul_rn(v0, v0), __fmul_rn(v1, v1));
                    }
                    const float ks = hi ? sv[1] : sv[0], gs = hi ? sv[0] : sv[1];
                    const float kq = hi ? qv[1] : qv[0], gq = hi ? qv[0] : qv[1];
                    ss[k] = __fadd_rn(ss[k], __fadd_rn(ks, lane_xor8(gs)));
                    sq[k] = __fadd_rn(sq[k], __fadd_rn(kq, lane_xor8(gq)));
                }
                if constexpr (SHPL_ROWS_STREG == 2) {
                    str[0] = ss;
                    str[1] = sq;
                } else {
                    s_st[lane] = ss;
                    s_st[64 + lane] = sq;
                }
            }
        } else if constexpr (ST) {
            // batch statistics of the pre-activation row (f32, as the tiled kernel): the accumulator through a
            // second transpose in the slot ([pixel][SPF floats]; LDS runs one wave's operations in order, so the
            // bf16 transpose's reads above are done first), then lane (cp, qt) sums channels 2cp, 2cp+1 over
            // pixels 8qt .. 8qt+7 of the row into its band sums (kept in LDS: the pooled form has no VGPR to spare)
            float *s_f = reinterpret_cast<float *>(s_o);
            if constexpr (m16<Q, ST>()) {
    #pragma unroll
                for (int t = 0; t < 4; ++t)
                    *reinterpret_cast<f32x4 *>(s_f + (16 * (t & 1) + (lane & 15)) * SPF + 16 * (t >> 1) +
                                               4 * (lane >> 4)) = tile4(a2, t);
            } else {
    #pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<f32x4 *>(s_f + pl * SPF + 8 * g + 4 * hf) =
                    f32x4{a2[4 * g], a2[4 * g + 1], a2[4 * g + 2], a2[4 * g + 3]};
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (row_ok) {
                const int cp = lane & 15, qt = lane >> 4, nv = r.w - x0;
                float t[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    #pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (k == 4) asm volatile("" ::: "memory");  // two batches of reads (transient registers)
                    const int px = 8 * qt + k;
                    f32x2 v = *reinterpret_cast<const f32x2 *>(s_f + px * SPF + 2 * cp);
                    if (px >= nv) v = f32x2{0.0f, 0.0f};
                    t[0] = __fadd_rn(t[0], v[0]);
                    t[1] = __fadd_rn(t[1], v[1]);
                    t[2] = __fadd_rn(t[2], __fmul_rn(v[0], v[0]));
                    t[3] = __fadd_rn(t[3], __fmul_rn(v[1], v[1]));
                }
                f32x4 a = s_st[lane];
    #pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = __fadd_rn(a[i], t[i]);
                s_st[lane] = a;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) a2[i] = 0.0f;
    // stage row j + RING into the slot (the transpose's reads of it are done first)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if SHPL_ROWS_PROBE == 3
    SHPL_STAMP(t3);
#endif
    if (SHPL_ROWS_PROBE == 2) return;
    const int jn = j + RING, y = ya - 1 + jn;
    const bool live = jn < n_in;
    uint64_t occ = 0;
    int32_t first = 0;
    if (CMP && live) {  // uniform LDS words (the band's halo-row windows)
        occ = s_occ[jn];
        first = s_first[jn];
    }
    // the pooled form with statistics keeps the lane offsets in LDS (OFFL: 6 VGPRs it does not have)
    uint32_t oa[L::NA];
    int32_t ob[L::NB > 0 ? L::NB : 1];
#pragma unroll
    for (int i = 0; i < L::NA; ++i) oa[i] = offsets_in_lds<Q, QA, CMP, ST>() ? s_offs[i * 64 + lane] : offa[i];
#pragma unroll
    for (int i = 0; i < (L::NB > 0 ? L::NB : 1); ++i)
        ob[i] = offsets_in_lds<Q, QA, CMP, ST>() ? (int32_t)s_offs[(L::NA + i) * 64 + lane] : offb[i];
    stage<Q, QA, CMP>(r, frame_row0 + (int64_t)y * r.w + x0 - 1, live && y >= 0 && y < r.h, occ, first, oa, ob,
                      s_ring + U * L::SLOT, lane);
#if SHPL_ROWS_PROBE == 3
    SHPL_STAMP(t4);
    ph[0] += t1 - t0;
    ph[1] += t2 - t1;
    ph[2] += t3 - t2;
    ph[3] += t4 - t3;
#endif
    (void)ph;
}

// Waves per SIMD: SHPL_ROWS_WPE, but the pooled 3 + 1 chunk form without ReLU on the 16x16 shape may drop to
// one (it needs 257 registers at two; the allocation differs from the ReLU form's by one register).
template <int Q, int QA, bool CMP, bool RELU, bool ST>
constexpr int rows_wpe_min() { return (m16<Q, ST>() && CMP && Q == 4 && QA == 3 && !RELU) ? 1 : SHPL_ROWS_WPE; }

template <int Q, int QA, bool CMP, bool RELU, bool ST>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(rows_wpe_min<Q, QA, CMP, RELU, ST>(),
                                                                    SHPL_ROWS_WPE))) void k_conv_rows(
    const RowArgs r) {
    typedef Layout<Q, QA, ST> L;
#if SHPL_ROWS_PROBE == 3
    uint64_t rt0;
    SHPL_RSTAMP(rt0);
#endif
    __shared__ __attribute__((aligned(16))) uint8_t s_ring[RING * L::SLOT];
    __shared__ __attribute__((aligned(16))) float s_par[2][NCO];
    // the halo rows' occupancy windows (entry j: input row ya - 1 + j): cells x0-1 .. x0+32 as bits 0..33, and
    // the frame-slot run index of the first of them
    __shared__ uint64_t s_occ[CMP ? 64 : 1];
    __shared__ int32_t s_first[CMP ? 64 : 1];
    const int lane = threadIdx.x;
    // (frame, band, strip, output block), output blocks fastest, then strips; each XCD (blocks b, b+8, ...)
    // takes one contiguous run of them, so the blocks of a strip read its rows together, and neighbouring
    // strips share their halo columns and neighbouring bands their halo rows, in that L2
#if SHPL_ROWS_XCD
    const int wi = (int)xcd_block(blockIdx.x, r.n_items * r.n_cob);
#else
    const int wi = blockIdx.x;
#endif
    const int cob = wi % r.n_cob, item = wi / r.n_cob;
    const int strip = item % r.strips, fb = item / r.strips;
    const int band = fb % r.n_bands, f = fb / r.n_bands;
    const bool second = r.out2 && cob * NCO >= r.c_split;
    uint16_t *const obase = second ? r.out2 + (cob * NCO - r.c_split) : r.out + cob * NCO;
    const int64_t ostr = second ? r.out2_stride : r.out_stride;
    // ST: lane (cp, qt)'s band sums of channels 2cp, 2cp+1 (sum, sum; square sum, square sum); with STREG the
    // lane's sums (s_st[lane]) and square sums (s_st[64 + lane]) of channels 16 ((lane / 8) % 2) + 4 (lane / 16) + k
    constexpr bool STREG = streg<Q, QA, CMP, ST>();
    __shared__ f32x4 s_st[ST ? (STREG ? 128 : 64) : 1];
    if constexpr (ST) s_st[lane] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (STREG) s_st[64 + lane] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int H = r.h;
    const int x0 = strip * TW, ya = band * r.band;
    const int n_out = min(r.band, H - ya), n_in = n_out + 2;
    const int64_t frame_row0 = (int64_t)f * H * r.w;
    if (lane < NCO) {  // scale (1 when absent) and shift - center * scale
        const int c = cob * NCO + lane;
        const float sc = r.scale ? r.scale[c] : 1.0f;
        const float ce = r.center ? r.center[c] : 0.0f;
        const float sh = r.shift ? r.shift[c] : 0.0f;
        s_par[0][lane] = sc;
        s_par[1][lane] = __fsub_rn(sh, __fmul_rn(ce, sc));
    }
    uint64_t b_rows = ~0ull;
    if constexpr (CMP) {
        const int y = ya - 1 + lane, w0 = x0 >> 5;
        uint64_t occ_row = 0;
        int32_t first_row = 0;
        if (lane < n_in && y >= 0 && y < H) {
            const int64_t wrow = ((int64_t)f * H + y) * r.wpr;
            const uint32_t ml = w0 > 0 ? r.occ[wrow + w0 - 1] : 0u, mc = r.occ[wrow + w0];
            const uint32_t mr = w0 + 1 < r.wpr ? r.occ[wrow + w0 + 1] : 0u;
            const int32_t bs = r.occ_base[wrow + (w0 > 0 ? w0 - 1 : w0)];
            occ_row = (uint64_t)(ml >> 31) | ((uint64_t)mc << 1) | ((uint64_t)(mr & 1u) << 33);
            first_row = (int32_t)r.frame_off[f] + bs + (w0 > 0 ? __popc(ml & 0x7fffffffu) : 0);
        }
        s_occ[lane] = occ_row;
        s_first[lane] = first_row;
        b_rows = __ballot(occ_row != 0);  // input rows with an occupied cell in their window
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS writes, in order
    }
    // out2 by occupancy: lane b holds the occupancy word of the strip's cells in output row ya + b (TW = 32: one
    // word), loaded before the weights' vmcnt(0) below retires it with them
    uint32_t m2row = 0u;
    const bool m2 = occ2_form<Q, CMP, RELU, ST>() && second && r.occ2 != nullptr;
    if (m2 && lane < n_out) m2row = r.occ2[((int64_t)f * H + ya + lane) * r.wpr + (x0 >> 5)];
    uint32_t offa[L::NA];
    int32_t offb[L::NB > 0 ? L::NB : 1];
    lane_offsets<Q, QA, CMP>(r, x0, lane, offa, offb);
    __shared__ uint32_t s_offs[offsets_in_lds<Q, QA, CMP, ST>() ? (L::NA + L::NB) * 64 : 1];
    if constexpr (offsets_in_lds<Q, QA, CMP, ST>()) {
#pragma unroll
        for (int i = 0; i < L::NA; ++i) s_offs[i * 64 + lane] = offa[i];
#pragma unroll
        for (int i = 0; i < L::NB; ++i) s_offs[(L::NA + i) * 64 + lane] = (uint32_t)offb[i];
    }
    // prologue: input rows 0 .. RING-1 in flight
#pragma unroll
    for (int j = 0; j < RING; ++j) {
        const int y = ya - 1 + j;
        stage<Q, QA, CMP>(r, frame_row0 + (int64_t)y * r.w + x0 - 1, j < n_in && y >= 0 && y < H, CMP ? s_occ[j] : 0,
                          CMP ? s_first[j] : 0, offa, offb, s_ring + j * L::SLOT, lane);
    }
    // the chunk weights of all taps stay in registers: A operands (32 output x 16 input channels)
    bf16x8 wr[Q][9];
    const uint16_t *wq = r.wp + (int64_t)cob * Q * W_ROWS * 16;
    if constexpr (m16<Q, ST>()) {
        // wr[2c + h][t]: the A operand of K-chunk c, output half h (lane: channel 16h + lane % 16, inputs
        // 8 (lane / 16) .. of the chunk: 16-channel chunk 2c + lane / 32, its half (lane / 16) % 2)
#pragma unroll
        for (int c = 0; c < Q / 2; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int t = 0; t < 9; ++t)
                    wr[2 * c + h][t] = *reinterpret_cast<const bf16x8 *>(
                        wq + (((2 * c + (lane >> 5)) * 9 + t) * NCO + 16 * h + (lane & 15)) * 16 + ((lane >> 4) & 1) * 8);
    } else {
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int t = 0; t < 9; ++t)
            wr[q][t] = *reinterpret_cast<const bf16x8 *>(wq + ((q * 9 + t) * NCO + (lane & 31)) * 16 + (lane >> 5) * 8);
    }
#if !SHPL_ROWS_WLATE
    // the weights have landed before the loop, as the compiler's wait model must know: its waitcnt pass
    // does not see the ring's asm DMAs, so weights still "pending" at the loop header made it put a ladder of
    // vmcnt waits down to vmcnt(0) among every row step's MFMAs -- draining the ring (the DMAs of the next two
    // rows and the stores) every row. The builtin clears its scoreboard (the prologue's DMAs land too)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
    const uint64_t m2live = m2 ? __ballot(m2row != 0u) : ~0ull;  // m2: the output rows with an occupied cell
    f32x16 acc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[k][i] = 0.0f;
    // B operand (pixels): lane (pl, hf) reads pixel pl (+ kx) of piece 2 q + hf
    const uint8_t *rd = s_ring + (lane >> 5) * HWD * 16 + (lane & 31) * 16;
    // 16x16x32 operand reads: K-chunk c's piece 4c + lane / 16 (from A below 2 QA, else B) at pixel lane % 16
    uint32_t rdq[2];  // byte offsets in s_ring
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int g = 4 * c + (lane >> 4);
        rdq[c] = (uint32_t)(((g < 2 * QA ? g * HWD : L::RB + (g - 2 * QA) * HWD) + (lane & 15)) * 16);
    }
    uint64_t ph[5] = {0, 0, 0, 0, 0};
    f32x4 str[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};  // STREG == 2: the band sums
#if SHPL_ROWS_PROBE == 3
    uint64_t tk0, rt1;
    SHPL_STAMP(tk0);
    SHPL_RSTAMP(rt1);
#endif
    for (int j = 0; j < n_in; j += RING) {
#define SHPL_ROWS_STEP(UU)                                                                                          \
    if (j + UU >= n_in) break;                                                                                      \
    step<Q, QA, CMP, RELU, ST, UU>(r, wr, acc, s_par, rd, s_ring, frame_row0, x0, ya, n_in, n_out, obase, ostr, s_st, \
                                   j + UU, s_occ, s_first, b_rows, offa, offb, s_offs, rdq, lane, str, ph, m2row, m2, m2live);
        SHPL_ROWS_STEP(0)
        SHPL_ROWS_STEP(1)
        SHPL_ROWS_STEP(2)
#undef SHPL_ROWS_STEP
    }
    asm volatile("s_waitcnt vmcnt(0) expcnt(5)" ::: "memory");  // the trailing DMAs land before the wave's LDS is released (expcnt(5): the ISA guard's exit marker)
#if SHPL_ROWS_PROBE == 3
    uint64_t tk1, rt2;
    SHPL_STAMP(tk1);
    SHPL_RSTAMP(rt2);
    if (lane == 0 && blockIdx.x < CPROBE_WAVES) {
        uint64_t *o = g_cprobe + 10 * (int64_t)blockIdx.x;
        o[6] = rt0;
        o[7] = rt1;
        o[8] = rt2;
        o[0] = ph[0];
        o[1] = ph[1];
        o[2] = ph[2];
        o[3] = ph[3];
        o[4] = tk1 - tk0;
        o[5] = (uint64_t)n_in;
    }
#endif
    if constexpr (STREG) {  // the band's sums over the 8 pixel lanes of each channel group, one double each
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        f32x4 ss = SHPL_ROWS_STREG == 2 ? str[0] : s_st[lane], sq = SHPL_ROWS_STREG == 2 ? str[1] : s_st[64 + lane];
#pragma unroll
        for (int o = 1; o < 8; o <<= 1)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ss[k] = __fadd_rn(ss[k], __shfl_xor(ss[k], o, 64));
                sq[k] = __fadd_rn(sq[k], __shfl_xor(sq[k], o, 64));
            }
        if ((lane & 7) == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int c = cob * NCO + 16 * ((lane >> 3) & 1) + 4 * (lane >> 4) + k;
                r.part[((int64_t)c * 2 + 0) * r.n_items + item] = (double)ss[k];
                r.part[((int64_t)c * 2 + 1) * r.n_items + item] = (double)sq[k];
            }
        }
    } else if constexpr (ST) {  // the band's sums over the 4 pixel quarters, then one double per (channel, statistic)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const f32x4 a = s_st[lane];
        float sst[4] = {a[0], a[1], a[2], a[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            sst[i] = __fadd_rn(sst[i], __shfl_xor(sst[i], 16, 64));
            sst[i] = __fadd_rn(sst[i], __shfl_xor(sst[i], 32, 64));
        }
        if (lane < 16) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = cob * NCO + 2 * lane + (i & 1), st = i >> 1;
                r.part[((int64_t)c * 2 + st) * r.n_items + item] = (double)sst[i];
            }
        }
    }
}


// ---- The bf16 weight gradient, row-streaming (k_wgrad_rows) ----
//
// dW[ky][kx][ci][co] = sum over pixels of X[y+ky-1][x+kx-1][ci] * G[y][x][co]
// as MFMAs with the pixels as K: D[ci][co] += Xᵀ[ci][px] G[px][co]. Both
// operands want 8 consecutive pixels of one channel per lane, i.e. the NHWC
// rows transposed; ds_read_b64_tr_b16 reads them so straight from the rows as
// the LDS-DMA lands them ([pixel][32 channels], 64 B per pixel: 4 rows of a
// read cover the 64 banks once). One wave per workgroup owns one 32-channel
// input tile x one 32-channel output tile, keeps the 9 taps' accumulators
// (144 VGPRs) for a whole run of items (frame, band, strip), and streams the
// band's input rows j through the per-wave ring of the forward (3 slots, 2
// rows ahead, counted vmcnt): row j of X (34 halo pixels) and row j of G
// arrive together; X row j meets G rows j, j-1, j-2 (ky = 0, 1, 2; the two
// older G fragments stay in registers), so each staged row is read once: 16
// transposed reads per 18 MFMAs. G rows outside the band read zeros (exact
// zero products). Per wave one f32 partial of the 9 x 32 x 32 tile; two
// fixed-order reductions (f64) give dW: deterministic.
#ifndef SHPL_WG_PROBE
#define SHPL_WG_PROBE 0
#endif
#ifndef SHPL_WG_PAIR
#define SHPL_WG_PAIR 1
#endif

constexpr int WX_PIECES = HWD * 4;                  // X row: 34 pixels x 4 pieces of 8 channels
constexpr int WG_PIECES = TW * 4;                   // G row: 32 pixels x 4 pieces
constexpr int WXB = WX_PIECES * 16, WGB = WG_PIECES * 16;  // 2176 + 2048 B
constexpr int WNX = (WX_PIECES + 63) / 64, WTX = WX_PIECES - 64 * (WNX - 1);  // 3 DMAs, the last one 8 lanes
constexpr int WNG = WG_PIECES / 64;                                         // 2 DMAs
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// PAIR: two waves per workgroup, input tiles 2p and 2p+1 of one output tile. They share each staged G row
// (wave w DMAs its half, pixels 16w .. 16w+15) and run in step: one s_barrier per row, after the ring wait.
// A ring slot then holds [X of wave 0][X of wave 1][G]; 4 slots, so that the row staged at step j (j + 3) goes
// into the slot of row j - 1, which both waves finished reading before step j's barrier. Alone (an odd number
// of input tiles) a wave DMAs the whole G row, and 3 slots suffice (row j + 3 into row j's own slot).
template <bool PAIR>
struct WgRing {
    static constexpr int NSLOT = PAIR ? 4 : 3;
    static constexpr int SLOT = (PAIR ? 2 : 1) * WXB + WGB;
    static constexpr int GOFF = (PAIR ? 2 : 1) * WXB;
    static constexpr int NG = PAIR ? 1 : WNG;  // G DMAs per wave
    static constexpr int NDMA = WNX + NG;
};

// The 32x16 operand fragment at pixel p0 (+ 8h + 4t + q) of an LDS image [pixel][64 B]: two transposed reads
// (lane 4q+p of 16-lane group g: row q, channels 16 (g & 1) + 4p .. + 3; lane i of the group gets channel
// 16 (g & 1) + i). `lb` holds the lane's part of the address; p0 a compile-time pixel offset.
template <int P0>
__device__ __forceinline__ bf16x8 tr_frag(const uint8_t *lb) {
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(lb + P0 * 64));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(lb + (P0 + 4) * 64));
    const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    bf16x8 out;
    __builtin_memcpy(&out, &v, 16);
    return out;
}

// pooled: X is the tile of the compact pooled rows (k_pool_runs): offx holds pixel << 16 | channel (-1: outside),
// cell pixel px of the row holds run  first + popc(occ below bit px)  when bit px of occ is set, else zeros.
// `xslot` is the wave's X part of the slot, `gslot` the G part (PAIR: this wave's half of it).
template <bool CMP, bool PAIR>
__device__ __forceinline__ void wstage(const WgRowArgs &r, const uint16_t *xsrc, int64_t xstride, int64_t pix0,
                                       bool xok, int64_t gpix, bool gok, const uint32_t (&offx)[WNX],
                                       const uint32_t (&offg)[WgRing<PAIR>::NG], uint8_t *xslot, uint8_t *gslot,
                                       int lane, bool pooled, uint64_t occ, int32_t first) {
    // one set of X DMAs whichever the source (selects, no branch: every path issues NDMA DMAs)
    const bool cmp = CMP && pooled;
    const i32x4 rx = rsrc(cmp ? static_cast<const void *>(r.cmp) : static_cast<const void *>(xsrc + pix0 * xstride),
                          xok ? OOB : 0u);
#pragma unroll
    for (int i = 0; i < WNX; ++i) {
        uint32_t o = offx[i];
        if (cmp) {
            const int32_t e = (int32_t)offx[i];
            const int px = (e >> 16) & 63;
            const bool hit = e >= 0 && ((occ >> px) & 1);
            const int rank = first + (int)__popcll(occ & ((1ull << px) - 1));
            o = hit ? (uint32_t)((rank * r.cmp_stride + (e & 0xffff)) * 2) : OOB;
        }
        if (i < WNX - 1 || lane < WTX) dma16(rx, o, xslot + i * 1024);
    }
    const i32x4 rg = rsrc(r.gy + gpix * r.gy_stride, gok ? OOB : 0u);
#pragma unroll
    for (int i = 0; i < WgRing<PAIR>::NG; ++i) dma16(rg, offg[i], gslot + i * 1024);
}

// One input row j of the band (slot U = j % NSLOT): 16 transposed reads, 18 MFMAs, then row j + 3 staged.
template <bool CMP, bool PAIR, int U>
__device__ __forceinline__ void wstep(const WgRowArgs &r, f32x16 (&acc)[9], bf16x8 (&g1)[2], bf16x8 (&g2)[2],
                                      uint8_t *s_ring, const uint8_t *lb, int xoff, int goff_w,
                                      const uint16_t *xsrc, int64_t xstride, int64_t frame_row0, int x0, int ya,
                                      int n_in, int n_out, int j, const uint32_t (&offx)[WNX],
                                      const uint32_t (&offg)[WgRing<PAIR>::NG], int lane, bool pooled,
                                      const uint64_t *s_occ, const int32_t *s_first) {
    typedef WgRing<PAIR> R;
    SHPL_RING_WAIT(R::NDMA * (RING - 1));  // rows j+1, j+2 may still be in flight
    if (PAIR) asm volatile("s_barrier" ::: "memory");  // the other wave's half of G row j has landed too
    const uint8_t *xs = lb + U * R::SLOT + xoff, *gs = lb + U * R::SLOT + R::GOFF;
    bf16x8 g0[2];
    g0[0] = tr_frag<0>(gs);
    g0[1] = tr_frag<16>(gs);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const bf16x8 xa = kx == 0 ? tr_frag<0>(xs + s * 1024) : kx == 1 ? tr_frag<1>(xs + s * 1024)
                                                                             : tr_frag<2>(xs + s * 1024);
            acc[kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, g0[s], acc[kx], 0, 0, 0);
            acc[3 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, g1[s], acc[3 + kx], 0, 0, 0);
            acc[6 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, g2[s], acc[6 + kx], 0, 0, 0);
        }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        g2[s] = g1[s];
        g1[s] = g0[s];
    }
    // the slot's reads are done before the DMAs refill it (PAIR: before the next barrier, after which the
    // other wave refills this slot)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int jn = j + RING, y = ya - 1 + jn;
    if (SHPL_WG_PROBE == 1) return;  // timing probe: no staging in the loop (wrong results)
    uint64_t occ = 0;
    int32_t first = 0;
    if (CMP && pooled && jn < n_in) {
        occ = s_occ[jn];
        first = s_first[jn];
    }
    uint8_t *ns = s_ring + ((U + RING) % R::NSLOT) * R::SLOT;
    wstage<CMP, PAIR>(r, xsrc, xstride, frame_row0 + (int64_t)y * r.w + x0 - 1, jn < n_in && y >= 0 && y < r.h,
                      frame_row0 + (int64_t)(ya + jn) * r.w + x0, jn < n_out, offx, offg, ns + xoff,
                      ns + R::GOFF + goff_w, lane, pooled, occ, first);
}

template <bool CMP, bool PAIR>
__global__ __launch_bounds__(PAIR ? 128 : 64) __attribute__((amdgpu_waves_per_eu(SHPL_ROWS_WPE, SHPL_ROWS_WPE)))
void k_wgrad_rows(const WgRowArgs r) {
    typedef WgRing<PAIR> R;
    constexpr int NW = PAIR ? 2 : 1;
    __shared__ __attribute__((aligned(16))) uint8_t s_ring[R::NSLOT * R::SLOT];
    __shared__ uint64_t s_occ_all[NW][CMP ? 64 : 1];  // pooled tile: the band rows' occupancy windows (as k_conv_rows)
    __shared__ int32_t s_first_all[NW][CMP ? 64 : 1];
    const int lane = threadIdx.x & 63, wv = PAIR ? (int)(threadIdx.x >> 6) : 0;
    uint64_t *s_occ = s_occ_all[wv];
    int32_t *s_first = s_first_all[wv];
    const int n_cw = r.n_cit / NW;  // workgroups per (group, output tile)
    const int total = r.n_groups * r.n_cot * n_cw;
    // (group, output tile, input tiles), input tiles fastest (they share the G rows), each XCD one contiguous run
    const int wi = (int)xcd_block(blockIdx.x, total);
    const int cit = (wi % n_cw) * NW + wv, cot = (wi / n_cw) % r.n_cot, grp = wi / (n_cw * r.n_cot);
    const int na = r.c_a / 32 + (r.c_a % 32 ? 1 : 0);  // input tiles of A (c_a % 32 == 0 when B is present)
    const bool from_a = cit < na;
    const uint16_t *xsrc = from_a ? r.a + cit * 32 : r.b + (cit - na) * 32;
    const int64_t xstride = from_a ? r.a_stride : r.b_stride;
    const int cn = from_a ? r.c_a - cit * 32 : r.c_b - (cit - na) * 32;  // channels of the tile (>= 32: whole)
    const bool pooled = CMP && !from_a;  // B pooled from the image through the cell-keyed CSR
    const int cg = r.c_out - cot * 32;
    const uint16_t *gsrc = r.gy + cot * 32;
    WgRowArgs rr = r;
    rr.gy = gsrc;
    const int64_t i0 = (int64_t)grp * r.n_items / r.n_groups, i1 = (int64_t)(grp + 1) * r.n_items / r.n_groups;
    // lane address part of the transposed reads: row q = (lane & 15) >> 2, channel 16 ((lane >> 4) & 1) + 4 (lane & 3),
    // pixel base 8 h (h = lane >> 5)
    const uint8_t *lb = s_ring + (8 * (lane >> 5) + ((lane & 15) >> 2)) * 64 + 32 * ((lane >> 4) & 1) + 8 * (lane & 3);
    const int xoff = wv * WXB, goff_w = PAIR ? wv * 1024 : 0;
    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.0f;
    for (int64_t it = i0; it < i1; ++it) {
        const int item = (int)it;
        const int strip = item % r.strips, fb = item / r.strips;
        const int band = fb % r.n_bands, f = fb / r.n_bands;
        const int x0 = strip * TW, ya = band * r.band;
        const int n_out = min(r.band, r.h - ya), n_in = n_out + 2;
        const int64_t frame_row0 = (int64_t)f * r.h * r.w;
        uint32_t offx[WNX], offg[R::NG];
#pragma unroll
        for (int i = 0; i < WNX; ++i) {
            const int pc = 64 * i + lane, px = pc >> 2, cq = pc & 3, x = x0 - 1 + px;
            const bool ok = pc < WX_PIECES && x >= 0 && x < r.w && 8 * cq < cn;
            if (pooled)
                offx[i] = ok ? (uint32_t)((px << 16) | ((cit - na) * 32 + 8 * cq)) : 0xffffffffu;
            else
                offx[i] = ok ? (uint32_t)((px * (int)xstride + 8 * cq) * 2) : OOB;
        }
        if (pooled) {  // lane j: halo row j's window (cells x0-1 .. x0+32 as bits 0..33) and its first run
            const int y = ya - 1 + lane, w0 = x0 >> 5;
            uint64_t occ_row = 0;
            int32_t first_row = 0;
            if (lane < n_in && y >= 0 && y < r.h) {
                const int64_t wrow = ((int64_t)f * r.h + y) * r.wpr;
                const uint32_t ml = w0 > 0 ? r.occ[wrow + w0 - 1] : 0u, mc = r.occ[wrow + w0];
                const uint32_t mr = w0 + 1 < r.wpr ? r.occ[wrow + w0 + 1] : 0u;
                const int32_t bs = r.occ_base[wrow + (w0 > 0 ? w0 - 1 : w0)];
                occ_row = (uint64_t)(ml >> 31) | ((uint64_t)mc << 1) | ((uint64_t)(mr & 1u) << 33);
                first_row = (int32_t)r.frame_off[f] + bs + (w0 > 0 ? __popc(ml & 0x7fffffffu) : 0);
            }
            s_occ[lane] = occ_row;
            s_first[lane] = first_row;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its own LDS writes, in order
        }
#pragma unroll
        for (int i = 0; i < R::NG; ++i) {
            const int pc = 64 * (PAIR ? wv : i) + lane, px = pc >> 2, cq = pc & 3, x = x0 + px;
            offg[i] = x < r.w && 8 * cq < cg ? (uint32_t)((px * (int)r.gy_stride + 8 * cq) * 2) : OOB;
        }
#pragma unroll
        for (int j = 0; j < RING; ++j) {
            const int y = ya - 1 + j;
            uint8_t *sl = s_ring + j * R::SLOT;
            wstage<CMP, PAIR>(rr, xsrc, xstride, frame_row0 + (int64_t)y * r.w + x0 - 1,
                              j < n_in && y >= 0 && y < r.h, frame_row0 + (int64_t)(ya + j) * r.w + x0, j < n_out,
                              offx, offg, sl + xoff, sl + R::GOFF + goff_w, lane, pooled, pooled ? s_occ[j] : 0,
                              pooled ? s_first[j] : 0);
        }
        bf16x8 g1[2], g2[2];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 8; ++i) g1[s][i] = g2[s][i] = (__bf16)0.0f;
        for (int j = 0; j < n_in; j += R::NSLOT) {
#define SHPL_WROWS_STEP(UU)                                                                                      \
    if (UU < R::NSLOT) {                                                                                         \
        if (j + UU >= n_in) break;                                                                               \
        wstep<CMP, PAIR, UU % R::NSLOT>(rr, acc, g1, g2, s_ring, lb, xoff, goff_w, xsrc, xstride, frame_row0, x0, \
                                        ya, n_in, n_out, j + UU, offx, offg, lane, pooled, s_occ, s_first);       \
    }
            SHPL_WROWS_STEP(0)
            SHPL_WROWS_STEP(1)
            SHPL_WROWS_STEP(2)
            SHPL_WROWS_STEP(3)
#undef SHPL_WROWS_STEP
        }
        asm volatile("s_waitcnt vmcnt(0) expcnt(5)" ::: "memory");  // the trailing DMAs land before the next item's prologue (exit marker)
        // PAIR: both waves are done with the item's slots before either stages the next item's rows into them
        if (PAIR) asm volatile("s_barrier" ::: "memory");
    }
// partial [group][cot][cit][tap][co][ci]: lane (co = lane & 31, h) holds ci 8 (i >> 2) + 4 h + (i & 3)
    float *out = r.part + (((int64_t)grp * r.n_cot + cot) * r.n_cit + cit) * (9 * 1024) + (lane & 31) * 32 +
                 4 * (lane >> 5);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4 *>(out + t * 1024 + 8 * g) =
                f32x4{acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]};
}

// Level 1: entries e of the partial tile set, summed over groups [c*WGC, (c+1)*WGC) in order (f64).
constexpr int WGC = 32;
__global__ __launch_bounds__(SHPL_BLOCK) void k_wgrad_rows_sum(const float *part, int64_t n_ent, int n_groups,
                                                               double *part2) {
    const int64_t e = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x;
    if (e >= n_ent) return;
    const int c = blockIdx.y, g0 = c * WGC, g1 = min(g0 + WGC, n_groups);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    int g = g0;
    for (; g + 3 < g1; g += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += (double)part[(int64_t)(g + u) * n_ent + e];
    }
    for (int u = 0; g < g1; ++g, ++u) acc[u] += (double)part[(int64_t)g * n_ent + e];
    part2[(int64_t)c * n_ent + e] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// Level 2: dW (HWIO f32) from the chunk sums, in order.
__global__ __launch_bounds__(SHPL_BLOCK) void k_wgrad_rows_final(const double *part2, int n_chunks, int64_t n_ent,
                                                                 int c_a, int c_b, int c_out, int n_cit, int n_cot,
                                                                 float *dw) {
    const int cin = c_a + c_b;
    const int64_t o = (int64_t)blockIdx.x * SHPL_BLOCK + threadIdx.x;
    if (o >= (int64_t)9 * cin * c_out) return;
    const int co = (int)(o % c_out), ci = (int)((o / c_out) % cin), tap = (int)(o / ((int64_t)c_out * cin));
    const int na = c_a / 32 + (c_a % 32 ? 1 : 0);
    const int cit = ci < c_a ? ci / 32 : na + (ci - c_a) / 32, lci = ci < c_a ? ci % 32 : (ci - c_a) % 32;
    const int64_t e = ((int64_t)(co / 32) * n_cit + cit) * (9 * 1024) + tap * 1024 + (co % 32) * 32 + lci;
    double s = 0.0;
    for (int c = 0; c < n_chunks; ++c) s += part2[(int64_t)c * n_ent + e];
    dw[o] = (float)s;
}
}  // namespace

bool supported(int q, int qa) {
    if (q < 1 || q > 4 || qa < 1 || qa > q) return false;
    return qa == q || q - qa >= 1;
}

// Statistics: not at 3 chunks from two sources (those spill at 256 VGPRs); pooled at 2 + 2 and 1 + 1 chunks
// (the lane offsets in LDS).
bool supported_st(int q, int qa, bool cmp) {
    if (!supported(q, qa)) return false;
    return cmp ? (q == 4 && qa == 2) || (q == 2 && qa == 1) : !(q == 3 && qa < 3);
}

int prep_pooled(int n_frames, int h, int w, int wpr, const int32_t *ent_dst, const int32_t *ent_src,
                const float *ent_val, int64_t nnz_cap, const int64_t *frame_off, const uint16_t *img,
                int64_t img_stride, int64_t img_off, int c_b, uint32_t *occ, int32_t *occ_base, uint16_t *cmp,
                hipStream_t s) {
    hipLaunchKernelGGL(k_occ_frame, dim3(n_frames), dim3(1024), 0, s, ent_dst, frame_off, h, w, wpr, occ, occ_base);
    SHPL_LAUNCH_CHECK();
    const int np = c_b / 8;
    if (nnz_cap > 0 && np > 0) {
        const dim3 grid((unsigned)((nnz_cap + SHPL_BLOCK - 1) / SHPL_BLOCK));
        switch (np) {
#define SHPL_POOL_RUNS(NP)                                                                                       \
    case NP:                                                                                                     \
        hipLaunchKernelGGL(k_pool_runs<NP>, grid, dim3(SHPL_BLOCK), 0, s, ent_dst, ent_src, ent_val, nnz_cap, img, \
                           img_stride, img_off, c_b, h, w, wpr, occ, occ_base, frame_off, cmp);                   \
        break;
            SHPL_POOL_RUNS(1)
            SHPL_POOL_RUNS(2)
            SHPL_POOL_RUNS(3)
            SHPL_POOL_RUNS(4)
            SHPL_POOL_RUNS(5)
            SHPL_POOL_RUNS(6)
            SHPL_POOL_RUNS(7)
            SHPL_POOL_RUNS(8)
#undef SHPL_POOL_RUNS
            default:
                return SHPL_ERR_ARG;
        }
        SHPL_LAUNCH_CHECK();
    }
    return SHPL_OK;
}

int launch(const RowArgs &r, int q, int qa, bool cmp, bool relu, bool st, hipStream_t s) {
    if (!supported(q, qa) || (cmp && qa == q) || (st && (relu || !r.part || !supported_st(q, qa, cmp))) || r.n_cob < 1)
        return SHPL_ERR_ARG;
    if ((int64_t)r.n_items * r.n_cob >= (1LL << 31)) return SHPL_ERR_BAD_SHAPE;
    if (r.out2 && r.c_split % NCO != 0) return SHPL_ERR_ARG;
    const dim3 grid((unsigned)(r.n_items * r.n_cob));
    const int key = (((q * 8 + qa) * 2 + (cmp ? 1 : 0)) * 2 + (relu ? 1 : 0)) * 2 + (st ? 1 : 0);
    switch (key) {
#define SHPL_ROWS_CASE(QQ, QQA, CMP, RELU, ST)                                                  \
    case (((QQ * 8 + QQA) * 2 + CMP) * 2 + RELU) * 2 + ST:                                      \
        hipLaunchKernelGGL((k_conv_rows<QQ, QQA, CMP, RELU, ST>), grid, dim3(64), 0, s, r);     \
        break;
    // statistics only beside the plain epilogue (the training forward writes the pre-activation output)
#define SHPL_ROWS_DENSE(QQ) SHPL_ROWS_CASE(QQ, QQ, 0, 0, 0) SHPL_ROWS_CASE(QQ, QQ, 0, 1, 0) SHPL_ROWS_CASE(QQ, QQ, 0, 0, 1)
#define SHPL_ROWS_TWO(QQ, QQA)                                                                                 \
    SHPL_ROWS_CASE(QQ, QQA, 0, 0, 0)                                                                          \
    SHPL_ROWS_CASE(QQ, QQA, 0, 1, 0) SHPL_ROWS_CASE(QQ, QQA, 1, 0, 0) SHPL_ROWS_CASE(QQ, QQA, 1, 1, 0)
        SHPL_ROWS_DENSE(1)
        SHPL_ROWS_DENSE(2)
        SHPL_ROWS_DENSE(3)
        SHPL_ROWS_DENSE(4)
        SHPL_ROWS_TWO(2, 1)
        SHPL_ROWS_TWO(3, 1)
        SHPL_ROWS_TWO(3, 2)
        SHPL_ROWS_TWO(4, 1)
        SHPL_ROWS_TWO(4, 2)
        SHPL_ROWS_TWO(4, 3)
        SHPL_ROWS_CASE(2, 1, 0, 0, 1)
        SHPL_ROWS_CASE(4, 1, 0, 0, 1)
        SHPL_ROWS_CASE(4, 2, 0, 0, 1)
        SHPL_ROWS_CASE(4, 3, 0, 0, 1)
        SHPL_ROWS_CASE(2, 1, 1, 0, 1)
        SHPL_ROWS_CASE(4, 2, 1, 0, 1)
#undef SHPL_ROWS_TWO
#undef SHPL_ROWS_DENSE
#undef SHPL_ROWS_CASE
        default:
            return SHPL_ERR_ARG;
    }
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}


bool wgrad_supported(int c_a, int c_b, int c_out) {
    if (c_a < 0 || c_b < 0 || c_a + c_b < 1 || c_out < 1) return false;
    if (c_a % 8 || c_b % 8 || c_out % 8) return false;
    return c_b == 0 || c_a % 32 == 0;  // an input tile never straddles the two sources
}

void wgrad_sizes(int n_items, int c_a, int c_b, int c_out, int *n_groups, size_t *part_bytes, size_t *part2_bytes) {
    const int n_cit = (c_a + 31) / 32 + (c_b + 31) / 32, n_cot = (c_out + 31) / 32;
    int g = 2048 / (n_cit * n_cot);  // 8 waves per CU
    if (g < 1) g = 1;
    if (g > n_items) g = n_items > 0 ? n_items : 1;
    *n_groups = g;
    const int64_t n_ent = (int64_t)n_cit * n_cot * 9 * 1024;
    *part_bytes = (size_t)g * n_ent * 4;
    *part2_bytes = (size_t)((g + WGC - 1) / WGC) * n_ent * 8;
}

int wgrad_launch(const WgRowArgs &r, float *dw, double *part2, hipStream_t s) {
    // pairs of input tiles share their G rows (SHPL_WG_PAIR 0: one wave per input tile)
    const bool pair = SHPL_WG_PAIR && r.n_cit % 2 == 0;
    const int total = r.n_groups * r.n_cot * (pair ? r.n_cit / 2 : r.n_cit);
    const dim3 grid((unsigned)total), block(pair ? 128 : 64);
    if (r.cmp) {
        if (pair)
            hipLaunchKernelGGL((k_wgrad_rows<true, true>), grid, block, 0, s, r);
        else
            hipLaunchKernelGGL((k_wgrad_rows<true, false>), grid, block, 0, s, r);
    } else {
        if (pair)
            hipLaunchKernelGGL((k_wgrad_rows<false, true>), grid, block, 0, s, r);
        else
            hipLaunchKernelGGL((k_wgrad_rows<false, false>), grid, block, 0, s, r);
    }
    SHPL_LAUNCH_CHECK();
    const int64_t n_ent = (int64_t)r.n_cit * r.n_cot * 9 * 1024;
    const int n_chunks = (r.n_groups + WGC - 1) / WGC;
    hipLaunchKernelGGL(k_wgrad_rows_sum, dim3((unsigned)((n_ent + SHPL_BLOCK - 1) / SHPL_BLOCK), (unsigned)n_chunks),
                       dim3(SHPL_BLOCK), 0, s, r.part, n_ent, r.n_groups, part2);
    SHPL_LAUNCH_CHECK();
    const int64_t n_out = (int64_t)9 * (r.c_a + r.c_b) * r.c_out;
    hipLaunchKernelGGL(k_wgrad_rows_final, dim3((unsigned)((n_out + SHPL_BLOCK - 1) / SHPL_BLOCK)), dim3(SHPL_BLOCK),
                       0, s, part2, n_chunks, n_ent, r.c_a, r.c_b, r.c_out, r.n_cit, r.n_cot, dw);
    SHPL_LAUNCH_CHECK();
    return SHPL_OK;
}

}  // namespace rows
}  // namespace shpl

#if SHPL_ROWS_PROBE == 3
// probe builds only: the last k_conv_rows launch's per-wave phase sums (s_memtime cycles: ring wait, operand
// reads + MFMA issue, epilogue, staging, whole loop; input rows; s_memrealtime at the wave's start, loop start
// and loop end)
extern "C" int shpl_probe_conv_phases(uint64_t *host, size_t n_waves) {
    if (n_waves > (size_t)shpl::rows::CPROBE_WAVES) n_waves = shpl::rows::CPROBE_WAVES;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(shpl::rows::g_cprobe), 80 * n_waves, 0, hipMemcpyDeviceToHost) ==
                   hipSuccess
               ? SHPL_OK
               : SHPL_ERR_HIP;
}
#endif
