// shpl_conv_wide.h -- the bf16 3x3 conv for wide channel counts (shpl_conv_wide.hip) as the conv's host
// code (shpl_conv.hip) launches it.
#pragma once

#include "shpl_common.h"

namespace shpl {
namespace wide {

constexpr int KC = 64;   // input channels per staged chunk
constexpr int NT = 256;  // output channels per workgroup

struct WideArgs {
    const uint16_t *a, *b;       // A / B rows (channel offsets applied); B NULL when c_b == 0
    int64_t a_stride, b_stride;  // elements
    int c_a, c_b;                // multiples of KC
    int n_frames, h, w;
    const uint16_t *wp;          // packed weights (k_pack_wide)
    const float *center, *scale, *shift;
    int act;
    uint16_t *out;
    int64_t out_stride;
    int c_out;                   // a multiple of NT
    // pooled B (cmp set): B's rows are the compact pooled runs of the cell-keyed CSR (prep), gathered per
    // pixel through the occupancy words: row frame_off[f] + occ_base[word] + popcount(bits below), zeros where
    // the bit is clear; b / b_stride unused
    const uint32_t *occ;
    const int32_t *occ_base;
    const int64_t *frame_off;
    const uint16_t *cmp;
    int wpr;
};

// Whether the wide kernel takes a bf16 forward of these channel counts (the row kernels' range, at most
// 64 input channels, stays theirs).
bool supported(int64_t c_a, int64_t c_b, int64_t c_out);
// Bytes of its packed weights.
size_t packed_bytes(int64_t c_a, int64_t c_b, int64_t c_out);
// The pooled operand of a fused call: occupancy words + prefix counts per frame (rows::prep_pooled's
// k_occ_frame), then every run's pooled vector into its compact row with shpl_pull's arithmetic -- one thread
// per (entry, 16-byte piece), so any channel count.
int prep(int n_frames, int h, int w, int wpr, const int32_t *ent_dst, const int32_t *ent_src, const float *ent_val,
         int64_t nnz_cap, const int64_t *frame_off, const uint16_t *img, int64_t img_stride, int64_t img_off, int c_b,
         uint32_t *occ, int32_t *occ_base, uint16_t *cmp, hipStream_t s);
// Pack the HWIO bf16 weights into wp, then the conv.
int launch(const WideArgs &a, const uint16_t *w_hwio, uint16_t *wp, hipStream_t s);

}  // namespace wide
}  // namespace shpl
