// shpl_conv_rows.h -- the row-streaming bf16 conv (shpl_conv_rows.hip) as the
// tiled conv's host code (shpl_conv.hip) launches it.
#pragma once

#include "shpl_common.h"

namespace shpl {
namespace rows {

constexpr int OCC_MAX_WORDS = 18432;  // k_occ_frame's LDS mask and prefixes: up to 589,824 cells per frame

struct RowArgs {
    const uint16_t *a, *b;       // A / B rows (the channel offsets applied)
    int64_t a_stride, b_stride;  // elements
    int c_a, c_b;
    int h, w, strips, band, n_bands, n_items;
    const uint16_t *wp;          // packed weights [co_block][chunk][tap][32][16] (k_pack_w)
    const float *center, *scale, *shift;
    uint16_t *out;
    int64_t out_stride;
    const uint32_t *occ;         // CMP: occupancy words, their prefix counts, compact pooled rows, entry slots
    const int32_t *occ_base;
    int wpr;
    const uint16_t *cmp;
    const int64_t *frame_off;
    uint16_t *junk;              // 32 x 32 channels: stores of rows / pixels outside the map land here
    uint16_t *out2;              // output blocks from channel c_split on go here (the input gradient's two maps)
    int64_t out2_stride;
    int c_split;                 // a multiple of 32 when out2 is set
    const uint32_t *occ2;        // out2 written only at the cells set in these occupancy words (wpr per row; NULL: all)
    int n_cob;                   // output blocks (the fastest index of a workgroup's item)
    double *part;                // ST: per-item channel sums [(co * 2 + stat) * n_items + item]
};

// k_conv_rows has an instantiation for q chunks of which qa come from A
// (supported_st: with the batch-statistics epilogue).
bool supported(int q, int qa);
bool supported_st(int q, int qa, bool cmp);

// Occupancy words + prefix counts of the cell-keyed CSR per frame, then the
// pooled vector of every run into its compact row (shpl_pull's arithmetic).
int prep_pooled(int n_frames, int h, int w, int wpr, const int32_t *ent_dst, const int32_t *ent_src,
                const float *ent_val, int64_t nnz_cap, const int64_t *frame_off, const uint16_t *img,
                int64_t img_stride, int64_t img_off, int c_b, uint32_t *occ, int32_t *occ_base, uint16_t *cmp,
                hipStream_t s);

// The conv: n_items * n_cob one-wave workgroups (ST: also the per-item
// channel sums of the pre-activation output, for k_stats_reduce).
int launch(const RowArgs &r, int q, int qa, bool cmp, bool relu, bool st, hipStream_t s);

// The bf16 weight gradient (k_wgrad_rows): dense sources, input tiles of 32
// channels within one source, outputs in tiles of 32.
struct WgRowArgs {
    const uint16_t *a, *b;
    int64_t a_stride, b_stride;
    int c_a, c_b;
    const uint16_t *gy;
    int64_t gy_stride;
    int c_out;
    int h, w, strips, band, n_bands, n_items;
    int n_cit, n_cot, n_groups;
    float *part;  // [group][cot][cit][9][32 co][32 ci]
    // pooled B (cmp set): the compact pooled rows of prep_pooled (cmp_stride = c_b channels per row), their
    // occupancy words and prefix counts, the frames' entry slots
    const uint16_t *cmp;
    int cmp_stride;
    const uint32_t *occ;
    const int32_t *occ_base;
    int wpr;
    const int64_t *frame_off;
};

bool wgrad_supported(int c_a, int c_b, int c_out);
void wgrad_sizes(int n_items, int c_a, int c_b, int c_out, int *n_groups, size_t *part_bytes, size_t *part2_bytes);
int wgrad_launch(const WgRowArgs &r, float *dw, double *part2, hipStream_t s);

}  // namespace rows
}  // namespace shpl
