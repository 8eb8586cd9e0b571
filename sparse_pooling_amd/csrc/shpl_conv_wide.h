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
};

// Whether the wide kernel takes a bf16 forward of these channel counts (the row kernels' range, at most
// 64 input channels, stays theirs).
bool supported(int64_t c_a, int64_t c_b, int64_t c_out);
// Bytes of its packed weights.
size_t packed_bytes(int64_t c_a, int64_t c_b, int64_t c_out);
// Pack the HWIO bf16 weights into wp, then the conv.
int launch(const WideArgs &a, const uint16_t *w_hwio, uint16_t *wp, hipStream_t s);

}  // namespace wide
}  // namespace shpl
