"""Post-fusion 3x3 convolution over the libshpl C ABI.

The reference follows the SHPL with a 3x3 conv on each fused map when
``rpn_sparse_pooling_conv_after_fusion`` is set (default true,
avod/avod/protos/model.proto:88):

    bev = slim.conv2d(bv_fused, feature_depths[0], [3, 3],
                      normalizer_fn=slim.batch_norm,
                      normalizer_params={'is_training': is_training},
                      scope='pyramid_fusion_pooled_bev')        # rpn_model.py:338-346
    img = slim.conv2d(img_fused, feature_depths[1], [3, 3], ...,
                      scope='pyramid_fusion_pooled_img')        # rpn_model.py:347-354

(RetinaNet: ``slim.conv2d(bev_fused, 256, [3, 3])`` with a bias and no BN,
retinanet_model.py:343-348). slim defaults: SAME padding, stride 1, ReLU,
no bias under a normalizer; slim.batch_norm: center (beta), no scale,
epsilon 1e-3, decay 0.999, fused kernel (batch moments when training, moving
averages with the Bessel-corrected variance).

``FusionConv.fused(bev, img, smap)`` computes the BEV conv of
[bev || pool(img)] straight from the img->BEV CSR (shpl_conv3x3 with a
pool CSR): bv_fused never reaches HBM, and the result is bitwise the conv of
the materialised map. The backward (TF autodiff of the same graph) runs on
the device too: BatchNorm/ReLU backward, the input gradient (the same conv
kernel on transposed weights) and the weight gradient (an MFMA reduction over
pixels that recomputes the pooled channels from the CSR), then the SHPL pull
that carries the pooled channels' gradient back to the image map.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L
from . import shpl_map as sm


def conv_ws_bytes(dtype, n_frames, h, w, c_a, c_b, c_out, pool_cap, stats):
    """Workspace of shpl_conv3x3; pool_cap: the pooling CSR's entry capacity
    (``Csr.nnz_cap``), or None without a pool."""
    out = ctypes.c_size_t()
    L.check(L.lib().shpl_conv3x3_workspace_bytes(dtype, int(n_frames), int(h), int(w), int(c_a), int(c_b),
                                                 int(c_out), -1 if pool_cap is None else int(pool_cap),
                                                 int(bool(stats)), ctypes.byref(out)), "shpl_conv3x3_workspace_bytes")
    return out.value


def rows_form(a, weights, b=None, pool=None, frame_off=None, relu=True, stats=False, out=None, c_out=None):
    """Whether conv3x3 with these arguments runs the row-streaming form (shpl_conv3x3_rows_form): only then
    does its workspace hold the pooled operand shpl_conv3x3_wgrad_reuse reads. ``out`` None: a fresh
    contiguous output (16-byte aligned, as torch allocates)."""
    B, H, W, Ca = (int(s) for s in a.shape)
    Cb = 0 if b is None else int(b.shape[-1])
    Cout = int(weights.shape[3]) if c_out is None else int(c_out)
    flag = ctypes.c_int(0)
    out_ptr = L.ptr(out) if out is not None else ctypes.c_void_p(256)  # a stand-in aligned address
    L.check(L.lib().shpl_conv3x3_rows_form(L.dtype_code(a), B, H, W, L.ptr(a), Ca, 0, Ca, L.ptr(b), Cb, 0, Cb,
                                           None if pool is None else pool.ref(), L.ptr(frame_off), L.ptr(weights),
                                           Cout, L.ACT_RELU if relu else L.ACT_NONE, out_ptr,
                                           Cout if out is None else int(out.stride(2)), int(bool(stats)),
                                           ctypes.byref(flag)), "shpl_conv3x3_rows_form")
    return bool(flag.value)


def conv3x3(a, weights, b=None, pool=None, frame_off=None, center=None, scale=None, shift=None, relu=True,
            stats=None, out=None, ws=None):
    """act((conv3x3_SAME([a || b], weights) - center) * scale + shift).

    a: [B,H,W,Ca] NHWC (f32 or bf16); weights: HWIO [3,3,Ca+Cb,Cout] of the
    same dtype; b: a second dense map [B,H,W,Cb], or -- with ``pool`` (the
    cell-keyed ``_lib.Csr`` of an img->BEV map) and ``frame_off`` -- the image
    map [Bi,Hi,Wi,Cb] that is pooled on the fly; stats: optional [2,Cout]
    float64 tensor receiving per-channel sum / sum of squares of the
    pre-epilogue output."""
    dt = L.dtype_code(a)
    a = a if a.is_contiguous() else a.contiguous()
    B, H, W, Ca = (int(s) for s in a.shape)
    Cb = 0
    if b is not None:
        b = b if b.is_contiguous() else b.contiguous()
        if b.dtype != a.dtype:
            raise TypeError("both inputs of the conv must share one dtype")
        Cb = int(b.shape[-1])
        if pool is None and tuple(b.shape[:3]) != (B, H, W):
            raise ValueError(f"dense second input {tuple(b.shape)} does not match {tuple(a.shape)}")
    if weights.dtype != a.dtype:
        weights = weights.to(a.dtype)
    weights = weights.contiguous()
    Cout = int(weights.shape[3])
    if tuple(weights.shape[:3]) != (3, 3, Ca + Cb):
        raise ValueError(f"weights {tuple(weights.shape)} do not match {Ca}+{Cb} input channels")
    if out is None:
        out = torch.empty((B, H, W, Cout), dtype=a.dtype, device=a.device)
    if ws is None:
        ws = L.workspace(conv_ws_bytes(dt, B, H, W, Ca, Cb, Cout, None if pool is None else pool.nnz_cap,
                                       stats is not None), a.device)
    f32 = [None if v is None else v.to(device=a.device, dtype=torch.float32).contiguous()
           for v in (center, scale, shift)]
    L.check(L.lib().shpl_conv3x3(dt, B, H, W, L.ptr(a), Ca, 0, Ca, L.ptr(b), Cb, 0, Cb,
                                 None if pool is None else pool.ref(), L.ptr(frame_off), L.ptr(weights), Cout,
                                 *[L.ptr(v) for v in f32], L.ACT_RELU if relu else L.ACT_NONE, L.ptr(out),
                                 int(out.stride(2)), L.ptr(stats), L.ptr(ws), ws.numel(),
                                 L.stream_of(a.device)), "shpl_conv3x3")
    return out


def batch_norm_train(x, stats, count, eps=1e-3, gamma=None, beta=None, relu=True, moving_mean=None,
                     moving_var=None, decay=0.999, batch_mean=None, batch_var=None, out=None, ws=None):
    """FusedBatchNorm (is_training) of x [..., C] from conv3x3's stats into
    ``out`` (None: in place). ``ws`` (2*C floats) receives the batch mean and
    scale the backward needs."""
    C = int(x.shape[-1])
    rows = x.numel() // C
    if ws is None:
        ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    L.check(L.lib().shpl_batch_norm(L.dtype_code(x), rows, L.ptr(x), L.ptr(out), C, C, L.ptr(stats), float(count),
                                    float(eps), L.ptr(gamma), L.ptr(beta), L.ACT_RELU if relu else L.ACT_NONE,
                                    L.ptr(moving_mean), L.ptr(moving_var), float(decay), L.ptr(batch_mean),
                                    L.ptr(batch_var), L.ptr(ws), L.stream_of(x.device)), "shpl_batch_norm")
    return x if out is None else out


def batch_norm_backward(gy, y=None, raw=None, mean=None, scale=None, gamma=None, relu=True, training=True,
                        beta=None):
    """(g_raw, dbeta, dgamma) of BatchNorm (+ ReLU) over [..., C]; mean / scale
    None -> 0 / 1 (a conv bias: dbeta is the bias gradient). With y None the
    ReLU mask is recomputed from raw (and beta), bitwise the forward's."""
    C = int(gy.shape[-1])
    rows = gy.numel() // C
    out = torch.empty_like(gy)
    dbeta = torch.empty(C, dtype=torch.float32, device=gy.device)
    dgamma = torch.empty(C, dtype=torch.float32, device=gy.device)
    nb = ctypes.c_size_t()
    L.check(L.lib().shpl_batch_norm_backward_workspace_bytes(rows, C, ctypes.byref(nb)),
            "shpl_batch_norm_backward_workspace_bytes")
    ws = L.workspace(nb.value, gy.device)
    L.check(L.lib().shpl_batch_norm_backward(L.dtype_code(gy), rows, L.ptr(y), L.ptr(raw), L.ptr(gy), C, C,
                                             L.ptr(mean), L.ptr(scale), L.ptr(gamma), L.ptr(beta),
                                             L.ACT_RELU if relu else L.ACT_NONE, int(bool(training)), L.ptr(out),
                                             L.ptr(dbeta), L.ptr(dgamma), L.ptr(ws), ws.numel(),
                                             L.stream_of(gy.device)), "shpl_batch_norm_backward")
    return out, dbeta, dgamma


def conv3x3_dgrad(gy, weights, c_dx, split=None, pool=None, fwd_ws=None, fwd_stats=False):
    """Input gradient [B,H,W,c_dx] of the SAME 3x3 conv with HWIO ``weights``;
    with ``split`` = c, the pair (channels [0, c), channels [c, c_dx)) as two
    dense maps written by the kernel's epilogue (no slicing copies). ``fwd_ws`` (with ``pool``, the pooled bf16
    forward's CSR, and ``split``): the workspace of that forward conv3x3 (taken with statistics: fwd_stats),
    whose occupancy words limit the second map to the occupied cells -- the only rows the pixel-keyed pull
    back to the image reads; its other cells are left unwritten (shpl_conv3x3_dgrad_reuse)."""
    gy = gy.contiguous()
    B, H, W, Cg = (int(s) for s in gy.shape)
    weights = weights.to(gy.dtype).contiguous()
    c_dx = int(c_dx)
    c0 = c_dx if split is None else int(split)
    dx = torch.empty((B, H, W, c0), dtype=gy.dtype, device=gy.device)
    dx_b = None if split is None else torch.empty((B, H, W, c_dx - c0), dtype=gy.dtype, device=gy.device)
    ws = L.workspace(conv_ws_bytes(L.dtype_code(gy), B, H, W, Cg, 0, c_dx, None, False), gy.device)
    args = (L.dtype_code(gy), B, H, W, L.ptr(gy), Cg, Cg, L.ptr(weights), c_dx, L.ptr(dx), max(c0, 1), c0,
            L.ptr(dx_b), max(c_dx - c0, 1), L.ptr(ws), ws.numel())
    if fwd_ws is not None:
        L.check(L.lib().shpl_conv3x3_dgrad_reuse(*args, pool.ref(), L.ptr(fwd_ws), fwd_ws.numel(),
                                                 int(bool(fwd_stats)), L.stream_of(gy.device)),
                "shpl_conv3x3_dgrad_reuse")
    else:
        L.check(L.lib().shpl_conv3x3_dgrad(*args, L.stream_of(gy.device)), "shpl_conv3x3_dgrad")
    return dx if split is None else (dx, dx_b)


def conv3x3_wgrad(a, gy, b=None, pool=None, frame_off=None, fwd_ws=None, fwd_stats=False):
    """Weight gradient (f32 HWIO [3,3,Ca+Cb,Cout]) of the SAME 3x3 conv of
    [a || b] (b dense, or the image map pooled through ``pool``). fwd_ws (pooled bf16): the workspace of
    the forward conv3x3 over the same inputs (taken with statistics: fwd_stats), whose pooled operand is
    read instead of prepared again (shpl_conv3x3_wgrad_reuse)."""
    a = a.contiguous()
    gy = gy.contiguous()
    dt = L.dtype_code(a)
    B, H, W, Ca = (int(s) for s in a.shape)
    Cb = 0 if b is None else int(b.shape[-1])
    if b is not None:
        b = b.contiguous()
    Cout = int(gy.shape[-1])
    dw = torch.empty((3, 3, Ca + Cb, Cout), dtype=torch.float32, device=a.device)
    nb = ctypes.c_size_t()
    L.check(L.lib().shpl_conv3x3_wgrad_workspace_bytes(dt, B, H, W, Ca, Cb, Cout, -1 if pool is None else pool.nnz_cap,
                                                       ctypes.byref(nb)), "shpl_conv3x3_wgrad_workspace_bytes")
    ws = L.workspace(nb.value, a.device)
    args = (dt, B, H, W, L.ptr(a), Ca, 0, Ca, L.ptr(b), Cb, 0, Cb, None if pool is None else pool.ref(),
            L.ptr(frame_off), L.ptr(gy), Cout, Cout, L.ptr(dw), L.ptr(ws), ws.numel())
    if fwd_ws is not None:
        L.check(L.lib().shpl_conv3x3_wgrad_reuse(*args, L.ptr(fwd_ws), fwd_ws.numel(), int(bool(fwd_stats)),
                                                 L.stream_of(a.device)), "shpl_conv3x3_wgrad_reuse")
    else:
        L.check(L.lib().shpl_conv3x3_wgrad(*args, L.stream_of(a.device)), "shpl_conv3x3_wgrad")
    return dw


class _FusionConvFn(torch.autograd.Function):
    """FusionConv forward + its TF-autodiff backward, all on the device.
    Inputs: a [B,H,W,Ca]; b: a dense [B,H,W,Cb], or the image map pooled
    through smap (pooled=True), or None; the conv weights; beta / bias."""

    @staticmethod
    def forward(ctx, a, b, weights, beta, bias, conv, smap, pooled, is_training, out):
        a = a.contiguous()
        b = None if b is None else b.contiguous()
        B, H, W, Ca = (int(s) for s in a.shape)
        Cb = 0 if b is None else int(b.shape[-1])
        dt = L.dtype_code(a)
        pool = smap.csr(L.BY_CELL, L.ORDER_ENTRY) if pooled else None
        frame_off = smap.frame_off if pooled else None
        train_bn = conv.batch_norm and is_training
        if pooled and ctx.needs_input_grad[1]:  # the image gradient's pixel-keyed CSR sorts beside the forward
            smap.prefetch_csr(L.BY_PIXEL, L.ORDER_COL_ENTRY)
        xb, b_img = None, b
        if pooled and train_bn and ctx.needs_input_grad[2] and a.dtype != torch.bfloat16:
            # f32: the weight gradient needs the pooled channels in HBM (see backward): pooled here, once, the
            # forward is the dense two-source conv (bf16 pools inside both convs: k_conv_rows / k_wgrad_rows)
            xb = sm.pool_img_to_bev(smap, b, (B, H, W, Cb))
            b, pool, frame_off = xb, None, None
        cap = pool.nnz_cap if pool is not None else None
        # bf16 pooled with a weight gradient to come: a workspace of this call's own, kept for the backward,
        # whose weight gradient reads the pooled operand the forward prepared in it (shpl_conv3x3_wgrad_reuse)
        # -- only when the forward runs the row-streaming form, which is what leaves that operand there
        reuse = (pooled and conv.WGRAD_REUSE and a.dtype == torch.bfloat16 and ctx.needs_input_grad[2] and
                 rows_form(a, weights.to(a.dtype), b=b, pool=pool, frame_off=frame_off,
                           relu=conv.relu if not train_bn else False, stats=train_bn,
                           out=out if not train_bn else None, c_out=conv.c_out))
        nbytes = conv_ws_bytes(dt, B, H, W, Ca, Cb, conv.c_out, cap, train_bn)
        ws = L.workspace(nbytes, a.device) if reuse else conv._ws_for((dt, B, H, W, Cb, cap, train_bn), nbytes)
        ctx.fwd_ws = ws if reuse else None
        raw, mean, scale = None, None, None
        if not train_bn:
            center, scale, shift = conv._inference_epilogue()
            if scale is not None:  # saved for the backward: a copy, not the buffer a training step rewrites
                scale = scale.clone()
            mean = center
            if not conv.batch_norm:
                shift = bias
            y = conv3x3(a, weights, b=b, pool=pool, frame_off=frame_off, center=center, scale=scale, shift=shift,
                        relu=conv.relu, out=out, ws=ws)
        else:
            stats = torch.empty((2, conv.c_out), dtype=torch.float64, device=a.device)
            raw = conv3x3(a, weights, b=b, pool=pool, frame_off=frame_off, relu=False, stats=stats, ws=ws)
            bn_ws = torch.empty(2 * conv.c_out, dtype=torch.float32, device=a.device)
            y = out if out is not None else torch.empty_like(raw)
            batch_norm_train(raw, stats, B * H * W, eps=conv.eps, beta=beta, relu=conv.relu,
                             moving_mean=conv.moving_mean, moving_var=conv.moving_var, decay=conv.decay, out=y,
                             ws=bn_ws)
            conv._refresh_scale()  # the moving statistics were updated through their device pointers
            mean, scale = bn_ws[:conv.c_out], bn_ws[conv.c_out:]
        ctx.conv, ctx.smap, ctx.pooled, ctx.train_bn = conv, smap, pooled, train_bn
        ctx.shapes = (Ca, Cb)
        ctx.xb = xb
        b = b_img
        # training BN: the backward recomputes the ReLU mask from raw and beta (bitwise y's), so y is not kept
        ctx.save_for_backward(a, b, weights, None if train_bn else y, raw, mean, scale,
                              beta if train_bn else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        a, b, weights, y, raw, mean, scale, beta = ctx.saved_tensors
        conv, smap, pooled = ctx.conv, ctx.smap, ctx.pooled
        Ca, Cb = ctx.shapes
        gy = gy.contiguous().to(a.dtype)
        if conv.batch_norm or conv.bias is not None or conv.relu:
            g_raw, dbeta, _ = batch_norm_backward(
                gy, y=y, raw=raw, mean=mean if (conv.batch_norm or ctx.train_bn) else None,
                scale=scale if conv.batch_norm else None, relu=conv.relu, training=ctx.train_bn, beta=beta)
        else:
            g_raw, dbeta = gy, None
        need_x = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        d_a = d_b = dw = None
        # side stream work beside the input gradient (FusionConv.IMG_ZERO_SIDE / WGRAD_SIDE): the image
        # gradient's zero rows (they need no index and no input gradient), then the weight gradient (it reads the
        # same g_raw as the input gradient and writes a disjoint output)
        side = zeros_done = None
        img_grad = need_x and pooled and b is not None and ctx.needs_input_grad[1]
        zero_side = img_grad and conv.IMG_ZERO_SIDE
        wgrad_side = need_x and ctx.needs_input_grad[2] and conv.WGRAD_SIDE
        # IMG_BESIDE_WGRAD: the image gradient (zero rows, then the pull) on the side stream after the input
        # gradient, beside the weight gradient, instead of its zero rows beside the input gradient
        late_zero = (zero_side and conv.IMG_BESIDE_WGRAD and ctx.needs_input_grad[2] and not wgrad_side and
                     g_raw.is_cuda)
        if g_raw.is_cuda and ((zero_side and not late_zero) or wgrad_side):
            cur = torch.cuda.current_stream(g_raw.device)
            side = _side_stream(g_raw.device)
            side.wait_stream(cur)
            if zero_side:
                d_b = torch.empty(b.shape, dtype=a.dtype, device=a.device)
            with torch.cuda.stream(side):
                if zero_side:
                    # (the dense half reads no source rows: any aligned map stands in for dx_b, not written yet)
                    sm.pull(smap, L.BY_PIXEL, L.ORDER_COL_ENTRY, d_b, Cb, 0, Cb, d_b, Cb, part="dense")
                    zeros_done = torch.cuda.Event()
                    zeros_done.record(side)
                if wgrad_side:
                    dw = _FusionConvFn._wgrad(ctx, a, b, weights, g_raw)
            for t in (a, b, g_raw, ctx.fwd_ws, ctx.xb, d_b):
                if t is not None:
                    t.record_stream(side)
        if need_x:
            if b is None:
                d_a = conv3x3_dgrad(g_raw, weights, Ca)
            else:  # the epilogue writes the two sources' gradients as separate dense maps
                occ = pooled and ctx.fwd_ws is not None and conv.DGRAD_OCC and ctx.needs_input_grad[1]
                d_a, dx_b = conv3x3_dgrad(g_raw, weights, Ca + Cb, split=Ca,
                                          pool=smap.csr(L.BY_CELL, L.ORDER_ENTRY) if occ else None,
                                          fwd_ws=ctx.fwd_ws if occ else None, fwd_stats=ctx.train_bn)
                if ctx.needs_input_grad[1]:
                    if late_zero:
                        cur = torch.cuda.current_stream(g_raw.device)
                        side = _side_stream(g_raw.device)
                        side.wait_stream(cur)
                        d_b = torch.empty(b.shape, dtype=a.dtype, device=a.device)
                        with torch.cuda.stream(side):
                            sm.pull(smap, L.BY_PIXEL, L.ORDER_COL_ENTRY, d_b, Cb, 0, Cb, d_b, Cb, part="dense")
                            sm.pull(smap, L.BY_PIXEL, L.ORDER_COL_ENTRY, dx_b, Cb, 0, Cb, d_b, Cb, part="sparse")
                        for t in (dx_b, d_b):
                            t.record_stream(side)
                    elif pooled and zeros_done is not None:  # its zero rows are on the side stream already
                        cur.wait_event(zeros_done)
                        sm.pull(smap, L.BY_PIXEL, L.ORDER_COL_ENTRY, dx_b, Cb, 0, Cb, d_b, Cb, part="sparse")
                    elif pooled:  # the pooled channels' gradient back to the image (a8's TF gradient)
                        d_b = torch.empty(b.shape, dtype=dx_b.dtype, device=dx_b.device)
                        sm.pull(smap, L.BY_PIXEL, L.ORDER_COL_ENTRY, dx_b, Cb, 0, Cb, d_b, Cb)
                    else:
                        d_b = dx_b
            if not ctx.needs_input_grad[0]:
                d_a = None
        if side is not None:
            if late_zero and dw is None and ctx.needs_input_grad[2]:  # on the main stream, beside the side's work
                dw = _FusionConvFn._wgrad(ctx, a, b, weights, g_raw)
            cur.wait_stream(side)
            if dw is not None and not late_zero:
                dw.record_stream(cur)
        if dw is None and ctx.needs_input_grad[2]:
            dw = _FusionConvFn._wgrad(ctx, a, b, weights, g_raw)
        d_beta = dbeta if (conv.batch_norm and ctx.needs_input_grad[3]) else None
        d_bias = dbeta if (not conv.batch_norm and ctx.needs_input_grad[4]) else None
        return d_a, d_b, dw, d_beta, d_bias, None, None, None, None, None

    @staticmethod
    def _wgrad(ctx, a, b, weights, g_raw):
        smap, pooled = ctx.smap, ctx.pooled
        if pooled and a.dtype == torch.bfloat16:
            # k_wgrad_rows gathers the pooled rows from a compact per-run buffer: bv_fused never stored
            dw = conv3x3_wgrad(a, g_raw, b=b, pool=smap.csr(L.BY_CELL, L.ORDER_ENTRY), frame_off=smap.frame_off,
                               fwd_ws=ctx.fwd_ws, fwd_stats=ctx.train_bn)
        elif pooled:
            # f32: the pooled channels once into HBM (shpl_pull): the dense two-source weight gradient
            # runs at twice the waves per SIMD of the one that recomputes them per tile (257 vs
            # 214 registers); conv3x3_wgrad(..., pool=...) stays the memory-lean form
            xb = ctx.xb if ctx.xb is not None else sm.pool_img_to_bev(smap, b, tuple(a.shape[:3]) + (ctx.shapes[1],))
            dw = conv3x3_wgrad(a, g_raw, b=xb)
        else:
            dw = conv3x3_wgrad(a, g_raw, b=b)
        return dw.to(weights.dtype)


_SIDE = {}


def _side_stream(dev):
    """One side stream per device for the weight gradient (created once: stream creation is not free)."""
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


class FusionConv:
    """slim.conv2d(x, c_out, [3,3]) with slim.batch_norm (or a bias) and ReLU:
    the variables of one ``pyramid_fusion_pooled_*`` scope and its forward."""

    # bf16 fused(): the weight gradient reads the pooled operand its forward prepared (False: prepares its own)
    WGRAD_REUSE = True
    # backward, beside the input gradient on a side stream: the image gradient's zero rows (IMG_ZERO_SIDE) and
    # the weight gradient (WGRAD_SIDE; False: after the input gradient on one stream -- the two convs side by
    # side measured slower: 7.34-7.35 vs 7.14-7.20 ms per bf16 training step, profiles/r05_wside_ab.log)
    IMG_ZERO_SIDE = True
    WGRAD_SIDE = False
    # bf16 fused() backward: the input gradient's pooled channels stored at the occupied cells only, by the
    # forward's occupancy words (shpl_conv3x3_dgrad_reuse; False: the whole map, shpl_conv3x3_dgrad)
    DGRAD_OCC = True
    # the image gradient (zero rows, then the pull of the pooled channels' gradient) on the side stream after the
    # input gradient, beside the weight gradient (False: only its zero rows, beside the input gradient): 6.93-7.00
    # against 6.98-7.04 ms per bf16 training step, interleaved (profiles/r06_ab/beside_*)
    IMG_BESIDE_WGRAD = True

    def __init__(self, c_in, c_out, batch_norm=True, bias=False, relu=True, eps=1e-3, decay=0.999,
                 dtype=torch.float32, device="cuda", seed=0):
        g = np.random.default_rng(seed)
        # xavier_initializer (uniform), slim.conv2d's default weights_initializer
        lim = float(np.sqrt(6.0 / (9 * c_in + 9 * c_out)))
        w = g.uniform(-lim, lim, size=(3, 3, c_in, c_out)).astype(np.float32)
        self.c_in, self.c_out = int(c_in), int(c_out)
        self.device, self.dtype = torch.device(device), dtype
        self.weights = torch.from_numpy(w).to(self.device, dtype)
        self.batch_norm, self.relu, self.eps, self.decay = batch_norm, relu, float(eps), float(decay)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.beta = torch.zeros(c_out, **f32) if batch_norm else None
        self.moving_mean = torch.zeros(c_out, **f32) if batch_norm else None
        self.moving_var = torch.ones(c_out, **f32) if batch_norm else None
        self.bias = torch.zeros(c_out, **f32) if (bias and not batch_norm) else None
        self._ws = {}
        self._scale = torch.empty(c_out, **f32) if batch_norm else None
        if batch_norm:
            self._refresh_scale()

    def _inference_epilogue(self):
        if not self.batch_norm:
            return None, None, self.bias
        # FusedBatchNorm inference: (x - moving_mean) * rsqrt(moving_var + eps) + beta. The scale lives in one
        # tensor, rewritten ON THE DEVICE right after every batch_norm_train (which updates moving_var through
        # its device pointer, bumping no tensor version), so a training step replayed from a captured graph
        # refreshes it too, and an inference graph reads the current one; an eager in-place update of moving_var
        # (its version) refreshes it here. An inference step launches nothing for it.
        if self._scale_key != (self.moving_var.data_ptr(), self.moving_var._version, self.eps):
            self._refresh_scale()
        return self.moving_mean, self._scale, self.beta

    def _refresh_scale(self):
        """self._scale = 1 / sqrt(moving_var + eps), in place (three launches, stream-ordered, capturable)."""
        torch.add(self.moving_var, self.eps, out=self._scale)
        self._scale.sqrt_().reciprocal_()
        self._scale_key = (self.moving_var.data_ptr(), self.moving_var._version, self.eps)

    def _ws_for(self, key, nbytes):
        t = self._ws.get(key)
        if t is None or t.numel() < nbytes:
            t = L.workspace(nbytes, self.device)
            self._ws[key] = t
        return t

    def _run(self, a, b, pool, frame_off, is_training, out):
        B, H, W = (int(s) for s in a.shape[:3])
        Cb = 0 if b is None else int(b.shape[-1])
        dt = L.dtype_code(a)
        train_bn = self.batch_norm and is_training
        cap = None if pool is None else pool.nnz_cap
        ws = self._ws_for((dt, B, H, W, Cb, cap, train_bn),
                          conv_ws_bytes(dt, B, H, W, int(a.shape[-1]), Cb, self.c_out, cap, train_bn))
        if not train_bn:
            center, scale, shift = self._inference_epilogue()
            return conv3x3(a, self.weights, b=b, pool=pool, frame_off=frame_off, center=center, scale=scale,
                           shift=shift, relu=self.relu, out=out, ws=ws)
        stats = torch.empty((2, self.c_out), dtype=torch.float64, device=a.device)
        y = conv3x3(a, self.weights, b=b, pool=pool, frame_off=frame_off, relu=False, stats=stats, out=out, ws=ws)
        y = batch_norm_train(y, stats, B * H * W, eps=self.eps, beta=self.beta, relu=self.relu,
                             moving_mean=self.moving_mean, moving_var=self.moving_var, decay=self.decay)
        self._refresh_scale()  # batch_norm_train updated the moving statistics through their device pointers
        return y

    def _grad_wanted(self, *tensors):
        return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in
                                               (*tensors, self.weights, self.beta, self.bias))

    def __call__(self, x, is_training=False, out=None):
        """The conv of a materialised map (bv_fused, img_fused, or img)."""
        if self._grad_wanted(x):
            return _FusionConvFn.apply(x, None, self.weights, self.beta, self.bias, self, None, False, is_training,
                                       out)
        return self._run(x, None, None, None, is_training, out)

    def fused(self, bev, img, smap, is_training=False, out=None):
        """The conv of [bev || _sparse_pool_op(M, img)] without writing the
        concat: ``smap`` is the ShplMap of the frames of ``bev``. Differentiable
        in bev, img, the weights and beta / bias."""
        if self._grad_wanted(bev, img):
            return _FusionConvFn.apply(bev, img, self.weights, self.beta, self.bias, self, smap, True, is_training,
                                       out)
        return self.fused_csr(bev, img, smap.csr(L.BY_CELL, L.ORDER_ENTRY), smap.frame_off, is_training, out)

    def fused_csr(self, bev, img, csr, frame_off, is_training=False, out=None):
        """fused() over an already built cell-keyed CSR (``_lib.Csr``) and the
        per-frame entry slots ``frame_off`` (FusedPipeline.csr / .frame_off);
        forward only."""
        return self._run(bev, img, csr, frame_off, is_training, out)
