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
the materialised map. Forward only: there is no autograd rule yet.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L


def conv_ws_bytes(dtype, n_frames, h, w, c_a, c_b, c_out, pooled, stats):
    out = ctypes.c_size_t()
    L.check(L.lib().shpl_conv3x3_workspace_bytes(dtype, int(n_frames), int(h), int(w), int(c_a), int(c_b),
                                                 int(c_out), int(bool(pooled)), int(bool(stats)),
                                                 ctypes.byref(out)), "shpl_conv3x3_workspace_bytes")
    return out.value


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
        ws = L.workspace(conv_ws_bytes(dt, B, H, W, Ca, Cb, Cout, pool is not None, stats is not None), a.device)
    f32 = [None if v is None else v.to(device=a.device, dtype=torch.float32).contiguous()
           for v in (center, scale, shift)]
    L.check(L.lib().shpl_conv3x3(dt, B, H, W, L.ptr(a), Ca, 0, Ca, L.ptr(b), Cb, 0, Cb,
                                 None if pool is None else pool.ref(), L.ptr(frame_off), L.ptr(weights), Cout,
                                 *[L.ptr(v) for v in f32], L.ACT_RELU if relu else L.ACT_NONE, L.ptr(out),
                                 int(out.stride(2)), L.ptr(stats), L.ptr(ws), ws.numel(),
                                 L.stream_of(a.device)), "shpl_conv3x3")
    return out


def batch_norm_train(x, stats, count, eps=1e-3, gamma=None, beta=None, relu=True, moving_mean=None,
                     moving_var=None, decay=0.999, batch_mean=None, batch_var=None):
    """In-place FusedBatchNorm (is_training) of x [..., C] from conv3x3's stats."""
    C = int(x.shape[-1])
    rows = x.numel() // C
    ws = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    L.check(L.lib().shpl_batch_norm(L.dtype_code(x), rows, L.ptr(x), C, C, L.ptr(stats), float(count), float(eps),
                                    L.ptr(gamma), L.ptr(beta), L.ACT_RELU if relu else L.ACT_NONE,
                                    L.ptr(moving_mean), L.ptr(moving_var), float(decay), L.ptr(batch_mean),
                                    L.ptr(batch_var), L.ptr(ws), L.stream_of(x.device)), "shpl_batch_norm")
    return x


class FusionConv:
    """slim.conv2d(x, c_out, [3,3]) with slim.batch_norm (or a bias) and ReLU:
    the variables of one ``pyramid_fusion_pooled_*`` scope and its forward."""

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

    def _inference_epilogue(self):
        if not self.batch_norm:
            return None, None, self.bias
        # FusedBatchNorm inference: (x - moving_mean) * rsqrt(moving_var + eps) + beta
        scale = 1.0 / torch.sqrt(self.moving_var + self.eps)
        return self.moving_mean, scale, self.beta

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
        ws = self._ws_for((dt, B, H, W, Cb, pool is not None, train_bn),
                          conv_ws_bytes(dt, B, H, W, int(a.shape[-1]), Cb, self.c_out, pool is not None, train_bn))
        if not train_bn:
            center, scale, shift = self._inference_epilogue()
            return conv3x3(a, self.weights, b=b, pool=pool, frame_off=frame_off, center=center, scale=scale,
                           shift=shift, relu=self.relu, out=out, ws=ws)
        stats = torch.empty((2, self.c_out), dtype=torch.float64, device=a.device)
        y = conv3x3(a, self.weights, b=b, pool=pool, frame_off=frame_off, relu=False, stats=stats, out=out, ws=ws)
        return batch_norm_train(y, stats, B * H * W, eps=self.eps, beta=self.beta, relu=self.relu,
                                moving_mean=self.moving_mean, moving_var=self.moving_var, decay=self.decay)

    def __call__(self, x, is_training=False, out=None):
        """The conv of a materialised map (bv_fused, img_fused, or img)."""
        return self._run(x, None, None, None, is_training, out)

    def fused(self, bev, img, smap, is_training=False, out=None):
        """The conv of [bev || _sparse_pool_op(M, img)] without writing the
        concat: ``smap`` is the ShplMap of the frames of ``bev``."""
        return self.fused_csr(bev, img, smap.csr(L.BY_CELL, L.ORDER_ENTRY), smap.frame_off, is_training, out)

    def fused_csr(self, bev, img, csr, frame_off, is_training=False, out=None):
        """fused() over an already built cell-keyed CSR (``_lib.Csr``) and the
        per-frame entry slots ``frame_off`` (FusedPipeline.csr / .frame_off)."""
        return self._run(bev, img, csr, frame_off, is_training, out)
