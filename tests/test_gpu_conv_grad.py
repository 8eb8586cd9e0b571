"""Backward of the post-fusion conv (shpl_conv3x3_dgrad / _wgrad,
shpl_batch_norm_backward, FusionConv autograd) vs the CPU oracle on MI355X.

Tolerances as in test_gpu_conv.py: 1e-5 plus the f32 summation error of the
products involved, 2^-19 * sum |a*b| for the 9*C-term dot products of the
input gradient, 2^-16 * sum |x*g| for the weight gradient (a reduction over
every pixel of the batch, summed in f32 per workgroup and in f64 across
workgroups). The oracle (double sums) is cross-checked against torch's CPU
autograd in tests/test_oracle_conv.py.
"""
import numpy as np
import pytest
import torch

from oracle import shpl_oracle as orc
from sparse_pooling_amd import synth

pytestmark = pytest.mark.gpu

TOL = 1e-5
ACC = 2.0 ** -19
ACC_W = 2.0 ** -16
DEV = "cuda"


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _weights(cin, cout, seed):
    rng = np.random.default_rng(seed)
    lim = np.sqrt(6.0 / (9 * cin + 9 * cout))
    return (3.0 * rng.uniform(-lim, lim, (3, 3, cin, cout))).astype(np.float32)


def _check(got, ref, bound, what):
    err = np.abs(_np(got).astype(np.float64) - ref)
    assert (err <= bound).all(), (what, float(err.max()), float((err / bound).max()))


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_pooling_amd import _lib as L
    L.lib()
    assert torch.cuda.is_available()


@pytest.mark.parametrize("shape", [(2, 9, 35, 24, 33), (1, 16, 64, 64, 32), (1, 3, 5, 5, 7)])
def test_dgrad_and_wgrad_dense(shape):
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = shape
    x = synth.make_features((B, H, W, Cin), 1)
    w = _weights(Cin, Cout, 2)
    g = synth.make_features((B, H, W, Cout), 3)
    dx = fc.conv3x3_dgrad(_t(g), _t(w), Cin)
    wt = np.ascontiguousarray(w[::-1, ::-1].transpose(0, 1, 3, 2))
    _, ab = orc.conv3x3(np.abs(g), np.abs(wt), raw=True)
    _check(dx, orc.conv3x3_dgrad(g, w), TOL + ACC * ab, "dx")
    # the two-output epilogue (the gradients of the conv's two sources) == one map, split
    c = Cin // 3
    da, db = fc.conv3x3_dgrad(_t(g), _t(w), Cin, split=c)
    assert da.shape[-1] == c and db.shape[-1] == Cin - c
    assert torch.equal(torch.cat([da, db], -1), dx)
    dw = fc.conv3x3_wgrad(_t(x), _t(g))
    _check(dw, orc.conv3x3_wgrad(x, g), TOL + ACC_W * orc.conv3x3_wgrad(np.abs(x), np.abs(g)), "dw")


def test_dgrad_and_wgrad_bf16():
    """bf16 storage: products of bf16 values are exact in f32, so the weight
    gradient keeps the f32 bound; the input gradient is stored in bf16 (plus
    half a bf16 ulp of the result: 2^-8 relative, 7 stored mantissa bits)."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = 2, 11, 37, 48, 32
    bf = lambda a: torch.from_numpy(a).to(torch.bfloat16)  # noqa: E731
    x = bf(synth.make_features((B, H, W, Cin), 41))
    w = bf(_weights(Cin, Cout, 42))
    g = bf(synth.make_features((B, H, W, Cout), 43))
    xf, wf, gf = (t.float().numpy() for t in (x, w, g))
    dx = fc.conv3x3_dgrad(g.to(DEV), w.to(DEV), Cin)
    assert dx.dtype == torch.bfloat16
    ref = orc.conv3x3_dgrad(gf, wf)
    wt = np.ascontiguousarray(wf[::-1, ::-1].transpose(0, 1, 3, 2))
    _, ab = orc.conv3x3(np.abs(gf), np.abs(wt), raw=True)
    _check(dx.float(), ref, TOL + ACC * ab + 2.0 ** -8 * np.abs(ref), "dx bf16")
    dw = fc.conv3x3_wgrad(x.to(DEV), g.to(DEV))
    _check(dw, orc.conv3x3_wgrad(xf, gf), TOL + ACC_W * orc.conv3x3_wgrad(np.abs(xf), np.abs(gf)), "dw bf16")


@pytest.mark.parametrize("shape,split", [((2, 16, 64, 32, 64), 32), ((1, 61, 70, 32, 64), 32),
                                         ((2, 9, 35, 32, 64), 16)])
def test_dgrad_bf16_two_maps(shape, split):
    """The bf16 input gradient of a 64-channel input from a 32-channel output
    gradient (the training workload's): k_conv_rows with two output blocks
    (blocks fastest in the item order, one per map when the split is at 32),
    vs the oracle within the bf16 bound; both maps bitwise the one-map form
    (a split inside an output block takes the tiled kernel: oracle bound only)."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cout, Cin = shape
    bf = lambda a: torch.from_numpy(a).to(torch.bfloat16)  # noqa: E731
    w = bf(_weights(Cin, Cout, 52))
    g = bf(synth.make_features((B, H, W, Cout), 53))
    wf, gf = (t.float().numpy() for t in (w, g))
    ref = orc.conv3x3_dgrad(gf, wf)
    wt = np.ascontiguousarray(wf[::-1, ::-1].transpose(0, 1, 3, 2))
    _, ab = orc.conv3x3(np.abs(gf), np.abs(wt), raw=True)
    bound = TOL + ACC * ab + 2.0 ** -8 * np.abs(ref)
    dx = fc.conv3x3_dgrad(g.to(DEV), w.to(DEV), Cin)
    _check(dx.float(), ref, bound, "dx bf16")
    da, db = fc.conv3x3_dgrad(g.to(DEV), w.to(DEV), Cin, split=split)
    _check(torch.cat([da, db], -1).float(), ref, bound, "dx bf16 split")
    if split % 32 == 0:
        assert torch.equal(torch.cat([da, db], -1), dx)


WGRAD_ROWS = [  # B, H, W, c_a, c_b, c_out: bf16 dense weight gradients on k_wgrad_rows
    (2, 16, 64, 32, 32, 32),   # the training workload's two sources
    (1, 130, 70, 64, 0, 64),   # three bands, a partial strip, two output tiles
    (3, 9, 33, 16, 0, 40),     # channel tails in both tiles (16 of 32 inputs, 8 of the second 32 outputs)
    (1, 61, 32, 32, 16, 32),   # one band of 61 rows; B's tile is a tail
    (1, 1, 1, 32, 0, 32),      # one pixel: every halo pixel and row outside the map
    (2, 2, 3, 8, 0, 8),        # 8-channel tiles, two frames of 2 rows
]


@pytest.mark.parametrize("shape", WGRAD_ROWS, ids=[str(s) for s in WGRAD_ROWS])
def test_wgrad_bf16_rows(shape):
    """k_wgrad_rows (transposed LDS reads of the NHWC rows, the 9 taps'
    accumulators resident over a run of bands, two fixed-order f64 reductions)
    vs the oracle's double sums: bf16 products are exact, so the f32 bound
    holds; two sources == their concat bitwise when A ends on a 32-channel tile."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, ca, cb, co = shape
    bf = lambda a: torch.from_numpy(a).to(torch.bfloat16)  # noqa: E731
    x = bf(synth.make_features((B, H, W, ca + cb), 71))
    g = bf(synth.make_features((B, H, W, co), 72))
    xf, gf = x.float().numpy(), g.float().numpy()
    bound = TOL + ACC_W * orc.conv3x3_wgrad(np.abs(xf), np.abs(gf))
    dw = fc.conv3x3_wgrad(x.to(DEV), g.to(DEV))
    _check(dw, orc.conv3x3_wgrad(xf, gf), bound, "dw bf16 rows")
    if cb > 0:
        xa = x[..., :ca].contiguous().to(DEV)
        xb = x[..., ca:].contiguous().to(DEV)
        dw2 = fc.conv3x3_wgrad(xa, g.to(DEV), b=xb)
        assert torch.equal(dw2, dw)


def test_fused_conv_training_bf16_rows():
    """bf16 FusionConv.fused in training (the bench's --train --dtype bf16 form
    at config-1 geometry, 32 + 32 -> 32 channels): the pooled map is built once
    in the forward and the conv runs dense on k_conv_rows with the statistics
    epilogue; output and every gradient bitwise those of the same autograd
    graph over the materialised bv_fused (conv(bv_fused) with the pooled
    channels' gradient pulled back to the image), and the output within the
    bf16 bound of the oracle chain."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    spec = synth.CONFIGS[1]
    fr = synth.make_frame(spec, seed=910, n_outside=10)
    gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                            tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb = Ci = 32
    bf = lambda a: torch.from_numpy(a).to(torch.bfloat16)  # noqa: E731
    bev = bf(synth.make_features((1, Hb, Wb, Cb), 21)).to(DEV)
    img = bf(synth.make_features((1, Hi, Wi, Ci), 22)).to(DEV)
    w = bf(_weights(Cb + Ci, Ci, 23)).to(DEV)
    g = bf(np.random.default_rng(24).standard_normal((1, Hb, Wb, Ci)).astype(np.float32)).to(DEV)
    smap = sm.pack_map(_t(ref["Mij_pool"]), _t(ref["M_val"].astype(np.float32)), ref["M_size"],
                       _t(ref["img_index_flip_pool"]), tuple(img.shape))
    beta = _t((0.1 * np.random.default_rng(25).standard_normal(Ci)).astype(np.float32))

    def run(fused):
        conv = fc.FusionConv(Cb + Ci, Ci, dtype=torch.bfloat16, device=DEV)
        conv.weights = w.clone().requires_grad_(True)
        conv.beta = beta.clone().requires_grad_(True)
        tb, ti = bev.clone().requires_grad_(True), img.clone().requires_grad_(True)
        if fused:
            y = conv.fused(tb, ti, smap, is_training=True)
        else:
            y = conv(sm.layer(tb, ti, smap)[0], is_training=True)
        y.backward(g)
        return y, tb.grad, ti.grad, conv.weights.grad, conv.beta.grad, conv.moving_mean, conv.moving_var

    got, want = run(True), run(False)
    for name, u, v in zip(("y", "d_bev", "d_img", "d_w", "d_beta", "moving_mean", "moving_var"), got, want):
        assert torch.equal(u, v), name
    eb, _ = orc.sparse_pool_layer(bev.float().cpu().numpy(), img.float().cpu().numpy(), ref["Mij_pool"],
                                  ref["M_val"], ref["M_size"], ref["img_index_flip_pool"])
    eb = orc.from_bf16_bits(orc.to_bf16_bits(eb))
    _, raw = orc.conv3x3(eb, w.float().cpu().numpy(), raw=True)
    ey, _, bvar, _, _ = orc.batch_norm_train(raw, 1e-3, None, beta.cpu().numpy(), True)
    _check(got[0].float(), ey, 1e-2 + 2.0 ** -7 * np.abs(ey), "y bf16")


def test_wgrad_two_sources_and_pooled():
    """wgrad of [a || b] with b dense, and with b pooled from the CSR (the
    pooled channels recomputed in the staging), == wgrad of the concat."""
    from sparse_pooling_amd import fusion_conv as fc, pipeline, shpl_map as sm
    spec = synth.CONFIGS[1]
    frames = [synth.make_frame(spec, seed=700 + f, n_outside=10) for f in range(2)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    ib = sm.build_index_batch(pts, vox, off, P, spec.im_size, spec.bv_size, spec.stride, maxp)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = synth.make_features((2, Hb, Wb, 16), 4)
    img = synth.make_features((2, Hi, Wi, 12), 5)
    g = synth.make_features((2, Hb, Wb, 40), 6)
    bv = sm.pool_img_to_bev(ib.map, _t(img), (2, Hb, Wb, 16), bev=_t(bev))
    x = _np(bv)
    ref = orc.conv3x3_wgrad(x, g)
    bound = TOL + ACC_W * orc.conv3x3_wgrad(np.abs(x), np.abs(g))
    _check(fc.conv3x3_wgrad(_t(x), _t(g)), ref, bound, "concat")
    _check(fc.conv3x3_wgrad(_t(bev), _t(g), b=_t(x[..., 16:])), ref, bound, "two dense")
    pooled = fc.conv3x3_wgrad(_t(bev), _t(g), b=_t(img), pool=ib.map.csr(0, 0), frame_off=ib.map.frame_off)
    _check(pooled, ref, bound, "pooled")


@pytest.mark.parametrize("training,C", [(True, 40), (False, 40), (True, 7), (False, 7)])
def test_batch_norm_backward(training, C):
    """C = 40: the 16-byte vector kernels; C = 7: the scalar ones."""
    from sparse_pooling_amd import fusion_conv as fc
    rng = np.random.default_rng(7)
    raw = (rng.standard_normal((3, 11, 13, C)) * 2.0 + 0.5).astype(np.float32)
    g = rng.standard_normal(raw.shape).astype(np.float32)
    beta = rng.standard_normal(C).astype(np.float32)
    if training:
        mean = raw.reshape(-1, C).astype(np.float64).mean(0)
        var = raw.reshape(-1, C).astype(np.float64).var(0)
    else:
        mean = rng.standard_normal(C)
        var = rng.uniform(0.5, 2.0, C)
    scale = (1.0 / np.sqrt(var + 1e-3)).astype(np.float32)
    y = np.maximum((raw - mean) * scale + beta, 0.0).astype(np.float32)
    gr, db, _ = fc.batch_norm_backward(_t(g), y=_t(y), raw=_t(raw), mean=_t(mean.astype(np.float32)),
                                       scale=_t(scale), relu=True, training=training)
    e_raw, e_db, _ = orc.batch_norm_backward(raw.astype(np.float64), g, training, mean, var, 1e-3, None, beta, True)
    # values of order |scale * g|; the training form subtracts two O(1) means in f32
    _check(gr, e_raw, 1e-5 + 1e-5 * np.abs(scale) * (np.abs(g) + 1.0), "g_raw")
    _check(db, e_db, 1e-4 + 1e-6 * np.abs(g).reshape(-1, C).sum(0), "dbeta")
    # the ReLU mask recomputed from raw (y not read) with the forward's rounding, (raw - mean) * scale + beta
    # one rounded op at a time (as torch's separate kernels do): bitwise the same result as reading y
    t_raw, t_mean, t_scale, t_beta = _t(raw), _t(mean.astype(np.float32)), _t(scale), _t(beta)
    y_dev = torch.clamp_min((t_raw - t_mean) * t_scale + t_beta, 0.0)
    a1 = fc.batch_norm_backward(_t(g), y=y_dev, raw=t_raw, mean=t_mean, scale=t_scale, relu=True, training=training)
    a2 = fc.batch_norm_backward(_t(g), y=None, raw=t_raw, mean=t_mean, scale=t_scale, relu=True, training=training,
                                beta=t_beta)
    for u, v in zip(a1, a2):
        assert torch.equal(u, v)


@pytest.mark.parametrize("train", [True, False])
def test_fused_conv_autograd_vs_oracle(train):
    """d(bev), d(img), d(weights), d(beta) of FusionConv.fused (pooling inside
    the conv) against the oracle chain: pooled map -> conv -> BatchNorm ->
    ReLU forward, and its TF gradients (BN / conv backward, then the
    gradient of _sparse_pool_op for the image)."""
    from sparse_pooling_amd import fusion_conv as fc, pipeline, shpl_map as sm
    spec = synth.CONFIGS[1]
    fr = synth.make_frame(spec, seed=900, n_outside=10)
    gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                            tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img
    bev = synth.make_features((1, Hb, Wb, Cb), 11)
    img = synth.make_features((1, Hi, Wi, Ci), 12)
    w = _weights(Cb + Ci, Ci, 13)
    rng = np.random.default_rng(14)
    beta = (0.1 * rng.standard_normal(Ci)).astype(np.float32)
    mm = (0.1 * rng.standard_normal(Ci)).astype(np.float32)
    mv = rng.uniform(0.5, 2.0, Ci).astype(np.float32)
    g = rng.standard_normal((1, Hb, Wb, Ci)).astype(np.float32)
    smap = sm.pack_map(_t(ref["Mij_pool"]), _t(ref["M_val"].astype(np.float32)), ref["M_size"],
                       _t(ref["img_index_flip_pool"]), img.shape)
    conv = fc.FusionConv(Cb + Ci, Ci, device=DEV)
    conv.weights = _t(w).requires_grad_(True)
    conv.beta = _t(beta).requires_grad_(True)
    conv.moving_mean, conv.moving_var = _t(mm), _t(mv)
    tb, ti = _t(bev).requires_grad_(True), _t(img).requires_grad_(True)
    y = conv.fused(tb, ti, smap, is_training=train)
    y.backward(_t(g))
    # oracle chain
    eb, _ = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"])
    _, raw = orc.conv3x3(eb, w, raw=True)
    mean = None if train else mm.astype(np.float64)
    var = None if train else mv.astype(np.float64)
    if train:
        ey, _, bvar, _, _ = orc.batch_norm_train(raw, 1e-3, None, beta, True)
        var_b = raw.reshape(-1, Ci).var(0)
        scale = 1.0 / np.sqrt(var_b + 1e-3)
    else:
        scale = 1.0 / np.sqrt(mv.astype(np.float64) + 1e-3)
        ey = np.maximum((raw - mm) * scale + beta, 0.0)
    g_raw, e_db, _ = orc.batch_norm_backward(raw, g, train, mean, var, 1e-3, None, beta, True)
    g_raw32 = g_raw.astype(np.float32)
    d_bv = orc.conv3x3_dgrad(g_raw32, w).astype(np.float64)
    d_img = orc.sparse_pool_grad_img(ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                     np.ascontiguousarray(d_bv[0, ..., Cb:].astype(np.float32)).reshape(-1, Ci),
                                     ref["img_index_flip_pool"], img.shape)
    d_w = orc.conv3x3_wgrad(eb, g_raw32)
    _, ab_y = orc.conv3x3(np.abs(eb), np.abs(w), raw=True)
    _check(y, ey, TOL + ACC * ab_y * np.abs(scale) + 1e-5 * np.abs(ey), "y")
    # g_raw is within ~1e-5 relative of the oracle's; the products carry it
    gr_mag = np.abs(g_raw) + 1e-3
    wt = np.ascontiguousarray(w[::-1, ::-1].transpose(0, 1, 3, 2))
    _, ab_dx = orc.conv3x3(gr_mag.astype(np.float32), np.abs(wt), raw=True)
    _check(tb.grad, d_bv[..., :Cb], TOL + 2e-5 * ab_dx[..., :Cb], "d_bev")
    # d_img sums several d_bv rows (TF order, f32) per pixel
    _check(ti.grad, d_img, 1e-4 + 1e-4 * np.abs(d_img), "d_img")
    _, ab_w = None, orc.conv3x3_wgrad(np.abs(eb), gr_mag.astype(np.float32))
    _check(conv.weights.grad, d_w, TOL + 2e-5 * ab_w, "d_w")
    _check(conv.beta.grad, e_db, 1e-4 + 1e-6 * np.abs(g).reshape(-1, Ci).sum(0), "d_beta")


@pytest.mark.parametrize("train,cb,ci,cout", [(True, 32, 32, 32), (False, 32, 32, 32),
                                               (True, 32, 16, 16), (False, 32, 16, 32), (True, 32, 16, 32),
                                               (True, 32, 32, 16), (False, 32, 32, 16)])
def test_fused_bf16_wgrad_reuses_forward_operand(train, cb, ci, cout):
    """bf16 FusionConv.fused: the weight gradient reading the forward's pooled operand
    (shpl_conv3x3_wgrad_reuse, WGRAD_REUSE) gives bitwise the gradients of the one that prepares its own.
    Config 1's geometry. 32 + 32 channels: the row-streaming forward and weight gradient. 32 + 16 with training
    BatchNorm (a 2 + 1 chunk statistics form k_conv_rows does not have) and c_out = 16 (not a whole output
    block) run the tiled forward, which leaves no pooled operand: the reuse must not be taken there
    (shpl_conv3x3_rows_form; ADVICE r04: it was, and dW read an unwritten workspace)."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    spec = synth.FrameSpec(2000, (1200, 360), (704, 800), (4, 4), cb, ci)
    fr = synth.make_frame(spec, seed=907, n_outside=10)
    gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                            tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img
    bev = _t(synth.make_features((1, Hb, Wb, Cb), 31)).to(torch.bfloat16)
    img = _t(synth.make_features((1, Hi, Wi, Ci), 32)).to(torch.bfloat16)
    g = _t(np.random.default_rng(33).standard_normal((1, Hb, Wb, cout)).astype(np.float32)).to(torch.bfloat16)
    grads = []
    for reuse in (False, True):
        smap = sm.pack_map(_t(ref["Mij_pool"]), _t(ref["M_val"].astype(np.float32)), ref["M_size"],
                           _t(ref["img_index_flip_pool"]), img.shape)
        conv = fc.FusionConv(Cb + Ci, cout, dtype=torch.bfloat16, device=DEV, seed=4)
        conv.WGRAD_REUSE = reuse
        conv.weights.requires_grad_(True)
        conv.beta.requires_grad_(True)
        tb, ti = bev.clone().requires_grad_(True), img.clone().requires_grad_(True)
        conv.fused(tb, ti, smap, is_training=train).backward(g)
        grads.append([x.grad.clone() for x in (tb, ti, conv.weights, conv.beta)])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_side_stream_backward_matches_one_stream(dtype):
    """FusionConv.IMG_ZERO_SIDE / WGRAD_SIDE / IMG_BESIDE_WGRAD: the image gradient's zero rows and / or the
    weight gradient on a side stream beside the input gradient, or the whole image gradient beside the weight
    gradient, give bitwise the gradients of the one-stream backward, over three steps (the side stream's
    allocations reused across steps)."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    spec = synth.FrameSpec(2000, (1200, 360), (704, 800), (4, 4), 32, 32)
    fr = synth.make_frame(spec, seed=911, n_outside=10)
    gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                            tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = _t(synth.make_features((1, Hb, Wb, 32), 41)).to(dtype)
    img = _t(synth.make_features((1, Hi, Wi, 32), 42)).to(dtype)
    grads = []
    for zero_side, wgrad_side, beside in ((False, False, False), (True, False, False), (False, True, False),
                                          (True, True, False), (True, False, True)):
        smap = sm.pack_map(_t(ref["Mij_pool"]), _t(ref["M_val"].astype(np.float32)), ref["M_size"],
                           _t(ref["img_index_flip_pool"]), img.shape)
        conv = fc.FusionConv(64, 32, dtype=dtype, device=DEV, seed=5)
        conv.IMG_ZERO_SIDE, conv.WGRAD_SIDE, conv.IMG_BESIDE_WGRAD = zero_side, wgrad_side, beside
        conv.weights.requires_grad_(True)
        conv.beta.requires_grad_(True)
        tb, ti = bev.clone().requires_grad_(True), img.clone().requires_grad_(True)
        out = []
        for k in range(3):
            for t in (tb, ti, conv.weights, conv.beta):
                t.grad = None
            g = _t(np.random.default_rng(50 + k).standard_normal((1, Hb, Wb, 32)).astype(np.float32)).to(dtype)
            conv.fused(tb, ti, smap, is_training=True).backward(g)
            out.append([x.grad.clone() for x in (tb, ti, conv.weights, conv.beta)])
        torch.cuda.synchronize()
        grads.append(out)
    for other in grads[1:]:
        for s0, s1 in zip(grads[0], other):
            for a, b in zip(s0, s1):
                assert torch.equal(a, b)


def test_wgrad_reuse_rejects_a_tiled_forward_workspace():
    """shpl_conv3x3_wgrad_reuse checks what it can of the forward's row-streaming predicate: a forward with
    training statistics over 32 + 16 bf16 channels runs the tiled kernel (no pooled operand in its workspace),
    so handing its workspace over is SHPL_ERR_ARG, not a silent read."""
    import ctypes
    from sparse_pooling_amd import _lib as L, fusion_conv as fc, shpl_map as sm
    spec = synth.FrameSpec(2000, (1200, 360), (704, 800), (4, 4), 32, 16)
    fr = synth.make_frame(spec, seed=907, n_outside=10)
    gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                            tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = _t(synth.make_features((1, Hb, Wb, 32), 31)).to(torch.bfloat16)
    img = _t(synth.make_features((1, Hi, Wi, 16), 32)).to(torch.bfloat16)
    smap = sm.pack_map(_t(ref["Mij_pool"]), _t(ref["M_val"].astype(np.float32)), ref["M_size"],
                       _t(ref["img_index_flip_pool"]), img.shape)
    pool = smap.csr(L.BY_CELL, L.ORDER_ENTRY)
    w = torch.zeros((3, 3, 48, 32), dtype=torch.bfloat16, device=DEV)
    assert not fc.rows_form(bev, w, b=img, pool=pool, frame_off=smap.frame_off, relu=False, stats=True)
    assert fc.rows_form(bev, w, b=img, pool=pool, frame_off=smap.frame_off, relu=False, stats=False)
    fws = L.workspace(fc.conv_ws_bytes(L.BF16, 1, Hb, Wb, 32, 16, 32, pool.nnz_cap, True), DEV)
    gy = torch.zeros((1, Hb, Wb, 32), dtype=torch.bfloat16, device=DEV)
    dw = torch.empty((3, 3, 48, 32), dtype=torch.float32, device=DEV)
    nb = ctypes.c_size_t()
    L.check(L.lib().shpl_conv3x3_wgrad_workspace_bytes(L.BF16, 1, Hb, Wb, 32, 16, 32, pool.nnz_cap,
                                                       ctypes.byref(nb)), "ws")
    ws = L.workspace(nb.value, DEV)
    rc = L.lib().shpl_conv3x3_wgrad_reuse(L.BF16, 1, Hb, Wb, L.ptr(bev), 32, 0, 32, L.ptr(img), 16, 0, 16, pool.ref(),
                                          L.ptr(smap.frame_off), L.ptr(gy), 32, 32, L.ptr(dw), L.ptr(ws), ws.numel(),
                                          L.ptr(fws), fws.numel(), 1, L.stream_of(DEV))
    assert rc == L.ERR_ARG


@pytest.mark.parametrize("stats,frames", [(True, 2), (False, 1)])
def test_dgrad_reuse_writes_occupied_cells_only(stats, frames):
    """shpl_conv3x3_dgrad_reuse: the input gradient's first map and, at every occupied cell of the pooled forward's
    CSR, its second map are bitwise shpl_conv3x3_dgrad's; every other cell of the second map keeps what it held
    (a NaN fill here). The forward (its workspace) with and without batch statistics; two frames: the occupancy
    words of frame 1 are found at its own rows. Config 1's geometry."""
    from sparse_pooling_amd import _lib as L, fusion_conv as fc, pipeline, shpl_map as sm
    spec = synth.CONFIGS[1]
    frs = [synth.make_frame(spec, seed=931 + f, n_outside=20 * f) for f in range(frames)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frs, DEV)
    ib = sm.build_index_batch(pts, vox, off, P, spec.im_size, spec.bv_size, spec.stride, maxp)
    smap = ib.map
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = _t(synth.make_features((frames, Hb, Wb, 32), 61)).to(torch.bfloat16)
    img = _t(synth.make_features((frames, Hi, Wi, 32), 62)).to(torch.bfloat16)
    pool = smap.csr(L.BY_CELL, L.ORDER_ENTRY)
    w = _t(np.random.default_rng(63).uniform(-0.1, 0.1, (3, 3, 64, 32)).astype(np.float32)).to(torch.bfloat16)
    assert fc.rows_form(bev, w, b=img, pool=pool, frame_off=smap.frame_off, relu=False, stats=stats)
    fws = L.workspace(fc.conv_ws_bytes(L.BF16, frames, Hb, Wb, 32, 32, 32, pool.nnz_cap, stats), DEV)
    st = torch.empty((2, 32), dtype=torch.float64, device=DEV) if stats else None
    fc.conv3x3(bev, w, b=img, pool=pool, frame_off=smap.frame_off, relu=False, stats=st, ws=fws)
    gy = _t(np.random.default_rng(64).standard_normal((frames, Hb, Wb, 32)).astype(np.float32)).to(torch.bfloat16)
    da, db = fc.conv3x3_dgrad(gy, w, 64, split=32)
    ws = L.workspace(fc.conv_ws_bytes(L.BF16, frames, Hb, Wb, 32, 0, 64, None, False), DEV)
    ra = torch.empty_like(da)
    rb = torch.full_like(db, float("nan"))
    L.check(L.lib().shpl_conv3x3_dgrad_reuse(L.BF16, frames, Hb, Wb, L.ptr(gy), 32, 32, L.ptr(w), 64, L.ptr(ra), 32,
                                             32, L.ptr(rb), 32, L.ptr(ws), ws.numel(), pool.ref(), L.ptr(fws),
                                             fws.numel(), int(stats), L.stream_of(DEV)), "shpl_conv3x3_dgrad_reuse")
    torch.cuda.synchronize()
    assert torch.equal(ra, da)
    dst, fo, fn = (_np(t) for t in (pool.ent_dst, smap.frame_off, ib.frame_nnz))
    occ = np.zeros(frames * Hb * Wb, dtype=bool)
    for f in range(frames):
        d = dst[fo[f]:fo[f] + fn[f]]
        occ[d[d >= 0]] = True
    occ = torch.from_numpy(occ).to(DEV)
    assert 0 < int(occ.sum()) < occ.numel()
    flat_b, flat_r = db.reshape(-1, 32), rb.reshape(-1, 32)
    assert torch.equal(flat_r[occ], flat_b[occ])
    assert bool(torch.isnan(flat_r[~occ].float()).all())
    # a workspace too small for the forward's plan is refused, not read
    rc = L.lib().shpl_conv3x3_dgrad_reuse(L.BF16, frames, Hb, Wb, L.ptr(gy), 32, 32, L.ptr(w), 64, L.ptr(ra), 32, 32,
                                          L.ptr(rb), 32, L.ptr(ws), ws.numel(), pool.ref(), L.ptr(fws), 256,
                                          int(stats), L.stream_of(DEV))
    assert rc == L.ERR_ARG
