"""Post-fusion 3x3 conv (shpl_conv3x3 / shpl_batch_norm)
vs the CPU oracle on MI355X.

The reference's Conv2D / FusedBatchNorm run through Eigen contractions that
fix no summation order, so the oracle sums in double and the HIP kernel in
f32 (exact f32 MFMA products, f32 accumulation). The tolerance is the
north_star's 1e-5 plus the f32 summation error of a K = 9*Cin term dot
product, 2^-19 * sum_k |a_k * w_k| (about 16 ulp of the absolute sum; TF's
own f32 Conv2D carries an error of the same order against the exact sum).
The fused form (pooled channels computed from the CSR inside the conv's
staging) must be BITWISE equal to the conv of the materialised bv_fused.
"""
import numpy as np
import pytest
import torch

from oracle import shpl_oracle as orc
from sparse_pooling_amd import synth

pytestmark = pytest.mark.gpu

TOL = 1e-5
ACC = 2.0 ** -19  # f32 accumulation term, relative to sum |a*w|
DEV = "cuda"


def _bound(x, w, scale=None):
    """Per-output tolerance: TOL + ACC * sum_k |x_k w_k| (times |scale|)."""
    _, ab = orc.conv3x3(np.abs(x), np.abs(w), raw=True)
    b = ACC * ab
    if scale is not None:
        b = b * np.abs(scale)
    return TOL + b


def _assert_within(got, ref, bound):
    err = np.abs(_np(got).astype(np.float64) - ref)
    assert (err <= bound).all(), (err.max(), (err / bound).max())


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def _weights(cin, cout, seed):
    rng = np.random.default_rng(seed)
    lim = np.sqrt(6.0 / (9 * cin + 9 * cout))
    # 3x xavier: outputs of a few units on N(0,1) inputs
    return (3.0 * rng.uniform(-lim, lim, (3, 3, cin, cout))).astype(np.float32)


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _bf16(a):
    return torch.from_numpy(orc.to_bf16_bits(a).view(np.int16)).to(DEV).view(torch.bfloat16)


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_pooling_amd import _lib as L
    L.lib()
    assert torch.cuda.is_available()


SHAPES = [  # B, H, W, Cin, Cout: partial tiles, channel tails, several output blocks
    (1, 9, 33, 10, 5),
    (2, 16, 64, 64, 32),
    (1, 5, 7, 3, 40),
    (3, 17, 70, 24, 33),
    (1, 1, 1, 8, 1),
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
@pytest.mark.parametrize("epi", ["none", "bias_relu", "bn_infer"])
def test_conv_dense_vs_oracle(shape, epi):
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = shape
    x = synth.make_features((B, H, W, Cin), 3)
    w = _weights(Cin, Cout, 4)
    rng = np.random.default_rng(5)
    center = scale = shift = None
    if epi == "bias_relu":
        shift = rng.standard_normal(Cout).astype(np.float32)
    elif epi == "bn_infer":
        center = rng.standard_normal(Cout).astype(np.float32)
        scale = rng.uniform(0.5, 2.0, Cout).astype(np.float32)
        shift = rng.standard_normal(Cout).astype(np.float32)
    relu = epi != "none"
    y = fc.conv3x3(_t(x), _t(w), center=None if center is None else _t(center),
                   scale=None if scale is None else _t(scale), shift=None if shift is None else _t(shift), relu=relu)
    ref = orc.conv3x3(x, w, center, scale, shift, relu)
    _assert_within(y, ref, _bound(x, w, scale))


def test_conv_two_dense_sources_equal_concat():
    """Channels split over two tensors == the conv of their concatenation,
    bitwise when the split falls on a staging chunk (8 f32 channels)."""
    from sparse_pooling_amd import fusion_conv as fc
    a = synth.make_features((2, 12, 40, 16), 6)
    b = synth.make_features((2, 12, 40, 24), 7)
    w = _weights(40, 32, 8)
    y2 = fc.conv3x3(_t(a), _t(w), b=_t(b), relu=False)
    y1 = fc.conv3x3(_t(np.concatenate([a, b], -1)), _t(w), relu=False)
    np.testing.assert_array_equal(_np(y2), _np(y1))
    ab = np.concatenate([a, b], -1)
    bound = _bound(ab, w)
    _assert_within(y1, orc.conv3x3(ab, w), bound)
    # a split off the chunk grid (12 + 28) still computes the same conv
    y3 = fc.conv3x3(_t(np.ascontiguousarray(ab[..., :12])), _t(w), b=_t(np.ascontiguousarray(ab[..., 12:])),
                    relu=False)
    _assert_within(y3, orc.conv3x3(ab, w), bound)


def _batch_map(cfg, n_frames, seed):
    from sparse_pooling_amd import pipeline, shpl_map as sm
    spec = synth.CONFIGS[cfg]
    frames = [synth.make_frame(spec, seed=seed + f, n_outside=20 * f) for f in range(n_frames)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    ib = sm.build_index_batch(pts, vox, off, P, spec.im_size, spec.bv_size, spec.stride, maxp)
    return spec, frames, ib


@pytest.mark.parametrize("cfg,n_frames", [(1, 3), (2, 2)])
def test_fused_pool_conv_is_the_conv_of_bv_fused(cfg, n_frames):
    """FusionConv.fused (pooling inside the conv's staging, bv_fused never
    written) == FusionConv(bv_fused) bitwise, and == the oracle's conv of the
    oracle's bv_fused within TOL (checked on a band of rows at config 2)."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    spec, frames, ib = _batch_map(cfg, n_frames, 500)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img
    bev = synth.make_features((n_frames, Hb, Wb, Cb), 11)
    img = synth.make_features((n_frames, Hi, Wi, Ci), 12)
    tb, ti = _t(bev), _t(img)
    conv = fc.FusionConv(Cb + Ci, Ci, device=DEV, seed=3)
    conv.weights = _t(_weights(Cb + Ci, Ci, 13))
    conv.moving_mean = _t(np.random.default_rng(1).standard_normal(Ci).astype(np.float32) * 0.1)
    conv.beta = _t(np.random.default_rng(2).standard_normal(Ci).astype(np.float32) * 0.1)
    bv_fused = sm.pool_img_to_bev(ib.map, ti, tb.shape, bev=tb)
    y_unf = conv(bv_fused)
    y_fus = conv.fused(tb, ti, ib.map)
    torch.cuda.synchronize()
    assert ib.map.error_bits() == 0
    np.testing.assert_array_equal(_np(y_fus), _np(y_unf))
    # oracle: bv_fused per frame (TF-order pooling), conv in double, on a band of rows
    center, scale, shift = (_np(v) for v in conv._inference_epilogue())
    y0, y1 = (0, Hb) if cfg == 1 else (300, 340)
    fo, fn = _np(ib.frame_off), _np(ib.frame_nnz)
    for f, fr in enumerate(frames):
        gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                                tuple(spec.bv_size))
        ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
        eb, _ = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                      ref["img_index_flip_pool"])
        np.testing.assert_array_equal(_np(bv_fused[f:f + 1]), eb)
        lo, hi = max(y0 - 1, 0), min(y1 + 1, Hb)
        band = orc.conv3x3(eb[:, lo:hi], _np(conv.weights), center, scale, shift, True)
        bound = _bound(eb[:, lo:hi], _np(conv.weights), scale)
        sl = slice(y0 - lo, y0 - lo + (y1 - y0))
        _assert_within(y_fus[f:f + 1, y0:y1], band[:, sl], bound[:, sl])


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_retinanet_fusion_conv_shape(dtype):
    """f4's second consumer at its own shape: RetinaNet's P2 SHPL followed by
    slim.conv2d(bev_fused, 256, [3, 3]) -- 256 BEV + 256 pooled image channels in, 256 out, bias + ReLU, no
    normalizer (retinanet_model.py:320-348) -- on config 6's 176 x 200 BEV grid, 2 frames. Fused == the conv
    of the materialised bv_fused (bitwise), and two bands of rows within the conv bound of the oracle's
    double-precision conv of the oracle's bv_fused (bf16: + one bf16 ulp of the result)."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    n_frames = 2
    spec, frames, ib = _batch_map(6, n_frames, 800)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci, Co = spec.c_bev, spec.c_img, 256
    bf = dtype == "bf16"
    dt = torch.bfloat16 if bf else torch.float32
    rd = (lambda a: orc.from_bf16_bits(orc.to_bf16_bits(a))) if bf else (lambda a: a)
    bev = rd(synth.make_features((n_frames, Hb, Wb, Cb), 61))
    img = rd(synth.make_features((n_frames, Hi, Wi, Ci), 62))
    w = rd(_weights(Cb + Ci, Co, 63))
    tb, ti = _t(bev).to(dt), _t(img).to(dt)
    conv = fc.FusionConv(Cb + Ci, Co, batch_norm=False, bias=True, relu=True, dtype=dt, device=DEV, seed=3)
    conv.weights = _t(w).to(dt)
    conv.bias = _t(np.random.default_rng(4).standard_normal(Co).astype(np.float32) * 0.5)
    bv_fused = sm.pool_img_to_bev(ib.map, ti, tb.shape, bev=tb)
    y_unf = conv(bv_fused)
    y_fus = conv.fused(tb, ti, ib.map)
    torch.cuda.synchronize()
    assert ib.map.error_bits() == 0
    assert torch.equal(y_fus, y_unf)
    _, _, shift = (None if v is None else _np(v) for v in conv._inference_epilogue())
    for f, fr in enumerate(frames):
        gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                                tuple(spec.bv_size))
        ref = orc.produce_sparse_pooling_input(gen, stride=spec.stride)
        eb, _ = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                      ref["img_index_flip_pool"])
        eb = rd(eb)
        np.testing.assert_array_equal(_np(bv_fused[f:f + 1].float()), eb)
        for y0, y1 in ((0, 5), (70, 76)):
            lo, hi = max(y0 - 1, 0), min(y1 + 1, Hb)
            band = orc.conv3x3(eb[:, lo:hi], w, None, None, shift, True)
            bound = _bound(eb[:, lo:hi], w)
            if bf:
                bound = bound + np.abs(band) * 2.0 ** -8
            sl = slice(y0 - lo, y0 - lo + (y1 - y0))
            _assert_within(y_fus[f:f + 1, y0:y1].float(), band[:, sl], bound[:, sl])


@pytest.mark.parametrize("shape", [(2, 17, 33, 128, 64, 256, "relu"), (1, 16, 16, 64, 64, 512, "none"),
                                   (1, 21, 9, 192, 0, 256, "bn"), (3, 5, 40, 64, 128, 256, "relu")])
def test_bf16_wide_conv_dense(shape):
    """The wide bf16 kernel (k_conv_wide: input chunks of 64 channels, 256-channel output blocks): partial
    16 x 16 tiles at every edge, one and two sources (== their concat, bitwise), two output blocks, the
    epilogue with and without center / scale / shift and ReLU, against the oracle's double-precision conv
    (bound: the f32 accumulation term + one bf16 ulp of the result)."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, ca, cb, co, epi = shape
    rd = lambda a: orc.from_bf16_bits(orc.to_bf16_bits(a))  # noqa: E731
    a = rd(synth.make_features((B, H, W, ca), 71))
    b = rd(synth.make_features((B, H, W, cb), 72)) if cb else None
    w = rd(_weights(ca + cb, co, 73))
    rng = np.random.default_rng(74)
    center = scale = shift = None
    if epi == "bn":
        center = rng.standard_normal(co).astype(np.float32) * 0.1
        scale = rng.uniform(0.5, 2.0, co).astype(np.float32)
    if epi != "none":
        shift = rng.standard_normal(co).astype(np.float32) * 0.5
    relu = epi != "none"
    ta, tw = _bf16(a), _bf16(w)
    tb = _bf16(b) if cb else None
    f32 = lambda v: None if v is None else _t(v)  # noqa: E731
    y = fc.conv3x3(ta, tw, b=tb, center=f32(center), scale=f32(scale), shift=f32(shift), relu=relu)
    x = np.concatenate([a, b], -1) if cb else a
    if cb:  # two sources == one concatenated source, bitwise (the same K order: 64-channel chunks)
        y1 = fc.conv3x3(_bf16(x), tw, center=f32(center), scale=f32(scale), shift=f32(shift), relu=relu)
        assert torch.equal(y, y1)
    ref = orc.conv3x3(x, w, center, scale, shift, relu)
    bound = _bound(x, w, scale) + np.abs(ref) * 2.0 ** -8
    _assert_within(y.float(), ref, bound)


def test_fused_conv_noncanonical_map():
    """Shuffled entries, cells with many entries (the run walk), negative
    weights, an empty frame-less corner, odd channel counts (scalar staging)."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    rng = np.random.default_rng(31)
    n, hb, wb, h, w, cb, ci, cout = 700, 20, 45, 15, 17, 5, 3, 7
    R = hb * wb
    idx = np.stack([np.zeros(n, np.int64), rng.integers(0, h, n), rng.integers(0, w, n)], 1)
    rows = rng.integers(0, R, n)
    rows[100:260] = rows[100]               # one cell with 160 entries
    rows[300:340] = rng.integers(0, wb, 40)  # a crowded first row
    extra = np.stack([rng.integers(0, R, 300), rng.integers(0, n, 300)], 1)
    mij = np.concatenate([np.stack([rows, np.arange(n)], 1), extra]).astype(np.int64)
    mij = mij[rng.permutation(len(mij))]
    mval = rng.uniform(-2, 2, len(mij)).astype(np.float32)
    img = rng.standard_normal((1, h, w, ci)).astype(np.float32)
    bev = rng.standard_normal((1, hb, wb, cb)).astype(np.float32)
    smap = sm.pack_map(_t(mij), _t(mval), [R, n], _t(idx), img.shape)
    wts = _weights(cb + ci, cout, 32)
    fused = fc.conv3x3(_t(bev), _t(wts), b=_t(img), pool=smap.csr(0, 0), frame_off=smap.frame_off, relu=False)
    bv = sm.pool_img_to_bev(smap, _t(img), (1, hb, wb, cb), bev=_t(bev))
    unf = fc.conv3x3(_t(_np(bv)[..., :cb]), _t(wts), b=_t(_np(bv)[..., cb:]), relu=False)
    np.testing.assert_array_equal(_np(fused), _np(unf))
    pooled = orc.sparse_pool_op(mij, mval, [R, n], img, idx).reshape(1, hb, wb, ci)
    x = np.concatenate([bev, pooled], -1)
    _assert_within(fused, orc.conv3x3(x, wts), _bound(x, wts))


def test_fused_conv_empty_map():
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    bev = synth.make_features((1, 6, 7, 8), 2)
    img = synth.make_features((1, 9, 11, 8), 1)
    smap = sm.pack_map(torch.zeros((0, 2), dtype=torch.int64, device=DEV), torch.zeros(0, device=DEV), [42, 0],
                       torch.zeros((0, 3), dtype=torch.int32, device=DEV), img.shape)
    wts = _weights(16, 8, 3)
    y = fc.conv3x3(_t(bev), _t(wts), b=_t(img), pool=smap.csr(0, 0), frame_off=smap.frame_off, relu=False)
    x = np.concatenate([bev, np.zeros_like(bev)], -1)
    _assert_within(y, orc.conv3x3(x, wts), _bound(x, wts))


def test_bf16_rows_empty_map_stats_and_wgrad():
    """An empty map through the bf16 pooled forms (k_conv_rows CMP + statistics, k_wgrad_rows with a pooled
    tile): every pooled chunk is zero, so both equal the dense forms over a zero second source, bitwise."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    bev = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((1, 6, 37, 32), 2)))
    img = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((1, 9, 11, 32), 1)))
    smap = sm.pack_map(torch.zeros((0, 2), dtype=torch.int64, device=DEV), torch.zeros(0, device=DEV), [222, 0],
                       torch.zeros((0, 3), dtype=torch.int32, device=DEV), img.shape)
    w = _bf16(orc.from_bf16_bits(orc.to_bf16_bits(_weights(64, 32, 3))))
    tb, ti = _bf16(bev), _bf16(img)
    zero = torch.zeros_like(tb)
    st_f, st_d = (torch.empty((2, 32), dtype=torch.float64, device=DEV) for _ in range(2))
    y_f = fc.conv3x3(tb, w, b=ti, pool=smap.csr(0, 0), frame_off=smap.frame_off, relu=False, stats=st_f)
    y_d = fc.conv3x3(tb, w, b=zero, relu=False, stats=st_d)
    assert torch.equal(y_f, y_d) and torch.equal(st_f, st_d)
    g = _bf16(synth.make_features((1, 6, 37, 32), 4))
    dw_f = fc.conv3x3_wgrad(tb, g, b=ti, pool=smap.csr(0, 0), frame_off=smap.frame_off)
    dw_d = fc.conv3x3_wgrad(tb, g, b=zero)
    assert torch.equal(dw_f, dw_d)
    assert not dw_f[:, :, 32:].any()


def test_batch_norm_training_vs_oracle():
    """is_training: conv statistics -> batch moments -> normalise + ReLU in
    place, moving averages with the Bessel-corrected variance."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = 2, 19, 37, 24, 40
    x = synth.make_features((B, H, W, Cin), 9) + 0.5
    w = _weights(Cin, Cout, 10)
    conv = fc.FusionConv(Cin, Cout, device=DEV)
    conv.weights = _t(w)
    rng = np.random.default_rng(3)
    beta = rng.standard_normal(Cout).astype(np.float32)
    mm0 = rng.standard_normal(Cout).astype(np.float32)
    mv0 = rng.uniform(0.5, 2, Cout).astype(np.float32)
    conv.beta, conv.moving_mean, conv.moving_var = _t(beta), _t(mm0), _t(mv0)
    conv(_t(x), is_training=False)  # an inference step first: its cached BN scale must not outlive the update
    y = conv(_t(x), is_training=True)
    _, raw = orc.conv3x3(x, w, raw=True)
    ey, bm, bv, emm, emv = orc.batch_norm_train(raw, 1e-3, None, beta, True, mm0, mv0, 0.999)
    k = 1.0 / np.sqrt(bv * (B * H * W - 1) / (B * H * W) + 1e-3)
    _assert_within(y, ey, _bound(x, w, k) + 1e-6 * np.abs(ey))
    np.testing.assert_allclose(_np(conv.moving_mean), emm, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(_np(conv.moving_var), emv, rtol=1e-6, atol=1e-7)
    # inference afterwards uses the moving statistics
    yi = conv(_t(x), is_training=False)
    k = 1.0 / np.sqrt(emv.astype(np.float64) + 1e-3)
    _assert_within(yi, orc.conv3x3(x, w, emm, k, beta, True), _bound(x, w, k))


def test_inference_scale_follows_graph_replayed_training():
    """The inference epilogue's scale 1/sqrt(moving_var + eps) follows moving_var when the training steps run
    from a captured HIP graph (no Python per step; batch_norm_train updates moving_var through its device
    pointer): after three replays of a captured training step, an eager inference call AND an inference graph
    captured before those replays both equal the conv with the scale recomputed from the current moving_var,
    bitwise."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = 1, 12, 20, 16, 32
    conv = fc.FusionConv(Cin, Cout, device=DEV, seed=5)
    conv.beta = _t(np.random.default_rng(4).standard_normal(Cout).astype(np.float32))
    x = _t(synth.make_features((B, H, W, Cin), 11) + 0.5)
    y_inf = torch.empty((B, H, W, Cout), device=DEV)
    conv(x, is_training=False, out=y_inf)  # the scale of the initial moving_var (all ones)
    gs = torch.cuda.Stream()
    gs.wait_stream(torch.cuda.current_stream())
    g_inf = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_inf, stream=gs):
        conv(x, is_training=False, out=y_inf)
    y_tr = torch.empty_like(y_inf)
    conv(x, is_training=True, out=y_tr)  # warm-up: workspaces allocated before the capture
    torch.cuda.synchronize()
    g_tr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_tr, stream=gs):
        conv(x, is_training=True, out=y_tr)
    mv_before = conv.moving_var.clone()
    for _ in range(3):
        g_tr.replay()
    torch.cuda.synchronize()
    assert not torch.equal(conv.moving_var, mv_before)  # the replays did move the statistics
    want = fc.conv3x3(x, conv.weights, center=conv.moving_mean, scale=1.0 / torch.sqrt(conv.moving_var + conv.eps),
                      shift=conv.beta, relu=True)
    assert torch.equal(conv(x, is_training=False), want)
    y_inf.fill_(float("nan"))
    g_inf.replay()
    torch.cuda.synchronize()
    assert torch.equal(y_inf, want)


def test_bf16_conv_and_fused():
    """bf16 storage: bf16 MFMA products are exact, f32 accumulation, one
    rounding at the store (|err| <= one bf16 ulp of the f32 result + TOL).
    Fused == unfused bitwise needs the BEV channels to end on a staging chunk
    (16 bf16 channels); a 24-channel BEV still agrees within the bound."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    spec, frames, ib = _batch_map(1, 2, 600)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    for cb, ci in ((16, 16), (24, 8)):
        bev = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((2, Hb, Wb, cb), 21)))
        img = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((2, Hi, Wi, ci), 22)))
        w = orc.from_bf16_bits(orc.to_bf16_bits(_weights(cb + ci, 16, 23)))
        tb, ti, tw = _bf16(bev), _bf16(img), _bf16(w)
        bv = sm.pool_img_to_bev(ib.map, ti, tb.shape, bev=tb)
        y_unf = fc.conv3x3(bv, tw, relu=False)
        y_fus = fc.conv3x3(tb, tw, b=ti, pool=ib.map.csr(0, 0), frame_off=ib.map.frame_off, relu=False)
        x = _np(bv.float())
        ref = orc.conv3x3(x, w)
        bound = _bound(x, w) + np.abs(ref) * 2.0 ** -8
        _assert_within(y_unf.float(), ref, bound)
        _assert_within(y_fus.float(), ref, bound)
        if cb % 16 == 0:
            np.testing.assert_array_equal(_np(y_fus.float()), _np(y_unf.float()))


ROWS_SHAPES = [  # bf16, <= 64 input channels, whole 32-channel output blocks: the row-streaming kernel
    (2, 16, 64, 64, 32),   # one band, two strips
    (3, 17, 70, 24, 64),   # a partial strip, two output blocks, a channel tail inside chunk 2
    (1, 1, 5, 8, 32),      # one row, one partial strip
    (2, 130, 40, 48, 32),  # three bands (band edges inside the map)
    (1, 61, 33, 16, 32),   # one band of 61 rows (every ring slot phase at the band end)
]


@pytest.mark.parametrize("shape", ROWS_SHAPES, ids=[str(s) for s in ROWS_SHAPES])
def test_bf16_rows_conv_dense(shape):
    """k_conv_rows (bf16, weights resident in VGPRs, per-wave LDS-DMA ring) vs
    the oracle, with the BatchNorm-inference epilogue; a two-source split on
    the chunk grid is bitwise the one-source conv."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = shape
    x = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((B, H, W, Cin), 41)))
    w = orc.from_bf16_bits(orc.to_bf16_bits(_weights(Cin, Cout, 42)))
    rng = np.random.default_rng(43)
    center = rng.standard_normal(Cout).astype(np.float32)
    scale = rng.uniform(0.5, 2.0, Cout).astype(np.float32)
    shift = rng.standard_normal(Cout).astype(np.float32)
    y = fc.conv3x3(_bf16(x), _bf16(w), center=_t(center), scale=_t(scale), shift=_t(shift), relu=True)
    ref = orc.conv3x3(x, w, center, scale, shift, True)
    _assert_within(y.float(), ref, _bound(x, w, scale) + np.abs(ref) * 2.0 ** -8)
    if Cin % 32 == 0:
        h = Cin // 2
        y2 = fc.conv3x3(_bf16(np.ascontiguousarray(x[..., :h])), _bf16(w), b=_bf16(np.ascontiguousarray(x[..., h:])),
                        center=_t(center), scale=_t(scale), shift=_t(shift), relu=True)
        np.testing.assert_array_equal(_np(y2.float()), _np(y.float()))


@pytest.mark.parametrize("relu", [True, False])
def test_bf16_rows_epilogue_equals_tiled(relu):
    """The same bf16 conv through k_conv_rows (16-byte aligned output) and the tiled
    k_conv3x3 (an output view 2 bytes off 16-byte alignment): bitwise the same with
    center, scale and shift all set (fma(acc, scale, shift - center * scale), rounded,
    then ReLU as an integer max on the bf16 bits), a NaN input pixel included. The two
    kernels sum the MFMA products in different orders, so inputs and weights are
    small integers: every accumulator is exact in f32 and only the epilogue can
    differ."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = 2, 16, 40, 32, 32
    rng = np.random.default_rng(53)
    x = rng.integers(-3, 4, (B, H, W, Cin)).astype(np.float32)
    x[1, 7, 9, 3] = np.nan
    w = rng.integers(-2, 3, (3, 3, Cin, Cout)).astype(np.float32)
    center = rng.standard_normal(Cout).astype(np.float32)
    scale = rng.uniform(0.5, 2.0, Cout).astype(np.float32)
    shift = rng.standard_normal(Cout).astype(np.float32)
    n = B * H * W * Cout
    flat = torch.empty(n + 16, dtype=torch.bfloat16, device=DEV)
    outs = []
    for off in (0, 1):  # 0: 16-byte aligned (row kernel), 1: 2 bytes off (tiled kernel)
        o = flat[off:off + n].view(B, H, W, Cout)
        fc.conv3x3(_bf16(x), _bf16(w), center=_t(center), scale=_t(scale), shift=_t(shift), relu=relu, out=o)
        torch.cuda.synchronize()
        outs.append(_np(o.view(torch.int16)).copy())
    np.testing.assert_array_equal(outs[0], outs[1])
    if not relu:  # the NaN pixel reached the outputs (the MFMA's NaN is negative: ReLU makes it +0)
        assert np.isnan(orc.from_bf16_bits(outs[0].view(np.uint16))).any()


STATS_SHAPES = [  # bf16 training forward on k_conv_rows: statistics epilogue (dense sources)
    (2, 16, 64, 64, 32),   # two sources of 32 (the training workload's Q = 4, QA = 2)
    (3, 17, 70, 24, 64),   # partial strip (masked pixels), two output blocks
    (2, 130, 40, 32, 32),  # three bands
]


@pytest.mark.parametrize("shape", STATS_SHAPES, ids=[str(s) for s in STATS_SHAPES])
def test_bf16_rows_conv_stats(shape):
    """The batch statistics of k_conv_rows' statistics epilogue (per band: f32
    sums of the f32 accumulators, per item a double; k_stats_reduce in a fixed
    order) vs the oracle's double sums of its double conv; the pre-activation
    output within the bf16 bound; a two-source split bitwise the one-source conv
    (output and statistics)."""
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, Cin, Cout = shape
    x = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((B, H, W, Cin), 61) + 0.25))
    w = orc.from_bf16_bits(orc.to_bf16_bits(_weights(Cin, Cout, 62)))
    stats = torch.empty((2, Cout), dtype=torch.float64, device=DEV)
    y = fc.conv3x3(_bf16(x), _bf16(w), relu=False, stats=stats)
    _, raw = orc.conv3x3(x, w, raw=True)
    bound = _bound(x, w)
    _assert_within(y.float(), raw, bound + np.abs(raw) * 2.0 ** -8)
    r2 = raw.reshape(-1, Cout)
    b2 = bound.reshape(-1, Cout)
    s = _np(stats)
    # per value the accumulator's error (bound), plus the f32 summation of the band sums
    _assert_within(s[0], r2.sum(0), b2.sum(0) + 1e-5 * np.abs(r2).sum(0))
    _assert_within(s[1], (r2 * r2).sum(0), (2.0 * np.abs(r2) * b2 + b2 * b2).sum(0) + 1e-5 * (r2 * r2).sum(0))
    if Cin % 32 == 0:
        h = Cin // 2
        st2 = torch.empty_like(stats)
        y2 = fc.conv3x3(_bf16(np.ascontiguousarray(x[..., :h])), _bf16(w), b=_bf16(np.ascontiguousarray(x[..., h:])),
                        relu=False, stats=st2)
        np.testing.assert_array_equal(_np(y2.float()), _np(y.float()))
        np.testing.assert_array_equal(_np(st2), s)


@pytest.mark.parametrize("cb,ci", [(32, 32), (16, 16)])
def test_bf16_rows_pooled_stats_and_wgrad(cb, ci):
    """The bf16 training pair without bv_fused: the pooled forward with the
    statistics epilogue (k_conv_rows, compact run buffer, lane offsets in LDS)
    and the pooled weight gradient (k_wgrad_rows gathering the same compact
    rows) are bitwise the dense two-source forms over the materialised pooled
    map (config 2 geometry, two frames; 16 + 16 -> 32 takes the 1 + 1 chunk
    instantiation). The dense forms are checked against the oracle elsewhere."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    spec, frames, ib = _batch_map(2, 2, 800)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((2, Hb, Wb, cb), 81)))
    img = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((2, Hi, Wi, ci), 82)))
    w = orc.from_bf16_bits(orc.to_bf16_bits(_weights(cb + ci, 32, 83)))
    tb, ti, tw = _bf16(bev), _bf16(img), _bf16(w)
    csr, foff = ib.map.csr(0, 0), ib.map.frame_off
    xb = sm.pool_img_to_bev(ib.map, ti, (2, Hb, Wb, ci))
    st_f = torch.empty((2, 32), dtype=torch.float64, device=DEV)
    st_d = torch.empty_like(st_f)
    y_f = fc.conv3x3(tb, tw, b=ti, pool=csr, frame_off=foff, relu=False, stats=st_f)
    y_d = fc.conv3x3(tb, tw, b=xb, relu=False, stats=st_d)
    torch.cuda.synchronize()
    assert ib.map.error_bits() == 0
    assert torch.equal(y_f, y_d)
    assert torch.equal(st_f, st_d)
    g = _bf16(synth.make_features((2, Hb, Wb, 32), 84))
    dw_f = fc.conv3x3_wgrad(tb, g, b=ti, pool=csr, frame_off=foff)
    dw_d = fc.conv3x3_wgrad(tb, g, b=xb)
    if cb % 32 == 0:
        assert torch.equal(dw_f, dw_d)
    else:  # A ends inside an input tile: the tiled kernels (their own summation orders), within the f32 bound
        ab = fc.conv3x3_wgrad(tb.abs(), g.abs(), b=xb.abs())
        _assert_within(dw_f, _np(dw_d).astype(np.float64), 1e-5 + 2.0 ** -15 * _np(ab))


def test_bf16_rows_fused_config2():
    """Config 2 in bf16 (32 + 32 -> 32 channels: k_conv_rows with the pooled
    half gathered from the compact run buffer): fused == the conv of the
    materialised bv_fused bitwise, and within the bf16 bound of the oracle's
    conv of the oracle's bv_fused on a band of rows."""
    from sparse_pooling_amd import fusion_conv as fc, shpl_map as sm
    spec, frames, ib = _batch_map(2, 2, 700)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img
    bev = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((2, Hb, Wb, Cb), 51)))
    img = orc.from_bf16_bits(orc.to_bf16_bits(synth.make_features((2, Hi, Wi, Ci), 52)))
    w = orc.from_bf16_bits(orc.to_bf16_bits(_weights(Cb + Ci, Ci, 53)))
    tb, ti, tw = _bf16(bev), _bf16(img), _bf16(w)
    conv = fc.FusionConv(Cb + Ci, Ci, dtype=torch.bfloat16, device=DEV, seed=3)
    conv.weights = tw
    conv.moving_mean = _t(np.random.default_rng(1).standard_normal(Ci).astype(np.float32) * 0.1)
    conv.beta = _t(np.random.default_rng(2).standard_normal(Ci).astype(np.float32) * 0.1)
    bv_fused = sm.pool_img_to_bev(ib.map, ti, tb.shape, bev=tb)
    y_unf = conv(bv_fused)
    y_fus = conv.fused(tb, ti, ib.map)
    torch.cuda.synchronize()
    assert ib.map.error_bits() == 0
    np.testing.assert_array_equal(_np(y_fus.float()), _np(y_unf.float()))
    center, scale, shift = (_np(v) for v in conv._inference_epilogue())
    y0, y1 = 296, 344
    for f in range(2):
        x = _np(bv_fused[f:f + 1, y0 - 1:y1 + 1].float())
        ref = orc.conv3x3(x, w, center, scale, shift, True)[:, 1:-1]
        bound = (_bound(x, w, scale) + np.abs(orc.conv3x3(x, w, center, scale, shift, True)) * 2.0 ** -8)[:, 1:-1]
        _assert_within(y_fus[f:f + 1, y0:y1].float(), ref, bound)


def test_conv_argument_errors():
    from sparse_pooling_amd import fusion_conv as fc, _lib as L
    x = _t(synth.make_features((1, 4, 4, 8), 1))
    with pytest.raises(ValueError):
        fc.conv3x3(x, _t(_weights(9, 4, 1)))
    with pytest.raises(L.ShplLibraryError):
        fc.conv3x3(x, _t(_weights(8, 4, 1)), ws=torch.empty(16, dtype=torch.uint8, device=DEV))
