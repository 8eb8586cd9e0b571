"""Seeded random shapes through the bf16 row-streaming conv kernels
(k_conv_rows: forward with / without statistics, the input gradient's two
maps; k_wgrad_rows: dense and pooled input tiles) against the CPU oracle's
double sums, with the bounds of test_gpu_conv.py / test_gpu_conv_grad.py:
1e-5 + 2^-19 * sum|a*w| per output (plus one bf16 ulp of a stored bf16
result), 1e-5 + 2^-16 * sum|x*g| per weight-gradient element. Shapes cover
partial strips, channel tails inside a 16-channel chunk, several bands and
frames, one or two output blocks.
"""
import numpy as np
import pytest
import torch

from oracle import shpl_oracle as orc
from sparse_pooling_amd import synth

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 1e-5


def _shapes(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        B = int(rng.integers(1, 3))
        H = int(rng.integers(1, 140))
        W = int(rng.integers(1, 90))
        cin = int(rng.choice([8, 16, 24, 32, 40, 48, 56, 64]))
        cout = int(rng.choice([32, 64]))
        out.append((B, H, W, cin, cout))
    return out


def _bf(a):
    return orc.from_bf16_bits(orc.to_bf16_bits(a))


def _dev(a):
    return torch.from_numpy(orc.to_bf16_bits(np.ascontiguousarray(a)).view(np.int16)).to(DEV).view(torch.bfloat16)


def _weights(cin, cout, seed):
    rng = np.random.default_rng(seed)
    lim = np.sqrt(6.0 / (9 * cin + 9 * cout))
    return _bf((3.0 * rng.uniform(-lim, lim, (3, 3, cin, cout))).astype(np.float32))


def _within(got, ref, bound, what):
    err = np.abs(got.astype(np.float64) - ref)
    assert (err <= bound).all(), (what, float(err.max()), float((err / bound).max()))


@pytest.mark.parametrize("shape", _shapes(2024, 6), ids=str)
def test_rows_forward_stats_dgrad_fuzz(shape):
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, cin, cout = shape
    x = _bf(synth.make_features((B, H, W, cin), 7) + 0.25)
    w = _weights(cin, cout, 8)
    stats = torch.empty((2, cout), dtype=torch.float64, device=DEV)
    y = fc.conv3x3(_dev(x), _dev(w), relu=False, stats=stats).float().cpu().numpy()
    _, raw = orc.conv3x3(x, w, raw=True)
    _, ab = orc.conv3x3(np.abs(x), np.abs(w), raw=True)
    bound = TOL + 2.0 ** -19 * ab
    _within(y, raw, bound + 2.0 ** -8 * np.abs(raw), "y")
    r2, b2 = raw.reshape(-1, cout), bound.reshape(-1, cout)
    s = stats.cpu().numpy()
    _within(s[0], r2.sum(0), b2.sum(0) + 1e-5 * np.abs(r2).sum(0), "sum")
    _within(s[1], (r2 * r2).sum(0), (2.0 * np.abs(r2) * b2 + b2 * b2).sum(0) + 1e-5 * (r2 * r2).sum(0), "sumsq")
    # the input gradient of a cout-channel output gradient into cin channels, split at a block when it can be
    if cin % 8 == 0:
        g = _bf(synth.make_features((B, H, W, cout), 9))
        wt = np.ascontiguousarray(w[::-1, ::-1].transpose(0, 1, 3, 2))  # the dgrad's forward weights: cout -> cin
        dx = fc.conv3x3_dgrad(_dev(g), _dev(w), cin).float().cpu().numpy()
        ref = orc.conv3x3_dgrad(g, w)
        _, abd = orc.conv3x3(np.abs(g), np.abs(wt), raw=True)
        _within(dx, ref, TOL + 2.0 ** -19 * abd + 2.0 ** -8 * np.abs(ref), "dx")


@pytest.mark.parametrize("shape", _shapes(4048, 6), ids=str)
def test_rows_wgrad_fuzz(shape):
    from sparse_pooling_amd import fusion_conv as fc
    B, H, W, cin, cout = shape
    x = _bf(synth.make_features((B, H, W, cin), 11))
    g = _bf(synth.make_features((B, H, W, cout), 12))
    dw = fc.conv3x3_wgrad(_dev(x), _dev(g)).cpu().numpy()
    bound = TOL + 2.0 ** -16 * orc.conv3x3_wgrad(np.abs(x), np.abs(g))
    _within(dw, orc.conv3x3_wgrad(x, g), bound, "dw")
    if cin > 32 and cin % 32 == 0:  # two sources on the 32-channel tile grid: bitwise the one-source form
        h = 32
        dw2 = fc.conv3x3_wgrad(_dev(x[..., :h]), _dev(g), b=_dev(x[..., h:])).cpu().numpy()
        np.testing.assert_array_equal(dw2, dw)
