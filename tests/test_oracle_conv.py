"""The oracle's post-fusion conv + BatchNorm (CPU) against an independent
restatement: torch's CPU conv2d / batch_norm in float64 (TensorFlow 1.8, the
reference's own runtime, is not installable here: parity unpinned by
reference fixtures, see oracle/shpl_oracle.c)."""
import numpy as np
import pytest
import torch

from oracle import shpl_oracle as orc


def _torch_conv(x, w):
    t = torch.nn.functional.conv2d(torch.from_numpy(x).double().permute(0, 3, 1, 2),
                                   torch.from_numpy(w).double().permute(3, 2, 0, 1), padding=1)
    return t.permute(0, 2, 3, 1).numpy()


@pytest.mark.parametrize("shape", [(1, 5, 7, 3, 4), (2, 9, 11, 16, 33), (1, 1, 1, 2, 2)])
def test_oracle_conv_matches_torch(shape):
    B, H, W, Cin, Cout = shape
    rng = np.random.default_rng(0)
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    w = rng.standard_normal((3, 3, Cin, Cout)).astype(np.float32)
    y, raw = orc.conv3x3(x, w, raw=True)
    t = _torch_conv(x, w)
    assert np.abs(raw - t).max() <= 1e-9 * max(1.0, np.abs(t).max())
    np.testing.assert_array_equal(y, t.astype(np.float32))
    c = rng.standard_normal(Cout).astype(np.float32)
    s = rng.uniform(0.5, 2, Cout).astype(np.float32)
    b = rng.standard_normal(Cout).astype(np.float32)
    y2 = orc.conv3x3(x, w, c, s, b, relu=True)
    e = np.maximum((t - c.astype(np.float64)) * s + b, 0.0).astype(np.float32)
    np.testing.assert_allclose(y2, e, rtol=1e-6, atol=1e-6)


def test_oracle_batch_norm_training_matches_torch():
    rng = np.random.default_rng(1)
    raw = rng.standard_normal((3, 7, 5, 6)) * 2.0 + 1.0
    beta = rng.standard_normal(6).astype(np.float32)
    mm = rng.standard_normal(6).astype(np.float32)
    mv = rng.uniform(0.5, 2, 6).astype(np.float32)
    y, bm, bv, emm, emv = orc.batch_norm_train(raw, 1e-3, None, beta, True, mm, mv, 0.999)
    rm, rv = torch.from_numpy(mm.astype(np.float64)), torch.from_numpy(mv.astype(np.float64))
    t = torch.nn.functional.batch_norm(torch.from_numpy(raw).permute(0, 3, 1, 2), rm, rv, None,
                                       torch.from_numpy(beta).double(), training=True, momentum=0.001, eps=1e-3)
    t = torch.relu(t).permute(0, 2, 3, 1).numpy()
    np.testing.assert_allclose(y, t.astype(np.float32), rtol=1e-6, atol=1e-6)
    # torch's running stats use the unbiased variance, as TF's FusedBatchNorm does
    np.testing.assert_allclose(emm, rm.numpy().astype(np.float32), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(emv, rv.numpy().astype(np.float32), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(bv, raw.reshape(-1, 6).var(0, ddof=1), rtol=1e-12)


def test_oracle_conv_and_bn_backward_match_torch_autograd():
    rng = np.random.default_rng(2)
    B, H, W, Cin, Cout = 2, 5, 7, 6, 4
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    w = rng.standard_normal((3, 3, Cin, Cout)).astype(np.float32)
    g = rng.standard_normal((B, H, W, Cout)).astype(np.float32)
    tx = torch.from_numpy(x).double().permute(0, 3, 1, 2).requires_grad_()
    tw = torch.from_numpy(w).double().permute(3, 2, 0, 1).requires_grad_()
    torch.nn.functional.conv2d(tx, tw, padding=1).backward(torch.from_numpy(g).double().permute(0, 3, 1, 2))
    np.testing.assert_allclose(orc.conv3x3_dgrad(g, w), tx.grad.permute(0, 2, 3, 1).numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(orc.conv3x3_wgrad(x, g), tw.grad.permute(2, 3, 1, 0).numpy(), rtol=1e-12, atol=1e-12)
    raw = rng.standard_normal((B, H, W, Cout)) * 2 + 1
    beta = rng.standard_normal(Cout).astype(np.float32)
    t = torch.from_numpy(raw).permute(0, 3, 1, 2).requires_grad_()
    tb = torch.from_numpy(beta).double().requires_grad_()
    tg = torch.ones(Cout, dtype=torch.float64, requires_grad=True)
    yy = torch.relu(torch.nn.functional.batch_norm(t, None, None, tg, tb, training=True, eps=1e-3))
    yy.backward(torch.from_numpy(g).double().permute(0, 3, 1, 2))
    dr, db, dg = orc.batch_norm_backward(raw, g, True, eps=1e-3, beta=beta)
    np.testing.assert_allclose(dr, t.grad.permute(0, 2, 3, 1).numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(db, tb.grad.numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(dg, tg.grad.numpy(), rtol=1e-10, atol=1e-12)
