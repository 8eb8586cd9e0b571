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
