"""The per-frame checksums bench.py reports (dist.frame_checksums) and the oracle tables it compares them with.

* the checksum is exact (integer arithmetic mod 2^64), independent of the batch, and sees positions: a row
  moved to another cell, two channels exchanged or two outputs swapped change it (the plain
  bit-pattern sum it replaced was blind to every permutation);
* the host mirror (frame_checksum_np, feature_values_np) equals the torch form bit for bit;
* profiles/frame_checksums.json's oracle tables hold, for a sample of their frames, the oracle's checksum of
  the bench's inputs for that global frame id (tests/checksum_tables.py; the generator
  tests/golden/make_checksum_tables.py computes every frame)."""
import json
import os

import numpy as np
import pytest
import torch

import checksum_tables as ct
from sparse_pooling_amd import dist as sd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table(key):
    with open(os.path.join(ROOT, "profiles", "frame_checksums.json")) as fh:
        return json.load(fh)[key]


def test_checksum_sees_row_and_channel_permutations():
    x = torch.randn(2, 6, 5, 8)
    cs = sd.frame_checksums(x)
    assert cs.dtype == torch.int64 and cs.shape == (2,)
    assert torch.equal(sd.frame_checksums(x[1:]), cs[1:])       # batch-independent
    rows = x.clone()
    rows[1, 2, 3], rows[1, 4, 0] = x[1, 4, 0], x[1, 2, 3]       # two pooled rows in each other's cells
    chans = x.clone()
    chans[1, ..., [2, 5]] = x[1, ..., [5, 2]]                   # two channels exchanged
    moved = x.clone()
    moved[1, 5, 4] = 0.0
    moved2 = moved.clone()
    moved2[1, 0, 0], moved2[1, 5, 4] = moved[1, 5, 4], moved[1, 0, 0]  # a row written to the wrong (empty) cell
    for y in (rows, chans):
        c = sd.frame_checksums(y)
        assert c[0] == cs[0] and c[1] != cs[1]
        # the plain bit sum of round 4 could not tell them apart
        assert y[1].view(torch.int32).to(torch.int64).sum() == x[1].view(torch.int32).to(torch.int64).sum()
    assert sd.frame_checksums(moved2)[1] != sd.frame_checksums(moved)[1]
    y = x.clone()
    y[1, 4, 2, 7] = torch.nextafter(y[1, 4, 2, 7], torch.tensor(1e9))  # one ulp in one element
    assert sd.frame_checksums(y)[1] != cs[1]
    b = x.to(torch.bfloat16)
    bs = sd.frame_checksums(b)
    bc = b.clone()
    bc[0, ..., [0, 1]] = b[0, ..., [1, 0]]
    assert sd.frame_checksums(bc)[0] != bs[0]


def test_combined_outputs_see_an_exchange():
    a, b = torch.randn(1, 4, 4, 2), torch.randn(1, 4, 4, 2)
    ca, cb = sd.frame_checksums(a), sd.frame_checksums(b)
    assert sd.combine_checksums([ca, cb]) != sd.combine_checksums([cb, ca])
    assert int(sd.combine_checksums([ca, cb])[0]) == sd.combine_checksums_int([int(ca[0]), int(cb[0])])


@pytest.mark.parametrize("bf16", [False, True])
def test_host_mirror_equals_torch(bf16):
    shape = (3, 7, 9, 16)
    dt = torch.bfloat16 if bf16 else torch.float32
    t = sd.fill_features(torch.empty((2,) + shape, dtype=dt), [11, 5], 3)
    for i, fid in enumerate((11, 5)):
        a = sd.feature_values_np(shape, fid, 3)
        if bf16:
            assert torch.equal(t[i], torch.from_numpy(a).to(torch.bfloat16))
        else:
            assert np.array_equal(t[i].numpy(), a)
        assert sd.frame_checksum_np(t[i].float().numpy(), bf16=bf16) == int(sd.frame_checksums(t[i:i + 1])[0])
    # large values: the products wrap mod 2^64 the same way on both sides
    x = torch.randn(1, 1 << 12, 64) * 3e38
    assert sd.frame_checksum_np(x[0].numpy()) == int(sd.frame_checksums(x)[0])


def test_features_are_frame_and_stream_keyed():
    a = sd.feature_values_np((64, 32), 0, 1)
    assert not np.array_equal(a, sd.feature_values_np((64, 32), 1, 1))
    assert not np.array_equal(a, sd.feature_values_np((64, 32), 0, 2))
    assert -1.0 <= a.min() and a.max() < 1.0 and abs(float(a.mean())) < 0.05


@pytest.mark.parametrize("key,fids", [("layer_config2_frames64", [0, 41]), ("layer_config3_frames4", [0, 3]),
                                      ("layer_config5_frames64", [17]), ("layer_config6_frames64", [0, 63]),
                                      ("frames_120000_frames64", [9])])
def test_stored_table_equals_oracle(key, fids):
    table = _table(key)
    assert len(table) == ct.ORACLE_TABLES[key] and len(set(table)) == len(table)
    for f in fids:
        assert table[f] == ct.table_entry(key, f), f"{key} frame {f}"
