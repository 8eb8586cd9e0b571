"""SHPL config switches, guards and feed filling (CPU only)."""
import os

import numpy as np
import pytest

from sparse_pooling_amd import config as C

RETINA = """
# comment
model_config {
    model_name: 'retinanet_model'
    input_config { bev_depth: 3 img_dims_w: 1200 }
    retinanet_config {
        nms_iou_thresh: 0.3
        nms_size: 100
        use_sparse_pooling: True
        use_pyramid_level_at_SHPL: 'P2'
    }
    layers_config { bev_feature_extractor { bev_resnet_fpn { pyramid_levels: ['P2', 'P3', 'P4'], load_from_pretrained: True } } }
}
dataset_config {
    name: 'kitti'
    aug_list: []
    output_indices: True
    use_pyramid_level_at_SHPL: 'P3'
    kitti_utils_config { area_extents: [-40, 40, -5, 3, 0, 70] voxel_size: 0.1 }
}
"""

RPN = """
model_config {
    model_name: 'avod_model'
    rpn_config {
        rpn_proposal_roi_crop_size: 3
        rpn_use_sparse_pooling: True
        rpn_sparse_pooling_use_batch_norm: False
        rpn_sparse_pooling_after_vgg: True
        rpn_dual_sparse_pooling_after_vgg: False
    }
}
dataset_config { output_indices: False }
"""


def test_text_format_parser():
    m = C.parse_text_config(RETINA)
    assert m["model_config"][0]["model_name"] == ["retinanet_model"]
    ext = m["dataset_config"][0]["kitti_utils_config"][0]["area_extents"]
    assert ext == [-40, 40, -5, 3, 0, 70]
    assert m["dataset_config"][0]["aug_list"] == []


def test_retinanet_switches_and_stride():
    cfg = C.load_shpl_config(RETINA)
    assert cfg.retinanet.use_sparse_pooling is True
    assert cfg.retinanet.use_pyramid_level_at_SHPL == 'P2'
    assert cfg.dataset.output_indices is True
    assert C.retinanet_uses_sparse_pooling(cfg)
    assert C.feat_stride(cfg.dataset.use_pyramid_level_at_SHPL) == 8


def test_rpn_switches_defaults_and_guard():
    cfg = C.load_shpl_config(RPN)
    assert cfg.rpn.rpn_use_sparse_pooling is True
    assert cfg.rpn.rpn_sparse_pooling_conv_after_fusion is True  # proto default
    assert cfg.rpn.rpn_sparse_pooling_after_vgg is True
    # rpn_model.py:111-118: silently off without dataset indices
    assert not C.rpn_uses_sparse_pooling(cfg)


def test_field_numbers_match_reference_protos():
    assert C.FIELD_NUMBERS["RpnConfig"]["rpn_use_sparse_pooling"] == 6
    assert C.FIELD_NUMBERS["RpnConfig"]["rpn_dual_sparse_pooling_after_vgg"] == 10
    assert C.FIELD_NUMBERS["RetinaNetConfig"]["use_pyramid_level_at_SHPL"] == 9
    assert C.FIELD_NUMBERS["KittiDatasetConfig"]["output_indices"] == 11


def test_feed_fill_on_and_off():
    sp = {"M_val": np.ones(3), "Mij_pool": np.zeros((3, 2), np.int64), "M_size": np.array([10, 3]),
          "img_index_flip_pool": np.zeros((3, 3), np.int64), "bev_index_flip_pool": np.zeros((0, 3))}
    feed = C.fill_sparse_pooling_feed({}, [sp], True)
    assert feed[C.PL_M_IJ] is sp["Mij_pool"] and feed[C.PL_M_SIZE] is sp["M_size"]
    off = C.fill_sparse_pooling_feed({}, None, False, after_vgg=True)
    assert off[C.PL_M_VAL].shape == (0,) and off[C.PL_IMG_POOL_IJ_VGG].shape == (0, 3)
    with pytest.raises(IndexError):  # the reference dataset emits one entry only
        C.fill_sparse_pooling_feed({}, [sp], True, after_vgg=True, use_after_vgg=True)


REF_CFG = "/root/reference/avod/avod/configs"


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference configs only in the survey container")
def test_parses_every_reference_config():
    n = 0
    for name in sorted(os.listdir(REF_CFG)):
        if name.endswith(".config"):
            cfg = C.load_shpl_config(open(os.path.join(REF_CFG, name)).read())
            assert isinstance(cfg.dataset.output_indices, bool)
            n += 1
    assert n > 10
    shpl = C.load_shpl_config(open(os.path.join(REF_CFG, "retinanet_car_SHPL.config")).read())
    assert C.retinanet_uses_sparse_pooling(shpl)


def test_mv3d_calib_to_P_matches_reference(golden_dir):
    """MV3D transform.calib_to_P / calib_to_L2C (transform.py:13-30) vs the reference run."""
    import numpy as np
    from sparse_pooling_amd import mv3d
    g = np.load(os.path.join(golden_dir, "mv3d_calib.npz"))
    np.testing.assert_array_equal(mv3d.calib_to_P(g["calib"]), g["P"])
    np.testing.assert_array_equal(mv3d.calib_to_P(g["calib"], from_camera=True), g["P_cam"])
    np.testing.assert_array_equal(mv3d.calib_to_L2C(g["calib"]), g["L2C"])
