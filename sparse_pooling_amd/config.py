"""SHPL configuration switches and feed keys, mirrored from the reference.

Field names and numbers are those of the reference protos, so existing
``.config`` files drive this build unchanged:

* ``RpnConfig``            (avod/avod/protos/model.proto:86-91)
      rpn_use_sparse_pooling = 6, rpn_sparse_pooling_use_batch_norm = 7,
      rpn_sparse_pooling_conv_after_fusion = 8 [default=true],
      rpn_sparse_pooling_after_vgg = 9, rpn_dual_sparse_pooling_after_vgg = 10
* ``RetinaNetConfig``      (model.proto:119-121)
      use_sparse_pooling = 6, use_pyramid_level_at_SHPL = 9 [default='P2']
* ``KittiDatasetConfig``   (avod/avod/protos/kitti_dataset.proto:38-40)
      output_indices = 11, use_pyramid_level_at_SHPL = 12 [default='P2']

There is no ``protoc`` here, so ``parse_text_config`` reads protobuf text
format directly (enough of it for the reference's config files).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, fields

import numpy as np

# Placeholder / feed keys (avod/avod/core/models/rpn_model.py:46-57,
# retinanet_model.py uses the first five).
PL_M_VAL = 'matrix_f2b_value'
PL_M_IJ = 'matrix_f2b_value_indices'
PL_M_SIZE = 'matrix_f2b_size'
PL_IMG_POOL_IJ = 'image_pool_indices'
PL_BEV_POOL_IJ = 'bev_pool_indices'
PL_M_VAL_VGG = 'matrix_f2b_value_after_vgg'
PL_M_IJ_VGG = 'matrix_f2b_value_indices_after_vgg'
PL_M_SIZE_VGG = 'matrix_f2b_size_after_vgg'
PL_IMG_POOL_IJ_VGG = 'image_pool_indices_after_vgg'
PL_BEV_POOL_IJ_VGG = 'bev_pool_indices_after_vgg'

# Sample-dict key (avod/avod/core/constants.py:19)
KEY_SPARSE_POOLING_INPUT = 'sparse_pooling_input'

# dtypes of the placeholders (rpn_model.py:220-242): numpy names
PLACEHOLDER_DTYPES = {
    PL_M_IJ: np.int64, PL_M_VAL: np.float32, PL_M_SIZE: np.int64,
    PL_IMG_POOL_IJ: np.int32, PL_BEV_POOL_IJ: np.int32,
}


@dataclass
class RpnConfig:
    rpn_use_sparse_pooling: bool = False                 # = 6
    rpn_sparse_pooling_use_batch_norm: bool = False      # = 7
    rpn_sparse_pooling_conv_after_fusion: bool = True    # = 8
    rpn_sparse_pooling_after_vgg: bool = False           # = 9
    rpn_dual_sparse_pooling_after_vgg: bool = False      # = 10


@dataclass
class RetinaNetConfig:
    use_sparse_pooling: bool = False                     # = 6
    use_pyramid_level_at_SHPL: str = 'P2'                # = 9


@dataclass
class KittiDatasetConfig:
    output_indices: bool = False                         # = 11
    use_pyramid_level_at_SHPL: str = 'P2'                # = 12


FIELD_NUMBERS = {
    "RpnConfig": {"rpn_use_sparse_pooling": 6, "rpn_sparse_pooling_use_batch_norm": 7,
                  "rpn_sparse_pooling_conv_after_fusion": 8, "rpn_sparse_pooling_after_vgg": 9,
                  "rpn_dual_sparse_pooling_after_vgg": 10},
    "RetinaNetConfig": {"use_sparse_pooling": 6, "use_pyramid_level_at_SHPL": 9},
    "KittiDatasetConfig": {"output_indices": 11, "use_pyramid_level_at_SHPL": 12},
}


# ------------------------------------------------------------ text format

_TOKEN = re.compile(r"""\s*(?:(\#[^\n]*)|([A-Za-z_][A-Za-z0-9_.]*)|("(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')|
                        ([-+]?(?:\d+\.?\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|inf|nan))|([{}\[\]:,;<>]))""",
                    re.X)


def _tokens(text):
    pos = 0
    out = []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ValueError(f"cannot parse config near: {text[pos:pos + 40]!r}")
        pos = m.end()
        if m.group(1):
            continue
        out.append(next(g for g in m.groups()[1:] if g is not None))
    return out


def _scalar(tok):
    if tok[0] in "\"'":
        return tok[1:-1]
    if tok in ("true", "True"):
        return True
    if tok in ("false", "False"):
        return False
    try:
        return int(tok)
    except ValueError:
        try:
            return float(tok)
        except ValueError:
            return tok  # enum identifier


def _parse_msg(toks, i, end):
    msg = {}
    while i < len(toks) and toks[i] != end:
        name = toks[i]
        i += 1
        if toks[i] == ":":
            i += 1
        if toks[i] in ("{", "<"):
            close = "}" if toks[i] == "{" else ">"
            sub, i = _parse_msg(toks, i + 1, close)
            msg.setdefault(name, []).append(sub)
            i += 1
        elif toks[i] == "[":
            i += 1
            vals = []
            while toks[i] != "]":
                if toks[i] == ",":
                    i += 1
                    continue
                if toks[i] == "{":
                    sub, i = _parse_msg(toks, i + 1, "}")
                    vals.append(sub)
                    i += 1
                else:
                    vals.append(_scalar(toks[i]))
                    i += 1
            msg.setdefault(name, []).extend(vals)
            i += 1
        else:
            msg.setdefault(name, []).append(_scalar(toks[i]))
            i += 1
        if i < len(toks) and toks[i] in (",", ";"):
            i += 1
    return msg, i


def parse_text_config(text):
    """protobuf text format -> nested dict {field: [values or sub-dicts]}."""
    msg, _ = _parse_msg(_tokens(text), 0, None)
    return msg


def _first(msg, *path):
    cur = msg
    for p in path:
        if not isinstance(cur, dict) or p not in cur:
            return None
        cur = cur[p][0]
    return cur


def _fill(cls, msg):
    obj = cls()
    if msg:
        for f in fields(cls):
            if f.name in msg:
                setattr(obj, f.name, msg[f.name][-1])
    return obj


@dataclass
class ShplConfig:
    rpn: RpnConfig
    retinanet: RetinaNetConfig
    dataset: KittiDatasetConfig
    model_name: str = ''


def load_shpl_config(text):
    """The SHPL-relevant switches of a reference pipeline config
    (model_config / dataset_config sections)."""
    msg = parse_text_config(text)
    mc = _first(msg, "model_config") or {}
    dc = _first(msg, "dataset_config") or {}
    return ShplConfig(rpn=_fill(RpnConfig, _first(mc, "rpn_config")),
                      retinanet=_fill(RetinaNetConfig, _first(mc, "retinanet_config")),
                      dataset=_fill(KittiDatasetConfig, dc),
                      model_name=_first(mc, "model_name") or '')


# ------------------------------------------------------------- guards

def rpn_uses_sparse_pooling(cfg: ShplConfig) -> bool:
    """RpnModel.__init__ (rpn_model.py:111-118): SHPL is silently disabled
    unless the dataset emits indices."""
    return bool(cfg.rpn.rpn_use_sparse_pooling and cfg.dataset.output_indices)


def retinanet_uses_sparse_pooling(cfg: ShplConfig) -> bool:
    """RetinanetModel.__init__ (retinanet_model.py:144)."""
    return bool(cfg.retinanet.use_sparse_pooling and cfg.dataset.output_indices)


def feat_stride(level: str) -> int:
    """KittiDataset.load_samples (kitti_dataset.py:375): 2 ** int(level[-1])."""
    return 2 ** int(level[-1])


def fill_sparse_pooling_feed(placeholder_inputs, sparse_pooling_inputs, use_sparse_pooling,
                             after_vgg=False, use_after_vgg=False):
    """RpnModel/RetinanetModel.create_feed_dict (rpn_model.py:841-868,
    retinanet_model.py:1206-1219): fill the five SHPL feeds from the
    dataset's sparse_pooling_input list, or with empty arrays when off.
    ``after_vgg`` also fills the *_after_vgg feeds from entry [1] (which the
    reference dataset never emits: an IndexError there)."""
    keys = [(PL_M_VAL, 'M_val'), (PL_M_IJ, 'Mij_pool'), (PL_M_SIZE, 'M_size'),
            (PL_IMG_POOL_IJ, 'img_index_flip_pool'), (PL_BEV_POOL_IJ, 'bev_index_flip_pool')]
    empty = {PL_M_VAL: np.zeros((0)), PL_M_IJ: np.zeros((0, 2)), PL_M_SIZE: np.zeros((2)),
             PL_IMG_POOL_IJ: np.zeros((0, 3)), PL_BEV_POOL_IJ: np.zeros((0, 3))}
    if use_sparse_pooling:
        sp = sparse_pooling_inputs[0]
        for pl, k in keys:
            placeholder_inputs[pl] = sp[k]
    else:
        placeholder_inputs.update(empty)
    if after_vgg:
        vgg = [(PL_M_VAL_VGG, PL_M_VAL), (PL_M_IJ_VGG, PL_M_IJ), (PL_M_SIZE_VGG, PL_M_SIZE),
               (PL_IMG_POOL_IJ_VGG, PL_IMG_POOL_IJ), (PL_BEV_POOL_IJ_VGG, PL_BEV_POOL_IJ)]
        if use_after_vgg:
            sp = sparse_pooling_inputs[1]
            for (pl, _), (_, k) in zip(vgg, keys):
                placeholder_inputs[pl] = sp[k]
        else:
            for pl, base in vgg:
                placeholder_inputs[pl] = empty[base]
    return placeholder_inputs
