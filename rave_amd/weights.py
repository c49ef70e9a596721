"""Weights: portable seeded init, checkpoint loading, weight-norm folding.

* ``init_params`` draws every parameter from its own numpy PCG64 stream keyed
  by (seed, crc32(reference name)), PyTorch-style ``U(-1/sqrt(fan_in),
  1/sqrt(fan_in))`` (fan_in from dim 1 x kernel, as torch computes it for both
  Conv1d and ConvTranspose1d weights).  Weight-norm gains are drawn around the
  norm of ``weight_v`` so the fold below is exercised, Snake ``alpha`` as
  ``1 + 0.1 N(0,1)`` and RVQ codebooks as ``N(0,1)``.
  Nothing has to be stored to reproduce a model: the golden fixtures, the
  oracle and the HIP path all rebuild the same tensors from the seed.
* ``fold_weight_norm`` is ``torch.nn.utils.weight_norm`` with ``dim=0``
  (rave/blocks.py:17-24, folded at export by scripts/export.py:598-600):
  ``w = g * v / ||v||`` with the norm over every dim but 0.  For a
  ConvTranspose1d dim 0 is ``in_channels`` (weight ``(C_in, C_out, k)``).
* ``load_checkpoint_state`` accepts a Lightning checkpoint dict (``state_dict``
  or ``callbacks.EMA``; scripts/export.py:558-569) or a bare state_dict, with
  the reference's strict=False semantics and weight-norm-folded weights.
"""
from __future__ import annotations

import zlib
from collections import OrderedDict
from typing import Dict, Mapping, Optional

import numpy as np

from .config import RaveConfig
from .graph import ConvNode, build_graph, param_shapes


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())]))


def init_params(cfg: RaveConfig, seed: int = 0, gain: float = 1.0) -> "OrderedDict[str, np.ndarray]":
    """Seeded random parameters under the reference's state_dict names.

    ``gain`` scales the uniform bound (1.0 = PyTorch's default init)."""
    shapes = param_shapes(cfg)
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for name, shape in shapes.items():
        rng = _rng(seed, name)
        if name.endswith(".weight_v") or name.endswith(".weight"):
            fan_in = shape[1] * int(np.prod(shape[2:]))
            b = gain / np.sqrt(fan_in)
            out[name] = rng.uniform(-b, b, size=shape).astype(np.float32)
        elif name.endswith(".weight_g"):
            continue  # drawn after its weight_v below
        elif name.endswith(".bias"):
            # fan_in of the owning weight
            base = name[: -len(".bias")]
            wshape = shapes.get(base + ".weight_v", shapes.get(base + ".weight"))
            fan_in = wshape[1] * int(np.prod(wshape[2:]))
            b = gain / np.sqrt(fan_in)
            out[name] = rng.uniform(-b, b, size=shape).astype(np.float32)
        elif name.endswith(".alpha"):
            out[name] = (1.0 + 0.1 * rng.standard_normal(size=shape)).astype(np.float32)
        elif name.endswith("._codebook.embed"):
            out[name] = rng.standard_normal(size=shape).astype(np.float32)
        else:
            raise KeyError(name)
    for name, shape in shapes.items():
        if name.endswith(".weight_g"):
            v = out[name[: -len("_g")] + "_v"].astype(np.float64)
            norm = np.sqrt((v.reshape(v.shape[0], -1) ** 2).sum(1)).reshape(shape)
            rng = _rng(seed, name)
            out[name] = (norm * rng.uniform(0.8, 1.2, size=shape)).astype(np.float32)
    # keep the reference's ordering (weight_g before weight_v)
    return OrderedDict((k, out[k]) for k in shapes)


def init_speaker(cfg: RaveConfig, seed: int = 0) -> np.ndarray:
    """Constant speaker embedding (rave/model.py:246-247 computes it once from
    an audio file with the pretrained SpeakerRAVE; here it is an input)."""
    return _rng(seed, "speaker").standard_normal(cfg.speaker_size).astype(np.float32)


def fold_weight_norm(g: np.ndarray, v: np.ndarray) -> np.ndarray:
    v64 = v.astype(np.float64)
    norm = np.sqrt((v64.reshape(v64.shape[0], -1) ** 2).sum(1))
    shape = (v.shape[0],) + (1,) * (v.ndim - 1)
    return (v64 * (g.astype(np.float64).reshape(shape) / norm.reshape(shape))).astype(np.float32)


def conv_weight(node: ConvNode, params: Mapping[str, np.ndarray]) -> np.ndarray:
    """Effective weight of one conv node in the torch layout
    ((C_out, C_in, k) for Conv1d, (C_in, C_out, k) for ConvTranspose1d)."""
    if node.weight_norm:
        return fold_weight_norm(np.asarray(params[node.name + ".weight_g"]),
                                np.asarray(params[node.name + ".weight_v"]))
    return np.asarray(params[node.name + ".weight"], dtype=np.float32)


def to_numpy_state(state: Mapping) -> Dict[str, np.ndarray]:
    out = {}
    for k, v in state.items():
        if hasattr(v, "detach"):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    return out


def load_checkpoint_state(ckpt: Mapping, use_ema: bool = False, cfg: Optional[RaveConfig] = None,
                          base: Optional[Mapping[str, np.ndarray]] = None) -> Dict[str, np.ndarray]:
    """Parameter dict from a Lightning checkpoint (scripts/export.py:558-569).

    * ``use_ema`` and an ``EMA`` entry under ``checkpoint["callbacks"]`` -> the
      EMA callback's weights, else ``checkpoint["state_dict"]`` (a bare
      state_dict is accepted too), as export.py chooses.
    * Without ``cfg`` every entry is returned (numpy).  With ``cfg`` the result
      holds exactly the hot path's parameters (graph.param_shapes), shapes
      checked.  Like the reference's ``load_state_dict(..., strict=False)``,
      keys of other modules (speaker encoder, discriminators) are ignored and
      a parameter the checkpoint lacks keeps its value in ``base`` (the EMA
      callback stores parameters only, not buffers such as RVQ codebooks);
      without ``base`` a missing parameter raises KeyError.
    * A weight already folded by ``remove_weight_norm`` (``<name>.weight``
      where the graph holds ``weight_g`` / ``weight_v``, scripts/export.py:
      598-600) is taken as ``weight_v = weight``, ``weight_g = ||weight||``
      (norm over every dim but 0), which folds back to the same weight."""
    callbacks = ckpt.get("callbacks") if isinstance(ckpt, Mapping) else None
    if use_ema and isinstance(callbacks, Mapping) and "EMA" in callbacks:
        state = callbacks["EMA"]
    elif "state_dict" in ckpt:
        state = ckpt["state_dict"]
    else:
        state = ckpt
    state = to_numpy_state(state)
    if cfg is None:
        return state
    out: Dict[str, np.ndarray] = {}
    for name, shape in param_shapes(cfg).items():
        if name in state:
            val = np.asarray(state[name], np.float32)
        elif name.endswith((".weight_g", ".weight_v")) and name.rsplit(".", 1)[0] + ".weight" in state:
            w = np.asarray(state[name.rsplit(".", 1)[0] + ".weight"], np.float32)
            if name.endswith("_v"):
                val = w
            else:
                w64 = w.astype(np.float64)
                val = np.sqrt((w64.reshape(w64.shape[0], -1) ** 2).sum(1)).reshape(shape).astype(np.float32)
        elif base is not None and name in base:
            val = np.asarray(base[name], np.float32)
        else:
            raise KeyError(f"checkpoint has no parameter {name} (and no base value was given)")
        if tuple(val.shape) != tuple(shape):
            raise ValueError(f"{name}: expected shape {shape}, got {val.shape}")
        out[name] = val
    return out


def check_params(cfg: RaveConfig, params: Mapping[str, np.ndarray]) -> None:
    """Raise if a hot-path parameter is missing or has the wrong shape."""
    for name, shape in param_shapes(cfg).items():
        if name not in params:
            raise KeyError(f"missing parameter {name}")
        if tuple(np.shape(params[name])) != tuple(shape):
            raise ValueError(f"{name}: expected shape {shape}, got {np.shape(params[name])}")
