"""Host-side pieces of the product that need no GPU: PQMF design (init-time,
rave_amd/pqmf.py) and the checkpoint loader (rave_amd/weights.py)."""
import hashlib

import numpy as np
import pytest
import torch

from rave_amd import config as rcfg
from rave_amd.pqmf import design_bank
from rave_amd.weights import conv_weight, fold_weight_norm, init_params, load_checkpoint_state
from rave_amd.graph import build_graph


def test_design_bank_bit_exact(golden):
    """get_qmf_bank's float32 torch arithmetic (rave/pqmf.py:32-52) reproduced
    bit for bit: the product's hk is the reference's hk."""
    hk = design_bank(100.0, 16)
    g = golden("pqmf")["hk"]
    assert hk.dtype == np.float32 and hk.shape == (16, 512)
    assert np.array_equal(hk, g)
    assert hashlib.sha256(hk.tobytes()).hexdigest()[:16] == "4d86cced7ee86762"


def _lightning(params, scale=1.0):
    """A Lightning-style checkpoint (scripts/train.py: state_dict + callback
    states), with torch tensors and keys of modules outside the hot path."""
    sd = {k: torch.from_numpy(np.asarray(v) * scale) for k, v in params.items()}
    sd["speaker_encoder.net.0.weight"] = torch.zeros(4, 4)
    sd["discriminator.convs.0.weight"] = torch.zeros(2)
    return sd


def test_checkpoint_state_dict_and_ema():
    cfg = rcfg.discrete(capacity=4)
    p = init_params(cfg, 0)
    ema = {k: v for k, v in _lightning(p, 0.5).items() if not k.endswith("_codebook.embed")}
    ckpt = {"state_dict": _lightning(p), "callbacks": {"EMA": ema, "ModelCheckpoint": {}}}
    a = load_checkpoint_state(ckpt, cfg=cfg)
    assert set(a) == set(p)
    assert all(np.array_equal(a[k], p[k]) for k in p)
    # EMA: parameters only; the codebook buffers keep the base values (strict=False)
    base = init_params(cfg, 1)
    b = load_checkpoint_state(ckpt, use_ema=True, cfg=cfg, base=base)
    w = [k for k in p if k.endswith(".weight_v")][0]
    assert np.allclose(b[w], 0.5 * p[w])
    cb = "encoder.rvq.layers.0._codebook.embed"
    assert np.array_equal(b[cb], base[cb])
    with pytest.raises(KeyError):
        load_checkpoint_state(ckpt, use_ema=True, cfg=cfg)       # no base for the buffers
    # use_ema without an EMA entry falls back to state_dict (export.py:559-569)
    c = load_checkpoint_state({"state_dict": _lightning(p), "callbacks": {}}, use_ema=True, cfg=cfg)
    assert np.array_equal(c[w], p[w])


def test_checkpoint_folded_weight_norm():
    """A state_dict after remove_weight_norm (scripts/export.py:598-600) holds
    <name>.weight; it loads into weight_g / weight_v that fold back to it."""
    cfg = rcfg.v2(capacity=4)
    p = init_params(cfg, 0)
    g = build_graph(cfg)
    folded = {}
    for k, v in p.items():
        if k.endswith(".weight_g"):
            continue
        if k.endswith(".weight_v"):
            n = k[:-len(".weight_v")]
            folded[n + ".weight"] = fold_weight_norm(p[n + ".weight_g"], v)
        else:
            folded[k] = v
    q = load_checkpoint_state(folded, cfg=cfg)
    for node in g.convs():
        np.testing.assert_allclose(conv_weight(node, q), conv_weight(node, p), rtol=2e-7, atol=1e-8)
    bad = dict(folded)
    bad[next(k for k in folded if k.endswith(".bias"))] = np.zeros(3, np.float32)
    with pytest.raises(ValueError):
        load_checkpoint_state(bad, cfg=cfg)
