#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the reference itself.

Runs ONLY in the build container (needs /root/reference).  It path-imports
``rave/{pqmf,core,blocks,quantization}.py`` as submodules of a synthetic
``rave`` package (``rave/__init__.py`` is not executed: it imports model.py,
whose module level loads a missing audio file, rave/model.py:29), with:

1. scipy shims: ``scipy.signal.kaiser`` -> ``scipy.signal.windows.kaiser`` and
   ``firwin(nyq=pi)`` -> ``fs=2*pi`` (scipy 1.15 here vs 1.10 pinned,
   requirements.txt:10; used at rave/pqmf.py:10,69);
2. a gin stub (refshim/gin.py) -- the .gin bindings are applied explicitly below;
3. empty stand-ins for GPUtil, librosa, lmdb, pytorch_lightning, torchaudio
   (imported at module level by rave/core.py:7-15 and rave/blocks.py:10, never
   called on the hot path);
4. refshim/cached_conv.py, a restatement of the unvendored cached_conv API.

Weights come from rave_amd.weights.init_params (seeded, portable); they are
loaded into the reference modules under the reference's own state_dict names,
so the fixtures store only inputs and outputs.  Nothing of the reference's
source is copied into the repo; the fixtures are data.

Usage:  python tests/golden/make_golden.py  [--out tests/golden]
"""
from __future__ import annotations

import argparse
import functools
import hashlib
import importlib
import json
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

sys.path.insert(0, REPO)
from rave_amd import config as rcfg  # noqa: E402
from rave_amd.graph import build_graph, param_shapes  # noqa: E402
from rave_amd.weights import init_params, init_speaker  # noqa: E402


# --------------------------------------------------------------------------- shims
def install_shims():
    sys.path.insert(0, os.path.join(HERE, "refshim"))
    import cached_conv  # noqa: F401  (refshim restatement)
    import gin  # noqa: F401  (refshim stub)
    import scipy.signal as ss
    import scipy.signal.windows as ssw

    if not hasattr(ss, "kaiser"):
        ss.kaiser = ssw.kaiser
    _firwin = ss.firwin

    def firwin(*args, nyq=None, **kw):
        if nyq is not None:
            kw["fs"] = 2 * nyq
        return _firwin(*args, **kw)

    ss.firwin = firwin

    def stub(name, **attrs):
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    class _Dummy:  # placeholder classes for annotations / base classes
        def __init__(self, *a, **k):
            pass

    stub("GPUtil")
    stub("librosa")
    stub("lmdb")
    stub("pytorch_lightning", Callback=_Dummy, LightningModule=nn.Module)
    ta = stub("torchaudio")
    ta.transforms = stub("torchaudio.transforms", Spectrogram=_Dummy)
    ta.functional = stub("torchaudio.functional")

    pkg = types.ModuleType("rave")
    pkg.__path__ = [os.path.join(REF, "rave")]
    sys.modules["rave"] = pkg
    mods = {}
    for name in ("pqmf", "core", "blocks", "quantization", "CombinedRave", "resampler"):
        mods[name] = importlib.import_module(f"rave.{name}")
    return mods


# --------------------------------------------------------------------------- model
def build_reference(mods, cfg: rcfg.RaveConfig, cached: bool):
    """Instantiate the reference modules for ``cfg`` with the gin bindings of
    v1/v2/causal/discrete/snake/adain/noise.gin applied explicitly."""
    import cached_conv as cc
    from torch.nn.utils import weight_norm

    blocks, pqmf, quant = mods["blocks"], mods["pqmf"], mods["quantization"]
    cc.use_cached_conv(cached)
    cc.set_padding_mode("causal" if cfg.causal else "centered")
    # v1.gin:41 blocks.normalization.mode = 'weight_norm'
    blocks.normalization = lambda module, mode="weight_norm": weight_norm(module)
    if cfg.activation == "snake":
        act = lambda dim: blocks.Snake(dim)  # noqa: E731
    else:
        act = lambda dim: nn.LeakyReLU(.2)  # noqa: E731
    # snake.gin:10-11 binds DilatedUnit's own activation
    if not hasattr(blocks, "_DilatedUnit"):
        blocks._DilatedUnit = blocks.DilatedUnit
    blocks.DilatedUnit = functools.partial(blocks._DilatedUnit, activation=act)
    adain = blocks.AdaptiveInstanceNormalization if cfg.adain else None

    def enc():
        return blocks.EncoderV2(data_size=cfg.enc_bands, capacity=cfg.capacity,
                                ratios=list(cfg.ratios), latent_size=cfg.latent_size, n_out=1,
                                kernel_size=cfg.kernel_size,
                                dilations=[list(d) for d in cfg.dilations],
                                activation=act, adain=adain)

    m = nn.Module()
    m.pqmf = pqmf.CachedPQMF(attenuation=cfg.pqmf_attenuation, n_band=cfg.n_band)
    if cfg.rvq is not None:
        m.encoder = blocks.DiscreteEncoder(
            encoder_cls=enc,
            vq_cls=lambda: quant.ResidualVectorQuantization(
                num_quantizers=cfg.rvq.num_quantizers, dim=cfg.latent_size,
                codebook_size=cfg.rvq.codebook_size),
            num_quantizers=cfg.rvq.num_quantizers)
    else:
        m.encoder = blocks.VariationalEncoder(enc)
    noise_module = None
    if cfg.noise is not None:
        noise_module = functools.partial(blocks.NoiseGeneratorV2, hidden_size=cfg.noise.hidden_size,
                                         data_size=cfg.n_band, ratios=list(cfg.noise.ratios),
                                         noise_bands=cfg.noise.noise_bands, activation=act)
    m.decoder = blocks.GeneratorV2(data_size=cfg.n_band, capacity=cfg.capacity,
                                   ratios=list(cfg.ratios), latent_size=cfg.dec_in,
                                   kernel_size=cfg.kernel_size,
                                   dilations=[list(d) for d in cfg.dilations],
                                   amplitude_modulation=cfg.amplitude_modulation,
                                   noise_module=noise_module, activation=act, adain=adain)
    m.eval()
    return m


def load_params(m: nn.Module, cfg, params):
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in params.items()}
    ref_params = dict(m.named_parameters())
    ref_buffers = dict(m.named_buffers())
    for k in sd:
        if k not in ref_params and k not in ref_buffers:
            raise KeyError(f"name mapping broken: {k} not in reference module")
    missing = [k for k in ref_params if k not in sd and not k.startswith("pqmf.")]
    if missing:
        raise KeyError(f"reference parameters not covered by rave_amd.graph: {missing[:5]}")
    m.load_state_dict(sd, strict=False)


def ref_encode(m, cfg, x, speaker):
    y = m.pqmf(x)
    z = m.encoder(y[:, :cfg.enc_bands, :])
    if cfg.rvq is not None:
        return z
    emb = speaker.reshape(1, -1, 1).repeat(z.shape[0], 1, z.shape[-1])
    return torch.cat((z, emb), 1)


def ref_decode(m, z):
    return m.pqmf.inverse(m.decoder(z))


def synth_audio(batch, t, seed0=0):
    n = np.arange(t)
    out = []
    for b in range(batch):
        rng = np.random.Generator(np.random.PCG64(seed0 + b))
        out.append(0.3 * np.sin(2 * np.pi * 440 * n / 48000) + 0.1 * rng.standard_normal(t))
    return np.stack(out)[:, None, :].astype(np.float32)


class NoiseInjector:
    """Replaces torch.rand_like inside NoiseGeneratorV2.forward (rave/blocks.py:287)."""

    def __init__(self, u01: torch.Tensor):
        self.u = u01
        self.orig = torch.rand_like

    def __enter__(self):
        def fake(t, *a, **k):
            assert tuple(t.shape) == tuple(self.u.shape), (t.shape, self.u.shape)
            return self.u.clone()
        torch.rand_like = fake

    def __exit__(self, *a):
        torch.rand_like = self.orig


def conv_hooks(m, cfg):
    names = {n.name for n in build_graph(cfg).convs()}
    store = {}
    hs = []
    for name, mod in m.named_modules():
        if name in names:
            hs.append(mod.register_forward_hook(
                lambda mod, inp, out, name=name: store.__setitem__(name, out.detach().numpy().copy())))
    return store, hs


# --------------------------------------------------------------------------- fixtures
def gen_pqmf(mods, out):
    import cached_conv as cc
    res = {}
    for mode in ("centered", "causal"):
        cc.use_cached_conv(False)
        cc.set_padding_mode(mode)
        p = mods["pqmf"].CachedPQMF(attenuation=100, n_band=16)
        if mode == "centered":
            res["hk"] = p.hk.numpy()
            res["h"] = p.h.numpy()
        x = torch.from_numpy(synth_audio(2, 4096, seed0=100))
        rng = np.random.Generator(np.random.PCG64(7))
        bands = torch.from_numpy(rng.standard_normal((2, 16, 256)).astype(np.float32))
        with torch.no_grad():
            res[f"x"] = x.numpy()
            res[f"bands"] = bands.numpy()
            res[f"analysis_{mode}"] = p(x).numpy()
            res[f"synthesis_{mode}"] = p.inverse(bands).numpy()
            res[f"roundtrip_{mode}"] = p.inverse(p(x)).numpy()
    np.savez_compressed(os.path.join(out, "pqmf.npz"), **res)
    return res


def gen_model(mods, cfg, out, fname, batch=2, t=8192, per_layer=False, seed=0):
    import cached_conv as cc
    m = build_reference(mods, cfg, cached=False)
    params = init_params(cfg, seed=seed)
    load_params(m, cfg, params)
    speaker = torch.from_numpy(init_speaker(cfg, seed=seed))
    x = torch.from_numpy(synth_audio(batch, t))
    res = {"x": x.numpy(), "speaker": speaker.numpy(), "seed": np.int64(seed)}
    store, hs = conv_hooks(m, cfg) if per_layer else ({}, [])
    noise_u = None
    with torch.no_grad():
        if cfg.rvq is not None:
            ze = ref_encode(m, cfg, x, speaker)
            idx = m.encoder.rvq.encode(ze)
            zq = m.encoder.rvq.decode(idx)
            emb = speaker.reshape(1, -1, 1).repeat(zq.shape[0], 1, zq.shape[-1])
            z = torch.cat((zq, emb), 1)
            res.update(z_enc=ze.numpy(), rvq_idx=idx.numpy(), z_q=zq.numpy())
            # top-2 gap of every quantizer decision (tie-margin rule for index parity)
            res["rvq_gap"] = rvq_gaps(m.encoder.rvq, ze)
        else:
            z = ref_encode(m, cfg, x, speaker)
        if cfg.noise is not None:
            frames = z.shape[-1] * cfg.hop // cfg.n_band
            n_fr = frames // int(np.prod(cfg.noise.ratios))
            ir = (z.shape[0], n_fr, cfg.n_band, 2 * (cfg.noise.noise_bands - 1))
            rng = np.random.Generator(np.random.PCG64(11))
            noise_u = torch.from_numpy(rng.uniform(0, 1, size=ir).astype(np.float32))
            res["noise_u"] = noise_u.numpy()
            with NoiseInjector(noise_u):
                y = ref_decode(m, z)
        else:
            y = ref_decode(m, z)
    for h in hs:
        h.remove()
    res.update(z=z.numpy(), y=y.numpy())
    for k, v in store.items():
        res["layer/" + k] = v
    np.savez_compressed(os.path.join(out, fname), **res)
    return res, m, params, speaker


def rvq_gaps(rvq, z):
    residual = z
    gaps = []
    for layer in rvq.layers:
        x = residual.permute(0, 2, 1).reshape(-1, residual.shape[1])
        embed = layer._codebook.embed.t()
        dist = -(x.pow(2).sum(1, keepdim=True) - 2 * x @ embed + embed.pow(2).sum(0, keepdim=True))
        top2 = dist.topk(2, dim=-1).values
        gaps.append((top2[:, 0] - top2[:, 1]).numpy())
        ind = layer.encode(residual)
        residual = residual - layer.decode(ind)
    return np.stack(gaps, 0)


def gen_rvq(mods, out, seed=0):
    """RVQ encode/decode on N(0,1) latents (the encoder-fed case in discrete.npz
    sits near the codebook origin; this one spreads the decisions)."""
    cfg = rcfg.discrete()
    m = build_reference(mods, cfg, cached=False)
    load_params(m, cfg, init_params(cfg, seed=seed))
    rng = np.random.Generator(np.random.PCG64(21))
    z = torch.from_numpy(rng.standard_normal((4, cfg.latent_size, 16)).astype(np.float32))
    with torch.no_grad():
        idx = m.encoder.rvq.encode(z)
        zq = m.encoder.rvq.decode(idx)
        gaps = rvq_gaps(m.encoder.rvq, z)
    np.savez_compressed(os.path.join(out, "rvq.npz"), z=z.numpy(), idx=idx.numpy(), zq=zq.numpy(),
                        gap=gaps, seed=np.int64(seed))


def gen_streaming(mods, cfg, out, seed=0, n_blocks=12, block=2048, fname="causal_stream.npz"):
    """Cached-conv streaming of the reference (cc.use_cached_conv(True)), causal
    or centred padding (the latter is the reference's default model exported
    with --streaming, README.md:187-190), next to the one-shot outputs."""
    m_s = build_reference(mods, cfg, cached=True)
    params = init_params(cfg, seed=seed)
    load_params(m_s, cfg, params)
    m_o = build_reference(mods, cfg, cached=False)
    load_params(m_o, cfg, params)
    speaker = torch.from_numpy(init_speaker(cfg, seed=seed))
    x = torch.from_numpy(synth_audio(1, n_blocks * block, seed0=3))
    frames = block // cfg.hop
    rng = np.random.Generator(np.random.PCG64(5))
    zlat = rng.standard_normal((1, cfg.latent_size, n_blocks * frames)).astype(np.float32)
    z = torch.cat([torch.from_numpy(zlat),
                   speaker.reshape(1, -1, 1).repeat(1, 1, zlat.shape[-1])], 1)
    res = {"x": x.numpy(), "z": z.numpy(), "speaker": speaker.numpy(),
           "block": np.int64(block), "seed": np.int64(seed)}
    with torch.no_grad():
        zs, ys, ys_rt = [], [], []
        for i in range(n_blocks):
            zs.append(ref_encode(m_s, cfg, x[..., i * block:(i + 1) * block], speaker))
        for i in range(n_blocks):
            ys.append(ref_decode(m_s, z[..., i * frames:(i + 1) * frames]))
        res["z_stream"] = torch.cat(zs, -1).numpy()
        res["y_stream"] = torch.cat(ys, -1).numpy()
        res["z_oneshot"] = ref_encode(m_o, cfg, x, speaker).numpy()
        res["y_oneshot"] = ref_decode(m_o, z).numpy()
    np.savez_compressed(os.path.join(out, fname), **res)
    return res


def gen_stream_discrete(mods, cfg, out, seed=0, n_blocks=8, block=2048, fname="discrete_stream.npz"):
    """DiscreteScriptedRAVE streamed (scripts/export.py:503-517 under
    cc.use_cached_conv(True)): per block, PQMF -> encoder -> rvq.encode
    (post_process_latent) with the top-2 gaps of every decision (tie margin),
    and, in a separate pass over fresh caches, the reference's own streamed
    codes -> rvq.decode (pre_process_latent's clamp) -> speaker concat ->
    decoder -> PQMF inverse."""
    m = build_reference(mods, cfg, cached=True)
    params = init_params(cfg, seed=seed)
    load_params(m, cfg, params)
    speaker = torch.from_numpy(init_speaker(cfg, seed=seed))
    x = torch.from_numpy(synth_audio(1, n_blocks * block, seed0=17))
    frames = block // cfg.hop
    res = {"x": x.numpy(), "speaker": speaker.numpy(), "block": np.int64(block), "seed": np.int64(seed)}
    with torch.no_grad():
        idxs, gaps = [], []
        for i in range(n_blocks):
            ze = ref_encode(m, cfg, x[..., i * block:(i + 1) * block], speaker)
            idxs.append(m.encoder.rvq.encode(ze))
            gaps.append(rvq_gaps(m.encoder.rvq, ze).reshape(cfg.rvq.num_quantizers, 1, frames))
        idx = torch.cat(idxs, -1)
        m2 = build_reference(mods, cfg, cached=True)     # fresh caches for the decoder pass
        load_params(m2, cfg, params)
        ys = []
        for i in range(n_blocks):
            zq = m2.encoder.rvq.decode(torch.clamp(idx[..., i * frames:(i + 1) * frames], 0,
                                                   cfg.rvq.codebook_size - 1).long())
            emb = speaker.reshape(1, -1, 1).repeat(zq.shape[0], 1, zq.shape[-1])
            ys.append(ref_decode(m2, torch.cat((zq, emb), 1)))
    res["idx_stream"] = idx.numpy()
    res["gap_stream"] = np.concatenate(gaps, -1)
    res["y_stream"] = torch.cat(ys, -1).numpy()
    np.savez_compressed(os.path.join(out, fname), **res)
    return res


def write_manifest(out, extra=None):
    """Hash every fixture (tests/golden/*.npz) into MANIFEST.json, keeping the
    keys an earlier full run wrote."""
    path = os.path.join(out, "MANIFEST.json")
    manifest = {}
    if os.path.exists(path):
        with open(path) as fh:
            manifest = json.load(fh)
    manifest.update(extra or {})
    manifest["generator"] = "tests/golden/make_golden.py"
    manifest["reference"] = "abargum/RAVE @ 2024-10-16 (path-imported, see docstring)"
    manifest["torch"] = torch.__version__
    files = sorted(f for f in os.listdir(out) if f.endswith(".npz"))
    manifest["files"] = {f: hashlib.sha256(open(os.path.join(out, f), "rb").read()).hexdigest()[:16]
                         for f in files}
    with open(path, "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    return manifest


def gen_stream_v3(mods, cfg, out, fname="v3_noise_causal_stream.npz", seed=0, n_blocks=6, block=2048):
    """Cached-conv streaming (cc.use_cached_conv(True)) of a causal v3 model with
    the noise synthesizer and AdaIN, block by block: blocks 0-1 learn the target
    statistics (learn_y), 2-3 learn the source (learn_x; the transfer turns on),
    4-5 transfer with frozen statistics -- the nn~ learn_target / learn_source
    sequence (scripts/export.py:248-265).  Encoder and decoder are streamed in
    separate passes over fresh caches; the decoder's uniform noise is injected
    per block (torch.rand_like, rave/blocks.py:287)."""
    m = build_reference(mods, cfg, cached=True)
    params = init_params(cfg, seed=seed)
    load_params(m, cfg, params)
    speaker = torch.from_numpy(init_speaker(cfg, seed=seed))
    x = torch.from_numpy(synth_audio(1, n_blocks * block, seed0=9))
    frames = block // cfg.hop
    rng = np.random.Generator(np.random.PCG64(13))
    zlat = rng.standard_normal((1, cfg.latent_size, n_blocks * frames)).astype(np.float32)
    z = torch.cat([torch.from_numpy(zlat), speaker.reshape(1, -1, 1).repeat(1, 1, zlat.shape[-1])], 1)
    F = block // cfg.n_band
    n_fr = F // int(np.prod(cfg.noise.ratios))
    u = rng.uniform(0, 1, size=(n_blocks, 1, n_fr, cfg.n_band, 2 * (cfg.noise.noise_bands - 1))).astype(np.float32)
    ada = [mod for mod in m.modules() if isinstance(mod, mods["blocks"].AdaptiveInstanceNormalization)]
    flags = [(0, 1), (0, 1), (1, 0), (1, 0), (0, 0), (0, 0)]

    def set_learn(lx, ly):
        for mod in ada:
            mod.learn_x.fill_(float(lx))
            mod.learn_y.fill_(float(ly))

    res = {"x": x.numpy(), "z": z.numpy(), "noise_u": u, "speaker": speaker.numpy(), "block": np.int64(block),
           "seed": np.int64(seed), "flags": np.array(flags, np.int64)}
    with torch.no_grad():
        zs = []
        for i in range(n_blocks):
            set_learn(*flags[i])
            zs.append(ref_encode(m, cfg, x[..., i * block:(i + 1) * block], speaker))
        for mod in ada:          # the decoder pass starts from fresh statistics too
            mod.reset_x()
            mod.reset_y()
        ys = []
        for i in range(n_blocks):
            set_learn(*flags[i])
            with NoiseInjector(torch.from_numpy(u[i])):
                ys.append(ref_decode(m, z[..., i * frames:(i + 1) * frames]))
    res["z_stream"] = torch.cat(zs, -1).numpy()
    res["y_stream"] = torch.cat(ys, -1).numpy()
    np.savez_compressed(os.path.join(out, fname), **res)
    return res


def gen_adain(mods, cfg, out, fname="v3_adain.npz", batch=2, t=8192, seed=0):
    """AdaIN style transfer in eval mode (rave/blocks.py:856-919), driven the
    way nn~'s learn_source / learn_target attributes drive it: learn the target
    statistics on x_tgt, learn the source statistics on x_src (the transfer
    turns on in that same call), transfer with frozen statistics, then learn the
    source again on a smaller batch (the buffers' [:bs] rows).  Every call is a
    full encode -> decode (AdaIN sits in both EncoderV2 and GeneratorV2)."""
    m = build_reference(mods, cfg, cached=False)
    params = init_params(cfg, seed=seed)
    load_params(m, cfg, params)
    speaker = torch.from_numpy(init_speaker(cfg, seed=seed))
    n = np.arange(t)
    rng = np.random.Generator(np.random.PCG64(100))
    x_tgt = torch.from_numpy((0.8 * np.sin(2 * np.pi * 3000 * n / 48000)[None, None, :]
                              * np.linspace(0.2, 1.0, batch)[:, None, None]
                              + 0.3 * rng.standard_normal((batch, 1, t))).astype(np.float32))
    x_src = torch.from_numpy(synth_audio(batch, t, seed0=200))
    ada = [mod for mod in m.modules() if isinstance(mod, mods["blocks"].AdaptiveInstanceNormalization)]
    names = [n for n, mod in m.named_modules() if isinstance(mod, mods["blocks"].AdaptiveInstanceNormalization)]

    def set_learn(lx, ly):
        for mod in ada:
            mod.learn_x.fill_(float(lx))
            mod.learn_y.fill_(float(ly))

    res = {"x_tgt": x_tgt.numpy(), "x_src": x_src.numpy(), "speaker": speaker.numpy(),
           "seed": np.int64(seed), "names": np.array(names)}
    steps = [("learn_y", (0, 1), x_tgt), ("learn_x", (1, 0), x_src), ("transfer", (0, 0), x_src),
             ("learn_x_bs1", (1, 0), x_src[:1])]
    with torch.no_grad():
        for i, (tag, (lx, ly), x) in enumerate(steps):
            set_learn(lx, ly)
            z = ref_encode(m, cfg, x, speaker)
            y = ref_decode(m, z)
            res[f"step{i}/z"] = z.numpy()
            res[f"step{i}/y"] = y.numpy()
    res["steps"] = np.array([s[0] for s in steps])
    for n, mod in zip(names, ada):
        for b in ("mean_x", "std_x", "mean_y", "std_y", "num_update_x", "num_update_y"):
            res[f"final/{n}.{b}"] = getattr(mod, b).numpy().copy()
    np.savez_compressed(os.path.join(out, fname), **res)
    return res


def gen_speaker(mods, out, seed=0):
    """SpeakerRAVE (rave/CombinedRave.py:200-328) in eval mode on the 16 PQMF
    bands of two synthetic clips (the reference's embedding call,
    scripts/export.py:84-90), centred and causal padding; seeded parameters
    (rave_amd.speaker.init_params) loaded under the module's own names."""
    import cached_conv as cc
    from rave_amd.speaker import init_params as speaker_params
    params = speaker_params(seed)
    res = {"seed": np.int64(seed)}
    for mode in ("centered", "causal"):
        cc.use_cached_conv(False)
        cc.set_padding_mode(mode)
        m = mods["CombinedRave"].SpeakerRAVE()
        sd = {k: torch.from_numpy(v) for k, v in params.items()}
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not unexpected, unexpected
        assert all(k.startswith("bn6.") or k.endswith("num_batches_tracked") for k in missing), missing
        m.eval()
        pq = mods["pqmf"].CachedPQMF(attenuation=100, n_band=16)
        x = torch.from_numpy(synth_audio(2, 16384, seed0=300))
        acts = {}
        hooks = [getattr(m, n).register_forward_hook(
            lambda mod, i, o, n=n: acts.__setitem__(n, o.detach().numpy().copy()))
            for n in ("layer2", "layer3", "layer4", "cat_layer", "out_layer")]
        with torch.no_grad():
            bands = pq(x)
            emb = m(bands)
        for h in hooks:
            h.remove()
        res[f"{mode}/x"] = x.numpy()
        res[f"{mode}/bands"] = bands.numpy()
        res[f"{mode}/emb"] = emb.numpy()
        for n, v in acts.items():
            res[f"{mode}/{n}"] = v
    cc.set_padding_mode("centered")
    np.savez_compressed(os.path.join(out, "speaker.npz"), **res)
    return res


def gen_resampler(mods, out):
    """Resampler (rave/resampler.py:9-66): its two filters, offline
    to/from_model_sampling_rate for ratios 2, 3 (centred) and 2 (causal), and
    the cached (streaming) form for ratio 2 over 2048-sample blocks.  These are
    the ratios the reference can build: for 4..8 the polyphase split of
    rave/resampler.py:41-44 pads len(h) % ratio taps and the reshape fails
    (rave_amd.resampler.design raises for them too), and streaming rejects odd
    ratios (:21-25)."""
    import cached_conv as cc
    res = {}
    rng = np.random.Generator(np.random.PCG64(400))
    x = torch.from_numpy(rng.standard_normal((2, 1, 4096)).astype(np.float32))
    for ratio, mode in ((2, "centered"), (3, "centered"), (2, "causal")):
        cc.use_cached_conv(False)
        cc.set_padding_mode(mode)
        r = mods["resampler"].Resampler(48000 * ratio, 48000)
        key = f"r{ratio}_{mode}"
        with torch.no_grad():
            res[f"{key}/down_w"] = r.downsample.weight.numpy().copy()
            res[f"{key}/up_w"] = r.upsample.weight.numpy().copy()
            res[f"{key}/down"] = r.to_model_sampling_rate(x).numpy()
            res[f"{key}/up"] = r.from_model_sampling_rate(x).numpy()
    res["x"] = x.numpy()
    n_blocks, block = 6, 2048
    xs = torch.from_numpy(rng.standard_normal((1, 1, n_blocks * block)).astype(np.float32))
    res["stream/x"] = xs.numpy()
    for ratio in (2,):
        for mode in ("centered", "causal"):
            cc.use_cached_conv(True)
            cc.set_padding_mode(mode)
            r = mods["resampler"].Resampler(48000 * ratio, 48000)
            with torch.no_grad():
                down = [r.to_model_sampling_rate(xs[..., i * block:(i + 1) * block]) for i in range(n_blocks)]
                up = [r.from_model_sampling_rate(xs[..., i * block:(i + 1) * block]) for i in range(n_blocks)]
            res[f"stream/r{ratio}_{mode}/down"] = torch.cat(down, -1).numpy()
            res[f"stream/r{ratio}_{mode}/up"] = torch.cat(up, -1).numpy()
    cc.use_cached_conv(False)
    cc.set_padding_mode("centered")
    np.savez_compressed(os.path.join(out, "resampler.npz"), **res)
    return res


def check_residual_semantics(mods):
    """The reference's tests/test_residual.py logic (streaming == one-shot,
    delay-shifted) run against the cached_conv restatement."""
    import cached_conv as cc
    blocks = mods["blocks"]
    cc.set_padding_mode("centered")
    if hasattr(blocks, "_DilatedUnit"):
        blocks.DilatedUnit = blocks._DilatedUnit
    results = {}
    torch.manual_seed(0)

    def run(make, tol):
        x = torch.randn(1, 16, 32)
        cc.use_cached_conv(False)
        a = make()
        cc.use_cached_conv(True)
        b = make()
        for p1, p2 in zip(a.parameters(), b.parameters()):
            p2.data.copy_(p1.data)
        d = b.cumulative_delay
        with torch.no_grad():
            ya, yb = a(x), b(x)
        if d:
            ya, yb = ya[..., d:-d], yb[..., d + d:]
        return bool(torch.allclose(ya, yb, tol[0], tol[1])), int(d)

    from torch.nn.utils import weight_norm
    blocks.normalization = lambda module, mode="weight_norm": weight_norm(module)
    results["residual_stack"] = run(lambda: blocks.ResidualStack(16, [3], [[1, 1], [3, 1], [5, 1]]), (1e-4, 1e-4))
    for k in (1, 3):
        for dl in ([1, 1], [3, 1]):
            results[f"residual_layer_k{k}_{dl}"] = run(lambda: blocks.ResidualLayer(16, k, dl), (1e-3, 1e-4))
    for r in (2, 4, 8):
        results[f"upsample_r{r}"] = run(lambda: blocks.UpsampleLayer(16, 16, r), (1e-3, 1e-4))
    cc.use_cached_conv(False)
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", default=None, help="regenerate one fixture group (e.g. adain)")
    a = ap.parse_args()
    torch.set_num_threads(8)
    mods = install_shims()
    if a.only == "stream_v3":
        gen_stream_v3(mods, rcfg.v3_noise(causal=True, capacity=16), a.out)
        gen_stream_v3(mods, rcfg.v3_noise(capacity=16), a.out, fname="v3_noise_stream.npz")
        write_manifest(a.out)
        return
    if a.only == "stream":
        gen_streaming(mods, rcfg.v2(), a.out, fname="v2_stream.npz")
        gen_stream_discrete(mods, rcfg.discrete(), a.out)
        gen_stream_v3(mods, rcfg.v3_noise(capacity=16), a.out, fname="v3_noise_stream.npz")
        write_manifest(a.out)
        return
    if a.only == "speaker":
        gen_speaker(mods, a.out)
        gen_resampler(mods, a.out)
        write_manifest(a.out)
        return
    if a.only == "adain":
        gen_adain(mods, rcfg.v3(), a.out)
        gen_adain(mods, rcfg.v3(capacity=8), a.out, fname="v3_adain_small.npz", t=4096)
        write_manifest(a.out)
        return
    if a.only == "manifest":
        write_manifest(a.out)
        return
    manifest = {}
    manifest["residual_semantics"] = check_residual_semantics(mods)
    assert all(v[0] for v in manifest["residual_semantics"].values()), manifest["residual_semantics"]

    pq = gen_pqmf(mods, a.out)
    manifest["pqmf_hk_sha16"] = hashlib.sha256(pq["hk"].tobytes()).hexdigest()[:16]
    gen_model(mods, rcfg.v2(capacity=8), a.out, "v2_small_layers.npz", batch=1, t=4096, per_layer=True)
    gen_model(mods, rcfg.v2(), a.out, "v2.npz")
    gen_model(mods, rcfg.causal(), a.out, "causal.npz")
    gen_streaming(mods, rcfg.causal(), a.out)
    gen_streaming(mods, rcfg.v2(), a.out, fname="v2_stream.npz")
    gen_model(mods, rcfg.discrete(), a.out, "discrete.npz")
    gen_rvq(mods, a.out)
    gen_model(mods, rcfg.v3_noise(), a.out, "v3_noise.npz")
    gen_model(mods, rcfg.v3_noise(capacity=8), a.out, "v3_noise_small_layers.npz", batch=1, t=4096,
              per_layer=True)
    gen_adain(mods, rcfg.v3(), a.out)
    gen_adain(mods, rcfg.v3(capacity=8), a.out, fname="v3_adain_small.npz", t=4096)
    gen_stream_v3(mods, rcfg.v3_noise(causal=True, capacity=16), a.out)
    gen_stream_v3(mods, rcfg.v3_noise(capacity=16), a.out, fname="v3_noise_stream.npz")
    gen_stream_discrete(mods, rcfg.discrete(), a.out)
    gen_speaker(mods, a.out)
    gen_resampler(mods, a.out)
    print(json.dumps(write_manifest(a.out, manifest), indent=1))


if __name__ == "__main__":
    main()
