"""Layer graph of the encode->decode path, named after the reference modules.

The graph is a flat, ordered list of operator nodes.  Every convolution node
carries the *reference state_dict prefix* of the module it replaces, so the
same table drives (a) the portable seeded weight init, (b) checkpoint loading
with weight-norm folding and (c) the native execution plan.

Module structure restated (no code copied):

* ``EncoderV2.net`` (rave/blocks.py:533-589): conv k=2*ks+1 -> per ratio r:
  [AdaIN]·Residual(DilatedUnit d) for d in dilations -> act -> conv(C, 2C,
  k=2r, stride r) -> act -> conv k=ks (C -> latent).
* ``GeneratorV2.net`` (rave/blocks.py:629-688): conv k=ks (latent+spk -> C0)
  -> per reversed ratio r: act -> ConvTranspose1d(C, C/2, 2r, stride r,
  padding r//2) -> [AdaIN]·Residual(DilatedUnit d) -> act -> waveform conv
  k=2*ks+1 (C -> 2*n_band); with a noise module the waveform conv lives in
  ``decoder.waveform_module`` (rave/blocks.py:679-686).
* ``Residual`` (rave/blocks.py:32-46) wraps ``cc.AlignBranches(module,
  Identity)``, so the DilatedUnit convs live at
  ``<residual>.aligned.branches.0.net.{1,3}``; its activations at
  ``.net.{0,2}`` (rave/blocks.py:94-107).
* ``NoiseGeneratorV2.net`` (rave/blocks.py:257-273): convs k=2r stride r
  padding (r, 0), activation between them, no weight norm.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .config import RaveConfig, get_padding


@dataclass
class ConvNode:
    """One convolution (or transposed convolution) with a fused prologue
    activation on its input and an optional residual add on its output."""
    name: str                 # reference module path (state_dict prefix)
    c_in: int
    c_out: int
    kernel: int
    stride: int = 1
    dilation: int = 1
    pad: Tuple[int, int] = (0, 0)
    transposed: bool = False
    weight_norm: bool = True
    bias: bool = True
    act: str = "none"         # activation applied to the input: none|leaky|snake
    alpha: Optional[str] = None   # Snake alpha parameter name when act == 'snake'
    src: str = ""             # input tensor id
    dst: str = ""             # output tensor id
    residual: Optional[str] = None  # tensor id added to the output
    adain: Optional[str] = None     # AdaIN module applied to the input before act
    kind: str = "conv"

    def out_len(self, t_in: int) -> int:
        if self.transposed:
            # nn.ConvTranspose1d: (T-1)*s - 2p + k with p = s//2, k = 2s
            p = self.stride // 2
            return (t_in - 1) * self.stride - 2 * p + self.kernel
        span = (self.kernel - 1) * self.dilation + 1
        return (t_in + self.pad[0] + self.pad[1] - span) // self.stride + 1


@dataclass
class Graph:
    cfg: RaveConfig
    encoder: List[ConvNode] = field(default_factory=list)
    decoder: List[ConvNode] = field(default_factory=list)
    noise: List[ConvNode] = field(default_factory=list)
    adain_modules: List[Tuple[str, int]] = field(default_factory=list)   # (prefix, dim)

    def convs(self) -> List[ConvNode]:
        return self.encoder + self.decoder + self.noise


def _act_param(cfg: RaveConfig, module: str) -> Tuple[str, Optional[str]]:
    if cfg.activation == "snake":
        return "snake", f"{module}.alpha"
    return "leaky", None


def build_graph(cfg: RaveConfig) -> Graph:
    g = Graph(cfg)
    ks = cfg.kernel_size
    c = cfg.causal

    # ------------------------------------------------------------ encoder
    pre = "encoder.encoder.net"
    idx = 0
    cur = "enc_in"
    tid = 0

    def new_t(prefix: str) -> str:
        nonlocal tid
        tid += 1
        return f"{prefix}{tid}"

    nxt = new_t("e")
    g.encoder.append(ConvNode(f"{pre}.{idx}", cfg.enc_bands, cfg.capacity, 2 * ks + 1,
                              pad=get_padding(2 * ks + 1, causal=c), act="none",
                              bias=cfg.conv_bias, src=cur, dst=nxt))
    cur = nxt
    idx += 1
    ch = cfg.capacity
    for r, dils in zip(cfg.ratios, cfg.dilations):
        for d in dils:
            adain = None
            if cfg.adain:
                adain = f"{pre}.{idx}"
                g.adain_modules.append((adain, ch))
                idx += 1
            _residual_unit(g.encoder, cfg, f"{pre}.{idx}", ch, d, cur, adain, new_t("e"), new_t("e"))
            cur = g.encoder[-1].dst
            idx += 1
        act, alpha = _act_param(cfg, f"{pre}.{idx}")
        idx += 1
        nxt = new_t("e")
        g.encoder.append(ConvNode(f"{pre}.{idx}", ch, 2 * ch, 2 * r, stride=r,
                                  pad=get_padding(2 * r, r, causal=c), act=act, alpha=alpha,
                                  bias=cfg.conv_bias, src=cur, dst=nxt))
        cur = nxt
        idx += 1
        ch *= 2
    act, alpha = _act_param(cfg, f"{pre}.{idx}")
    idx += 1
    g.encoder.append(ConvNode(f"{pre}.{idx}", ch, cfg.latent_size, ks,
                              pad=get_padding(ks, causal=c), act=act, alpha=alpha,
                              bias=cfg.conv_bias, src=cur, dst="latent"))

    # ------------------------------------------------------------ decoder
    pre = "decoder.net"
    idx = 0
    ch = cfg.dec_channels
    nxt = new_t("d")
    g.decoder.append(ConvNode(f"{pre}.{idx}", cfg.dec_in, ch, ks, pad=get_padding(ks, causal=c),
                              act="none", bias=cfg.conv_bias, src="dec_in", dst=nxt))
    cur = nxt
    idx += 1
    for r, dils in zip(cfg.ratios[::-1], cfg.dilations[::-1]):
        act, alpha = _act_param(cfg, f"{pre}.{idx}")
        idx += 1
        nxt = new_t("d")
        g.decoder.append(ConvNode(f"{pre}.{idx}", ch, ch // 2, 2 * r, stride=r,
                                  pad=(r // 2, r // 2), transposed=True, act=act, alpha=alpha,
                                  bias=cfg.convt_bias, src=cur, dst=nxt))
        cur = nxt
        idx += 1
        ch //= 2
        for d in dils:
            adain = None
            if cfg.adain:
                adain = f"{pre}.{idx}"
                g.adain_modules.append((adain, ch))
                idx += 1
            _residual_unit(g.decoder, cfg, f"{pre}.{idx}", ch, d, cur, adain, new_t("d"), new_t("d"))
            cur = g.decoder[-1].dst
            idx += 1
    act, alpha = _act_param(cfg, f"{pre}.{idx}")
    idx += 1
    wave_name = "decoder.waveform_module" if cfg.noise is not None else f"{pre}.{idx}"
    g.decoder.append(ConvNode(wave_name, ch, cfg.dec_out, 2 * ks + 1,
                              pad=get_padding(2 * ks + 1, causal=c), act=act, alpha=alpha,
                              bias=cfg.conv_bias, src=cur, dst="wave"))

    # ------------------------------------------------------------ noise synth
    if cfg.noise is not None:
        nz = cfg.noise
        chans = [ch] + [nz.hidden_size] * (len(nz.ratios) - 1) + [cfg.n_band * nz.noise_bands]
        src = cur
        npre = "decoder.noise_module.net"
        j = 0
        for i, r in enumerate(nz.ratios):
            if i == 0:
                # the noise module consumes the activated decoder features:
                # same activation (and Snake alpha) as the waveform conv
                act_i, alpha_i = act, alpha
            else:
                act_i, alpha_i = _act_param(cfg, f"{npre}.{j - 1}")
            dst = "noise_amp" if i == len(nz.ratios) - 1 else new_t("n")
            g.noise.append(ConvNode(f"{npre}.{j}", chans[i], chans[i + 1], 2 * r, stride=r,
                                    pad=(r, 0), weight_norm=False, act=act_i, alpha=alpha_i,
                                    bias=cfg.conv_bias, src=src, dst=dst))
            src = dst
            j += 2 if i != len(nz.ratios) - 1 else 1
    return g


def _residual_unit(out: List[ConvNode], cfg: RaveConfig, res: str, ch: int, d: int,
                   src: str, adain: Optional[str], mid: str, dst: str) -> None:
    """Residual(DilatedUnit(ch, ks, d)) -- rave/blocks.py:32-46, 84-113."""
    ks = cfg.kernel_size
    unit = f"{res}.aligned.branches.0.net"
    act0, alpha0 = _act_param(cfg, f"{unit}.0")
    act2, alpha2 = _act_param(cfg, f"{unit}.2")
    out.append(ConvNode(f"{unit}.1", ch, ch, ks, dilation=d,
                        pad=get_padding(ks, dilation=d, causal=cfg.causal),
                        act=act0, alpha=alpha0, bias=cfg.conv_bias, src=src, dst=mid, adain=adain))
    out.append(ConvNode(f"{unit}.3", ch, ch, 1, act=act2, alpha=alpha2,
                        bias=cfg.conv_bias, src=mid, dst=dst, residual=src))


def param_shapes(cfg: RaveConfig) -> Dict[str, Tuple[int, ...]]:
    """Reference state_dict parameter names -> shapes for the hot path."""
    g = build_graph(cfg)
    shapes: Dict[str, Tuple[int, ...]] = {}
    for n in g.convs():
        wshape = (n.c_in, n.c_out, n.kernel) if n.transposed else (n.c_out, n.c_in, n.kernel)
        if n.weight_norm:
            shapes[f"{n.name}.weight_g"] = (wshape[0], 1, 1)
            shapes[f"{n.name}.weight_v"] = wshape
        else:
            shapes[f"{n.name}.weight"] = wshape
        if n.bias:
            shapes[f"{n.name}.bias"] = (n.c_out,)
        if n.act == "snake" and n.alpha not in shapes:
            shapes[n.alpha] = (n.c_in, 1)
    if cfg.rvq is not None:
        for i in range(cfg.rvq.num_quantizers):
            shapes[f"encoder.rvq.layers.{i}._codebook.embed"] = (cfg.rvq.codebook_size, cfg.latent_size)
    return shapes
