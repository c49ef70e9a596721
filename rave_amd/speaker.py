"""``SpeakerRAVE``: the speaker encoder whose output is RAVE's constant 256-d
speaker embedding (rave/CombinedRave.py:200-328; used once at model init,
rave/model.py:246-247, and by the nn~ export for its four reference speakers
and the recorded target, scripts/export.py:84-93, 281-282).

Forward (rave/CombinedRave.py:301-328), x = the 16 PQMF bands of the
embedding audio, (B, 16, T):

    in_layer   Conv1d(16, 128, 7)                              (:208-213)
    layer2     Residual(DilatedUnit(128, 3, d=1)) -> LeakyReLU -> Conv1d(128, 256, 8, s=4)
    layer3     Residual(DilatedUnit(256, 3, d=3)) -> LeakyReLU -> Conv1d(256, 256, 8, s=4)
    layer4     Residual(DilatedUnit(256, 3, d=5)) -> LeakyReLU -> Conv1d(256, 256, 4, s=2)
    cat_layer  Conv1d(256, 256, 1)
    out_layer  Conv1d(768, 768, 3) over cat(MaxPool1d(2)(x2), x3, x4) -> LeakyReLU
    attentive statistics pooling: global_x = cat(x, mean_t(x), sqrt(clamp(var_t(x))))
      w = softmax_t(Conv1d(128, 768, 1)(BN(ReLU(Conv1d(2304, 128, 1)(global_x)))))
      mu = sum_t x w,  sg = sqrt(clamp(sum_t x^2 w - mu^2))
    fc6(bn5(cat(mu, sg)))  -> (B, 256)

The module's ``normalization`` defaults to identity (rave/CombinedRave.py:18-24),
so the convs carry plain ``weight``/``bias``; BatchNorm runs in eval mode
(running statistics, eps 1e-5).  Every conv runs on the HIP conv kernels
(``rave_conv1d``, exact fp32), the residual units on the fused unit kernel, and
the pooling head on the kernels of csrc/speaker.hip (``rave_row_stats``,
``rave_attn_pool``, ``rave_linear``, ``rave_maxpool``).  Host-side work is
parameter folding only: BN into the neighbouring affine maps, the time-constant
mean/std columns of the 2304-channel attention input into a per-row bias.
"""
from __future__ import annotations

import ctypes as C
import zlib
from collections import OrderedDict
from typing import Dict, Mapping, Optional

import numpy as np

from .config import get_padding

BANDS, C1, C2, EMB = 16, 128, 256, 256
ATT, ATT_HID = 768, 128
BN_EPS = 1e-5
VAR_MIN, VAR_MAX = 1e-4, 1e4
LEAKY = 0.2
# (name, c_in, c_out, kernel, stride) of the strided head of layer2..4, and the unit's dilation
STAGES = (("layer2", C1, C2, 8, 4, 1), ("layer3", C2, C2, 8, 4, 3), ("layer4", C2, C2, 4, 2, 5))


def _unit(prefix: str) -> str:
    return f"{prefix}.0.aligned.branches.0.net"


def param_shapes() -> "OrderedDict[str, tuple]":
    """SpeakerRAVE's state_dict entries the forward uses, in module order."""
    s: "OrderedDict[str, tuple]" = OrderedDict()
    s["in_layer.weight"], s["in_layer.bias"] = (C1, BANDS, 7), (C1,)
    for name, ci, co, k, _, _ in STAGES:
        u = _unit(name)
        s[f"{u}.1.weight"], s[f"{u}.1.bias"] = (ci, ci, 3), (ci,)
        s[f"{u}.3.weight"], s[f"{u}.3.bias"] = (ci, ci, 1), (ci,)
        s[f"{name}.2.weight"], s[f"{name}.2.bias"] = (co, ci, k), (co,)
    s["cat_layer.weight"], s["cat_layer.bias"] = (EMB, EMB, 1), (EMB,)
    s["out_layer.weight"], s["out_layer.bias"] = (ATT, 3 * EMB, 3), (ATT,)
    s["attention.0.weight"], s["attention.0.bias"] = (ATT_HID, 3 * ATT, 1), (ATT_HID,)
    for b, n in (("attention.2", ATT_HID), ("bn5", 2 * ATT)):
        s[f"{b}.weight"], s[f"{b}.bias"] = (n,), (n,)
        s[f"{b}.running_mean"], s[f"{b}.running_var"] = (n,), (n,)
    s["attention.3.weight"], s["attention.3.bias"] = (ATT, ATT_HID, 1), (ATT,)
    s["fc6.weight"], s["fc6.bias"] = (EMB, 2 * ATT), (EMB,)
    return s


def init_params(seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """Seeded parameters under SpeakerRAVE's names (the pretrained blob,
    rave/pretrained/model000000075.model, is not in the reference): PyTorch's
    default uniform bound for weights and biases; BatchNorm affine and running
    statistics drawn away from their identity init so the folds are exercised."""
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    shapes = param_shapes()
    for name, shape in shapes.items():
        rng = np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())]))
        owner = name.rsplit(".", 1)[0]
        if name.endswith("running_mean"):
            v = 0.1 * rng.standard_normal(shape)
        elif name.endswith("running_var"):
            v = rng.uniform(0.5, 2.0, shape)
        elif owner in ("attention.2", "bn5"):
            v = (1.0 + 0.1 * rng.standard_normal(shape)) if name.endswith("weight") else 0.1 * rng.standard_normal(shape)
        else:
            w = shapes[owner + ".weight"]
            bound = 1.0 / np.sqrt(w[1] * int(np.prod(w[2:])))
            v = rng.uniform(-bound, bound, shape)
        out[name] = v.astype(np.float32)
    return out


def load_state(state: Mapping) -> Dict[str, np.ndarray]:
    """Parameters from a speaker-encoder checkpoint as RAVE.load_speaker_statedict
    reads it (rave/model.py:278-300): the ``__S__.`` prefix is dropped and
    ``pqmf.*`` entries are set aside (the embedding uses the model's own PQMF).
    Entries the forward does not use (``bn6``, ``num_batches_tracked``) are
    ignored, as load_state_dict would keep them unused; missing or misshaped
    entries raise."""
    flat = {}
    for k, v in state.items():
        k = k.replace("__S__.", "")
        if "pqmf" in k:
            continue
        flat[k] = np.asarray(v.detach().cpu().numpy() if hasattr(v, "detach") else v, np.float32)
    out = {}
    for name, shape in param_shapes().items():
        if name not in flat:
            raise KeyError(f"speaker checkpoint has no {name}")
        if tuple(flat[name].shape) != tuple(shape):
            raise ValueError(f"{name}: expected {shape}, got {flat[name].shape}")
        out[name] = flat[name]
    return out


def _bn_affine(p: Mapping[str, np.ndarray], name: str):
    """Eval BatchNorm as y = s * x + t (float64)."""
    s = p[f"{name}.weight"].astype(np.float64) / np.sqrt(p[f"{name}.running_var"].astype(np.float64) + BN_EPS)
    t = p[f"{name}.bias"].astype(np.float64) - s * p[f"{name}.running_mean"].astype(np.float64)
    return s, t


def fold_head(p: Mapping[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Host folds of the pooling head (float64, cast once to float32):

    * attention.0 over cat(x, mean, std): W = [Wx | Wm | Ws]; the mean/std
      columns are constant over time, so ``att0_stat`` = [Wm | Ws] (128, 1536)
      turns (mean, std) into a per-row bias added to attention.0.bias;
    * BN(attention.2) after the ReLU folds into attention.3:
      W3 diag(s) and b3 + W3 t;
    * bn5 before fc6 folds into fc6: W6 diag(s5) and b6 + W6 t5."""
    w0 = p["attention.0.weight"].reshape(ATT_HID, 3 * ATT).astype(np.float64)
    s2, t2 = _bn_affine(p, "attention.2")
    w3 = p["attention.3.weight"].reshape(ATT, ATT_HID).astype(np.float64)
    s5, t5 = _bn_affine(p, "bn5")
    w6 = p["fc6.weight"].astype(np.float64)
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    return {
        "att0_x": f32(w0[:, :ATT].reshape(ATT_HID, ATT, 1)),
        "att0_stat": f32(w0[:, ATT:]),
        "att0_b": f32(p["attention.0.bias"]),
        "att3_w": f32((w3 * s2[None, :]).reshape(ATT, ATT_HID, 1)),
        "att3_b": f32(p["attention.3.bias"].astype(np.float64) + w3 @ t2),
        "fc_w": f32(w6 * s5[None, :]),
        "fc_b": f32(p["fc6.bias"].astype(np.float64) + w6 @ t5),
    }


class SpeakerRAVE:
    """HIP SpeakerRAVE forward.  ``forward(bands)`` takes the (B, 16, T) PQMF
    bands (the reference's call, scripts/export.py:90) and returns (B, 256);
    ``embed(audio)`` runs the centred PQMF analysis first (all 16 bands).
    T must be a multiple of 64 (the three strided stages and the max-pool).
    ``causal`` selects cached_conv's causal padding (causal.gin)."""

    def __init__(self, params: Mapping[str, np.ndarray], device=None, causal: bool = False,
                 pqmf_attenuation: float = 100.0):
        import torch
        from . import _native as N
        from . import pqmf as P
        self.N, self.torch = N, torch
        self.dev = torch.device(device or "cuda")
        self.causal = bool(causal)
        shapes = param_shapes()
        for name, shape in shapes.items():
            if name not in params:
                raise KeyError(f"missing speaker parameter {name}")
            if tuple(np.shape(params[name])) != tuple(shape):
                raise ValueError(f"{name}: expected {shape}, got {np.shape(params[name])}")
        p = {k: np.asarray(v, np.float32) for k, v in params.items()}
        d = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(self.dev)  # noqa: E731
        self._pk = {}       # packed conv weights (fp32 MFMA layout)
        self._b = {}

        def conv(name, w, b, ci, co, k, s=1, dil=1):
            self._pk[name] = (d(N.pack_conv_weight(w, ci, co, k, s, dil, False)), ci, co, k, s, dil)
            self._b[name] = d(b)

        conv("in_layer", p["in_layer.weight"], p["in_layer.bias"], BANDS, C1, 7)
        self._units = {}
        for name, ci, co, k, s, dil in STAGES:
            u = _unit(name)
            if N.unit_supported(ci):
                self._units[name] = (d(N.pack_unit_weight(p[f"{u}.1.weight"], p[f"{u}.3.weight"], ci)),
                                     d(p[f"{u}.1.bias"]), d(p[f"{u}.3.bias"]), ci, dil)
            else:   # pragma: no cover - every SpeakerRAVE width has a fused unit
                raise NotImplementedError(f"no fused residual unit for C={ci}")
            conv(name, p[f"{name}.2.weight"], p[f"{name}.2.bias"], ci, co, k, s)
        conv("cat_layer", p["cat_layer.weight"], p["cat_layer.bias"], EMB, EMB, 1)
        conv("out_layer", p["out_layer.weight"], p["out_layer.bias"], 3 * EMB, ATT, 3)
        h = fold_head(p)
        conv("att0", h["att0_x"], np.zeros(ATT_HID, np.float32), ATT, ATT_HID, 1)
        conv("att3", h["att3_w"], h["att3_b"], ATT_HID, ATT, 1)
        self._att0_stat, self._att0_b = d(h["att0_stat"]), d(h["att0_b"])
        self._fc_w, self._fc_b = d(h["fc_w"]), d(h["fc_b"])
        self._hkf = None
        self._pqmf_att = pqmf_attenuation
        self._P = P

    # ------------------------------------------------------------ launches
    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def _conv(self, name, x, y, act="none", bias=None, batch=None, x_off=0, y_off=0):
        N = self.N
        w, ci, co, k, s, dil = self._pk[name]
        B = x.shape[0] if batch is None else batch
        t_in, t_out = x.shape[-1], y.shape[-1]
        pad = get_padding(k, s, dil, causal=self.causal)
        if (t_in + pad[0] + pad[1] - ((k - 1) * dil + 1)) // s + 1 != t_out:
            raise ValueError(f"{name}: output length {t_out} does not follow from {t_in}")
        # ReLU is the leaky prologue with slope 0
        a = N.ConvArgs(c_in=ci, c_out=co, kernel=k, stride=s, dilation=dil, pad_left=pad[0],
                       pad_right=pad[1], transposed=0, out_shift=0, act=N.ACT["leaky" if act == "relu" else act],
                       leaky_slope=LEAKY if act == "leaky" else 0.0, batch=B, t_in=t_in, t_out=t_out,
                       precision=N.PREC_F32,
                       x=x.data_ptr() + 4 * x_off, x_sb=x.stride(0), x_sc=x.stride(1),
                       y=y.data_ptr() + 4 * y_off, y_sb=y.stride(0), y_sc=y.stride(1),
                       weight=w.data_ptr(), bias=(bias if bias is not None else self._b[name]).data_ptr(),
                       config=0)
        nws = int(N.lib.rave_conv1d_workspace(C.byref(a)))
        ws = None
        if nws > 0:
            ws = self.torch.zeros(nws, dtype=self.torch.float32, device=self.dev)
            a.partial = ws.data_ptr()
        N.check(N.lib.rave_conv1d(C.byref(a), self._stream()), f"speaker {name}")
        return ws    # keep the workspace alive until the stream has used it

    def _unit_run(self, name, x, y):
        N = self.N
        w, b1, b2, ch, dil = self._units[name]
        pad = get_padding(3, 1, dil, causal=self.causal)
        a = N.UnitArgs(channels=ch, batch=x.shape[0], t_len=x.shape[-1], dilation=dil, pad_left=pad[0],
                       act=N.ACT["leaky"], leaky_slope=LEAKY, precision=N.PREC_F32,
                       x=x.data_ptr(), x_sb=x.stride(0), x_sc=x.stride(1),
                       y=y.data_ptr(), y_sb=y.stride(0), y_sc=y.stride(1),
                       weight=w.data_ptr(), bias1=b1.data_ptr(), bias2=b2.data_ptr())
        N.check(N.lib.rave_residual_unit(C.byref(a), self._stream()), f"speaker {name} unit")

    # ------------------------------------------------------------ API
    def forward(self, bands):
        """(B, 16, T) fp32 PQMF bands on this device -> (B, 256)."""
        torch, N = self.torch, self.N
        if bands.dim() != 3 or bands.shape[1] != BANDS:
            raise ValueError(f"expected (B, {BANDS}, T) bands, got {tuple(bands.shape)}")
        if bands.dtype != torch.float32 or bands.device != self.dev:
            raise ValueError("bands must be float32 on the model's device")
        B, _, T = bands.shape
        if T % 64 or T < 64:
            raise ValueError(f"band length {T} must be a positive multiple of 64")
        x = bands.contiguous()
        e = lambda c, t: torch.empty(B, c, t, device=self.dev)  # noqa: E731
        keep = []
        h0 = e(C1, T)
        keep.append(self._conv("in_layer", x, h0))
        t2, t3, t4 = T // 4, T // 16, T // 32
        u = e(C1, T)
        self._unit_run("layer2", h0, u)
        x1 = e(C2, t2)
        keep.append(self._conv("layer2", u, x1, act="leaky"))
        u = e(C2, t2)
        self._unit_run("layer3", x1, u)
        x2 = e(C2, t3)
        keep.append(self._conv("layer3", u, x2, act="leaky"))
        u = e(C2, t3)
        self._unit_run("layer4", x2, u)
        cat = e(3 * EMB, t4)                              # cat(mp2(x2), x3, x4) as channel slices
        x3 = cat[:, EMB:2 * EMB]
        keep.append(self._conv("layer4", u, x3, act="leaky"))
        keep.append(self._conv("cat_layer", x3, cat[:, 2 * EMB:]))
        mp = N.MaxPoolArgs(batch=B, channels=EMB, t_out=t4, kernel=2,
                           x=x2.data_ptr(), x_sb=x2.stride(0), x_sc=x2.stride(1),
                           y=cat.data_ptr(), y_sb=cat.stride(0), y_sc=cat.stride(1))
        N.check(N.lib.rave_maxpool(C.byref(mp), self._stream()), "speaker maxpool")
        xo = e(ATT, t4)                                   # out_layer before its LeakyReLU
        keep.append(self._conv("out_layer", cat, xo))
        # attentive statistics pooling; the LeakyReLU is applied where xo is read
        stats = torch.empty(B, 2 * ATT, device=self.dev)
        rs = N.RowStatsArgs(batch=B, channels=ATT, t_len=t4, act=N.ACT["leaky"], leaky_slope=LEAKY,
                            var_min=VAR_MIN, var_max=VAR_MAX,
                            x=xo.data_ptr(), x_sb=xo.stride(0), x_sc=xo.stride(1),
                            y=stats.data_ptr(), y_sb=stats.stride(0))
        N.check(N.lib.rave_row_stats(C.byref(rs), self._stream()), "speaker row stats")
        bias0 = torch.empty(B, ATT_HID, device=self.dev)  # attention.0.bias + [Wm | Ws] (mean, std)
        self._linear(stats, self._att0_stat, self._att0_b, bias0)
        hid = e(ATT_HID, t4)
        for b in range(B):                                # per-row bias: one launch per clip
            keep.append(self._conv("att0", xo, hid, act="leaky", bias=bias0[b], batch=1,
                                   x_off=b * xo.stride(0), y_off=b * hid.stride(0)))
        logits = e(ATT, t4)
        keep.append(self._conv("att3", hid, logits, act="relu"))
        pooled = torch.empty(B, 2 * ATT, device=self.dev)
        ap = N.AttnPoolArgs(batch=B, channels=ATT, t_len=t4, act=N.ACT["leaky"], leaky_slope=LEAKY,
                            var_min=VAR_MIN, var_max=VAR_MAX,
                            x=xo.data_ptr(), x_sb=xo.stride(0), x_sc=xo.stride(1),
                            logits=logits.data_ptr(), l_sb=logits.stride(0), l_sc=logits.stride(1),
                            y=pooled.data_ptr(), y_sb=pooled.stride(0))
        N.check(N.lib.rave_attn_pool(C.byref(ap), self._stream()), "speaker attention pooling")
        out = torch.empty(B, EMB, device=self.dev)
        self._linear(pooled, self._fc_w, self._fc_b, out)
        self._keep = keep                                 # workspaces live until the next call
        return out

    def _linear(self, x, w, b, y):
        N = self.N
        a = N.LinearArgs(batch=x.shape[0], n_in=w.shape[1], n_out=w.shape[0],
                         x=x.data_ptr(), x_sb=x.stride(0), w=w.data_ptr(), bias=b.data_ptr(),
                         y=y.data_ptr(), y_sb=y.stride(0))
        N.check(N.lib.rave_linear(C.byref(a), self._stream()), "speaker linear")

    def pqmf_bands(self, audio):
        """Centred 16-band PQMF analysis of (B, 1, T) audio, T a multiple of 16."""
        torch, N = self.torch, self.N
        if self._hkf is None:
            hkf, _ = self._P.kernels(self._P.design_bank(self._pqmf_att, BANDS))
            self._hkf = torch.from_numpy(hkf).to(self.dev)
        B, _, T = audio.shape
        if T % BANDS:
            raise ValueError(f"audio length {T} must be a multiple of {BANDS}")
        x = audio.contiguous()
        taps = self._hkf.shape[-1]
        pad = get_padding(taps, causal=self.causal)
        y = torch.empty(B, BANDS, T // BANDS, device=self.dev)
        a = N.AnalysisArgs(n_band=BANDS, taps=taps, n_out_bands=BANDS, batch=B, t_in=T, pad_left=pad[0],
                           t_out=T // BANDS, x=x.data_ptr(), x_sb=x.stride(0),
                           y=y.data_ptr(), y_sb=y.stride(0), y_sc=y.stride(1), hkf=self._hkf.data_ptr())
        N.check(N.lib.rave_pqmf_analysis(C.byref(a), self._stream()), "speaker pqmf")
        return y

    def embed(self, audio):
        """(B, 1, T) audio -> (B, 256): PQMF analysis (rave/model.py:246) then forward."""
        return self.forward(self.pqmf_bands(audio))
