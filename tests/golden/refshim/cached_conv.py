"""Restatement of the third-party ``cached_conv`` operator API.

Used ONLY by tests/golden/make_golden.py to path-import the reference blocks in
this container (the package, ``cached-conv>=2.5.0`` per
/root/reference/requirements.txt:14, is unpinned, not vendored and not
installed).  Written from the package's published behaviour; the semantics
pinned here:

* ``get_padding(k, stride, dilation, mode)``: p=(k-1)d+1; centered
  ((p-1)//2, p//2); causal (p-1, 0); k==1 -> (0,0).
* non-cached ``Conv1d``: explicit ``F.pad(x, padding)`` then conv;
  ``cumulative_delay = 0``.  Non-cached ``ConvTranspose1d`` = torch's.
* ``CachedConv1d``: left cache of ``l+r`` input samples, extra
  ``stride_delay = (s - ((r + cd) % s)) % s`` crop-pad, ``cumulative_delay =
  (r + stride_delay + cd) // s``.
* ``CachedConvTranspose1d``: transposed conv with padding 0, overlap-add of a
  ``2*padding`` cache, crop right, bias after; delay ``padding + cd*stride``.
* ``AlignBranches`` delays each branch's input by ``max(delays) - delay``.
* Caches hold ``MAX_BATCH_SIZE`` rows and are created on first call.

Validated by make_golden.py against the reference's own
tests/test_residual.py semantics (streaming == one-shot shifted by delay).
"""
import torch
import torch.nn as nn

MAX_BATCH_SIZE = 64
_USE_CACHED = False
USE_BUFFER_CONV = False       # the package's public flag (read by rave/resampler.py:21)
_PAD_MODE = "centered"
_CONVT_BIAS_DEFAULT = False   # v1.gin:34 cc.ConvTranspose1d.bias = False
_CONV_BIAS_DEFAULT = True     # v1.gin:33 cc.Conv1d.bias = True


def use_cached_conv(state: bool):
    global _USE_CACHED, USE_BUFFER_CONV
    _USE_CACHED = bool(state)
    USE_BUFFER_CONV = _USE_CACHED


def set_padding_mode(mode: str):
    global _PAD_MODE
    _PAD_MODE = mode


def get_padding(kernel_size, stride=1, dilation=1, mode=None):
    mode = mode or _PAD_MODE
    if kernel_size == 1:
        return (0, 0)
    p = (kernel_size - 1) * dilation + 1
    if mode == "centered":
        return ((p - 1) // 2, p // 2)
    if mode == "causal":
        return (p - 1, 0)
    raise ValueError(mode)


class CachedSequential(nn.Sequential):

    def __init__(self, *args, **kwargs):
        cumulative_delay = kwargs.pop("cumulative_delay", 0)
        stride = kwargs.pop("stride", 1)
        super().__init__(*args, **kwargs)
        self.cumulative_delay = int(cumulative_delay) * stride
        last = 0
        for i in range(1, len(self) + 1):
            if hasattr(self[-i], "cumulative_delay"):
                last = self[-i].cumulative_delay
                break
        self.cumulative_delay += last


class CachedPadding1d(nn.Module):

    def __init__(self, padding, crop=False):
        super().__init__()
        self.padding = int(padding)
        self.crop = crop
        self.initialized = 0

    def forward(self, x):
        if not self.initialized:
            self.register_buffer("pad", torch.zeros(MAX_BATCH_SIZE, x.shape[1], self.padding).to(x))
            self.initialized = 1
        if self.padding:
            x = torch.cat([self.pad[:x.shape[0]], x], -1)
            self.pad[:x.shape[0]].copy_(x[..., -self.padding:])
            if self.crop:
                x = x[..., :-self.padding]
        return x


class _Conv1d(nn.Conv1d):

    def __init__(self, *args, **kwargs):
        self._pad = tuple(kwargs.pop("padding", (0, 0)))
        kwargs.pop("cumulative_delay", None)
        kwargs.setdefault("bias", _CONV_BIAS_DEFAULT)
        super().__init__(*args, **kwargs)
        self.cumulative_delay = 0

    def forward(self, x):
        x = nn.functional.pad(x, self._pad)
        return nn.functional.conv1d(x, self.weight, self.bias, self.stride, 0, self.dilation, self.groups)


class CachedConv1d(nn.Conv1d):

    def __init__(self, *args, **kwargs):
        padding = kwargs.pop("padding", 0)
        cd = kwargs.pop("cumulative_delay", 0)
        kwargs.setdefault("bias", _CONV_BIAS_DEFAULT)
        super().__init__(*args, padding=0, **kwargs)
        if isinstance(padding, int):
            r_pad = padding
        else:
            r_pad = padding[1]
            padding = padding[0] + padding[1]
        s = self.stride[0]
        stride_delay = (s - ((r_pad + cd) % s)) % s
        self.cumulative_delay = (r_pad + stride_delay + cd) // s
        self.cache = CachedPadding1d(padding)
        self.downsampling_delay = CachedPadding1d(stride_delay, crop=True)

    def forward(self, x):
        x = self.downsampling_delay(x)
        x = self.cache(x)
        return nn.functional.conv1d(x, self.weight, self.bias, self.stride, 0, self.dilation, self.groups)


class _ConvTranspose1d(nn.ConvTranspose1d):

    def __init__(self, *args, **kwargs):
        kwargs.pop("cumulative_delay", None)
        kwargs.setdefault("bias", _CONVT_BIAS_DEFAULT)
        super().__init__(*args, **kwargs)
        self.cumulative_delay = 0


class CachedConvTranspose1d(nn.ConvTranspose1d):

    def __init__(self, *args, **kwargs):
        cd = kwargs.pop("cumulative_delay", 0)
        kwargs.setdefault("bias", _CONVT_BIAS_DEFAULT)
        super().__init__(*args, **kwargs)
        self.cumulative_delay = self.padding[0] + cd * self.stride[0]
        self.initialized = 0

    def forward(self, x):
        x = nn.functional.conv_transpose1d(x, self.weight, None, self.stride, 0,
                                           self.output_padding, self.groups, self.dilation)
        p = 2 * self.padding[0]
        if not self.initialized:
            self.register_buffer("cache", torch.zeros(MAX_BATCH_SIZE, x.shape[1], p).to(x))
            self.initialized = 1
        x[..., :p] += self.cache[:x.shape[0]]
        self.cache[:x.shape[0]].copy_(x[..., -p:])
        x = x[..., :-p]
        if self.bias is not None:
            x = x + self.bias.unsqueeze(-1)
        return x


def Conv1d(*args, **kwargs):
    return CachedConv1d(*args, **kwargs) if _USE_CACHED else _Conv1d(*args, **kwargs)


def ConvTranspose1d(*args, **kwargs):
    return CachedConvTranspose1d(*args, **kwargs) if _USE_CACHED else _ConvTranspose1d(*args, **kwargs)


class AlignBranches(nn.Module):

    def __init__(self, *branches, delays=None, cumulative_delay=0, stride=1):
        super().__init__()
        self.branches = nn.ModuleList(branches)
        if delays is None:
            delays = [b.cumulative_delay for b in self.branches]
        max_delay = max(delays)
        self.paddings = nn.ModuleList([CachedPadding1d(max_delay - d, crop=True) for d in delays])
        self.cumulative_delay = int(cumulative_delay * stride) + max_delay

    def forward(self, x):
        return [b(p(x)) for b, p in zip(self.branches, self.paddings)]
