"""``RAVE``: the reference's encode / decode / forward surface on HIP kernels.

Mirrors ``rave.model.RAVE`` (rave/model.py:594-634):

* ``encode(x)``  x (B, 1, T) -> PQMF analysis -> bands[:, :6] -> EncoderV2 ->
  cat(z, speaker) = (B, latent + 256, T / hop)          (model.py:594-622)
* ``decode(z)``  GeneratorV2 -> PQMF synthesis -> (B, 1, T)   (model.py:624-629)
* ``forward(x)`` = decode(encode(x))                          (model.py:631-634)

and, for the discrete config, the nn~ export path of DiscreteScriptedRAVE
(scripts/export.py:503-517): ``encode_codes`` (encoder -> rvq.encode) and
``decode_codes`` (rvq.decode -> cat speaker -> decoder -> PQMF inverse).

Every call runs a pre-recorded launch plan (one ctypes call, all launches
issued from C++ on torch's current stream).  Tensors are torch CUDA tensors;
PyTorch only provides device memory and the stream.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Mapping, Optional, Tuple

import numpy as np
import torch

from . import _native as N
from . import pqmf as P
from .adain import AdainState
from .config import RaveConfig, get_padding
from .graph import ConvNode, build_graph
from .weights import check_params, conv_weight


# ============================================================ device constants
class Arena:
    """All constants of a model (packed conv weights, biases, Snake alphas,
    PQMF kernels, speaker embedding, codebooks) in one device allocation."""

    ALIGN = 64  # floats (256 B)

    def __init__(self):
        self._parts: List[np.ndarray] = []
        self.size = 0
        self.tensor: Optional[torch.Tensor] = None

    def add(self, arr: np.ndarray) -> int:
        arr = np.ascontiguousarray(arr, np.float32).reshape(-1)
        off = self.size
        self._parts.append((off, arr))
        self.size = off + ((arr.size + self.ALIGN - 1) // self.ALIGN) * self.ALIGN
        return off

    def upload(self, device) -> None:
        host = np.zeros(max(self.size, 1), np.float32)
        for off, arr in self._parts:
            host[off:off + arr.size] = arr
        self.tensor = torch.from_numpy(host).to(device)
        self._parts = []

    def ptr(self, off: int) -> int:
        return self.tensor.data_ptr() + 4 * off


# ============================================================ plans
@dataclass(frozen=True)
class View:
    """A (B, C, T) time-contiguous view: slot 'ws' (workspace), 'arena', 'abs'
    (``off`` is an absolute device address in bytes, elem 1), or an integer I/O
    slot bound at run time."""
    slot: object
    off: int          # elements from the slot base
    sb: int
    sc: int
    elem: int = 4     # bytes per element


class Workspace:
    """First-fit allocator with liveness-based reuse (sizes in floats)."""

    ALIGN = 64

    def __init__(self):
        self.free: List[Tuple[int, int]] = []
        self.top = 0

    def alloc(self, n: int) -> int:
        n = ((n + self.ALIGN - 1) // self.ALIGN) * self.ALIGN
        for i, (off, sz) in enumerate(self.free):
            if sz >= n:
                if sz == n:
                    self.free.pop(i)
                else:
                    self.free[i] = (off + n, sz - n)
                return off
        off = self.top
        self.top += n
        return off

    def release(self, off: int, n: int) -> None:
        n = ((n + self.ALIGN - 1) // self.ALIGN) * self.ALIGN
        self.free.append((off, n))
        self.free.sort()
        merged: List[Tuple[int, int]] = []
        for o, s in self.free:
            if merged and merged[-1][0] + merged[-1][1] == o:
                merged[-1] = (merged[-1][0], merged[-1][1] + s)
            else:
                merged.append((o, s))
        self.free = merged


def splitk_floats(scalars: dict, has_res: bool = False) -> int:
    """Split-K slab floats the native launcher wants for a conv (0 = unsplit)."""
    a = N.ConvArgs(**scalars)
    a.x = a.y = a.weight = a.alpha = 16   # placeholders: only shapes are inspected
    a.residual = 16 if has_res else None
    n = int(N.lib.rave_conv1d_workspace(C.byref(a)))
    if n < 0:
        N.check(N.RAVE_ERR_ARG, "conv1d_workspace")
    return n


class Plan:
    """Symbolic op list -> native rave_plan with relocations for I/O slots."""

    def __init__(self, arena: Arena):
        self.arena = arena
        self.ws = Workspace()
        self.splitk_off = -1
        self.sym: List[Tuple[int, type, dict, dict]] = []
        self.labels: List[str] = []
        self.flops: List[float] = []
        self.nbytes: List[float] = []     # algorithmic HBM bytes (tensors read/written once)
        self.handle = None
        self.ws_tensor: Optional[torch.Tensor] = None
        self._splitk: List[View] = []
        self.splitk_max = 0

    def splitk_view(self, floats: int) -> Optional[View]:
        """One shared split-K slab (dead after each conv's reduce), sized at
        finalize time to the largest request."""
        if floats <= 0:
            return None
        self.splitk_max = max(self.splitk_max, floats)
        v = View("splitk", 0, 0, 0)
        return v

    def add(self, kind: int, st: type, scalars: dict, ptrs: Dict[str, Optional[View]],
            label: str = "", flops: float = 0.0, nbytes: float = 0.0):
        self.sym.append((kind, st, scalars, ptrs))
        self.labels.append(label or {N.OP_CONV: "conv", N.OP_PQMF_ANALYSIS: "pqmf_analysis",
                                     N.OP_PQMF_SYNTHESIS: "pqmf_synthesis", N.OP_FILL: "fill",
                                     N.OP_RVQ_ENCODE: "rvq_encode", N.OP_RVQ_DECODE: "rvq_decode",
                                     N.OP_SHIFT_HISTORY: "shift_history", N.OP_COPY: "copy",
                                     N.OP_NOISE: "noise_synth", N.OP_ADAIN: "adain"}.get(kind, "op"))
        self.flops.append(float(flops))
        self.nbytes.append(float(nbytes))

    def finalize(self, device) -> "Plan":
        # The slab is live at different points of the plan than any tensor, so it
        # must not come from the free list (regions free at the END of planning
        # are in use mid-plan): bump-allocate past everything.
        splitk_off = self.splitk_off = self.ws.top
        self.ws.top += ((self.splitk_max + Workspace.ALIGN - 1) // Workspace.ALIGN) * Workspace.ALIGN
        self.ws_tensor = torch.empty(max(self.ws.top, 1), dtype=torch.float32, device=device)
        if self.splitk_max > 0:     # split-K arrival counters start (and stay) zero
            self.ws_tensor[splitk_off:splitk_off + N.SPLITK_TICKETS].zero_()
        n = len(self.sym)
        ops = (N.PlanOp * max(n, 1))()
        relocs = []
        for i, (kind, st, scalars, ptrs) in enumerate(self.sym):
            args = st()
            for k, v in scalars.items():
                setattr(args, k, v)
            for field, view in ptrs.items():
                if view is None:
                    setattr(args, field, None)
                    continue
                if view.slot == "ws":
                    setattr(args, field, self.ws_tensor.data_ptr() + view.elem * view.off)
                elif view.slot == "splitk":
                    setattr(args, field, self.ws_tensor.data_ptr() + 4 * splitk_off)
                elif view.slot == "arena":
                    setattr(args, field, self.arena.ptr(view.off))
                elif view.slot == "abs":
                    setattr(args, field, view.off)
                else:
                    setattr(args, field, None)
                    relocs.append(N.Reloc(i, getattr(st, field).offset, int(view.slot), 0,
                                          view.elem * view.off))
            ops[i].kind = kind
            C.memmove(ops[i].raw, C.addressof(args), C.sizeof(args))
        rl = (N.Reloc * max(len(relocs), 1))(*relocs)
        h = C.c_void_p()
        N.check(N.lib.rave_plan_create(ops, n, rl, len(relocs), C.byref(h)), "plan_create")
        self.handle = h
        return self

    def run(self, slots: List[int], stream: Optional[int] = None) -> None:
        arr = (C.c_void_p * len(slots))(*slots)
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        N.check(N.lib.rave_plan_run(self.handle, arr, len(slots), C.c_void_p(stream)), "plan_run")

    def profile(self, runs: int = 1) -> None:
        """Arm per-op timing for the next ``runs`` runs (0 disarms)."""
        N.check(N.lib.rave_plan_profile(self.handle, int(runs)), "plan_profile")

    def op_times(self, acc: Optional[np.ndarray] = None) -> Tuple[np.ndarray, int]:
        """(per-op milliseconds summed over the recorded runs, added into ``acc``;
        number of runs).  Re-arms the recorder."""
        n = len(self.sym)
        buf = (C.c_float * n)()
        if acc is not None:
            for i in range(n):
                buf[i] = float(acc[i])
        runs = N.lib.rave_plan_op_times(self.handle, buf, n)
        if runs < 0:
            N.check(runs, "plan_op_times")
        return np.array(list(buf), np.float64), runs

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and N is not None and N.lib is not None:
            N.lib.rave_plan_destroy(h)
            self.handle = None


# ============================================================ model
class RAVE:
    """HIP implementation of RAVE.encode / decode / forward for one config."""

    def __init__(self, cfg: RaveConfig, params: Mapping[str, np.ndarray], speaker: np.ndarray,
                 device=None, hk: Optional[np.ndarray] = None,
                 adain_stats: Optional[Mapping] = None, fuse_units: bool = True,
                 precision: str = "f32", tuning: Optional[list] = None,
                 autotune: Optional[bool] = None):
        check_params(cfg, params)
        if precision not in list(N.PRECISION) + ["auto"]:
            raise ValueError(f"precision must be one of {sorted(N.PRECISION) + ['auto']}")
        self.precision = precision
        # "auto": every conv / fused-unit op is timed in both arithmetic paths at
        # plan-build time on scratch tensors of its own shape; the faster is kept
        self.precs = [N.PREC_F32, N.PREC_SPLIT16] if precision == "auto" else [N.PRECISION[precision]]
        self.prec = self.precs[-1]
        # launch configurations (tile, K-splits) timed per conv op at plan build:
        # by default with "auto" precision, else the launchers' heuristics
        self.autotune = precision == "auto" if autotune is None else bool(autotune)
        self._tuned: Dict[tuple, Tuple[int, float]] = {}   # op key -> (choice, ms)
        if tuning:                  # choices recorded by tuning() of an earlier model
            self._tuned = {tuple(k): (c, ms) for k, c, ms in tuning}
        self.cfg = cfg
        self.graph = build_graph(cfg)
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("rave_amd.RAVE runs on the GPU only (device must be cuda)")
        ar = Arena()
        # packed conv weights per precision: (name, prec) -> arena offset
        self.w_off: Dict[str, Tuple[int, Optional[int], Optional[int]]] = {}   # f32 / first precision
        self.w_pack: Dict[Tuple[str, int], int] = {}
        self.w_pack_stream: Dict[Tuple[str, int], int] = {}
        for n in self.graph.convs():
            w = conv_weight(n, params)
            for pr in self.precs:
                self.w_pack[(n.name, pr)] = ar.add(N.pack_conv_weight(
                    w, n.c_in, n.c_out, n.kernel, n.stride, n.dilation, n.transposed, precision=pr))
                if n.transposed:   # cached (streaming) form: overlap-add cache, no r//2 crop
                    self.w_pack_stream[(n.name, pr)] = ar.add(N.pack_conv_weight(
                        w, n.c_in, n.c_out, n.kernel, n.stride, n.dilation, True, out_shift=0, precision=pr))
            bo = ar.add(params[n.name + ".bias"]) if n.bias else None
            ao = ar.add(params[n.alpha]) if n.act == "snake" else None
            self.w_off[n.name] = (self.w_pack[(n.name, self.precs[0])], bo, ao)
        # fused Residual(DilatedUnit) weights: (k=3 node name, prec) -> arena offset
        self.unit_pack: Dict[Tuple[str, int], int] = {}
        self.unit_off: Dict[str, int] = {}
        if fuse_units:
            for k3, k1 in self._unit_pairs(self.graph.convs()):
                for pr in self.precs:
                    if N.unit_supported(k3.c_in, pr):
                        self.unit_pack[(k3.name, pr)] = ar.add(N.pack_unit_weight(
                            conv_weight(k3, params), conv_weight(k1, params), k3.c_in, precision=pr))
                cands = [pr for pr in self.precs if (k3.name, pr) in self.unit_pack]
                if cands:
                    self.unit_off[k3.name] = self.unit_pack[(k3.name, cands[0])]
        self.noise_target = int(np.prod(cfg.noise.ratios)) if cfg.noise is not None else 0
        self.hk = P.design_bank(cfg.pqmf_attenuation, cfg.n_band) if hk is None else np.asarray(hk, np.float32)
        hkf, hki = P.kernels(self.hk)
        self.taps_a, self.taps_s = hkf.shape[-1], hki.shape[-1]
        self.hkf_off = ar.add(hkf)
        self.hki_off = ar.add(hki)
        spk = np.asarray(speaker, np.float32).reshape(-1)
        if spk.size != cfg.speaker_size:
            raise ValueError(f"speaker embedding must have {cfg.speaker_size} values")
        self.spk_off = ar.add(spk)
        self.cb_off = None
        if cfg.rvq is not None:
            cbs = np.stack([np.asarray(params[f"encoder.rvq.layers.{i}._codebook.embed"], np.float32)
                            for i in range(cfg.rvq.num_quantizers)])
            self.cb_off = ar.add(cbs)
        ar.upload(self.device)
        self.arena = ar
        self._plans: Dict[tuple, Plan] = {}
        # AdaIN buffers (rave/blocks.py:856-919): identity until statistics are
        # loaded or learned; ``adain_row0`` is the first buffer row this
        # process's batch uses (batch shards of a data-parallel job).
        self.adain: Optional[AdainState] = None
        self.adain_row0 = 0
        if cfg.adain:
            self.adain = AdainState(self.graph.adain_modules, self.device)
            if adain_stats:
                self.adain.load(adain_stats)
        elif adain_stats:
            raise ValueError("adain_stats given for a config without AdaIN")

    @staticmethod
    def _unit_pairs(nodes: List[ConvNode]) -> List[Tuple[ConvNode, ConvNode]]:
        """(k=3 dilated conv, 1x1 conv) pairs forming Residual(DilatedUnit)
        (rave/blocks.py:32-46, 84-113): the 1x1 reads the k=3 output and adds
        the k=3 input back."""
        out = []
        for a, b in zip(nodes, nodes[1:]):
            if (a.kernel == 3 and a.stride == 1 and not a.transposed and b.kernel == 1
                    and b.src == a.dst and b.residual == a.src and a.c_in == a.c_out == b.c_out
                    and a.act == b.act and a.bias == b.bias):
                out.append((a, b))
        return out

    # ------------------------------------------------------------ per-op precision choice
    def tuning(self) -> list:
        """The autotuner's choices so far, JSON-serialisable; pass it back as
        ``RAVE(..., tuning=...)`` to build the same plans without timing runs."""
        return [[list(k), int(c), float(ms)] for k, (c, ms) in self._tuned.items()]

    def _time_native(self, fn, args, reps: int = 5) -> float:
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(2):
            N.check(fn(C.byref(args), st), "autotune")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn(C.byref(args), st)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def _bind_scratch(self, args, ptrs: Dict[str, Optional[View]], shapes: Dict[str, tuple],
                      keep: list) -> None:
        """Point an op's pointer fields at scratch tensors (tensor fields) or the
        arena (constants) for a timing run."""
        for field, view in ptrs.items():
            if view is None:
                setattr(args, field, None)
            elif view.slot == "arena":
                setattr(args, field, self.arena.ptr(view.off))
            elif view.slot == "abs":
                setattr(args, field, view.off)
            else:
                t = torch.randn(shapes[field], device=self.device) * 0.5
                keep.append(t)
                setattr(args, field, t.data_ptr())

    def _pick(self, key: tuple, cands: List[int], run, timed: bool = False) -> int:
        """The faster precision of ``cands`` for the op ``key`` (cached with its
        time); ``run(prec)`` returns milliseconds.  A single candidate is only
        timed when ``timed`` (its time is wanted by a fusion decision)."""
        if len(cands) == 1 and not timed:
            return cands[0]
        if key not in self._tuned:
            times = {pr: run(pr) for pr in cands}
            best = min(times, key=times.get)
            self._tuned[key] = (best, times[best])
        return self._tuned[key][0]

    def _fuse_unit(self, k3: ConvNode, k1: ConvNode, B: int, T: int, src: View) -> bool:
        """Run Residual(DilatedUnit) as the fused kernel (True) or as its two
        convs (False): with several precisions the faster by measurement
        (e.g. exact-fp32 fused against two split-f16 convs at C=512)."""
        if len(self.precs) == 1:
            return True
        key = ("fuse", k3.name, B, T)
        if key not in self._tuned:
            fused_ms = self._unit_time(k3, k1, B, T)
            tmp = View("t", 0, k3.c_out * T, T)
            s3, p3 = self._conv_desc(k3, B, T, src, tmp, None)
            self.conv_launch(k3, s3, p3, timed=True)
            s1, p1 = self._conv_desc(k1, B, T, tmp, tmp, src)
            self.conv_launch(k1, s1, p1, timed=True)
            split_ms = (self._tuned[self._conv_key(k3, False, s3)][1]
                        + self._tuned[self._conv_key(k1, False, s1)][1])
            self._tuned[key] = (fused_ms <= split_ms, min(fused_ms, split_ms))
        return bool(self._tuned[key][0])

    def _unit_best_ms(self, k3: ConvNode, k1: ConvNode, B: int, T: int) -> float:
        """Measured time of a unit as the plan would run it (fused or two convs)."""
        if len(self.precs) > 1:
            self._fuse_unit(k3, k1, B, T, View("t", 0, k3.c_in * T, T))
            return float(self._tuned[("fuse", k3.name, B, T)][1])
        return self._unit_time(k3, k1, B, T)

    def _stack_runs(self, nodes: List[ConvNode]) -> Dict[str, List[Tuple[ConvNode, ConvNode]]]:
        """Runs of N.STACK_UNITS consecutive Residual(DilatedUnit)s of one width
        (the residual stacks of EncoderV2 / GeneratorV2, rave/blocks.py:533-558,
        647-664) that rave_residual_stack can run: first k=3 node name -> units."""
        pairs, out, i, U = self._unit_pairs(nodes), {}, 0, N.STACK_UNITS
        adain_on = self.adain is not None and self.adain.active
        while i + U <= len(pairs):
            run = pairs[i:i + U]
            a0 = run[0][0]
            ok = (all(run[k + 1][0].src == run[k][1].dst for k in range(U - 1))
                  and all(k3.c_in == a0.c_in and k3.act == a0.act and k3.bias == a0.bias for k3, _ in run)
                  and N.stack_supported(a0.c_in)
                  and all((k3.name, N.PREC_SPLIT16) in self.unit_pack for k3, _ in run)
                  and not (adain_on and any(k3.adain for k3, _ in run)))
            if ok:
                out[a0.name] = run
                i += U
            else:
                i += 1
        return out

    def _stack_parts(self, run: List[Tuple[ConvNode, ConvNode]], B: int, T: int):
        """(scalars, pointer views, timing run) of one residual-stack op."""
        arena = lambda o: View("arena", o, 0, 0) if o is not None else None  # noqa: E731
        C_ = run[0][0].c_in
        s = dict(channels=C_, batch=B, t_len=T, act=N.ACT[run[0][0].act], leaky_slope=self.cfg.leaky_slope)
        p: Dict[str, Optional[View]] = {}
        for u, (k3, k1) in enumerate(run):
            _, b1, a0 = self.w_off[k3.name]
            _, b2, a2 = self.w_off[k1.name]
            s[f"dilation{u}"], s[f"pad_left{u}"] = k3.dilation, k3.pad[0]
            p.update({f"weight{u}": arena(self.unit_pack[(k3.name, N.PREC_SPLIT16)]),
                      f"bias1{u}": arena(b1), f"bias2{u}": arena(b2),
                      f"alpha0{u}": arena(a0), f"alpha2{u}": arena(a2)})

        def run_t():
            args = N.StackArgs(**s, x_sb=C_ * T, x_sc=T, y_sb=C_ * T, y_sc=T)
            keep: list = []
            self._bind_scratch(args, dict(p, x=View("t", 0, 0, 0), y=View("t", 0, 0, 0)),
                               {"x": (B, C_, T), "y": (B, C_, T)}, keep)
            return self._time_native(N.lib.rave_residual_stack, args)

        return s, p, run_t

    def _use_stack(self, run: List[Tuple[ConvNode, ConvNode]], B: int, T: int) -> bool:
        """One rave_residual_stack launch instead of the units: always in
        split16-only mode, else when it measures faster than the units' best."""
        if N.PREC_SPLIT16 not in self.precs:
            return False
        if len(self.precs) == 1 and not self.autotune:
            return True
        key = ("stack", run[0][0].name, B, T)
        if key not in self._tuned:
            try:
                st_ms = self._stack_parts(run, B, T)[2]()
            except (NotImplementedError, ValueError):
                self._tuned[key] = (0, 0.0)
                return False
            units_ms = sum(self._unit_best_ms(k3, k1, B, T) for k3, k1 in run)
            self._tuned[key] = (int(st_ms <= units_ms), min(st_ms, units_ms))
        return bool(self._tuned[key][0])

    def _stack(self, plan: Plan, run: List[Tuple[ConvNode, ConvNode]], B: int, T: int, src: View,
               dst: View) -> None:
        s, p, _ = self._stack_parts(run, B, T)
        s.update(x_sb=src.sb, x_sc=src.sc, y_sb=dst.sb, y_sc=dst.sc)
        C_ = run[0][0].c_in
        plan.add(N.OP_STACK, N.StackArgs, s, dict(p, x=src, y=dst),
                 label=run[0][0].name.rsplit(".net.", 2)[0] + ".stack",
                 flops=2.0 * B * T * C_ * C_ * 4 * len(run),
                 nbytes=4.0 * (2 * B * C_ * T + 4 * C_ * C_ * len(run)))

    def _unit_parts(self, k3: ConvNode, k1: ConvNode, B: int, T: int):
        """(descriptor builder, fused-kernel precisions, timing run) of one unit."""
        _, b1, a0 = self.w_off[k3.name]
        _, b2, a2 = self.w_off[k1.name]
        arena = lambda o: View("arena", o, 0, 0) if o is not None else None  # noqa: E731
        C_ = k3.c_in
        cands = [pr for pr in self.precs if (k3.name, pr) in self.unit_pack]

        def desc(pr, x_sb, x_sc, y_sb, y_sc):
            s = dict(channels=C_, batch=B, t_len=T, dilation=k3.dilation, pad_left=k3.pad[0],
                     act=N.ACT[k3.act], leaky_slope=self.cfg.leaky_slope, precision=pr,
                     x_sb=x_sb, x_sc=x_sc, y_sb=y_sb, y_sc=y_sc)
            p = dict(weight=arena(self.unit_pack[(k3.name, pr)]), bias1=arena(b1), bias2=arena(b2),
                     alpha0=arena(a0), alpha2=arena(a2))
            return s, p

        def run(pr):
            s, p = desc(pr, C_ * T, T, C_ * T, T)
            args = N.UnitArgs(**s)
            keep: list = []
            self._bind_scratch(args, dict(p, x=View("t", 0, 0, 0), y=View("t", 0, 0, 0)),
                               {"x": (B, C_, T), "y": (B, C_, T)}, keep)
            return self._time_native(N.lib.rave_residual_unit, args)

        return desc, cands, run

    def _unit_time(self, k3: ConvNode, k1: ConvNode, B: int, T: int) -> float:
        _, cands, run = self._unit_parts(k3, k1, B, T)
        key = ("unit", k3.name, B, T)
        self._pick(key, cands, run, timed=True)
        return self._tuned[key][1]

    def _unit(self, plan: Plan, k3: ConvNode, k1: ConvNode, B: int, T: int, src: View,
              dst: View) -> None:
        desc, cands, run = self._unit_parts(k3, k1, B, T)
        C_ = k3.c_in
        pr = self._pick(("unit", k3.name, B, T), cands, run)
        s, p = desc(pr, src.sb, src.sc, dst.sb, dst.sc)
        plan.add(N.OP_UNIT, N.UnitArgs, s, dict(p, x=src, y=dst),
                 label=k3.name.rsplit(".net.", 1)[0] + ".unit",
                 flops=2.0 * B * T * C_ * C_ * 4, nbytes=4.0 * (2 * B * C_ * T + 4 * C_ * C_))

    def _adain_key(self) -> tuple:
        return self.adain.key() + (self.adain_row0,) if self.adain is not None else ()

    def _adain_op(self, plan: Plan, name: str, B: int, C: int, T: int, x: View) -> None:
        """AdaIN in place on the residual unit's input (it is both the unit's
        conv input and its residual, and has no other reader)."""
        ad = self.adain
        if self.adain_row0 + B > ad.max_batch:
            raise ValueError(f"AdaIN statistics hold {ad.max_batch} batch rows "
                             f"(cc.MAX_BATCH_SIZE); batch {B} at row {self.adain_row0} exceeds them")
        st, cnt, tk = ad.ptrs(name)
        plan.add(N.OP_ADAIN, N.AdainArgs,
                 dict(batch=B, channels=C, t_len=T, mode=ad.mode, max_batch=ad.max_batch,
                      row0=self.adain_row0, x_sb=x.sb, x_sc=x.sc, y_sb=x.sb, y_sc=x.sc),
                 dict(x=x, y=x, stats=View("abs", st, 0, 0, elem=1),
                      counters=View("abs", cnt, 0, 0, elem=1), ticket=View("abs", tk, 0, 0, elem=1)),
                 label="adain:" + name)

    # ------------------------------------------------------------ plan pieces
    @staticmethod
    def _conv_key(n: ConvNode, stream_form: bool, scalars: dict) -> tuple:
        return ("conv", n.name, stream_form, scalars["batch"], scalars["t_in"])

    def conv_launch(self, n: ConvNode, scalars: dict, ptrs: Dict[str, Optional[View]],
                    stream_form: bool = False, timed: bool = False) -> Tuple[int, int]:
        """(precision, launch config) of one conv op.  With ``autotune`` every
        precision and every launch configuration rave_conv1d_configs() lists
        (tile shape, K-splits, split-K combine) is timed once on scratch tensors
        of the op's shape and the fastest kept; else config 0 (the launcher's
        heuristic).  ``scalars`` / ``ptrs`` describe the op without them."""
        pack = self.w_pack_stream if stream_form else self.w_pack
        key = self._conv_key(n, stream_form, scalars)
        if key not in self._tuned and (len(self.precs) > 1 or timed or self.autotune):
            B, t_in, t_out = scalars["batch"], scalars["t_in"], scalars["t_out"]
            shapes = {"x": (B, n.c_in, t_in), "y": (B, n.c_out, t_out), "residual": (B, n.c_out, t_out)}
            keep: list = []
            p = dict(ptrs, partial=None)
            for f in ("x", "y", "residual"):
                if p.get(f) is not None:
                    p[f] = View("t", 0, 0, 0)
            base = N.ConvArgs(**scalars)
            base.x_sb, base.x_sc = n.c_in * t_in, t_in
            base.y_sb = base.r_sb = n.c_out * t_out
            base.y_sc = base.r_sc = t_out
            self._bind_scratch(base, p, shapes, keep)
            cands = []
            for pr in self.precs:
                base.precision = pr
                base.weight = self.arena.ptr(pack[(n.name, pr)])
                cfgs = N.conv_configs(base) if (self.autotune or len(self.precs) > 1) else []
                cands += [(pr, c) for c in [0] + cfgs]
            nws = 0
            for pr, c in cands:
                base.precision, base.config = pr, c
                base.weight = self.arena.ptr(pack[(n.name, pr)])
                nws = max(nws, int(N.lib.rave_conv1d_workspace(C.byref(base))))
            ws = torch.zeros(max(nws, 1), device=self.device)   # counters zero, slabs free
            times = {}
            for pr, c in cands:
                args = N.ConvArgs.from_buffer_copy(base)
                args.precision, args.config = pr, c
                args.weight = self.arena.ptr(pack[(n.name, pr)])
                args.partial = ws.data_ptr() if nws > 0 else None
                try:
                    times[(pr, c)] = self._time_native(N.lib.rave_conv1d, args)
                except (NotImplementedError, ValueError):
                    if c == 0:
                        raise               # the default configuration must run

            best = min(times, key=times.get)
            self._tuned[key] = (best[0] * self.CFG_BASE + best[1], times[best])
        if key in self._tuned:
            v = int(self._tuned[key][0])
            return v // self.CFG_BASE, v % self.CFG_BASE
        return self.precs[0], 0

    CFG_BASE = 1 << 16          # tuned conv choice = precision * CFG_BASE + config

    def _conv_desc(self, n: ConvNode, B: int, t_in: int, src: View, dst: View,
                   res: Optional[View]) -> Tuple[dict, Dict[str, Optional[View]]]:
        """Scalars and pointer views of one conv op, without precision / weight."""
        _, bo, ao = self.w_off[n.name]
        t_out = n.out_len(t_in)
        s = dict(c_in=n.c_in, c_out=n.c_out, kernel=n.kernel, stride=n.stride, dilation=n.dilation,
                 act=N.ACT[n.act], leaky_slope=self.cfg.leaky_slope, batch=B, t_in=t_in, t_out=t_out,
                 x_sb=src.sb, x_sc=src.sc, y_sb=dst.sb, y_sc=dst.sc,
                 r_sb=res.sb if res else 0, r_sc=res.sc if res else 0)
        if n.transposed:
            s.update(pad_left=0, pad_right=0, transposed=1, out_shift=n.stride // 2)
        else:
            s.update(pad_left=n.pad[0], pad_right=n.pad[1], transposed=0, out_shift=0)
        ptrs = dict(x=src, y=dst, residual=res,
                    bias=View("arena", bo, 0, 0) if bo is not None else None,
                    alpha=View("arena", ao, 0, 0) if ao is not None else None)
        return s, ptrs

    def _conv(self, plan: Plan, n: ConvNode, B: int, t_in: int, src: View, dst: View,
              res: Optional[View]) -> int:
        t_out = n.out_len(t_in)
        s, ptrs = self._conv_desc(n, B, t_in, src, dst, res)
        pr, cfg = self.conv_launch(n, s, ptrs)
        s["precision"], s["config"] = pr, cfg
        ptrs["weight"] = View("arena", self.w_pack[(n.name, pr)], 0, 0)
        ptrs["partial"] = plan.splitk_view(splitk_floats(s, res is not None))
        if n.transposed:
            flops = 2.0 * B * n.c_out * t_out * n.c_in * 2          # 2 taps per output sample
        else:
            flops = 2.0 * B * n.c_out * t_out * n.c_in * n.kernel
        nbytes = 4.0 * (B * n.c_in * t_in + B * n.c_out * t_out * (2 if res is not None else 1)
                        + n.c_in * n.c_out * n.kernel)
        plan.add(N.OP_CONV, N.ConvArgs, s, ptrs, label=n.name, flops=flops, nbytes=nbytes)
        return t_out

    def _run_stack(self, plan: Plan, nodes: List[ConvNode], B: int, inputs: Dict[str, Tuple[View, int]],
                   outputs: Dict[str, View]) -> Dict[str, Tuple[View, int, int]]:
        """Lay a conv sequence into the plan, allocating workspace tensors with
        liveness-based reuse.  inputs: name -> (view, T)."""
        last_use: Dict[str, int] = {}
        for i, n in enumerate(nodes):
            last_use[n.src] = i
            if n.residual:
                last_use[n.residual] = i
        tensors: Dict[str, Tuple[View, int, int]] = {k: (v, t, -1) for k, (v, t) in inputs.items()}
        fused = {a.name: b for a, b in self._unit_pairs(nodes) if a.name in self.unit_off}
        stacks = self._stack_runs(nodes) if self.unit_off else {}
        skip = set()
        for i, n in enumerate(nodes):
            if n.name in skip:
                continue
            src, t_in, _ = tensors[n.src]
            if n.adain and self.adain is not None and self.adain.active:
                self._adain_op(plan, n.adain, B, n.c_in, t_in, src)
            if n.name in stacks and self._use_stack(stacks[n.name], B, t_in):
                # the whole residual stack in one kernel; unit outputs never reach HBM
                run = stacks[n.name]
                last = run[-1][1]
                for k3, k1 in run:
                    skip.update((k3.name, k1.name))
                if last.dst in outputs:
                    dst, size = outputs[last.dst], -1
                else:
                    size = B * last.c_out * t_in
                    dst = View("ws", plan.ws.alloc(size), last.c_out * t_in, t_in)
                self._stack(plan, run, B, t_in, src, dst)
                tensors[last.dst] = (dst, t_in, size)
                if last_use.get(n.src, -1) <= i + 2 * len(run) - 1 and n.src in tensors:
                    v, _, sz = tensors[n.src]
                    if sz > 0 and v.slot == "ws" and n.src not in outputs:
                        plan.ws.release(v.off, sz)
                continue
            if n.name in fused and self._fuse_unit(n, fused[n.name], B, t_in, src):
                # Residual(DilatedUnit) in one kernel; the k=3 output never exists in HBM
                k1 = fused[n.name]
                skip.add(k1.name)
                if k1.dst in outputs:
                    dst, size = outputs[k1.dst], -1
                else:
                    size = B * k1.c_out * t_in
                    dst = View("ws", plan.ws.alloc(size), k1.c_out * t_in, t_in)
                self._unit(plan, n, k1, B, t_in, src, dst)
                tensors[k1.dst] = (dst, t_in, size)
                for name in {n.src}:
                    if last_use.get(name) == i + 1 and name in tensors:
                        v, _, sz = tensors[name]
                        if sz > 0 and v.slot == "ws" and name not in outputs:
                            plan.ws.release(v.off, sz)
                continue
            t_out = n.out_len(t_in)
            if n.dst in outputs:
                dst = outputs[n.dst]
                size = -1
            else:
                size = B * n.c_out * t_out
                dst = View("ws", plan.ws.alloc(size), n.c_out * t_out, t_out)
            res = tensors[n.residual][0] if n.residual else None
            self._conv(plan, n, B, t_in, src, dst, res)
            tensors[n.dst] = (dst, t_out, size)
            for name in {n.src, n.residual}:
                if name and last_use.get(name) == i and name in tensors:
                    v, _, sz = tensors[name]
                    if sz > 0 and v.slot == "ws" and name not in outputs:
                        plan.ws.release(v.off, sz)
        return tensors

    def _analysis(self, plan: Plan, B: int, T: int, x: View, y: View, n_out: int) -> int:
        cfg = self.cfg
        F = T // cfg.n_band
        pad = get_padding(self.taps_a, causal=cfg.causal)[0]
        plan.add(N.OP_PQMF_ANALYSIS, N.AnalysisArgs,
                 dict(n_band=cfg.n_band, taps=self.taps_a, n_out_bands=n_out, batch=B, t_in=T,
                      pad_left=pad, t_out=F, x_sb=x.sb, y_sb=y.sb, y_sc=y.sc),
                 dict(x=x, y=y, hkf=View("arena", self.hkf_off, 0, 0)),
                 flops=2.0 * B * n_out * F * self.taps_a, nbytes=4.0 * (B * T + B * n_out * F))
        return F

    def _synthesis(self, plan: Plan, B: int, F: int, x: View, y: View, mode: int,
                   noise: Optional[View] = None, frame0: int = 0) -> None:
        cfg = self.cfg
        pad = get_padding(self.taps_s, causal=cfg.causal)[0]
        plan.add(N.OP_PQMF_SYNTHESIS, N.SynthesisArgs,
                 dict(n_band=cfg.n_band, taps=self.taps_s, batch=B, t_in=F, pad_left=pad, mode=mode,
                      frame0=frame0, x_sb=x.sb, x_sc=x.sc,
                      n_sb=noise.sb if noise else 0, n_sc=noise.sc if noise else 0, y_sb=y.sb),
                 dict(x=x, y=y, noise=noise, hki=View("arena", self.hki_off, 0, 0)),
                 flops=2.0 * B * F * cfg.n_band * cfg.n_band * self.taps_s,
                 nbytes=4.0 * (2 * B * F * cfg.n_band + (B * F * cfg.n_band if noise else 0)))

    def _fill_speaker(self, plan: Plan, B: int, Fz: int, z: View) -> None:
        cfg = self.cfg
        plan.add(N.OP_FILL, N.FillArgs,
                 dict(batch=B, channels=cfg.speaker_size, t_len=Fz, y_sb=z.sb, y_sc=z.sc),
                 dict(y=z, values=View("arena", self.spk_off, 0, 0)))

    # ------------------------------------------------------------ plans
    def _encode_plan(self, B: int, T: int, codes: bool = False) -> Plan:
        key = ("enc_codes" if codes else "enc", B, T) + self._adain_key()
        if key in self._plans:
            return self._plans[key]
        cfg = self.cfg
        plan = Plan(self.arena)
        F = T // cfg.n_band
        Fz = T // cfg.hop
        bands_sz = B * cfg.enc_bands * F
        bands = View("ws", plan.ws.alloc(bands_sz), cfg.enc_bands * F, F)
        self._analysis(plan, B, T, View(0, 0, T, T), bands, cfg.enc_bands)
        if codes:
            lat = View("ws", plan.ws.alloc(B * cfg.latent_size * Fz), cfg.latent_size * Fz, Fz)
        else:
            zc = cfg.latent_size + cfg.speaker_size
            lat = View(1, 0, zc * Fz, Fz)
        self._run_stack(plan, self.graph.encoder, B, {"enc_in": (bands, F)}, {"latent": lat})
        if codes:
            rq = cfg.rvq
            sc = dict(n_q=rq.num_quantizers, codebook_size=rq.codebook_size, dim=cfg.latent_size,
                      batch=B, t_len=Fz, z_sb=lat.sb, z_sc=lat.sc,
                      i_sb=rq.num_quantizers * Fz, i_sq=Fz, y_sb=0, y_sc=0)
            nw = int(N.lib.rave_rvq_workspace(C.byref(N.RvqArgs(**sc))))
            if nw < 0:
                N.check(nw, "rvq_workspace")
            plan.add(N.OP_RVQ_ENCODE, N.RvqArgs, sc,
                     dict(codebooks=View("arena", self.cb_off, 0, 0), z=lat,
                          idx=View(1, 0, 0, 0, elem=8), y=None,
                          work=View("ws", plan.ws.alloc(max(nw, 1)), 0, 0)))
        else:
            self._fill_speaker(plan, B, Fz, View(1, cfg.latent_size * Fz, lat.sb, Fz))
        self._plans[key] = plan.finalize(self.device)
        return plan

    def _decode_plan(self, B: int, Fz: int, codes: bool = False) -> Plan:
        key = ("dec_codes" if codes else "dec", B, Fz) + self._adain_key()
        if key in self._plans:
            return self._plans[key]
        cfg = self.cfg
        plan = Plan(self.arena)
        zc = cfg.dec_in
        if codes:
            rq = cfg.rvq
            z = View("ws", plan.ws.alloc(B * zc * Fz), zc * Fz, Fz)
            plan.add(N.OP_RVQ_DECODE, N.RvqArgs,
                     dict(n_q=rq.num_quantizers, codebook_size=rq.codebook_size, dim=cfg.latent_size,
                          batch=B, t_len=Fz, z_sb=0, z_sc=0, i_sb=rq.num_quantizers * Fz, i_sq=Fz,
                          y_sb=z.sb, y_sc=z.sc),
                     dict(codebooks=View("arena", self.cb_off, 0, 0), z=None,
                          idx=View(0, 0, 0, 0, elem=8), y=z))
            self._fill_speaker(plan, B, Fz, View("ws", z.off + cfg.latent_size * Fz, z.sb, Fz))
        else:
            z = View(0, 0, zc * Fz, Fz)
        F = Fz * cfg.hop // cfg.n_band
        wave = View("ws", plan.ws.alloc(B * cfg.dec_out * F), cfg.dec_out * F, F)
        outputs = {"wave": wave}
        noise = None
        if cfg.noise is not None:
            nz = cfg.noise
            Fn = F // self.noise_target
            na = cfg.n_band * nz.noise_bands
            outputs["noise_amp"] = View("ws", plan.ws.alloc(B * na * Fn), na * Fn, Fn)
        self._run_stack(plan, self.graph.decoder + self.graph.noise, B, {"dec_in": (z, Fz)}, outputs)
        if cfg.noise is not None:
            # NoiseGeneratorV2 filter stage; the uniform noise is I/O slot 2
            noise = View("ws", plan.ws.alloc(B * cfg.n_band * F), cfg.n_band * F, F)
            amp = outputs["noise_amp"]
            plan.add(N.OP_NOISE, N.NoiseArgs,
                     dict(batch=B, frames=Fn, n_band=cfg.n_band, noise_bands=nz.noise_bands,
                          target=self.noise_target, a_sb=amp.sb, a_sc=amp.sc,
                          u_sb=Fn * cfg.n_band * self.noise_target, y_sb=noise.sb, y_sc=noise.sc),
                     dict(amp=amp, u=View(2, 0, 0, 0), y=noise))
        T = F * cfg.n_band
        self._synthesis(plan, B, F, wave, View(1, 0, T, T), 1 if cfg.amplitude_modulation else 2,
                        noise=noise)
        self._plans[key] = plan.finalize(self.device)
        return plan

    # ------------------------------------------------------------ public API
    def _check_audio(self, x: torch.Tensor) -> Tuple[int, int]:
        if not isinstance(x, torch.Tensor) or x.device.type != "cuda" or x.dtype != torch.float32:
            raise ValueError("x must be a float32 CUDA tensor")
        if x.dim() != 3 or x.shape[1] != 1:
            raise ValueError(f"x must be (B, 1, T), got {tuple(x.shape)}")
        B, _, T = x.shape
        if T % self.cfg.hop:
            raise ValueError(f"T={T} must be a multiple of {self.cfg.hop} (n_band * prod(ratios))")
        return B, T

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        B, T = self._check_audio(x)
        x = x.contiguous()
        Fz = T // self.cfg.hop
        z = torch.empty(B, self.cfg.latent_size + self.cfg.speaker_size, Fz, device=x.device)
        self._encode_plan(B, T).run([x.data_ptr(), z.data_ptr()])
        return z

    def noise_shape(self, B: int, Fz: int) -> Tuple[int, int, int, int]:
        """Shape of NoiseGeneratorV2's uniform noise (torch.rand_like(ir),
        rave/blocks.py:287): (B, frames, n_band, target_size)."""
        F = Fz * self.cfg.hop // self.cfg.n_band
        return (B, F // self.noise_target, self.cfg.n_band, self.noise_target)

    def _noise_slot(self, B: int, Fz: int, noise_u: Optional[torch.Tensor], dev) -> List[int]:
        if self.cfg.noise is None:
            if noise_u is not None:
                raise ValueError("noise_u given for a config without a noise synthesizer")
            return []
        shape = self.noise_shape(B, Fz)
        if noise_u is None:
            noise_u = torch.rand(shape, device=dev)      # rand_like on the device RNG
        elif (noise_u.dtype != torch.float32 or noise_u.device.type != "cuda"
              or tuple(noise_u.shape) != shape):
            raise ValueError(f"noise_u must be a float32 CUDA tensor of shape {shape}")
        self._noise_keep = noise_u = noise_u.contiguous()
        return [noise_u.data_ptr()]

    def decode(self, z: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        """GeneratorV2 -> PQMF inverse.  For a noise config, ``noise_u`` (U[0,1),
        ``noise_shape``) replaces the reference's torch.rand_like draw; when
        omitted it is drawn on the device."""
        if not isinstance(z, torch.Tensor) or z.device.type != "cuda" or z.dtype != torch.float32:
            raise ValueError("z must be a float32 CUDA tensor")
        if z.dim() != 3 or z.shape[1] != self.cfg.dec_in:
            raise ValueError(f"z must be (B, {self.cfg.dec_in}, T), got {tuple(z.shape)}")
        z = z.contiguous()
        B, _, Fz = z.shape
        y = torch.empty(B, 1, Fz * self.cfg.hop, device=z.device)
        slots = [z.data_ptr(), y.data_ptr()] + self._noise_slot(B, Fz, noise_u, z.device)
        self._decode_plan(B, Fz).run(slots)
        return y

    def forward(self, x: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.decode(self.encode(x), noise_u)

    __call__ = forward

    def encode_codes(self, x: torch.Tensor) -> torch.Tensor:
        """encoder -> rvq.encode: (B, n_q, T/hop) int64 (discrete config)."""
        if self.cfg.rvq is None:
            raise ValueError("encode_codes needs a discrete (RVQ) config")
        B, T = self._check_audio(x)
        x = x.contiguous()
        idx = torch.empty(B, self.cfg.rvq.num_quantizers, T // self.cfg.hop, dtype=torch.int64,
                          device=x.device)
        self._encode_plan(B, T, codes=True).run([x.data_ptr(), idx.data_ptr()])
        return idx

    def decode_codes(self, idx: torch.Tensor) -> torch.Tensor:
        """rvq.decode (indices clamped as DiscreteScriptedRAVE) -> cat speaker ->
        decoder -> PQMF inverse."""
        if self.cfg.rvq is None:
            raise ValueError("decode_codes needs a discrete (RVQ) config")
        if idx.dtype != torch.int64 or idx.device.type != "cuda" or idx.dim() != 3 \
                or idx.shape[1] != self.cfg.rvq.num_quantizers:
            raise ValueError("idx must be an int64 CUDA tensor (B, n_q, T)")
        idx = idx.contiguous()
        B, _, Fz = idx.shape
        y = torch.empty(B, 1, Fz * self.cfg.hop, device=idx.device)
        slots = [idx.data_ptr(), y.data_ptr()] + self._noise_slot(B, Fz, None, idx.device)
        self._decode_plan(B, Fz, codes=True).run(slots)
        return y

    def forward_codes(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode_codes(self.encode_codes(x))
