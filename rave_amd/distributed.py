"""Batch data parallelism for offline encode/decode.

RAVE inference has no cross-sample coupling (no BatchNorm in EncoderV2 /
GeneratorV2, AdaIN statistics are per sample, RVQ is per frame), so the
utterance batch is sharded across ranks (one process per GPU) and every rank
runs the whole encode->decode path on its shard.  The one exchange step is an
all-gather of the latents over xGMI (RCCL, backend "nccl"), which makes the
full batch's ``encode`` output (B_global, C, T/hop) available on every rank;
each rank then decodes its own shard, so audio is never gathered.

The collective is latency-bound at these sizes (C2: 164 KB per rank), a single
``all_gather_into_tensor`` per step.  Every backend runs the same code: RCCL
(backend "nccl") on the GPU box and gloo in the CPU tests take the same
``all_gather_into_tensor`` calls on the same dtypes (RVQ codes narrowed to
int16 and carried as bytes), so the world-2 gloo tests exercise the RCCL path's
logic.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(n: int, rank: int, size: int) -> Tuple[int, int]:
    """Contiguous, balanced shard [lo, hi) of n items for ``rank``."""
    base, extra = divmod(n, size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_latents(z_local: torch.Tensor, out: Optional[torch.Tensor] = None,
                   group=None) -> torch.Tensor:
    """All-gather equally sized per-rank latent shards along dim 0.  Without a
    process group this is the identity; with one (any size, world size 1
    included) the shards always go through the backend's collective."""
    if not (dist.is_available() and dist.is_initialized()):
        return z_local
    size = dist.get_world_size(group)
    z_local = z_local.contiguous()
    if out is None:
        out = torch.empty((size * z_local.shape[0],) + tuple(z_local.shape[1:]),
                          dtype=z_local.dtype, device=z_local.device)
    dist.all_gather_into_tensor(out, z_local, group=group)
    return out


class ShardedRunner:
    """One data-parallel step on this rank's shard of the utterance batch.

    ``mode``:
      * ``"latent"`` (C2) -- encode -> all-gather latents -> decode;
      * ``"codes"`` (C4, DiscreteScriptedRAVE, scripts/export.py:503-517) --
        encode_codes -> all-gather the RVQ indices -> decode_codes.  Over RCCL
        the indices travel as int16 when the codebook fits (1024 entries: a
        quarter of the int64 bytes) and are widened back after the gather;
      * ``"decode"`` (C5) -- decode of the local latent shard; no exchange.

    Shards may differ in size (``shard_bounds`` of a batch that does not divide
    by the world size).  ``shard_sizes`` -- every rank's shard size, identical
    on all ranks -- fixes them up front; without it the sizes are all-gathered
    at every step (one 8-byte collective).  Unequal shards travel padded to the
    largest and are compacted after the gather.  Each rank decodes its own
    rows (the local tensor, so the decode does not wait for the exchange) and
    addresses AdaIN buffer rows by its global batch offset.  ``model`` is
    anything with the matching methods (rave_amd.RAVE on GPU)."""

    MODES = ("latent", "codes", "decode")

    def __init__(self, model, group=None, mode: str = "latent", shard_sizes: Optional[List[int]] = None):
        if mode not in self.MODES:
            raise ValueError(f"mode must be one of {self.MODES}")
        self.model = model
        self.group = group
        self.mode = mode
        self.shard_sizes = list(shard_sizes) if shard_sizes is not None else None
        self._all: Optional[torch.Tensor] = None

    def _narrow_codes(self) -> bool:
        rvq = getattr(getattr(self.model, "cfg", None), "rvq", None)
        return self.mode == "codes" and rvq is not None and rvq.codebook_size <= 32767

    def sizes(self, b: int, device) -> List[int]:
        """Every rank's shard size."""
        rank, size = world()
        if size == 1:
            return [b]
        if self.shard_sizes is not None:
            if len(self.shard_sizes) != size or self.shard_sizes[rank] != b:
                raise ValueError(f"shard_sizes {self.shard_sizes} do not match rank {rank}'s batch {b} "
                                 f"at world size {size}")
            return self.shard_sizes
        dev = device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        mine = torch.tensor([b], dtype=torch.int64, device=dev)
        out = torch.empty(size, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, mine, group=self.group)
        return [int(v) for v in out.tolist()]

    def _gather(self, t: torch.Tensor, sizes: List[int]) -> torch.Tensor:
        rank, size = world()
        if not (dist.is_available() and dist.is_initialized()):
            return t
        narrow = self._narrow_codes()
        # codes travel as int16 (1024-entry codebooks), viewed as bytes: every
        # backend moves uint8 (gloo has no int16 collectives)
        src = t.to(torch.int16).view(torch.uint8) if narrow else t
        bmax = max(sizes)
        if src.shape[0] < bmax:                  # unequal shards travel padded to the largest
            pad = torch.zeros((bmax - src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
            src = torch.cat([src, pad], 0)
        shape = (size * bmax,) + tuple(src.shape[1:])
        if self._all is None or tuple(self._all.shape) != shape or self._all.dtype != src.dtype:
            self._all = torch.empty(shape, dtype=src.dtype, device=src.device)
        out = gather_latents(src, self._all, self.group)
        if any(n != bmax for n in sizes):
            out = torch.cat([out[r * bmax:r * bmax + n] for r, n in enumerate(sizes)], 0)
        return out.view(torch.int16).to(t.dtype) if narrow else out

    def verify(self, x_local: torch.Tensor) -> dict:
        """One step's exchange checked end to end (call it outside any timed
        region): this rank's rows of the gathered tensor equal its own encode
        output bitwise, and every rank's rows match that rank's own checksum
        (float64 sum and abs-sum, all-gathered separately).  The verdict is
        reduced over ranks (MIN), so every rank returns the global result; a
        mismatch raises.  The latents are what the all-gather delivers to every
        rank, so this is what makes a wrong collective visible at N > 1."""
        rank, size = world()
        if self.mode == "decode":
            return {"checked": False, "reason": "decode mode has no exchange"}
        sizes = self.sizes(x_local.shape[0], x_local.device)
        local = self.model.encode_codes(x_local) if self.mode == "codes" else self.model.encode(x_local)
        allt = self._gather(local, sizes)
        off = sum(sizes[:rank])
        own = bool(torch.equal(allt[off:off + local.shape[0]], local))
        ld = local.double()
        mine = torch.stack([ld.sum(), ld.abs().sum()])
        if size > 1:
            dev = local.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
            sums = torch.empty(2 * size, dtype=torch.float64, device=dev)
            dist.all_gather_into_tensor(sums, mine.to(dev), group=self.group)
            sums = sums.view(size, 2).to(local.device)
        else:
            sums = mine.view(1, 2)
        worst = 0.0
        o = 0
        for r, n in enumerate(sizes):
            got = allt[o:o + n].double()
            ref = sums[r]
            err = torch.abs(torch.stack([got.sum(), got.abs().sum()]) - ref) / torch.clamp(ref[1].abs(), min=1.0)
            worst = max(worst, float(err.max()))
            o += n
        ok = own and worst <= 1e-12
        if size > 1:
            dev = local.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            ok = bool(flag.item())
        res = {"checked": True, "ranks": size, "rows": int(sum(sizes)), "own_rows_bitwise": own,
               "max_rel_checksum_err": worst, "ok": ok}
        if not ok:
            raise RuntimeError(f"all-gather check failed: {res}")
        return res

    def step(self, x_local: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(what every rank holds after the exchange, this rank's decoded audio)."""
        if self.mode == "decode":
            return x_local, self.model.decode(x_local)
        rank, _ = world()
        sizes = self.sizes(x_local.shape[0], x_local.device)
        if getattr(self.model, "adain", None) is not None:
            # AdaIN buffer rows follow the global batch index (rave/blocks.py:886-891)
            self.model.adain_row0 = sum(sizes[:rank])
        if self.mode == "codes":
            t = self.model.encode_codes(x_local)
            return self._gather(t, sizes), self.model.decode_codes(t)
        t = self.model.encode(x_local)
        return self._gather(t, sizes), self.model.decode(t)
