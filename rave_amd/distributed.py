"""Batch data parallelism for offline encode/decode.

RAVE inference has no cross-sample coupling (no BatchNorm in EncoderV2 /
GeneratorV2, AdaIN statistics are per sample, RVQ is per frame), so the
utterance batch is sharded across ranks (one process per GPU) and every rank
runs the whole encode->decode path on its shard.  The one exchange step is an
all-gather of the latents over xGMI (RCCL, backend "nccl"), which makes the
full batch's ``encode`` output (B_global, C, T/hop) available on every rank;
each rank then decodes its own shard, so audio is never gathered.

The collective is latency-bound at these sizes (C2: 164 KB per rank), a single
``all_gather_into_tensor`` per step.  With the gloo backend (CPU tests) the
list form of all_gather is used.
"""
from __future__ import annotations

from typing import Optional, Tuple

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
    """All-gather equally sized per-rank latent shards along dim 0."""
    rank, size = world()
    if size == 1:
        return z_local
    z_local = z_local.contiguous()
    if out is None:
        out = torch.empty((size * z_local.shape[0],) + tuple(z_local.shape[1:]),
                          dtype=z_local.dtype, device=z_local.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, z_local, group=group)
    else:
        parts = list(out.chunk(size, 0))
        dist.all_gather(parts, z_local, group=group)
    return out


class ShardedRunner:
    """encode (local shard) -> all-gather latents -> decode (local shard).

    ``model`` is anything with ``encode``/``decode`` (rave_amd.RAVE on GPU)."""

    def __init__(self, model, group=None):
        self.model = model
        self.group = group
        self._z_all: Optional[torch.Tensor] = None

    def step(self, x_local: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        rank, size = world()
        if getattr(self.model, "adain", None) is not None:
            # AdaIN buffer rows follow the global batch index (rave/blocks.py:886-891)
            self.model.adain_row0 = rank * x_local.shape[0]
        z = self.model.encode(x_local)
        if size > 1:
            shape = (size * z.shape[0],) + tuple(z.shape[1:])
            if self._z_all is None or tuple(self._z_all.shape) != shape:
                self._z_all = torch.empty(shape, dtype=z.dtype, device=z.device)
            z_all = gather_latents(z, self._z_all, self.group)
            zl = z_all[rank * z.shape[0]:(rank + 1) * z.shape[0]]
        else:
            z_all = zl = z
        return z_all, self.model.decode(zl)
