"""Multi-process (gloo, world_size 2, CPU) coverage of the batch-sharded
encode -> all-gather latents -> decode path of rave_amd.distributed.  The
model here is the CPU oracle restricted to its encode/decode (the HIP model
needs a GPU); what is tested is the sharding, the collective and that the
sharded result equals the single-process result."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _OracleModel:
    """encode/decode on torch CPU tensors through the oracle (test stand-in)."""

    def __init__(self):
        from oracle.rave_oracle import Oracle
        from rave_amd import config as rcfg
        from rave_amd.weights import init_params, init_speaker
        cfg = rcfg.v2(capacity=4)
        self.o = Oracle(cfg, init_params(cfg, 0), init_speaker(cfg, 0))

    def encode(self, x):
        return torch.from_numpy(self.o.encode(x.numpy()).astype(np.float32))

    def decode(self, z):
        return torch.from_numpy(self.o.decode(z.numpy()).astype(np.float32))


def _worker(rank, size, port, x_all, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        from rave_amd.distributed import ShardedRunner, shard_bounds
        lo, hi = shard_bounds(x_all.shape[0], rank, size)
        runner = ShardedRunner(_OracleModel())
        z_all, y = runner.step(x_all[lo:hi])
        q.put((rank, z_all.numpy(), y.numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_encode_gather_decode_matches_single_process():
    rng = np.random.default_rng(0)
    x_all = torch.from_numpy((0.2 * rng.standard_normal((4, 1, 2048))).astype(np.float32))
    ref_model = _OracleModel()
    z_ref = ref_model.encode(x_all)
    y_ref = ref_model.decode(z_ref)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, x_all, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    for rank, z_all, y in res:
        np.testing.assert_allclose(z_all, z_ref.numpy(), atol=1e-6)     # every rank holds all latents
        np.testing.assert_allclose(y, y_ref.numpy()[rank * 2:(rank + 1) * 2], atol=1e-6)


def test_shard_bounds_cover_batch():
    from rave_amd.distributed import shard_bounds
    for n in (1, 7, 16, 64, 128):
        for size in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, size) for r in range(size)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(size - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
