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


class _OracleCodesModel:
    """encode_codes/decode_codes (DiscreteScriptedRAVE, scripts/export.py:503-517)
    through the oracle on the discrete config (test stand-in)."""

    def __init__(self):
        from oracle.rave_oracle import Oracle
        from rave_amd import config as rcfg
        from rave_amd.weights import init_params, init_speaker
        self.cfg = rcfg.discrete(capacity=4)
        self.o = Oracle(self.cfg, init_params(self.cfg, 0), init_speaker(self.cfg, 0))

    def encode_codes(self, x):
        return torch.from_numpy(self.o.rvq_encode(self.o.encode(x.numpy())).astype(np.int64))

    def decode_codes(self, idx):
        z = self.o.cat_speaker(self.o.rvq_decode(idx.numpy()))
        return torch.from_numpy(self.o.decode(z).astype(np.float32))

    def decode(self, z):
        return torch.from_numpy(self.o.decode(z.numpy()).astype(np.float32))


def _worker(rank, size, port, x_all, q, mode="latent", fixed_sizes=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        from rave_amd.distributed import ShardedRunner, shard_bounds
        spans = [shard_bounds(x_all.shape[0], r, size) for r in range(size)]
        lo, hi = spans[rank]
        model = _OracleModel() if mode == "latent" else _OracleCodesModel()
        sizes = [h - l for l, h in spans] if fixed_sizes else None
        runner = ShardedRunner(model, mode=mode, shard_sizes=sizes)
        z_all, y = runner.step(x_all[lo:hi])
        chk = runner.verify(x_all[lo:hi])          # the exchange self-check bench.py runs
        assert chk["ok"] and chk["ranks"] == size and chk["rows"] == x_all.shape[0], chk
        q.put((rank, z_all.numpy(), y.numpy()))
    finally:
        dist.destroy_process_group()


def _run_world2(x_all, mode, fixed_sizes=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, x_all, q, mode, fixed_sizes)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda t: t[0])


@pytest.mark.parametrize("n", [4, 3])
def test_sharded_codes_gather_matches_single_process(n):
    """C4's path: encode_codes per shard -> all-gather of the RVQ indices (as
    int16 bytes, the RCCL path's own code) -> decode_codes of the local rows;
    every rank holds the batch's indices.  n=3: unequal shards travel padded."""
    from rave_amd.distributed import shard_bounds
    rng = np.random.default_rng(1)
    x_all = torch.from_numpy((0.2 * rng.standard_normal((n, 1, 2048))).astype(np.float32))
    m = _OracleCodesModel()
    idx_ref = m.encode_codes(x_all)
    y_ref = m.decode_codes(idx_ref)
    for rank, idx_all, y in _run_world2(x_all, "codes"):
        lo, hi = shard_bounds(n, rank, 2)
        assert idx_all.dtype == np.int64
        np.testing.assert_array_equal(idx_all, idx_ref.numpy())
        np.testing.assert_allclose(y, y_ref.numpy()[lo:hi], atol=1e-6)


def test_sharded_decode_mode_has_no_exchange():
    """C5's path: each rank decodes its own latent shard; nothing is gathered."""
    from rave_amd.distributed import ShardedRunner
    m = _OracleCodesModel()
    z = torch.from_numpy(np.random.default_rng(2).standard_normal((1, 384, 2)).astype(np.float32))
    held, y = ShardedRunner(m, mode="decode").step(z)
    assert held is z
    np.testing.assert_allclose(y.numpy(), m.decode(z).numpy(), atol=0)
    with pytest.raises(ValueError):
        ShardedRunner(m, mode="tokens")


@pytest.mark.parametrize("n,fixed", [(4, True), (3, False)])
def test_sharded_encode_gather_decode_matches_single_process(n, fixed):
    """Equal shards with the sizes given up front, and an odd batch (2 + 1
    clips) whose sizes are exchanged and whose shards travel padded."""
    from rave_amd.distributed import shard_bounds
    rng = np.random.default_rng(0)
    x_all = torch.from_numpy((0.2 * rng.standard_normal((n, 1, 2048))).astype(np.float32))
    ref_model = _OracleModel()
    z_ref = ref_model.encode(x_all)
    y_ref = ref_model.decode(z_ref)
    for rank, z_all, y in _run_world2(x_all, "latent", fixed_sizes=fixed):
        lo, hi = shard_bounds(n, rank, 2)
        np.testing.assert_allclose(z_all, z_ref.numpy(), atol=1e-6)     # every rank holds all latents
        np.testing.assert_allclose(y, y_ref.numpy()[lo:hi], atol=1e-6)


def test_shard_sizes_must_match():
    from rave_amd.distributed import ShardedRunner
    r = ShardedRunner(_OracleModel(), shard_sizes=[2, 2])
    assert r.sizes(5, torch.device("cpu")) == [5]          # single process: no exchange


def test_shard_bounds_cover_batch():
    from rave_amd.distributed import shard_bounds
    for n in (1, 7, 16, 64, 128):
        for size in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, size) for r in range(size)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(size - 1))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _bench_worker(rank, size, port, x_all, sizes, q):
    """bench.py's own timed region (bench.timed_region: warmup, barrier +
    sync, K steps, MAX over ranks) around a codes-mode ShardedRunner step with
    unequal shards fixed up front, then the exchange self-check."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        import time
        from bench import timed_region
        from rave_amd.distributed import ShardedRunner
        lo = sum(sizes[:rank])
        x = x_all[lo:lo + sizes[rank]]
        runner = ShardedRunner(_OracleCodesModel(), mode="codes", shard_sizes=sizes)
        held = []

        def step():
            if rank == 1:
                time.sleep(0.05)                  # the slow rank sets the job's time
            idx_all, y = runner.step(x)
            held.append(idx_all)
            return y

        el, y = timed_region(step, 2, 1, size, lambda: None, torch.device("cpu"))
        chk = runner.verify(x)
        q.put((rank, el, held[-1].numpy(), y.numpy(), chk))
    finally:
        dist.destroy_process_group()


def test_bench_timed_region_codes_unequal_shards():
    """C4's codes mode at world size 2 with shards of 2 and 1 clips, through
    bench.py's timed region: every rank reports the same (max) elapsed time,
    which covers the slow rank's two timed steps; every rank holds the whole
    batch's indices; each decodes its own rows; the exchange check passes."""
    rng = np.random.default_rng(3)
    x_all = torch.from_numpy((0.2 * rng.standard_normal((3, 1, 2048))).astype(np.float32))
    sizes = [2, 1]
    m = _OracleCodesModel()
    idx_ref = m.encode_codes(x_all)
    y_ref = m.decode_codes(idx_ref)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, x_all, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    els = [r[1] for r in res]
    assert els[0] == els[1] and els[0] >= 2 * 0.05
    for rank, _, idx_all, y, chk in res:
        lo = sum(sizes[:rank])
        np.testing.assert_array_equal(idx_all, idx_ref.numpy())
        np.testing.assert_allclose(y, y_ref.numpy()[lo:lo + sizes[rank]], atol=1e-6)
        assert chk["ok"] and chk["rows"] == 3 and chk["ranks"] == 2
