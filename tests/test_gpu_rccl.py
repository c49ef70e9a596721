"""The RCCL (backend "nccl") branch of rave_amd.distributed on the GPU box.

The box has one GPU, and RCCL refuses two ranks on one device, so this runs a
world-size-1 "nccl" process group: the shards still travel through RCCL's
``all_gather_into_tensor`` (ShardedRunner gathers whenever a process group
exists), on the dtypes the product sends -- fp32 latents (C2) and RVQ codes
narrowed to int16 and carried as bytes (C4).  The world-2 logic (uneven shards,
padding, per-rank decode) is covered on gloo by tests/test_distributed_gloo.py.
Expected results: the same model's direct encode/decode on the same input."""
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    assert dist.get_backend() == "nccl"
    yield dev
    dist.destroy_process_group()


def _synth(B, T, seed):
    rng = np.random.default_rng(seed)
    n = np.arange(T)
    x = 0.3 * np.sin(2 * np.pi * 440 * n / 48000)[None, None, :] + 0.1 * rng.standard_normal((B, 1, T))
    return x.astype(np.float32)


def test_rccl_latent_gather(nccl_group):
    from rave_amd import config as rcfg
    from rave_amd.distributed import ShardedRunner
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    dev = nccl_group
    cfg = rcfg.get_config("v2")
    m = RAVE(cfg, init_params(cfg, seed=0), init_speaker(cfg, seed=0), device=dev, precision="auto")
    x = torch.from_numpy(_synth(2, 8192, 0)).to(dev)
    runner = ShardedRunner(m, shard_sizes=[2])
    z_all, y = runner.step(x)
    torch.cuda.synchronize()
    assert runner._all is not None and runner._all.data_ptr() == z_all.data_ptr()   # the RCCL output buffer
    z = m.encode(x)
    assert torch.equal(z_all, z)
    assert torch.equal(y, m.decode(z))
    chk = runner.verify(x)                    # bench.py's exchange self-check, through RCCL
    assert chk["ok"] and chk["own_rows_bitwise"] and chk["max_rel_checksum_err"] == 0.0


def test_rccl_codes_gather_int16(nccl_group):
    from rave_amd import config as rcfg
    from rave_amd.distributed import ShardedRunner
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    dev = nccl_group
    cfg = rcfg.discrete(capacity=8)
    m = RAVE(cfg, init_params(cfg, seed=1), init_speaker(cfg, seed=1), device=dev, precision="auto")
    x = torch.from_numpy(_synth(2, 8192, 1)).to(dev)
    runner = ShardedRunner(m, mode="codes")
    assert runner._narrow_codes()
    idx_all, y = runner.step(x)
    torch.cuda.synchronize()
    assert runner._all.dtype == torch.uint8                 # int16 codes carried as bytes over RCCL
    idx = m.encode_codes(x)
    assert idx_all.dtype == idx.dtype and torch.equal(idx_all, idx)
    assert runner.verify(x)["ok"]
    assert torch.equal(y, m.decode_codes(idx))
