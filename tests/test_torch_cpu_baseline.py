"""bench.py's CPU baseline (oracle/torch_cpu.py: the reference's module graph on
torch fp32 CPU / oneDNN) against the golden fixtures made by running the
reference itself, so the CPU number bench.py reports is the same computation."""
import numpy as np
import pytest
import torch

from oracle.torch_cpu import TorchCPURave
from rave_amd import config as rcfg
from rave_amd.weights import init_params

TOL = 1e-4


@pytest.mark.parametrize("name,cfg", [("v2", rcfg.v2()), ("causal", rcfg.causal())])
def test_torch_cpu_matches_reference_fixtures(golden, name, cfg):
    g = golden(name)
    hk = golden("pqmf")["hk"]
    m = TorchCPURave(cfg, init_params(cfg, seed=int(g["seed"])), g["speaker"], hk=hk)
    with torch.no_grad():
        z = m.encode(torch.from_numpy(np.asarray(g["x"], np.float32))).numpy()
        y = m.decode(torch.from_numpy(np.asarray(g["z"], np.float32))).numpy()
    assert np.abs(z - g["z"]).max() < TOL
    assert np.abs(y - g["y"]).max() < TOL


def test_torch_cpu_rejects_unsupported():
    cfg = rcfg.discrete()
    with pytest.raises(NotImplementedError):
        TorchCPURave(cfg, {}, np.zeros(256))
