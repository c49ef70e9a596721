"""Host-side contract of the operator seam (rave_amd.cc / rave_amd.modules):
the module tree carries the reference's state_dict names, scripts for
TorchScript (nn~), keeps cached_conv's delay bookkeeping, and refuses CPU
tensors (no CPU fallback).  No GPU needed; the kernels run in test_gpu_cc.py."""
import pytest
import torch

from rave_amd import cc
from rave_amd import config as rcfg
from rave_amd.modules import DilatedUnit, RAVEModules, Residual, load_reference_state
from rave_amd.weights import init_params, init_speaker


@pytest.mark.parametrize("name", ["v2", "causal", "discrete", "v3", "v3_noise"])
def test_tree_names_match_reference_state_dict(name):
    cfg = rcfg.get_config(name, capacity=8)
    m = RAVEModules(cfg, init_speaker(cfg, 0))
    params = init_params(cfg, 0)
    expected = set()
    for k in params:
        if k.startswith("encoder.rvq."):
            continue
        expected.add(k[:-len("_g")] if k.endswith(".weight_g") else k)
    expected = {k for k in expected if not k.endswith(".weight_v")}
    buffers = {k for k, _ in m.named_buffers()}
    own = {k for k in m.state_dict() if k not in ("speaker", "pqmf.hk") and k not in buffers}
    assert own == expected, (sorted(own - expected)[:4], sorted(expected - own)[:4])
    if cfg.adain:   # AdaIN buffers under the reference's names (rave/blocks.py:858-868)
        assert "encoder.encoder.net.1.mean_x" in buffers and "decoder.net.3.num_update_y" in buffers
    load_reference_state(m, params)


@pytest.mark.parametrize("name", ["causal", "v3_noise"])
@pytest.mark.parametrize("cached", [False, True])
def test_tree_scripts(cached, name):
    cc.use_cached_conv(cached)
    try:
        m = RAVEModules(rcfg.get_config(name, capacity=8))
    finally:
        cc.use_cached_conv(False)
    ts = torch.jit.script(m)
    assert hasattr(ts, "encode") and hasattr(ts, "decode")


def test_cached_delay_bookkeeping():
    """cached_conv's cumulative delays: a centred k3
    conv with dilation d lags d, Residual aligns its identity branch by the
    unit's delay, a strided k 2r conv lags one output frame, ConvTranspose r//2."""
    cc.use_cached_conv(True)
    try:
        unit = DilatedUnit(8, 3, 3)
        res = Residual(DilatedUnit(8, 3, 9))
        down = cc.Conv1d(8, 16, 8, stride=4, padding=cc.get_padding(8, 4))
        up = cc.ConvTranspose1d(16, 8, 8, stride=4, padding=2)
        cc.set_padding_mode("causal")
        causal_unit = DilatedUnit(8, 3, 3)
    finally:
        cc.use_cached_conv(False)
        cc.set_padding_mode("centered")
    assert unit.cumulative_delay == 3
    assert res.cumulative_delay == 9 and res.aligned.paddings[1].padding == 9
    assert down.cumulative_delay == 1 and down.stride_delay == 0
    assert up.cumulative_delay == 2
    assert causal_unit.cumulative_delay == 0


def test_cpu_tensors_are_refused():
    conv = cc.Conv1d(4, 4, 3, padding=1)
    with pytest.raises((ValueError, RuntimeError)):
        conv(torch.zeros(1, 4, 16))
    with pytest.raises(NotImplementedError):
        cc.Conv1d(4, 4, 3, groups=2)
