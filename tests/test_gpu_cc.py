"""The operator-level seam (rave_amd.cc + rave_amd.modules): the reference's
module tree written against ``cc.Conv1d`` / ``cc.ConvTranspose1d`` /
``CachedPQMF`` runs on the HIP kernels through torch.ops.rave_amd.* and
reproduces the reference's fixtures -- per layer (offline), block for block
(cached_conv streaming, causal and centred), and RVQ indices.  Runs on an
MI355X only (``-m gpu``)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

TOL = 1e-4


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _conv_hooks(m, got):
    """Forward hooks recording every cc conv's output under its module name.  A
    conv that carries its Residual's sum in its epilogue (``forward(h,
    residual, ...)``: each DilatedUnit's last conv) reports the conv alone --
    output minus the residual it was given -- which is what the reference's
    hook on that nn.Conv1d saw (rave/blocks.py:44-46 adds after the module)."""
    from rave_amd import cc

    def hook(mod, i, o, n):
        r = i[1] if len(i) > 1 else None
        got[n] = (o - r if r is not None else o).detach().cpu().numpy()
    return [mod.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n))
            for n, mod in m.named_modules() if isinstance(mod, (cc.Conv1d, cc.ConvTranspose1d))]


def _tree(cfg, g, golden, dev, cached=False, precision="f32"):
    from rave_amd import cc
    from rave_amd.modules import RAVEModules, load_reference_state
    from rave_amd.weights import init_params
    cc.use_cached_conv(cached)
    cc.set_precision(precision)
    try:
        m = RAVEModules(cfg, g["speaker"], hk=golden("pqmf")["hk"])
    finally:
        cc.use_cached_conv(False)
        cc.set_precision("f32")
    load_reference_state(m, init_params(cfg, seed=int(g["seed"])))
    return m.to(dev).eval()


@pytest.mark.parametrize("precision", ["f32", "split16"])
def test_cc_tree_per_layer_golden(dev, golden, precision):
    """Every conv of the v2 tree (capacity 8) against the reference's per-layer
    outputs (tests/golden/v2_small_layers.npz, forward hooks on the reference
    modules of the same names); z and y within 1e-4; the scripted tree equal."""
    from rave_amd import config as rcfg
    cfg = rcfg.v2(capacity=8)
    g = golden("v2_small_layers")
    m = _tree(cfg, g, golden, dev, precision=precision)
    got = {}
    hooks = _conv_hooks(m, got)
    with torch.no_grad():
        z = m.encode(torch.from_numpy(g["x"]).to(dev))
        y = m.decode(torch.from_numpy(g["z"]).to(dev))
    for h in hooks:
        h.remove()
    layers = [k[len("layer/"):] for k in g if k.startswith("layer/")]
    assert layers and set(layers) <= set(got), sorted(set(layers) - set(got))[:5]
    worst = 0.0
    for name in layers:
        ref = g["layer/" + name]
        err = maxabs(got[name], ref)
        worst = max(worst, err / max(1.0, float(np.abs(ref).max())))
        assert err <= 2e-5 * max(1.0, float(np.abs(ref).max())), (name, err)
    ez = maxabs(z.cpu().numpy()[:, :cfg.latent_size], g["z"][:, :cfg.latent_size])
    ey = maxabs(y.cpu().numpy(), g["y"])
    print(f"\n[cc] v2 cap 8 {precision}: {len(layers)} layers, worst rel {worst:.2e}; z {ez:.2e} y {ey:.2e}")
    assert ez < TOL and ey < TOL
    ts = torch.jit.script(m)
    with torch.no_grad():
        ys = ts.decode(torch.from_numpy(g["z"]).to(dev))
    assert maxabs(ys.cpu().numpy(), y.cpu().numpy()) == 0.0


@pytest.mark.parametrize("name,fixture", [("causal", "causal_stream"), ("v2", "v2_stream")])
def test_cc_cached_tree_streams_reference(dev, golden, name, fixture):
    """cc.use_cached_conv(True) before construction: the tree streams 2048-sample
    blocks and matches the reference's cached_conv run block for block
    (causal, and the reference's default centred model)."""
    from rave_amd import config as rcfg
    cfg = rcfg.get_config(name)
    g = golden(fixture)
    m = _tree(cfg, g, golden, dev, cached=True)
    blk = int(g["block"])
    Fz = blk // cfg.hop
    x = torch.from_numpy(g["x"]).to(dev)
    z = torch.from_numpy(g["z"]).to(dev)
    nb = x.shape[-1] // blk
    with torch.no_grad():
        zs = torch.cat([m.encode(x[..., i * blk:(i + 1) * blk]) for i in range(nb)], -1)
        ys = torch.cat([m.decode(z[..., i * Fz:(i + 1) * Fz]) for i in range(nb)], -1)
    ez, ey = maxabs(zs.cpu().numpy(), g["z_stream"]), maxabs(ys.cpu().numpy(), g["y_stream"])
    print(f"\n[cc] cached {name} tree vs reference streaming: z {ez:.2e} y {ey:.2e}")
    assert ez < TOL and ey < TOL


def test_cc_rvq_ops_golden(dev, golden):
    """cc.rvq_encode / rvq_decode against the reference's RVQ fixture (indices
    exact outside the tie margin)."""
    from rave_amd import cc
    from rave_amd import config as rcfg
    from rave_amd.weights import init_params
    g = golden("rvq")
    cfg = rcfg.discrete()
    params = init_params(cfg, seed=int(g["seed"]))
    cbs = torch.from_numpy(np.stack([params[f"encoder.rvq.layers.{i}._codebook.embed"] for i in range(16)])).to(dev)
    z = torch.from_numpy(g["z"]).to(dev)
    idx = cc.rvq_encode(z, cbs)
    zq = cc.rvq_decode(torch.from_numpy(g["idx"]).to(dev), cbs)
    torch.cuda.synchronize()
    got, ref = idx.cpu().numpy(), g["idx"]
    B, _, T = z.shape
    gap = g["gap"].reshape(16, B, T).transpose(1, 0, 2)
    mism = got != ref
    assert (gap[mism] < 1e-3).all()
    assert maxabs(zq.cpu().numpy(), g["zq"]) < 1e-5


def test_cc_conv_module_contract(dev):
    """cc.Conv1d / ConvTranspose1d keep torch's parameter layout (weight_norm
    applies; a changed weight is re-packed) and refuse shapes the kernels do
    not take."""
    from rave_amd import cc
    from oracle.rave_oracle import conv1d, conv_transpose1d
    conv = cc.Conv1d(16, 32, 3, padding=cc.get_padding(3, dilation=2), dilation=2).to(dev)
    assert tuple(conv.weight.shape) == (32, 16, 3)
    x = torch.randn(2, 16, 100, device=dev)
    ref = conv1d(x.cpu().double().numpy(), conv.weight.detach().cpu().numpy(), conv.bias.detach().cpu().numpy(),
                 1, 2, (2, 2))
    assert maxabs(conv(x).detach().cpu().numpy(), ref) < 1e-5
    with torch.no_grad():
        conv.weight.mul_(2.0)                          # in-place change: re-packed on the next call
    assert maxabs(conv(x).detach().cpu().numpy(), conv1d(x.cpu().double().numpy(),
                  conv.weight.detach().cpu().numpy(), conv.bias.detach().cpu().numpy(), 1, 2, (2, 2))) < 1e-5
    wn = torch.nn.utils.weight_norm(cc.Conv1d(16, 8, 1).to(dev))
    assert hasattr(wn, "weight_g") and tuple(wn(x).shape) == (2, 8, 100)
    ct = cc.ConvTranspose1d(16, 8, 8, stride=4, padding=2).to(dev)
    refc = conv_transpose1d(x.cpu().double().numpy(), ct.weight.detach().cpu().numpy(), 4, 2, None)
    assert maxabs(ct(x).detach().cpu().numpy(), refc) < 1e-5
    with pytest.raises(NotImplementedError):
        cc.ConvTranspose1d(16, 8, 5, stride=2, padding=1)


def _set_adain(m, lx, ly, reset=False):
    """nn~'s learn / reset attributes on every AdaIN module (eager or scripted):
    the reference's buffer names (rave/blocks.py:858-884)."""
    vals = {"learn_x": float(lx), "learn_y": float(ly)}
    if reset:
        vals.update(mean_x=0.0, std_x=1.0, num_update_x=0.0, mean_y=0.0, std_y=1.0, num_update_y=0.0)
    n = 0
    for name, buf in m.named_buffers():
        leaf = name.rsplit(".", 1)[-1]
        if leaf in vals and (".net." in name or name.startswith("net.")):
            buf.fill_(vals[leaf])
            n += leaf == "learn_x"
    assert n > 0


@pytest.mark.parametrize("precision", ["f32", "split16"])
def test_cc_v3_noise_tree_per_layer_golden(dev, golden, precision):
    """The v3 tree with AdaIN, Snake and NoiseGeneratorV2 (capacity 8) on the
    operator seam, every conv against the reference's per-layer outputs
    (tests/golden/v3_noise_small_layers.npz: the residual convs, the noise
    module's three convs, the waveform module), z and y within 1e-4 with the
    reference's uniform noise injected; the scripted tree equal."""
    from rave_amd import config as rcfg
    cfg = rcfg.v3_noise(capacity=8)
    g = golden("v3_noise_small_layers")
    m = _tree(cfg, g, golden, dev, precision=precision)
    got = {}
    hooks = _conv_hooks(m, got)
    u = torch.from_numpy(g["noise_u"]).to(dev)
    with torch.no_grad():
        z = m.encode(torch.from_numpy(g["x"]).to(dev))
        y = m.decode(torch.from_numpy(g["z"]).to(dev), u)
    for h in hooks:
        h.remove()
    layers = [k[len("layer/"):] for k in g if k.startswith("layer/")]
    assert {"decoder.noise_module.net.4", "decoder.waveform_module"} <= set(layers)
    assert layers and set(layers) <= set(got), sorted(set(layers) - set(got))[:5]
    worst = 0.0
    for name in layers:
        ref = g["layer/" + name]
        err = maxabs(got[name], ref)
        worst = max(worst, err / max(1.0, float(np.abs(ref).max())))
        assert err <= 2e-5 * max(1.0, float(np.abs(ref).max())), (name, err)
    ez = maxabs(z.cpu().numpy()[:, :cfg.latent_size], g["z"][:, :cfg.latent_size])
    ey = maxabs(y.cpu().numpy(), g["y"])
    print(f"\n[cc] v3+noise cap 8 {precision}: {len(layers)} layers, worst rel {worst:.2e}; z {ez:.2e} y {ey:.2e}")
    assert ez < TOL and ey < TOL
    ts = torch.jit.script(m)
    with torch.no_grad():
        ys = ts.decode(torch.from_numpy(g["z"]).to(dev), u)
    assert maxabs(ys.cpu().numpy(), y.cpu().numpy()) == 0.0


@pytest.mark.parametrize("fixture,causal", [("v3_noise_causal_stream", True), ("v3_noise_stream", False)])
def test_cc_cached_v3_noise_tree_streams_reference(dev, golden, fixture, causal):
    """cc.use_cached_conv(True): the v3 + noise + AdaIN tree (capacity 16),
    scripted, streams 2048-sample blocks against the reference's cached_conv
    run block for block, AdaIN learning the target, then the source, then
    transferring (nn~'s learn flags switched between blocks), the reference's
    per-block uniform noise injected."""
    from rave_amd import config as rcfg
    cfg = rcfg.v3_noise(causal=causal, capacity=16)
    g = golden(fixture)
    m = torch.jit.script(_tree(cfg, g, golden, dev, cached=True))
    blk = int(g["block"])
    Fz = blk // cfg.hop
    x = torch.from_numpy(g["x"]).to(dev)
    z = torch.from_numpy(g["z"]).to(dev)
    u = torch.from_numpy(g["noise_u"]).to(dev)
    zs, ys = [], []
    with torch.no_grad():
        for i, (lx, ly) in enumerate(g["flags"]):
            _set_adain(m, lx, ly)
            zs.append(m.encode(x[..., i * blk:(i + 1) * blk]))
        _set_adain(m, 0, 0, reset=True)
        for i, (lx, ly) in enumerate(g["flags"]):
            _set_adain(m, lx, ly)
            ys.append(m.decode(z[..., i * Fz:(i + 1) * Fz], u[i]))
    ez = maxabs(torch.cat(zs, -1).cpu().numpy(), g["z_stream"])
    ey = maxabs(torch.cat(ys, -1).cpu().numpy(), g["y_stream"])
    print(f"\n[cc] cached v3+noise+AdaIN tree ({'causal' if causal else 'centred'}) vs reference: z {ez:.2e} y {ey:.2e}")
    assert ez < TOL and ey < TOL


def test_cc_adain_modes_match_reference_semantics(dev):
    """AdaptiveInstanceNormalization on rave_adain against the reference's eval
    forward restated in torch fp64 (rave/blocks.py:886-919): learn_y updates the
    y statistics and passes x through, learn_x updates the x statistics and
    then transfers (once both counters are set), batch rows [:bs] only."""
    from rave_amd.modules import AdaptiveInstanceNormalization
    C, T = 16, 300
    m = AdaptiveInstanceNormalization(C).to(dev).eval()
    r = {k: v.detach().cpu().double() for k, v in m.state_dict().items()}

    def ref_forward(x):
        bs = x.shape[0]
        if r["learn_y"].item():
            for k, v in (("mean_y", x.mean(-1, keepdim=True)), ("std_y", x.std(-1, keepdim=True))):
                r[k][:bs] += (v - r[k][:bs]) / (r["num_update_y"] + 1)
            r["num_update_y"] += 1
            return x
        if r["learn_x"].item():
            for k, v in (("mean_x", x.mean(-1, keepdim=True)), ("std_x", x.std(-1, keepdim=True))):
                r[k][:bs] += (v - r[k][:bs]) / (r["num_update_x"] + 1)
            r["num_update_x"] += 1
        if r["num_update_x"].item() and r["num_update_y"].item():
            x = (x - r["mean_x"][:bs]) / (r["std_x"][:bs] + 1e-5) * r["std_y"][:bs] + r["mean_y"][:bs]
        return x

    gen = torch.Generator().manual_seed(3)
    for step, (lx, ly, bs) in enumerate([(0, 1, 3), (0, 1, 3), (1, 0, 3), (1, 0, 2), (0, 0, 3)]):
        for t in (m, ):
            t.learn_x.fill_(lx)
            t.learn_y.fill_(ly)
        r["learn_x"].fill_(lx)
        r["learn_y"].fill_(ly)
        x = (torch.randn(bs, C, T, generator=gen) * (1 + step) + step).to(dev)
        with torch.no_grad():
            y = m(x)
        ref = ref_forward(x.cpu().double())
        assert maxabs(y.cpu().numpy(), ref.numpy()) < 1e-4, step
        for k in ("mean_x", "std_x", "mean_y", "std_y", "num_update_x", "num_update_y"):
            assert maxabs(getattr(m, k).cpu().numpy(), r[k].numpy()) < 1e-5, (step, k)
