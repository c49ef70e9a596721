"""Streaming (cached_conv mode) beyond the causal v2 case: centred (non-causal)
configs, discrete configs, stream construction details.  Runs on an MI355X
only (``-m gpu``).

Reference fixtures: tests/golden/make_golden.py runs the reference's own
modules under cc.use_cached_conv(True) (gen_streaming, gen_stream_v3,
gen_stream_discrete).  Tolerance: the north star's 1e-4 max-abs on model
outputs; RVQ indices exact outside the fp32 tie margin (top-2 gap < 1e-3)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

TOL = 1e-4
PRECISIONS = ["f32", "split16", "auto", "f32_tuned", "f32_bf3"]   # f32_tuned: exact fp32 incl. the ring kernels


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _model(cfg, g, dev, golden, precision="f32"):
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params
    return RAVE(cfg, init_params(cfg, seed=int(g["seed"])), g["speaker"], device=dev,
                hk=golden("pqmf")["hk"], precision=precision)


# ------------------------------------------------------------------ centred (non-causal) v2
@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_noncausal_streaming_golden(dev, golden, precision, graph):
    """The reference's default (centred) v2 model exported with --streaming
    (README.md:187-190): cached convs with (l + r)-column caches and Residual's
    AlignBranches delays (rave/blocks.py:32-46), block for block against the
    reference's cached mode."""
    from rave_amd import config as rcfg
    from rave_amd.streaming import StreamingRAVE
    cfg = rcfg.v2()
    g = golden("v2_stream")
    m = _model(cfg, g, dev, golden, precision)
    blk = int(g["block"])
    s = StreamingRAVE(m, batch=1, block=blk, graph=graph)
    x = torch.from_numpy(g["x"]).to(dev)
    z = torch.from_numpy(g["z"]).to(dev)
    nb = x.shape[-1] // blk
    Fz = blk // cfg.hop
    zs = torch.cat([s.encode(x[..., i * blk:(i + 1) * blk].contiguous()) for i in range(nb)], -1)
    ys = torch.cat([s.decode(z[..., i * Fz:(i + 1) * Fz].contiguous()) for i in range(nb)], -1)
    torch.cuda.synchronize()
    ez = maxabs(zs.cpu().numpy(), g["z_stream"])
    ey = maxabs(ys.cpu().numpy(), g["y_stream"])
    print(f"\n[parity] v2 centred streaming {precision} graph={graph}: z {ez:.3e}, y {ey:.3e}")
    assert ez < TOL and ey < TOL
    assert s.decode_delay == 8672


def test_noncausal_streaming_matches_oneshot_shifted(dev):
    """tests/test_residual.py:37-122's property on the HIP stack, at model
    scale: the streamed centred decoder equals one-shot decoding shifted by its
    cumulative delay (8672 samples: ConvTranspose r//2 caches, the dilated
    units' AlignBranches delays, the waveform and PQMF-inverse convs' right
    pads), once the left receptive field has filled."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2()
    m = RAVE(cfg, init_params(cfg, 3), init_speaker(cfg, 3), device=dev)
    B, blk, nb = 2, 2048, 40
    gen = torch.Generator().manual_seed(11)
    z = torch.randn(B, cfg.dec_in, nb * blk // cfg.hop, generator=gen).to(dev)
    s = StreamingRAVE(m, batch=B, block=blk, direction="decode")
    Fz = blk // cfg.hop
    ys = torch.cat([s.decode(z[..., i * Fz:(i + 1) * Fz].contiguous()) for i in range(nb)], -1)
    y1 = m.decode(z)
    torch.cuda.synchronize()
    d, warm = s.decode_delay, 12288
    assert d == 8672
    err = float((ys[..., d + warm:] - y1[..., warm:y1.shape[-1] - d]).abs().max())
    print(f"\n[parity] centred streamed decode vs one-shot shifted by {d}: {err:.3e}")
    assert err < TOL
    # the shift is exactly d: one sample either way breaks it
    assert float((ys[..., d + 1 + warm:] - y1[..., warm:y1.shape[-1] - d - 1]).abs().max()) > 1e-3


@pytest.mark.parametrize("precision", ["f32", "auto", "f32_bf3"])
def test_noncausal_v3_noise_adain_streaming_golden(dev, golden, precision):
    """Centred v3 + noise + AdaIN streamed against the reference's cached
    mode: the noise branch (padding (r, 0) convs, no AlignBranches) and the
    waveform conv (3-frame lag) are summed unaligned, as the reference does."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params
    g = golden("v3_noise_stream")
    cfg = rcfg.v3_noise(capacity=16)
    m = RAVE(cfg, init_params(cfg, int(g["seed"])), g["speaker"], device=dev, hk=golden("pqmf")["hk"],
             precision=precision)
    blk = int(g["block"])
    s = StreamingRAVE(m, batch=1, block=blk)
    x = torch.from_numpy(g["x"]).to(dev)
    z = torch.from_numpy(g["z"]).to(dev)
    u = torch.from_numpy(g["noise_u"]).to(dev)
    Fz = blk // cfg.hop
    zs, ys = [], []
    for i, (lx, ly) in enumerate(g["flags"]):
        m.adain.set_learn(learn_x=bool(lx), learn_y=bool(ly))
        zs.append(s.encode(x[..., i * blk:(i + 1) * blk].contiguous()))
    m.adain.reset_x()
    m.adain.reset_y()
    for i, (lx, ly) in enumerate(g["flags"]):
        m.adain.set_learn(learn_x=bool(lx), learn_y=bool(ly))
        ys.append(s.decode(z[..., i * Fz:(i + 1) * Fz].contiguous(), noise_u=u[i]))
    torch.cuda.synchronize()
    ez = maxabs(torch.cat(zs, -1).cpu().numpy(), g["z_stream"])
    ey = maxabs(torch.cat(ys, -1).cpu().numpy(), g["y_stream"])
    print(f"\n[parity] v3+noise+AdaIN centred streaming {precision}: z {ez:.3e}, y {ey:.3e}")
    assert ez < TOL and ey < TOL


# ------------------------------------------------------------------ discrete (RVQ) streaming
@pytest.mark.parametrize("precision", ["f32", "auto", "f32_bf3"])
def test_discrete_streaming_golden(dev, golden, precision):
    """DiscreteScriptedRAVE streamed (scripts/export.py:503-517 under
    cc.use_cached_conv(True)): per-block indices equal the reference's outside
    the tie margin; the reference's streamed indices decode to its audio."""
    from rave_amd import config as rcfg
    from rave_amd.streaming import StreamingRAVE
    cfg = rcfg.discrete()
    g = golden("discrete_stream")
    m = _model(cfg, g, dev, golden, precision)
    blk = int(g["block"])
    s = StreamingRAVE(m, batch=1, block=blk)
    x = torch.from_numpy(g["x"]).to(dev)
    nb = x.shape[-1] // blk
    Fz = blk // cfg.hop
    idx = torch.cat([s.encode_codes(x[..., i * blk:(i + 1) * blk].contiguous()) for i in range(nb)], -1)
    ref = torch.from_numpy(g["idx_stream"]).to(dev)
    ys = torch.cat([s.decode_codes(ref[..., i * Fz:(i + 1) * Fz].contiguous()) for i in range(nb)], -1)
    torch.cuda.synchronize()
    got = idx.cpu().numpy()
    mism = got != g["idx_stream"]
    gap = g["gap_stream"].transpose(1, 0, 2)          # (1, n_q, frames)
    assert (gap[mism] < 1e-3).all(), int(mism.sum())
    ey = maxabs(ys.cpu().numpy(), g["y_stream"])
    print(f"\n[parity] discrete streaming {precision}: index mismatches {int(mism.sum())} (tie margin), "
          f"y {ey:.3e}")
    assert ey < TOL
    with pytest.raises(ValueError):
        s.encode(x[..., :blk].contiguous())          # float latents are not this stream's output


def test_scripted_discrete_streaming_golden(dev, golden, tmp_path):
    """A scripted discrete model (DiscreteScriptedRAVE surface: float indices
    out of encode, clamp + truncation into decode), saved and loaded as nn~
    does, streams the reference's codes and audio."""
    from rave_amd import config as rcfg
    from rave_amd.scripted import ScriptedRAVE
    from rave_amd.weights import init_params
    cfg = rcfg.discrete()
    g = golden("discrete_stream")
    blk = int(g["block"])
    m = ScriptedRAVE(cfg, init_params(cfg, seed=int(g["seed"])), g["speaker"], hk=golden("pqmf")["hk"],
                     streaming=True, block=blk)
    path = str(tmp_path / "discrete_streaming.ts")
    m.export_to_ts(path)
    ts = torch.jit.load(path)
    assert ts.get_method_params("encode") == [1, 1, 16, 1024]
    x = torch.from_numpy(g["x"]).to(dev)
    codes = ts.encode(x)                               # whole buffer, split into blocks inside
    assert codes.dtype == torch.float32
    mism = codes.cpu().numpy().astype(np.int64) != g["idx_stream"]
    assert (g["gap_stream"].transpose(1, 0, 2)[mism] < 1e-3).all()
    y = ts.decode(torch.from_numpy(g["idx_stream"]).float().to(dev) + 0.25)   # truncation toward zero
    torch.cuda.synchronize()
    assert maxabs(y.cpu().numpy(), g["y_stream"]) < TOL


# ------------------------------------------------------------------ stream construction
def test_stream_warmup_leaves_adain_state(dev):
    """Creating a stream while AdaIN learns must not fold the warm-up block
    into the statistics: learning first and then streaming gives bitwise the
    statistics of streaming first and then learning."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3(causal=True, capacity=8)
    p, spk = init_params(cfg, 12), init_speaker(cfg, 12)
    gen = torch.Generator().manual_seed(12)
    xs = [(0.3 * torch.randn(1, 1, 2048, generator=gen)).to(dev) for _ in range(2)]
    states = []
    for learn_first in (True, False):
        m = RAVE(cfg, p, spk, device=dev)
        if learn_first:
            m.adain.set_learn(learn_x=True, learn_y=True)
            s = StreamingRAVE(m, batch=1, block=2048)
        else:
            s = StreamingRAVE(m, batch=1, block=2048)
            m.adain.set_learn(learn_x=True, learn_y=True)
        for x in xs:
            s.decode(s.encode(x))
        torch.cuda.synchronize()
        states.append(m.adain.state_dict())
    a, b = states
    assert a.keys() == b.keys()
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    name = next(k for k in a if k.endswith("num_update_y"))
    assert a[name][0] == 2                      # one update per streamed block


def test_stream_direction_flags_and_row0(dev):
    """ENCODE_ONLY / DECODE_ONLY streams refuse the other direction; a row0
    change after creation moves an existing stream's AdaIN rows."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3(causal=True, capacity=8)
    m = RAVE(cfg, init_params(cfg, 13), init_speaker(cfg, 13), device=dev)
    se = StreamingRAVE(m, batch=1, block=2048, direction="encode")
    sd = StreamingRAVE(m, batch=1, block=2048, direction="decode")
    x = (0.3 * torch.randn(1, 1, 2048, generator=torch.Generator().manual_seed(13))).to(dev)
    z = se.encode(x)
    y = sd.decode(z)
    with pytest.raises(RuntimeError):
        sd.encode(x)
    with pytest.raises(RuntimeError):
        se.decode(z)
    full = StreamingRAVE(m, batch=1, block=2048)
    torch.cuda.synchronize()
    assert torch.equal(full.decode(full.encode(x)), y)
    # rave_stream_launches (ABI 18): kernels per block; graph-captured kernel
    # nodes cover the plan's ops (an op can add a split-K reduce) except the
    # block's input copy, which a graph-mode call does itself straight into the
    # history buffer, and the encoder's speaker fill, run once per speaker
    # (round 6); a direction the stream lacks is refused
    eager = StreamingRAVE(m, batch=1, block=2048, graph=False)
    for w in ("encode", "decode"):
        assert full.launches(w) >= eager.launches(w) - (2 if w == "encode" else 1) >= 3
    assert se.launches("encode") == full.launches("encode")
    with pytest.raises(Exception):
        se.launches("decode")
    # row0: learn on row 3 through the existing stream
    m.adain_row0 = 3
    m.adain.set_learn(learn_y=True)
    se.encode(x)
    torch.cuda.synchronize()
    st = m.adain.state_dict()
    name = m.adain.modules[0][0]
    assert st[f"{name}.num_update_y"][0] == 1
    assert np.allclose(st[f"{name}.mean_y"][0], 0) and not np.allclose(st[f"{name}.mean_y"][3], 0)


def test_noise_frames_must_divide(dev):
    """NoiseGeneratorV2 reshapes per noise frame (rave/blocks.py:283-285): a
    decode whose band frames do not divide by prod(noise ratios) is refused
    instead of leaving workspace garbage in the noise tail."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3_noise(capacity=8, ratios=(2, 2, 2, 2), dilations=((1,), (1,), (1,), (1,)))
    # hop = 16 * 16 = 256; one latent frame = 16 band frames, prod(noise ratios) = 8: fine;
    cfg_bad = rcfg.v3_noise(capacity=8, ratios=(2, 2), dilations=((1,), (1,)))
    for c, ok in ((cfg, True), (cfg_bad, False)):
        m = RAVE(c, init_params(c, 1), init_speaker(c, 1), device=dev)
        z = torch.zeros(1, c.dec_in, 1, device=dev)
        if ok:
            m.decode(z)
        else:                            # 1 frame * 64 / 16 = 4 band frames, not a multiple of 8
            with pytest.raises(ValueError):
                m.decode(z)


def test_stream_graph_speaker_change(dev):
    """A graph-mode stream fills the latents' speaker channels outside its graph,
    once per speaker (round 6): a speaker change between blocks reaches the
    next block's latents and output exactly as in an eager stream."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.causal(capacity=8)
    p = init_params(cfg, 21)
    spk = [init_speaker(cfg, 21), init_speaker(cfg, 22)]
    gen = torch.Generator().manual_seed(21)
    xs = [(0.3 * torch.randn(1, 1, 2048, generator=gen)).to(dev) for _ in range(4)]
    outs = []
    for graph in (True, False):
        m = RAVE(cfg, p, spk[0], device=dev)
        s = StreamingRAVE(m, batch=1, block=2048, graph=graph)
        zs, ys = [], []
        for i, x in enumerate(xs):
            if i == 2:
                m.set_speaker(spk[1])
            z = s.encode(x)
            zs.append(z.clone())
            ys.append(s.decode(z).clone())
        torch.cuda.synchronize()
        outs.append((zs, ys))
    (zg, yg), (ze, ye) = outs
    lat = cfg.latent_size
    for i in range(4):
        assert torch.equal(zg[i], ze[i]), i
        assert torch.equal(yg[i], ye[i]), i
    # the speaker channels follow the change
    assert not torch.equal(zg[1][:, lat:], zg[2][:, lat:])
    assert torch.equal(zg[2][:, lat:], zg[3][:, lat:])
