"""SpeakerRAVE and the Resampler on the HIP path, against the reference's own
outputs (tests/golden/speaker.npz, resampler.npz) and the float64 oracle.

Tolerances: the embedding and resampled audio within 1e-5 max-abs of the
reference fp32 CPU output (|emb| ~ 0.2, audio ~ N(0,1)); kernels against the
float64 oracle within 1e-5 relative to max|ref|."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("mode", ["centered", "causal"])
def test_speaker_embedding_golden(dev, golden, mode):
    import torch
    from rave_amd.speaker import SpeakerRAVE, init_params
    g = golden("speaker")
    m = SpeakerRAVE(init_params(int(g["seed"])), device=dev, causal=mode == "causal")
    emb = m.forward(torch.from_numpy(g[f"{mode}/bands"]).to(dev))
    torch.cuda.synchronize()
    assert tuple(emb.shape) == (2, 256)
    assert maxabs(emb.cpu().numpy(), g[f"{mode}/emb"]) < 1e-5
    # from audio: PQMF analysis (all 16 bands) on the GPU, then the encoder
    emb2 = m.embed(torch.from_numpy(g[f"{mode}/x"]).to(dev))
    assert maxabs(emb2.cpu().numpy(), g[f"{mode}/emb"]) < 1e-5
    # repeatable
    emb3 = m.forward(torch.from_numpy(g[f"{mode}/bands"]).to(dev))
    assert torch.equal(emb, emb3)


def test_speaker_longer_clip_vs_oracle(dev):
    """The nn~ embedding length (131072 samples -> 8192 frames, scripts/export.py:79-90)."""
    import torch
    from oracle.speaker_oracle import speaker_forward
    from rave_amd.speaker import SpeakerRAVE, init_params
    p = init_params(5)
    rng = np.random.default_rng(8)
    bands = (0.3 * rng.standard_normal((1, 16, 8192))).astype(np.float32)
    m = SpeakerRAVE(p, device=dev)
    emb = m.forward(torch.from_numpy(bands).to(dev)).cpu().numpy()
    ref = speaker_forward(p, bands)
    assert maxabs(emb, ref) < 1e-5


def test_speaker_rejects_bad_shapes(dev):
    import torch
    from rave_amd.speaker import SpeakerRAVE, init_params
    m = SpeakerRAVE(init_params(0), device=dev)
    with pytest.raises(ValueError):
        m.forward(torch.zeros(1, 8, 256, device=dev))
    with pytest.raises(ValueError):
        m.forward(torch.zeros(1, 16, 100, device=dev))


@pytest.mark.parametrize("ratio,mode", [(2, "centered"), (3, "centered"), (2, "causal")])
def test_resampler_golden(dev, golden, ratio, mode):
    import torch
    from rave_amd.resampler import Resampler
    g = golden("resampler")
    key = f"r{ratio}_{mode}"
    r = Resampler(48000 * ratio, 48000, device=dev, causal=mode == "causal")
    x = torch.from_numpy(g["x"]).to(dev)
    down = r.to_model_sampling_rate(x).cpu().numpy()
    up = r.from_model_sampling_rate(x).cpu().numpy()
    assert down.shape == g[f"{key}/down"].shape and up.shape == g[f"{key}/up"].shape
    assert maxabs(down, g[f"{key}/down"]) < 1e-5
    assert maxabs(up, g[f"{key}/up"]) < 1e-5


@pytest.mark.parametrize("mode", ["centered", "causal"])
def test_resampler_streaming_golden(dev, golden, mode):
    import torch
    from rave_amd.resampler import Resampler
    g = golden("resampler")
    xs = torch.from_numpy(g["stream/x"]).to(dev)
    r = Resampler(96000, 48000, device=dev, causal=mode == "causal", streaming=True)
    n = xs.shape[-1] // 2048
    down = torch.cat([r.to_model_sampling_rate(xs[..., i * 2048:(i + 1) * 2048]) for i in range(n)], -1)
    up = torch.cat([r.from_model_sampling_rate(xs[..., i * 2048:(i + 1) * 2048]) for i in range(n)], -1)
    assert maxabs(down.cpu().numpy(), g[f"stream/r2_{mode}/down"]) < 1e-5
    assert maxabs(up.cpu().numpy(), g[f"stream/r2_{mode}/up"]) < 1e-5
    r.reset()                                   # fresh caches reproduce the first block
    d0 = r.to_model_sampling_rate(xs[..., :2048])
    assert torch.equal(d0, down[..., :1024])
    with pytest.raises(ValueError):
        Resampler(144000, 48000, device=dev, streaming=True)     # odd ratio (rave/resampler.py:21-25)


@pytest.mark.parametrize("B,T,P,K,S,pad", [(3, 1000, 1, 39, 2, 19), (2, 777, 3, 21, 1, 10),
                                           (1, 5000, 1, 57, 3, 56), (2, 64, 2, 7, 1, 6)])
def test_fir_kernel_vs_numpy(dev, B, T, P, K, S, pad):
    """Ragged lengths, several phases/strides, windows past both ends."""
    import torch
    from rave_amd import _native as N
    rng = np.random.default_rng(B * T + K)
    x = rng.standard_normal((B, T)).astype(np.float32)
    h = rng.standard_normal((P, K)).astype(np.float32)
    t_out = (T + pad - K) // S + 1 + 3                     # a few frames past the right end too
    xp = np.pad(x.astype(np.float64), ((0, 0), (pad, t_out * S + K)))
    ref = np.zeros((B, t_out, P))
    for t in range(t_out):
        ref[:, t, :] = xp[:, t * S:t * S + K] @ h.astype(np.float64).T
    xd, hd = torch.from_numpy(x).to(dev), torch.from_numpy(h).to(dev)
    y = torch.full((B, t_out * P), float("nan"), device=dev)
    a = N.FirArgs(batch=B, t_in=T, t_out=t_out, phases=P, taps=K, stride=S, pad_left=pad,
                  x=xd.data_ptr(), x_sb=T, y=y.data_ptr(), y_sb=t_out * P, h=hd.data_ptr())
    N.check(N.lib.rave_fir(C.byref(a), C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    out = y.cpu().numpy().reshape(B, t_out, P)
    assert maxabs(out, ref) / np.abs(ref).max() < 1e-5


def test_pooling_kernels_vs_numpy(dev):
    import torch
    from rave_amd import _native as N
    rng = np.random.default_rng(2)
    B, Ch, T = 3, 40, 333
    x = rng.standard_normal((B, Ch, T)).astype(np.float32)
    lg = (3 * rng.standard_normal((B, Ch, T))).astype(np.float32)
    a = np.where(x > 0, x, 0.2 * x).astype(np.float64)
    st = torch.cuda.current_stream().cuda_stream
    xd, ld = torch.from_numpy(x).to(dev), torch.from_numpy(lg).to(dev)
    y = torch.zeros(B, 2 * Ch, device=dev)
    rs = N.RowStatsArgs(batch=B, channels=Ch, t_len=T, act=N.ACT["leaky"], leaky_slope=0.2, var_min=1e-4,
                        var_max=1e4, x=xd.data_ptr(), x_sb=Ch * T, x_sc=T, y=y.data_ptr(), y_sb=2 * Ch)
    N.check(N.lib.rave_row_stats(C.byref(rs), C.c_void_p(st)))
    ref = np.concatenate([a.mean(-1), np.sqrt(np.clip(a.var(-1, ddof=1), 1e-4, 1e4))], 1)
    assert maxabs(y.cpu().numpy(), ref) < 1e-5
    w = np.exp(lg - lg.max(-1, keepdims=True))
    w /= w.sum(-1, keepdims=True)
    mu = (a * w).sum(-1)
    ref = np.concatenate([mu, np.sqrt(np.clip((a * a * w).sum(-1) - mu ** 2, 1e-4, 1e4))], 1)
    ap = N.AttnPoolArgs(batch=B, channels=Ch, t_len=T, act=N.ACT["leaky"], leaky_slope=0.2, var_min=1e-4,
                        var_max=1e4, x=xd.data_ptr(), x_sb=Ch * T, x_sc=T, logits=ld.data_ptr(), l_sb=Ch * T,
                        l_sc=T, y=y.data_ptr(), y_sb=2 * Ch)
    N.check(N.lib.rave_attn_pool(C.byref(ap), C.c_void_p(st)))
    assert maxabs(y.cpu().numpy(), ref) < 1e-5
    # linear and max-pool
    W = rng.standard_normal((37, 2 * Ch)).astype(np.float32)
    bias = rng.standard_normal(37).astype(np.float32)
    Wd, bd = torch.from_numpy(W).to(dev), torch.from_numpy(bias).to(dev)
    out = torch.zeros(B, 37, device=dev)
    ln = N.LinearArgs(batch=B, n_in=2 * Ch, n_out=37, x=y.data_ptr(), x_sb=2 * Ch, w=Wd.data_ptr(),
                      bias=bd.data_ptr(), y=out.data_ptr(), y_sb=37)
    N.check(N.lib.rave_linear(C.byref(ln), C.c_void_p(st)))
    assert maxabs(out.cpu().numpy(), y.cpu().numpy().astype(np.float64) @ W.T + bias) < 1e-4
    mp = torch.zeros(B, Ch, T // 2, device=dev)
    m = N.MaxPoolArgs(batch=B, channels=Ch, t_out=T // 2, kernel=2, x=xd.data_ptr(), x_sb=Ch * T, x_sc=T,
                      y=mp.data_ptr(), y_sb=Ch * (T // 2), y_sc=T // 2)
    N.check(N.lib.rave_maxpool(C.byref(m), C.c_void_p(st)))
    assert np.array_equal(mp.cpu().numpy(), x[..., :T // 2 * 2].reshape(B, Ch, T // 2, 2).max(-1))


def test_model_set_speaker_and_nntilde_selection(dev, golden):
    """RAVE.set_speaker swaps the embedding encode concatenates; the nn~
    ``speaker`` attribute picks speaker1..N or speaker5 (scripts/export.py:384-396)."""
    import torch
    from rave_amd import config as rcfg
    from rave_amd.export import NNTildeRAVE
    from rave_amd.model import RAVE
    from rave_amd.speaker import SpeakerRAVE, init_params as sp_params
    from rave_amd.weights import init_params, init_speaker
    g = golden("speaker")
    embs = SpeakerRAVE(sp_params(0), device=dev).embed(torch.from_numpy(g["centered/x"]).to(dev))
    cfg = rcfg.v2(capacity=8)
    m = RAVE(cfg, init_params(cfg, 2), init_speaker(cfg, 2), device=dev)
    x = (0.1 * torch.randn(1, 1, 4096, generator=torch.Generator().manual_seed(1))).to(dev)
    z0 = m.encode(x)
    m.set_speaker(embs[1])
    z1 = m.encode(x)
    assert torch.equal(z0[:, :cfg.latent_size], z1[:, :cfg.latent_size])
    assert torch.equal(z1[0, cfg.latent_size:, 0], embs[1])
    w = NNTildeRAVE(m, speakers=[embs[0], embs[1]])
    w.set_speaker(0)
    assert torch.equal(w.encode(x)[0, cfg.latent_size:, 1], embs[0])
    w.set_speaker(5)                                          # beyond the list: speaker5 (ones)
    assert torch.equal(w.encode(x)[0, cfg.latent_size:, 2], torch.ones(256, device=dev))


def test_scripted_speakers_and_resampler(dev, golden, tmp_path):
    """The .ts carries its speaker embeddings and the Resampler (torch.ops.rave_amd.fir):
    encode at 96 kHz == model.encode(to_model_sampling_rate(x)); decode ==
    from_model_sampling_rate(model.decode(z)); the speaker attribute selects."""
    import torch
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.resampler import Resampler
    from rave_amd.scripted import ScriptedRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2(capacity=8)
    p, spk = init_params(cfg, 3), init_speaker(cfg, 3)
    rng = np.random.default_rng(0)
    e = [rng.standard_normal(256).astype(np.float32) for _ in range(2)]
    m = ScriptedRAVE(cfg, p, spk, speakers=e, target_sr=96000)
    path = str(tmp_path / "rs.ts")
    m.export_to_ts(path)
    ts = torch.jit.load(path)
    assert ts.get_method_params("encode") == [1, 1, 320, 2048]
    ref = RAVE(cfg, p, spk, device=dev)
    rs = Resampler(96000, 48000, device=dev)
    x = (0.1 * torch.randn(2, 1, 8192, generator=torch.Generator().manual_seed(2))).to(dev)
    ts.set_speaker(1)
    z = ts.encode(x)
    ref.set_speaker(e[1])
    z_ref = ref.encode(rs.to_model_sampling_rate(x))
    assert torch.equal(z, z_ref)
    y = ts.decode(z)
    assert torch.equal(y, rs.from_model_sampling_rate(ref.decode(z_ref)))
    assert y.shape == x.shape


def test_scripted_streaming_resampler_matches_python(dev):
    """Causal streaming with a 96 kHz host: the scripted module's cached FIRs
    equal rave_amd.Resampler(streaming=True) around StreamingRAVE."""
    import torch
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.resampler import Resampler
    from rave_amd.scripted import ScriptedRAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.causal(capacity=8)
    p, spk = init_params(cfg, 4), init_speaker(cfg, 4)
    ts = torch.jit.script(ScriptedRAVE(cfg, p, spk, block=2048, target_sr=96000))
    st = StreamingRAVE(RAVE(cfg, p, spk, device=dev), batch=1, block=2048)
    rs = Resampler(96000, 48000, device=dev, causal=True, streaming=True)
    x = (0.2 * torch.randn(1, 1, 3 * 4096, generator=torch.Generator().manual_seed(5))).to(dev)
    for i in range(3):
        xi = x[..., i * 4096:(i + 1) * 4096]
        y = ts.forward(xi)
        y_ref = rs.from_model_sampling_rate(st.forward(rs.to_model_sampling_rate(xi)))
        assert float((y - y_ref).abs().max()) < 1e-6
