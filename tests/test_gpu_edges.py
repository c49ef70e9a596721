"""The fused path edges (csrc/edge_split.hip) against the float64 oracle and
against the separate ops they replace.

* rave_encoder_head = CachedPQMF.forward + band slice (rave/pqmf.py:269-273,
  rave/model.py:613) -> EncoderV2's first conv (rave/blocks.py:533-536), + the
  speaker concat (rave/model.py:618-620);
* rave_decoder_tail = GeneratorV2's act -> conv -> `x*sigmoid(a) (+noise) ->
  tanh` (rave/blocks.py:691-707) -> CachedPQMF.inverse (rave/pqmf.py:275-284).

Tolerances: layer outputs 2e-5 relative to max|ref| (as the single-layer tests);
model outputs 1e-4 max-abs (north star).  Ragged lengths (frames not a
multiple of the 256-frame tiles) and both padding modes are covered, in both
arithmetics: split-f16 and exact fp32 (precision RAVE_PREC_F32_RING: the
ring weight image and the fp32 filter image)."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def N():
    from rave_amd import _native
    return _native


def _st():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _filters(golden):
    from oracle.rave_oracle import pqmf_filters
    hk = golden("pqmf")["hk"]
    return pqmf_filters(hk)


HEAD_CASES = [(600, 2, 1.0, 6), (4096, 3, 1.0, 6), (257, 1, 3e6, 6),
              (600, 2, 1.0, 5), (600, 1, 1.0, 8)]     # odd / full band counts: the fp32 conv's channel pairs


@pytest.mark.parametrize("prec", ["split16", "f32_ring", "bf16x3"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("F,B,scale,nb", HEAD_CASES)
def test_encoder_head(N, dev, golden, causal, F, B, scale, nb, prec):
    """bf16x3 (round 6): the analysis on the bf16 matrix cores (filter and audio
    split exactly into three bf16 parts), the conv in exact fp32 on the ring
    image; held to the fp32-class bound as the bf16x3 tail."""
    from oracle.rave_oracle import conv1d, get_padding, reverse_half
    hkf, _ = _filters(golden)
    rng = np.random.default_rng(F + 7 * causal + nb)
    T = 16 * F
    x = (scale * (0.3 * np.sin(np.arange(T) * 0.05)[None, None] + 0.1 * rng.standard_normal((B, 1, T)))).astype(np.float32)
    co, k = 64, 7
    w = (rng.uniform(-1, 1, (co, nb, k)) / np.sqrt(nb * k)).astype(np.float32)
    b = (0.1 * rng.standard_normal(co)).astype(np.float32)
    bands = reverse_half(conv1d(x.astype(np.float64), hkf.astype(np.float64), None, stride=16,
                                pad=get_padding(hkf.shape[-1], causal=causal)))[:, :nb]
    cpad = get_padding(k, causal=causal)
    ref = conv1d(bands, w.astype(np.float64), b.astype(np.float64), pad=cpad)
    P = N.PRECISION[prec]
    wprec = N.PREC_F32_RING if P == N.PREC_BF16X3 else P      # the bf16x3 head's conv: exact fp32, ring image
    packed = torch.from_numpy(N.pack_conv_weight(w, nb, co, k, 1, 1, 0, precision=wprec)).to(dev)
    xd = torch.from_numpy(x).to(dev)
    y = torch.full((B, co, F), float("nan"), device=dev)
    spk = torch.from_numpy(rng.standard_normal(256).astype(np.float32)).to(dev)
    Fz = max(1, F // 64)
    z = torch.full((B, 320, Fz), float("nan"), device=dev)
    hd = torch.from_numpy(N.pack_edge_filter(hkf, head=True, n_out_bands=nb,
                                             f32=P in (N.PREC_F32_RING, N.PREC_BF16X3))).to(dev)
    bd = torch.from_numpy(b).to(dev)
    a = N.EdgeArgs(batch=B, frames=F, conv_c_in=nb, conv_c_out=co, conv_kernel=k, conv_pad_left=cpad[0],
                   pqmf_taps=hkf.shape[-1], pqmf_pad_left=get_padding(hkf.shape[-1], causal=causal)[0],
                   x=xd.data_ptr(), x_sb=T, y=y.data_ptr(), y_sb=co * F, y_sc=F,
                   weight=packed.data_ptr(), bias=bd.data_ptr(), filter=hd.data_ptr(),
                   fill_channels=256, fill_t=Fz, fill_y=z[:, 64:].data_ptr(), f_sb=320 * Fz, f_sc=Fz,
                   fill_values=spk.data_ptr(), precision=P)
    N.check(N.lib.rave_encoder_head(C.byref(a), _st()), "encoder_head")
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    assert np.isfinite(got).all()
    err = maxabs(got, ref)
    assert err <= 2e-5 * float(np.abs(ref).max()), err
    if prec == "bf16x3":                   # fp32-class arithmetic
        assert err <= 2e-6 * max(1.0, float(np.abs(ref).max())), err
    zz = z.cpu().numpy()
    assert np.array_equal(zz[:, 64:], np.broadcast_to(spk.cpu().numpy()[None, :, None], (B, 256, Fz)))
    assert np.isnan(zz[:, :64]).all()            # the latent rows are the encoder's, untouched


@pytest.mark.parametrize("prec", ["split16", "f32_ring", "bf16x3"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("am,act,noise", [(True, "leaky", False), (False, "snake", True), (True, "snake", True)])
@pytest.mark.parametrize("F,B", [(600, 2), (4096, 2), (100, 1)])
def test_decoder_tail(N, dev, golden, causal, am, act, noise, F, B, prec):
    from oracle.rave_oracle import conv1d, get_padding, leaky_relu, reverse_half, snake
    _, hki = _filters(golden)
    rng = np.random.default_rng(F + 3 * am + 5 * causal)
    ci, k = 64, 7
    co = 32 if am else 16
    x = rng.standard_normal((B, ci, F)).astype(np.float32)
    w = (rng.uniform(-1, 1, (co, ci, k)) / np.sqrt(ci * k)).astype(np.float32)
    b = (0.1 * rng.standard_normal(co)).astype(np.float32)
    alpha = (1 + 0.1 * rng.standard_normal(ci)).astype(np.float32)
    nz = (0.05 * rng.standard_normal((B, 16, F))).astype(np.float32) if noise else None
    xa = leaky_relu(x.astype(np.float64)) if act == "leaky" else snake(x.astype(np.float64), alpha.reshape(-1, 1))
    cpad = get_padding(k, causal=causal)
    wv = conv1d(xa, w.astype(np.float64), b.astype(np.float64), pad=cpad)
    if am:
        v, amp = np.split(wv, 2, axis=1)
        wv = v * (1.0 / (1.0 + np.exp(-amp)))
    wv = np.tanh(wv + (nz if noise else 0.0))
    spad = get_padding(hki.shape[-1], causal=causal)
    ys = conv1d(reverse_half(wv), hki.astype(np.float64), None, pad=spad) * 16
    ref = ys[:, ::-1, :].transpose(0, 2, 1).reshape(B, 1, F * 16)
    P = N.PRECISION[prec]
    packed = torch.from_numpy(N.pack_conv_weight(w, ci, co, k, 1, 1, 0, precision=P)).to(dev)
    xd = torch.from_numpy(x).to(dev)
    y = torch.full((B, 1, 16 * F), float("nan"), device=dev)
    bd, ad = (torch.from_numpy(v).to(dev) for v in (b, alpha))
    # (bf16x3: the conv on the bf16 matrix cores, the synthesis on the exact-fp32 filter image)
    hd = torch.from_numpy(N.pack_edge_filter(hki, head=False, f32=P in (N.PREC_F32_RING, N.PREC_BF16X3))).to(dev)
    nd = torch.from_numpy(nz).to(dev) if noise else None
    a = N.EdgeArgs(batch=B, frames=F, conv_c_in=ci, conv_c_out=co, conv_kernel=k, conv_pad_left=cpad[0],
                   pqmf_taps=hki.shape[-1], pqmf_pad_left=spad[0], mode=1 if am else 2, act=N.ACT[act],
                   leaky_slope=0.2, x=xd.data_ptr(), x_sb=ci * F, x_sc=F, y=y.data_ptr(), y_sb=16 * F,
                   weight=packed.data_ptr(), bias=bd.data_ptr(), alpha=ad.data_ptr(), filter=hd.data_ptr(),
                   noise=nd.data_ptr() if noise else None, n_sb=16 * F, n_sc=F, precision=P)
    N.check(N.lib.rave_decoder_tail(C.byref(a), _st()), "decoder_tail")
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    assert np.isfinite(got).all()
    err = maxabs(got, ref)
    assert err <= 2e-5 * max(1.0, float(np.abs(ref).max())), err
    if prec != "split16":                  # fp32-class arithmetics
        assert err <= 2e-6 * max(1.0, float(np.abs(ref).max())), err


def test_edges_refuse_unsupported(N):
    a = N.EdgeArgs(batch=1, frames=64, conv_c_in=96, conv_c_out=32, conv_kernel=7, pqmf_taps=33, mode=1,
                   act=N.ACT["leaky"], x=16, y=16, weight=16, filter=16)
    assert N.lib.rave_decoder_tail(C.byref(a), None) == N.RAVE_ERR_UNSUPPORTED     # capacity 96 (discrete)
    a = N.EdgeArgs(batch=1, frames=64, conv_c_in=16, conv_c_out=64, conv_kernel=7, pqmf_taps=513, x=16, y=16,
                   weight=16, filter=16)
    assert N.lib.rave_encoder_head(C.byref(a), None) == N.RAVE_ERR_UNSUPPORTED     # > 8 bands


@pytest.mark.parametrize("cfg_name,precision", [("v2", "split16"), ("v3_noise", "split16"), ("v2", "f32_tuned"),
                                                ("v3_noise", "f32_tuned"), ("v2", "f32_bf3"),
                                                ("v3_noise", "f32_bf3")])
def test_model_uses_edges_and_matches_oracle(dev, golden, cfg_name, precision):
    """A split16 model lays both fused edges into its plans (an exact-fp32
    f32_tuned model: where they time faster than the separate ops), and its
    forward matches the float64 oracle (the model golden tests cover auto /
    split16 against the reference fixtures)."""
    from oracle.rave_oracle import Oracle
    from rave_amd import _native as N
    from rave_amd import config as rcfg
    from rave_amd.model import DECODE, ENCODE, RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.get_config(cfg_name)
    params = init_params(cfg, seed=3)
    spk = init_speaker(cfg, seed=3)
    m = RAVE(cfg, params, spk, device=dev, hk=golden("pqmf")["hk"], precision=precision)
    B, T = 2, 16384
    Fz = T // cfg.hop
    kinds_e = [o["kind"] for o in m.ops(ENCODE, B, T)]
    kinds_d = [o["kind"] for o in m.ops(DECODE, B, Fz)]
    if precision == "split16":
        assert N.OP_HEAD in kinds_e and N.OP_PQMF_ANALYSIS not in kinds_e and N.OP_FILL not in kinds_e
        assert N.OP_TAIL in kinds_d and N.OP_PQMF_SYNTHESIS not in kinds_d
    else:
        assert (N.OP_HEAD in kinds_e) != (N.OP_PQMF_ANALYSIS in kinds_e)
        assert (N.OP_TAIL in kinds_d) != (N.OP_PQMF_SYNTHESIS in kinds_d)
    rng = np.random.default_rng(4)
    x = (0.3 * np.sin(np.arange(T) * 2 * np.pi * 440 / 48000)[None, None]
         + 0.1 * rng.standard_normal((B, 1, T))).astype(np.float32)
    o = Oracle(cfg, params, spk, hk=golden("pqmf")["hk"])
    z = m.encode(torch.from_numpy(x).to(dev))
    assert maxabs(z.cpu().numpy(), o.encode(x.astype(np.float64))) <= 1e-4
    noise_u = None
    if cfg.noise is not None:
        noise_u = torch.from_numpy(rng.uniform(0, 1, m.noise_shape(B, Fz)).astype(np.float32)).to(dev)
    y = m.decode(z, noise_u=noise_u)
    ref = o.decode(z.cpu().numpy().astype(np.float64),
                   noise_u=noise_u.cpu().numpy().astype(np.float64) if noise_u is not None else None)
    assert maxabs(y.cpu().numpy(), ref) <= 1e-4
