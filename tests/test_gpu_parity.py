"""HIP path vs the CPU oracle (and the reference's golden fixtures), through
the C-ABI.  Runs on an MI355X only (``-m gpu``).

Tolerances: the north star is <= 1e-4 max-abs vs the reference fp32 CPU path
on model outputs; single layers are checked at 2e-5 relative to max|ref|
(fp32 accumulation over K <= 3072 against a float64 oracle)."""
import ctypes as C
import ctypes as C_
import os

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


@pytest.fixture(scope="module")
def N():
    from rave_amd import _native
    return _native


def _golden_hk(golden):
    return golden("pqmf")["hk"]


# ------------------------------------------------------------------ single conv
CONV_CASES = [
    # c_in, c_out, k, s, d, transposed, act, residual, B, T
    (64, 64, 3, 1, 1, 0, "leaky", False, 2, 300),
    (64, 64, 3, 1, 9, 0, "leaky", False, 3, 1000),
    (128, 128, 1, 1, 1, 0, "leaky", True, 2, 257),
    (6, 64, 7, 1, 1, 0, "none", False, 2, 512),
    (64, 128, 8, 4, 1, 0, "leaky", False, 2, 1024),
    (256, 512, 4, 2, 1, 0, "snake", False, 2, 64),
    (1024, 64, 3, 1, 1, 0, "leaky", False, 4, 16),
    (320, 1024, 3, 1, 1, 0, "none", False, 2, 8),
    (1024, 512, 4, 2, 1, 1, "leaky", False, 2, 8),
    (128, 64, 8, 4, 1, 1, "snake", False, 2, 100),
    (64, 32, 7, 1, 1, 0, "snake", False, 2, 4096),
    (96, 96, 3, 1, 3, 0, "snake", True, 2, 700),
    (512, 512, 3, 1, 3, 0, "leaky", False, 16, 128),
    # small-capacity shapes (capacity 8 models)
    (8, 8, 3, 1, 1, 0, "leaky", False, 2, 300),
    (8, 8, 1, 1, 1, 0, "snake", True, 2, 300),
    (6, 8, 7, 1, 1, 0, "none", False, 1, 256),
    (8, 16, 8, 4, 1, 0, "leaky", False, 2, 256),
    (16, 32, 4, 2, 1, 0, "leaky", False, 2, 64),
    (32, 16, 4, 2, 1, 1, "leaky", False, 2, 16),
    (16, 8, 8, 4, 1, 1, "snake", False, 2, 32),
    (8, 16, 7, 1, 1, 0, "leaky", False, 2, 256),
    (8, 32, 7, 1, 1, 0, "snake", False, 2, 256),
    (8, 16, 4, 2, 1, 0, "snake", False, 2, 256),
    (64, 8, 3, 1, 1, 0, "leaky", False, 2, 8),
    (40, 64, 3, 1, 1, 0, "none", False, 2, 8),
    # v2's short-N layers at bench size (wide-chunk K-group tiles)
    (512, 512, 1, 1, 1, 0, "leaky", True, 16, 128),
    (1024, 128, 3, 1, 1, 0, "leaky", False, 16, 64),
]


def run_conv(N, dev, x, w, b, alpha, res, c_in, c_out, k, s, d, pad, transposed, act, split=True,
             precision=0, config=0):
    B, _, T = x.shape
    packed = torch.from_numpy(N.pack_conv_weight(w, c_in, c_out, k, s, d, transposed,
                                                 precision=precision)).to(dev)
    xd = torch.from_numpy(x).to(dev)
    if transposed:
        t_out = T * s
    else:
        t_out = (T + pad[0] + pad[1] - ((k - 1) * d + 1)) // s + 1
    y = torch.full((B, c_out, t_out), float("nan"), device=dev)
    bd = torch.from_numpy(b).to(dev) if b is not None else None
    ad = torch.from_numpy(alpha).to(dev) if alpha is not None else None
    rd = torch.from_numpy(res).to(dev) if res is not None else None
    a = N.ConvArgs(c_in=c_in, c_out=c_out, kernel=k, stride=s, dilation=d,
                   pad_left=0 if transposed else pad[0], pad_right=0 if transposed else pad[1],
                   transposed=transposed, out_shift=s // 2 if transposed else 0, act=N.ACT[act],
                   leaky_slope=0.2, batch=B, t_in=T, t_out=t_out, precision=precision,
                   x=xd.data_ptr(), x_sb=c_in * T, x_sc=T, y=y.data_ptr(), y_sb=c_out * t_out, y_sc=t_out,
                   residual=rd.data_ptr() if rd is not None else None, r_sb=c_out * t_out, r_sc=t_out,
                   weight=packed.data_ptr(), bias=bd.data_ptr() if bd is not None else None,
                   alpha=ad.data_ptr() if ad is not None else None, config=config)
    ws = None
    if split:
        nws = N.lib.rave_conv1d_workspace(C.byref(a))
        assert nws >= 0
        if nws > 0:
            ws = torch.full((nws,), float("nan"), device=dev)   # slabs need no initialisation,
            ws[:N.SPLITK_TICKETS] = 0                              # the arrival counters start zero
            a.partial = ws.data_ptr()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib.rave_conv1d(C.byref(a), st), "conv1d")
    torch.cuda.synchronize()
    out = y.cpu().numpy()
    if ws is not None:
        # the call left the counters zero, and a second call gives bitwise the same output
        assert int((ws[:N.SPLITK_TICKETS].view(torch.int32) != 0).sum()) == 0
        y.fill_(float("nan"))
        N.check(N.lib.rave_conv1d(C.byref(a), st), "conv1d")
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy(), out)
    return out


def conv_case(case):
    """Seeded inputs of a CONV_CASES row and the oracle's output (float64)."""
    from oracle.rave_oracle import conv1d, conv_transpose1d, leaky_relu, snake
    c_in, c_out, k, s, d, transposed, act, has_res, B, T = case
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    x = rng.standard_normal((B, c_in, T)).astype(np.float32)
    bound = 1 / np.sqrt(c_in * k)
    if transposed:
        w = rng.uniform(-bound, bound, (c_in, c_out, k)).astype(np.float32)
    else:
        w = rng.uniform(-bound, bound, (c_out, c_in, k)).astype(np.float32)
    b = rng.uniform(-bound, bound, c_out).astype(np.float32)
    alpha = (1 + 0.1 * rng.standard_normal((c_in, 1))).astype(np.float32) if act == "snake" else None
    xa = x.astype(np.float64)
    if act == "leaky":
        xa = leaky_relu(xa)
    elif act == "snake":
        xa = snake(xa, alpha)
    if transposed:
        ref = conv_transpose1d(xa, w, s, s // 2, b)
        pad = (0, 0)
    else:
        p = (k - 1) * d + 1
        pad = ((p - 1) // 2, p // 2)
        ref = conv1d(xa, w, b, s, d, pad)
    res = rng.standard_normal(ref.shape).astype(np.float32) if has_res else None
    if has_res:
        ref = ref + res
    return x, w, b, alpha.reshape(-1) if alpha is not None else None, res, pad, ref


def _ring_skip(precision, T):
    if precision in ("f32_ring", "bf16x3") and T % 4:
        pytest.skip("the fp32 ring kernels need 16-byte aligned rows (refusal: test_conv_ring_refuses_unaligned)")


@pytest.mark.parametrize("precision", ["f32", "split16", "f32_ring", "bf16x3"])
@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("case", CONV_CASES, ids=[str(c[:8]) for c in CONV_CASES])
def test_conv_layer(N, dev, case, split, precision):
    c_in, c_out, k, s, d, transposed, act, has_res, B, T = case
    _ring_skip(precision, T)
    x, w, b, alpha, res, pad, ref = conv_case(case)
    got = run_conv(N, dev, x, w, b, alpha, res,
                   c_in, c_out, k, s, d, pad, transposed, act, split, N.PRECISION[precision])
    assert np.isfinite(got).all()
    assert maxabs(got, ref) <= 2e-5 * max(1.0, np.abs(ref).max())


# v2's conv shapes at bench size (T % 4 == 0): the strided down-convs, a ConvT,
# a C = 512 k3 and the k1 with residual
BF3_CONV_CASES = [CONV_CASES[i] for i in (4, 5, 8, 12)] + CONV_CASES[-2:]


@pytest.mark.parametrize("case", BF3_CONV_CASES, ids=[str(c[:8]) for c in BF3_CONV_CASES])
def test_conv_bf16x3_is_fp32_class(N, dev, case):
    """The bf16x3 conv (conv1d_bf3_kernel) against the exact-fp32 ring conv on
    the same inputs: its error against the float64 oracle is within 1.5x (+1e-7
    of the output scale) of the exact-fp32 MFMA kernel's, and the two differ by
    fp32 ulps of the output scale (<= 1e-6), not by bf16 rounding (~4e-3)."""
    c_in, c_out, k, s, d, transposed, act, has_res, B, T = case
    x, w, b, alpha, res, pad, ref = conv_case(case)
    x = 4.0 * x                                  # operands well past 1
    from oracle.rave_oracle import conv1d, conv_transpose1d, leaky_relu, snake
    xa = x.astype(np.float64)
    xa = leaky_relu(xa) if act == "leaky" else snake(xa, alpha.reshape(-1, 1)) if act == "snake" else xa
    ref = conv_transpose1d(xa, w, s, s // 2, b) if transposed else conv1d(xa, w, b, s, d, pad)
    if has_res:
        ref = ref + res
    outs = {p: run_conv(N, dev, x, w, b, alpha, res, c_in, c_out, k, s, d, pad, transposed, act, True,
                        N.PRECISION[p]) for p in ("f32_ring", "bf16x3")}
    scale = float(np.abs(ref).max())
    e_ring = maxabs(outs["f32_ring"], ref) / scale
    e_bf3 = maxabs(outs["bf16x3"], ref) / scale
    d_rb = maxabs(outs["bf16x3"], outs["f32_ring"]) / scale
    print(f"\n[bf16x3] conv {case[:8]}: rel err vs float64 ring {e_ring:.2e} bf16x3 {e_bf3:.2e}; "
          f"bf16x3 vs ring {d_rb:.2e}")
    assert np.isfinite(outs["bf16x3"]).all()
    assert e_bf3 <= 1.5 * e_ring + 1e-7
    assert d_rb <= 1e-6


CONFIG_CASES = [CONV_CASES[i] for i in (1, 2, 4, 5, 8, 9, 11, 12, 14)] + CONV_CASES[-2:]


@pytest.mark.parametrize("precision", ["f32", "split16", "f32_ring", "bf16x3"])
@pytest.mark.parametrize("case", CONFIG_CASES, ids=[str(c[:8]) for c in CONFIG_CASES])
def test_conv_every_config(N, dev, case, precision):
    """Every launch configuration rave_conv1d_configs() offers the autotuner
    (tile shape x K-splits x split-K combine) meets the layer tolerance."""
    c_in, c_out, k, s, d, transposed, act, has_res, B, T = case
    _ring_skip(precision, T)
    x, w, b, alpha, res, pad, ref = conv_case(case)
    t_out = ref.shape[-1]
    a = N.ConvArgs(c_in=c_in, c_out=c_out, kernel=k, stride=s, dilation=d,
                   pad_left=0 if transposed else pad[0], pad_right=0 if transposed else pad[1],
                   transposed=transposed, out_shift=s // 2 if transposed else 0, act=N.ACT[act],
                   batch=B, t_in=T, t_out=t_out, precision=N.PRECISION[precision], x=16, y=16, weight=16,
                   alpha=16 if alpha is not None else None, residual=16 if res is not None else None)
    cfgs = N.conv_configs(a)
    assert cfgs, "no configurations listed"
    outs = {}
    for cfg in cfgs:
        got = run_conv(N, dev, x, w, b, alpha, res, c_in, c_out, k, s, d, pad, transposed, act, True,
                       N.PRECISION[precision], config=cfg)
        err = maxabs(got, ref)
        assert np.isfinite(got).all() and err <= 2e-5 * max(1.0, np.abs(ref).max()), (cfg, err)
        outs[cfg] = got
    if precision == "f32":
        # exact-fp32 MFMA tiles (0..4): bit 9 = the in-launch combine (round 6),
        # bitwise the separate reduce launch (both sum the splits in split order)
        pairs = [(c, c + 512) for c in outs if (c - 1) & 15 < 5 and not ((c - 1) >> 9) & 1 and c + 512 in outs]
        for c0, c1 in pairs:
            assert np.array_equal(outs[c0], outs[c1]), (c0, c1)


GEMV_CASES = [
    # c_in, c_out, k, s, d, transposed, act, residual, B, T   -- the streaming shapes (U <= 32)
    (1024, 64, 3, 1, 1, 0, "leaky", False, 1, 4),
    (512, 512, 3, 1, 9, 0, "snake", True, 1, 4),
    (512, 1024, 4, 2, 1, 0, "leaky", False, 1, 8),
    (128, 256, 8, 4, 1, 0, "snake", False, 2, 128),
    (1024, 512, 4, 2, 1, 1, "leaky", False, 1, 4),
    (256, 128, 8, 4, 1, 1, "snake", False, 2, 8),
    (64, 32, 7, 1, 1, 0, "snake", False, 1, 32),
    (128, 128, 1, 1, 1, 0, "leaky", True, 1, 32),
    (320, 1024, 3, 1, 1, 0, "none", False, 1, 2),
    (96, 200, 3, 1, 3, 0, "leaky", True, 3, 13),
    (64, 64, 3, 1, 9, 0, "leaky", False, 1, 128),        # 128 columns: one row per lane
    (64, 64, 1, 1, 1, 0, "snake", True, 1, 128),
    (128, 128, 3, 1, 3, 0, "leaky", True, 2, 50),        # 64 columns: two rows per lane
    (128, 64, 8, 4, 1, 1, "leaky", False, 1, 32),        # ConvT to 128 columns
]


@pytest.mark.parametrize("case", GEMV_CASES, ids=[str(c[:8]) for c in GEMV_CASES])
def test_conv_gemv_configs(N, dev, case):
    """The skinny-N exact-fp32 family (conv_gemv.hip: weights spread over the
    chip, all output columns per workgroup), every configuration
    rave_conv1d_configs lists for it (column width x K splits x in-launch or
    separate combine), against the float64 oracle at the layer tolerance: k1 /
    k3 dilated / k7 / strided k4 s2 and k8 s4 / ConvT (both phase groups),
    LeakyReLU / Snake / none, residual, batch > 1, ragged channel counts."""
    c_in, c_out, k, s, d, transposed, act, has_res, B, T = case
    x, w, b, alpha, res, pad, ref = conv_case(case)
    t_out = ref.shape[-1]
    a = N.ConvArgs(c_in=c_in, c_out=c_out, kernel=k, stride=s, dilation=d,
                   pad_left=0 if transposed else pad[0], pad_right=0 if transposed else pad[1],
                   transposed=transposed, out_shift=s // 2 if transposed else 0, act=N.ACT[act],
                   batch=B, t_in=T, t_out=t_out, precision=N.PREC_F32, x=16, y=16, weight=16,
                   alpha=16 if alpha is not None else None, residual=16 if res is not None else None)
    # tiles 8..13: K-split over workgroups; 14 / 15: row-sliced, whole K per workgroup (round 6)
    gemv = [c for c in N.conv_configs(a) if 8 <= ((c - 1) & 15) <= 15]
    assert gemv, "no skinny-N configurations listed"
    assert T > 32 or {(c - 1) & 15 for c in gemv} >= {14, 15}, "no row-sliced configuration listed"
    outs = {}
    for cfg in gemv:
        got = run_conv(N, dev, x, w, b, alpha, res, c_in, c_out, k, s, d, pad, transposed, act, True,
                       N.PREC_F32, config=cfg)
        err = maxabs(got, ref)
        assert np.isfinite(got).all() and err <= 2e-5 * max(1.0, np.abs(ref).max()), (cfg, err)
        outs[cfg] = got
    # the in-launch combine (sc1 slabs, last arriver; round 6) sums the K splits in
    # split order, as the separate reduce launch does: bitwise the same
    pairs = [(c, c + 512) for c in outs if (c - 1) & 15 < 14 and not ((c - 1) >> 9) & 1 and c + 512 in outs]
    for c0, c1 in pairs:
        assert np.array_equal(outs[c0], outs[c1]), (c0, c1)


def test_conv_ring_refuses_unaligned(N, dev):
    """RAVE_PREC_F32_RING refuses rows it cannot DMA in 16-byte pieces (the
    autotuner then keeps the register-staged fp32 kernel for that op)."""
    c_in, c_out, k, T = 64, 64, 3, 257
    x, w = np.zeros((1, c_in, T), np.float32), np.zeros((c_out, c_in, k), np.float32)
    with pytest.raises(NotImplementedError, match="16-byte aligned"):
        run_conv(N, dev, x, w, None, None, None, c_in, c_out, k, 1, 1, (1, 1), 0, "leaky", False,
                 N.PREC_F32_RING)


# ------------------------------------------------------------------ PQMF
@pytest.mark.parametrize("precision", ["f32", "split16"])
@pytest.mark.parametrize("causal", [False, True])
def test_pqmf_golden(N, dev, golden, causal, precision):
    """rave_pqmf_analysis / rave_pqmf_synthesis (CachedPQMF.forward / inverse)
    through the C-ABI against the reference's PQMF fixtures, both paddings, in
    both arithmetics."""
    prec = N.PRECISION[precision]
    from oracle.rave_oracle import get_padding
    from rave_amd.pqmf import kernels
    g = golden("pqmf")
    mode = "causal" if causal else "centered"
    hkf, hki = kernels(g["hk"])
    hkf_d, hki_d = torch.from_numpy(hkf).to(dev), torch.from_numpy(hki).to(dev)
    x = torch.from_numpy(g["x"]).to(dev)
    B, _, T = x.shape
    F = T // 16
    y = torch.empty(B, 16, F, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = N.AnalysisArgs(n_band=16, taps=hkf.shape[-1], n_out_bands=16, batch=B, t_in=T,
                       pad_left=get_padding(hkf.shape[-1], causal=causal)[0], t_out=F, x=x.data_ptr(), x_sb=T,
                       y=y.data_ptr(), y_sb=16 * F, y_sc=F, hkf=hkf_d.data_ptr(), precision=prec)
    N.check(N.lib.rave_pqmf_analysis(C.byref(a), st))
    bands = torch.from_numpy(g["bands"]).to(dev)
    Fb = bands.shape[-1]
    out = torch.empty(B, 1, Fb * 16, device=dev)
    s_ = N.SynthesisArgs(n_band=16, taps=hki.shape[-1], batch=B, t_in=Fb,
                         pad_left=get_padding(hki.shape[-1], causal=causal)[0], mode=0, frame0=0, x_len=0,
                         x=bands.data_ptr(), x_sb=16 * Fb, x_sc=Fb, y=out.data_ptr(), y_sb=16 * Fb,
                         hki=hki_d.data_ptr(), precision=prec)
    N.check(N.lib.rave_pqmf_synthesis(C.byref(s_), st))
    torch.cuda.synchronize()
    ref_a = g[f"analysis_{mode}"]
    ref_s = g[f"synthesis_{mode}"]
    assert maxabs(y.cpu().numpy(), ref_a) <= 1e-5 * max(1, np.abs(ref_a).max())
    assert maxabs(out.cpu().numpy(), ref_s) <= 1e-5 * max(1, np.abs(ref_s).max())


@pytest.mark.parametrize("precision", ["f32", "split16"])
@pytest.mark.parametrize("causal", [False, True])
def test_pqmf_roundtrip_golden(N, dev, golden, causal, precision):
    """PQMF round trip on the GPU: rave_pqmf_analysis of the fixture audio,
    then rave_pqmf_synthesis of those device-resident bands (CachedPQMF.forward
    then .inverse, rave/pqmf.py:269-284), against the reference's own
    ``roundtrip_{centered,causal}`` outputs, in both arithmetics.  (The fused
    path edges carry a conv between the two filterbanks, so they have no pure
    round trip; tests/test_gpu_edges.py checks them against the oracle.)"""
    prec = N.PRECISION[precision]
    from oracle.rave_oracle import get_padding
    from rave_amd.pqmf import kernels
    g = golden("pqmf")
    mode = "causal" if causal else "centered"
    hkf, hki = kernels(g["hk"])
    hkf_d, hki_d = torch.from_numpy(hkf).to(dev), torch.from_numpy(hki).to(dev)
    x = torch.from_numpy(g["x"]).to(dev)
    B, _, T = x.shape
    F = T // 16
    bands = torch.empty(B, 16, F, device=dev)
    out = torch.full((B, 1, T), float("nan"), device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    a = N.AnalysisArgs(n_band=16, taps=hkf.shape[-1], n_out_bands=16, batch=B, t_in=T,
                       pad_left=get_padding(hkf.shape[-1], causal=causal)[0], t_out=F, x=x.data_ptr(), x_sb=T,
                       y=bands.data_ptr(), y_sb=16 * F, y_sc=F, hkf=hkf_d.data_ptr(), precision=prec)
    N.check(N.lib.rave_pqmf_analysis(C.byref(a), st))
    s_ = N.SynthesisArgs(n_band=16, taps=hki.shape[-1], batch=B, t_in=F,
                         pad_left=get_padding(hki.shape[-1], causal=causal)[0], mode=0, frame0=0, x_len=0,
                         x=bands.data_ptr(), x_sb=16 * F, x_sc=F, y=out.data_ptr(), y_sb=T,
                         hki=hki_d.data_ptr(), precision=prec)
    N.check(N.lib.rave_pqmf_synthesis(C.byref(s_), st))
    torch.cuda.synchronize()
    ref = g[f"roundtrip_{mode}"]
    got = out.cpu().numpy()
    assert np.isfinite(got).all()
    assert maxabs(got, ref) <= 1e-5 * max(1, np.abs(ref).max())


@pytest.mark.parametrize("case", [
    # (B, frames, mode, noise, pad, x_len, frame0, n_out)  -- offline and streaming shapes
    (3, 300, 1, True, 16, 0, 0, 6), (2, 257, 2, True, 32, 0, 0, 16), (1, 2, 1, False, 0, 34, -32, 6),
    (2, 4096, 1, False, 16, 0, 0, 6), (1, 64, 0, False, 0, 96, 7, 16)])
def test_pqmf_split16_matches_f32(N, dev, golden, case):
    """The split-f16 PQMF kernels against the exact-fp32 ones on every staging
    path the plans use: amplitude modulation / noise / plain synthesis, cached
    history (pad 0, x_len > frames, odd frame0), ragged lengths, 6 or 16 bands."""
    from rave_amd.pqmf import kernels
    B, Fr, mode, with_noise, pad, x_len, frame0, n_out = case
    hkf, hki = kernels(golden("pqmf")["hk"])
    hkf_d, hki_d = torch.from_numpy(hkf).to(dev), torch.from_numpy(hki).to(dev)
    g = torch.Generator().manual_seed(7)
    xl = x_len if x_len else Fr
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    # synthesis
    z = torch.randn(B, 32, xl, generator=g).to(dev)
    nz = (0.1 * torch.rand(B, 16, xl, generator=g)).to(dev) if with_noise else None
    outs = []
    for prec in (N.PREC_F32, N.PREC_SPLIT16):
        y = torch.empty(B, 1, Fr * 16, device=dev)
        a = N.SynthesisArgs(n_band=16, taps=hki.shape[-1], batch=B, t_in=Fr, pad_left=pad, mode=mode,
                            frame0=frame0, x_len=x_len, x=z.data_ptr(), x_sb=32 * xl, x_sc=xl,
                            noise=nz.data_ptr() if nz is not None else None, n_sb=16 * xl, n_sc=xl,
                            y=y.data_ptr(), y_sb=16 * Fr, hki=hki_d.data_ptr(), precision=prec)
        N.check(N.lib.rave_pqmf_synthesis(C.byref(a), st))
        outs.append(y)
    torch.cuda.synchronize()
    ref = outs[0].cpu().numpy()
    assert maxabs(outs[1].cpu().numpy(), ref) <= 2e-6 * max(1.0, np.abs(ref).max())
    # analysis over the same number of frames
    T = Fr * 16
    x = (0.5 * torch.randn(B, 1, T, generator=g)).to(dev)
    outs = []
    for prec in (N.PREC_F32, N.PREC_SPLIT16):
        y = torch.full((B, n_out, Fr), 7.0, device=dev)
        a = N.AnalysisArgs(n_band=16, taps=hkf.shape[-1], n_out_bands=n_out, batch=B, t_in=T, pad_left=256,
                           t_out=Fr, x=x.data_ptr(), x_sb=T, y=y.data_ptr(), y_sb=n_out * Fr, y_sc=Fr,
                           hkf=hkf_d.data_ptr(), precision=prec)
        N.check(N.lib.rave_pqmf_analysis(C.byref(a), st))
        outs.append(y)
    torch.cuda.synchronize()
    ref = outs[0].cpu().numpy()
    assert maxabs(outs[1].cpu().numpy(), ref) <= 2e-6 * max(1.0, np.abs(ref).max())


# ------------------------------------------------------------------ full model vs golden
def _model(cfg, g, dev, golden, precision="f32"):
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params
    return RAVE(cfg, init_params(cfg, seed=int(g["seed"])), g["speaker"], device=dev,
                hk=_golden_hk(golden), precision=precision)


PRECISIONS = ["f32", "split16", "auto"]
# model-level modes: + exact fp32 with autotuned launch choices (bench.py's headline mode)
MODEL_PRECISIONS = PRECISIONS + ["f32_tuned", "f32_bf3"]


@pytest.mark.parametrize("precision", MODEL_PRECISIONS)
@pytest.mark.parametrize("name", ["v2", "causal", "discrete"])
def test_model_golden(dev, golden, name, precision):
    from rave_amd import config as rcfg
    cfg = rcfg.get_config(name)
    g = golden(name)
    m = _model(cfg, g, dev, golden, precision)
    x = torch.from_numpy(g["x"]).to(dev)
    z = m.encode(x)
    ref_z = g["z_enc"] if name == "discrete" else g["z"]
    zz = z.cpu().numpy()
    ez = maxabs(zz[:, :cfg.latent_size], ref_z[:, :cfg.latent_size])
    assert ez < TOL
    assert maxabs(zz[:, cfg.latent_size:], g["speaker"][None, :, None]) == 0.0
    y = m.decode(torch.from_numpy(g["z"]).to(dev))
    torch.cuda.synchronize()
    ey = maxabs(y.cpu().numpy(), g["y"])
    print(f"\n[parity] {name} {precision}: z max-abs {ez:.3e}, y max-abs {ey:.3e}")
    assert ey < TOL


def test_discrete_codes_golden(dev, golden):
    """rvq.encode indices match the reference except where its own top-2
    distance gap is below the fp32 tie margin; decode_codes matches."""
    from rave_amd import config as rcfg
    from oracle.rave_oracle import Oracle
    cfg = rcfg.discrete()
    g = golden("discrete")
    m = _model(cfg, g, dev, golden)
    idx = m.encode_codes(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    ref = g["rvq_idx"]
    gap = g["rvq_gap"].reshape(cfg.rvq.num_quantizers, ref.shape[0], ref.shape[2]).transpose(1, 0, 2)
    mism = idx != ref
    assert (gap[mism] < 1e-3).all(), (mism.sum(), gap[mism])
    y = m.decode_codes(torch.from_numpy(ref).to(dev))
    torch.cuda.synchronize()
    assert maxabs(y.cpu().numpy(), g["y"]) < TOL


def test_rvq_kernels_golden(dev, golden, N):
    from rave_amd import config as rcfg
    from rave_amd.weights import init_params
    g = golden("rvq")
    cfg = rcfg.discrete()
    params = init_params(cfg, seed=int(g["seed"]))
    cbs = np.stack([params[f"encoder.rvq.layers.{i}._codebook.embed"] for i in range(16)])
    cb = torch.from_numpy(cbs).to(dev)
    z = torch.from_numpy(g["z"]).to(dev)
    B, D, T = z.shape
    idx = torch.empty(B, 16, T, dtype=torch.int64, device=dev)
    y = torch.empty(B, D, T, device=dev)
    a = N.RvqArgs(n_q=16, codebook_size=1024, dim=D, batch=B, t_len=T, codebooks=cb.data_ptr(),
                  z=z.data_ptr(), z_sb=D * T, z_sc=T, idx=idx.data_ptr(), i_sb=16 * T, i_sq=T,
                  y=y.data_ptr(), y_sb=D * T, y_sc=T)
    work = torch.empty(int(N.lib.rave_rvq_workspace(C.byref(a))), device=dev)
    a.work = work.data_ptr()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib.rave_rvq_encode(C.byref(a), st))
    N.check(N.lib.rave_rvq_decode(C.byref(a), st))
    torch.cuda.synchronize()
    got = idx.cpu().numpy()
    ref = g["idx"]
    gap = g["gap"].reshape(16, B, T).transpose(1, 0, 2)
    mism = got != ref
    assert (gap[mism] < 1e-3).all()
    assert mism.mean() < 0.01
    if not mism.any():
        assert maxabs(y.cpu().numpy(), g["zq"]) < 1e-5


# ------------------------------------------------------------------ larger sizes vs oracle
@pytest.mark.parametrize("precision", MODEL_PRECISIONS)
def test_v2_full_clip_vs_oracle(dev, precision):
    """One 65536-sample clip (BASELINE config 1 size) against the oracle."""
    from oracle.rave_oracle import Oracle
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2()
    params, spk = init_params(cfg, 0), init_speaker(cfg, 0)
    T = 65536
    n = np.arange(T)
    x = (0.3 * np.sin(2 * np.pi * 440 * n / 48000)
         + 0.1 * np.random.default_rng(0).standard_normal(T)).astype(np.float32)[None, None]
    m = RAVE(cfg, params, spk, device=dev, precision=precision)
    z = m.encode(torch.from_numpy(x).to(dev))
    y = m.decode(z)
    torch.cuda.synchronize()
    o = Oracle(cfg, params, spk, hk=m.hk)
    zr = o.encode(x)
    ez = maxabs(z.cpu().numpy(), zr)
    yr = o.decode(zr)
    ey = maxabs(y.cpu().numpy(), yr)
    print(f"\n[parity] v2 1x65536 {precision} vs float64 oracle: z {ez:.3e}, y {ey:.3e}")
    assert ez < TOL
    assert ey < TOL


@pytest.mark.parametrize("precision", ["f32", "auto", "f32_bf3"])
def test_discrete_codes_c4_shard_vs_oracle(dev, precision):
    """BASELINE config 4's per-GPU shard (8 x 65536 of the B=64 batch): the
    whole encode_codes -> decode_codes path, two clips checked against the
    float64 oracle.  Indices equal the oracle's wherever its top-2 distance
    gap exceeds the fp32 tie margin; decode_codes of the GPU's own indices
    matches the oracle's decode of those indices within 1e-4."""
    from oracle.rave_oracle import Oracle
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.discrete()
    params, spk = init_params(cfg, 3), init_speaker(cfg, 3)
    B, T = 8, 65536
    n = np.arange(T)
    rng = np.random.default_rng(4)
    x = np.stack([0.3 * np.sin(2 * np.pi * (220 + 55 * b) * n / 48000) + 0.1 * rng.standard_normal(T)
                  for b in range(B)])[:, None, :].astype(np.float32)
    m = RAVE(cfg, params, spk, device=dev, precision=precision)
    idx = m.encode_codes(torch.from_numpy(x).to(dev))
    y = m.decode_codes(idx)
    torch.cuda.synchronize()
    idx, y = idx.cpu().numpy(), y.cpu().numpy()
    o = Oracle(cfg, params, spk, hk=m.hk)
    for b in (0, 5):
        ref, gap = o.rvq_encode(o.encode(x[b:b + 1]), return_gaps=True)
        gap = gap.reshape(cfg.rvq.num_quantizers, 1, -1).transpose(1, 0, 2)
        mism = idx[b:b + 1] != ref
        assert (gap[mism] < 1e-3).all(), (b, int(mism.sum()))
        yr = o.decode(o.cat_speaker(o.rvq_decode(idx[b:b + 1])))
        ey = maxabs(y[b:b + 1], yr)
        print(f"\n[parity] discrete C4 shard clip {b} {precision}: index mismatches {int(mism.sum())} "
              f"(all within the tie margin), y max-abs {ey:.3e}")
        assert ey < TOL


@pytest.mark.parametrize("precision", ["f32", "auto", "f32_bf3"])
def test_batch_independence_and_determinism(dev, precision):
    """At BASELINE config 2 size (16 x 65536), in the bench's precision mode too:
    each clip of the batch equals the same clip run alone (no cross-sample
    coupling), and reruns are bitwise equal."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2()
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=precision)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (0.1 * torch.randn(16, 1, 65536, generator=g)).to(dev)
    y1 = m.forward(x)
    y2 = m.forward(x)
    y3 = m.forward(x[5:6].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.isfinite(y1).all()
    assert float((y1[5:6] - y3).abs().max()) < 1e-5


# ------------------------------------------------------------------ streaming (BASELINE config 3)
@pytest.mark.parametrize("precision", MODEL_PRECISIONS)
def test_causal_streaming_golden(dev, golden, precision):
    """Block streaming (2048-sample blocks, persistent caches) reproduces the
    reference's cached_conv streaming outputs block for block."""
    from rave_amd import config as rcfg
    from rave_amd.streaming import StreamingRAVE
    cfg = rcfg.causal()
    g = golden("causal_stream")
    m = _model(cfg, g, dev, golden, precision)
    blk = int(g["block"])
    s = StreamingRAVE(m, batch=1, block=blk)
    x = torch.from_numpy(g["x"]).to(dev)
    z = torch.from_numpy(g["z"]).to(dev)
    nb = x.shape[-1] // blk
    Fz = blk // cfg.hop
    zs = torch.cat([s.encode(x[..., i * blk:(i + 1) * blk].contiguous()) for i in range(nb)], -1)
    ys = torch.cat([s.decode(z[..., i * Fz:(i + 1) * Fz].contiguous()) for i in range(nb)], -1)
    torch.cuda.synchronize()
    assert maxabs(zs.cpu().numpy(), g["z_stream"]) < TOL
    assert maxabs(ys.cpu().numpy(), g["y_stream"]) < TOL
    assert s.decode_delay == 928


def test_streaming_matches_oneshot_long(dev):
    """64 blocks of batch 4: streamed decode == one-shot causal decode delayed by
    928 samples past the receptive field; streamed encode == one-shot encode."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.causal()
    m = RAVE(cfg, init_params(cfg, 3), init_speaker(cfg, 3), device=dev)
    B, blk, nb = 4, 2048, 64
    gen = torch.Generator().manual_seed(1)
    x = (0.2 * torch.randn(B, 1, blk * nb, generator=gen)).to(dev)
    s = StreamingRAVE(m, batch=B, block=blk)
    zs = torch.cat([s.encode(x[..., i * blk:(i + 1) * blk].contiguous()) for i in range(nb)], -1)
    z1 = m.encode(x)
    ys = torch.cat([s.decode(z1[..., i * 2:(i + 1) * 2].contiguous()) for i in range(nb)], -1)
    y1 = m.decode(z1)
    torch.cuda.synchronize()
    assert float((zs - z1).abs().max()) < 1e-4
    d, warm = 928, 12288
    assert float((ys[..., d + warm:] - y1[..., warm:-d]).abs().max()) < 1e-4
    s.reset()
    ys2 = s.decode(z1[..., :2].contiguous())
    assert torch.equal(ys2, ys[..., :blk])


def test_streaming_graph_equals_eager(dev):
    """RAVE_STREAM_GRAPH (captured hipGraph per block, staging buffers) gives
    bitwise the blocks of the eager plan replay, across a reset too."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.causal()
    m = RAVE(cfg, init_params(cfg, 4), init_speaker(cfg, 4), device=dev, precision="auto")
    sg = StreamingRAVE(m, batch=2, block=4096, graph=True)
    se = StreamingRAVE(m, batch=2, block=4096, graph=False)
    gen = torch.Generator().manual_seed(2)
    for i in range(6):
        if i == 3:
            sg.reset()
            se.reset()
        x = (0.2 * torch.randn(2, 1, 4096, generator=gen)).to(dev)
        zg, ze = sg.encode(x), se.encode(x)
        yg, ye = sg.decode(zg), se.decode(ze)
        torch.cuda.synchronize()
        assert torch.equal(zg, ze) and torch.equal(yg, ye), i


@pytest.mark.parametrize("precision", ["f32", "auto", "f32_bf3"])
@pytest.mark.parametrize("graph", [True, False])
def test_stream_v3_noise_adain_golden(dev, golden, precision, graph):
    """Streaming a causal v3 model with the noise synthesizer and AdaIN against
    the reference run in cached_conv streaming mode (make_golden.py
    gen_stream_v3): blocks learn the target statistics, then the source, then
    transfer (nn~'s learn_target / learn_source flags switched between
    blocks); the decoder's per-block uniform noise is the reference's."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params
    g = golden("v3_noise_causal_stream")
    cfg = rcfg.v3_noise(causal=True, capacity=16)
    m = RAVE(cfg, init_params(cfg, int(g["seed"])), g["speaker"], device=dev, hk=_golden_hk(golden),
             precision=precision)
    blk = int(g["block"])
    s = StreamingRAVE(m, batch=1, block=blk, graph=graph)
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
    print(f"\n[parity] v3+noise+AdaIN causal streaming {precision} graph={graph}: z {ez:.3e}, y {ey:.3e}")
    assert ez < TOL and ey < TOL


def test_engine_forward_and_device_noise(dev):
    """rave_model_forward == decode(encode(x)) bitwise; a noise config with no
    noise tensor draws it on the device (a fresh draw per call, finite output,
    same statistics as the injected-noise path)."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    N = pytest.importorskip("rave_amd._native")
    cfg = rcfg.v2(capacity=8)
    m = RAVE(cfg, init_params(cfg, 1), init_speaker(cfg, 1), device=dev)
    x = (0.2 * torch.randn(2, 1, 8192, generator=torch.Generator().manual_seed(5))).to(dev)
    y = torch.empty_like(x)
    N.check(N.lib.rave_model_forward(m.handle, x.data_ptr(), 2, 8192, y.data_ptr(), None,
                                     C.c_void_p(torch.cuda.current_stream().cuda_stream)), "forward")
    assert torch.equal(y, m.decode(m.encode(x)))
    cfgn = rcfg.v3_noise(capacity=8)
    mn = RAVE(cfgn, init_params(cfgn, 1), init_speaker(cfgn, 1), device=dev)
    z = torch.randn(2, cfgn.dec_in, 8, generator=torch.Generator().manual_seed(6)).to(dev)
    y1, y2 = mn.decode(z), mn.decode(z)
    u = torch.rand(mn.noise_shape(2, 8), device=dev)
    y3 = mn.decode(z, noise_u=u)
    torch.cuda.synchronize()
    assert torch.isfinite(y1).all() and not torch.equal(y1, y2)
    assert float((y1 - y3).abs().max()) < 0.5 and float((y1 - y3).abs().max()) > 0


# ------------------------------------------------------------------ v3 noise / AdaIN (BASELINE config 5)
@pytest.mark.parametrize("precision", PRECISIONS + ["f32_bf3"])
@pytest.mark.parametrize("name,capacity", [("v3_noise", None), ("v3_noise_small_layers", 8)])
def test_v3_noise_golden(dev, golden, name, capacity, precision):
    """Snake + NoiseGeneratorV2 decode with the reference's injected uniform noise."""
    from rave_amd import config as rcfg
    cfg = rcfg.v3_noise() if capacity is None else rcfg.v3_noise(capacity=capacity)
    g = golden(name)
    m = _model(cfg, g, dev, golden, precision)
    x = torch.from_numpy(g["x"]).to(dev)
    u = torch.from_numpy(g["noise_u"]).to(dev)
    if "z" in g:
        z = m.encode(x)
        torch.cuda.synchronize()
        assert maxabs(z.cpu().numpy(), g["z"]) < TOL
        y = m.decode(torch.from_numpy(g["z"]).to(dev), u)
    else:
        y = m.forward(x, u)
    torch.cuda.synchronize()
    assert maxabs(y.cpu().numpy(), g["y"]) < TOL


def test_noise_synth_kernel_vs_oracle(dev, N):
    """The filter stage alone (mod_sigmoid -> impulse response -> fft_convolve)
    on wide-range amplitudes against the oracle's float64 FFT restatement."""
    from oracle.rave_oracle import Oracle
    from rave_amd import config as rcfg
    cfg = rcfg.v3_noise()
    rng = np.random.default_rng(5)
    B, Fn, nb, tgt = 3, 700, 5, 8
    amp = (rng.standard_normal((B, 16 * nb, Fn)) * 4 + 3).astype(np.float32)
    u = rng.uniform(0, 1, (B, Fn, 16, tgt)).astype(np.float32)
    o = Oracle(cfg, {}, np.zeros(256))
    # oracle filter stage: noise_generator with its convs bypassed
    o._conv = lambda x, *a, **k: x
    o._act = lambda x, *a, **k: x
    ref = o.noise_generator(amp.astype(np.float64), u)
    a_t, u_t = torch.from_numpy(amp).to(dev), torch.from_numpy(u).to(dev)
    y = torch.empty(B, 16, Fn * tgt, device=dev)
    a = N.NoiseArgs(batch=B, frames=Fn, n_band=16, noise_bands=nb, target=tgt, amp=a_t.data_ptr(),
                    a_sb=16 * nb * Fn, a_sc=Fn, u=u_t.data_ptr(), u_sb=Fn * 16 * tgt,
                    y=y.data_ptr(), y_sb=16 * Fn * tgt, y_sc=Fn * tgt)
    N.check(N.lib.rave_noise_synth(C.byref(a), C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    assert maxabs(got, ref) < 2e-6 * max(1.0, float(np.abs(ref).max()))


@pytest.mark.parametrize("precision", ["f32", "f32_bf3"])
def test_v3_noise_decode_c5_shard_vs_oracle(dev, precision):
    """BASELINE config 5 per-GPU shard geometry (16 x 64 latent frames) on two
    samples against the oracle, plus device-drawn noise statistics."""
    from oracle.rave_oracle import Oracle
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3_noise()
    params, spk = init_params(cfg, 3), init_speaker(cfg, 3)
    m = RAVE(cfg, params, spk, device=dev, precision=precision)
    rng = np.random.default_rng(9)
    z = rng.standard_normal((16, cfg.dec_in, 64)).astype(np.float32)
    u = rng.uniform(0, 1, m.noise_shape(16, 64)).astype(np.float32)
    y = m.decode(torch.from_numpy(z).to(dev), torch.from_numpy(u).to(dev))
    y_rand = m.decode(torch.from_numpy(z).to(dev))          # device-drawn noise
    torch.cuda.synchronize()
    o = Oracle(cfg, params, spk, hk=m.hk)
    yr = o.decode(z[[0, 11]], u[[0, 11]])
    assert maxabs(y.cpu().numpy()[[0, 11]], yr) < TOL
    d = (y_rand - y).abs()
    assert torch.isfinite(y_rand).all() and float(d.max()) < 0.05   # noise is a small additive term


@pytest.mark.parametrize("precision", PRECISIONS + ["f32_bf3"])
def test_adain_style_transfer_golden(dev, golden, precision):
    """learn_y -> learn_x -> transfer -> learn_x(bs=1) against the reference's
    AdaIN run, including the device-resident buffers and counters."""
    from rave_amd import config as rcfg
    from tests.test_oracle_golden import adain_sequence
    for name, cfg in [("v3_adain_small", rcfg.v3(capacity=8)), ("v3_adain", rcfg.v3())]:
        g = golden(name)
        m = _model(cfg, g, dev, golden, precision)
        assert not m.adain.active
        for i, (tag, lx, ly, x) in enumerate(adain_sequence(g)):
            m.adain.set_learn(lx, ly)
            z = m.encode(torch.from_numpy(np.ascontiguousarray(x)).to(dev))
            y = m.decode(z)
            torch.cuda.synchronize()
            zr = g[f"step{i}/z"]
            assert maxabs(z.cpu().numpy(), zr) < TOL * max(1.0, float(np.abs(zr).max())), (name, tag)
            assert maxabs(y.cpu().numpy(), g[f"step{i}/y"]) < TOL, (name, tag)
        sd = m.adain.state_dict()
        for n, _ in m.graph.adain_modules:
            for b in ("mean_x", "std_x", "mean_y", "std_y"):
                ref = g[f"final/{n}.{b}"]
                assert maxabs(sd[f"{n}.{b}"], ref) < 1e-4 * max(1.0, float(np.abs(ref).max())), (n, b)
            for b in ("num_update_x", "num_update_y"):
                assert float(sd[f"{n}.{b}"][0]) == float(g[f"final/{n}.{b}"][0])


def test_adain_state_roundtrip(dev):
    """AdaIN buffers held by the engine: reference init, load/state_dict under
    the reference's names, learn flags -> kernel mode (learn_y wins, as
    forward checks it first), reset_y."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3(capacity=4)
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev)
    st = m.adain
    assert not st.active and st.mode == 0 and len(st.modules) == 22
    (a, ca), (b, cb) = st.modules[0], st.modules[-1]
    sd = st.state_dict()
    assert sd[f"{a}.mean_x"].shape == (64, ca, 1) and (sd[f"{b}.std_y"] == 1).all()
    rng = np.random.default_rng(0)
    new = {f"{b}.mean_y": rng.standard_normal((64, cb, 1)), f"{b}.num_update_y": np.array([3.0])}
    st.load(new)
    assert st.active
    sd = st.state_dict()
    assert np.allclose(sd[f"{b}.mean_y"], new[f"{b}.mean_y"]) and sd[f"{b}.num_update_y"][0] == 3.0
    assert (sd[f"{a}.mean_y"] == 0).all()
    st.set_learn(learn_x=True, learn_y=True)
    assert st.mode == 2
    st.set_learn(learn_y=False)
    assert st.mode == 1
    st.reset_y()
    assert (st.state_dict()[f"{b}.mean_y"] == 0).all() and st.state_dict()[f"{b}.num_update_y"][0] == 0


def test_adain_loaded_stats_and_batch_limit(dev):
    """Stats loaded from a state_dict transfer like the oracle; a batch past
    the buffers' MAX_BATCH_SIZE rows raises like the reference."""
    from oracle.rave_oracle import Oracle
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3(capacity=8)
    params, spk = init_params(cfg, 1), init_speaker(cfg, 1)
    m0 = RAVE(cfg, params, spk, device=dev)
    rng = np.random.default_rng(4)
    state = {}
    for n, c in m0.graph.adain_modules:
        state[f"{n}.mean_x"] = rng.standard_normal((64, c, 1)) * 0.1
        state[f"{n}.std_x"] = rng.uniform(0.5, 2.0, (64, c, 1))
        state[f"{n}.mean_y"] = rng.standard_normal((64, c, 1)) * 0.1
        state[f"{n}.std_y"] = rng.uniform(0.5, 2.0, (64, c, 1))
        state[f"{n}.num_update_x"] = np.ones(1)
        state[f"{n}.num_update_y"] = np.ones(1)
    m = RAVE(cfg, params, spk, device=dev, adain_stats=state)
    x = (0.1 * rng.standard_normal((3, 1, 4096))).astype(np.float32)
    y = m.forward(torch.from_numpy(x).to(dev))
    torch.cuda.synchronize()
    ost = {n: {k.split(".")[-1]: np.array(v, np.float64) if np.ndim(v) > 1 else float(v[0])
               for k, v in state.items() if k.rsplit(".", 1)[0] == n} for n, _ in m.graph.adain_modules}
    o = Oracle(cfg, params, spk, hk=m.hk, adain_stats=ost)
    assert maxabs(y.cpu().numpy(), o.forward(x)) < TOL
    with pytest.raises(ValueError):
        m.forward(torch.zeros(65, 1, 4096, device=dev))


def test_no_amplitude_modulation_epilogue(dev):
    """GeneratorV2 without amplitude modulation still ends in tanh (mode 2)."""
    from oracle.rave_oracle import Oracle
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2(capacity=8, amplitude_modulation=False)
    params, spk = init_params(cfg, 2), init_speaker(cfg, 2)
    m = RAVE(cfg, params, spk, device=dev)
    x = (0.2 * np.random.default_rng(1).standard_normal((2, 1, 4096))).astype(np.float32)
    y = m.forward(torch.from_numpy(x).to(dev))
    torch.cuda.synchronize()
    o = Oracle(cfg, params, spk, hk=m.hk)
    assert maxabs(y.cpu().numpy(), o.forward(x)) < TOL


# ------------------------------------------------------------------ fused Residual(DilatedUnit)
UNIT_CASES = [
    # C, d, act, causal, B, T
    (64, 1, "leaky", False, 2, 4096),
    (64, 9, "leaky", False, 2, 1000),
    (64, 3, "snake", True, 1, 300),
    (128, 3, "leaky", False, 3, 1024),
    (128, 9, "snake", False, 2, 200),
    (256, 1, "leaky", False, 2, 256),
    (256, 9, "snake", True, 2, 77),
    (512, 3, "leaky", False, 2, 128),
    (512, 1, "snake", False, 1, 40),
]


@pytest.mark.parametrize("precision", PRECISIONS + ["f32_ring", "bf16x3"])
@pytest.mark.parametrize("case", UNIT_CASES, ids=[str(c) for c in UNIT_CASES])
def test_residual_unit_kernel(N, dev, case, precision):
    """rave_residual_unit == x + conv1x1(act(conv3_d(act(x)) + b1)) + b2 (oracle, float64)."""
    from oracle.rave_oracle import conv1d, leaky_relu, snake
    C, d, act, causal, B, T = case
    rng = np.random.default_rng(C + d)
    x = rng.standard_normal((B, C, T)).astype(np.float32)
    w1 = (rng.standard_normal((C, C, 3)) / np.sqrt(3 * C)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, 1)) / np.sqrt(C)).astype(np.float32)
    b1 = rng.standard_normal(C).astype(np.float32) * 0.1
    b2 = rng.standard_normal(C).astype(np.float32) * 0.1
    a0 = (1 + 0.3 * rng.standard_normal(C)).astype(np.float32)
    a2 = (1 + 0.3 * rng.standard_normal(C)).astype(np.float32)
    pad = (2 * d, 0) if causal else (d, d)
    f = (lambda v, al: snake(v, al.reshape(-1, 1))) if act == "snake" else (lambda v, al: leaky_relu(v, 0.2))
    h = f(conv1d(f(x.astype(np.float64), a0), w1, b1, 1, d, pad), a2)
    ref = x + conv1d(h, w2, b2, 1, 1, (0, 0))
    if precision == "auto":
        pytest.skip("auto is a per-op choice between the two kernels tested here")
    prec = N.PRECISION[precision]
    if not N.unit_supported(C, prec):
        pytest.skip(f"no fused {precision} unit for C={C} (the model runs it as two convs)")
    packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C, precision=prec)).to(dev)
    xd = torch.from_numpy(x).to(dev)
    y = torch.full_like(xd, float("nan"))
    dd = {k: torch.from_numpy(v).to(dev) for k, v in dict(b1=b1, b2=b2, a0=a0, a2=a2).items()}
    a = N.UnitArgs(channels=C, batch=B, t_len=T, dilation=d, pad_left=pad[0], act=N.ACT[act],
                   leaky_slope=0.2, precision=prec, x=xd.data_ptr(), x_sb=C * T, x_sc=T, y=y.data_ptr(), y_sb=C * T,
                   y_sc=T, weight=packed.data_ptr(), bias1=dd["b1"].data_ptr(), bias2=dd["b2"].data_ptr(),
                   alpha0=dd["a0"].data_ptr() if act == "snake" else None,
                   alpha2=dd["a2"].data_ptr() if act == "snake" else None)
    N.check(N.lib.rave_residual_unit(C_.byref(a), C_.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    assert np.isfinite(got).all()
    assert maxabs(got, ref) <= 2e-5 * max(1.0, float(np.abs(ref).max()))


BF3_CASES = [(64, 9, "snake", False, 4, 1000), (128, 3, "leaky", True, 3, 517), (256, 1, "leaky", False, 16, 256)]


@pytest.mark.parametrize("case", BF3_CASES, ids=[str(c) for c in BF3_CASES])
def test_residual_unit_bf16x3_is_fp32_class(N, dev, case):
    """bf16x3 (exact 3-way bf16 operand split, six products, fp32 accumulation)
    against the exact-fp32 ring kernel on the same inputs: its error against the
    float64 oracle is that of fp32 (within 1.5x + 1e-7 of the ring kernel's) and
    the two differ by a few fp32 ulps of the output scale, not by f16/bf16
    rounding (~1e-3)."""
    from oracle.rave_oracle import conv1d, leaky_relu, snake
    C, d, act, causal, B, T = case
    rng = np.random.default_rng(7 * C + d)
    x = (4.0 * rng.standard_normal((B, C, T))).astype(np.float32)   # operands well past 1
    w1 = (rng.standard_normal((C, C, 3)) / np.sqrt(3 * C)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, 1)) / np.sqrt(C)).astype(np.float32)
    b1 = rng.standard_normal(C).astype(np.float32) * 0.1
    b2 = rng.standard_normal(C).astype(np.float32) * 0.1
    a0 = (1 + 0.3 * rng.standard_normal(C)).astype(np.float32)
    a2 = (1 + 0.3 * rng.standard_normal(C)).astype(np.float32)
    pad = (2 * d, 0) if causal else (d, d)
    f = (lambda v, al: snake(v, al.reshape(-1, 1))) if act == "snake" else (lambda v, al: leaky_relu(v, 0.2))
    h = f(conv1d(f(x.astype(np.float64), a0), w1, b1, 1, d, pad), a2)
    ref = x + conv1d(h, w2, b2, 1, 1, (0, 0))
    xd = torch.from_numpy(x).to(dev)
    dd = {k: torch.from_numpy(v).to(dev) for k, v in dict(b1=b1, b2=b2, a0=a0, a2=a2).items()}
    outs = {}
    for name in ("f32_ring", "bf16x3"):
        prec = N.PRECISION[name]
        packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C, precision=prec)).to(dev)
        y = torch.full_like(xd, float("nan"))
        a = N.UnitArgs(channels=C, batch=B, t_len=T, dilation=d, pad_left=pad[0], act=N.ACT[act],
                       leaky_slope=0.2, precision=prec, x=xd.data_ptr(), x_sb=C * T, x_sc=T, y=y.data_ptr(),
                       y_sb=C * T, y_sc=T, weight=packed.data_ptr(), bias1=dd["b1"].data_ptr(),
                       bias2=dd["b2"].data_ptr(), alpha0=dd["a0"].data_ptr() if act == "snake" else None,
                       alpha2=dd["a2"].data_ptr() if act == "snake" else None)
        N.check(N.lib.rave_residual_unit(C_.byref(a), C_.c_void_p(torch.cuda.current_stream().cuda_stream)))
        torch.cuda.synchronize()
        outs[name] = y.cpu().numpy()
    scale = float(np.abs(ref).max())
    e_ring = maxabs(outs["f32_ring"], ref) / scale
    e_bf3 = maxabs(outs["bf16x3"], ref) / scale
    d_rb = maxabs(outs["bf16x3"], outs["f32_ring"]) / scale
    print(f"\n[bf16x3] C={C}: rel err vs float64 ring {e_ring:.2e} bf16x3 {e_bf3:.2e}; bf16x3 vs ring {d_rb:.2e}")
    assert np.isfinite(outs["bf16x3"]).all()
    assert e_bf3 <= 1.5 * e_ring + 1e-7
    assert d_rb <= 1e-6


COOP_CASES = [
    # C, d, act, causal, B, T (C, rb: the wide group, coop_rb = 4 at C = 256, round 6)
    (256, 3, "leaky", False, 16, 256),
    (256, 9, "snake", True, 3, 77),
    (512, 3, "leaky", False, 16, 128),
    (512, 1, "snake", False, 2, 40),
    (512, 9, "leaky", True, 5, 333),
    ((256, 4), 3, "leaky", False, 16, 256),
    ((256, 4), 9, "snake", True, 3, 77),
    ((256, 4), 1, "leaky", False, 1, 8),
]


@pytest.mark.parametrize("precision", ["split16", "f32_ring", "bf16x3"])
@pytest.mark.parametrize("case", COOP_CASES, ids=[str(c) for c in COOP_CASES])
def test_residual_unit_cooperative(N, dev, case, precision):
    """The cooperative fused unit (groups of C/128 workgroups handing act2(h) rows
    to each other inside the launch, rave_unit_workspace) matches the one-
    workgroup-per-slab kernel (same operands; its K-steps alternate over two
    accumulator chains, so sums differ in the last bits only), meets the
    oracle, leaves its counters zero (three calls on one workspace) and never
    gives up waiting (a give-up writes NaN)."""
    from oracle.rave_oracle import conv1d, leaky_relu, snake
    C, d, act, causal, B, T = case
    C, rb = C if isinstance(C, tuple) else (C, 0)
    prec = N.PRECISION[precision]
    if precision == "f32_ring" and T % 4:
        pytest.skip("fp32 ring units need whole 16-byte rows")
    if precision == "bf16x3" and C == 512 and d > 4:
        pytest.skip("the bf16x3 unit takes dilations <= 4 at C = 512 (three planes in LDS)")
    rng = np.random.default_rng(C + d + T)
    x = rng.standard_normal((B, C, T)).astype(np.float32)
    w1 = (rng.standard_normal((C, C, 3)) / np.sqrt(3 * C)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, 1)) / np.sqrt(C)).astype(np.float32)
    b1, b2 = (rng.standard_normal(C).astype(np.float32) * 0.1 for _ in range(2))
    a0, a2 = ((1 + 0.3 * rng.standard_normal(C)).astype(np.float32) for _ in range(2))
    pad = (2 * d, 0) if causal else (d, d)
    f = (lambda v, al: snake(v, al.reshape(-1, 1))) if act == "snake" else (lambda v, al: leaky_relu(v, 0.2))
    h = f(conv1d(f(x.astype(np.float64), a0), w1, b1, 1, d, pad), a2)
    ref = x + conv1d(h, w2, b2, 1, 1, (0, 0))
    packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C, precision=prec)).to(dev)
    xd = torch.from_numpy(x).to(dev)
    dd = {k: torch.from_numpy(v).to(dev) for k, v in dict(b1=b1, b2=b2, a0=a0, a2=a2).items()}

    def args(y, ws):
        return N.UnitArgs(channels=C, batch=B, t_len=T, dilation=d, pad_left=pad[0], act=N.ACT[act],
                          leaky_slope=0.2, precision=prec, x=xd.data_ptr(), x_sb=C * T, x_sc=T, y=y.data_ptr(),
                          y_sb=C * T, y_sc=T, weight=packed.data_ptr(), bias1=dd["b1"].data_ptr(),
                          bias2=dd["b2"].data_ptr(), alpha0=dd["a0"].data_ptr() if act == "snake" else None,
                          alpha2=dd["a2"].data_ptr() if act == "snake" else None,
                          workspace=ws.data_ptr() if ws is not None else None, coop_rb=rb)
    st = C_.c_void_p(torch.cuda.current_stream().cuda_stream)
    y1 = torch.full_like(xd, float("nan"))
    N.check(N.lib.rave_residual_unit(C_.byref(args(y1, None)), st))
    nws = N.lib.rave_unit_workspace(C_.byref(args(y1, None)))
    assert nws > N.SPLITK_TICKETS
    ws = torch.zeros(nws, device=dev)
    for _ in range(3):
        y2 = torch.full_like(xd, float("nan"))
        N.check(N.lib.rave_residual_unit(C_.byref(args(y2, ws)), st))
        torch.cuda.synchronize()
        assert float((y1 - y2).abs().max()) <= 1e-6 * float(y1.abs().max())
        assert int(torch.count_nonzero(ws[:N.SPLITK_TICKETS])) == 0      # counters re-armed, no give-up
    got = y2.cpu().numpy()
    assert np.isfinite(got).all()
    assert maxabs(got, ref) <= 2e-5 * max(1.0, float(np.abs(ref).max()))


CACHED_UNIT_CASES = [
    # C, d, act, causal, B, T, coop
    (64, 1, "leaky", True, 1, 1, False),
    (64, 9, "snake", False, 2, 16, False),
    (128, 3, "leaky", True, 1, 128, False),
    (128, 9, "leaky", False, 2, 37, False),
    (128, 1, "snake", False, 2, 126, False),      # x_len % 4 == 0: 16-byte window loads
    (256, 3, "snake", True, 1, 32, False),
    (256, 9, "leaky", True, 2, 64, True),
    (512, 1, "leaky", False, 1, 8, True),
    (256, 3, "leaky", True, 1, 8, 4),             # the wide cooperative group (coop_rb = 4)
    (256, 9, "snake", False, 1, 16, 4),
]


@pytest.mark.parametrize("precision", ["f32", "split16", "f32_ring", "bf16x3"])
@pytest.mark.parametrize("case", CACHED_UNIT_CASES, ids=[str(c) for c in CACHED_UNIT_CASES])
def test_residual_unit_cached_form(N, dev, case, precision):
    """The cached (streaming) fused unit: x holds need = 2d history columns then
    the block (x_len = 2d + T, pad_left 0, rows wider than x_len), the residual
    is x shifted by res_shift = 2d - delay (AlignBranches: causal delay 0,
    centred d; rave/blocks.py:32-46, cached_conv convs pad nothing), against
    the oracle on the same window."""
    from oracle.rave_oracle import conv1d, leaky_relu, snake
    C, d, act, causal, B, T, coop = case
    prec = N.PRECISION[precision]
    if not N.unit_supported(C, prec):
        pytest.skip(f"no fused {precision} unit for C={C}")
    need = 2 * d
    rs = need - (0 if causal else d)
    XL = need + T
    SC = (XL + 3) // 4 * 4 + 4                    # 16-byte rows, wider than x_len
    rng = np.random.default_rng(C + d + T)
    xw = np.zeros((B, C, SC), np.float32)
    xw[:, :, :XL] = rng.standard_normal((B, C, XL))
    xw[:, :, XL:] = np.nan                        # row padding past x_len is never read
    w1 = (rng.standard_normal((C, C, 3)) / np.sqrt(3 * C)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, 1)) / np.sqrt(C)).astype(np.float32)
    b1, b2 = (rng.standard_normal(C).astype(np.float32) * 0.1 for _ in range(2))
    a0, a2 = ((1 + 0.3 * rng.standard_normal(C)).astype(np.float32) for _ in range(2))
    f = (lambda v, al: snake(v, al.reshape(-1, 1))) if act == "snake" else (lambda v, al: leaky_relu(v, 0.2))
    x = xw[:, :, :XL].astype(np.float64)
    h = f(conv1d(f(x, a0), w1, b1, 1, d, (0, 0)), a2)
    ref = x[:, :, rs:rs + T] + conv1d(h, w2, b2, 1, 1, (0, 0))
    packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C, precision=prec)).to(dev)
    xd = torch.from_numpy(xw).to(dev)
    dd = {k: torch.from_numpy(v).to(dev) for k, v in dict(b1=b1, b2=b2, a0=a0, a2=a2).items()}
    y = torch.full((B, C, T), float("nan"), device=dev)

    def args(ws):
        return N.UnitArgs(channels=C, batch=B, t_len=T, dilation=d, pad_left=0, act=N.ACT[act],
                          leaky_slope=0.2, precision=prec, x=xd.data_ptr(), x_sb=C * SC, x_sc=SC, y=y.data_ptr(),
                          y_sb=C * T, y_sc=T, weight=packed.data_ptr(), bias1=dd["b1"].data_ptr(),
                          bias2=dd["b2"].data_ptr(), alpha0=dd["a0"].data_ptr() if act == "snake" else None,
                          alpha2=dd["a2"].data_ptr() if act == "snake" else None,
                          workspace=ws.data_ptr() if ws is not None else None, x_len=XL, res_shift=rs,
                          coop_rb=4 if coop == 4 else 0)
    ws = None
    if coop:
        nws = N.lib.rave_unit_workspace(C_.byref(args(None)))
        if nws > 0:
            ws = torch.zeros(nws, device=dev)
    N.check(N.lib.rave_residual_unit(C_.byref(args(ws)), C_.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    assert np.isfinite(got).all()
    assert maxabs(got, ref) <= 2e-5 * max(1.0, float(np.abs(ref).max()))
    if ws is not None:
        assert int(torch.count_nonzero(ws[:N.SPLITK_TICKETS])) == 0


@pytest.mark.parametrize("precision,n_fused", [("f32", 22), ("split16", 22), ("auto", 22)])
def test_fused_units_match_unfused_model(N, dev, precision, n_fused):
    """The v2 plan with fused residual units equals the conv-by-conv plan."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2()
    params, spk = init_params(cfg, 0), init_speaker(cfg, 0)
    from rave_amd.model import DECODE, ENCODE
    mf = RAVE(cfg, params, spk, device=dev, precision=precision)
    mu = RAVE(cfg, params, spk, device=dev, fuse_units=False, precision=precision)

    def units(m):
        ops = m.ops(ENCODE, 4, 65536) + m.ops(DECODE, 4, 64)
        return sum(1 for o in ops if o["kind"] == N.OP_UNIT) + 3 * sum(1 for o in ops if o["kind"] == N.OP_STACK)
    assert units(mu) == 0
    if precision == "auto":
        assert 0 < units(mf) <= n_fused          # fused where it measured faster
    else:
        assert units(mf) == n_fused
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (0.1 * torch.randn(4, 1, 65536, generator=g)).to(dev)
    zf, zu = mf.encode(x), mu.encode(x)
    yf, yu = mf.decode(zf), mu.decode(zf)
    torch.cuda.synchronize()
    assert float((zf - zu).abs().max()) < 1e-4
    assert float((yf - yu).abs().max()) < 1e-4


def test_auto_tuning_roundtrip(dev):
    """RAVE.tuning() replayed into a new model builds the same plans (same
    per-op choices, no timing runs) and gives bitwise the same output."""
    import json
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2()
    params, spk = init_params(cfg, 0), init_speaker(cfg, 0)
    m1 = RAVE(cfg, params, spk, device=dev, precision="auto")
    g = torch.Generator(device="cpu").manual_seed(3)
    x = (0.1 * torch.randn(2, 1, 32768, generator=g)).to(dev)
    y1 = m1.forward(x)
    tun = json.loads(json.dumps(m1.tuning()))
    kinds = {k.split("|")[0] for k, _, _ in tun}
    assert {"fuse", "conv", "unit"} <= kinds
    m2 = RAVE(cfg, params, spk, device=dev, precision="auto", tuning=tun)
    y2 = m2.forward(x)
    torch.cuda.synchronize()
    assert m2.tuning() == m1.tuning()
    assert torch.equal(y1, y2)


STACK_CASES = [
    # C, dilations, act, causal, B, T
    (64, (1, 3, 9), "leaky", False, 2, 1000),
    (64, (1, 3, 9), "snake", True, 1, 300),
    (128, (1, 3, 9), "leaky", False, 2, 257),
    (128, (1, 3, 9), "snake", False, 1, 64),
    (64, (1, 3, 9), "leaky", True, 3, 20),
    (128, (2, 5, 11), "leaky", False, 1, 500),
]


@pytest.mark.parametrize("precision", ["split16", "bf16x3"])
@pytest.mark.parametrize("case", STACK_CASES, ids=[str(c) for c in STACK_CASES])
def test_residual_stack_kernel(N, dev, case, precision):
    """rave_residual_stack == the three units one after the other (oracle,
    float64, and the unit kernel of the same arithmetic run three times): the
    split16 stack, and the bf16x3 one the f32_bf3 plans run (round 5)."""
    from oracle.rave_oracle import conv1d, leaky_relu, snake
    C, dils, act, causal, B, T = case
    prec = N.PRECISION[precision]
    rng = np.random.default_rng(C + sum(dils) + T)
    x = rng.standard_normal((B, C, T)).astype(np.float32)
    xd = torch.from_numpy(x).to(dev)
    units, args = [], N.StackArgs(channels=C, batch=B, t_len=T, act=N.ACT[act], leaky_slope=0.2,
                                  precision=prec)
    keep = []
    for u, d in enumerate(dils):
        w1 = (rng.standard_normal((C, C, 3)) / np.sqrt(3 * C)).astype(np.float32)
        w2 = (rng.standard_normal((C, C, 1)) / np.sqrt(C)).astype(np.float32)
        b1 = (rng.standard_normal(C) * 0.1).astype(np.float32)
        b2 = (rng.standard_normal(C) * 0.1).astype(np.float32)
        a0 = (1 + 0.3 * rng.standard_normal(C)).astype(np.float32)
        a2 = (1 + 0.3 * rng.standard_normal(C)).astype(np.float32)
        pad = (2 * d, 0) if causal else (d, d)
        units.append((w1, w2, b1, b2, a0, a2, d, pad))
        tens = [torch.from_numpy(N.pack_unit_weight(w1, w2, C, precision=prec)).to(dev)] + \
               [torch.from_numpy(v).to(dev) for v in (b1, b2, a0, a2)]
        keep += tens
        setattr(args, f"dilation{u}", d)
        setattr(args, f"pad_left{u}", pad[0])
        for f, t in zip(("weight", "bias1", "bias2", "alpha0", "alpha2"), tens):
            setattr(args, f"{f}{u}", t.data_ptr())
    y = torch.full_like(xd, float("nan"))
    args.x, args.x_sb, args.x_sc = xd.data_ptr(), C * T, T
    args.y, args.y_sb, args.y_sc = y.data_ptr(), C * T, T
    st = C_.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib.rave_residual_stack(C_.byref(args), st), "residual_stack")
    # the same three units through the single-unit kernel
    cur = xd
    for u, (w1, w2, b1, b2, a0, a2, d, pad) in enumerate(units):
        nxt = torch.empty_like(xd)
        ua = N.UnitArgs(channels=C, batch=B, t_len=T, dilation=d, pad_left=pad[0], act=N.ACT[act],
                        leaky_slope=0.2, precision=prec, x=cur.data_ptr(), x_sb=C * T, x_sc=T,
                        y=nxt.data_ptr(), y_sb=C * T, y_sc=T, weight=getattr(args, f"weight{u}"),
                        bias1=getattr(args, f"bias1{u}"), bias2=getattr(args, f"bias2{u}"),
                        alpha0=getattr(args, f"alpha0{u}"), alpha2=getattr(args, f"alpha2{u}"))
        N.check(N.lib.rave_residual_unit(C_.byref(ua), st), "residual_unit")
        cur = nxt
    torch.cuda.synchronize()
    got, seq = y.cpu().numpy(), cur.cpu().numpy()
    ref = x.astype(np.float64)
    for w1, w2, b1, b2, a0, a2, d, pad in units:
        xa = snake(ref, a0[:, None]) if act == "snake" else leaky_relu(ref, 0.2)
        h = conv1d(xa, w1, b1, 1, d, pad)
        h = snake(h, a2[:, None]) if act == "snake" else leaky_relu(h, 0.2)
        ref = ref + conv1d(h, w2, b2, 1, 1, (0, 0))
    assert np.isfinite(got).all()
    assert maxabs(got, seq) <= 1e-5 * max(1.0, np.abs(seq).max())
    assert maxabs(got, ref) <= 2e-5 * max(1.0, np.abs(ref).max())
    if precision == "bf16x3":      # fp32-class: the exact three-way split, no ~22-bit operands
        print(f"\n[parity] stack bf16x3 {case}: rel err vs float64 {maxabs(got, ref) / np.abs(ref).max():.2e}")
        assert maxabs(got, ref) <= 2e-6 * max(1.0, np.abs(ref).max())


def test_residual_stack_bf16x3_halo_limit(N, dev):
    """The bf16x3 stack keeps a 24-row plane halo: a unit whose taps reach
    further is refused (RAVE_ERR_UNSUPPORTED), never computed wrong."""
    C, B, T = 64, 1, 256
    x = torch.zeros(B, C, T, device=dev)
    y = torch.zeros_like(x)
    w = torch.from_numpy(N.pack_unit_weight(np.zeros((C, C, 3), np.float32), np.zeros((C, C, 1), np.float32), C,
                                            precision=N.PREC_BF16X3)).to(dev)
    args = N.StackArgs(channels=C, batch=B, t_len=T, act=N.ACT["leaky"], leaky_slope=0.2,
                       precision=N.PREC_BF16X3, x=x.data_ptr(), x_sb=C * T, x_sc=T, y=y.data_ptr(),
                       y_sb=C * T, y_sc=T)
    for u, d in enumerate((1, 3, 13)):
        setattr(args, f"dilation{u}", d)
        setattr(args, f"pad_left{u}", 2 * d)          # causal: 26 > 24 at d = 13
        setattr(args, f"weight{u}", w.data_ptr())
    rc = N.lib.rave_residual_stack(C_.byref(args), C_.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == N.RAVE_ERR_UNSUPPORTED


# ------------------------------------------------------------------ streaming history shift
def _shift_ref(a, hist, t_new):
    """cached_conv's cache update: the newest ``hist`` columns move to the front."""
    out = a.copy()
    out[..., :hist] = a[..., t_new:t_new + hist]
    return out


def test_shift_history_batched(dev, N):
    """rave_shift_history alone and as a run of consecutive plan ops (one
    batched launch of up to 24 buffers, more split over launches): hist below,
    equal to and above t_new (in-place overlap), one-channel rows with long
    histories, padded channel strides, hist 0."""
    rng = np.random.default_rng(7)
    shapes = [(1, 1, 512, 2048), (2, 64, 6, 128), (1, 512, 130, 64), (3, 16, 200, 200),
              (1, 8, 0, 32), (2, 33, 70, 5)]
    shapes = shapes + [(1, 4 + i, 3 + 7 * i, 11 + i) for i in range(26)]
    bufs, refs = [], []
    for (B, Cc, h, t) in shapes:
        a = rng.standard_normal((B, Cc + 1, h + t + 3)).astype(np.float32)  # padded strides
        refs.append(a.copy())
        bufs.append(torch.from_numpy(a).to(dev))
    # single op through the public entry point
    b0 = bufs[2].clone()
    B, Cc, h, t = shapes[2]
    s = N.ShiftArgs(batch=B, channels=Cc, hist=h, t_new=t, buf=b0.data_ptr(),
                    sb=b0.stride(0), sc=b0.stride(1))
    N.check(N.lib.rave_shift_history(C.byref(s), C.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    exp = refs[2].copy()
    exp[:, :Cc] = _shift_ref(refs[2][:, :Cc], h, t)
    assert np.array_equal(b0.cpu().numpy(), exp)
    # all of them as consecutive plan ops
    ops = (N.PlanOp * len(shapes))()
    for i, ((B, Cc, h, t), buf) in enumerate(zip(shapes, bufs)):
        sa = N.ShiftArgs(batch=B, channels=Cc, hist=h, t_new=t, buf=buf.data_ptr(), sb=buf.stride(0),
                         sc=buf.stride(1))
        ops[i].kind = N.OP_SHIFT_HISTORY
        C.memmove(ops[i].raw, C.addressof(sa), C.sizeof(sa))
    hp = C.c_void_p()
    N.check(N.lib.rave_plan_create(ops, len(shapes), None, 0, C.byref(hp)), "plan_create")
    N.check(N.lib.rave_plan_run(hp, None, 0, C.c_void_p(torch.cuda.current_stream().cuda_stream)), "plan_run")
    torch.cuda.synchronize()
    N.lib.rave_plan_destroy(hp)
    for (B, Cc, h, t), buf, r in zip(shapes, bufs, refs):
        exp = r.copy()
        exp[:, :Cc] = _shift_ref(r[:, :Cc], h, t)
        assert np.array_equal(buf.cpu().numpy(), exp), (B, Cc, h, t)


def _rvq_encode_np(z, cbs):
    """float64 RVQ encode (rave/quantization.py:131-140,302-318) with each
    layer's top-2 distance gap, for tie-tolerant index comparison."""
    B, D, T = z.shape
    r = z.transpose(0, 2, 1).reshape(-1, D).astype(np.float64)
    idx, gaps = [], []
    for E in cbs.astype(np.float64):
        d = (E * E).sum(1)[None] - 2.0 * r @ E.T
        o = np.argsort(d, 1, kind="stable")[:, :2]
        i = o[:, 0]
        gaps.append(np.take_along_axis(d, o[:, 1:2], 1)[:, 0] - np.take_along_axis(d, o[:, :1], 1)[:, 0])
        idx.append(i)
        r = r - E[i]
    idx = np.stack(idx, 0).reshape(len(cbs), B, T).transpose(1, 0, 2)
    gaps = np.stack(gaps, 0).reshape(len(cbs), B, T).transpose(1, 0, 2)
    return idx, gaps


@pytest.mark.parametrize("B,D,T,K,nq", [(8, 128, 64, 1024, 16), (3, 64, 37, 1000, 5), (1, 128, 1, 64, 2)])
def test_rvq_encode_sizes_vs_numpy(dev, N, B, D, T, K, nq):
    """The per-layer split RVQ encode at the C4 per-GPU shard (512 frames) and
    at ragged sizes (frames not a multiple of the 32-frame tile, codebook not a
    multiple of the 64-code split, dim 64, one frame): indices equal the float64
    argmin wherever its top-2 gap exceeds the fp32 tie margin; decode of the
    indices equals the sum of the selected codewords."""
    rng = np.random.default_rng(B * 1000 + K)
    cbs = rng.standard_normal((nq, K, D)).astype(np.float32)
    z = rng.standard_normal((B, D, T)).astype(np.float32) * 2.0
    cb = torch.from_numpy(cbs).to(dev)
    zt = torch.from_numpy(z).to(dev)
    idx = torch.full((B, nq, T), -1, dtype=torch.int64, device=dev)
    y = torch.empty(B, D, T, device=dev)
    a = N.RvqArgs(n_q=nq, codebook_size=K, dim=D, batch=B, t_len=T, codebooks=cb.data_ptr(),
                  z=zt.data_ptr(), z_sb=D * T, z_sc=T, idx=idx.data_ptr(), i_sb=nq * T, i_sq=T,
                  y=y.data_ptr(), y_sb=D * T, y_sc=T)
    work = torch.empty(int(N.lib.rave_rvq_workspace(C.byref(a))), device=dev)
    a.work = work.data_ptr()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib.rave_rvq_encode(C.byref(a), st))
    N.check(N.lib.rave_rvq_decode(C.byref(a), st))
    torch.cuda.synchronize()
    got = idx.cpu().numpy()
    assert got.min() >= 0 and got.max() < K
    ref, gap = _rvq_encode_np(z, cbs)
    mism = got != ref
    assert (gap[mism] < 1e-3).all()
    # decode sums the codewords of the returned indices in layer order
    zq = np.zeros((B, T, D), np.float32)
    for q in range(nq):
        zq = zq + cbs[q][got[:, q, :]]
    assert maxabs(y.cpu().numpy(), zq.transpose(0, 2, 1)) < 1e-5


# ------------------------------------------------------------------ nn~ method surface
def test_nn_tilde_surface_streaming_and_stereo(dev):
    """rave_amd.export.NNTildeRAVE (scripts/export.py:298-339): streaming
    encode/decode/forward equal StreamingRAVE block for block; stereo decode
    puts two identical channels side by side; offline encode == RAVE.encode."""
    from rave_amd import config as rcfg
    from rave_amd.export import NNTildeRAVE
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.causal()
    m = RAVE(cfg, init_params(cfg, 5), init_speaker(cfg, 5), device=dev)
    w = NNTildeRAVE(m, stereo=True)
    ref = StreamingRAVE(m, batch=1, block=2048)
    gen = torch.Generator().manual_seed(3)
    for _ in range(4):
        x = (0.2 * torch.randn(1, 1, 2048, generator=gen)).to(dev)
        y = w.forward(x)
        y_ref = ref.forward(x)
        assert tuple(y.shape) == (1, 2, 2048)
        assert torch.equal(y[:, :1], y[:, 1:])                 # L == R bitwise
        # batch 2 vs batch 1 may pick other tiles / K-splits: equal up to summation order
        assert float((y[:, :1] - y_ref).abs().max()) < 1e-6
    cfg2 = rcfg.v2()
    m2 = RAVE(cfg2, init_params(cfg2, 6), init_speaker(cfg2, 6), device=dev)
    w2 = NNTildeRAVE(m2)
    x = (0.2 * torch.randn(2, 1, 8192, generator=gen)).to(dev)
    assert torch.equal(w2.encode(x), m2.encode(x))
    assert w2.get_method_params("encode") == [1, 1, 320, 1024]


def test_nn_tilde_learn_target_drives_adain(dev):
    """nn~'s learn_target / reset_target attributes reach the model's AdaIN
    modules on encode (ScriptedRAVE.update_adain, scripts/export.py:248-265):
    statistics are learned, then a reset clears them once."""
    from rave_amd import config as rcfg
    from rave_amd.export import NNTildeRAVE
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3(capacity=8)
    m = RAVE(cfg, init_params(cfg, 2), init_speaker(cfg, 2), device=dev)
    w = NNTildeRAVE(m)
    x = (0.3 * torch.randn(1, 1, 4096, generator=torch.Generator().manual_seed(1))).to(dev)
    name = m.adain.modules[0][0]
    w.encode(x)
    assert m.adain.state_dict()[f"{name}.num_update_y"][0] == 0
    w.set_learn_target(True)
    w.encode(x)
    w.encode(x)
    sd = m.adain.state_dict()
    assert sd[f"{name}.num_update_y"][0] == 2 and not np.allclose(sd[f"{name}.mean_y"][0], 0)
    w.set_learn_target(False)
    w.set_reset_target(True)
    w.encode(x)
    assert m.adain.state_dict()[f"{name}.num_update_y"][0] == 0 and w.get_reset_target() is False


def _stream_conv_cases(cfg):
    """(node, t_src, extra history) of every conv of a causal graph at a 2048-sample
    block, with the operand views the streaming engine gives it: x starts
    `need` columns before the block inside a [history | block] row, row widths
    not a multiple of 4 (the unaligned window-DMA path)."""
    from rave_amd.graph import build_graph
    g = build_graph(cfg)
    t = {"enc_in": 2048 // cfg.n_band, "dec_in": 2048 // cfg.hop}
    out = []
    for n in g.encoder + g.decoder + g.noise:
        ts = t[n.src]
        t[n.dst] = ts * n.stride if n.transposed else ts // n.stride
        out.append((n, ts))
    return out


@pytest.mark.parametrize("capacity", [8, 16, 64])
def test_stream_conv_shapes_split16_vs_f32(N, dev, capacity):
    """Every streaming conv shape of a causal v3+noise graph: split-f16 ==
    exact fp32 (layer tolerance), with the cached views (history offset, odd
    row widths, the cached ConvTranspose form with one history column)."""
    from rave_amd import config as rcfg
    cfg = rcfg.v3_noise(causal=True, capacity=capacity)
    rng = np.random.default_rng(capacity)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for n, ts in _stream_conv_cases(cfg):
        need = 1 if n.transposed else n.pad[0]
        h = need + 3                                   # history columns in the row
        width = h + ts
        t_in = need + ts
        t_out = ts * n.stride if n.transposed else ts // n.stride
        B = 2
        xbuf = torch.from_numpy(rng.standard_normal((B, n.c_in, width)).astype(np.float32)).to(dev)
        wshape = (n.c_in, n.c_out, n.kernel) if n.transposed else (n.c_out, n.c_in, n.kernel)
        w = (rng.uniform(-1, 1, wshape) / np.sqrt(n.c_in * n.kernel)).astype(np.float32)
        bias = torch.from_numpy(rng.uniform(-0.1, 0.1, n.c_out).astype(np.float32)).to(dev)
        alpha = torch.from_numpy((1 + 0.1 * rng.standard_normal(n.c_in)).astype(np.float32)).to(dev)
        outs = []
        for prec in (N.PREC_F32, N.PREC_SPLIT16):
            packed = torch.from_numpy(N.pack_conv_weight(w, n.c_in, n.c_out, n.kernel, n.stride, n.dilation,
                                                         n.transposed, out_shift=0, precision=prec)).to(dev)
            y = torch.full((B, n.c_out, t_out + 5), float("nan"), device=dev)
            a = N.ConvArgs(c_in=n.c_in, c_out=n.c_out, kernel=n.kernel, stride=n.stride, dilation=n.dilation,
                           pad_left=1 if n.transposed else 0, pad_right=0, transposed=int(n.transposed),
                           out_shift=0, act=N.ACT[n.act], leaky_slope=0.2, batch=B, t_in=t_in, t_out=t_out,
                           precision=prec, x=xbuf.data_ptr() + 4 * (h - need), x_sb=n.c_in * width, x_sc=width,
                           y=y.data_ptr(), y_sb=n.c_out * (t_out + 5), y_sc=t_out + 5,
                           weight=packed.data_ptr(), bias=bias.data_ptr() if n.bias else None,
                           alpha=alpha.data_ptr() if n.act == "snake" else None)
            nws = int(N.lib.rave_conv1d_workspace(C.byref(a)))
            ws = torch.zeros(max(nws, 1), device=dev)
            a.partial = ws.data_ptr() if nws > 0 else None
            N.check(N.lib.rave_conv1d(C.byref(a), st), n.name)
            torch.cuda.synchronize()
            outs.append(y[..., :t_out].cpu().numpy())
            assert torch.isnan(y[..., t_out:]).all(), n.name           # nothing written past t_out
        ref = outs[0]
        assert np.isfinite(ref).all(), n.name
        err = maxabs(outs[1], ref)
        assert err <= 2e-5 * max(1.0, np.abs(ref).max()), (n.name, n.c_in, n.c_out, n.kernel, ts, err)


# ------------------------------------------------------------------ TorchScript (nn~) export
@pytest.mark.parametrize("precision", ["f32", "f32_bf3"])
def test_scripted_export_roundtrip_golden(dev, golden, tmp_path, precision):
    """ScriptedRAVE -> torch.jit.script -> save -> torch.jit.load (what nn~
    does with the .ts, scripts/export.py:618): the loaded module's encode /
    decode match the reference fixtures and its nn~ metadata is intact."""
    from rave_amd import config as rcfg
    from rave_amd.scripted import ScriptedRAVE
    from rave_amd.weights import init_params
    g = golden("v2")
    cfg = rcfg.v2()
    m = ScriptedRAVE(cfg, init_params(cfg, seed=int(g["seed"])), g["speaker"], hk=_golden_hk(golden),
                     precision=precision)
    path = str(tmp_path / "rave_v2.ts")
    m.export_to_ts(path)
    ts = torch.jit.load(path)
    assert ts.get_methods() == ["encode", "decode", "forward"]
    assert ts.get_method_params("encode") == [1, 1, 320, 1024]
    assert ts.set_speaker(3) == 0 and ts.get_speaker() == 3
    z = ts.encode(torch.from_numpy(g["x"]).to(dev))
    y = ts.decode(torch.from_numpy(g["z"]).to(dev))
    torch.cuda.synchronize()
    assert maxabs(z.cpu().numpy()[:, :64], g["z"][:, :64]) < TOL
    assert maxabs(y.cpu().numpy(), g["y"]) < TOL


def test_scripted_streaming_matches_streaming_rave(dev):
    """A scripted causal model streams block by block through the engine's
    hipGraph streams: equal to rave_amd.StreamingRAVE; a 2-block buffer is
    split into blocks."""
    from rave_amd import config as rcfg
    from rave_amd.scripted import ScriptedRAVE
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.causal()
    p, spk = init_params(cfg, 7), init_speaker(cfg, 7)
    ts = torch.jit.script(ScriptedRAVE(cfg, p, spk, block=2048))
    ref = StreamingRAVE(RAVE(cfg, p, spk, device=dev), batch=1, block=2048)
    gen = torch.Generator().manual_seed(4)
    x = (0.2 * torch.randn(1, 1, 3 * 4096, generator=gen)).to(dev)
    for i in range(3):
        xi = x[..., i * 4096:(i + 1) * 4096]
        y = ts.forward(xi)
        y_ref = torch.cat([ref.forward(xi[..., :2048].contiguous()), ref.forward(xi[..., 2048:].contiguous())], -1)
        torch.cuda.synchronize()
        assert float((y - y_ref).abs().max()) < 1e-6


def test_scripted_adain_attributes(dev):
    """set_learn_target on the scripted module drives the engine's AdaIN (the
    output changes once target statistics exist and transfer is on)."""
    from rave_amd import config as rcfg
    from rave_amd.scripted import ScriptedRAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v3(capacity=8)
    ts = torch.jit.script(ScriptedRAVE(cfg, init_params(cfg, 1), init_speaker(cfg, 1)))
    gen = torch.Generator().manual_seed(8)
    x_tgt = (0.5 * torch.randn(1, 1, 4096, generator=gen)).to(dev)
    x = (0.2 * torch.randn(1, 1, 4096, generator=gen)).to(dev)
    y0 = ts.forward(x)
    ts.set_learn_target(True)
    ts.encode(x_tgt)
    ts.set_learn_target(False)
    ts.set_learn_source(True)
    ts.encode(x)
    ts.set_learn_source(False)
    y1 = ts.forward(x)
    torch.cuda.synchronize()
    assert float((y1 - y0).abs().max()) > 1e-3
    ts.set_reset_target(True)
    ts.set_reset_source(True)
    ts.encode(x)
    assert ts.get_reset_target() is False
    y2 = ts.forward(x)
    torch.cuda.synchronize()
    assert float((y2 - y0).abs().max()) < 1e-6
