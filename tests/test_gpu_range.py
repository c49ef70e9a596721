"""Split-f16 range guard (rave_amd/csrc/common.h "range guard").

RAVE_PREC_SPLIT16 carries an fp32 operand as an f16 pair, which holds
|v| < 2^15 only.  Every split kernel converts optimistically and votes per
wave; a staged operand block that reaches 2^15 is re-converted as v * 2^-s and
the GEMM result takes the exact 2^s back.  These tests drive activations far
past f16's 65504 -- scaled inputs, scaled weights, overflow in some K-chunks
only, at a fused unit's seam only -- and check the split16 kernels against the
float64 oracle at the layer tolerance (2e-5 of max |ref|, as the in-range
tests), never inf; and at model level, a v2 model whose interior activations
exceed 65504 everywhere matches the oracle within the north star's 1e-4 in
split16 and auto.  Runs on an MI355X only (``-m gpu``)."""
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


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


# ------------------------------------------------------------------ conv
RANGE_CONV_CASES = [
    # c_in, c_out, k, s, d, transposed, act, residual, B, T, which channels are blown up
    (64, 64, 3, 1, 1, 0, "leaky", False, 2, 300, "all"),
    (128, 128, 1, 1, 1, 0, "leaky", True, 2, 257, "some"),
    (512, 512, 3, 1, 3, 0, "leaky", False, 16, 128, "some"),
    (64, 128, 8, 4, 1, 0, "leaky", False, 2, 1024, "all"),
    (1024, 512, 4, 2, 1, 1, "leaky", False, 2, 8, "some"),
    (256, 512, 4, 2, 1, 0, "snake", False, 2, 64, "some"),
    (64, 32, 7, 1, 1, 0, "snake", False, 2, 4096, "all"),
    (256, 256, 3, 1, 9, 0, "leaky", True, 2, 300, "mid"),
]


@pytest.mark.parametrize("case", RANGE_CONV_CASES, ids=[str(c) for c in RANGE_CONV_CASES])
def test_conv_range_guard(N, dev, case):
    """rave_conv1d in split16 with inputs up to 3e6: every chunk (all) or a few
    K-chunks only (some: the per-chunk rescue runs next to unscaled chunks)."""
    from oracle.rave_oracle import conv1d, conv_transpose1d, leaky_relu, snake
    from tests.test_gpu_parity import run_conv
    c_in, c_out, k, s, d, transposed, act, has_res, B, T, which = case
    rng = np.random.default_rng(c_in * 7 + k)
    x = rng.standard_normal((B, c_in, T)).astype(np.float32)
    if which == "all":
        x *= 3e6
    elif which == "mid":
        # |act| in [2^15, 65504]: no f16 overflow, so no second attempt; the
        # split itself must stay exact to ~2^-22 there
        x = rng.uniform(-65000, 65000, x.shape).astype(np.float32)
    else:
        x[:, c_in // 3:c_in // 3 + 5] *= 3e6
    bound = 1 / np.sqrt(c_in * k)
    wshape = (c_in, c_out, k) if transposed else (c_out, c_in, k)
    w = rng.uniform(-bound, bound, wshape).astype(np.float32)
    b = rng.uniform(-bound, bound, c_out).astype(np.float32)
    alpha = (1 + 0.1 * rng.standard_normal((c_in, 1))).astype(np.float32) if act == "snake" else None
    xa = x.astype(np.float64)
    xa = leaky_relu(xa) if act == "leaky" else snake(xa, alpha)
    if transposed:
        ref = conv_transpose1d(xa, w, s, s // 2, b)
        pad = (0, 0)
    else:
        p = (k - 1) * d + 1
        pad = ((p - 1) // 2, p // 2)
        ref = conv1d(xa, w, b, s, d, pad)
    res = (1e5 * rng.standard_normal(ref.shape)).astype(np.float32) if has_res else None
    if has_res:
        ref = ref + res
    got = run_conv(N, dev, x, w, b, alpha.reshape(-1) if alpha is not None else None, res, c_in, c_out, k, s, d,
                   pad, transposed, act, precision=N.PREC_SPLIT16)
    assert np.isfinite(got).all()
    err = maxabs(got, ref)
    assert err <= 2e-5 * float(np.abs(ref).max()), err


def test_conv_range_guard_every_config(N, dev):
    """Every launch configuration the autotuner may pick keeps the guard (tile
    shapes, K-groups, wide chunks, split-K slabs and their combine)."""
    from oracle.rave_oracle import conv1d, leaky_relu
    c_in, c_out, k, d, B, T = 512, 512, 3, 1, 16, 128
    rng = np.random.default_rng(5)
    x = rng.standard_normal((B, c_in, T)).astype(np.float32)
    x[:, 200:210] *= 1e6
    w = (rng.uniform(-1, 1, (c_out, c_in, k)) / np.sqrt(c_in * k)).astype(np.float32)
    b = (0.1 * rng.standard_normal(c_out)).astype(np.float32)
    ref = conv1d(leaky_relu(x.astype(np.float64)), w, b, 1, d, (1, 1))
    from tests.test_gpu_parity import run_conv
    a = N.ConvArgs(c_in=c_in, c_out=c_out, kernel=k, stride=1, dilation=d, pad_left=1, pad_right=1, act=N.ACT["leaky"],
                   leaky_slope=0.2, batch=B, t_in=T, t_out=T, precision=N.PREC_SPLIT16, x=16, y=16, weight=16)
    cfgs = N.conv_configs(a)
    assert cfgs
    for cfg in cfgs:
        got = run_conv(N, dev, x, w, b, None, None, c_in, c_out, k, 1, d, (1, 1), 0, "leaky",
                       precision=N.PREC_SPLIT16, config=cfg)
        assert np.isfinite(got).all(), cfg
        assert maxabs(got, ref) <= 2e-5 * float(np.abs(ref).max()), cfg


# ------------------------------------------------------------------ fused unit / stack
def _unit_ref(x, w1, w2, b1, b2, d, pad):
    from oracle.rave_oracle import conv1d, leaky_relu
    h = leaky_relu(conv1d(leaky_relu(x.astype(np.float64), 0.2), w1, b1, 1, d, pad), 0.2)
    return x + conv1d(h, w2, b2, 1, 1, (0, 0))


@pytest.mark.parametrize("C_,where,coop", [(64, "input", False), (128, "seam", False), (256, "input", False),
                                           (512, "seam", False), (256, "input", True), (512, "seam", True),
                                           (256, "seam_one", True), (512, "seam_one", True)])
def test_unit_range_guard(N, dev, C_, where, coop):
    """rave_residual_unit (split16): the act0(x) window past f16 (input), or
    in-range input whose k3 output h is (the seam's own guard); cooperative
    form (rave_unit_workspace): h past f16 in every member, or only in the rows
    of one member (seam_one: the group-wide guard)."""
    d, B, T = 3, 2, 200
    rng = np.random.default_rng(C_)
    x = rng.standard_normal((B, C_, T)).astype(np.float32)
    w1 = (rng.standard_normal((C_, C_, 3)) / np.sqrt(3 * C_)).astype(np.float32)
    w2 = (rng.standard_normal((C_, C_, 1)) / np.sqrt(C_)).astype(np.float32)
    if where == "input":
        x *= 1e6
    elif where == "seam_one":
        w1[:128] *= 1e6                   # rows of the group's first member only
        w2 *= 1e-3
    else:
        w1 *= 1e6
        w2 *= 1e-3
    b1 = (0.1 * rng.standard_normal(C_)).astype(np.float32)
    b2 = (0.1 * rng.standard_normal(C_)).astype(np.float32)
    ref = _unit_ref(x, w1, w2, b1, b2, d, (d, d))
    packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C_, precision=N.PREC_SPLIT16)).to(dev)
    xd = torch.from_numpy(x).to(dev)
    y = torch.full_like(xd, float("nan"))
    bd1, bd2 = torch.from_numpy(b1).to(dev), torch.from_numpy(b2).to(dev)
    a = N.UnitArgs(channels=C_, batch=B, t_len=T, dilation=d, pad_left=d, act=N.ACT["leaky"], leaky_slope=0.2,
                   precision=N.PREC_SPLIT16, x=xd.data_ptr(), x_sb=C_ * T, x_sc=T, y=y.data_ptr(), y_sb=C_ * T,
                   y_sc=T, weight=packed.data_ptr(), bias1=bd1.data_ptr(), bias2=bd2.data_ptr())
    ws = None
    if coop:
        nws = N.lib.rave_unit_workspace(C.byref(a))
        assert nws > 0
        ws = torch.zeros(nws, device=dev)
        a.workspace = ws.data_ptr()
    N.check(N.lib.rave_residual_unit(C.byref(a), _stream()))
    torch.cuda.synchronize()
    if coop:
        assert int(torch.count_nonzero(ws[:N.SPLITK_TICKETS])) == 0
    got = y.cpu().numpy()
    assert np.isfinite(got).all()
    err = maxabs(got, ref)
    assert err <= 2e-5 * float(np.abs(ref).max()), err


@pytest.mark.parametrize("C_,where", [(64, "input"), (64, "seam"), (128, "between")])
def test_stack_range_guard(N, dev, C_, where):
    """rave_residual_stack (split16): overflow in the unit-0 window, at the
    seams, or only in the running sum between units."""
    dils = (1, 3, 9)
    B, T = 2, 700
    rng = np.random.default_rng(C_ + len(where))
    x = rng.standard_normal((B, C_, T)).astype(np.float32)
    if where == "input":
        x *= 1e6
    args = N.StackArgs(channels=C_, batch=B, t_len=T, act=N.ACT["leaky"], leaky_slope=0.2)
    keep, units = [], []
    for u, d in enumerate(dils):
        w1 = (rng.standard_normal((C_, C_, 3)) / np.sqrt(3 * C_)).astype(np.float32)
        w2 = (rng.standard_normal((C_, C_, 1)) / np.sqrt(C_)).astype(np.float32)
        if where == "seam":
            w1 *= 1e6
            w2 *= 1e-6
        if where == "between" and u == 0:
            w2 *= 1e7                      # unit 0's output (unit 1's input) leaves f16's range
        b1 = (0.1 * rng.standard_normal(C_)).astype(np.float32)
        b2 = (0.1 * rng.standard_normal(C_)).astype(np.float32)
        units.append((w1, w2, b1, b2, d))
        tens = [torch.from_numpy(N.pack_unit_weight(w1, w2, C_, precision=N.PREC_SPLIT16)).to(dev),
                torch.from_numpy(b1).to(dev), torch.from_numpy(b2).to(dev)]
        keep += tens
        setattr(args, f"dilation{u}", d)
        setattr(args, f"pad_left{u}", d)
        for f, t in zip(("weight", "bias1", "bias2"), tens):
            setattr(args, f"{f}{u}", t.data_ptr())
    xd = torch.from_numpy(x).to(dev)
    y = torch.full_like(xd, float("nan"))
    args.x, args.x_sb, args.x_sc = xd.data_ptr(), C_ * T, T
    args.y, args.y_sb, args.y_sc = y.data_ptr(), C_ * T, T
    N.check(N.lib.rave_residual_stack(C.byref(args), _stream()), "residual_stack")
    torch.cuda.synchronize()
    ref = x.astype(np.float64)
    for w1, w2, b1, b2, d in units:
        ref = _unit_ref(ref, w1, w2, b1, b2, d, (d, d))
    got = y.cpu().numpy()
    assert np.isfinite(got).all()
    err = maxabs(got, ref)
    assert err <= 2e-5 * float(np.abs(ref).max()), err


# ------------------------------------------------------------------ PQMF
def test_pqmf_range_guard(N, dev, golden):
    """Analysis of audio at 3e6 and plain synthesis of bands at 3e6 (split16)
    against the exact-fp32 kernels."""
    from rave_amd.pqmf import kernels
    hkf, hki = kernels(golden("pqmf")["hk"])
    hkf_d, hki_d = torch.from_numpy(hkf).to(dev), torch.from_numpy(hki).to(dev)
    g = torch.Generator().manual_seed(9)
    B, Fr = 2, 512
    T = Fr * 16
    x = (3e6 * torch.randn(B, 1, T, generator=g)).to(dev)
    z = (3e6 * torch.randn(B, 16, Fr, generator=g)).to(dev)
    outs_a, outs_s = [], []
    for prec in (N.PREC_F32, N.PREC_SPLIT16):
        ya = torch.empty(B, 16, Fr, device=dev)
        a = N.AnalysisArgs(n_band=16, taps=hkf.shape[-1], n_out_bands=16, batch=B, t_in=T, pad_left=256, t_out=Fr,
                           x=x.data_ptr(), x_sb=T, y=ya.data_ptr(), y_sb=16 * Fr, y_sc=Fr, hkf=hkf_d.data_ptr(),
                           precision=prec)
        N.check(N.lib.rave_pqmf_analysis(C.byref(a), _stream()))
        ys = torch.empty(B, 1, T, device=dev)
        s_ = N.SynthesisArgs(n_band=16, taps=hki.shape[-1], batch=B, t_in=Fr, pad_left=16, mode=0, frame0=0,
                             x_len=0, x=z.data_ptr(), x_sb=16 * Fr, x_sc=Fr, y=ys.data_ptr(), y_sb=T,
                             hki=hki_d.data_ptr(), precision=prec)
        N.check(N.lib.rave_pqmf_synthesis(C.byref(s_), _stream()))
        outs_a.append(ya)
        outs_s.append(ys)
    torch.cuda.synchronize()
    for ref, got in ((outs_a[0], outs_a[1]), (outs_s[0], outs_s[1])):
        ref, got = ref.cpu().numpy(), got.cpu().numpy()
        assert np.isfinite(got).all()
        assert maxabs(got, ref) <= 2e-6 * float(np.abs(ref).max())


# ------------------------------------------------------------------ model
@pytest.mark.parametrize("precision", ["split16", "auto"])
def test_model_range_guard_vs_oracle(dev, precision):
    """A v2 model driven past f16's range inside: audio at 1e6 scale (the PQMF
    input and every encoder activation far past 65504) with the encoder's last
    conv scaled down by 1e-6, and latents at 1e6 (every decoder activation past
    65504) with the waveform conv scaled down by 1e-6, so z and y are O(1)
    again.  The
    split16 / auto plans match the float64 oracle within 1e-4 and stay finite,
    as the exact-fp32 plan does."""
    from oracle.rave_oracle import Oracle
    from rave_amd import config as rcfg
    from rave_amd.graph import build_graph
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2()
    params, spk = init_params(cfg, 0), init_speaker(cfg, 0)
    g = build_graph(cfg)
    params = dict(params)
    for name in (g.encoder[-1].name, g.decoder[-1].name):
        params[name + ".weight_g"] = (params[name + ".weight_g"] * np.float32(1e-6)).astype(np.float32)
    T = 16384
    n = np.arange(T)
    x = (1e6 * (0.3 * np.sin(2 * np.pi * 440 * n / 48000)
                + 0.1 * np.random.default_rng(0).standard_normal(T))).astype(np.float32)[None, None]
    zin = (1e6 * np.random.default_rng(1).standard_normal((1, cfg.dec_in, T // cfg.hop))).astype(np.float32)
    m = RAVE(cfg, params, spk, device=dev, precision=precision)
    z = m.encode(torch.from_numpy(x).to(dev)).cpu().numpy()
    y = m.decode(torch.from_numpy(zin).to(dev)).cpu().numpy()
    mf = RAVE(cfg, params, spk, device=dev, precision="f32")
    zf = mf.encode(torch.from_numpy(x).to(dev)).cpu().numpy()
    yf = mf.decode(torch.from_numpy(zin).to(dev)).cpu().numpy()
    o = Oracle(cfg, params, spk, hk=m.hk)
    zr, yr = o.encode(x), o.decode(zin)
    assert np.isfinite(z).all() and np.isfinite(y).all()
    ez, ey = maxabs(z, zr), maxabs(y, yr)
    print(f"\n[range] v2 {precision}: |z| max {np.abs(zr).max():.2f}, z err {ez:.3e} (f32 {maxabs(zf, zr):.3e}); "
          f"y err {ey:.3e} (f32 {maxabs(yf, yr):.3e})")
    assert ez < 1e-4 and ey < 1e-4


# ------------------------------------------------------------------ bf16x3: no guard needed
@pytest.mark.parametrize("scale", [3e6, 1e-20])
@pytest.mark.parametrize("C_", [64, 256, 512])
def test_unit_bf16x3_wide_range(N, dev, C_, scale):
    """rave_residual_unit in bf16x3: the three bf16 parts keep fp32's exponent
    range, so operands far past f16's (3e6) or far below it (1e-20) need no
    range guard and stay fp32-exact relative to the output scale."""
    d, B, T = 3, 2, 200
    rng = np.random.default_rng(C_ + 11)
    x = (scale * rng.standard_normal((B, C_, T))).astype(np.float32)
    w1 = (rng.standard_normal((C_, C_, 3)) / np.sqrt(3 * C_)).astype(np.float32)
    w2 = (rng.standard_normal((C_, C_, 1)) / np.sqrt(C_)).astype(np.float32)
    b1 = (0.1 * scale * rng.standard_normal(C_)).astype(np.float32)
    b2 = (0.1 * scale * rng.standard_normal(C_)).astype(np.float32)
    ref = _unit_ref(x, w1, w2, b1, b2, d, (d, d))
    packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C_, precision=N.PREC_BF16X3)).to(dev)
    xd = torch.from_numpy(x).to(dev)
    y = torch.full_like(xd, float("nan"))
    bd1, bd2 = torch.from_numpy(b1).to(dev), torch.from_numpy(b2).to(dev)
    a = N.UnitArgs(channels=C_, batch=B, t_len=T, dilation=d, pad_left=d, act=N.ACT["leaky"], leaky_slope=0.2,
                   precision=N.PREC_BF16X3, x=xd.data_ptr(), x_sb=C_ * T, x_sc=T, y=y.data_ptr(), y_sb=C_ * T,
                   y_sc=T, weight=packed.data_ptr(), bias1=bd1.data_ptr(), bias2=bd2.data_ptr())
    N.check(N.lib.rave_residual_unit(C.byref(a), _stream()))
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    assert np.isfinite(got).all()
    assert maxabs(got, ref) <= 2e-6 * float(np.abs(ref).max())


@pytest.mark.parametrize("scale", [3e6, 1e-20])
def test_conv_bf16x3_wide_range(N, dev, scale):
    """rave_conv1d in bf16x3 far outside f16's range (no guard pass exists)."""
    from oracle.rave_oracle import conv1d, leaky_relu
    from tests.test_gpu_parity import run_conv
    c_in, c_out, k, d, B, T = 256, 512, 4, 1, 4, 64
    rng = np.random.default_rng(3)
    x = (scale * rng.standard_normal((B, c_in, T))).astype(np.float32)
    bound = 1 / np.sqrt(c_in * k)
    w = rng.uniform(-bound, bound, (c_out, c_in, k)).astype(np.float32)
    b = (scale * rng.uniform(-bound, bound, c_out)).astype(np.float32)
    ref = conv1d(leaky_relu(x.astype(np.float64)), w, b, 2, d, (1, 1))
    got = run_conv(N, dev, x, w, b, None, None, c_in, c_out, k, 2, d, (1, 1), 0, "leaky", precision=N.PREC_BF16X3)
    assert np.isfinite(got).all()
    assert maxabs(got, ref) <= 2e-6 * float(np.abs(ref).max())
