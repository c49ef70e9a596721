"""CPU-side checks of the C-ABI library: it loads, exports every symbol that
include/rave_amd.h declares, its struct layouts match the ctypes mirrors, the
host-side weight packer lays weights out as the kernels read them, and argument
validation maps to Python exceptions (no GPU needed: nothing here launches)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from oracle.rave_oracle import conv1d, conv_transpose1d
from rave_amd import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "rave_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rave_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_header_symbol():
    names = header_functions()
    assert len(names) >= 15
    for name in names:
        assert hasattr(N.lib, name), name
    assert sorted(N.EXPORTS) == names


def test_struct_sizes_match():
    n = N.lib.rave_struct_sizes(None, 0)
    buf = (C.c_int64 * n)()
    N.lib.rave_struct_sizes(buf, n)
    assert list(buf) == [C.sizeof(s) for s in N.STRUCTS]
    assert C.sizeof(N.PlanOp) == 248


def _emulate_packed_conv(packed, x, c_in, c_out, k, s, d, pad, transposed, out_shift=None):
    """Run the GEMM the kernel runs, from the packed layout (kk = tap*CI_T + ci).
    ConvTranspose: rows [0, split) are phases q < r-P with window offset -1,
    rows [split, M) phases q >= r-P with offset 0; output t = u*r + q."""
    ci_t = N.conv_chunk(c_in, k, s, d, transposed)
    taps = 2 if transposed else k
    R = s if transposed else 1
    P = R // 2 if out_shift is None else out_shift
    q0 = R - P
    # group 1 starts on a 64-row tile boundary (rows in between are padding)
    split = c_out * q0 if (not transposed or q0 == R) else -(-c_out * q0 // 64) * 64
    M = split + c_out * (R - q0) if transposed else c_out
    Mpad = -(-M // 128) * 128
    nch = -(-c_in // ci_t)
    W = packed.reshape(nch, taps, ci_t, Mpad)[..., :M]
    xc = np.pad(x.astype(np.float64), ((0, 0), (0, nch * ci_t - c_in), (0, 0)))
    B, _, T = x.shape
    if not transposed:
        xp = np.pad(xc, ((0, 0), (0, 0), pad))
        U = (xp.shape[-1] - ((taps - 1) * d + 1)) // s + 1
        y = np.zeros((B, M, U))
        for c in range(nch):
            for j in range(taps):
                xs = xp[:, c * ci_t:(c + 1) * ci_t, j * d: j * d + (U - 1) * s + 1: s]
                y += np.einsum("im,bin->bmn", W[c, j], xs)
        return y
    xp = np.pad(xc, ((0, 0), (0, 0), (1, 1)))        # x[-1] and x[T] are zero
    out = np.zeros((B, c_out, T * R))
    for m in range(M):
        if m < split:
            co, q, off = m // q0, m % q0, -1
            if co >= c_out:
                assert not W[..., m].any()           # padding rows are zero
                continue
        else:
            co, q, off = (m - split) // (R - q0), q0 + (m - split) % (R - q0), 0
        acc = np.zeros((B, T))
        for c in range(nch):
            for j in range(taps):
                xs = xp[:, c * ci_t:(c + 1) * ci_t, 1 + off + j: 1 + off + j + T]
                acc += np.einsum("i,bit->bt", W[c, j, :, m], xs)
        out[:, co, q::R] = acc
    return out


@pytest.mark.parametrize("c_in,c_out,k,s,d,transposed", [
    (64, 64, 3, 1, 9, 0), (64, 64, 1, 1, 1, 0), (6, 64, 7, 1, 1, 0), (64, 128, 8, 4, 1, 0),
    (256, 512, 4, 2, 1, 0), (320, 1024, 3, 1, 1, 0), (64, 32, 7, 1, 1, 0), (96, 96, 3, 1, 3, 0),
    (64, 48, 4, 2, 1, 1), (32, 16, 8, 4, 1, 1), (96, 40, 4, 2, 1, 1)])
def test_pack_layout(c_in, c_out, k, s, d, transposed):
    rng = np.random.default_rng(1)
    T = 40
    x = rng.standard_normal((2, c_in, T)).astype(np.float32)
    if transposed:
        w = rng.standard_normal((c_in, c_out, k)).astype(np.float32)
        ref = conv_transpose1d(x, w, s, s // 2)
        pad = (0, 0)
    else:
        w = rng.standard_normal((c_out, c_in, k)).astype(np.float32)
        p = (k - 1) * d + 1
        pad = ((p - 1) // 2, p // 2)
        ref = conv1d(x, w, None, s, d, pad)
    packed = N.pack_conv_weight(w, c_in, c_out, k, s, d, transposed)
    got = _emulate_packed_conv(packed, x, c_in, c_out, k, s, d, pad, transposed)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() < 1e-9 * max(1, np.abs(ref).max()) * 1e4


def test_validation_errors():
    a = N.ConvArgs()
    with pytest.raises(ValueError):
        N.check(N.lib.rave_conv1d(C.byref(a), None), "conv1d")
    with pytest.raises(NotImplementedError):
        N.pack_conv_weight(np.zeros((4, 4, 3), np.float32), 4, 4, 3, 2, 1, 1)  # transposed needs k == 2s
    with pytest.raises(NotImplementedError):
        N.pack_conv_weight(np.zeros((4, 4, 5), np.float32), 4, 4, 5, 1, 1, 0)  # no 5-tap family
    # workspace query validates like the launcher
    a = N.ConvArgs(c_in=64, c_out=64, kernel=3, stride=1, dilation=1, pad_left=1, pad_right=1,
                   batch=1, t_in=100, t_out=99, x=16, y=16, weight=16)
    assert N.lib.rave_conv1d_workspace(C.byref(a)) == -1   # t_out inconsistent
    a.t_out = 100
    assert N.lib.rave_conv1d_workspace(C.byref(a)) >= 0


@pytest.mark.parametrize("precision", [0, 1])
def test_conv_configs_listing(precision):
    """rave_conv1d_configs lists configurations the launcher accepts (host-side
    validation only: the workspace query resolves each), and rejects others."""
    a = N.ConvArgs(c_in=128, c_out=128, kernel=3, stride=1, dilation=3, pad_left=3, pad_right=3,
                   batch=16, t_in=1024, t_out=1024, precision=precision, x=16, y=16, weight=16)
    cfgs = N.conv_configs(a)
    assert len(cfgs) >= 4 and 0 not in cfgs and len(set(cfgs)) == len(cfgs)
    for c in cfgs:
        a.config = c
        assert N.lib.rave_conv1d_workspace(C.byref(a)) >= 0
    a.config = 1 + 16 * 30    # 31 K-splits: more than the layer has chunks
    assert N.lib.rave_conv1d_workspace(C.byref(a)) == -1
    a.config = -3
    assert N.lib.rave_conv1d_workspace(C.byref(a)) == -1


def test_conv_f32_inlaunch_configs():
    """Exact-fp32 MFMA tiles (0..4) with K splits are listed twice (round 6): the
    separate reduce launch and, bit 9 set, the in-launch combine; the launcher
    accepts both and refuses the in-launch bit without K splits."""
    a = N.ConvArgs(c_in=512, c_out=512, kernel=3, stride=1, dilation=1, pad_left=1, pad_right=1,
                   batch=1, t_in=64, t_out=64, precision=N.PREC_F32, x=16, y=16, weight=16)
    cfgs = N.conv_configs(a)
    tile = lambda c: (c - 1) & 15
    splits = lambda c: ((c - 1) >> 4 & 31) + 1
    inl = [c for c in cfgs if tile(c) < 5 and ((c - 1) >> 9) & 1]
    assert inl and all(splits(c) > 1 and c - 512 in cfgs for c in inl)
    for c in inl:
        a.config = c
        assert N.lib.rave_conv1d_workspace(C.byref(a)) > 0
    a.config = 1 + 4 + 512        # 64 x 64 tile, one K split, in-launch bit: nothing to combine
    assert N.lib.rave_conv1d_workspace(C.byref(a)) == -1


def test_conv_gemv_rows_configs():
    """The row-sliced skinny-N form (tiles 14 / 15, round 6: 8, 16 or 32 rows
    per workgroup over the whole K, one launch) is listed for up to 32 output
    columns, with one K split only."""
    def args(T, c_in=512):
        return N.ConvArgs(c_in=c_in, c_out=512, kernel=3, stride=1, dilation=1, pad_left=2, pad_right=0,
                          batch=1, t_in=T, t_out=T, precision=N.PREC_F32, x=16, y=16, weight=16)
    rows = lambda a: [c for c in N.conv_configs(a) if (c - 1) & 15 >= 14]
    a = args(8)
    assert sorted(rows(a)) == [15, 16, 15 + 512]                 # 16, 8 and 32 rows per workgroup
    for c in rows(a):
        a.config = c
        assert N.lib.rave_conv1d_workspace(C.byref(a)) == 0      # nothing to combine
    a.config = 15 + 16                                            # two K splits: refused
    assert N.lib.rave_conv1d_workspace(C.byref(a)) == -1
    a.config = 16 + 512                                           # tile 15 has no bit-9 form
    assert N.lib.rave_conv1d_workspace(C.byref(a)) == -1
    assert not rows(args(33))                                     # more columns than the form holds
    assert not rows(args(32, c_in=4096))                          # window beyond the staging area


def test_plan_create_and_relocation_bounds():
    ops = (N.PlanOp * 1)()
    ops[0].kind = N.OP_FILL
    good = (N.Reloc * 1)(N.Reloc(0, N.FillArgs.y.offset, 0, 0, 0))
    h = C.c_void_p()
    N.check(N.lib.rave_plan_create(ops, 1, good, 1, C.byref(h)), "plan_create")
    assert N.lib.rave_plan_size(h) == 1
    # unbound slot is reported before anything is launched
    with pytest.raises(ValueError):
        N.check(N.lib.rave_plan_run(h, None, 0, None), "plan_run")
    N.lib.rave_plan_destroy(h)
    bad = (N.Reloc * 1)(N.Reloc(0, 4, 0, 0, 0))   # misaligned pointer field
    with pytest.raises(ValueError):
        N.check(N.lib.rave_plan_create(ops, 1, bad, 1, C.byref(h)), "plan_create")


@pytest.mark.parametrize("c_in,c_out,r", [(64, 32, 2), (32, 16, 4)])
def test_pack_layout_transposed_cached_form(c_in, c_out, r):
    """out_shift = 0 (cached_conv's overlap-add form): output = the uncropped
    transposed conv's first T*r samples (cache = zeros)."""
    rng = np.random.default_rng(2)
    T = 20
    x = rng.standard_normal((2, c_in, T)).astype(np.float32)
    w = rng.standard_normal((c_in, c_out, 2 * r)).astype(np.float32)
    ref = conv_transpose1d(x, w, r, 0)[..., :T * r]
    packed = N.pack_conv_weight(w, c_in, c_out, 2 * r, r, 1, 1, out_shift=0)
    got = _emulate_packed_conv(packed, x, c_in, c_out, 2 * r, r, 1, (0, 0), 1, out_shift=0)
    assert np.abs(got - ref).max() < 1e-9 * max(1, np.abs(ref).max()) * 1e4


@pytest.mark.parametrize("name", ["v2", "causal", "discrete", "v3", "v3_noise"])
def test_engine_parameter_table_matches_graph(name):
    """The native engine's module graph (rave_amd/csrc/engine.cpp) asks for
    exactly the reference state_dict names and shapes that rave_amd.graph
    restates -- the table the golden fixtures load into the reference modules."""
    from rave_amd import config as rcfg
    from rave_amd.graph import param_shapes
    cfg = rcfg.get_config(name)
    ccfg = N.model_config(cfg)
    n = N.lib.rave_model_param_count(C.byref(ccfg))
    assert n > 0
    buf = C.create_string_buffer(256)
    numel = C.c_int64()
    got = {}
    for i in range(n):
        N.check(N.lib.rave_model_param_info(C.byref(ccfg), i, buf, 256, C.byref(numel)), "param_info")
        got[buf.value.decode()] = numel.value
    assert got.pop("pqmf.hk") == -1                   # any (n_band, L): the checkpoint's buffer
    exp = {k: int(np.prod(v)) for k, v in param_shapes(cfg).items()}
    assert got == exp


def test_engine_config_validation():
    from rave_amd import config as rcfg
    ccfg = N.model_config(rcfg.v2())
    ccfg.activation = 7
    assert N.lib.rave_model_param_count(C.byref(ccfg)) == N.RAVE_ERR_ARG
    ccfg = N.model_config(rcfg.v2())
    ccfg.n_ratios = 0
    with pytest.raises(ValueError):
        N.check(N.lib.rave_model_param_count(C.byref(ccfg)), "param_count")
    h = C.c_void_p()
    with pytest.raises(ValueError):   # rejected before any device work
        N.check(N.lib.rave_model_create(C.byref(ccfg), None, 0, None, 0, C.byref(h)), "model_create")


def test_unit_workspace_sizes():
    """rave_unit_workspace (host logic, no GPU): the cooperative form exists for
    C = 256 / 512 in split16 and the exact-fp32 ring arithmetic only; its
    counters fit the split-K ticket words and the exchange follows them."""
    def ws(ch, prec, B=16, T=256):
        a = N.UnitArgs(channels=ch, batch=B, t_len=T, dilation=3, pad_left=3, act=N.ACT["leaky"],
                       leaky_slope=0.2, precision=prec)
        return N.lib.rave_unit_workspace(C.byref(a))
    assert ws(128, N.PREC_SPLIT16) == 0 and ws(64, N.PREC_SPLIT16) == 0
    assert ws(256, N.PREC_F32) == 0
    for C_, prec in [(256, N.PREC_SPLIT16), (512, N.PREC_SPLIT16), (512, N.PREC_F32_RING)]:
        n = ws(C_, prec)
        groups = -(-256 // 32) * 16
        assert n >= N.SPLITK_TICKETS + groups * 32 * C_
    # more groups than the ticket words can count: no cooperative form
    assert ws(512, N.PREC_SPLIT16, B=512, T=4096) == 0

    # the wide group (coop_rb = 4, C = 256 only, round 6): twice the members' maxima words
    def wsr(ch, rb, B=1, T=8):
        a = N.UnitArgs(channels=ch, batch=B, t_len=T, dilation=3, pad_left=3, act=N.ACT["leaky"],
                       leaky_slope=0.2, precision=N.PREC_BF16X3, coop_rb=rb)
        return N.lib.rave_unit_workspace(C.byref(a))
    assert wsr(256, 4) >= wsr(256, 0) > 0 and wsr(256, 2) == wsr(256, 0)
    assert wsr(512, 2) == 0                      # no such group: no cooperative form
    a = N.UnitArgs(channels=256, batch=1, t_len=8, dilation=3, pad_left=3, act=N.ACT["leaky"], leaky_slope=0.2,
                   precision=N.PREC_BF16X3, coop_rb=3, x=16, y=16, weight=16)
    assert N.lib.rave_residual_unit(C.byref(a), None) == N.RAVE_ERR_ARG   # refused before any launch


def test_edge_precision_and_f32_filter_images(golden):
    """rave_edge_args.precision is validated before any launch, and the fp32
    filter images are the plain filter rows (scale word 1)."""
    from oracle.rave_oracle import pqmf_filters
    hkf, hki = pqmf_filters(golden("pqmf")["hk"])
    a = N.EdgeArgs(batch=1, frames=64, conv_c_in=6, conv_c_out=64, conv_kernel=7, pqmf_taps=513,
                   x=16, y=16, weight=16, filter=16, precision=2)
    assert N.lib.rave_encoder_head(C.byref(a), None) == N.RAVE_ERR_ARG
    img = N.pack_edge_filter(hkf, head=True, n_out_bands=6, f32=True)
    rows = img[:16 * 552].reshape(16, 552)
    assert img[16 * 552] == 1.0
    h2 = np.asarray(hkf, np.float32).reshape(16, -1)
    np.testing.assert_array_equal(rows[0, :513], h2[0])
    np.testing.assert_array_equal(rows[8, 16:16 + 513], h2[0])                       # phase 1 row
    assert not rows[6].any() and not rows[7].any()                                   # bands past 6
    timg = N.pack_edge_filter(hki, head=False, f32=True)
    trows = timg[:16 * 552].reshape(16, 552)
    h3 = np.asarray(hki, np.float32).reshape(16, 16, -1)
    np.testing.assert_array_equal(trows[3, 5 * 16 + 2], h3[3, 2, 5])


def test_gemv_configs_listing():
    """The skinny-N family (conv_gemv.hip) is listed for the exact-fp32
    precision when the output has at most 128 columns: the narrowest column
    width that holds them, K splits that each stage a bounded window, in-launch
    and separate combines; its workspace is the tickets plus S fp32 slabs.
    Wider outputs list none (host logic only; config codes are per precision:
    the split-f16 tile table has its own tiles 8..11)."""
    def args(T, t_out, prec=N.PREC_F32, c_in=512, c_out=512, k=3, d=3, B=1):
        return N.ConvArgs(c_in=c_in, c_out=c_out, kernel=k, stride=1, dilation=d, pad_left=0, pad_right=0,
                          batch=B, t_in=T, t_out=t_out, precision=prec, x=16, y=16, weight=16)

    def tile(c):
        return (c - 1) & 15

    a = args(10, 4)
    gemv = [c for c in N.conv_configs(a) if 8 <= tile(c) <= 11]
    assert gemv and all(tile(c) == 8 for c in gemv)              # NMAX 4 holds 4 columns
    assert any(((c - 1) >> 9) & 1 for c in gemv) and any(not ((c - 1) >> 9) & 1 for c in gemv)
    for c in gemv:
        a.config = c
        S = (((c - 1) >> 4) & 31) + 1
        want = 0 if S == 1 else N.SPLITK_TICKETS + S * 1 * 512 * 4
        assert N.lib.rave_conv1d_workspace(C.byref(a)) == want, c
    b = args(23, 17)
    assert {tile(c) for c in N.conv_configs(b) if 8 <= tile(c) <= 11} == {11}   # 17 columns: NMAX 32
    assert {tile(c) for c in N.conv_configs(args(40, 34)) if 8 <= tile(c) <= 13} == {12}   # NMAX 64
    assert {tile(c) for c in N.conv_configs(args(130, 128, d=1)) if 8 <= tile(c) <= 13} == {13}   # 128
    assert not [c for c in N.conv_configs(args(140, 134)) if 8 <= tile(c) <= 13]                  # > 128
