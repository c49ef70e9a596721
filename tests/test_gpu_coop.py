"""The cooperative fused unit's failure path (rave_amd/csrc/unit_split.hip,
cooperative form): a group member whose bounded wait for its partners gives up
must surface as an error, never as silent NaN audio with RAVE_OK.

The reference unit (rave/blocks.py:84-113, Residual :32-46) has no failure
mode; this is the MI355X design's own contract (include/rave_amd.h:
RAVE_SPLITK_STATUS_WORD, rave_unit_args.status, rave_model_check,
RAVE_ERR_COOP).  rave_debug_coop(-1, 1) forces every group to report a give-up
after a normal hand-off, so the path runs deterministically."""
import ctypes as C_

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def N():
    from rave_amd import _native
    return _native


@pytest.fixture
def forced(N):
    N.check(N.lib.rave_debug_coop(-1, 1))
    yield
    N.check(N.lib.rave_debug_coop(-1, 0))


# (arithmetic, C, dilation): the split16 cooperative unit, and the bf16x3 one
# that the f32_bf3 headline runs at C = 256 / 512 (unit_bf3_kernel, RB = 2 / 4;
# its C = 512 window is sized for dilations <= 4)
COOP_FORMS = [("split16", 512, 3), ("bf16x3", 512, 3), ("bf16x3", 256, 9)]


def _unit(N, dev, C=512, B=4, T=96, d=3, precision="split16"):
    prec = N.PRECISION[precision]
    rng = np.random.default_rng(7)
    x = torch.from_numpy(rng.standard_normal((B, C, T)).astype(np.float32)).to(dev)
    w1 = (rng.standard_normal((C, C, 3)) / np.sqrt(3 * C)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, 1)) / np.sqrt(C)).astype(np.float32)
    packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C, precision=prec)).to(dev)
    b = torch.zeros(C, device=dev)

    def args(y, ws, status):
        return N.UnitArgs(channels=C, batch=B, t_len=T, dilation=d, pad_left=d, act=N.ACT["leaky"],
                          leaky_slope=0.2, precision=prec, x=x.data_ptr(), x_sb=C * T, x_sc=T,
                          y=y.data_ptr(), y_sb=C * T, y_sc=T, weight=packed.data_ptr(), bias1=b.data_ptr(),
                          bias2=b.data_ptr(), workspace=ws.data_ptr() if ws is not None else None,
                          status=status.data_ptr() if status is not None else None)
    return x, args


@pytest.mark.parametrize("form", COOP_FORMS, ids=[f"{p}-C{c}" for p, c, _ in COOP_FORMS])
def test_coop_giveup_sets_status_words(N, dev, forced, form):
    """Direct C-ABI: a forced give-up sets the workspace's reserved status word
    and the caller's status word, writes NaN outputs, and still re-arms the
    group counters (every ticket word but the status word is zero after)."""
    precision, C, d = form
    x, args = _unit(N, dev, C=C, d=d, precision=precision)
    st = C_.c_void_p(torch.cuda.current_stream().cuda_stream)
    y = torch.zeros_like(x)
    nws = N.lib.rave_unit_workspace(C_.byref(args(y, None, None)))
    assert nws > N.SPLITK_TICKETS
    ws = torch.zeros(nws, device=dev)
    status = torch.zeros(4, dtype=torch.int32, device=dev)
    N.check(N.lib.rave_residual_unit(C_.byref(args(y, ws, status)), st))
    torch.cuda.synchronize()
    words = ws.view(torch.int32)[:N.SPLITK_TICKETS].cpu().numpy()
    assert words[N.SPLITK_STATUS_WORD] == 1
    assert np.count_nonzero(words[:N.SPLITK_STATUS_WORD]) == 0
    assert int(status[0]) == 1 and int(status[1:].abs().sum()) == 0
    assert torch.isnan(y).all()


@pytest.mark.parametrize("form", COOP_FORMS, ids=[f"{p}-C{c}" for p, c, _ in COOP_FORMS])
def test_coop_no_giveup_leaves_status_clear(N, dev, form):
    """Without the debug override the same launch never gives up: finite
    outputs, both status words zero."""
    precision, C, d = form
    x, args = _unit(N, dev, C=C, d=d, precision=precision)
    st = C_.c_void_p(torch.cuda.current_stream().cuda_stream)
    y = torch.zeros_like(x)
    nws = N.lib.rave_unit_workspace(C_.byref(args(y, None, None)))
    ws = torch.zeros(nws, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(3):
        N.check(N.lib.rave_residual_unit(C_.byref(args(y, ws, status)), st))
    torch.cuda.synchronize()
    assert int(ws.view(torch.int32)[N.SPLITK_STATUS_WORD]) == 0 and int(status[0]) == 0
    assert torch.isfinite(y).all()


def _coop_tuning(model):
    """model.tuning() with every fused unit in its cooperative form (value bit 8;
    the engine takes it where rave_unit_workspace offers one: C = 256 / 512)."""
    out = []
    for k, c, ms in model.tuning():
        if k.startswith("unit|"):
            c = int(c) | 256
        elif k.startswith("fuse|"):
            c = 1
        out.append([k, int(c), ms])
    return out


def _coop_tuning_bf3(model):
    """As _coop_tuning for an f32_bf3 model: every fused unit in bf16x3 (value
    RAVE_PREC_BF16X3), in its cooperative form where the engine offers one."""
    out = []
    for k, c, ms in model.tuning():
        if k.startswith("unit|"):
            c = 5 | 256
        elif k.startswith("fuse|"):
            c = 1
        out.append([k, int(c), ms])
    return out


@pytest.fixture(scope="module", params=["split16", "f32_bf3"])
def coop_model(N, dev, request):
    """A v2 model whose plans run every C = 256 / 512 unit cooperatively: in
    split16, and in the f32_bf3 headline's arithmetic (bf16x3 cooperative
    units)."""
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker
    precision = request.param
    cfg = rcfg.v2()
    params, spk = init_params(cfg, 0), init_speaker(cfg, 0)
    x = torch.from_numpy(np.random.default_rng(1).standard_normal((2, 1, 16384)).astype(np.float32) * 0.3).to(dev)
    probe = RAVE(cfg, params, spk, device=dev, precision=precision)
    ref = probe.forward(x)
    tuning = _coop_tuning(probe) if precision == "split16" else _coop_tuning_bf3(probe)
    m = RAVE(cfg, params, spk, device=dev, precision=precision, tuning=tuning)
    n_coop = sum(1 for k, c, _ in tuning if k.startswith("unit|") and (c >> 8))
    return m, x, ref, tuning, n_coop, (cfg, params, spk, precision)


def test_coop_giveup_raises_through_forward(N, dev, coop_model):
    """RAVE.forward: a give-up inside the call makes RAVE.check() raise
    NativeError (RAVE_ERR_COOP) naming a cooperative unit; a later call on the
    model raises it too when check() was not called; the status is cleared once
    reported, and the next clean call matches the non-cooperative plan."""
    m, x, ref, _, n_coop, _ = coop_model
    assert n_coop > 0
    y = m.forward(x)
    m.check()                                         # clean run first
    assert float((y - ref).abs().max()) < 1e-4
    N.check(N.lib.rave_debug_coop(-1, 1))
    try:
        y = m.forward(x)
        torch.cuda.synchronize()
    finally:
        N.check(N.lib.rave_debug_coop(-1, 0))
    assert torch.isnan(y).any()
    with pytest.raises(N.NativeError, match="cooperative residual unit"):
        m.check()
    m.check()                                         # reported once, then clear
    y = m.forward(x)
    m.check()
    assert float((y - ref).abs().max()) < 1e-4
    # without an explicit check: the next call raises on entry
    N.check(N.lib.rave_debug_coop(-1, 1))
    try:
        m.forward(x)
        torch.cuda.synchronize()
    finally:
        N.check(N.lib.rave_debug_coop(-1, 0))
    with pytest.raises(N.NativeError, match="status -5"):
        m.forward(x)
    m.check()


def test_coop_giveup_raises_through_torchscript_engine(N, dev, coop_model):
    """The TorchScript Engine (nn~ export, csrc/torch_ops.cpp) raises the same
    error from check() and from its next call."""
    from rave_amd.scripted import ScriptedRAVE
    _, x, ref, tuning, _, (cfg, params, spk, precision) = coop_model
    sm = ScriptedRAVE(cfg, params, spk, precision=precision, streaming=False)
    text = "".join(f"{k} {int(c)} {float(ms)!r}\n" for k, c, ms in tuning)
    sm.engine.set_tuning(text)
    y = sm.engine.forward(x)
    sm.engine.check()
    assert float((y - ref).abs().max()) < 1e-4
    N.check(N.lib.rave_debug_coop(-1, 1))
    try:
        sm.engine.forward(x)
        torch.cuda.synchronize()
    finally:
        N.check(N.lib.rave_debug_coop(-1, 0))
    with pytest.raises(RuntimeError, match="cooperative residual unit"):
        sm.engine.check()
    N.check(N.lib.rave_debug_coop(-1, 1))
    try:
        sm.engine.forward(x)
        torch.cuda.synchronize()
    finally:
        N.check(N.lib.rave_debug_coop(-1, 0))
    with pytest.raises(RuntimeError, match="cooperative residual unit"):
        sm.engine.forward(x)
    y = sm.engine.forward(x)
    sm.engine.check()
    assert float((y - ref).abs().max()) < 1e-4


def test_coop_concurrent_engines_make_progress(N, dev, coop_model):
    """Three engine instances of the cooperative plan on three HIP streams at
    once (bench.py's pipelined leg; several nn~ instances in one process): the
    groups of concurrent launches share the XCDs' workgroup slots, and the
    launch-time fit check (unit_split.hip us_launch: slots per XCD >= Q (RB - 1)
    + RB for Q = the process's hardware queues) keeps a whole group resident
    somewhere at all times.  No hand-off may give up, and every output matches
    the single-stream reference."""
    from rave_amd.model import RAVE
    m, x, ref, tuning, n_coop, (cfg, params, spk, precision) = coop_model
    assert n_coop > 0
    models = [m] + [RAVE(cfg, params, spk, device=dev, precision=precision, tuning=tuning) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in models]
    ev = torch.cuda.Event()
    ev.record()
    outs = []
    for s in streams:
        s.wait_event(ev)
    for i in range(12):
        with torch.cuda.stream(streams[i % 3]):
            outs.append(models[i % 3].forward(x))
    for s in streams:
        torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    for mm in models:
        mm.check()
    for y in outs:
        assert torch.isfinite(y).all()
        assert float((y - ref).abs().max()) < 1e-4
