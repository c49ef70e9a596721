"""The hand-counted weight register rings of the built gfx950 code object are
structurally safe (tools/ring_hazard_check.py): for every `bload16` (inline-asm
buffer_load_dwordx4 that hipcc does not see) no instruction reads, copies or
writes its destination registers before the covering `s_waitcnt vmcnt(N)`, on
any control-flow path.  CPU only: the check reads the disassembly, it runs
nothing on a GPU.  The synthetic cases pin what the checker detects."""
import os

import pytest

from tools import ring_hazard_check as R

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "rave_amd", "librave_amd.so")


def _prog(lines):
    insts = [R.Inst(0x1000 + 4 * i, t) for i, t in enumerate(lines)]
    R.link(insts)
    return insts


def _hazards(lines):
    insts = _prog(lines)
    out = []
    for k, ins in enumerate(insts):
        if ins.hidden:
            out += R.check_load(insts, k)
    return out


LOAD = ["s_nop 4", "buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen"]


def test_copy_before_wait_is_flagged():
    # the round-5 fault: the compiler copies the refill's destination early
    h = _hazards(LOAD + ["v_mov_b32_e32 v20, v5", "s_waitcnt vmcnt(0)", "s_endpgm"])
    assert len(h) == 1 and "v_mov_b32_e32 v20, v5" in h[0][3]


def test_write_before_wait_is_flagged():
    # a dead ring register reused while its load can still land (WAW)
    h = _hazards(LOAD + ["v_accvgpr_read_b32 v6, a3", "s_waitcnt vmcnt(0)", "s_endpgm"])
    assert len(h) == 1


def test_insufficient_wait_is_flagged():
    # vmcnt(1) with no younger memory op does not cover the load
    h = _hazards(LOAD + ["s_waitcnt vmcnt(1)", "v_mfma_f32_32x32x16_bf16 a[0:15], v[4:7], v[8:11], a[0:15]",
                         "s_endpgm"])
    assert len(h) == 1


def test_counted_wait_covers():
    h = _hazards(LOAD + ["buffer_load_dwordx4 v[8:11], v2, s[0:3], 0 offen",
                         "buffer_load_dwordx4 v2, s[0:3], 0 offen lds",
                         "s_waitcnt vmcnt(2)", "v_mov_b32_e32 v20, v5", "s_endpgm"])
    assert h == []


def test_loop_back_edge_paths():
    # refill at the loop bottom, waited at the loop top: clean; a use on the
    # exit path before the drain: flagged
    body = ["s_waitcnt vmcnt(0)",                       # top: covers the previous refill
            "v_mov_b32_e32 v20, v5",
            "s_nop 4", "buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen",
            "s_cbranch_scc1 65531"]                     # back to the top (-5 dwords)
    assert _hazards(["s_nop 0"] + body + ["s_waitcnt vmcnt(0)", "v_mov_b32_e32 v21, v6", "s_endpgm"]) == []
    h = _hazards(["s_nop 0"] + body + ["v_mov_b32_e32 v21, v6", "s_waitcnt vmcnt(0)", "s_endpgm"])
    assert len(h) == 1 and "v21" in h[0][3]


def test_both_branch_targets_are_followed():
    h = _hazards(LOAD + ["s_cbranch_scc0 2", "s_waitcnt vmcnt(0)", "s_branch 1",
                         "v_mov_b32_e32 v20, v4", "s_endpgm"])
    assert len(h) == 1


@pytest.mark.skipif(not os.path.exists(LIB), reason="librave_amd.so not built (__graft_entry__.build())")
def test_built_library_rings_are_safe():
    loads, kernels, hazards = R.check_library(LIB)
    # every conv1d_{split,ring_f32,bf3}_kernel instantiation carries rings
    assert kernels >= 100 and loads >= 1000, (loads, kernels)
    assert hazards == [], hazards[:5]
