#!/usr/bin/env python3
"""Static check of the hand-counted weight register rings in the built gfx950
code object (test infrastructure: tests/test_ring_hazard.py runs it on every
build; it never runs on the product path).

The split / ring / bf16x3 conv kernels (rave_amd/csrc/conv_split.hip) stream
weight fragments into registers with `bload16`: an inline-asm
`buffer_load_dwordx4 vD, voff, rsrc, 0 offen` (preceded by `s_nop 4`) whose
destination hipcc believes is defined as soon as the asm statement ends.  The
matching `s_waitcnt vmcnt(N)` comes later, in `wait_vm_regs{,3}`.  Correctness
rests on the compiler never reading, copying, spilling or overwriting vD in
between: round 5 faulted a GPU run when a scheduling change let the compiler
copy a refill's destination before the hardware wrote it.

For every such load this tool follows every control-flow path of the
disassembly from the load until a covering wait -- an `s_waitcnt vmcnt(N)` with
at least N younger vector-memory operations issued since the load (vmcnt counts
loads, stores, atomics and LDS-DMA together, in issue order) -- and reports any
instruction on the way that names one of vD's registers.

    python tools/ring_hazard_check.py [rave_amd/librave_amd.so]

Exit status 0 when no hazard is found.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# kernels that use bload16 (hand-counted register rings)
KERNEL_RE = re.compile(r"conv1d_(bf3|split|ring_f32)_kernel|decoder_tail_kernel|stack_|unit_")

_VMEM_PREFIX = ("buffer_", "global_", "scratch_", "flat_", "tbuffer_")
_VREG_RE = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_VMCNT_RE = re.compile(r"vmcnt\((\d+)\)")


def code_objects(lib):
    """The gfx950 code objects (ELF bytes) embedded in a HIP shared library or object."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib, os.devnull],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    out = []
    i = data.find(BUNDLE_MAGIC)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", data, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if "gfx950" in triple:
                out.append(data[i + off:i + off + size])
        i = data.find(BUNDLE_MAGIC, i + 1)
    return out


def disassemble(elf_bytes):
    with tempfile.NamedTemporaryFile(suffix=".co") as fh:
        fh.write(elf_bytes)
        fh.flush()
        r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", fh.name],
                           check=True, capture_output=True, text=True)
    return r.stdout


class Inst:
    __slots__ = ("addr", "mnem", "ops", "text", "regs", "vmem", "vmcnt", "branch", "target", "end", "hidden")

    def __init__(self, addr, text):
        self.addr = addr
        self.text = text
        parts = text.split(None, 1)
        self.mnem = parts[0]
        self.ops = parts[1] if len(parts) > 1 else ""
        regs = set()
        for a, b, c in _VREG_RE.findall(self.ops):
            if c:
                regs.add(int(c))
            else:
                regs.update(range(int(a), int(b) + 1))
        self.regs = frozenset(regs)
        self.vmem = self.mnem.startswith(_VMEM_PREFIX)
        self.vmcnt = None
        if self.mnem == "s_waitcnt":
            m = _VMCNT_RE.search(self.ops)
            if m:
                self.vmcnt = int(m.group(1))
        self.branch = self.mnem.startswith("s_branch") or self.mnem.startswith("s_cbranch")
        self.target = None
        self.end = self.mnem in ("s_endpgm", "s_setpc_b64", "s_trap")
        self.hidden = False


def parse_functions(asm, name_filter=KERNEL_RE):
    """{symbol: [Inst]} for the functions whose names match name_filter."""
    funcs, cur, name = {}, None, None
    for line in asm.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            name = m.group(2)
            cur = [] if name_filter.search(name) else None
            if cur is not None:
                funcs[name] = cur
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s or s.startswith(";"):
            continue
        m = re.match(r"^(.*?)\s*//\s*([0-9A-Fa-f]+):", s)
        if not m:
            continue
        body = m.group(1).strip()
        if not body:
            continue
        cur.append(Inst(int(m.group(2), 16), body))
    return funcs


def link(insts):
    """Resolve branch targets to instruction indices; mark the hidden ring loads."""
    at = {ins.addr: k for k, ins in enumerate(insts)}
    for k, ins in enumerate(insts):
        if ins.branch:
            # SOPP branch: simm16 in dwords, relative to the next instruction
            simm = int(ins.ops.split()[0], 0)
            if simm >= 0x8000:
                simm -= 0x10000
            ins.target = at.get(ins.addr + 4 + 4 * simm)
            if ins.target is None:
                raise ValueError(f"branch target outside the function: {ins.addr:#x} {ins.text}")
        if (ins.mnem == "buffer_load_dwordx4" and " lds" not in (" " + ins.ops) and "offen" in ins.ops
                and k > 0 and insts[k - 1].mnem == "s_nop" and insts[k - 1].ops.strip() == "4"):
            ins.hidden = True


def dest_regs(ins):
    m = _VREG_RE.match(ins.ops)
    if not m:
        return frozenset()
    a, b, c = m.groups()
    return frozenset([int(c)]) if c else frozenset(range(int(a), int(b) + 1))


def _is_load(ins):
    return "_load" in ins.mnem and " lds" not in (" " + ins.ops)


def src_regs(ins):
    """VGPRs named after the first (destination) operand."""
    m = _VREG_RE.match(ins.ops)
    rest = ins.ops[m.end():] if m else ins.ops
    regs = set()
    for a, b, c in _VREG_RE.findall(rest):
        regs.update([int(c)] if c else range(int(a), int(b) + 1))
    return regs


def check_load(insts, k, max_vm=63):
    """Hazards of hidden load k: list of (load, offending instruction) texts."""
    dst = dest_regs(insts[k])
    bad = []
    seen = set()
    stack = [(k + 1, 0)]
    while stack:
        j, y = stack.pop()
        while j < len(insts):
            key = (j, y)
            if key in seen:
                break
            seen.add(key)
            ins = insts[j]
            if ins.vmcnt is not None and y >= ins.vmcnt:
                break                                   # covered on this path
            if ins.vmem and _is_load(ins) and dst <= dest_regs(ins) and not (src_regs(ins) & dst):
                break                                   # a younger load rewrites them (loads return in order)
            if ins.regs & dst:
                bad.append((insts[k].addr, insts[k].text, ins.addr, ins.text))
                break
            if ins.vmem:
                y = min(y + 1, max_vm)
            if ins.end:
                break
            if ins.branch:
                if ins.target is not None:
                    stack.append((ins.target, y))
                if ins.mnem.startswith("s_branch"):
                    break                               # unconditional
            j += 1
    return bad


def check_code_object(co):
    """(hidden loads checked, kernels checked, hazards) of one code object."""
    loads = kernels = 0
    hazards = []
    for name, insts in parse_functions(disassemble(co)).items():
        link(insts)
        ks = [k for k, ins in enumerate(insts) if ins.hidden]
        if not ks:
            continue
        kernels += 1
        for k in ks:
            loads += 1
            for h in check_load(insts, k):
                hazards.append((name,) + h)
    return loads, kernels, hazards


def check_library(lib, workers=None):
    """(hidden loads checked, kernels checked, hazards) over every gfx950 code
    object of the library (one process per code object)."""
    from concurrent.futures import ProcessPoolExecutor
    cos = code_objects(lib)
    workers = workers or min(8, os.cpu_count() or 1)
    loads = kernels = 0
    hazards = []
    with ProcessPoolExecutor(max_workers=workers) as ex:
        for l, k, h in ex.map(check_code_object, cos):
            loads += l
            kernels += k
            hazards += h
    return loads, kernels, hazards


def main():
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(repo, "rave_amd", "librave_amd.so")
    loads, kernels, hazards = check_library(lib)
    print(f"{lib}: {loads} hidden ring loads in {kernels} kernels; {len(hazards)} hazards")
    for name, la, lt, ia, it in hazards[:20]:
        print(f"  {name}\n    load  {la:#x}: {lt}\n    reads {ia:#x}: {it}")
    return 1 if hazards or loads == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
