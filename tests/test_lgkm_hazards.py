"""No instruction of the shipped gfx950 code touches a register an LDS / scalar-memory load is still writing.

The F16 kernels issue LDS reads in inline asm whose results are waited for later, in another statement
(`k_wgrad_s`'s `ds_read_b64_tr_b16` fragments, settled one k-step later: wgrad.hip `frag` / `settle`).
The compiler takes an asm output as written when its statement ends, so correctness rests on register
allocation: it must not copy, spill, or reuse such a register before the `s_waitcnt lgkmcnt` that retires
the read (round 3 faulted the GPU exactly that way with a scalar load, commit 926e7d7).  This test
disassembles every gfx950 code object in lib/libnof.so and replays the LGKM counter over each kernel:

  * every LDS op (reads, writes, permutes) and scalar-memory op is queued in issue order;
  * `s_waitcnt lgkmcnt(N)` retires all but the youngest N LDS ops (LDS ops complete in order among
    themselves); a scalar load or message (out of order) retires only at lgkmcnt(0);
  * an instruction that reads a destination register of a pending op, or writes one (other than a newer LDS
    op over an older LDS op's destination), is a hazard.

Control flow is followed (a worklist over each kernel's branches, pending states joined where paths
meet), so a load left in flight across a branch or a loop back-edge is tracked too.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "nerf-or-nothing_amd", "lib", "libnof.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

REG = re.compile(r"(?<![\w\[])([vsa])(?:\[(\d+):(\d+)\]|(\d+))(?![\w])")
LGKM_WAIT = re.compile(r"lgkmcnt\((\d+)\)")


def _regs(text):
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        lo, hi = (int(m.group(2)), int(m.group(3))) if m.group(2) else (int(m.group(4)), int(m.group(4)))
        out.update((kind, r) for r in range(lo, hi + 1))
    return out


def _lgkm_kind(mn):
    """'ds' (in-order LDS), 'smem' / 'msg' (out of order), or None for instructions outside the LGKM counter."""
    if mn.startswith("ds_"):
        return "ds"
    if mn.startswith(("s_load_", "s_buffer_load_", "s_scratch_load_", "s_memtime", "s_memrealtime", "s_dcache_",
                      "s_atc_probe")):
        return "smem"
    if mn.startswith(("s_sendmsg", "s_sendmsghalt")):
        return "msg"
    return None


def _dst(mn, ops):
    """destination registers of an LGKM op (loads and returning LDS ops write their first operand)"""
    if mn.startswith("ds_") and not (mn.startswith("ds_write") or mn.startswith("ds_store") or
                                     mn in ("ds_nop",) or ("_rtn" not in mn and mn.startswith(("ds_add_", "ds_sub_",
                                            "ds_max", "ds_min", "ds_and", "ds_or", "ds_xor", "ds_inc", "ds_dec",
                                            "ds_cmpst", "ds_mskor", "ds_cmpswap", "ds_wrxchg"))) or
                                     mn.startswith("ds_gws") or mn.startswith("ds_barrier")):
        return _regs(ops.split(",")[0]) if ops else set()
    if mn.startswith(("s_load_", "s_buffer_load_", "s_scratch_load_", "s_memtime", "s_memrealtime")):
        return _regs(ops.split(",")[0]) if ops else set()
    return set()


INSN = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<([^>+]+)\+(0x[0-9a-f]+)>")
SYM = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
MAX_AGES = 64


def _parse(lines):
    """kernels -> list of (addr, mnemonic, operands, branch target addr or None)"""
    funcs, cur, base = {}, None, {}
    for raw in lines:
        m = SYM.match(raw.strip())
        if m:
            cur = m.group(2)
            base[cur] = int(m.group(1), 16)
            funcs[cur] = []
            continue
        m = INSN.match(raw)
        if not m or cur is None:
            continue
        mn, ops, addr = m.group(1), m.group(2).strip(), int(m.group(3), 16)
        tgt = None
        if mn.startswith(("s_branch", "s_cbranch")):
            t = TARGET.search(raw)
            if t and t.group(1) in base:
                tgt = base[t.group(1)] + int(t.group(2), 16)
        funcs[cur].append((addr, mn, ops, tgt))
    return funcs


# A state is (ds, oo): ds = the pending LDS ops by age, a tuple of frozensets oldest -> youngest (slot i holds
# every op that is the i-th oldest on some path into this point); oo = the pending out-of-order ops (scalar
# loads, messages).  LDS ops retire in order among themselves whatever else is pending, so lgkmcnt(n) leaves
# at most the youngest n LDS slots; an out-of-order op retires only at lgkmcnt(0).
EMPTY = ((), frozenset())


def _wait(state, n):
    ds, oo = state
    return EMPTY if n == 0 else (ds[len(ds) - n:] if len(ds) > n else ds, oo)


def _issue(state, op):
    ds, oo = state
    if op[1] != "ds":
        return ds, oo | {op}
    ds = ds + (frozenset([op]),)
    if len(ds) > MAX_AGES:  # fold the oldest slots together: they then retire later, never earlier
        ds = (ds[0] | ds[1],) + ds[2:]
    return ds, oo


def _merge(a, b):
    """join: LDS slots aligned from the youngest and united, out-of-order sets united"""
    if a == b:
        return a
    (da, oa), (db, ob) = a, b
    n = max(len(da), len(db))
    da = (frozenset(),) * (n - len(da)) + da
    db = (frozenset(),) * (n - len(db)) + db
    return tuple(x | y for x, y in zip(da, db)), oa | ob


def check_disassembly(lines):
    """Replays the LGKM counter over `llvm-objdump -d` output, following branches (a worklist over each
    kernel's control flow, states joined at merges); returns the hazards found."""
    hazards = {}
    for func, insns in _parse(lines).items():
        if not insns:
            continue
        idx = {a: i for i, (a, _, _, _) in enumerate(insns)}
        state_in = {0: EMPTY}
        work = [0]
        while work:
            i = work.pop()
            st = state_in[i]
            addr, mn, ops, tgt = insns[i]
            kind = _lgkm_kind(mn)
            if mn == "s_waitcnt" or mn.startswith("s_waitcnt_lgkmcnt"):
                m = LGKM_WAIT.search(ops) if mn == "s_waitcnt" else re.search(r",\s*(0x[0-9a-f]+|\d+)", ops)
                out = _wait(st, int(m.group(1), 0)) if m else st
            else:
                ds, oo = st
                busy_ds = {r: op for slot in ds for op in slot for r in op[2]}
                busy_oo = {r: op for op in oo for r in op[2]}
                dst = _dst(mn, ops) if kind else set()
                src = _regs(ops) - dst if kind else _regs(ops)
                # reads of any pending destination, and writes over one — except an LDS op's write over an
                # older LDS op's destination (LDS ops retire in order)
                hit = {r: busy_ds.get(r) or busy_oo[r] for r in src if r in busy_ds or r in busy_oo}
                hit.update({r: busy_oo[r] for r in dst if r in busy_oo})
                if kind != "ds":
                    hit.update({r: busy_ds[r] for r in dst if r in busy_ds})
                if hit:
                    r0 = sorted(hit)[0]
                    hazards[(func, addr)] = (f"{func} @{addr:#x}: `{mn} {ops}` touches {sorted(hit)[:4]} of "
                                             f"in-flight `{hit[r0][3]}`")
                out = _issue(st, (addr, kind, frozenset(dst), f"{mn} {ops}")) if kind else st
            succ = []
            if mn == "s_endpgm" or mn.startswith(("s_setpc", "s_trap")):
                pass
            elif mn == "s_branch":
                succ.append(idx.get(tgt))
            else:
                if tgt is not None:
                    succ.append(idx.get(tgt))
                succ.append(i + 1 if i + 1 < len(insns) else None)
            for j in succ:
                if j is None:
                    continue
                new = out if j not in state_in else _merge(state_in[j], out)
                if j not in state_in or new != state_in[j]:
                    state_in[j] = new
                    work.append(j)
    return list(hazards.values())


def _disassemble(lib, tmp):
    shutil.copy(lib, os.path.join(tmp, "lib.so"))
    subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=tmp, check=True, capture_output=True)
    cos = sorted(f for f in os.listdir(tmp) if "gfx950" in f)
    assert cos, "no gfx950 code object in the library"
    out = []
    for co in cos:
        r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], cwd=tmp, check=True, capture_output=True, text=True)
        out.append(r.stdout.splitlines())
    return out


def _asm(*insns):
    """a fake kernel in llvm-objdump's format (addresses 8 bytes apart, branch targets as <k+0xoff>)"""
    out = ["0000000000001000 <_ZN3nof1kE>:"]
    for i, t in enumerate(insns):
        t = t.replace("@", "// ")
        out.append(f"\t{t:<60}// {0x1000 + 8 * i:012X}: 00000000" + (f" <_ZN3nof1kE+{t.split('->')[1]}>"
                                                                          if "->" in t else ""))
    return [l.split("->")[0] if "->" in l and not l.startswith("\t") else l for l in out]


def test_checker_sees_a_planted_hazard():
    """The replay itself: a copy of an in-flight transposed read is a hazard; after its wait it is not;
    counted waits retire in order; a scalar load makes them order nothing; branches are followed."""
    bad = _asm("ds_read_b64_tr_b16 v[130:131], v4", "v_mov_b32_e32 v7, v131", "s_waitcnt lgkmcnt(0)", "s_endpgm")
    good = _asm("ds_read_b64_tr_b16 v[130:131], v4", "s_waitcnt lgkmcnt(0)", "v_mov_b32_e32 v7, v131", "s_endpgm")
    counted = _asm("ds_read_b128 v[0:3], v9", "ds_read_b128 v[4:7], v9 offset:16", "s_waitcnt lgkmcnt(1)",
                   "v_mov_b32_e32 v8, v3", "v_mov_b32_e32 v8, v4", "s_endpgm")
    mixed = _asm("s_load_dword s4, s[0:1], 0x0", "ds_read_b32 v1, v9", "s_waitcnt lgkmcnt(1)",
                 "s_add_u32 s5, s4, 1", "s_endpgm")
    # the read is in flight on the branch's path only: seen through the jump over the wait
    branchy = _asm("ds_read_b32 v1, v9", "s_cbranch_scc1 2 ->0x20", "s_waitcnt lgkmcnt(0)", "s_nop 0",
                   "v_mov_b32_e32 v2, v1", "s_endpgm")
    assert check_disassembly(bad) and not check_disassembly(good)
    h = check_disassembly(counted)
    assert len(h) == 1 and "v8, v4" in h[0], h  # v3 retired by lgkmcnt(1), v4 still in flight
    assert check_disassembly(mixed), "lgkmcnt(N > 0) orders nothing when a scalar load is pending"
    assert check_disassembly(branchy), "the path through the branch is followed"


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="llvm-objdump not installed")
@pytest.mark.parametrize("name", ["libnof.so", "libnof_check.so"])
def test_no_register_touched_while_its_lgkm_load_is_in_flight(name):
    """the product library and the device-check build the GPU suite also loads"""
    lib = os.path.join(os.path.dirname(LIB), name)
    assert os.path.exists(lib), f"lib/{name} not built (make -C nerf-or-nothing_amd all check)"
    with tempfile.TemporaryDirectory() as tmp:
        objs = _disassemble(lib, tmp)
    hazards, n_tr = [], 0
    for lines in objs:
        n_tr += sum("ds_read_b64_tr_b16" in l for l in lines)
        hazards += check_disassembly(lines)
    assert n_tr > 0, "k_wgrad_s's transposed reads not found: the check no longer covers them"
    assert not hazards, f"{len(hazards)} LGKM hazards:\n" + "\n".join(hazards[:20])
