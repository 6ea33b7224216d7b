#!/usr/bin/env python3
"""Static check of the counted vector-memory waits in the device assembly.

A counted ``s_waitcnt vmcnt(N)`` retires an LDS-DMA (or load) only if at least N vector-memory instructions were
issued after it -- in the instruction stream the COMPILER emitted, on every path to the wait.  The kernels say which
group each counted wait must retire with the markers of csrc/common.h:

    SV_VMTAG("w1")             -> ``; svtag w1``        after the group's last vector-memory instruction
    SV_VMWAIT(N, "w1:1 w2:2")  -> ``s_waitcnt vmcnt(N) ; svwait w1:1 w2:2``
    SV_VMCHECK("bias:1")       -> ``; svcheck bias:1``  (assert retired, no wait)

``name:k`` = the k-th most recent instance of the group (1 = the latest); ``name:k@c`` checks only the paths on
which group c was tagged after that instance (a wait whose count includes another group's instructions only where
the source guarantees they lie between, e.g. gemm9's epilogue stores: "p1:2@epi").  For every kernel that carries markers the
checker builds the control-flow graph of its assembly and runs a forward dataflow analysis: per group and instance,
the MINIMUM over all paths of the number of vector-memory instructions issued since that instance's marker
(retired = infinite; an s_waitcnt vmcnt(n) retires every instance with >= n younger; 64 younger retire it too, the
counter's capacity).  A wait passes when each listed instance is retired by it on every path.

Vector-memory instructions counted: buffer_/global_/scratch_/flat_ loads, stores and atomics (LDS-DMA included);
cache-maintenance ones (buffer_wbl2 / buffer_inv) are not counted, which can only make the check stricter.

Usage:  check_vmcnt.py FILE.s [...]            (device assembly: hipcc --cuda-device-only -S)
        check_vmcnt.py --build                 compile the checked sources with build_native()'s flags and check them
Exit status 1 if any wait leaves its target outstanding (or a marker names an unknown group).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

INF = 10**9
MAXI = 4  # instances tracked per group
VMEM = re.compile(r"^(buffer_(load|store|atomic)|global_(load|store|atomic)|scratch_(load|store)|flat_(load|store|atomic))")
BRANCH = re.compile(r"^s_(c?branch)")
LABEL = re.compile(r"^(\.LBB\d+_\d+):")
CHECKED_SOURCES = ("mlp.hip", "gemm9.hip")


def split_kernels(text: str) -> dict[str, list[str]]:
    """Kernel symbol -> its assembly lines (from the symbol's label to its .Lfunc_end)."""
    lines = text.splitlines()
    out: dict[str, list[str]] = {}
    i = 0
    while i < len(lines):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", lines[i])
        if m and not m.group(1).startswith(".") and i > 0 and any(
                ".type" in lines[j] and m.group(1) in lines[j] and "@function" in lines[j] for j in range(max(0, i - 4), i)):
            name = m.group(1)
            j = i + 1
            while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
                j += 1
            out[name] = lines[i + 1:j]
            i = j
        i += 1
    return out


def parse(lines: list[str]):
    """-> list of basic blocks {label, ins: [(kind, payload, lineno)], succ_idx: [(block, edge)]}; a conditional
    branch's two edges carry ('taken'|'fall', opcode) so the path-sensitive pass can follow scc / vcc facts."""
    blocks = []
    cur = {"label": "<entry>", "ins": [], "succ": [], "fall": True}
    blocks.append(cur)

    def new_block(label):
        nonlocal cur
        cur = {"label": label, "ins": [], "succ": [], "fall": True}
        blocks.append(cur)

    for ln, raw in enumerate(lines):
        s = raw.strip()
        if not s:
            continue
        m = LABEL.match(s)
        if m:
            new_block(m.group(1))
            continue
        if s.startswith(";;#ASM") or s.startswith("."):
            continue
        if s.startswith(";"):
            mm = re.match(r";\s*(svtag|svcheck)\s+(.*)$", s)
            if mm:
                cur["ins"].append((mm.group(1), mm.group(2).split(), ln))
            continue
        body, _, comment = s.partition(";")
        body = body.strip()
        op = body.split()[0] if body else ""
        if op == "s_waitcnt":
            mv = re.search(r"vmcnt\((\d+)\)", body)
            mw = re.match(r"\s*svwait\s+(.*)$", comment)
            cur["ins"].append(("wait", (int(mv.group(1)) if mv else None, mw.group(1).split() if mw else []), ln))
            continue
        if VMEM.match(op):
            cur["ins"].append(("vmem", op, ln))
            continue
        if op == "s_endpgm" or op.startswith("s_setpc"):
            cur["fall"] = False
            new_block(f"<after{ln}>")
            continue
        if BRANCH.match(op):
            tgt = body.split()[-1]
            cur["succ"].append((tgt, op))
            if op == "s_branch":
                cur["fall"] = False
            new_block(f"<after{ln}>")
            continue
        if op:
            cur["ins"].append(("op", body, ln))
    # keep only the scalar-relevant ops: SALU, VALU writing an SGPR / vcc, and the VGPRs of the uniform-bool idiom
    idiom_v = set()
    for b in blocks:
        for k, p, _ in b["ins"]:
            if k == "op" and p.startswith("v_cndmask_b32_e64"):
                a = p.replace(",", " ").split()
                if len(a) == 5 and a[2] == "0" and a[3] == "1":
                    idiom_v.add(a[1])
    skip = ("s_nop", "s_barrier", "s_setprio", "s_sleep", "s_waitcnt", "s_memtime", "s_memrealtime", "s_sendmsg")
    for b in blocks:
        kept = []
        for ins in b["ins"]:
            if ins[0] != "op":
                kept.append(ins)
                continue
            a = ins[1].replace(",", " ").split()
            op = a[0]
            if op.startswith(skip):
                continue
            if op.startswith("s_") or (len(a) > 1 and (_regset(a[1]) is not None or a[1] in idiom_v)) or (
                    len(a) > 2 and a[2] in ("vcc", "vcc_lo")):
                kept.append(ins)
        b["ins"] = kept
    index = {b["label"]: k for k, b in enumerate(blocks)}
    for k, b in enumerate(blocks):
        succ = []
        for t, op in b["succ"]:
            if t in index:
                succ.append((index[t], ("taken", op)))
        if b["fall"] and k + 1 < len(blocks):
            cond = [op for _, op in b["succ"] if op != "s_branch"]
            succ.append((k + 1, ("fall", cond[0]) if cond else None))
        b["succ_idx"] = succ
    return blocks


# ---- scalar facts: just enough symbolic evaluation to follow the uniform branches hipcc correlates through SGPR
# masks (s_mov_b64 s[0:1], -1 / 0 ... s_andn2_b64 vcc, exec, s[0:1]; s_cbranch_vccnz) and repeated s_cmp of an unchanged
# register (if (grp == 0) ... if (grp == 0)).  Unknown instructions only ever forget facts (more paths, stricter).
_SREG = re.compile(r"^(s\[(\d+):(\d+)\]|s(\d+)|vcc|vcc_lo|vcc_hi|exec|exec_lo|exec_hi|m0)$")
_NO_SCC = ("s_mov_", "s_movk_", "s_cselect_", "s_mul_i32", "s_mul_hi", "s_waitcnt", "s_nop", "s_barrier", "s_setprio",
           "s_sleep", "s_getpc", "s_memtime", "s_memrealtime", "s_load", "s_buffer_load", "s_sendmsg", "s_dcache",
           "s_sethalt", "s_trap", "s_icache", "s_set_gpr_idx", "s_denorm", "s_round")


def _regset(tok: str):
    tok = tok.rstrip(",")
    m = _SREG.match(tok)
    if not m:
        return None
    if m.group(2) is not None:
        return frozenset(range(int(m.group(2)), int(m.group(3)) + 1))
    if m.group(4) is not None:
        return frozenset([int(m.group(4))])
    base = tok.split("_")[0]
    return frozenset([base])


def _imm(tok: str):
    tok = tok.rstrip(",")
    try:
        return int(tok, 0)
    except ValueError:
        return None


def _cmp_pred(op: str, args: list[str], ver) -> tuple | None:
    """('p', key, polarity) of an s_cmp: normalised so that complementary compares of the same operands share a key
    (lt x / ge x / gt x-1 / le x-1 of an immediate; a > b as b < a; eq / lg).  The key carries the version (defining
    line) of every register it reads, so a fact about a value never applies to a later value of the register."""
    m = re.match(r"s_cmpk?_(eq|lg|gt|ge|lt|le)_([iu]\d+)$", op)
    if not m or len(args) < 2:
        return None
    rel, ty = m.groups()
    a, b = args[0], args[1]
    regs = tuple(sorted((str(x), ver(str(x))) for x in (_regset(a) or frozenset()) | (_regset(b) or frozenset())))
    ib = _imm(b)
    if rel in ("eq", "lg"):
        x, y = sorted([a, b])
        return ("p", ("eq", ty, x, y, regs), rel == "eq")
    if ib is not None:
        if rel in ("lt", "ge"):
            return ("p", ("lt", ty, a, str(ib), regs), rel == "lt")
        return ("p", ("lt", ty, a, str(ib + 1), regs), rel == "le")
    if rel in ("lt", "ge"):
        return ("p", ("lt", ty, a, b, regs), rel == "lt")
    return ("p", ("lt", ty, b, a, regs), rel == "gt")


_CAP = 3  # exact small-counter values tracked up to this, then a lower bound (enough for "kt < 2"-style tests)


def _mentions(v, pairs) -> bool:
    return isinstance(v, tuple) and len(v) == 3 and any(p in pairs for p in v[1][4])


def interesting_regs(blocks) -> frozenset:
    """Register tokens whose values can decide a branch: compare operands, mask operands, the uniform-bool idiom, and
    (closure) the sources of the moves / adds / selects that define them.  Only these are given values, which keeps the
    number of distinct path classes small."""
    ops = [p.replace(",", " ").split() for b in blocks for k, p, _ in b["ins"] if k == "op"]
    want = set()
    for a in ops:
        if a[0].startswith(("s_cmp_", "s_cmpk_")):
            want.update(a[1:3])
        elif a[0] in ("s_and_b64", "s_or_b64", "s_andn2_b64") or (a[0] == "s_mov_b64" and a[1] == "vcc"):
            want.update(a[1:4])
        elif a[0].startswith(("v_cndmask_b32_e64", "v_cmp_ne_u32_e64", "v_cmp_eq_u32_e64", "s_cselect_b64")):
            want.update(a[1:])
    changed = True
    while changed:
        changed = False
        for a in ops:
            if a[0] in ("s_mov_b32", "s_mov_b64", "s_add_i32", "s_add_u32") and len(a) > 2 and a[1] in want:
                for x in a[2:]:
                    if x not in want and _imm(x) is None:
                        want.add(x)
                        changed = True
    out = set()
    for x in want:
        rs = _regset(x)
        if rs is not None:
            out |= set(rs)
        elif _imm(x) is None:
            out.add(x)  # VGPR tokens of the idiom
    return frozenset(out)


class Ctx:
    """Scalar facts of one path class: regs (register set -> -1 / 0 / ('p', key, pol)), scc / vcc values, known
    predicates, and the version (defining line) of every register written so far."""
    __slots__ = ("regs", "scc", "vcc", "facts", "ver")
    keep: frozenset = frozenset()  # set per kernel: interesting_regs()
    counters: frozenset = frozenset()  # registers compared against an immediate: the only ones given integer values

    def __init__(self, regs=None, scc=None, vcc=None, facts=None, ver=None):
        self.regs = dict(regs or {})
        self.scc, self.vcc = scc, vcc
        self.facts = dict(facts or {})
        self.ver = dict(ver or {})

    def v(self, name: str):
        return self.ver.get(name, "in")

    def key(self):
        self._prune()
        if Ctx.keep:
            for k in [k for k in self.regs if not (k & Ctx.keep)]:
                del self.regs[k]
        return (tuple(sorted(((tuple(sorted(map(str, k))), v) for k, v in self.regs.items()), key=str)),
                self.scc, self.vcc, tuple(sorted(self.facts.items(), key=str)))

    def _prune(self):
        """Drop facts nothing can test any more (a register they read has been redefined, and no value holds them)."""
        held = {v[1] for v in list(self.regs.values()) + [self.scc, self.vcc] if isinstance(v, tuple)}
        for k in list(self.facts):
            if k not in held and any(self.v(n) != ver for n, ver in k[4]):
                del self.facts[k]

    def copy(self):
        return Ctx(self.regs, self.scc, self.vcc, self.facts, self.ver)

    def clobber(self, rs, line):
        if not rs:
            return
        for k in [k for k in self.regs if k & rs]:
            del self.regs[k]
        pairs = {(str(x), line) for x in rs}  # a value of this same version would alias the new one
        for k in [k for k in self.facts if any(p in pairs for p in k[4])]:
            del self.facts[k]
        for k in [k for k, v in self.regs.items() if _mentions(v, pairs)]:
            del self.regs[k]
        for attr in ("scc", "vcc"):
            if _mentions(getattr(self, attr), pairs):
                setattr(self, attr, None)
        for x in rs:
            self.ver[str(x)] = line
        if "vcc" in rs:
            self.vcc = None

    def value_of(self, tok):
        rs = _regset(tok)
        if rs is None:
            return None
        return self.regs.get(rs)

    def resolve(self, v):
        """bool, or ('p', key, pol) still unknown, or None."""
        if v is None or isinstance(v, bool):
            return v
        if isinstance(v, int):
            return v != 0
        if v[0] != "p":
            return None
        _, k, pol = v
        if k in self.facts:
            return self.facts[k] == pol
        t = self._implied(k)
        if t is not None:
            return t == pol
        return v

    @staticmethod
    def _reg_const(k):
        """(register token, constant) of a compare key against an immediate, else None."""
        if k[0] == "eq":
            a, b = k[2], k[3]
            if _imm(a) is not None and _imm(b) is None:
                return b, _imm(a)
            if _imm(b) is not None and _imm(a) is None:
                return a, _imm(b)
            return None
        if _imm(k[3]) is not None and _imm(k[2]) is None:
            return k[2], _imm(k[3])
        return None

    def _implied(self, k):
        """The value of compare k implied by known facts about the same register value (eq c => lt x is c < x;
        lt x true and c >= x => eq c false; lt x false and c < x => eq c false), or None."""
        rc = self._reg_const(k)
        if rc is None:
            return None
        reg, c = rc
        for f, val in self.facts.items():
            if f[4] != k[4]:
                continue
            frc = self._reg_const(f)
            if frc is None or frc[0] != reg:
                continue
            fc = frc[1]
            if f[1] != k[1] and (fc < 0 or c < 0):  # signed / unsigned agree only on non-negative constants
                continue
            if f[0] == "eq" and val and k[0] == "lt":
                return fc < c
            if f[0] == "eq" and val and k[0] == "eq":
                return fc == c
            if f[0] == "lt" and k[0] == "eq":
                if val and c >= fc:
                    return False
                if not val and c < fc:
                    return False
            if f[0] == "lt" and k[0] == "lt":
                if val and fc <= c:
                    return True
                if not val and c <= fc:
                    return False
        return None

    def op(self, body: str, line: int):
        toks = body.replace(",", " ").split()
        op, args = toks[0], toks[1:]
        if op.startswith("s_cmp_") or op.startswith("s_cmpk_"):
            pr = _cmp_pred(op, args, self.v)
            # operands of known constant value (s_mov_b32 s71, 0 before a loop): evaluate
            vals = [(_imm(x) if _imm(x) is not None else self.regs.get(_regset(x) or frozenset([x]))) for x in args[:2]]
            if pr is not None and isinstance(vals[0], tuple) and vals[0][0] == "ge" and isinstance(vals[1], int):
                lo, c = vals[0][1], vals[1]  # a >= lo against the constant c
                rel = pr[1][0]
                known = None
                if rel == "eq" and c < lo:
                    known = False
                elif rel == "lt" and pr[1][2] == args[0]:
                    bound = int(pr[1][3])  # a < bound
                    if lo >= bound:
                        known = False
                if known is not None:
                    self.scc = known == pr[2]
                    return
            if pr is not None and all(isinstance(x, int) for x in vals):
                a, b = vals
                rel = pr[1][0]
                if rel == "eq":
                    self.scc = (a == b) == pr[2]
                else:
                    lt = (a < b) if pr[1][2] == args[0] else (b < a)
                    if pr[1][2] == args[0] and pr[1][3] != args[1]:  # the le / gt forms compare against b + 1
                        lt = a < b + 1
                    self.scc = lt == pr[2]
                return
            self.scc = self.resolve(pr)
            return
        if op in ("s_cselect_b64", "s_cselect_b32") and len(args) == 3 and _imm(args[1]) == -1 and _imm(args[2]) == 0:
            rs = _regset(args[0])
            val = self.scc
            self.clobber(rs, line)
            if rs is not None and val is not None:
                self.regs[rs] = val if isinstance(val, tuple) else (-1 if val else 0)
            return
        if op in ("s_add_i32", "s_add_u32") and len(args) == 3:
            # small loop counters: exact up to CAP, then a lower bound ('ge', CAP)
            rs = _regset(args[0])
            ia, ib = _imm(args[1]), _imm(args[2])
            src, inc = (args[1], ib) if ib is not None else (args[2], ia)
            v = self.regs.get(_regset(src) or frozenset([src])) if inc is not None else None
            self.clobber(rs, line)
            self.scc = None
            if rs is not None and rs <= Ctx.counters and inc is not None and inc >= 0 and v is not None and not (
                    isinstance(v, tuple) and v[0] == "p"):
                lo = v[1] if isinstance(v, tuple) else v
                if isinstance(v, int) and v + inc <= _CAP:
                    self.regs[rs] = v + inc
                elif lo >= 0:
                    self.regs[rs] = ("ge", min(lo + inc, _CAP))
            return
        if op in ("s_mov_b64", "s_mov_b32") and len(args) == 2:
            rs = _regset(args[0])
            imm = _imm(args[1])
            src = self.value_of(args[1]) if imm is None else None
            self.clobber(rs, line)
            if rs is not None:
                if imm is not None and (imm in (-1, 0) or (rs <= Ctx.counters and 0 <= imm <= _CAP)):
                    self.regs[rs] = imm
                elif src is not None:
                    self.regs[rs] = src
                if args[0] == "vcc":
                    v = imm if imm is not None else src
                    self.vcc = self.resolve(v) if v is not None else None
            return
        if op in ("s_and_b64", "s_or_b64") and len(args) == 3 and args[0] not in ("vcc", "exec"):
            # masks combined: a known-false (and) / known-true (or) operand decides; a known-neutral one passes the other
            # (exec counts as true: these uniform masks are formed with every lane active)
            rs = _regset(args[0])
            va = True if args[1] == "exec" else self.resolve(self.value_of(args[1]))
            vb = True if args[2] == "exec" else self.resolve(self.value_of(args[2]))
            self.clobber(rs, line)
            self.scc = None
            if rs is None:
                return
            absorb, neutral = (False, True) if op == "s_and_b64" else (True, False)
            res = None
            if va is absorb or vb is absorb:
                res = absorb
            elif va is neutral:
                res = vb
            elif vb is neutral:
                res = va
            if isinstance(res, bool):
                self.regs[rs] = -1 if res else 0
            elif isinstance(res, tuple):
                self.regs[rs] = res
            return
        if op in ("s_and_b64", "s_andn2_b64") and len(args) == 3 and args[0] == "vcc":
            other = args[2] if args[1] == "exec" else (args[1] if args[2] == "exec" and op == "s_and_b64" else None)
            val = self.value_of(other) if other else None
            val = self.resolve(val) if val is not None else None
            if val is not None and op == "s_andn2_b64":
                val = (not val) if isinstance(val, bool) else ("p", val[1], not val[2])
            self.clobber(frozenset(["vcc"]), line)
            self.vcc = val
            self.scc = None
            return
        # the uniform-bool-through-a-VGPR idiom: v_cndmask_b32_e64 vX, 0, 1, S ; v_cmp_{ne,eq}_u32_e64 D, 1, vX
        if op == "v_cndmask_b32_e64" and len(args) == 4 and args[1] == "0" and args[2] == "1":
            val = self.value_of(args[3])
            val = self.resolve(val) if val is not None else None
            self.regs.pop(frozenset([args[0]]), None)
            if val is not None:
                self.regs[frozenset([args[0]])] = val if isinstance(val, tuple) else (-1 if val else 0)
            return
        if op in ("v_cmp_ne_u32_e64", "v_cmp_eq_u32_e64") and len(args) == 3 and args[1] in ("0", "1"):
            rs = _regset(args[0])
            val = self.regs.get(frozenset([args[2]]))
            self.clobber(rs, line)
            if rs is not None and val is not None:
                t = val if isinstance(val, tuple) else (val != 0)
                same = (op == "v_cmp_eq_u32_e64") == (args[1] == "1")  # D = vX (== 1 / != 0) or its negation
                if isinstance(t, tuple):
                    self.regs[rs] = t if same else ("p", t[1], not t[2])
                else:
                    self.regs[rs] = -1 if (t == same) else 0
            return
        # generic: the first operand of most instructions is the destination
        if args and re.match(r"^v(\d+|\[)", args[0]):
            self.regs.pop(frozenset([args[0]]), None)
        if args:
            rs = _regset(args[0])
            if rs is not None and not op.startswith(("s_cmp", "s_bitcmp")):
                self.clobber(rs, line)
            if op.startswith("v_") and len(args) > 1 and args[1] in ("vcc", "vcc_lo"):
                self.clobber(frozenset(["vcc"]), line)
        if op.startswith("s_") and not op.startswith(_NO_SCC):
            self.scc = None

    def branch(self, edge) -> "Ctx | None":
        """This context along a CFG edge, or None if the scalar facts rule the edge out."""
        if edge is None:
            return self
        kind, op = edge
        cond = {"s_cbranch_scc1": ("scc", True), "s_cbranch_scc0": ("scc", False),
                "s_cbranch_vccnz": ("vcc", True), "s_cbranch_vccz": ("vcc", False)}.get(op)
        if cond is None:
            return self
        attr, want = cond
        if kind == "fall":
            want = not want
        val = self.resolve(getattr(self, attr))
        if isinstance(val, bool):
            return self if val == want else None
        if isinstance(val, tuple):
            c = self.copy()
            c.facts[val[1]] = want == val[2]
            setattr(c, attr, want)
            return c
        return self


def join(a: dict | None, b: dict) -> dict:
    """Elementwise min of two tag states {tag: [instance {cond: younger-min}]} (cond None = every path)."""
    if a is None:
        return {t: [dict(i) for i in v] for t, v in b.items()}
    out = {}
    for t in set(a) | set(b):
        va, vb = a.get(t, []), b.get(t, [])
        n = max(len(va), len(vb))
        lst = []
        for i in range(n):
            x = va[i] if i < len(va) else {}
            y = vb[i] if i < len(vb) else {}
            lst.append({c: min(x.get(c, INF), y.get(c, INF)) for c in set(x) | set(y)})
        out[t] = lst
    return out


def step(state: dict, ins, report=None, known=frozenset(), conds=frozenset()) -> dict:
    """Tag-state transfer of one instruction.  An instance is {None: min younger over all paths, c: min younger over
    the paths on which group c was tagged after the instance} for the conditions c the waits name ("p1:2@epi")."""
    kind, pay, ln = ins
    if kind == "vmem":
        for t, v in state.items():
            state[t] = [{c: (INF if (d == INF or d + 1 >= 64) else d + 1) for c, d in inst.items()} for inst in v]
    elif kind == "svtag":
        for t in pay:
            if t in conds:  # every instance of every group now has t after it on these paths
                for u, v in state.items():
                    for inst in v:
                        inst[t] = min(inst.get(t, INF), inst.get(None, INF))
            state[t] = ([{None: 0}] + state.get(t, []))[:MAXI]
    elif kind in ("wait", "svcheck"):
        n, targets = (pay if kind == "wait" else (None, pay))
        if report is not None:
            for tk in targets:
                tk0, _, cond = tk.partition("@")
                name, _, k = tk0.partition(":")
                k = int(k or 1)
                v = state.get(name)
                inst = v[k - 1] if v is not None and k - 1 < len(v) else {}
                have = inst.get(cond or None, INF)
                ok = have == INF or (n is not None and have >= n)
                report.append({"line": ln, "target": tk, "vmcnt": n, "younger_min": None if have == INF else have,
                               "ok": ok, "known": name in known and (not cond or cond in known)})
        if n is not None:
            for t, v in state.items():
                state[t] = [{c: (INF if (d == INF or d >= n) else d) for c, d in inst.items()} for inst in v]
    return state


def check_kernel(lines: list[str], max_ctx: int = 256, witness: bool = False) -> list[dict]:
    blocks = parse(lines)
    known = frozenset(t for b in blocks for k, p, _ in b["ins"] if k == "svtag" for t in p)
    conds = frozenset(tk.partition("@")[2] for b in blocks for k, p, _ in b["ins"] if k in ("wait", "svcheck")
                      for tk in (p[1] if k == "wait" else p) if "@" in tk)
    if not any(k in ("wait", "svcheck") and (k == "svcheck" or p[1]) for b in blocks for k, p, _ in b["ins"]):
        return []
    Ctx.keep = interesting_regs(blocks)
    cnt = set()
    for b in blocks:
        for k, p, _ in b["ins"]:
            if k == "op" and p.startswith(("s_cmp_", "s_cmpk_")):
                a = p.replace(",", " ").split()
                if len(a) == 3 and (_imm(a[1]) is not None) != (_imm(a[2]) is not None):
                    rs = _regset(a[2] if _imm(a[1]) is not None else a[1])
                    if rs is not None:
                        cnt |= set(rs)
    Ctx.counters = frozenset(cnt)
    for b in blocks:
        b["tag_ins"] = [i for i in b["ins"] if i[0] != "op"]
        b["ops"] = [i for i in b["ins"] if i[0] == "op"]
    # the scalar-fact transfer of a block depends only on its input context: memoised per (block, context)
    ctx_memo: dict = {}

    def ctx_edges(k, ctx, key):
        r = ctx_memo.get((k, key))
        if r is None:
            c = ctx.copy()
            for ins in blocks[k]["ops"]:
                c.op(ins[1], ins[2])
            r = []
            for s_, edge in blocks[k]["succ_idx"]:
                c3 = c.branch(edge)
                if c3 is not None:
                    r.append((s_, c3, c3.key()))
            ctx_memo[(k, key)] = r
        return r

    def tags(k, st, report=None):
        st = {t: [dict(i) for i in v] for t, v in st.items()}
        for ins in blocks[k]["tag_ins"]:
            st = step(st, ins, report, known, conds)
        return st

    # per block: {ctx key: (Ctx, tag state)}; path classes with equal scalar facts are merged (min)
    inp: list[dict] = [dict() for _ in blocks]
    src: list[dict] = [dict() for _ in blocks]
    c0 = Ctx()
    inp[0][c0.key()] = (c0, {})
    work = {0}
    while work:
        k = min(work)
        work.discard(k)
        for key, (ctx, st) in list(inp[k].items()):
            st2 = tags(k, st)
            for s_, c3, key3 in ctx_edges(k, ctx, key):
                cur = inp[s_].get(key3)
                if cur is None and len(inp[s_]) >= max_ctx:  # too many path classes: merge into a fact-free one
                    c3 = Ctx()
                    key3 = c3.key()
                    cur = inp[s_].get(key3)
                nj = join(cur[1] if cur else None, st2)
                if cur is None or nj != cur[1]:
                    inp[s_][key3] = (c3, nj)
                    src[s_][key3] = (k, key)
                    work.add(s_)
    rep: list[dict] = []
    for k in range(len(blocks)):
        for key, (ctx, st) in inp[k].items():
            n0 = len(rep)
            tags(k, st, rep)
            if witness:
                for r in rep[n0:]:
                    if not r["ok"]:
                        path, b, kk = [], k, key
                        while kk in src[b] and len(path) < 80:
                            path.append(blocks[b]["label"])
                            b, kk = src[b][kk]
                        r["witness"] = list(reversed(path))
    worst: dict = {}
    for r in rep:
        key = (r["line"], r["target"])
        if key not in worst or (not r["ok"] and worst[key]["ok"]) or (
                r["ok"] == worst[key]["ok"] and (r["younger_min"] or INF) < (worst[key]["younger_min"] or INF)):
            worst[key] = r
    return sorted(worst.values(), key=lambda r: (r["line"], r["target"]))


def _check_one(args):
    name, lines, witness = args
    return name, check_kernel(lines, witness=witness)


def check_text(text: str, witness: bool = False, only: str | None = None, jobs: int | None = None) -> dict[str, list[dict]]:
    """Per kernel (that carries checked waits): its report rows.  Kernels are checked in parallel processes."""
    todo = [(n, ln, witness) for n, ln in split_kernels(text).items()
            if (only is None or only in n) and any("svwait" in x or "svcheck" in x for x in ln)]
    jobs = jobs or min(len(todo), os.cpu_count() or 1, 8)
    if jobs <= 1:
        res = [_check_one(t) for t in todo]
    else:
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(max_workers=jobs) as ex:
            res = list(ex.map(_check_one, todo, chunksize=1))
    return {n: r for n, r in res if r}


# Groups whose LOADED REGISTERS must not be touched above the group's own counted wait (``svwait g:1``): the
# compiler waits for such a consumer with a vmcnt of its own, counted on in-order retirement behind the younger
# stores and LDS-DMA, and the fused MLP backward's dz / dw then differed run to run (DESIGN "Round 6", r15a-c).
# group -> the load opcodes that make it up (the contiguous run of those loads just before ``svtag g``).
EARLY_USE_GROUPS = {"zl": ("buffer_load_dword", "buffer_load_dwordx2")}
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _vregs(text: str) -> set[int]:
    out: set[int] = set()
    for m in _VREG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def check_early_use(lines: list[str], groups=EARLY_USE_GROUPS) -> list[dict]:
    """Per group tag found in the kernel: the instructions between the group's loads and its ``svwait g:1`` (text
    order) that read or write a register those loads fill.  A row with ``uses`` non-empty fails."""
    body = [ln.split(";")[0].strip() if not re.search(r";\s*sv(tag|wait)", ln) else ln.strip() for ln in lines]
    rows = []
    for g, ops in groups.items():
        for ti, ln in enumerate(body):
            if not re.search(rf";\s*svtag\s+{re.escape(g)}\b", ln):
                continue
            loads, regs, j = [], set(), ti - 1
            while j >= 0:
                op = body[j].split()[0] if body[j] else ""
                if VMEM.match(op) or body[j].startswith(";") and "svtag" in body[j]:
                    if op not in ops:
                        break
                    loads.append(j)
                    regs |= _vregs(body[j].split(None, 1)[1].split(",")[0])
                j -= 1
            if not loads:
                rows.append({"group": g, "line": ti, "loads": 0, "uses": [], "wait": None})
                continue
            wait = next((k for k in range(ti + 1, len(body)) if re.search(rf"svwait\b.*\b{re.escape(g)}:1\b", body[k])),
                        None)
            end = wait if wait is not None else len(body)
            uses = []
            for k in range(min(loads) + 1, end):
                if k in loads or not body[k] or body[k].startswith((";", ".")) or body[k].endswith(":"):
                    continue
                parts = body[k].split(None, 1)
                if len(parts) > 1 and _vregs(parts[1]) & regs:
                    uses.append((k, body[k]))
            rows.append({"group": g, "line": ti, "loads": len(loads), "uses": uses, "wait": wait})
    return rows


def check_early_use_text(text: str) -> dict[str, list[dict]]:
    """Kernel symbol -> check_early_use rows, for every kernel carrying a tag of an EARLY_USE_GROUPS group."""
    out = {}
    for n, ln in split_kernels(text).items():
        if any(re.search(rf";\s*svtag\s+{re.escape(g)}\b", x) for x in ln for g in EARLY_USE_GROUPS):
            out[n] = check_early_use(ln)
    return out


def build_asm(srcs=CHECKED_SOURCES, defines=()) -> dict[str, str]:
    """Device assembly of the checked sources with build_native()'s flags (hipcc -S --cuda-device-only), plus
    ``defines`` (e.g. ``("-DSV_MLPB_PIN=0",)`` for an A/B build)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge

    from concurrent.futures import ThreadPoolExecutor

    out = {}
    with tempfile.TemporaryDirectory() as td:
        def one(src):
            path = os.path.join(ge.CSRC, src)
            s_out = os.path.join(td, src + ".s")
            cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")] + ge.compile_flags(src) + list(defines) + [
                "--cuda-device-only", "-S", path, "-o", s_out]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc -S failed on {src}:\n{r.stderr}")
            return src, open(s_out).read()

        with ThreadPoolExecutor(max_workers=len(srcs)) as ex:
            out = dict(ex.map(one, srcs))
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("files", nargs="*")
    ap.add_argument("--build", action="store_true", help="compile csrc/{mlp,gemm9}.hip to assembly and check them")
    ap.add_argument("--json", help="write the per-kernel report here")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--witness", action="store_true", help="print a block path for each failing wait")
    ap.add_argument("--only", help="check only kernels whose symbol contains this string")
    a = ap.parse_args()
    texts = {f: open(f).read() for f in a.files}
    if a.build:
        texts.update(build_asm())
    bad = 0
    full = {}
    for f, text in texts.items():
        res = check_text(text, a.witness, a.only)
        full[f] = res
        for kern, rows in res.items():
            nbad = sum(1 for r in rows if not r["ok"] or not r["known"])
            bad += nbad
            slack = [r["younger_min"] - r["vmcnt"] for r in rows if r["younger_min"] is not None and r["vmcnt"] is not None]
            print(f"{'FAIL' if nbad else 'ok  '} {f}: {kern[:90]}  {len(rows)} checked waits"
                  + (f", min slack {min(slack)}" if slack else ""))
            if nbad or a.v:
                for r in rows:
                    if a.v or not r["ok"] or not r["known"]:
                        print(f"      line {r['line']}: vmcnt({r['vmcnt']}) must retire {r['target']}: "
                              f"{'retired' if r['younger_min'] is None else str(r['younger_min']) + ' younger (min over paths)'}"
                              f"{'' if r['known'] else '  [unknown group]'}{'' if r['ok'] else '  <-- OUTSTANDING'}")
                        if r.get("witness"):
                            print("        witness (block labels):", " ".join(r["witness"][-40:]))
        for kern, rows in check_early_use_text(text).items():
            for r in rows:
                ok = r["loads"] and r["wait"] is not None and not r["uses"]
                bad += not ok
                print(f"{'ok  ' if ok else 'FAIL'} {f}: {kern[:90]}  group {r['group']}: {r['loads']} loads, "
                      f"{len(r['uses'])} uses above their svwait")
                for k, ins in r["uses"][:8]:
                    print(f"      line {k}: {ins}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(full, fh, indent=1)
    if not any(full.values()):
        print("no checked waits found")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
