#!/usr/bin/env python3
"""Static float data-flow extraction from a reference object file (study tool; build container
only — it needs /root/reference, which never reaches the GPU box).

The reference's objects are READ AS DATA (`objdump -d` text): nothing is executed, emulated on
concrete values or linked.  The tool walks one straight-line instruction range symbolically and
prints, as SSA, the expression every scalar float/double store, compare and return value is
made of — which products GCC 9.3 contracted into FMAs (`-O3 -march=native`, reference
evaluation/CMakeFiles/ORB_SLAM3.dir/flags.make:5), in which order sums associate, where float
is widened to double.  The oracle's and the kernels' restatements (explicit fmaf / fma) are
written from this listing; tests/test_fp_sites.py checks them against C code emitted by
`--emit-c` from the same listing (oracle/_ref/, git-ignored, only when /root/reference exists).

    python3 tools/disasm/fptrace.py OBJ 'FUNC substring' START END [--names a=rdx+0x0,...]
                                    [--emit-c NAME --inputs v1,v2,... --outputs o1,o2,...]

Branches are not followed: a conditional jump falls through, which is what the gates of the
traced functions do on their accepting path.  Supported: the scalar SSE/AVX/FMA subset GCC
emits for these functions (vmov*, vadd/sub/mul/div/sqrt ss/sd, vfm*/vfnm* 132/213/231,
vcvt*, vxorps sign flips, vucomis/vcomis, 32-bit GPR moves and stack copies).
"""
from __future__ import annotations

import argparse
import re
import struct
import subprocess
import sys

REG64 = {"rax", "rbx", "rcx", "rdx", "rsi", "rdi", "rbp", "rsp", "r8", "r9", "r10", "r11", "r12",
         "r13", "r14", "r15"}
R32 = {"eax": "rax", "ebx": "rbx", "ecx": "rcx", "edx": "rdx", "esi": "rsi", "edi": "rdi",
       "ebp": "rbp", "r8d": "r8", "r9d": "r9", "r10d": "r10", "r11d": "r11", "r12d": "r12",
       "r13d": "r13", "r14d": "r14", "r15d": "r15"}


class Node:
    __slots__ = ("op", "args", "ty", "id", "name")

    def __init__(self, op, args, ty, name=None):
        self.op, self.args, self.ty, self.id, self.name = op, tuple(args), ty, None, name


class Tracer:
    def __init__(self, obj, names, packed=False):
        self.obj = obj
        self.packed = packed    # round 5: packed-double instructions and untyped vector moves
        self.sret_slots = {"_transformVector": 6, "cam_project": 6, "*0x50": 12} if packed else {}
        self.nodes = []
        self.memo = {}
        self.regs = {}          # xmmN -> [lane0..lane3] (lane0 of a double holds the f64 node)
        self.gpr = {"rsp": ("rsp", 0)}
        self.mem = {}           # (base, off) -> node (4-byte granularity; f64 at off, 'hi' at off+4)
        self.events = []
        self.names = names
        self.consts = self._load_consts()
        self.ncall = 0

    # ---- constants from .rodata.cst* (read as data) ----
    def _load_consts(self):
        syms = {}
        out = subprocess.run(["objdump", "-t", self.obj], capture_output=True, text=True).stdout
        for line in out.splitlines():
            m = re.match(r"^([0-9a-f]+)\s+l\s+(\S+)\s+[0-9a-f]+\s+(\.LC\d+)$", line.strip())
            if m:
                syms[m.group(3)] = (m.group(2), int(m.group(1), 16))
        secs = {}
        out = subprocess.run(["objdump", "-s", "-j", ".rodata.cst4", "-j", ".rodata.cst8",
                              "-j", ".rodata.cst16", "-j", ".rodata.cst32", self.obj],
                             capture_output=True, text=True).stdout
        cur = None
        for line in out.splitlines():
            m = re.match(r"^Contents of section (\S+):", line)
            if m:
                cur = m.group(1)
                secs[cur] = bytearray()
                continue
            m = re.match(r"^ ([0-9a-f]{4,}) ((?:[0-9a-f]{2,8} ?)+)", line)
            if cur and m:
                hexs = "".join(m.group(2).split())
                secs[cur] += bytes.fromhex(hexs)
        self.secs = secs
        return syms

    def const_bytes(self, reloc, n):
        m = re.match(r"(\.LC\d+|\.rodata\.cst\d+)([+-]0x[0-9a-f]+)?", reloc)
        sym, add = m.group(1), int(m.group(2) or "0", 16)
        # RIP-relative PC32: target = S + A + 4 (the displacement ends the instruction)
        sec, off = self.consts[sym] if sym.startswith(".LC") else (sym, 0)
        base = off + add + 4
        return bytes(self.secs[sec][base: base + n])

    # ---- node construction with hash-consing ----
    def mk(self, op, args, ty, name=None):
        key = (op, tuple(id(a) for a in args), ty, name)
        if key in self.memo:
            return self.memo[key]
        n = Node(op, args, ty, name)
        self.memo[key] = n
        self.nodes.append(n)
        return n

    def inp(self, where, ty):
        nm = self.names.get(where, where)
        return self.mk("in", [], ty, nm)

    def const(self, val, ty):
        return self.mk("const", [], ty, repr(val))

    # ---- operands ----
    def addr(self, s, reloc):
        if "%rip" in s:
            return ("const", reloc)
        m = re.match(r"^(-?0x[0-9a-f]+|-?\d+)?\(%(\w+)(?:,%(\w+),(\d))?\)$", s)
        if not m:
            raise ValueError("addr " + s)
        disp = int(m.group(1), 16) if m.group(1) and "x" in m.group(1) else int(m.group(1) or 0)
        base = m.group(2)
        if m.group(3):
            return ("dyn", s)
        b = self.gpr.get(base)
        if b is None:
            b = ("arg_" + base, 0)
            self.gpr[base] = b
        return (b[0], b[1] + disp)

    @staticmethod
    def where(a):
        if isinstance(a[1], str):
            return a[1]
        return f"{a[0]}+0x{a[1]:x}" if a[1] >= 0 else f"{a[0]}-0x{-a[1]:x}"

    def load32(self, a, ty="f32"):
        if a[0] == "const":
            return None
        key = (a[0], a[1])
        v = self.mem.get(key)
        if v is None:
            v = self.inp(self.where(a), ty)
            self.mem[key] = v
        elif v.ty == "raw" and ty != "raw":
            v = self.inp(v.name, ty)
        return v

    # ---- untyped 4-byte slots (round 5: packed doubles) ----
    # Vector moves copy memory without saying what it holds: a slot never written is read as a
    # "raw" node named by its address, typed when an instruction consumes it (f32: the slot, f64:
    # the slot pair whose low half it is).  A double lives in slot 2k of a register (slot 2k + 1 is
    # its high half, None).
    def raw(self, a):
        key = (a[0], a[1])
        v = self.mem.get(key)
        if v is None:
            v = self.mk("in", [], "raw", self.names.get(self.where(a), self.where(a)))
            self.mem[key] = v
        return v

    def as_f64(self, lanes, k):
        lo = lanes[2 * k]
        if lo is None:
            raise ValueError("f64 lane %d empty" % k)
        if lo.ty == "raw":
            return self.inp(lo.name, "f64")
        if lo.ty == "f32" and lo.op == "const":  # a constant moved as f32 slots, consumed as f64
            hi = lanes[2 * k + 1]
            lo_b = struct.pack("<f", float(lo.name))
            hi_b = struct.pack("<f", float(hi.name)) if hi is not None and hi.op == "const" else b"\0\0\0\0"
            return self.const(struct.unpack("<d", lo_b + hi_b)[0], "f64")
        if lo.ty != "f64":
            raise ValueError("f64 use of %s" % lo.ty)
        return lo

    def sv(self, n, ty):
        """A scalar operand of type ty (a raw slot typed on use)."""
        if n is not None and n.ty == "raw":
            return self.inp(n.name, ty)
        return n

    def as_f32(self, n):
        if n is not None and n.ty == "raw":
            return self.inp(n.name, "f32")
        return n

    def load_pd(self, s, reloc, w):
        """w doubles from memory (or a RIP-relative constant) as register slots."""
        a = self.addr(s, reloc)
        lanes = [None] * 8
        if a[0] == "const":
            b = self.const_bytes(reloc, 8 * w)
            for k in range(w):
                lanes[2 * k] = self.const(struct.unpack("<d", b[8 * k:8 * k + 8])[0], "f64")
            return lanes
        for k in range(w):
            v = self.mem.get((a[0], a[1] + 8 * k))
            if v is None or v.ty == "raw":
                v = self.inp(v.name if v is not None else self.where((a[0], a[1] + 8 * k)), "f64")
                self.mem[(a[0], a[1] + 8 * k)] = v
            lanes[2 * k] = v
        return lanes

    def pd_operand(self, o, reloc, w):
        if o.endswith("}") and "{1to" in o:  # AVX-512 embedded broadcast of one double
            v = self.load_pd(o[:o.index("{")], reloc, 1)[0]
            return [v] * w
        if o[:4] in ("%xmm", "%ymm", "%zmm"):
            lanes = self.reg("xmm" + o[4:])
            return [self.as_f64(lanes, k) if lanes[2 * k] is not None else None for k in range(w)]
        lanes = self.load_pd(o, reloc, w)
        return [lanes[2 * k] for k in range(w)]

    def set_pd(self, d, vals):
        lanes = [None] * 8
        for k, v in enumerate(vals):
            lanes[2 * k] = v
        self.regs["xmm" + d[4:]] = lanes

    def step_pd(self, ins, ops, reloc):
        """Packed-double instructions (Eigen's vectorised 2x3 / 3x3 products).  Returns True when
        handled."""
        X = lambda o: o[:4] in ("%xmm", "%ymm", "%zmm")
        wid = lambda o: 4 if o.startswith("%ymm") else 2
        binop = {"vaddpd": "+", "vsubpd": "-", "vmulpd": "*", "vdivpd": "/"}
        if ins in binop:
            s2, s1, d = ops
            w = wid(d)
            b = self.pd_operand(s2, reloc, w)
            a = self.pd_operand(s1, reloc, w)
            self.set_pd(d, [self.mk(binop[ins], [x, y], "f64") if x is not None and y is not None else None
                            for x, y in zip(a, b)])
            return True
        m = re.match(r"^v(fn?m)(add|sub)(132|213|231)pd$", ins)
        if m:
            neg, sub, form = m.group(1) == "fnm", m.group(2) == "sub", m.group(3)
            o1, o2, d = ops
            w = wid(d)
            v1 = self.pd_operand(o1, reloc, w)
            v2 = self.pd_operand(o2, reloc, w)
            vd = self.pd_operand(d, reloc, w)
            out = []
            for k in range(w):
                if form == "132":
                    p, q, c = vd[k], v1[k], v2[k]
                elif form == "213":
                    p, q, c = v2[k], vd[k], v1[k]
                else:
                    p, q, c = v2[k], v1[k], vd[k]
                if p is None or q is None or c is None:
                    out.append(None)
                    continue
                if neg:
                    p = self.mk("neg", [p], "f64")
                if sub:
                    c = self.mk("neg", [c], "f64")
                out.append(self.mk("fma", [p, q, c], "f64"))
            self.set_pd(d, out)
            return True
        if ins == "vmovddup":
            s, d = ops
            v = self.pd_operand(s, reloc, 1)[0] if not X(s) else self.as_f64(self.reg("xmm" + s[4:]), 0)
            self.set_pd(d, [v, v] if wid(d) == 2 else [v, v, v, v])
            return True
        if ins in ("vunpckhpd", "vunpcklpd"):
            s2, s1, d = ops
            a = self.pd_operand(s1, reloc, 2)
            b = self.pd_operand(s2, reloc, 2)
            k = 1 if ins == "vunpckhpd" else 0
            self.set_pd(d, [a[k], b[k]])
            return True
        if ins == "vpermilpd":
            imm, s, d = ops
            imm = int(imm[1:], 16)
            w = wid(d)
            a = self.pd_operand(s, reloc, w)
            out = [a[(imm >> 0) & 1], a[(imm >> 1) & 1]]
            if w == 4:
                out += [a[2 + ((imm >> 2) & 1)], a[2 + ((imm >> 3) & 1)]]
            self.set_pd(d, out)
            return True
        if ins == "vpermpd":  # 4-lane permute by immediate (the packed quaternion products)
            imm, s_, d = ops
            imm = int(imm[1:], 16)
            a = self.pd_operand(s_, reloc, 4)
            self.set_pd(d, [a[(imm >> (2 * k)) & 3] for k in range(4)])
            return True
        if ins == "vblendpd":  # AT&T: $imm, src2, src1, dst -- lane k from src2 where bit k is set
            imm, s2, s1, d = ops
            imm = int(imm[1:], 16)
            w = wid(d)
            a = self.pd_operand(s1, reloc, w)
            b = self.pd_operand(s2, reloc, w)
            self.set_pd(d, [b[k] if (imm >> k) & 1 else a[k] for k in range(w)])
            return True
        if ins in ("vextractf64x2", "vextractf128"):
            imm, s_, d = ops
            imm = int(imm[1:], 16)
            a = self.pd_operand(s_, reloc, 4)
            self.set_pd(d, a[2 * imm:2 * imm + 2])
            return True
        if ins == "vbroadcastsd":
            s_, d = ops
            v = self.as_f64(self.reg("xmm" + s_[4:]), 0) if X(s_) else self.pd_operand(s_, reloc, 1)[0]
            self.set_pd(d, [v] * wid(d))
            return True
        if ins == "vmovq" and X(ops[0]) and X(ops[1]):  # low double kept, upper lane zeroed
            v = self.as_f64(self.reg("xmm" + ops[0][4:]), 0)
            self.set_pd(ops[1], [v, self.const(0.0, "f64")])
            return True
        if ins == "vxorpd" and ops[0] != ops[1]:
            s2, s1, d = ops
            w = wid(d)
            a = self.pd_operand(s1, reloc, w)
            b = self.pd_operand(s2, reloc, w)
            out = []
            for x, y in zip(a, b):
                if x is None or y is None:
                    out.append(None)
                    continue
                # one operand is the sign-mask constant (-0.0: negate) or +0.0 (no-op)
                mask, val = (x, y) if x.op == "const" else (y, x)
                if mask.op != "const" or float(mask.name) != 0.0:
                    raise ValueError("vxorpd without a sign-mask operand")
                neg = struct.pack("<d", float(mask.name)) == struct.pack("<d", -0.0)
                out.append(self.mk("neg", [val], "f64") if neg else val)
            self.set_pd(d, out)
            return True
        if ins in ("vmovapd", "vmovupd") and X(ops[1]) and not X(ops[0]):
            w = wid(ops[1])
            self.regs["xmm" + ops[1][4:]] = self.load_pd(ops[0], reloc, w)
            return True
        if ins == "vmovq" and "%rip" in ops[0] and X(ops[1]):
            b = self.const_bytes(reloc, 8)
            self.set_pd(ops[1], [self.const(struct.unpack("<d", b)[0], "f64"), self.const(0.0, "f64")])
            return True
        return False

    def load_scalar(self, s, reloc, ty):
        a = self.addr(s, reloc)
        if a[0] == "const":
            b = self.const_bytes(reloc, 4 if ty == "f32" else 8)
            return self.const(struct.unpack("<f" if ty == "f32" else "<d", b)[0], ty)
        if ty == "f64":
            v = self.mem.get((a[0], a[1]))
            if v is not None and v.ty == "f64":
                return v
            if v is not None and v.ty == "raw":
                return self.inp(v.name, "f64")
            if v is None:
                v = self.inp(self.where(a), "f64")
                self.mem[(a[0], a[1])] = v
                return v
            raise ValueError("f64 load of f32 data at %r" % (a,))
        return self.load32(a)

    def reg(self, r):
        if r not in self.regs:
            self.regs[r] = [self.inp("%" + r, "f32")] + [None] * 7
        lanes = self.regs[r]
        if len(lanes) < 8:
            lanes = self.regs[r] = list(lanes) + [None] * (8 - len(lanes))
        return lanes

    # ---- events ----
    def event(self, kind, *nodes, extra=""):
        self.events.append((kind, nodes, extra))

    def run(self, lines):
        for addr, ins, ops, reloc in lines:
            try:
                self.step(addr, ins, ops, reloc)
            except Exception as e:  # pragma: no cover - study tool
                print(f"# {addr:x}: unsupported {ins} {ops}: {e}", file=sys.stderr)

    def step(self, addr, ins, ops, reloc):
        X = lambda o: o[:4] in ("%xmm", "%ymm", "%zmm")
        R = lambda o: "xmm" + o[4:] if o[:4] in ("%xmm", "%ymm", "%zmm") else o[1:]
        W = lambda o: 8 if o.startswith("%ymm") else 4
        binop = {"vaddss": "+", "vsubss": "-", "vmulss": "*", "vdivss": "/",
                 "vaddsd": "+", "vsubsd": "-", "vmulsd": "*", "vdivsd": "/",
                 "vminss": "min", "vmaxss": "max", "vminsd": "min", "vmaxsd": "max"}
        if self.packed and self.step_pd(ins, ops, reloc):
            return
        if ins in ("vmovss", "vmovsd"):
            ty = "f32" if ins == "vmovss" else "f64"
            if len(ops) == 2 and X(ops[1]) and not X(ops[0]):
                v = self.load_scalar(ops[0], reloc, ty)
                self.regs[R(ops[1])] = [v, None, None, None]
            elif len(ops) == 2 and X(ops[0]) and not X(ops[1]):
                a = self.addr(ops[1], reloc)
                v = self.reg(R(ops[0]))[0]
                self.mem[(a[0], a[1])] = v
                if ty == "f64":
                    self.mem[(a[0], a[1] + 4)] = None
                self.event("store", v, extra=self.where(a))
            elif len(ops) == 2:
                self.regs[R(ops[1])] = list(self.reg(R(ops[0])))
            else:
                src, other, dst = ops
                lanes = list(self.reg(R(other)))
                lanes[0] = self.reg(R(src))[0]
                self.regs[R(dst)] = lanes
            return
        if ins in ("vmovaps", "vmovups", "vmovdqa64", "vmovdqu64", "vmovdqa", "vmovdqu",
                   "vmovapd", "vmovupd", "vmovdqa32", "vmovdqu32"):
            src, dst = ops
            w = max(W(src), W(dst))
            if X(src) and X(dst):
                self.regs[R(dst)] = list(self.reg(R(src)))
            elif X(dst):
                a = self.addr(src, reloc)
                if a[0] == "const":
                    cb = self.const_bytes(reloc, 4 * w)
                    self.regs[R(dst)] = [self.const(struct.unpack("<f", cb[4 * k:4 * k + 4])[0], "f32") for k in range(w)] + [None] * (8 - w)
                elif self.packed:
                    self.regs[R(dst)] = [self.raw((a[0], a[1] + 4 * k)) for k in range(w)] + [None] * (8 - w)
                else:
                    self.regs[R(dst)] = [self.load32((a[0], a[1] + 4 * k)) for k in range(w)] + [None] * (8 - w)
            else:
                a = self.addr(dst, reloc)
                lanes = self.reg(R(src))
                for k in range(w):
                    self.mem[(a[0], a[1] + 4 * k)] = lanes[k]
                    if lanes[k] is not None and lanes[k].op not in ("in", "const"):
                        self.event("store", lanes[k], extra=self.where((a[0], a[1] + 4 * k)))
            return
        if ins in ("vmovq", "vmovd"):
            src, dst = ops
            n = 2 if ins == "vmovq" else 1
            if X(src) and not X(dst):
                if dst.startswith("%"):
                    self.gpr[R(dst)] = ("xmmval", self.reg(R(src))[:n])
                    return
                a = self.addr(dst, reloc)
                lanes = self.reg(R(src))
                for k in range(n):
                    self.mem[(a[0], a[1] + 4 * k)] = lanes[k]
            elif X(dst):
                if src.startswith("%"):
                    g = self.gpr.get(R(src))
                    if g and g[0] == "constq":
                        self.regs[R(dst)] = [self.const(g[1], "f64")] + [None] * 7
                        return
                    self.regs[R(dst)] = (list(g[1]) + [None] * 4)[:4] if g and g[0] == "xmmval" else [None] * 4
                    return
                a = self.addr(src, reloc)
                self.regs[R(dst)] = [self.load32((a[0], a[1] + 4 * k)) for k in range(n)] + [None] * (4 - n)
            return
        if ins in ("vandps", "vandpd"):
            a, b, d = ops  # and with an abs mask constant: fabs
            src = self.reg(R(b))
            if "%rip" in a:
                word = struct.unpack("<I", self.const_bytes(reloc, 4))[0]
                assert word == 0x7fffffff, hex(word)
            lanes = list(src)
            lanes[0] = self.mk("fabs", [src[0]], src[0].ty)
            self.regs[R(d)] = lanes
            return
        if ins in ("vxorps", "vxorpd", "vpxor", "vpxord", "vpxorq"):
            a, b, d = ops
            if a == b:
                ty = "f64" if ins == "vxorpd" else "f32"
                self.regs[R(d)] = [self.const(0.0, ty)] * 8
            else:
                # xor with a sign-mask constant: lane-wise negation (checked against the bytes)
                w = W(d)
                mask = self.const_bytes(reloc, 4 * w) if "%rip" in a else None
                src = self.reg(R(b))
                lanes = []
                for k in range(8):
                    if k < w and src[k] is not None:
                        if mask is not None:
                            word = struct.unpack("<I", mask[4 * k:4 * k + 4])[0]
                            if ins == "vxorpd":
                                assert mask[4 * k:4 * k + 4] in (b"\x00\x00\x00\x00", b"\x00\x00\x00\x80"), mask
                            else:
                                assert word == 0x80000000, hex(word)
                        lanes.append(self.mk("neg", [src[k]], src[k].ty))
                    else:
                        lanes.append(None)
                self.regs[R(d)] = lanes
            return
        if ins in binop:
            s2, s1, d = ops
            ty = "f32" if ins.endswith("ss") else "f64"
            b = self.sv(self.reg(R(s2))[0], ty) if X(s2) else self.load_scalar(s2, reloc, ty)
            a = self.reg(R(s1))
            lanes = list(a)
            lanes[0] = self.mk(binop[ins], [self.sv(a[0], ty), b], ty)
            self.regs[R(d)] = lanes
            return
        if ins in ("vsqrtss", "vsqrtsd"):
            s2, s1, d = ops
            ty = "f32" if ins.endswith("ss") else "f64"
            b = self.reg(R(s2))[0] if X(s2) else self.load_scalar(s2, reloc, ty)
            lanes = list(self.reg(R(s1)))
            lanes[0] = self.mk("sqrt", [b], ty)
            self.regs[R(d)] = lanes
            return
        m = re.match(r"^v(fn?m)(add|sub)(132|213|231)s([sd])$", ins)
        if m:
            neg = m.group(1) == "fnm"
            sub = m.group(2) == "sub"
            form = m.group(3)
            ty = "f32" if m.group(4) == "s" else "f64"
            o1, o2, d = ops
            v1 = self.sv(self.reg(R(o1))[0], ty) if X(o1) else self.load_scalar(o1, reloc, ty)
            v2 = self.sv(self.reg(R(o2))[0], ty)
            vd = self.sv(self.reg(R(d))[0], ty)
            if form == "132":  # AT&T operand order: (op1, op2, dst)
                p, q, c = vd, v1, v2
            elif form == "213":
                p, q, c = v2, vd, v1
            else:
                p, q, c = v2, v1, vd
            if neg:
                p = self.mk("neg", [p], ty)
            if sub:
                c = self.mk("neg", [c], ty)
            lanes = list(self.reg(R(d)))
            lanes[0] = self.mk("fma", [p, q, c], ty)
            self.regs[R(d)] = lanes
            return
        if ins in ("vcvtss2sd", "vcvtsd2ss"):
            s, o, d = ops
            src_ty, ty = ("f32", "f64") if ins == "vcvtss2sd" else ("f64", "f32")
            v = self.sv(self.reg(R(s))[0], src_ty) if X(s) else self.load_scalar(s, reloc, src_ty)
            lanes = list(self.reg(R(o)))
            lanes[0] = self.mk("cvt", [v], ty)
            self.regs[R(d)] = lanes
            return
        if ins in ("vcvtsi2ss", "vcvtsi2sd", "vcvtsi2ssl", "vcvtsi2sdl"):
            s, o, d = ops
            ty = "f32" if "ss" in ins else "f64"
            g = self.gpr.get(R(s)) if s.startswith("%") else None
            v = g[1] if g and g[0] == "ival" else self.inp("int " + s, "i32")
            lanes = list(self.reg(R(o)))
            lanes[0] = self.mk("i2f", [v], ty)
            self.regs[R(d)] = lanes
            return
        if ins in ("vcvttss2si", "vcvtss2si", "vcvttsd2si", "vcvtsd2si"):
            s, d = ops
            v = self.reg(R(s))[0] if X(s) else self.load_scalar(s, reloc, "f64" if "sd2" in ins else "f32")
            op = "trunc" if "tt" in ins else "rint"
            n = self.mk(op, [v], "i32")
            self.gpr[R32.get(R(d), R(d))] = ("ival", n)
            self.event("int", n, extra=d)
            return
        if ins in ("vrndscaless", "vrndscalesd", "vroundss", "vroundsd"):
            imm, s, o, d = ops
            mode = {"$0xa": "ceil", "$0x9": "floor", "$0xb": "trunc", "$0x8": "rint", "$0xc": "rint",
                    "$0x4": "rint", "$0x1": "floor", "$0x2": "ceil"}.get(imm, "round" + imm)
            v = self.reg(R(s))[0]
            lanes = list(self.reg(R(o)))
            lanes[0] = self.mk(mode, [v], v.ty)
            self.regs[R(d)] = lanes
            return
        if ins in ("vucomiss", "vcomiss", "vucomisd", "vcomisd"):
            a, b = ops
            ty = "f32" if ins.endswith("ss") else "f64"
            va = self.reg(R(a))[0] if X(a) else self.load_scalar(a, reloc, ty)
            vb = self.reg(R(b))[0]
            self.event("cmp", vb, va, extra="(first ? second; branch follows)")
            return
        if ins in ("mov", "movl", "movq", "movabs", "lea"):
            src, dst = ops
            if ins == "lea":
                self.gpr[R(dst)] = self.addr(src, reloc)
                return
            if src.startswith("$"):
                imm = int(src[1:], 16)
                if dst.startswith("%"):
                    self.gpr[R32.get(R(dst), R(dst))] = ("imm", imm)
                    return
                a = self.addr(dst, reloc)
                if ins == "movl":
                    self.mem[(a[0], a[1])] = self.const(struct.unpack("<f", struct.pack("<I", imm & 0xffffffff))[0], "f32")
                else:
                    lo = imm & 0xffffffff
                    hi = (imm >> 32) & 0xffffffff if imm >= 0 else 0xffffffff
                    self.mem[(a[0], a[1])] = self.const(struct.unpack("<f", struct.pack("<I", lo))[0], "f32")
                    self.mem[(a[0], a[1] + 4)] = self.const(struct.unpack("<f", struct.pack("<I", hi))[0], "f32")
                return
            if src.startswith("%") and dst.startswith("%"):
                s = R32.get(R(src), R(src))
                self.gpr[R32.get(R(dst), R(dst))] = self.gpr.get(s, ("arg_" + s, 0))
                return
            if dst.startswith("%"):
                d = R(dst)
                a = self.addr(src, reloc)
                if a[0] == "const":
                    # a 64-bit constant moved through a GPR (`mov .LCn(%rip),%rax; vmovq %rax,%xmm0`)
                    try:
                        self.gpr[R32.get(d, d)] = ("constq", struct.unpack("<d", self.const_bytes(reloc, 8))[0])
                    except Exception:
                        self.gpr[R32.get(d, d)] = ("got:" + str(reloc), 0)
                    return
                if d in R32:
                    self.gpr[R32[d]] = ("m32", self.load32(a) if a[0] != "const" else None)
                else:
                    self.gpr[d] = (f"*({a[0]}+0x{a[1]:x})" if a[0] != "dyn" else a[1], 0)
                return
            s = R(src)
            a = self.addr(dst, reloc)
            g = self.gpr.get(R32.get(s, s))
            if s in R32 and g and g[0] == "m32":
                self.mem[(a[0], a[1])] = g[1]
            elif g and g[0] == "imm":
                self.mem[(a[0], a[1])] = self.const(struct.unpack("<f", struct.pack("<I", g[1] & 0xffffffff))[0], "f32")
                if s not in R32:
                    hi = (g[1] >> 32) & 0xffffffff
                    self.mem[(a[0], a[1] + 4)] = self.const(struct.unpack("<f", struct.pack("<I", hi))[0], "f32")
            return
        if ins.startswith("call"):
            self.ncall += 1
            callee = (reloc or " ".join(ops)).split("(")[0].replace("-0x4", "").split("::")[-1]
            tag = f"{callee}#{self.ncall}"
            self.event("call", extra=tag)
            if callee in ("sincos", "pow") and self.packed:
                # glibc's sincos(x, &s, &c) / pow(x, y) as pure functions of their arguments (the
                # emitted C calls the same glibc; SE3Quat::exp, round 6)
                x = self.as_f64(self.reg("xmm0"), 0)
                if callee == "pow":
                    y = self.as_f64(self.reg("xmm1"), 0)
                    res = self.mk("pow", [x, y], "f64")
                    for k in range(32):
                        self.regs.pop(f"xmm{k}", None)
                    self.set_pd("%xmm0", [res, None])
                    return
                for reg, fn in (("rdi", "sin"), ("rsi", "cos")):
                    g = self.gpr.get(reg)
                    a = (g[0], g[1])
                    self.mem[a] = self.mk(fn, [x], "f64")
                    self.mem[(a[0], a[1] + 4)] = None
                for k in range(32):
                    self.regs.pop(f"xmm{k}", None)
                return
            if callee in ("roundf", "round", "floorf", "ceilf"):  # pure libm: its value, not an input
                x = self.reg("xmm0")[0]
                res = self.mk(callee, [x], "f32" if callee.endswith("f") else "f64")
                for k in range(32):
                    self.regs.pop(f"xmm{k}", None)
                self.regs["xmm0"] = [res] + [None] * 7
                return
            for k in range(32):
                self.regs.pop(f"xmm{k}", None)
            dret = any(k in callee for k in ("normL2Sqr", "sqrt", "pow", "log", "exp"))
            self.regs["xmm0"] = ([self.inp(f"{tag}.xmm0d", "f64")] if dret else
                                 [self.inp(f"{tag}.xmm0[{k}]", "f32") for k in range(4)]) + [None] * 4
            self.regs["xmm1"] = [self.inp(f"{tag}.xmm1[{k}]", "f32") for k in range(4)] + [None] * 4
            rdi = self.gpr.get("rdi")
            # a callee returning a class by value writes it through the hidden pointer in rdi
            # (Matx33f, Point2f); normL2Sqr only reads its rdi argument
            sret = "normL2Sqr" not in callee
            if sret and rdi and isinstance(rdi[1], int) and rdi[0] in ("rsp", "arg_rbp", "rbp"):
                # slots the callee writes: the Eigen Vector3d / 2x3 results of the FP64 sites are
                # smaller than 16 slots, and the caller keeps its own stack data right above them
                nslots = next((v for k, v in self.sret_slots.items() if k in callee), 16)
                for k in range(nslots):
                    self.mem[(rdi[0], rdi[1] + 4 * k)] = self.mk("in", [], "raw", f"{tag}.out[{k}]") if self.packed \
                        else self.inp(f"{tag}.out[{k}]", "f32")
            return
        if ins in ("ret", "retq"):
            self.event("ret", *(x for x in [self.regs.get("xmm0", [None])[0]] if x is not None))
            return
        # control flow / integer ops are not followed

    # ---- printing ----
    def expr(self, n):
        a = [self.name_of(x) for x in n.args]
        fm = "fmaf" if n.ty == "f32" else "fma"
        if n.op == "fma":
            return f"{fm}({a[0]}, {a[1]}, {a[2]})"
        if n.op in "+-*/":
            return f"{a[0]} {n.op} {a[1]}"
        if n.op == "neg":
            return f"-{a[0]}"
        if n.op == "cvt":
            return f"({'double' if n.ty == 'f64' else 'float'}){a[0]}"
        return f"{n.op}({', '.join(a)})"

    def report(self):
        self.counter = 0
        out = []

        def need(n):
            if n is None or n.op in ("in", "const") or n.id is not None:
                return
            for a in n.args:
                need(a)
            self.counter += 1
            n.id = f"t{self.counter}"
            out.append(f"  {n.id:>5} : {n.ty} = {self.expr(n)}")

        for kind, nodes, extra in self.events:
            for n in nodes:
                need(n)
            out.append(f"  {kind:>5} : {', '.join(self.name_of(n) for n in nodes)} {extra}")
        return "\n".join(out)

    def name_of(self, n):
        if n is None:
            return "?"
        if n.op == "in":
            return n.name
        if n.op == "const":
            return n.name + ("f" if n.ty == "f32" else "")
        return n.id


def read_range(obj, func, start, end, section=".text"):
    out = subprocess.run(["objdump", "-d", "-C", "-r", "--no-show-raw-insn", "-j", section,
                          f"--start-address={start}", f"--stop-address={end}", obj],
                         capture_output=True, text=True, check=True).stdout
    res = []
    pending = None
    for line in out.splitlines():
        m = re.match(r"^\s+([0-9a-f]+):\s+(\S+)\s*(.*)$", line)
        if not m:
            continue
        if m.group(2).startswith("R_X86_64"):
            if pending is not None:
                pending[3] = m.group(3).strip()
            continue
        ins = m.group(2)
        rest = m.group(3).split("#")[0].strip()
        ops = re.findall(r"(?:[^,(]|\([^)]*\))+", rest) if rest else []
        ops = [o.strip() for o in ops]
        pending = [int(m.group(1), 16), ins, ops, None]
        res.append(pending)
    return res


def trace(obj, ranges, names=None, packed=False, f64_regs=()):
    """Walk the address ranges ["0xA:0xB", ...] of obj in order; returns the Tracer.  packed=True
    (the FP64 sites, round 5) follows packed-double instructions and types vector-moved slots on
    use; the float sites of rounds 2-4 are traced without it, exactly as before."""
    t = Tracer(obj, names or {}, packed)
    for r in f64_regs:  # registers holding double arguments at entry (%xmm0 = "%xmm0" input)
        t.regs[r] = [t.inp("%" + r, "f64")] + [None] * 7
    for r in ranges:
        # "0xA:0xB" in .text, or "0xA:0xB@SECTION" (a COMDAT function: inline members, Eigen)
        r, _, sec = r.partition("@")
        a, b = r.split(":")
        t.run(read_range(obj, None, a, b, sec or ".text"))
    for k in range(32):
        lanes = t.regs.get(f"xmm{k}")
        if lanes and lanes[0] is not None and lanes[0].op not in ("in", "const"):
            t.event("live", lanes[0], extra=f"%xmm{k}")
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj")
    ap.add_argument("ranges", nargs="+", help="START:END address ranges, walked in order")
    ap.add_argument("--names", default="")
    args = ap.parse_args()
    names = dict(kv.split("=", 1)[::-1] for kv in args.names.split(",") if kv)
    print(trace(args.obj, args.ranges, names).report())


if __name__ == "__main__":
    main()


# ---------------------------------------------------------------------------------------------
# C emission (for tests/test_fp_sites.py): the traced data flow as a C function
#     void NAME(const double* in, double* out)
# in[k] = the k-th named input (converted to its traced type), out[k] = the k-th selected value
# (an event operand) widened to double.  Every operation is spelled out (fmaf / fma, casts), and
# the file must be compiled with -ffp-contract=off.
def emit_c(tr: Tracer, fname: str, inputs: list[str], outputs: list[tuple[str, int]]) -> str:
    byname = {}
    for n in tr.nodes:
        if n.op == "in" and n.ty != "raw":  # a raw slot is typed on use: its typed node is the input
            byname.setdefault(n.name, n)
    sel = []
    for kind_key, idx in outputs:
        # kind_key: "store:LOC", "laststore:LOC", "cmp#K", "live:%xmmN", "ret", "int#K"
        found = None
        if kind_key.startswith("cmp#") or kind_key.startswith("int#"):
            kind, k = kind_key.split("#")
            evs = [e for e in tr.events if e[0] == kind]
            found = evs[int(k)][1][idx]
        else:
            kind, _, loc = kind_key.partition(":")
            last = kind == "laststore"  # the final value stored at LOC (a stack slot reused)
            kind = "store" if last else kind
            for e in tr.events:
                if e[0] == kind and (not loc or e[2] == loc):
                    found = e[1][idx]
                    if not last:
                        break
        if found is None:
            raise KeyError(kind_key)
        sel.append(found)
    ctype = {"f32": "float", "f64": "double", "i32": "int"}
    lines = [f"void {fname}(const double* in, double* out) {{"]
    names = {}
    for k, nm in enumerate(inputs):
        n = byname.get(nm)
        if n is None:
            continue
        names[id(n)] = f"i{k}"
        lines.append(f"    const {ctype[n.ty]} i{k} = ({ctype[n.ty]})in[{k}];")
    cnt = [0]

    def ref(n):
        if id(n) in names:
            return names[id(n)]
        if n.op == "const":
            return f"(({ctype[n.ty]}){float(n.name)!r})"
        if n.op == "in":
            raise KeyError(f"unbound input {n.name}")
        a = [ref(x) for x in n.args]
        cnt[0] += 1
        v = f"v{cnt[0]}"
        t = ctype[n.ty]
        if n.op == "fma":
            e = f"{'fmaf' if n.ty == 'f32' else 'fma'}({a[0]}, {a[1]}, {a[2]})"
        elif n.op in "+-*/":
            e = f"{a[0]} {n.op} {a[1]}"
        elif n.op == "neg":
            e = f"-{a[0]}"
        elif n.op == "cvt":
            e = f"({t}){a[0]}"
        elif n.op == "sqrt":
            e = f"{'sqrtf' if n.ty == 'f32' else 'sqrt'}({a[0]})"
        elif n.op == "fabs":
            e = f"{'fabsf' if n.ty == 'f32' else 'fabs'}({a[0]})"
        elif n.op in ("ceil", "floor", "trunc", "rint"):
            e = f"{n.op}{'f' if n.ty == 'f32' else ''}({a[0]})"
        elif n.op in ("roundf", "round", "floorf", "ceilf", "sin", "cos"):
            e = f"{n.op}({a[0]})"
        elif n.op == "pow":
            e = f"pow({a[0]}, {a[1]})"
        elif n.op == "i2f":
            e = f"({t}){a[0]}"
        else:
            raise ValueError(n.op)
        lines.append(f"    const {t} {v} = {e};")
        names[id(n)] = v
        return v

    for k, n in enumerate(sel):
        lines.append(f"    out[{k}] = (double){ref(n)};")
    lines.append("}")
    return "\n".join(lines)
