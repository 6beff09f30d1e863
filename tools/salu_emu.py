"""A one-lane emulator of the gfx950 instructions the k_min<0> reproducer's
code uses: scalar ALU, compares, scalar branches,
s_load, the exec / vcc bookkeeping of one active lane, and the handful of
vector moves, v_cndmask / v_readfirstlane and the global store it ends with.
Emulating the committed assembly decides whether a wrong record comes from
the instructions themselves (the compiler) or from how the hardware runs
them.  Investigation tool: no product code uses it.

    prog = Program(open("kmin_slp_O3.s").read())
    out = prog.run(kernarg={0: dst_ptr, 0x20: action}, memory=Memory(...))
"""
import re

M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1


def _s32(x):
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


class Memory:
    """Byte-addressed little-endian memory (dict of 32-bit words at 4-byte addresses)."""

    def __init__(self):
        self.w = {}

    def load32(self, a):
        assert a % 4 == 0, hex(a)
        return self.w.get(a, 0)

    def store32(self, a, v):
        assert a % 4 == 0, hex(a)
        self.w[a] = v & M32


class Fault(Exception):
    pass


_REG = re.compile(r"^(s|v|a)(\d+)$")
_RANGE = re.compile(r"^(s|v|a)\[(\d+):(\d+)\]$")


class Program:
    def __init__(self, text, symbol=None):
        self.ins = []
        self.labels = {}
        started = symbol is None
        for raw in text.split("\n"):
            line = raw.split(";")[0].rstrip()
            if not line.strip():
                continue
            if symbol is not None and line.startswith(symbol + ":"):
                started = True
                continue
            if not started:
                continue
            m = re.match(r"^(\.?[\w.$]+):", line)
            if m and not line.startswith("\t"):
                self.labels[m.group(1)] = len(self.ins)
                continue
            s = line.strip()
            if s.startswith("."):
                if s.startswith(".Lfunc_end") or s.startswith(".size"):
                    break
                continue
            op, _, rest = s.partition(" ")
            args = [a.strip() for a in rest.split(",")] if rest.strip() else []
            self.ins.append((op, args))

    # -- register file ------------------------------------------------------------------------
    def _get(self, a, width=32):
        st = self.st
        if width == 64:
            m = _RANGE.match(a)
            if m:
                kind, lo, hi = m.group(1), int(m.group(2)), int(m.group(3))
                assert hi == lo + 1, a
                f = st[kind]
                return f[lo] | (f[hi] << 32)
            if a == "vcc":
                return st["vcc"]
            if a == "exec":
                return st["exec"]
            return self._imm(a) & M64
        m = _REG.match(a)
        if m:
            return st[m.group(1)][int(m.group(2))]
        if a == "vcc_lo":
            return st["vcc"] & M32
        if a == "vcc_hi":
            return st["vcc"] >> 32
        if a == "exec_lo":
            return st["exec"] & M32
        if a == "exec_hi":
            return st["exec"] >> 32
        if a == "scc":
            return st["scc"]
        return self._imm(a) & M32

    def _imm(self, a):
        if re.match(r"^-?0x[0-9a-fA-F]+$", a) or re.match(r"^-?\d+$", a):
            return int(a, 0)
        raise Fault("operand " + a)

    def _set(self, a, v, width=32):
        st = self.st
        if width == 64:
            v &= M64
            m = _RANGE.match(a)
            if m:
                kind, lo = m.group(1), int(m.group(2))
                f = st[kind]
                f[lo], f[lo + 1] = v & M32, v >> 32
                return
            if a in ("vcc", "exec"):
                st[a] = v
                return
            raise Fault("dest " + a)
        v &= M32
        m = _REG.match(a)
        if m:
            st[m.group(1)][int(m.group(2))] = v
            return
        if a == "vcc_lo":
            st["vcc"] = (st["vcc"] & ~M32 & M64) | v
        elif a == "vcc_hi":
            st["vcc"] = (st["vcc"] & M32) | (v << 32)
        elif a == "exec_lo":
            st["exec"] = (st["exec"] & ~M32 & M64) | v
        elif a == "exec_hi":
            st["exec"] = (st["exec"] & M32) | (v << 32)
        else:
            raise Fault("dest " + a)

    # -- execution ------------------------------------------------------------------------------
    def run(self, kernarg, memory, tid=0, max_steps=200000, trace=None):
        """kernarg: {byte offset: 32/64-bit value} of the kernel arguments
        (placed at address 0x1000); returns the memory after s_endpgm."""
        self.st = {"s": [0] * 106, "v": [0] * 256, "a": [0] * 256, "vcc": 0, "exec": M64, "scc": 0, "lanes": {}}
        ka = 0x1000
        for off, val in kernarg.items():
            memory.store32(ka + off, val & M32)
            memory.store32(ka + off + 4, (val >> 32) & M32)
        self.st["s"][0], self.st["s"][1] = ka, 0
        self.st["v"][0] = tid
        self.mem = memory
        pc = 0
        for _ in range(max_steps):
            op, a = self.ins[pc]
            if trace is not None:
                trace.append((pc, op, a))
            try:
                nxt = self._exec(op, a, pc)
            except Fault as e:
                raise Fault("%s (at %d: %s %s)" % (e, pc, op, ", ".join(a))) from None
            if nxt == "end":
                return memory
            pc = pc + 1 if nxt is None else nxt
        raise Fault("step limit")

    def _lane0(self):
        return self.st["exec"] & 1

    def _exec(self, op, a, pc):
        st, g, s = self.st, self._get, self._set
        if op == "s_endpgm":
            return "end"
        if op in ("s_waitcnt", "s_nop"):
            return None
        if op == "s_branch":
            return self.labels[a[0]]
        if op.startswith("s_cbranch_"):
            c = op[len("s_cbranch_"):]
            take = {"scc0": st["scc"] == 0, "scc1": st["scc"] == 1, "vccz": st["vcc"] == 0,
                    "vccnz": st["vcc"] != 0, "execz": st["exec"] == 0, "execnz": st["exec"] != 0}[c]
            return self.labels[a[0]] if take else None
        if op.startswith("s_load_dword"):
            n = {"s_load_dword": 1, "s_load_dwordx2": 2, "s_load_dwordx4": 4, "s_load_dwordx8": 8}[op]
            base = g(a[1], 64) + self._imm(a[2])
            m = _RANGE.match(a[0]) or _REG.match(a[0])
            lo = int(m.group(2))
            for k in range(n):
                st["s"][lo + k] = self.mem.load32(base + 4 * k)
            return None
        if op.startswith("global_load_dword"):
            n = {"global_load_dword": 1, "global_load_dwordx2": 2, "global_load_dwordx3": 3, "global_load_dwordx4": 4}[op]
            sbase, *mods = a[2].split()
            addr = g(a[1], 64) if sbase == "off" else g(sbase, 64) + g(a[1])
            for x in mods + a[3:]:
                if x.startswith("offset:"):
                    addr += int(x.split(":")[1], 0)
            m = _RANGE.match(a[0]) or _REG.match(a[0])
            lo = int(m.group(2))
            if self._lane0():
                for k in range(n):
                    st[m.group(1)][lo + k] = self.mem.load32(addr + 4 * k)
            return None
        if op.startswith("global_store_dword"):
            n = {"global_store_dword": 1, "global_store_dwordx2": 2, "global_store_dwordx4": 4}[op]
            if not self._lane0():
                return None
            sbase, *mods = a[2].split()
            addr = g(a[0], 64) if sbase == "off" else g(sbase, 64) + g(a[0])
            for x in mods + a[3:]:
                if x.startswith("offset:"):
                    addr += int(x.split(":")[1], 0)
            m = _RANGE.match(a[1]) or _REG.match(a[1])
            lo = int(m.group(2))
            for k in range(n):
                self.mem.store32(addr + 4 * k, st["v"][lo + k])
            return None
        m = re.match(r"^v_cmp_(eq|ne|lg|gt|ge|lt|le)_(u32|i32)_(e32|e64)$", op)
        if m:  # lane 0's bit; the other lanes are not modelled
            rel, ty, enc = m.groups()
            if enc == "e32":
                dst, (x, y) = "vcc", (a[1:3] if a[0] == "vcc" else a[0:2])
            else:
                dst, x, y = a[0], a[1], a[2]
            x, y = g(x), g(y)
            if ty == "i32":
                x, y = _s32(x), _s32(y)
            r = {"eq": x == y, "ne": x != y, "lg": x != y, "gt": x > y, "ge": x >= y, "lt": x < y, "le": x <= y}[rel]
            s(dst, int(r), 64)
            return None
        if op == "v_mov_b32_e32":
            if self._lane0():
                s(a[0], g(a[1]))
            return None
        if op == "v_cndmask_b32_e64":
            if self._lane0():
                s(a[0], g(a[2]) if g(a[3], 64) & 1 else g(a[1]))
            return None
        if op == "v_writelane_b32":  # spills of SGPRs into VGPR lanes (-O0)
            lane = g(a[2]) & 63
            st["lanes"][(a[0], lane)] = g(a[1])
            if lane == 0:
                s(a[0], g(a[1]))
            return None
        if op == "v_readlane_b32":
            lane = g(a[2]) & 63
            s(a[0], g(a[1]) if lane == 0 else st["lanes"].get((a[1], lane), 0))
            return None
        if op == "v_readfirstlane_b32":
            s(a[0], g(a[1]))
            return None
        if op in ("v_accvgpr_write_b32", "v_accvgpr_read_b32"):
            if self._lane0():
                s(a[0], g(a[1]))
            return None
        if op == "v_mov_b64_e32":
            if self._lane0():
                s(a[0], g(a[1], 64), 64)
            return None
        if op == "v_cndmask_b32_e32":  # vD, a, b, vcc
            if self._lane0():
                s(a[0], g(a[2]) if g(a[3], 64) & 1 else g(a[1]))
            return None
        if op == "s_or_saveexec_b64":
            old = st["exec"]
            s(a[0], old, 64)
            st["exec"] = g(a[1], 64) | old
            st["scc"] = int(st["exec"] != 0)
            return None
        if op == "s_and_saveexec_b64":
            old = st["exec"]
            s(a[0], old, 64)
            st["exec"] = g(a[1], 64) & old
            st["scc"] = int(st["exec"] != 0)
            return None
        w = 64 if op.endswith("_b64") or op.endswith("_u64") else 32
        if op in ("s_mov_b32", "s_mov_b64"):
            s(a[0], g(a[1], w), w)
            return None
        if op == "s_movk_i32":
            s(a[0], ((self._imm(a[1]) & 0xFFFF) ^ 0x8000) - 0x8000)
            return None
        if op in ("s_cselect_b32", "s_cselect_b64"):
            s(a[0], g(a[1], w) if st["scc"] else g(a[2], w), w)
            return None
        logic = {"s_and": lambda x, y: x & y, "s_or": lambda x, y: x | y, "s_xor": lambda x, y: x ^ y,
                 "s_andn2": lambda x, y: x & ~y, "s_orn2": lambda x, y: x | ~y}
        base = op.rsplit("_", 1)[0]
        if base in logic and op.rsplit("_", 1)[1] in ("b32", "b64"):
            mask = M64 if w == 64 else M32
            r = logic[base](g(a[1], w), g(a[2], w)) & mask
            s(a[0], r, w)
            st["scc"] = int(r != 0)
            return None
        if op == "s_not_b32":
            r = ~g(a[1]) & M32
            s(a[0], r)
            st["scc"] = int(r != 0)
            return None
        if op == "s_lshl_b32":
            r = (g(a[1]) << (g(a[2]) & 31)) & M32
            s(a[0], r)
            st["scc"] = int(r != 0)
            return None
        if op == "s_lshr_b32":
            r = g(a[1]) >> (g(a[2]) & 31)
            s(a[0], r)
            st["scc"] = int(r != 0)
            return None
        if op == "s_ashr_i32":
            r = (_s32(g(a[1])) >> (g(a[2]) & 31)) & M32
            s(a[0], r)
            st["scc"] = int(r != 0)
            return None
        if op == "s_add_i32":
            x, y = _s32(g(a[1])), _s32(g(a[2]))
            r = x + y
            s(a[0], r)
            st["scc"] = int(r != _s32(r))
            return None
        if op == "s_sub_i32":
            x, y = _s32(g(a[1])), _s32(g(a[2]))
            r = x - y
            s(a[0], r)
            st["scc"] = int(r != _s32(r))
            return None
        if op == "s_add_u32":
            r = g(a[1]) + g(a[2])
            s(a[0], r)
            st["scc"] = int(r > M32)
            return None
        if op == "s_addc_u32":
            r = g(a[1]) + g(a[2]) + st["scc"]
            s(a[0], r)
            st["scc"] = int(r > M32)
            return None
        m = re.match(r"^s_lshl([1-4])_add_u32$", op)
        if m:
            r = ((g(a[1]) << int(m.group(1))) & M32) + g(a[2])
            s(a[0], r)
            st["scc"] = int(r > M32)
            return None
        if op == "s_addk_i32":  # d += simm16
            x, y = _s32(g(a[0])), ((self._imm(a[1]) & 0xFFFF) ^ 0x8000) - 0x8000
            r = x + y
            s(a[0], r)
            st["scc"] = int(r != _s32(r))
            return None
        if op == "s_mul_i32":
            s(a[0], _s32(g(a[1])) * _s32(g(a[2])))
            return None
        if op == "s_bfe_u32":
            x, c = g(a[1]), g(a[2])
            off, width = c & 31, (c >> 16) & 0x7F
            r = (x >> off) & ((1 << width) - 1) if width else 0
            s(a[0], r)
            st["scc"] = int(r != 0)
            return None
        if op == "s_bfe_i32":
            x, c = g(a[1]), g(a[2])
            off, width = c & 31, (c >> 16) & 0x7F
            r = 0
            if width:
                r = (x >> off) & ((1 << width) - 1)
                if r >> (width - 1):
                    r -= 1 << width
            s(a[0], r)
            st["scc"] = int(r & M32 != 0)
            return None
        if op == "s_ff1_i32_b32":
            x = g(a[1])
            r = (x & -x).bit_length() - 1 if x else -1
            s(a[0], r)
            return None
        if op == "s_bitset1_b32":
            s(a[0], g(a[0]) | (1 << (g(a[1]) & 31)))
            return None
        if op == "s_bitcmp0_b32":
            st["scc"] = int(((g(a[0]) >> (g(a[1]) & 31)) & 1) == 0)
            return None
        if op == "s_bitcmp1_b32":
            st["scc"] = int(((g(a[0]) >> (g(a[1]) & 31)) & 1) == 1)
            return None
        m = re.match(r"^s_cmp(k?)_(eq|lg|gt|ge|lt|le)_(u32|i32|u64)$", op)
        if m:
            k, rel, ty = m.groups()
            if ty == "u64":
                x, y = g(a[0], 64), g(a[1], 64)
            elif k:
                imm = self._imm(a[1]) & 0xFFFF
                y = ((imm ^ 0x8000) - 0x8000) if ty == "i32" else imm
                x = _s32(g(a[0])) if ty == "i32" else g(a[0])
            elif ty == "i32":
                x, y = _s32(g(a[0])), _s32(g(a[1]))
            else:
                x, y = g(a[0]), g(a[1])
            st["scc"] = int({"eq": x == y, "lg": x != y, "gt": x > y, "ge": x >= y, "lt": x < y, "le": x <= y}[rel])
            return None
        raise Fault("opcode %s %s at %d" % (op, a, pc))
