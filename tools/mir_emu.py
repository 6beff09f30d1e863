"""A one-lane interpreter of AMDGPU machine IR as llc prints it between
passes (`-print-after-all`), for the k_min<0> reproducer (DESIGN.md section
12): virtual and physical registers as 32-bit words, `None` for an undefined
word (IMPLICIT_DEF, `undef` operands) so that a value the program stores
without ever defining shows up as such; PHIs by predecessor, COPY,
REG_SEQUENCE, the scalar ALU, compares and branches, the SI_IF / SI_END_CF
pseudos for the one active lane, and the few vector forms the kernel uses.
Run on the dump after every pass, it names the first pass whose output
stores a wrong or undefined record.  Investigation tool: no product code
uses it.
"""
import re

M32 = 0xFFFFFFFF

_SUB = {"sub0": (0, 1), "sub1": (1, 1), "sub2": (2, 1), "sub3": (3, 1), "sub0_sub1": (0, 2), "sub1_sub2": (1, 2),
        "sub2_sub3": (2, 2), "sub0_sub1_sub2": (0, 3), "sub1_sub2_sub3": (1, 3), "sub0_sub1_sub2_sub3": (0, 4),
        "lo16": (0, 1), "hi16": (0, 1)}
_WIDTH = {"sreg_32": 1, "sreg_32_xm0": 1, "sreg_32_xm0_xexec": 1, "sgpr_32": 1, "vgpr_32": 1, "av_32": 1,
          "sreg_64": 2, "sreg_64_xexec": 2, "sgpr_64": 2, "vreg_64": 2, "vreg_64_align2": 2, "av_64": 2,
          "av_64_align2": 2, "sreg_64_xexec_xnull": 2, "sgpr_96": 3, "sgpr_128": 4, "sreg_128": 4,
          "vreg_128": 4, "vreg_128_align2": 4, "av_128": 4, "av_128_align2": 4}


class Fault(Exception):
    pass


def _s32(x):
    return x - (1 << 32) if x & 0x80000000 else x


class Function:
    """Blocks of one function from a -print-after-all dump (or a .mir body)."""

    def __init__(self, text):
        self.blocks = {}  # number -> list of instruction strings
        self.order = []
        self.succ = {}
        cur = None
        for raw in text.split("\n"):
            ln = re.sub(r"^\s*\d+B\s+", "", raw).strip()
            if not ln or ln.startswith(";") or ln.startswith("#") or ln.startswith("liveins:"):
                continue
            m = re.match(r"^bb\.(\d+)\b.*:$", ln)
            if m:
                cur = int(m.group(1))
                self.blocks[cur] = []
                self.order.append(cur)
                self.succ[cur] = []
                continue
            if cur is None:
                continue
            if ln.startswith("successors:"):
                self.succ[cur] = [int(x) for x in re.findall(r"%bb\.(\d+)", ln.split(";")[0])]
                continue
            if ln.startswith("End machine code") or ln.startswith("..."):
                break
            if ln == "}" or (ln.startswith("BUNDLE") and ln.endswith("{")):
                continue  # a bundle's members run in order
            self.blocks[cur].append(ln.split(" :: ")[0].split(", debug-location")[0])


class Machine:
    def __init__(self, fn):
        self.fn = fn

    # -- operands --------------------------------------------------------------------------------
    @staticmethod
    def _strip(op):
        op = re.sub(r"\((?:s|p)\d+\)$|\(tied-def \d+\)$", "", op.strip())
        while True:
            m = re.match(r"^(killed|undef|dead|implicit-def|implicit|renamable|internal|early-clobber|debug-use)\s+(.*)$",
                         op)
            if not m:
                return op
            op = m.group(2)

    def _phys(self, name):
        """$sgpr4_sgpr5 -> [('s', 4), ('s', 5)]"""
        out = []
        for part in name.split("_"):
            m = re.match(r"^(sgpr|vgpr|agpr)(\d+)$", part)
            if m:
                out.append((m.group(1)[0], int(m.group(2))))
            elif part in ("vcc", "exec"):
                out += [(part, 0), (part, 1)]
            elif part in ("lo", "hi") and out:
                key = out[-2][0]
                out = out[:-2] + [(key, 0 if part == "lo" else 1)]
            elif part in ("scc", "m0", "null"):
                out.append((part, 0))
            else:
                raise Fault("register " + name)
        return out

    def read(self, op):
        """operand -> list of 32-bit words (None = undefined) or an int immediate"""
        flags_undef = "undef " in (" " + op.strip() + " ")
        op = self._strip(op)
        if re.match(r"^-?\d+$", op):
            return int(op)
        m = re.match(r"^%(\d+)(?:\.(\w+))?(?::[\w]+)?$", op)
        if m:
            words = self.vr.get(int(m.group(1)))
            if words is None:
                return [None] * (2 if not m.group(2) else _SUB[m.group(2)][1])
            if m.group(2):
                lo, n = _SUB[m.group(2)]
                words = (words + [None] * 4)[lo:lo + n]
            return [None] * len(words) if flags_undef else list(words)
        m = re.match(r"^\$(\w+?)(?:\.(\w+))?$", op)
        if m:
            regs = self._phys(m.group(1))
            if m.group(2):
                lo, n = _SUB[m.group(2)]
                regs = regs[lo:lo + n]
            return [self.pr.get(r) for r in regs]
        raise Fault("operand " + op)

    def write(self, op, words):
        undef = op.strip().startswith("undef ")
        op = self._strip(op)
        m = re.match(r"^%(\d+)(?:\.(\w+))?(?::([\w]+))?$", op)
        if m:
            v = int(m.group(1))
            if m.group(2):
                lo, n = _SUB[m.group(2)]
                cur = [None] * 4 if undef or v not in self.vr else (self.vr[v] + [None] * 4)[:4]
                for k in range(n):
                    cur[lo + k] = words[k] if k < len(words) else None
                w = max(_WIDTH.get(m.group(3) or "", 0), lo + n, len([x for x in self.vr.get(v, [])]))
                self.vr[v] = cur[:max(w, lo + n)]
            else:
                self.vr[v] = list(words)
            return
        m = re.match(r"^\$(\w+?)(?:\.(\w+))?$", op)
        if m:
            regs = self._phys(m.group(1))
            if m.group(2):
                lo, n = _SUB[m.group(2)]
                regs = regs[lo:lo + n]
            for r, w in zip(regs, words):
                self.pr[r] = w
            return
        raise Fault("dest " + op)

    # -- execution -------------------------------------------------------------------------------
    def run(self, kernarg, memory, max_steps=400000):
        self.vr, self.pr = {}, {}
        ka = 0x1000
        for off, val in kernarg.items():
            memory[ka + off] = val & M32
            memory[ka + off + 4] = (val >> 32) & M32
        self.mem = memory
        self.pr[("s", 0)], self.pr[("s", 1)] = ka, 0  # kernarg segment pointer (first user SGPRs)
        self.pr[("v", 0)] = 0  # thread 0
        self.pr[("exec", 0)], self.pr[("exec", 1)] = M32, M32
        self.stored = None
        fn = self.fn
        bb, prev, steps = fn.order[0], None, 0
        while True:
            ins = fn.blocks[bb]
            # PHIs read their inputs together, by the edge taken
            phis = [i for i in ins if re.search(r"= PHI ", i)]
            vals = []
            for i in phis:
                d, rhs = i.split(" = PHI ", 1)
                ops = [x.strip() for x in rhs.split(",")]
                src = None
                for k in range(0, len(ops), 2):
                    if ops[k + 1] == "%%bb.%d" % prev:
                        src = ops[k]
                if src is None:
                    raise Fault("PHI without edge from bb.%s in bb.%d" % (prev, bb))
                vals.append((d, self.read(src)))
            for d, v in vals:
                self.write(d, v)
            nxt = None
            for i in ins:
                if " = PHI " in i:
                    continue
                steps += 1
                if steps > max_steps:
                    raise Fault("step limit")
                self.last = i
                r = self.exec(i)
                if r == "end":
                    return self.stored
                if r is not None:
                    nxt = r
                    break
            if nxt is None:  # fall through to the layout successor
                k = fn.order.index(bb)
                nxt = fn.order[k + 1]
            prev, bb = bb, nxt

    def exec(self, i):
        if " = " in i:
            lhs, rhs = i.split(" = ", 1)
            defs = [d.strip() for d in lhs.split(",")]
        else:
            defs, rhs = [], i
        rhs = re.sub(r"^((nuw|nsw|exact|disjoint|samesign|nnan|ninf|nsz|arcp|contract|afn|reassoc|nofpexcept)\s+)*", "", rhs)
        op, _, rest = rhs.partition(" ")
        ops = [x.strip() for x in rest.split(",")] if rest.strip() else []
        expl = [x for x in ops if not re.match(r"^(implicit|implicit-def)\b", x)]
        R, W = self.read, self.write

        def w1(x):
            if isinstance(x, int):
                return x & M32
            return x[0]

        def w64(x):
            if isinstance(x, int):
                return [x & M32, (x >> 32) & M32]
            return (x + [None])[:2]

        def scc(v):
            self.pr[("scc", 0)] = v

        if op == "S_ENDPGM":
            return "end"
        if op in ("KILL", "CFI_INSTRUCTION", "S_WAITCNT", "S_NOP", "BUNDLE", "SCHED_BARRIER", "S_SETPRIO",
                  "S_WAITCNT_soft", "S_WAITCNT_VSCNT", "S_DELAY_ALU") and not defs:
            return None
        if rhs.startswith("frame-setup") or rhs.startswith("frame-destroy"):
            return None
        if op in ("S_AND_SAVEEXEC_B64", "S_OR_SAVEEXEC_B64"):
            old = R("$exec")
            src = w64(R(expl[0]))
            e = [None if x is None else (x & o if op.startswith("S_AND") else x | o) for x, o in zip(src, old)]
            W(defs[0], old)
            W("$exec", e)
            scc(None if None in e else int((e[0] | e[1]) != 0))
            return None
        if op == "S_BRANCH":
            return int(expl[0][4:])
        if op.startswith("S_CBRANCH_"):
            c = op[len("S_CBRANCH_"):]
            if c.startswith("SCC"):
                s = self.pr.get(("scc", 0))
                if s is None:
                    raise Fault("branch on undefined scc")
                take = s == (1 if c == "SCC1" else 0)
            elif c.startswith("VCC"):
                v = R("$vcc")
                if None in v:
                    raise Fault("branch on undefined vcc")
                nz = (v[0] | v[1]) != 0
                take = nz if c == "VCCNZ" else not nz
            elif c.startswith("EXEC"):
                v = R("$exec")
                nz = (v[0] | v[1]) != 0
                take = nz if c == "EXECNZ" else not nz
            else:
                raise Fault(op)
            return int(expl[0][4:]) if take else None
        if op in ("COPY", "KILL", "S_MOV_B32", "S_MOV_B64", "V_MOV_B32_e32", "V_MOV_B64_e32", "AV_MOV_B32_IMM_PSEUDO",
                  "S_MOV_B64_IMM_PSEUDO", "V_READFIRSTLANE_B32", "PRED_COPY", "S_MOV_B32_term", "S_MOV_B64_term",
                  "V_MOV_B64_PSEUDO"):
            x = R(expl[0])
            if isinstance(x, int):
                x = w64(x) if "64" in op else [x & M32]
            if self._strip(expl[0]) == "$scc":  # a lane mask of the condition (si-fix-sgpr-copies: S_CSELECT -1, 0)
                m = re.search(r":(\w+)$", self._strip(defs[0]))
                n = _WIDTH.get(m.group(1), 2) if m else 2
                x = [None] * n if x[0] is None else [M32 if x[0] else 0] * n
            W(defs[0], x)
            return None
        if op == "S_BITSET1_B32":  # $d = S_BITSET1_B32 bit, $d(tied)
            b, d = w1(R(expl[0])), w1(R(expl[1]))
            W(defs[0], [None if b is None or d is None else d | (1 << (b & 31))])
            return None
        if op == "S_MOVK_I32":
            W(defs[0], [((R(expl[0]) & 0xFFFF) ^ 0x8000) - 0x8000 & M32])
            return None
        if op == "IMPLICIT_DEF":
            W(defs[0], [None] * 4)
            return None
        if op == "REG_SEQUENCE":
            words = [None] * 4
            hi = 0
            for k in range(0, len(expl), 2):
                lo, n = _SUB[expl[k + 1].split(".")[1]]
                v = R(expl[k])
                v = [v & M32] if isinstance(v, int) else v
                for j in range(n):
                    words[lo + j] = v[j] if j < len(v) else None
                hi = max(hi, lo + n)
            W(defs[0], words[:hi])
            return None
        if op.startswith("S_LOAD_DWORD"):
            n = {"S_LOAD_DWORD_IMM": 1, "S_LOAD_DWORDX2_IMM": 2, "S_LOAD_DWORDX4_IMM": 4}[op]
            base = w64(R(expl[0]))
            if None in base:
                raise Fault("load through undefined address")
            a = base[0] | (base[1] << 32)
            a += R(expl[1])
            W(defs[0], [self.mem.get(a + 4 * k, 0) for k in range(n)])
            return None
        m = re.match(r"^GLOBAL_LOAD_DWORD(X2|X3|X4)?_SADDR$", op)
        if m:  # vD = [saddr + voffset + offset]
            n = {None: 1, "X2": 2, "X3": 3, "X4": 4}[m.group(1)]
            sb, v, off = w64(R(expl[0])), R(expl[1]), R(expl[2])
            v = v if isinstance(v, int) else v[0]
            if None in sb or v is None:
                raise Fault("load through undefined address")
            a = (sb[0] | (sb[1] << 32)) + v + off
            W(defs[0], [self.mem.get(a + 4 * k, 0) for k in range(n)])
            return None
        m = re.match(r"^GLOBAL_STORE_DWORD(X2|X3|X4)?_SADDR$", op)
        if m:
            n = {None: 1, "X2": 2, "X3": 3, "X4": 4}[m.group(1)]
            v, data, sb = R(expl[0]), R(expl[1]), w64(R(expl[2]))
            off = R(expl[3])
            if None in sb or (isinstance(v, list) and None in v):
                raise Fault("store through undefined address")
            data = [data & M32] if isinstance(data, int) else data
            a = (sb[0] | (sb[1] << 32)) + (v if isinstance(v, int) else v[0]) + off
            self.stored = (a, list(data))
            for k in range(n):
                self.mem[a + 4 * k] = data[k] if k < len(data) else None
            return None
        if op == "SI_IF":
            cond = w64(R(expl[0]))
            if cond[0] is None:
                raise Fault("SI_IF on undefined mask")
            W(defs[0], [M32, M32])  # the lanes to restore (not modelled beyond lane 0)
            if cond[0] & 1:
                self.pr[("exec", 0)], self.pr[("exec", 1)] = 1, 0
                return None
            return int(expl[1][4:])
        if op == "SI_END_CF":
            self.pr[("exec", 0)], self.pr[("exec", 1)] = M32, M32
            return None
        m = re.match(r"^V_CMP_(EQ|NE|LG|GT|GE|LT|LE)_(U32|I32)_(e64|e32)$", op)
        if m:
            if m.group(3) == "e32":
                defs = ["$vcc"]
            a, b = w1(R(expl[0])), w1(R(expl[1]))
            if a is None or b is None:
                W(defs[0], [None, None])
                return None
            if m.group(2) == "I32":
                a, b = _s32(a), _s32(b)
            r = {"EQ": a == b, "NE": a != b, "LG": a != b, "GT": a > b, "GE": a >= b, "LT": a < b, "LE": a <= b}[m.group(1)]
            W(defs[0], [int(r), 0])
            return None
        if op == "V_CNDMASK_B32_e64":  # src0_mod, src0, src1_mod, src1, mask
            s0, s1, mk = R(expl[1]), R(expl[3]), w64(R(expl[4]))
            if mk[0] is None:
                W(defs[0], [None])
                return None
            W(defs[0], [w1(s1) if mk[0] & 1 else w1(s0)])
            return None
        if op in ("S_ADD_CO_PSEUDO",):  # dst, carry-out = a + b + carry-in (a lane mask)
            a, b, c = w1(R(expl[0])), w1(R(expl[1])), w64(R(expl[2]))
            if None in (a, b, c[0]):
                W(defs[0], [None]); W(defs[1], [None, None])
                return None
            r = a + b + (1 if (c[0] | (c[1] or 0)) else 0)
            W(defs[0], [r & M32])
            W(defs[1], [1 if r > M32 else 0, 0])
            return None
        # scalar ALU
        w = 2 if op.endswith("_B64") or op.endswith("_U64") else 1
        get = (lambda x: w64(R(x))) if w == 2 else (lambda x: [w1(R(x))])

        def join(ws):
            if None in ws:
                return None
            return ws[0] | (ws[1] << 32) if len(ws) == 2 else ws[0]

        def split(x, n):
            return [None] * n if x is None else ([x & M32, (x >> 32) & M32] if n == 2 else [x & M32])

        logic = {"S_AND": lambda x, y: x & y, "S_OR": lambda x, y: x | y, "S_XOR": lambda x, y: x ^ y,
                 "S_ANDN2": lambda x, y: x & ~y, "S_ORN2": lambda x, y: x | ~y}
        base = op.rsplit("_", 1)[0]
        mask = (1 << (32 * w)) - 1
        if base in logic and op.rsplit("_", 1)[1] in ("B32", "B64"):
            # bitwise: word by word, so an undefined word of one half leaves the other half defined
            xs, ys = get(expl[0]), get(expl[1])
            r = [None if x is None or y is None else logic[base](x, y) & M32 for x, y in zip(xs, ys)]
            W(defs[0], r)
            scc(None if None in r else int(any(r)))
            return None
        if op == "S_NOT_B32":
            x = join(get(expl[0]))
            r = None if x is None else ~x & M32
            W(defs[0], split(r, 1)); scc(None if r is None else int(r != 0))
            return None
        if op == "S_CSELECT_B32" or op == "S_CSELECT_B64":
            s = self.pr.get(("scc", 0))
            x, y = get(expl[0]), get(expl[1])
            W(defs[0], ([None] * w) if s is None else (x if s else y))
            return None
        two = {"S_LSHL_B32": lambda x, y: (x << (y & 31)) & M32, "S_LSHR_B32": lambda x, y: x >> (y & 31),
               "S_ASHR_I32": lambda x, y: (_s32(x) >> (y & 31)) & M32,
               "S_MUL_I32": lambda x, y: (_s32(x) * _s32(y)) & M32}
        if op in two:
            x, y = join(get(expl[0])), join(get(expl[1]))
            r = None if x is None or y is None else two[op](x, y)
            W(defs[0], split(r, 1))
            if op != "S_MUL_I32":
                scc(None if r is None else int(r != 0))
            return None
        if op in ("S_ADD_I32", "S_SUB_I32", "S_ADD_U32", "S_ADDC_U32", "S_SUB_U32"):
            x, y = join(get(expl[0])), join(get(expl[1]))
            c = self.pr.get(("scc", 0)) if op == "S_ADDC_U32" else 0
            if x is None or y is None or c is None:
                W(defs[0], [None]); scc(None)
                return None
            if op == "S_ADD_I32":
                r = _s32(x) + _s32(y); sc = int(r != _s32(r & M32))
            elif op == "S_SUB_I32":
                r = _s32(x) - _s32(y); sc = int(r != _s32(r & M32))
            elif op == "S_SUB_U32":
                r = x - y; sc = int(r < 0)
            else:
                r = x + y + c; sc = int(r > M32)
            W(defs[0], [r & M32]); scc(sc)
            return None
        if op == "S_BFE_U32":
            x, c = join(get(expl[0])), join(get(expl[1]))
            r = None if x is None or c is None else ((x >> (c & 31)) & ((1 << ((c >> 16) & 0x7F)) - 1))
            W(defs[0], split(r, 1)); scc(None if r is None else int(r != 0))
            return None
        if op == "S_FF1_I32_B32":
            x = join(get(expl[0]))
            r = None if x is None else (((x & -x).bit_length() - 1) & M32 if x else M32)
            W(defs[0], split(r, 1))
            return None
        if op == "S_BITCMP0_B32":
            x, b = join(get(expl[0])), join(get(expl[1]))
            scc(None if x is None or b is None else int(((x >> (b & 31)) & 1) == 0))
            return None
        m = re.match(r"^S_CMP(K?)_(EQ|LG|GT|GE|LT|LE)_(U32|I32|U64)$", op)
        if m:
            k, rel, ty = m.groups()
            if ty == "U64":
                x, y = join(w64(R(expl[0]))), join(w64(R(expl[1])))
            else:
                x, y = w1(R(expl[0])), R(expl[1])
                if k:
                    y = ((y & 0xFFFF) ^ 0x8000) - 0x8000 if ty == "I32" else y & 0xFFFF
                else:
                    y = w1(y)
            if x is None or y is None:
                scc(None)
                return None
            if ty == "I32":
                x, y = _s32(x), _s32(y & M32) if not k else y
            r = {"EQ": x == y, "LG": x != y, "GT": x > y, "GE": x >= y, "LT": x < y, "LE": x <= y}[rel]
            scc(int(r))
            return None
        raise Fault("opcode " + i)
