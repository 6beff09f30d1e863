"""Round 4's deterministic k_min<0> defect: split
chosen `<2 x i32>` phis of the committed SLP IR into two `i32` phis, every
other vector operation left as it is.  Each incoming vector is taken apart
by two `extractelement`s in its predecessor block (before the terminator);
the vector is rebuilt by two `insertelement`s after the block's phis, so
every use is unchanged.  Numbered values are renamed (%N -> %vN) first so
that instructions can be inserted.  Investigation tool: the variants run
through llc and the code-object checker (tools/kmin_phi_split.sh).

    python tools/kmin_phi_split.py IN.ll OUT.ll [PHI ...]    # PHI: 810 811 ...
"""
import re
import sys


def rename(lines):
    out = []
    in_fn = False
    for ln in lines:
        if ln.startswith("define "):
            in_fn = True
            out.append(re.sub(r"%(\d+)\b", r"%v\1", ln))
            out.append("v1:")
            continue
        if in_fn:
            if ln.startswith("}"):
                in_fn = False
                out.append(ln)
                continue
            m = re.match(r"^(\d+):(.*)$", ln)
            if m:
                out.append("v%s:%s" % (m.group(1), m.group(2)))
                continue
            code, sep, comment = ln.partition(";")
            out.append(re.sub(r"%(\d+)\b", r"%v\1", code) + sep + comment)
        else:
            out.append(ln)
    return out


def parse_incoming(body):
    # "[ %v203, %v161 ], [ <i32 1, i32 2>, %v5 ], ..."
    items = re.findall(r"\[\s*(.+?),\s*(%[\w.]+)\s*\]", body)
    return [(v.strip(), b) for v, b in items]


def const_lanes(v):
    if v in ("zeroinitializer",):
        return "0", "0"
    if v in ("poison", "undef"):
        return "poison", "poison"
    m = re.match(r"<\s*i32\s+(\S+),\s*i32\s+(\S+)\s*>", v)
    if m:
        return m.group(1), m.group(2)
    return None


def block_ranges(lines):
    """label -> (first line index after the label, index of the block's last line + 1)"""
    labels = [(i, re.match(r"^(v\d+):", ln).group(1)) for i, ln in enumerate(lines) if re.match(r"^v\d+:", ln)]
    end_fn = next(i for i in range(labels[0][0], len(lines)) if lines[i].startswith("}"))
    out = {}
    for k, (i, name) in enumerate(labels):
        j = labels[k + 1][0] if k + 1 < len(labels) else end_fn
        out[name] = (i + 1, j)
    return out


def terminator_index(lines, lo, hi):
    j = hi - 1
    while j >= lo and not lines[j].strip():
        j -= 1
    if lines[j].strip() == "]":
        while not lines[j].lstrip().startswith("switch "):
            j -= 1
    return j


def split_phis(lines, phis):
    inserts = {}  # line index -> lines to insert before it
    after_phis = {}  # block label -> lines after its phis
    for x in phis:
        name = "%v" + x
        idx = next(i for i, ln in enumerate(lines) if ln.startswith("  %s = phi <2 x i32> " % name))
        blk = None
        for i in range(idx, -1, -1):
            m = re.match(r"^(v\d+):", lines[i])
            if m:
                blk = m.group(1)
                break
        inc = parse_incoming(lines[idx].split("phi <2 x i32>", 1)[1])
        ranges = block_ranges(lines)
        s0, s1 = [], []
        for n, (v, b) in enumerate(inc):
            c = const_lanes(v)
            if c is not None:
                s0.append("[ %s, %s ]" % (c[0], b))
                s1.append("[ %s, %s ]" % (c[1], b))
                continue
            lo, hi = ranges[b[1:]]
            t = terminator_index(lines, lo, hi)
            e0, e1 = "%s.e%d.0" % (name, n), "%s.e%d.1" % (name, n)
            inserts.setdefault(t, []).extend(["  %s = extractelement <2 x i32> %s, i64 0" % (e0, v),
                                              "  %s = extractelement <2 x i32> %s, i64 1" % (e1, v)])
            s0.append("[ %s, %s ]" % (e0, b))
            s1.append("[ %s, %s ]" % (e1, b))
        lines[idx] = "  %s.s0 = phi i32 %s\n  %s.s1 = phi i32 %s" % (name, ", ".join(s0), name, ", ".join(s1))
        after_phis.setdefault(blk, []).extend(["  %s.r0 = insertelement <2 x i32> poison, i32 %s.s0, i64 0" % (name, name),
                                               "  %s = insertelement <2 x i32> %s.r0, i32 %s.s1, i64 1" % (name, name, name)])
    ranges = block_ranges(lines)
    for blk, new in after_phis.items():
        lo, hi = ranges[blk]
        k = lo
        while k < hi and " = phi " in lines[k]:
            k += 1
        inserts.setdefault(k, []).extend(new)
    out = []
    for i, ln in enumerate(lines):
        out.extend(inserts.get(i, []))
        out.append(ln)
    return out


def main():
    src, dst, phis = sys.argv[1], sys.argv[2], sys.argv[3:]
    lines = rename(open(src).read().split("\n"))
    if phis:
        lines = split_phis(lines, phis)
    open(dst, "w").write("\n".join(lines))


if __name__ == "__main__":
    main()
