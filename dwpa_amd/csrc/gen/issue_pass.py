"""gfx950 VALU issue pass: insert s_nop spacers into the main (4096-iteration) loop of a device assembly file.

Why (measured on MI355X, tools/valu_mix*, tools/asm/asm_lab, profiles/r01/): a wave64 VALU stream that mixes 4-cycle
ops (v_alignbit_b32, v_add3_u32, v_xad_u32, ...) with 2-cycle ops (v_xor_b32, v_bitop3_b32, v_add_u32) issues
EVERY instruction at the 4-cycle rate, even with 8 waves per SIMD; homogeneous streams run at 2 / 4 cycles.  A
scalar `s_nop 0` in front of each 4-cycle op restores near-additive issue: the PBKDF2 loop goes from 3.9 to ~3.4
SIMD-cycles per VALU instruction (+15.7 % PMK/s) with the instruction stream otherwise unchanged.  Source-level
`asm volatile("s_nop 0")` cannot do this -- LLVM hoists the register-only VALU ops over it -- hence the pass on
the compiler's assembly.  The product rule (the Makefile's ISSUE_RULE) is `sched=1:alt:orig:asmnop,before_half`
since round 5 (`before_half` before it; profiles/r05/issue_rules_sched/, profiles/r05/sched_identities/).

Rules (comma-separated, applied in the loop body only):
  after_half      s_nop after every 4-cycle VALU (alignbit, add3, xad, bfi, ...)
  after_full_h    s_nop after a 2-cycle VALU that follows a 4-cycle VALU
  before_half     s_nop before every 4-cycle VALU
  every=K         s_nop after every K-th VALU
  after_alb       s_nop after every v_alignbit_b32
  before_half_trans  s_nop before a 4-cycle VALU that follows a 2-cycle VALU
  before_alb / before_ad3  s_nop before every alignbit / add3
  before_full_trans  s_nop before a 2-cycle VALU that follows a 4-cycle VALU
  nop1            use s_nop 1 instead of s_nop 0
  split_add3      rewrite every v_add3_u32 as two v_add_u32_e32 (same adds, mod 2^32; 4-cycle op -> two 2-cycle
                  ops), applied before the nop rules (A/B: fewer half-rate ops in the stream)
  sched=D[:alt|:group][:orig][:asmnop]  list-schedule the loop body again (VGPR/SGPR/SCC dependences kept, registers
                  unchanged) so that an instruction issues at least D VALU slots after the producers of its operands
                  where the dependences allow; `alt` also prefers alternating 2-/4-cycle ops, `group` runs of one
                  rate (fewer 2 <-> 4-cycle transitions, for lone waves); ties go to the longest remaining critical
                  path, or with `orig` to the compiler's order; `asmnop` first drops the s_nop LLVM places after
                  inline-asm blocks where provably dead (drop_asm_nops); `bank` then renames loop-local values so that fewer
                  v_bitop3_b32 read sources from one VGPR bank (bank_rename; A/B only, profiles/r05/vgpr_bank/).
                  Applied before the nop rules (A/B).  Fails closed: an instruction outside SCHED_VALU (a second
                  destination, an implicit operand, a transcendental op, DPP/SDWA) stops the build
  none            copy through

The Makefile runs tools/issue_equiv.py on every scheduled kernel after the pass: the scheduled loop body must compute
the same registers as the compiler's on random inputs, or the build stops.
"""
import re
import sys

HALF = ("v_alignbit_b32", "v_add3_u32", "v_xad_u32", "v_bfi_b32", "v_lshl_add_u32", "v_lshl_or_b32",
        "v_lshlrev_b32", "v_perm_b32", "v_or3_b32", "v_and_or_b32", "v_add_co_u32", "v_alignbyte_b32")


def main_loop_range(lines, kernel):
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    best = None
    for h in range(start, end):
        if "Loop Header" in lines[h]:
            lab = lines[h].split(":")[0].strip()
            if not lab.startswith(".LBB"):
                lab = lines[h - 1].split(":")[0].strip()
            # the backedge is a conditional branch to the header below it; a loop entered by fallthrough from a
            # latch placed above the header (an outer loop around the hot one) is skipped
            e = next((n for n in range(h + 1, end) if "s_cbranch" in lines[n] and lines[n].split()[-1] == lab), None)
            if e is None:
                continue
            nv = sum(1 for l in lines[h:e] if re.match(r"\s+v_", l))
            if best is None or nv > best[2]:
                best = (h, e, nv)
    return best


def _vgpr(x):
    return re.fullmatch(r"v\d+", x) is not None


def split_add3(line):
    """v_add3_u32 D, A, B, C -> v_add_u32_e32 D, X, Y ; v_add_u32_e32 D, Z, D.  The first add takes every operand
    that is D itself (it is overwritten), and VOP2 takes a non-VGPR operand only as src0.  Returns the lines, or None
    when the operands do not fit that form (the line is then kept as it is)."""
    m = re.match(r"(\s+)v_add3_u32\s+(v\d+),\s*(\S+),\s*(\S+),\s*(\S+)\s*$", line)
    if not m:
        return None
    ind, d, ops = m.group(1), m.group(2), list(m.groups()[2:])
    if sum(1 for o in ops if not _vgpr(o)) > 1:
        return None
    # the operand left for the second add: never D (it is overwritten by the first), preferably the non-VGPR one
    cand = [i for i, o in enumerate(ops) if o != d]
    if not cand:  # D + D + D
        return None
    z = next((i for i in cand if not _vgpr(ops[i])), cand[-1])
    x, y = [o for i, o in enumerate(ops) if i != z]
    if not _vgpr(y):
        x, y = y, x
    if not _vgpr(y):
        return None
    return [f"{ind}v_add_u32_e32 {d}, {x}, {y}", f"{ind}v_add_u32_e32 {d}, {ops[z]}, {d}"]


_REG = re.compile(r"^(v\d+|s\d+|vcc|exec|scc)$")

# The VALU ops the schedule may move (fail closed): each writes exactly one VGPR -- its first
# operand -- and reads only its other operands, with no implicit operand (VCC, EXEC, M0), no second destination (the
# _co_ carry-out ops, v_cmp*, v_readlane / v_readfirstlane, v_div_scale write an SGPR pair or VCC as well), no
# transcendental unit (its results need wait states) and no DPP / SDWA lane crossing.  The PBKDF2 loop uses the first
# five; any other op in a loop body stops the build instead of being list-scheduled on an assumption.
SCHED_VALU = {"v_add3_u32", "v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_bitop3_b32", "v_mov_b32", "v_or_b32",
              "v_and_b32", "v_xor3_b32", "v_or3_b32", "v_xad_u32", "v_bfi_b32", "v_lshl_add_u32", "v_lshl_or_b32",
              "v_and_or_b32", "v_lshlrev_b32", "v_lshrrev_b32", "v_alignbyte_b32", "v_perm_b32"}
_MODIFIER_OK = re.compile(r"^bitop3:0x[0-9a-fA-F]+$")


def _valu_base(op):
    return op.replace("_e32", "").replace("_e64", "")


def _safe_valu(line):
    """(op, dst, [sources]) of a VALU the schedule may move, or a ValueError naming why it may not."""
    m = re.match(r"\s+(v_\w+)\s+(.*)$", line)
    if not m:
        raise ValueError(f"not a VALU: {line!r}")
    op, rest = m.group(1), m.group(2)
    if _valu_base(op) not in SCHED_VALU:
        raise ValueError(f"VALU outside the schedulable set (second destination, implicit operand, transcendental or "
                         f"unknown): {line!r}")
    parts = [p.strip() for p in rest.split(",")]
    last = parts[-1].split()
    parts[-1] = last[0]
    for mod in last[1:]:
        if not (_valu_base(op) == "v_bitop3_b32" and _MODIFIER_OK.match(mod)):
            raise ValueError(f"VALU modifier the schedule does not model ({mod}): {line!r}")
    if not re.fullmatch(r"v\d+", parts[0]):
        raise ValueError(f"VALU destination is not one VGPR: {line!r}")
    for t in parts[1:]:
        if not (re.fullmatch(r"[vs]\d+", t) or re.fullmatch(r"-?(0x[0-9a-fA-F]+|\d+)", t)):
            raise ValueError(f"VALU operand the schedule does not model ({t}): {line!r}")
    return op, parts[0], parts[1:]


def _defs_uses(line):
    """(op, defs, uses) of one loop-body instruction; None for a line that is not an instruction.  Raises ValueError
    for anything the list schedule cannot prove safe to move (see SCHED_VALU): the pass then fails the build."""
    m = re.match(r"\s+([vs]_\w+)\s*(.*)", line)
    if not m:
        return None
    op = m.group(1)
    if op.startswith("v_"):
        _, dst, srcs = _safe_valu(line)
        return op, {dst}, {t for t in srcs if re.fullmatch(r"[vs]\d+", t)}
    toks = [t.strip().split()[0] for t in m.group(2).split(",") if t.strip()]
    regs = [t if _REG.match(t) else None for t in toks]
    if op.startswith("s_cmp"):
        return op, {"scc"}, {r for r in regs if r}
    if op in ("s_add_i32", "s_sub_i32", "s_add_u32", "s_sub_u32"):
        return op, {regs[0], "scc"}, {r for r in regs[1:] if r}
    raise ValueError(f"unexpected instruction in the loop body: {line!r}")


def drop_asm_nops(body):
    """`asmnop`: LLVM puts an `s_nop 0` after every inline-asm block, whose contents it cannot see.  It is dropped only
    where that is provably dead: the block holds only schedulable VALUs (one VGPR out, VGPR / SGPR / constant in) and
    the next instruction is a schedulable VALU reading VGPRs and constants only.  Elsewhere it stays."""
    out = []
    for k, l in enumerate(body):
        if l.strip() == "s_nop 0" and k and body[k - 1].strip() == ";;#ASMEND":
            j = k - 2
            block = []
            while j >= 0 and body[j].strip() != ";;#ASMSTART":
                if body[j].strip() and not body[j].strip().startswith(";"):
                    block.append(body[j])
                j -= 1
            nxt = next((x for x in body[k + 1:] if x.strip() and not x.strip().startswith(";")), None)

            def vgpr_only_valu(x):
                try:
                    _, _, srcs = _safe_valu(x)
                except ValueError:
                    return False
                return not any(re.fullmatch(r"s\d+", t) for t in srcs)

            def safe(x):
                try:
                    _safe_valu(x)
                    return True
                except ValueError:
                    return False
            if j >= 0 and block and all(safe(b) for b in block) and nxt is not None and vgpr_only_valu(nxt):
                continue
        out.append(l)
    return out


def reschedule(body, dmin, alt, group=False, orig=False):
    """Greedy list schedule of a straight-line loop body (see the sched rule)."""
    ins = []
    for l in body:
        du = _defs_uses(l)
        if du:
            ins.append((l,) + du)
    n = len(ins)
    preds = [set() for _ in range(n)]
    raw = [set() for _ in range(n)]
    last_w, readers = {}, {}
    for i, (_, op, defs, uses) in enumerate(ins):
        for r in uses:
            if r in last_w:
                preds[i].add(last_w[r])
                raw[i].add(last_w[r])
        for r in defs:
            if r in last_w:
                preds[i].add(last_w[r])
            for j in readers.get(r, ()):
                if j != i:
                    preds[i].add(j)
        for r in uses:
            readers.setdefault(r, set()).add(i)
        for r in defs:
            last_w[r] = i
            readers[r] = set()
    salu = [i for i in range(n) if ins[i][1].startswith("s_")]
    for i in salu:  # the loop counter stays at the end, next to the branch
        for j in range(n):
            if j not in salu and (ins[i][2] & (ins[j][2] | ins[j][3]) - {"scc"}):
                raise ValueError("a VALU touches the loop counter")
    succs = [[] for _ in range(n)]
    for i in range(n):
        for j in preds[i]:
            succs[j].append(i)
    cp = [0] * n  # longest path to the end (critical path)
    for i in range(n - 1, -1, -1):
        cp[i] = 1 + max((cp[j] for j in succs[i]), default=0)
    left = [len(preds[i]) for i in range(n)]
    ready = {i for i in range(n) if not left[i] and i not in salu}
    pos, order, prev_half = {}, [], None
    while ready:
        def key(i):
            dist = min((len(order) - pos[j] for j in raw[i]), default=dmin)
            half = ins[i][1].replace("_e32", "").replace("_e64", "") in HALF
            return (min(dist, dmin), alt and prev_half is not None and half != prev_half,
                    group and prev_half is not None and half == prev_half, *((-i, cp[i]) if orig else (cp[i], -i)))
        i = max(ready, key=key)
        ready.discard(i)
        pos[i] = len(order)
        order.append(i)
        prev_half = ins[i][1].replace("_e32", "").replace("_e64", "") in HALF
        for j in succs[i]:
            left[j] -= 1
            if not left[j] and j not in salu:
                ready.add(j)
    if len(order) + len(salu) != n:
        raise ValueError("schedule incomplete")
    return [ins[i][0] for i in order + salu]


def _bop3_conflicts(srcs):
    """Source VGPR pairs of one v_bitop3_b32 that share a bank (v % 4)."""
    vs = [int(s[1:]) for s in srcs if _vgpr(s)]
    return sum(1 for a in range(len(vs)) for b in range(a + 1, len(vs)) if vs[a] % 4 == vs[b] % 4 and vs[a] != vs[b])


def bank_rename(body, maxv):
    """Rename loop-local VGPR values so that fewer v_bitop3_b32 read two sources from one bank.  Measured with
    tools/vgpr_bank.hip (profiles/r05/vgpr_bank/): a v_bitop3_b32 whose three sources all sit in one bank (v % 4)
    issues at the half rate; two in one bank cost nothing extra.  Cutting the pairs (99 -> 36 in the q kernel) also
    cuts those triples (4 -> 1); the C2 kernel gained 0.08 %, so this stays an A/B option.  A value is local when the body
    writes its register again later (so it dies inside the body); it moves to a register in [0, maxv] that no
    instruction touches between the value's def and its last use and whose next access after that is a pure write.
    Dependences between instructions only lose false (WAR/WAW) edges; the order is unchanged."""
    if any("v[" in l for l in body):
        raise ValueError("register tuples in the loop body")
    ops = []  # per line: None, or [op, [operand tokens], text prefix]
    for l in body:
        m = re.match(r"(\s+)([vs]_\w+)(\s+)(.*)$", l)
        if not m or _defs_uses(l) is None:
            ops.append(None)
            continue
        parts = m.group(4).split(",")
        ops.append([m.group(2), parts, m.group(1) + m.group(2) + m.group(3)])

    def tok(p):
        return p.strip().split()[0] if p.strip() else ""

    def acc(k):  # (defs, uses) of VGPRs at line k
        if ops[k] is None:
            return set(), set()
        op, parts, _ = ops[k]
        ts = [tok(p) for p in parts]
        if op.startswith("v_"):
            return {ts[0]}, {t for t in ts[1:] if _vgpr(t)}
        return set(), set()

    def value_at(k, reg):
        """(def line, use lines, next def line) of the value register reg gets at line k, or None if not local."""
        uses = []
        for j in range(k + 1, len(body)):
            d, u = acc(j)
            if reg in u:
                uses.append(j)
            if reg in d:
                return k, uses, j
        return None

    def free(reg, a, b):
        """reg holds nothing live over lines [a, b]: no access there, and its next access after b is a pure write."""
        for j in range(a, len(body)):
            d, u = acc(j)
            if j <= b:
                if reg in d or reg in u:
                    return False
            elif reg in u:
                return False
            elif reg in d:
                return True
        return False

    def conflicts():
        return sum(_bop3_conflicts([tok(p) for p in o[1][1:]]) for o in ops if o and o[0] == "v_bitop3_b32")

    def rename(k, uses, old, new):
        op, parts, pre = ops[k]
        parts[0] = parts[0].replace(old, new, 1) if tok(parts[0]) == old else parts[0]
        for j in uses:
            p = ops[j][1]
            for x in range(1, len(p)):
                if tok(p[x]) == old:
                    p[x] = p[x].replace(old, new, 1)

    before = conflicts()
    for k in range(len(body)):
        o = ops[k]
        if not o or o[0] != "v_bitop3_b32":
            continue
        srcs = [tok(p) for p in o[1][1:]]
        if not _bop3_conflicts(srcs):
            continue
        # try to move one source value of a conflicting pair to a bank none of the other sources use
        done = False
        for s in srcs:
            if done or not _vgpr(s):
                continue
            dl = max((j for j in range(k) if s in acc(j)[0]), default=None)
            if dl is None:
                continue
            v = value_at(dl, s)
            if v is None:
                continue
            _, uses, _ = v
            last = max(uses)
            others = {int(t[1:]) % 4 for t in srcs if _vgpr(t) and t != s}
            for r in range(maxv + 1):
                nr = f"v{r}"
                if r % 4 in others or nr == s or not free(nr, dl, last):
                    continue
                # the move must not add conflicts at the value's other bitop3 readers
                old_c = sum(_bop3_conflicts([tok(p) for p in ops[j][1][1:]]) for j in uses if ops[j][0] == "v_bitop3_b32")
                saved = [(j, list(ops[j][1])) for j in [dl] + uses]
                rename(dl, uses, s, nr)
                new_c = sum(_bop3_conflicts([tok(p) for p in ops[j][1][1:]]) for j in uses if ops[j][0] == "v_bitop3_b32")
                if new_c < old_c:
                    done = True
                    break
                for j, p in saved:
                    ops[j][1] = p
    out = [l if ops[k] is None else ops[k][2] + ",".join(ops[k][1]) for k, l in enumerate(body)]
    sys.stderr.write(f"issue_pass: bank: v_bitop3_b32 same-bank source pairs {before} -> {conflicts()}\n")
    return out


def nopify(lines, kernel, rules):
    h, e, nv = main_loop_range(lines, kernel)
    for r in rules:
        if r.startswith("sched="):
            arg = r.split("=", 1)[1].split(":")
            body = lines[h + 1:e]
            if "asmnop" in arg[1:]:
                body = drop_asm_nops(body)
            # fail closed: an instruction the schedule cannot model raises here and stops the build (ISSUE_RULE=none
            # builds the compiler's schedule unchanged)
            body = reschedule(body, int(arg[0]), "alt" in arg[1:], "group" in arg[1:], "orig" in arg[1:])
            if "bank" in arg[1:]:
                start = next(i for i, l in enumerate(lines) if l.startswith(kernel + ":"))
                end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
                maxv = max(int(x) for l in lines[start:end] for x in re.findall(r"\bv(\d+)\b", l))
                body = bank_rename(body, maxv)
            lines = lines[:h + 1] + body + lines[e:]
            e = h + 1 + len(body)
    if "split_add3" in rules:
        body = []
        for l in lines[h + 1:e]:
            body += split_add3(l) or [l]
        lines = lines[:h + 1] + body + lines[e:]
        e = h + 1 + len(body)
    sys.stderr.write(f"issue_pass: {kernel}: main loop {nv} VALU, rules {','.join(rules)}\n")
    out = lines[:h + 1]
    k = 0
    prev_half = False
    every = [int(r.split("=")[1]) for r in rules if r.startswith("every=")]
    for l in lines[h + 1:e]:
        m = re.match(r"\s+(v_\w+)", l)
        if not m:
            out.append(l)
            continue
        op = m.group(1).replace("_e32", "").replace("_e64", "")
        half = op in HALF
        nopw = "\ts_nop 1" if "nop1" in rules else "\ts_nop 0"
        if "before_half" in rules and half:
            out.append(nopw)
        elif "before_half_trans" in rules and half and not prev_half:
            out.append(nopw)
        elif "before_alb" in rules and op == "v_alignbit_b32":
            out.append(nopw)
        elif "before_ad3" in rules and op == "v_add3_u32":
            out.append(nopw)
        elif "before_full_trans" in rules and not half and prev_half:
            out.append(nopw)
        out.append(l)
        k += 1
        ins = False
        if "after_half" in rules and half:
            ins = True
        if "after_full_h" in rules and not half and prev_half:
            ins = True
        if "after_alb" in rules and op == "v_alignbit_b32":
            ins = True
        if every and k % every[0] == 0:
            ins = True
        if ins:
            out.append("\ts_nop 0")
        prev_half = half
    out += lines[e:]
    return out


if __name__ == "__main__":
    src, dst, kernel, rules = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4].split(",")
    lines = open(src).read().split("\n")
    if rules != ["none"]:
        for k in kernel.split("+"):  # several kernels may share one .s
            try:
                lines = nopify(lines, k, rules)
            except ValueError as err:
                sys.stderr.write(f"issue_pass: {k}: {err}\nissue_pass: refusing to schedule this loop; fix the pass "
                                 f"or build with ISSUE_RULE=none\n")
                sys.exit(1)
    open(dst, "w").write("\n".join(lines))
