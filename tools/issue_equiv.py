"""Checks that the issue pass leaves a PBKDF2 loop body's results unchanged: both bodies run on the same random
register file, in a small interpreter of the loop's VALU ops. After one pass through the body every register must
match. That holds for the schedule (same instructions, dependences kept) and for the bank renaming (a renamed value
lives in a register the body writes again before reading it).

    python3 tools/issue_equiv.py build/pbkdf2/pbkdf2_gfx950.s KERNEL[+KERNEL...] RULES [trials]

`make` runs it on every kernel the pass schedules (build/pbkdf2/issue_equiv.ok): the library is not linked unless
the scheduled loops compute what the compiler's do.
"""
import random
import re
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dwpa_amd", "csrc", "gen"))
import issue_pass as P  # noqa: E402

M = 0xFFFFFFFF


def _val(t, regs):
    if re.fullmatch(r"[vs]\d+", t):
        return regs[t]
    return int(t, 0) & M


def run(body, regs):
    for l in body:
        m = re.match(r"\s+([vs]_\w+)\s*(.*)$", l)
        if not m:
            continue
        op = m.group(1)
        if op.startswith("s_"):
            continue  # the loop counter
        parts = [p.strip() for p in m.group(2).split(",")]
        mod = parts[-1].split()[1:] if len(parts[-1].split()) > 1 else []
        parts[-1] = parts[-1].split()[0]
        d, a = parts[0], [_val(t, regs) for t in parts[1:]]
        base = op.replace("_e32", "").replace("_e64", "")
        if base == "v_add3_u32":
            r = (a[0] + a[1] + a[2]) & M
        elif base == "v_add_u32":
            r = (a[0] + a[1]) & M
        elif base == "v_xor_b32":
            r = a[0] ^ a[1]
        elif base == "v_alignbit_b32":
            r = (((a[0] << 32) | a[1]) >> (a[2] & 31)) & M
        elif base == "v_bitop3_b32":
            tt = int(mod[0].split(":")[1], 0)
            r = 0
            for bit in range(32):
                x, y, z = (a[0] >> bit) & 1, (a[1] >> bit) & 1, (a[2] >> bit) & 1
                r |= ((tt >> (x * 4 + y * 2 + z)) & 1) << bit
        elif base == "v_mov_b32":
            r = a[0]
        else:
            raise ValueError(f"op not modelled: {l!r}")
        regs[d] = r
    return regs


def check(path, kernel, rules, trials=3):
    lines = open(path).read().split("\n")
    h, e, _ = P.main_loop_range(lines, kernel)
    ref = lines[h + 1:e]
    out = P.nopify(lines, kernel, rules)
    h2, e2, _ = P.main_loop_range(out, kernel)
    new = out[h2 + 1:e2]
    for t in range(trials):
        rng = random.Random(t)
        init = {f"{c}{i}": rng.getrandbits(32) for c in "vs" for i in range(256)}
        r1 = run(ref, dict(init))
        r2 = run(new, dict(init))
        keys = set(r1) | set(r2)
        bad = [k for k in keys if r1.get(k) != r2.get(k)]
        if bad:
            return False, bad
    return True, []


if __name__ == "__main__":
    # kernels "+"-separated (the Makefile checks every kernel the pass scheduled); exit 1 on any difference
    trials = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    failed = False
    for kern in sys.argv[2].split("+"):
        ok, bad = check(sys.argv[1], kern, sys.argv[3].split(","), trials)
        print(f"issue_equiv: {kern}: " + ("equal" if ok else f"DIFFERENT: {sorted(bad)[:10]}"))
        failed |= not ok
    sys.exit(1 if failed else 0)
