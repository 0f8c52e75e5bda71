"""CPU: the gfx950 issue pass (dwpa_amd/csrc/gen/issue_pass.py) keeps the PBKDF2 loop's results.

tools/issue_equiv.py runs the compiler's loop body and the pass's output on the same random register file in a
small interpreter of the loop's VALU ops, and compares every register after one pass through the body. Covered:
the product rule, and the rule with the `bank` renaming step (an A/B option, not the product). A mutated body must
be caught. Needs the compiler's assembly from `make` (build/pbkdf2/pbkdf2_gfx950.s); skipped without it."""
import os

import pytest

from tools import issue_equiv as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM = os.path.join(ROOT, "build", "pbkdf2", "pbkdf2_gfx950.s")
PRODUCT = "sched=1:alt:orig:asmnop,before_half"

pytestmark = pytest.mark.skipif(not os.path.exists(ASM), reason="build/pbkdf2/pbkdf2_gfx950.s not built")


@pytest.mark.parametrize("rule", [PRODUCT, "sched=1:alt:orig:asmnop:bank,before_half"])
def test_issue_pass_keeps_the_loop_results(rule):
    ok, bad = E.check(ASM, "k_pbkdf2_gfx950_q", rule.split(","), trials=2)
    assert ok, bad


def test_the_checker_catches_a_wrong_operand():
    lines = open(ASM).read().split("\n")
    h, e, _ = E.P.main_loop_range(lines, "k_pbkdf2_gfx950_q")
    body = lines[h + 1:e]
    k = next(i for i, l in enumerate(body) if "v_bitop3_b32" in l)
    parts = body[k].split(",")
    mutated = body[:k] + [",".join([parts[0], parts[2], parts[1]] + parts[3:])] + body[k + 1:]
    if mutated[k] == body[k]:
        pytest.skip("symmetric operands")
    init = {f"{c}{i}": (i * 2654435761 + (c == "s")) & 0xFFFFFFFF for c in "vs" for i in range(256)}
    r1 = E.run(body, dict(init))
    r2 = E.run(mutated, dict(init))
    assert r1 != r2
