"""CPU: the gfx950 issue pass fails closed.

dwpa_amd/csrc/gen/issue_pass.py list-schedules the PBKDF2 loop body again.  It may only move VALU ops whose one
destination is their first operand (SCHED_VALU); a loop holding anything else -- a carry pair (_co_ ops write VCC as a
second destination), a v_cmp, a v_readlane, a transcendental op, DPP -- must stop the build, not be scheduled on an
assumption.  `asmnop` drops LLVM's s_nop after an inline-asm block only where the block and the next instruction are
plain VGPR VALUs.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dwpa_amd", "csrc", "gen"))
import issue_pass as P  # noqa: E402

RULE = "sched=1:alt:orig:asmnop,before_half"


def _kernel(body):
    return ["k_test:", "\ts_mov_b32 s4, 4096", ".LBB0_1:                                ; =>This Inner Loop Header: Depth=1",
            *body, "\ts_add_i32 s4, s4, -1", "\ts_cmp_lg_u32 s4, 0", "\ts_cbranch_scc1 .LBB0_1", "\ts_endpgm", ""]


PLAIN = ["\tv_add_u32_e32 v1, v2, v3", "\tv_alignbit_b32 v4, v1, v1, 27", "\tv_xor_b32_e32 v5, v4, v2",
         "\tv_add3_u32 v6, v5, s8, v1"]


def test_plain_loop_is_scheduled():
    out = P.nopify(_kernel(PLAIN), "k_test", RULE.split(","))
    assert sum(1 for l in out if l.strip() == "s_nop 0") == 2  # before the two 4-cycle ops


@pytest.mark.parametrize("bad", [
    ["\tv_add_co_u32_e32 v1, vcc, v2, v3", "\tv_addc_co_u32_e32 v4, vcc, v5, v6, vcc"],  # carry pair
    ["\tv_add_co_u32_e64 v1, s[10:11], v2, v3"],                                         # carry into an SGPR pair
    ["\tv_cmp_eq_u32_e32 vcc, v1, v2"],
    ["\tv_readlane_b32 s9, v1, 3"],
    ["\tv_readfirstlane_b32 s9, v1"],
    ["\tv_rcp_f32_e32 v1, v2"],                                                            # transcendental
    ["\tv_mov_b32_dpp v1, v2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"],
    ["\tv_cndmask_b32_e32 v1, v2, v3, vcc"],                                              # implicit VCC read
    ["\tv_xor_b32_e32 v1, vcc_lo, v2"],
])
def test_unmodelled_instruction_stops_the_pass(bad, tmp_path):
    lines = _kernel(PLAIN[:2] + bad + PLAIN[2:])
    with pytest.raises(ValueError):
        P.nopify(lines, "k_test", RULE.split(","))
    src, dst = tmp_path / "in.s", tmp_path / "out.s"
    src.write_text("\n".join(lines))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "dwpa_amd", "csrc", "gen", "issue_pass.py"), str(src),
                        str(dst), "k_test", RULE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "refusing to schedule" in r.stderr
    assert not dst.exists()
    # ISSUE_RULE=none still builds (the compiler's schedule, unchanged)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "dwpa_amd", "csrc", "gen", "issue_pass.py"), str(src),
                        str(dst), "k_test", "none"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and dst.read_text() == src.read_text()


def test_asm_nop_dropped_only_when_provably_dead():
    blk = ["\t;;#ASMSTART", "\tv_bitop3_b32 v7, v1, v2, v3 bitop3:0x96", "\t;;#ASMEND", "\ts_nop 0"]
    # next instruction reads VGPRs only: the nop goes
    body = PLAIN[:2] + blk + ["\tv_xor_b32_e32 v8, v7, v4"]
    assert "\ts_nop 0" not in P.drop_asm_nops(body)
    # next instruction reads an SGPR: kept
    body = PLAIN[:2] + blk + ["\tv_add3_u32 v8, v7, s8, v4"]
    assert "\ts_nop 0" in P.drop_asm_nops(body)
    # the block writes an SGPR (v_readlane): kept, and the schedule then refuses the body
    bad = ["\t;;#ASMSTART", "\tv_readlane_b32 s9, v1, 3", "\t;;#ASMEND", "\ts_nop 0"]
    body = PLAIN[:2] + bad + ["\tv_xor_b32_e32 v8, v7, v4"]
    assert "\ts_nop 0" in P.drop_asm_nops(body)
    with pytest.raises(ValueError):
        P.nopify(_kernel(body), "k_test", RULE.split(","))


def test_makefile_runs_the_equivalence_check():
    mk = open(os.path.join(ROOT, "Makefile")).read()
    assert "build/pbkdf2/pbkdf2_gfx950.hsaco: build/pbkdf2/pbkdf2_issue.s build/pbkdf2/issue_equiv.ok" in mk
    assert "python3 tools/issue_equiv.py $< $(PBKDF2_KERNELS) $(ISSUE_RULE)" in mk
