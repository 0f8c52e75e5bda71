"""The issue-cost roofline of the PBKDF2 kernel from measured gfx950 VALU issue costs.

`tools/bin/valu_peak` measures SIMD-cycles per wave64 instruction for each VALU op the SHA-1 loop uses
(profiles/rNN/valu_issue_costs.json).  With f = the full-rate cost (v_xor / v_bitop3 / v_add_u32) and h = the
half-rate cost (v_alignbit / v_add3), the cheapest HMAC inner-loop compression of PBKDF2's 84-byte message costs

    78 rounds x (rotl5 h + rotl30 h + f() f + 4 adds min(4f, 2h))
  - one add in each of the 14 rounds whose K+W or e+K is loop-invariant      (-14 f)
  + rounds 0-1 folded into midstate invariants                                (5 f)
  + schedule: 64 rotates + SCHED_XORS xor/bitop3                             (64 h + SCHED_XORS f)
  + digest adds                                                               (5 f)
  + T ^= U, 5 xors per two compressions (one of them folded)                  (1.25 f)

SCHED_XORS is the schedule's XOR-type op count (tools/sched_identities.py).  The plain recurrence needs 112; rounds 1-4
priced the model on that, C_min = 1,878.5.  Round 5 found that the recurrence applied 2^j times reaches the message's
zero words: 99 ops with j <= 1, which is what the kernel runs (DWPA_SCHED_WIDE=1, 61 VGPRs), and 84 with j <= 2, whose
longer live ranges spill at 8 waves.  The model takes the cheapest known form, 84: C_min = 1,822.5 at f = 2, h = 4.
Peak = SIMDs x clock x 64 / C_min.

    python tools/cmin.py profiles/r02/valu_issue_costs.json     # prints the peak from a fresh measurement
"""
from __future__ import annotations

import json
import sys

FULL_OPS = ("v_xor_b32", "v_bitop3_b32", "v_add_u32")
HALF_OPS = ("v_alignbit_b32", "v_add3_u32")
SIMDS, CLOCK_HZ, COMPRESSIONS_PER_PMK = 1024, 2.4e9, 16388


SCHED_XORS = 84  # the cheapest known schedule (j <= 2); the kernel's j <= 1 form has 99


def c_min(f: float = 2.0, h: float = 4.0, sched_xors: int = SCHED_XORS) -> float:
    return 78 * (2 * h + f + min(4 * f, 2 * h)) - 14 * f + 5 * f + (64 * h + sched_xors * f) + 5 * f + 1.25 * f


def from_costs(path: str) -> dict:
    with open(path) as fh:
        d = json.load(fh)
    cyc = {r["op"]: r["simd_cycles_per_wave_inst"] for r in d["results"]}
    f = max(cyc[o] for o in FULL_OPS if o in cyc)
    h = max(cyc[o] for o in HALF_OPS if o in cyc)
    model = c_min(round(f), round(h))
    measured = c_min(f, h)
    peak = SIMDS * CLOCK_HZ * 64 / model
    return {"source": path, "full_rate_cycles": round(f, 3), "half_rate_cycles": round(h, 3),
            "c_min_model": model, "c_min_measured_costs": round(measured, 1),
            "peak_compressions_per_s": peak, "peak_pmk_per_s": peak / COMPRESSIONS_PER_PMK,
            "peak_pmk_per_s_measured_costs": SIMDS * CLOCK_HZ * 64 / measured / COMPRESSIONS_PER_PMK}


if __name__ == "__main__":
    print(json.dumps(from_costs(sys.argv[1]) if len(sys.argv) > 1 else {"c_min_model": c_min()}))
