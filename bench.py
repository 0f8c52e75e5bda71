"""bench.py -- PMK/s (PBKDF2-HMAC-SHA1 x4096) of the m22000 engine on MI355X, BASELINE.json configs[1] (C2).

Workload (per GPU): one ESSID, one EAPOL keyver-2 hashline (message_pair 0x80, planted nonce correction +3 LE,
hashcat nonce mode --nonce-error-corrections=8 -> 33 attempts, as help_crack.py:773 runs it), a 100M-word
synthetic dictionary resident in HBM (uint64 offsets + bytes, lengths geometric around 10 clipped to [8, 63];
the true PSK is word 99,999,000).  A step = one batch
of the dictionary through the hot path: candidates -> HMAC midstates -> PBKDF2 -> verify.  Rank r of N scans its
own 100M-word shard of an N x 100M-word node dictionary (rank 0's is the one above; no two ranks derive the same
PMK, no collective on the data path): weak scaling.

The JSON line carries the PBKDF2 kernel's roofline (integer VALU bound) from HIP events recorded around each
launch on the stream it runs on, and the CPU baseline (the OpenSSL restatement of check_key_m22000 from
oracle/, timed on this host's cores on a bounded sample of the same workload: 1 thread = one PHP request, and
the box's CPU share).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "PMK/s (PBKDF2-HMAC-SHA1 x4096) per GPU and per 8×MI355X node, m22000"
DICT_WORDS = 100_000_000
PLANT_INDEX = 99_999_000
NC = 8          # nonce-error-corrections of the client (help_crack.py:773); the CPU baseline's PHP window
NC_MODE = 1     # DWPA_NC_HASHCAT: N+0 then +-1..+-8 in both endians = 33 attempts per candidate
# Roofline.  Work unit: 16,388 SHA-1 compressions per PMK (north_star).  Bound: integer
# VALU issue.  Measured on gfx950 (tools/valu_peak, profiles/r01/valu_issue_costs.json): xor/bitop3/add_u32 take
# 2 SIMD cycles per wave64 instruction, alignbit (rotate) and add3 take 4, so the cheapest known HMAC inner-loop
# compression costs C_MIN = 1822.5 SIMD-cycles per wave (64 lanes; derivation in DESIGN.md section 4 and
# tools/cmin.py: with the schedule identities of round 5; rounds 1-4 priced it at 1878.5 with the plain recurrence).
COMPRESSIONS_PER_PMK = 16388
SIMDS, CLOCK_HZ = 256 * 4, 2.4e9
from tools.cmin import c_min  # noqa: E402  (the C_min model; tools/regen_peak.sh re-measures its inputs)
C_MIN_CYCLES = c_min()  # 1822.5 at full rate 2 / half rate 4 SIMD-cycles per wave instruction
PEAK_COMPRESSIONS = SIMDS * CLOCK_HZ * 64 / C_MIN_CYCLES
# HBM traffic per PMK of the kernel each workload's roofline names, from the PMC passes of tools/profile_traffic.sh
# over that workload's bench command (FETCH_SIZE doubled as MI355X_MICROARCH.md "HBM [CDNA4]" prescribes, plus
# WRITE_SIZE; per-launch medians divided by the PMKs of the launch).  PMC counters cannot be read inside a timed
# run, so the bench scales the measured per-PMK figure to its launches.
#   c2/c4: k_pbkdf2_gfx950_q (the work-queue kernel multi-round scans run), profiles/r06/pmc (round 6's last code,
#          tools/profile_traffic.sh, median of the full 16,777,216-PMK launches): FETCH 360,959,040 B x 2 = 43.0 B/PMK
#          (a slot range's two output-block items are taken back to back, so the second read of each 40-byte key
#          midstate is an L2 hit) + WRITE 553,910,272 B = 33.0 B/PMK (round 5, profiles/r05/pmc_final: FETCH
#          358,833,216 B; round 4: 356,765,120 B; round 2: 365,219,648 B; the same WRITE)
#   c3:    k_pbkdf2_gfx950_mg_q + k_verify<PMKID> + k_verify<keyver 2> per dwpa_scan_run (the roofline's events
#          bracket all three), profiles/r02/traffic_q3: 463.9 + 446.6 + 1,093.9 MB for 13,445,190 PMKs
TRAFFIC_BYTES_PER_PMK = {"c2": (2 * 360959040 + 553910272) / 16777216, "c4": (2 * 360959040 + 553910272) / 16777216,
                         "c3": (463.935e6 + 446.650e6 + 1093.884e6) / 13445190}
TRAFFIC_SOURCE = {"c2": "k_pbkdf2_gfx950_q, profiles/r06/pmc",
                  "c4": "k_pbkdf2_gfx950_q per PMK as measured on c2, profiles/r06/pmc",
                  "c3": "k_pbkdf2_gfx950_mg_q + k_verify, profiles/r02/traffic_q3"}
# Algorithmic bytes per PMK: PBKDF2 reads the 40-byte key midstate once and writes the 32-byte PMK (c2/c4, the
# kernel the roofline names).  c3's events also bracket the verify, which reads each PMK (32 B) and candidate id
# (8 B) once per hashline of its ESSID; its midstates are shared by all ESSID groups.
ALGO_BYTES_PER_PMK = 40 + 32
# Guide view (MI355X_MICROARCH.md: 4 SIMD-32 per CU, one VALU per 2 cycles = 128 int32 lane-ops/clk/CU at 2.4 GHz,
# every op full rate).  Reported beside the issue-cost roofline, with SURVEY.md 8(d)'s ideal 617 ops per compression
# and with the 558 VALU the kernel issues per compression (1,116 per loop iteration of two compressions with round 5's
# schedule identities in k_pbkdf2_gfx950_q; 575.5 before them, 4,714,742 per wave / 8,192 compressions in PMC).  Not
# attainable on gfx950, where v_alignbit/v_add3/v_bfi issue at half rate (profiles/r01/valu_issue_costs.json).
SURVEY_OPS_PER_COMPRESSION = 617
ISSUED_OPS_PER_COMPRESSION = 558
PEAK_LANE_OPS = 256 * 128 * CLOCK_HZ


def roofline_block(kernel, kernel_pmk_s, pmk_per_launch, kernel_ms, traffic_pmk, traffic_src, algo_bytes_per_pmk,
                   peak_costs=None):
    """The bench line's roofline object.  Headline (`achieved` / `peak` / `frac`): the guide's integer-VALU peak
    (MI355X_MICROARCH.md: 256 CU x 128 int32 lane-ops/clk x 2.4 GHz = 78.64 T lane-ops/s) against SURVEY.md 8(d)'s
    ideal 617 ops per SHA-1 compression x 16,388 compressions per PMK, so frac = PMKs per launch x 16,388 x 617 /
    mean launch duration / 78.64e12.  Beside it: the same kernel against the issue-cost model measured on gfx950
    (rotates and 3-input adds issue at half rate), and the most the guide basis can show under
    that model."""
    comp_s = kernel_pmk_s * COMPRESSIONS_PER_PMK
    ops_s = comp_s * SURVEY_OPS_PER_COMPRESSION
    return {
        "bound": "valu",
        "kernel": kernel,
        "achieved": round(ops_s / 1e12, 3),
        "peak": round(PEAK_LANE_OPS / 1e12, 3),
        "unit": f"T int32 lane-ops/s ({SURVEY_OPS_PER_COMPRESSION} ops per SHA-1 compression x "
                f"{COMPRESSIONS_PER_PMK} compressions per PMK)",
        "frac": round(ops_s / PEAK_LANE_OPS, 4),
        "peak_basis": "MI355X_MICROARCH.md: 256 CU x 128 int32 lane-ops/clk x 2.4 GHz = 78.64 T lane-ops/s; "
                      f"SURVEY.md 8(d): {SURVEY_OPS_PER_COMPRESSION} ideal VALU ops per SHA-1 compression",
        "roofline_pmk_per_s": round(PEAK_LANE_OPS / SURVEY_OPS_PER_COMPRESSION / COMPRESSIONS_PER_PMK, 1),
        "traffic": round(traffic_pmk * pmk_per_launch) if traffic_pmk else None,
        "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE of this workload, "
                        + (traffic_src or "not measured") + ")",
        "algorithmic_bytes": round(algo_bytes_per_pmk * pmk_per_launch),
        "hbm_gbs": round(traffic_pmk * pmk_per_launch / (kernel_ms * 1e-3) / 1e9, 3) if traffic_pmk else None,
        "kernel_ms": round(kernel_ms, 3),
        "pmk_per_launch": pmk_per_launch,
        "kernel_pmk_per_s": round(kernel_pmk_s, 1),
        # the most the guide basis can show on gfx950: the cheapest compression under the measured issue costs
        "frac_attainable_on_gfx950": round(PEAK_COMPRESSIONS * SURVEY_OPS_PER_COMPRESSION / PEAK_LANE_OPS, 4),
        "frac_issue_cost_model": round(comp_s / PEAK_COMPRESSIONS, 4),
        "issue_cost_model": {
            "achieved": round(comp_s / 1e9, 3), "peak": round(PEAK_COMPRESSIONS / 1e9, 3),
            "unit": "G SHA-1 compressions/s",
            "roofline_pmk_per_s": round(PEAK_COMPRESSIONS / COMPRESSIONS_PER_PMK, 1),
            "basis": f"{SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz x 64 lanes / {C_MIN_CYCLES} SIMD-cycles per compression "
                     "(measured gfx950 issue costs: full rate 2, half rate 4 SIMD-cycles per wave64 instruction; "
                     "tools/cmin.py, " + (peak_costs or "profiles/r01/valu_issue_costs.json") + ")"},
        "frac_nominal_ops": round(comp_s * ISSUED_OPS_PER_COMPRESSION / PEAK_LANE_OPS, 4),
        "frac_nominal_ops_basis": f"{ISSUED_OPS_PER_COMPRESSION} VALU issued per compression (PMC) / "
                                  "78.64 T int32 lane-ops/s",
    }


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node.  Under a launcher (WORLD_SIZE set) it must equal WORLD_SIZE; "
                         "without one, N > 1 starts N rank processes of this script itself (one per GPU, "
                         "LOCAL_RANK = device) and prints rank 0's line.  Default: WORLD_SIZE, else 1")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak (default): every rank scans its own batches, fixed work per GPU per step.  strong "
                         "(c4 only): a step exhausts the whole 10^8 keyspace once, rank g of G taking the "
                         "contiguous range [g*10^8/G, (g+1)*10^8/G) (SURVEY.md 8(d) C4); value = node PMK/s")
    ap.add_argument("--t1-s", type=float, default=None,
                    help="strong scaling: the one-GPU time to exhaust the keyspace (a previous --gpus 1 run's "
                         "t_exhaust_s); the line then reports speedup S(G) = T1 / TG")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: every rank builds its shard schedule and runs the control plane only (gloo "
                         "barrier, max/sum reductions); rank 0 prints the ranks' coverage (tests the N-rank path)")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 24,
                    help="candidates per step per GPU (one PBKDF2 launch of 64 wave rounds; 4M-candidate steps "
                         "measured 0.2 %% slower per PMK: one launch tail per 16 rounds, profiles/r02/batch_size)")
    ap.add_argument("--dict-words", type=int, default=DICT_WORDS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--peak-costs", default=None,
                    help="price the roofline from a fresh tools/bin/valu_peak measurement (tools/regen_peak.sh output)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="batches in flight (c2/c3/c4), each on its own scan working set and HIP stream.  Measured "
                         "A/B (profiles/r01/pipeline/): 2 gains 0.2 %% -- the next batch's PBKDF2 waves hold the "
                         "SIMDs, so the verify runs starved beside it -- and blurs the per-kernel events; default 1")
    ap.add_argument("--rule-words", type=int, default=1_000_000,
                    help="c3files: base words of the gz dictionary the WPA rule set is applied to")
    ap.add_argument("--workload", choices=["c1", "c2", "c3", "c4", "c5", "c2files", "c3files", "c1lat", "c1cold",
                                           "expand"],
                    default="c2",
                    help="c2 = BASELINE configs[1] (the bench line); c3/c4 = configs[2]/[3] legs; "
                         "c1/c5 = the FFI check path (host buffers, PCIe-inclusive); c2files = C2 through "
                         "dwpa_crack_files from a gz dictionary on disk (the help_crack client path); c3files = "
                         "the client's rule pass: a gz dictionary x the WPA rule set through dwpa_crack_files; "
                         "c1lat = server call latency at 1/16/202 keys per call beside one CPU core; c1cold = the "
                         "server path as PHP-FPM runs it: fresh worker processes, first-call cost, per-worker "
                         "footprint, K concurrent workers; expand = help_crack's `hashcat --stdout -r` wordlist "
                         "expansion (dwpa_rules_expand_file)")
    ap.add_argument("--cold-role", choices=["parent", "worker", "context"], default="parent",
                    help=argparse.SUPPRESS)  # c1cold: the child processes the parent starts
    ap.add_argument("--cold-id", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--cold-warmup", action="store_true",
                    help="c1cold workers start the HIP runtime before their first call (dwpa22000_warmup()'s model) "
                         "instead of the PHP wrapper's default (dwpa_init with the host backend allowed, no probe)")
    ap.add_argument("--cold-k", default="4,8,16",
                    help="c1cold: concurrent worker counts (each a fresh process; the box allows 16 GPU processes)")
    ap.add_argument("--rules-set", choices=["wpa", "server"], default="wpa",
                    help="c3files: the rules file -- wpa (148 rules of bestWPA.rule's ops) or server (those plus 67 "
                         "lines of the rest of hashcat's rule language: title case, inserts, memory, reject ...)")
    ap.add_argument("--rule-mode", choices=["hashcat", "full"], default="hashcat",
                    help="c3files: the rules file's loader -- hashcat (default: lines with reject / memory functions "
                         "are skipped, as hashcat's -r loader does) or full (they run too)")
    ap.add_argument("--essids", type=int, default=1000, help="c3: number of ESSIDs (BASELINE: 1000)")
    ap.add_argument("--scan-run", action="store_true",
                    help="c2/c4: derive + verify through dwpa_scan_run (the multi-group kernel C3 uses) instead of "
                         "the per-group calls (A/B of the two PBKDF2 entry points)")
    ap.add_argument("--short-words", action="store_true",
                    help="c2files: lengths geometric(0.3)+6 so ~30 %% of the words are shorter than 8 and dropped "
                         "by the m22000 filter (as in real wordlists); PMK/s counts only 8..63-byte words")
    ap.add_argument("--start-at", type=float, default=None,
                    help="c1/c5: after the warmup, wait until this Unix time before the timed calls, so that separate "
                         "bench processes on one GPU (PHP-FPM workers) time the same window; the line then carries "
                         "the window's Unix start and end")
    ap.add_argument("--callers", type=int, default=1,
                    help="c1/c5: concurrent callers (host threads, as PHP ZTS workers or a threaded server), each "
                         "making the step's call on its own argument block; the library runs up to "
                         "DWPA_CALLS_PER_DEVICE (default 2) calls per GPU at once.  value = all callers' PMKs / wall")
    return ap.parse_args()


_JSON_FD = None


def quiet_stdout() -> None:
    """Keep stdout for the one JSON line: fd 1 goes to stderr from here on (gloo prints its connection banner and
    runtimes may print notices there) and emit() writes the line to the original stdout."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def emit(obj) -> None:
    data = (json.dumps(obj) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(data.decode())
        sys.stdout.flush()
        return
    while data:
        data = data[os.write(_JSON_FD, data):]


def make_dictionary(n, seed=2):
    """Host-side synthetic dictionary in the HBM layout (uint64 offsets + bytes), lengths geometric(0.3)+7 -> [8, 63].
    Weak scaling gives rank r the seed 2 + r: its own shard of the node dictionary."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lens = np.clip(rng.geometric(0.3, n) + 7, 8, 63).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0x21, 0x7F, int(off[-1]) + 64, dtype=np.uint8)
    return off, data


def _pmk_cache(S, essid):
    cache = {}

    def pmk_of(psk):
        if psk not in cache:
            cache[psk] = S.pmk(psk, essid)
        return cache[psk]
    return pmk_of


def verify_timed_hits(w, hits, batches):
    """The hits of the timed steps (untimed check): every reported hit is genuine (w.genuine
    re-derives it: the candidate at the reported id is the line's PSK and the PMK is the oracle's), and every expected
    (line, candidate) -- the plant, and in C3 every line whose PSK is in the keyspace -- is reported exactly once per
    timed scan of the batch that holds it."""
    from collections import Counter
    got = Counter((h["line"], h["cand"]) for h in hits)
    false_hits = sum(1 for h in hits if not w.genuine(h))
    scans = Counter(batches)
    missing = extra = 0
    for key, b in w.expected.items():
        want, have = scans.get(b, 0), got.get(key, 0)
        missing += max(0, want - have)
        extra += max(0, have - want)
    plant_scans = scans.get(w.plant_batch, 0)
    return (false_hits == 0 and missing == 0 and extra == 0), {
        "timed_hits": len(hits), "timed_hits_false": false_hits, "timed_expected_missing": missing,
        "timed_expected_extra": extra, "timed_plant_scans": plant_scans,
        "expected_pairs": len(w.expected), "timed_expected_reports": sum(scans.get(b, 0) for b in w.expected.values())}


class Workload:
    """One BASELINE.json config as a sequence of steps over HBM-resident candidates."""
    name = ""
    description = ""


def build_c2(args, local, S, Scan, Dictionary, shard=0):
    """configs[1]: one ESSID, one EAPOL keyver-2 line, 100M-word dictionary.  Shard r (weak scaling, rank r) is its
    own 100M-word dictionary (seed 2 + r) with its own planted PSK at the same index, so the ranks' (ESSID, word)
    units are disjoint."""
    import random
    w = Workload()
    n = args.dict_words
    w.plant = min(PLANT_INDEX, n - 1)
    w.off, w.data = make_dictionary(n, seed=2 + shard)
    w.psk = w.data[int(w.off[w.plant]):int(w.off[w.plant + 1])].tobytes()
    rng = random.Random(1)
    w.essid, ap, sta, an, sn = S.random_net(rng, essid_len=10)
    w.line = S.eapol_line(w.psk, w.essid, ap, sta, an, sn, 2, 3, "LE", mp=0x80, rng=rng)
    w.dict = Dictionary(w.off, w.data, device=local)
    w.B = (args.batch + 63) & ~63
    w.nbatches = (n + w.B - 1) // w.B
    w.scans = [Scan([w.line], device=local, nc=NC, nc_mode=NC_MODE, batch=w.B) for _ in range(args.pipeline)]
    w.groups = 1
    w.name = "C2"
    w.description = ("C2: one ESSID, one EAPOL keyver-2 line (mp 0x80, planted NC +3 LE), 100M-word synthetic "
                     "dictionary resident in HBM, hashcat nonce mode --nonce-error-corrections=8 (33 attempts)")
    w.extra = {"dict_words": n, "shards": "weak: rank r scans its own dict_words-word shard (seed 2 + r) of the node "
                                         "dictionary, one batch per step"}

    def load(i, hs, sc):
        first = (i % w.nbatches) * w.B
        cnt = min(w.B, n - first)
        sc.load_dict(w.dict.off.ptr, w.dict.data.ptr, first, cnt, 8, 63, hs)
        return cnt

    def check(hits):
        return any(h["cand"] == w.plant and h["nc"] == 3 and h["endian"] == "LE" and h["pmk"] == S.pmk(w.psk, w.essid)
                   for h in hits)

    def genuine(h):  # the reported word is the line's PSK (the plant, or a dictionary duplicate of it)
        word = w.data[int(w.off[h["cand"]]):int(w.off[h["cand"] + 1])].tobytes()
        return h["line"] == 0 and word == w.psk and (h["nc"], h["endian"]) == (3, "LE") and h["pmk"] == pmk_of(w.psk)

    def cpu_keys(m):  # the m dictionary words ending at the planted PSK
        lo = w.plant - m + 1
        o = w.off[lo:w.plant + 2].astype("int64")
        raw = w.data[o[0]:o[-1]].tobytes()
        return [raw[o[i] - o[0]:o[i + 1] - o[0]] for i in range(m)]
    pmk_of = _pmk_cache(S, w.essid)
    w.load, w.check, w.plant_batch = load, check, w.plant // w.B
    w.genuine, w.expected = genuine, {(0, w.plant): w.plant_batch}
    w.cpu_line, w.cpu_keys, w.cpu_what = w.line, cpu_keys, "dictionary words"
    w.algo_bytes_per_pmk = ALGO_BYTES_PER_PMK
    return w


def build_c4(args, local, S, Scan, Dictionary, shard=0):
    """configs[3]: 8-digit numeric keyspace 00000000..99999999 generated in-kernel, one ESSID (PMKID line).  Weak
    scaling gives rank r its own ESSID (shard r), strong scaling splits shard 0's keyspace."""
    import random
    w = Workload()
    n = 10 ** 8
    w.plant = 73019412
    rng = random.Random(3 if shard == 0 else 3000 + shard)
    w.essid, ap, sta, an, sn = S.random_net(rng, essid_len=8)
    w.line = S.pmkid_line(b"%08d" % w.plant, w.essid, ap, sta)
    w.B = (args.batch + 63) & ~63
    w.nbatches = (n + w.B - 1) // w.B
    w.scans = [Scan([w.line], device=local, nc=NC, nc_mode=0, batch=w.B) for _ in range(args.pipeline)]
    w.groups = 1
    w.name = "C4"
    w.description = "C4: 8-digit numeric keyspace (10^8) generated on the GPU, one ESSID, PMKID line"
    w.extra = {"keyspace": n, "shards": "weak: rank r scans the keyspace of its own ESSID, one batch per step"}

    def load(i, hs, sc):
        first = (i % w.nbatches) * w.B
        cnt = min(w.B, n - first)
        sc.load_numeric(first, cnt, 8, hs)
        return cnt

    def check(hits):
        return any(h["cand"] == w.plant and h["pmk"] == S.pmk(b"%08d" % w.plant, w.essid) for h in hits)

    def genuine(h):
        return h["line"] == 0 and h["cand"] == w.plant and h["pmk"] == pmk_of(b"%08d" % w.plant)
    pmk_of = _pmk_cache(S, w.essid)
    w.load, w.check, w.plant_batch = load, check, w.plant // w.B
    w.genuine, w.expected = genuine, {(0, w.plant): w.plant_batch}
    w.cpu_line, w.cpu_keys = w.line, lambda m: [b"%08d" % v for v in range(w.plant - m + 1, w.plant + 1)]
    w.cpu_what = "8-digit candidates"
    w.algo_bytes_per_pmk = ALGO_BYTES_PER_PMK
    return w


def build_c3(args, local, S, Scan, Dictionary, shard=0):
    """configs[2]: 10k-word dictionary x WPA rule set amplified on the GPU, across E ESSIDs with 1-4 lines each;
    each PMK is derived once per ESSID x candidate and tested against every line of that ESSID.  Weak scaling gives
    rank r its own E ESSIDs (shard r; same words, rules and planted PSKs)."""
    import random
    from dwpa_amd.rulesets import wpa_rules
    from dwpa_amd.device import dictionary_arrays
    import dwpa_amd
    w = Workload()
    rng = random.Random(4)
    net_rng = rng if shard == 0 else random.Random(4000 + shard)
    base = [S.random_psk(rng, 6, 12) for _ in range(10000)]
    rules = wpa_rules()
    picks = [(rng.randrange(len(base)), rng.randrange(len(rules))) for _ in range(4 * args.essids)]
    expanded = dwpa_amd.rules_expand("\n".join(rules), [base[wi] for wi, _ in picks], device=local)
    w.off, w.data = dictionary_arrays(base)
    w.dict = Dictionary(w.off, w.data, device=local)
    lines, w.plants = [], []
    line_psk = []  # per line: (PSK or None when it is outside the keyspace, ESSID, candidate id)
    for e in range(args.essids):
        essid, ap, sta, an, sn = S.random_net(net_rng)
        for k in range(rng.randint(1, 4)):
            wi, ri = picks[4 * e + k]
            psk = expanded[4 * e + k][ri]
            if not psk or not 8 <= len(psk) <= 63:
                psk = b"not-in-keyspace-%d" % k
                line_psk.append((None, essid, None))
            else:
                line_psk.append((psk, essid, wi * len(rules) + ri))
                if e == 0 and k == 0:
                    w.plants.append((len(lines), wi * len(rules) + ri, essid, psk))
            if k % 2:
                lines.append(S.pmkid_line(psk, essid, rng.randbytes(6), sta))
            else:
                lines.append(S.eapol_line(psk, essid, ap, sta, an, sn, 2, rng.randint(-3, 3), "LE", rng=rng))
    # one step = args.batch PMKs spread over every ESSID: batch/E candidates x E ESSID groups, derived by
    # multi-group PBKDF2 launches (dwpa_scan_run).  Rule filtering makes the per-step count data-dependent, so the
    # last wave round of each launch is partial; a 16M-candidate step keeps that tail near 2 %.
    w.B = max(len(rules) + 63, args.batch // max(1, args.essids)) // 64 * 64
    w.scans = [Scan(lines, device=local, nc=NC, nc_mode=NC_MODE, batch=w.B) for _ in range(args.pipeline)]
    w.nrules = [sc.set_rules("\n".join(rules)) for sc in w.scans][0]
    w.words_per_step = max(1, w.B // w.nrules)
    w.nbatches = (len(base) + w.words_per_step - 1) // w.words_per_step
    w.groups = w.scans[0].groups
    w.name = "C3"
    w.description = (f"C3: 10k-word dictionary x {w.nrules} WPA rules amplified on the GPU (8..63 filter), "
                     f"{w.groups} ESSIDs x 1-4 lines, one PMK per ESSID x candidate")
    w.extra = {"essids": w.groups, "lines": len(lines), "rules": w.nrules,
               "shards": "weak: rank r scans the candidates against its own ESSIDs, one batch per step"}

    def load(i, hs, sc):
        first = (i % w.nbatches) * w.words_per_step
        nw = min(w.words_per_step, len(base) - first)
        sc.load_rules(w.dict.off.ptr, w.dict.data.ptr, first, nw, hs)
        return sc.loaded(hs) * w.groups

    def check(hits):
        return all(any(h["line"] == li and h["pmk"] == S.pmk(psk, essid) for h in hits)
                   for li, cand, essid, psk in w.plants)

    from oracle import rules as R
    parsed_rules = [R.parse(r) for r in rules]
    pmks = {}

    def genuine(h):  # the reported (word, rule) candidate is the line's PSK, and the PMK is the oracle's
        psk, essid, _ = line_psk[h["line"]]
        wi, ri = divmod(h["cand"], w.nrules)
        if psk is None or R.apply(parsed_rules[ri], base[wi]) != psk:
            return False
        if h["line"] not in pmks:
            pmks[h["line"]] = S.pmk(psk, essid)
        return h["pmk"] == pmks[h["line"]]
    # every in-keyspace line is reported once per scan of the batch holding its (word, rule) candidate
    w.genuine = genuine
    assert w.nrules == len(rules), "every rule of the WPA set parses, so candidate ids are word * len(rules) + rule"
    w.expected = {(li, c): (c // w.nrules) // w.words_per_step
                  for li, (psk, _, c) in enumerate(line_psk) if psk is not None}

    def cpu_keys(m):  # the m rule candidates (word-major, 8..63 only) ending at the first planted one
        from oracle import rules as R
        _, cand, _, psk = w.plants[0]
        wi, ri = divmod(cand, w.nrules)
        parsed = [R.parse(r) for r in rules]
        out = [c for c in (R.apply(parsed[r], base[wi]) for r in range(ri + 1)) if c and 8 <= len(c) <= 63]
        j = wi - 1
        while len(out) < m and j >= 0:
            row = [c for c in (R.apply(pr, base[j]) for pr in parsed) if c and 8 <= len(c) <= 63]
            out = row + out
            j -= 1
        return out[-m:]
    w.load, w.check = load, check
    w.cpu_line, w.cpu_keys = (lines[w.plants[0][0]], cpu_keys) if w.plants else (None, None)
    w.cpu_what = "rule candidates (word-major, 8..63) of one ESSID's line"
    w.algo_bytes_per_pmk = 32 + 40 * len(lines) / w.groups
    w.plant_batch = (w.plants[0][1] // w.nrules) // w.words_per_step if w.plants else 0
    return w


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK = LOCAL_RANK = r,
    WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free port for the gloo control plane), one per GPU, as
    torch.distributed.run would.  This parent never touches a GPU.  It relays rank 0's stdout (the JSON line),
    stops the other ranks as soon as one fails, and fails unless all N ranks exited 0 and the line reports
    n_gpus == N.  Returns the exit code."""
    import signal
    import socket
    import subprocess
    import threading
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]

    def die_with_parent():  # a rank gets SIGTERM if this parent is killed (e.g. by a time limit): no orphan ranks
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True, preexec_fn=die_with_parent))
    lines = []

    def relay():
        for raw in procs[0].stdout:
            lines.append(raw.decode(errors="replace").rstrip("\n"))
    reader = threading.Thread(target=relay, daemon=True)
    reader.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            for p, c in zip(procs, codes):
                if c is None:  # our own child's process group (start_new_session), never a pattern
                    os.killpg(p.pid, signal.SIGTERM)
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
                    p.wait()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.2)
    reader.join(timeout=30)
    result = None
    for ln in lines:
        try:
            obj = json.loads(ln)
        except ValueError:
            print(ln, file=sys.stderr, flush=True)
            continue
        result = obj
    if rc != 0:
        print(f"bench.py: a rank failed with exit code {rc}", file=sys.stderr)
        return rc if rc > 0 else 1
    if result is None or result.get("n_gpus") != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but rank 0 reported "
              f"{None if result is None else result.get('n_gpus')} ranks", file=sys.stderr)
        return 4
    emit(result)
    return 0


def check_device(local: int, rank: int) -> int:
    """This rank's device index.  LOCAL_RANK when every GPU is visible; 0 when the launcher gave the rank its own GPU
    (HIP/ROCR/CUDA_VISIBLE_DEVICES naming exactly one); otherwise fail loudly (a node with fewer GPUs than --gpus)."""
    import dwpa_amd
    n = dwpa_amd.device_count()
    if local < n:
        return local
    vis = next((os.environ[v] for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
                if os.environ.get(v)), None)
    if n == 1 and vis is not None and len(vis.split(",")) == 1:
        return 0
    raise SystemExit(f"bench.py rank {rank}: device {local} not visible ({n} gfx950 devices); "
                     "DWPA_BENCH_ONE_DEVICE=1 rehearses N ranks on one GPU")


def main():
    args = parse()
    if args.workload == "c2files":  # the client's node mode: one process over N devices, never rank processes
        os.environ.setdefault("DWPA_DICT_CACHE_MB", "0")
    elif os.environ.get("WORLD_SIZE") is None and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args))
    quiet_stdout()
    if args.workload == "c1cold":  # before anything touches the GPU: the parent never does
        return {"parent": main_cold, "worker": cold_worker, "context": cold_context}[args.cold_role](args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world and not (args.workload == "c2files" and world == 1):
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.scaling == "strong" and args.workload != "c4":
        sys.exit("bench.py: --scaling strong is defined for --workload c4 (the numeric keyspace)")
    if args.peak_costs:
        global C_MIN_CYCLES, PEAK_COMPRESSIONS
        from tools.cmin import from_costs
        C_MIN_CYCLES = from_costs(args.peak_costs)["c_min_model"]
        PEAK_COMPRESSIONS = SIMDS * CLOCK_HZ * 64 / C_MIN_CYCLES
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DWPA_BENCH_ONE_DEVICE") == "1":
        local = 0  # rehearsal of the N>1 control path with every rank on one GPU (not a scaling measurement)
    if args.dry_run:
        return main_dry(args, world, rank)
    local = check_device(local, rank)
    if args.workload in ("c1", "c5"):
        return main_ffi(args, world, rank, local)
    if args.workload == "c2files":
        return main_files(args, world, rank, local)
    if args.workload == "c3files":
        return main_files_rules(args, world, rank, local)
    if args.workload == "c1lat":
        return main_latency(args, world, rank, local)
    if args.workload == "expand":
        return main_expand(args, world, rank, local)
    if args.scaling == "strong":
        return main_strong(args, world, rank, local)
    if world > 1:
        # control plane only (barrier, max-over-ranks time, sum of PMKs): the data path shards the keyspace and
        # never exchanges data, so there is no RCCL collective on the GPU.
        dist.init_process_group("gloo")

    import dwpa_amd
    from tests import synth as S
    from dwpa_amd.device import Dictionary, Event, Stream
    from dwpa_amd.shard import reduce_timing, weak_units

    build = {"c2": build_c2, "c3": build_c3, "c4": build_c4}[args.workload]
    w = build(args, local, S, dwpa_amd.Scan, Dictionary, shard=rank)
    # pipeline slot k: its own scan working set (batch buffers, hit buffer) and stream; batch s goes to slot
    # s % P, so batch s+1's PBKDF2 is queued while batch s's verify still runs
    P = len(w.scans)
    streams = [Stream(local) for _ in range(P)]

    def sync_all():
        for st in streams:
            st.synchronize()

    def step(i, k, ev=None):
        sc, stream = w.scans[k], streams[k]
        hs = stream.handle
        cnt = w.load(i, hs, sc)
        if w.groups > 1 or args.scan_run:
            # all ESSID groups per launch; the events bracket PBKDF2 + verify (conservative for the roofline)
            if ev is not None:
                ev[0].record(stream)
            sc.run(hs)
            if ev is not None:
                ev[1].record(stream)
            return cnt
        if ev is not None:
            ev[0].record(stream)
        sc.pbkdf2(0, hs)
        if ev is not None:
            ev[1].record(stream)
        sc.verify(0, hs)
        return cnt

    # the batch order is rotated so that the first timed step scans the planted batch: every timed window, however
    # short, holds at least one scan whose hits verify_timed_hits checks against the plant
    rot = (getattr(w, "plant_batch", 0) - args.warmup) % w.nbatches
    for s, (_, b) in enumerate(weak_units(rank, 0, args.warmup, w.nbatches, rot)):
        step(b, s % P)
    sync_all()
    for k in range(P):
        w.scans[k].hits(streams[k].handle)  # drop warmup hits

    kev = [(Event(local), Event(local)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    done = 0
    counts = []
    for s, (_, b) in enumerate(weak_units(rank, args.warmup, args.steps, w.nbatches, rot)):
        counts.append(step(b, s % P, kev[s]))
        done += counts[-1]
    sync_all()
    elapsed_local = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms = [a.elapsed_ms(b) for a, b in kev]
    kernel_ms = sum(kms) / len(kms)

    if world > 1:
        elapsed, total = reduce_timing(dist, elapsed, done)
    else:
        total = float(done)

    # correctness (untimed): the hits of the timed steps, each re-derived, and every timed scan of the planted batch
    # reporting the plant; then one more scan of the planted batch, which must report it too
    timed_hits = []
    for k in range(P):
        timed_hits += w.scans[k].hits(streams[k].handle)
    timed_ok, hits_check = verify_timed_hits(w, timed_hits,
                                             [b for _, b in weak_units(rank, args.warmup, args.steps, w.nbatches,
                                                                       rot)])
    step(w.plant_batch, 0)
    plant_ok = bool(w.check(w.scans[0].hits(streams[0].handle)))
    hits_check["plant_rescan_ok"] = plant_ok
    verified = timed_ok and plant_ok
    if world > 1:  # every rank's own planted PSK must come back (each rank scans its own shard)
        from dwpa_amd.shard import all_ranks
        verified = all_ranks(dist, verified)

    per_launch = list(counts) if w.groups > 1 else [c / w.groups for c in counts]
    pmk_per_launch = sum(per_launch) / len(per_launch)
    kernel_pmk_s = sum(per_launch) / (sum(kms) * 1e-3)
    traffic_pmk = TRAFFIC_BYTES_PER_PMK.get(args.workload)
    if rank == 0:
        value = total / elapsed
        cpu = None
        if not args.no_cpu_baseline and world == 1 and w.cpu_keys:
            cpu = cpu_baseline(w.cpu_line, w.cpu_keys, args.cpu_seconds, w.cpu_what)
        result = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "PMK/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": dict({"workload": w.description, "batch_per_step": w.B,
                            "parallelism": f"keyspace shards x{world}, no collective on the data path"}, **w.extra),
            "roofline": roofline_block("k_pbkdf2_gfx950_q" if w.groups == 1 else
                                       "k_pbkdf2_mg + k_verify (per dwpa_scan_run)", kernel_pmk_s, pmk_per_launch,
                                       kernel_ms, traffic_pmk, TRAFFIC_SOURCE.get(args.workload),
                                       w.algo_bytes_per_pmk, args.peak_costs),
            "cpu_baseline": cpu,
            "hits_verified": verified,
            "hits_check": hits_check,
            "pbkdf2_kernel": "k_pbkdf2 (hipcc schedule)" if os.environ.get("DWPA_PBKDF2_PLAIN", "0") not in ("", "0")
                             else "k_pbkdf2_gfx950 (gfx950 VALU issue pass)",
            "rank0_local_s": round(elapsed_local, 4),
            "pipeline": P,
        }
        emit(result)
    for sc in w.scans:
        sc.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not verified:
        sys.exit(3)


def main_dry(args, world, rank):
    """--dry-run: the N-rank control path with no GPU.  Every rank builds the shard schedule its workload would
    scan (weak: (its own shard r, batch) of every timed step; strong c4: its contiguous keyspace
    range), then the gloo barrier and the max/sum reductions run as in a measured run; rank 0 prints the coverage
    of every rank.  tests/test_bench_spawn.py checks N ranks and disjoint coverage through `--gpus N`."""
    if args.workload == "c2files":
        return dry_node(args)
    import torch.distributed as dist
    from dwpa_amd.shard import reduce_timing, strong_batches, weak_units
    if os.environ.get("DWPA_TEST_RANK_SLEEP"):  # tests/test_bench_spawn.py: keep the ranks alive while it kills the parent
        time.sleep(float(os.environ["DWPA_TEST_RANK_SLEEP"]))
    if world > 1:
        dist.init_process_group("gloo")
    B = (args.batch + 63) & ~63
    if args.scaling == "strong":
        mine = [list(x) for x in strong_batches(10 ** 8, rank, world, B)]
        units = sum(c for _, c in mine)
    else:
        n = 10 ** 8 if args.workload == "c4" else args.dict_words
        nb = (n + B - 1) // B
        mine = [list(u) for u in weak_units(rank, args.warmup, args.steps, nb)]
        units = len(mine) * B
    gathered = [mine]
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        dist.barrier()
        _, total = reduce_timing(dist, 0.0, units)
    else:
        total = float(units)
    if rank == 0:
        emit({"metric": METRIC, "value": None, "unit": "PMK/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "scaling": args.scaling,
                          "config": {"workload": args.workload, "batch_per_step": B},
                          "units_all_ranks": total, "coverage": gathered, "pid": os.getpid()})
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def dry_node(args):
    """--workload c2files --dry-run: the node mode's work distribution with no GPU.  One process (no ranks); a scaled
    C2 gzip dictionary (at most 2M words) goes through the library's own reader and item queue (dict_reader.hpp:
    ChunkSource + ItemQueue, in tools/bin/item_queue_check) to N x DWPA_CRACK_SHARDS_PER_DEVICE workers that hold
    each item for a time proportional to its size, with crack.cpp's item sizes for a batch scaled to the dictionary.
    Reports every worker's words and items and whether every word went out exactly once."""
    import copy
    import subprocess
    import tempfile
    ngpu = args.gpus or 1
    spd = int(os.environ.get("DWPA_CRACK_SHARDS_PER_DEVICE", "1") or 1)
    W = ngpu * spd
    a = copy.copy(args)
    a.dict_words = min(args.dict_words, 2_000_000)
    tmp = tempfile.mkdtemp(prefix="dwpa_node_dry_")
    path, _, _, _, _ = _c2_gz_dictionary(a, tmp)
    B = max(64, a.dict_words // (16 * W))  # batch scaled so every worker takes several items
    first = max(1, B // 16)
    most = min(16 * B, max(first, 2 * B)) if W > 1 else 16 * B  # crack.cpp: items of at most 2 batches when W > 1
    tool = os.path.join(ROOT, "tools", "bin", "item_queue_check")
    r = subprocess.run([tool, str(W), str(first), str(most), "200000", path], capture_output=True, text=True,
                       timeout=300)
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    if r.returncode != 0:
        raise SystemExit(f"item_queue_check failed: {r.stderr[-1000:]}")
    q = json.loads(r.stdout)
    emit({"metric": METRIC, "value": None, "unit": "PMK/s", "n_gpus": ngpu, "steps": args.steps,
          "warmup": args.warmup, "dry_run": True, "scaling": "weak",
          "config": {"workload": "c2files", "device_mask": (1 << ngpu) - 1, "workers": W,
                     "shard_workers_per_device": spd, "dict_words": a.dict_words, "batch_scaled": B,
                     "items_first_most": [first, most], "parallelism": f"one process, {ngpu} device(s) x {spd} worker(s)"},
          "words_total": q["words_total"], "every_word_once": q["unique"] and q["words_total"] == a.dict_words,
          "workers": q["workers"], "pid": os.getpid()})


def main_strong(args, world, rank, local):
    """C4 strong scaling: a step exhausts the 10^8 keyspace 00000000..99999999 once; rank g
    of G scans [g*10^8/G, (g+1)*10^8/G) in equal batches (generated in-kernel, PBKDF2 + PMKID verify).  Time per
    step = max over ranks (gloo), value = node PMK/s; with --t1-s the line carries S(G) = T1 / TG.  The planted
    PSK 73019412 must be reported by the rank whose range holds it, in every timed pass."""
    import torch.distributed as dist
    import dwpa_amd
    from tests import synth as S
    from dwpa_amd.device import Event, Stream
    from dwpa_amd.shard import contiguous_shard, reduce_timing, strong_batches

    if world > 1:
        dist.init_process_group("gloo")
    w = build_c4(args, local, S, dwpa_amd.Scan, None)
    sc = w.scans[0]
    stream = Stream(local)
    hs = stream.handle
    n = 10 ** 8
    sched = strong_batches(n, rank, world, w.B)
    lo, hi = contiguous_shard(n, rank, world)

    def scan(first, cnt, ev=None):
        sc.load_numeric(first, cnt, 8, hs)
        if ev is not None:
            ev[0].record(stream)
        sc.pbkdf2(0, hs)
        if ev is not None:
            ev[1].record(stream)
        sc.verify(0, hs)

    for _ in range(args.warmup):
        scan(*sched[0])
    stream.synchronize()
    sc.hits(hs)
    kev = [[(Event(local), Event(local)) for _ in sched] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    stream.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        for j, (first, cnt) in enumerate(sched):
            scan(first, cnt, kev[s][j])
    stream.synchronize()
    elapsed_local = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    done = float(sum(c for _, c in sched) * args.steps)
    hits = sc.hits(hs)
    want = args.steps if lo <= w.plant < hi else 0
    good = sum(1 for h in hits if h["cand"] == w.plant and h["pmk"] == S.pmk(b"%08d" % w.plant, w.essid))
    ok_local = good == want and len(hits) == want
    kms = [a.elapsed_ms(b) for step in kev for a, b in step]
    kernel_ms = sum(kms) / len(kms)
    kernel_pmk_s = sum(c for _, c in sched) * args.steps / (sum(kms) * 1e-3)
    if world > 1:
        from dwpa_amd.shard import all_ranks
        elapsed, total = reduce_timing(dist, elapsed, done)
        verified = all_ranks(dist, ok_local)
        shards = [None] * world
        dist.all_gather_object(shards, [lo, hi, len(sched), round(elapsed_local, 4)])
    else:
        total, verified, shards = done, ok_local, [[lo, hi, len(sched), round(elapsed_local, 4)]]
    if rank == 0:
        t_exhaust = elapsed / args.steps
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(w.cpu_line, w.cpu_keys, args.cpu_seconds, w.cpu_what)
        pmk_per_launch = sum(c for _, c in sched) / len(sched)
        traffic_pmk = TRAFFIC_BYTES_PER_PMK["c4"]
        emit({
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "PMK/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "C4 strong scaling: the 8-digit keyspace 00000000..99999999 (10^8, generated on "
                                   "the GPU) exhausted once per step, rank g of G scanning [g*10^8/G, (g+1)*10^8/G); "
                                   "one ESSID, PMKID line", "keyspace": n, "batch_max": w.B,
                       "parallelism": f"contiguous keyspace shards x{world}, no collective on the data path"},
            "t_exhaust_s": round(t_exhaust, 4),
            "speedup": round(args.t1_s / t_exhaust, 4) if args.t1_s else None,
            "speedup_basis": f"S(G) = T1 / TG with T1 = {args.t1_s} s (--t1-s)" if args.t1_s else None,
            "shards": shards,
            "roofline": roofline_block("k_pbkdf2_gfx950_q (rank 0)", kernel_pmk_s, pmk_per_launch, kernel_ms,
                                       traffic_pmk, TRAFFIC_SOURCE["c4"], ALGO_BYTES_PER_PMK, args.peak_costs),
            "cpu_baseline": cpu, "hits_verified": verified,
            "hits_checked": "the planted PSK 73019412 with its PMK, once per timed pass, on the rank holding it; "
                            "no other hit on any rank"})
    sc.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not verified:
        sys.exit(3)


def main_ffi(args, world, rank, local):
    """C1 / C5 legs: the server-side FFI call (dwpa_check_m22000 / dwpa_check_batch) on host buffers, as PHP
    makes it (common.php:157, :902).  A step = one call over the whole config: C1 = 10k keys x 1 PMKID line,
    C5 = 1,010 mixed jobs x 202 keys at nc=128 (261 NC attempts).  The rate includes parsing, the key upload
    and the result download (PCIe-inclusive, unlike the HBM-resident C2 line).  N>1 runs N replicas."""
    import ctypes
    import torch.distributed as dist
    import dwpa_amd
    from dwpa_amd import _lib as L
    from tests import synth as S
    from dwpa_amd.shard import reduce_timing

    if world > 1:
        dist.init_process_group("gloo")
    cfg = L.Config(ctypes.sizeof(L.Config), 1 << local, 0, 0)
    L.check(L.load().dwpa_init(ctypes.byref(cfg)), "init")
    if args.workload == "c1":
        line, keys, psk = S.c1_workload()
        jobs = [(line, keys, False, 128)]
        desc = "C1: 10,000 PSKs (1 % $HEX[]) vs one PMKID line, dwpa_check_m22000 per step (FFI, host buffers)"
    else:
        jobs, plants = S.c5_plan()
        desc = ("C5: 250 PMKID + 250 x keyver 1/2/3 EAPOL lines (NC offsets 0..+-8, LE/BE) + 10 zero-PMK jobs, "
                "202 keys per job, nc=128 (261 attempts), dwpa_check_batch per step (FFI, host buffers)")
    import threading
    callers = max(1, args.callers)
    batches = [dwpa_amd.BatchJobs(jobs) for _ in range(callers)]
    batch = batches[0]
    go = threading.Barrier(callers)  # the main thread is caller 0
    errors = []

    def caller(b):  # warmup, wait for the start, then args.steps calls back to back (ctypes drops the GIL)
        try:
            for _ in range(args.warmup):
                b.run()
            go.wait()
            for _ in range(args.steps):
                b.run()
        except Exception as e:  # noqa: BLE001 -- reported below, the run fails
            errors.append(e)
            go.abort()

    threads = [threading.Thread(target=caller, args=(b,)) for b in batches[1:]]
    for t in threads:
        t.start()
    for _ in range(args.warmup):
        batch.run()
    if world > 1:
        dist.barrier()
    if args.start_at:
        time.sleep(max(0.0, args.start_at - time.time()))
    go.wait()
    t0, u0 = time.perf_counter(), time.time()
    for _ in range(args.steps):
        batch.run()
    for t in threads:
        t.join()
    elapsed = time.perf_counter() - t0
    window = [round(u0, 4), round(u0 + elapsed, 4)]
    if errors:
        raise errors[0]
    call_stats = dwpa_amd.check_stats()  # the main thread's last timed call (dwpa_check_last_stats)
    keys_all = float(batch.nkeys * args.steps * callers)
    if world > 1:
        dist.barrier()
        elapsed, total = reduce_timing(dist, time.perf_counter() - t0, keys_all)
    else:
        total = keys_all
    got = batch.results()
    same = all(b.results() == got for b in batches[1:])
    mismatches = None
    if args.workload == "c1":
        verified = bool(got[0]) and got[0][0] == psk and got[0][3] == S.pmk(psk, bytes.fromhex(line.split(b"*")[5].decode()))
    else:
        # every job exactly: the planted key's [PSK, NC, endian, PMK] tuple re-derived by the oracle from that key
        # alone, or False where no key was planted (tests/test_gpu_configs.py adds the first-key prefix checks)
        from concurrent.futures import ThreadPoolExecutor
        from oracle import oracle as O

        def expected(i):
            line, keys, pmk, nc = jobs[i]
            p = plants[i]
            return False if p is None else O.c_check_key_m22000(line, [keys[p]], pmk if p == 0 else False, nc)
        with ThreadPoolExecutor(host_cpu()["threads_all"]) as ex:
            exp = list(ex.map(expected, range(len(jobs))))
        mismatches = sum(1 for g, e in zip(got, exp) if g != e)
        verified = mismatches == 0 and sum(1 for e in exp if e) >= 0.85 * len(jobs)
    verified = verified and same
    if world > 1:  # every replica's results must check
        from dwpa_amd.shard import all_ranks
        verified = all_ranks(dist, verified)
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline_jobs(jobs, args.cpu_seconds)
        emit({
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "PMK/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": desc, "jobs": len(jobs), "keys_per_step": batch.nkeys * callers,
                       "callers": callers, "parallelism": f"replicas x{world}"},
            "roofline": None, "cpu_baseline": cpu, "hits_verified": verified,
            "hits": sum(1 for g in got if g),
            "mismatches": mismatches if args.workload == "c5" else None,
            "window_unix": window,
            "last_call": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in call_stats.items()},
            "hits_checked": "every job's result against its planted key's [PSK, NC, endian, PMK] (re-derived by the "
                            "CPU oracle) or False" if args.workload == "c5" else "the planted PSK and its PMK"})
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not verified:
        sys.exit(3)


def main_latency(args, world, rank, local):
    """Server call latency.  put_work checks each submitted PSK with its own
    check_key_m22000($struct, [$psk]) call, default nc=128 (common.php:902), for at most ~202 submissions per
    request (:937).  Measured here per FFI call: 1, 16 and 202 keys against one PMKID line and one EAPOL keyver-2
    line at nc=128 (dwpa_check_m22000, the true key last), and the whole 202-submission request as one
    dwpa_check_batch of 202 one-key jobs -- each beside the same call on one CPU core (the OpenSSL restatement,
    one PHP request).  A call that derives k PMKs on the GPU cannot finish before one PBKDF2
    chain does (8,194 dependent SHA-1 compressions per lane, a lone wave on its SIMD), so the library runs small
    calls on its host backend: each row reports the library's default routing (lib_ms,
    lib_backend) and the GPU alone (gpu_ms)."""
    import random
    import statistics
    import dwpa_amd
    from dwpa_amd import _lib as L
    from dwpa_amd import m22000 as M
    from tests import synth as S
    from oracle import oracle as O
    rng = random.Random(7)
    essid, ap, sta, an, sn = S.random_net(rng, essid_len=10)
    rows = []
    reps = max(3, args.steps)

    def timed(fn, n):
        fn()  # warm (first call of a shape: staging buffers)
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            r = fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e3, r

    # Each server-call row twice: as the library routes it by default (small calls on its host backend, DESIGN.md
    # 1.1; which backend answered is read back from dwpa_check_last_stats) and with the host backend off (the GPU).
    BACKENDS = {L.DWPA_BACKEND_DEVICE: "device", L.DWPA_BACKEND_HOST_SMALL: "host",
                L.DWPA_BACKEND_HOST_FALLBACK: "host_fallback"}

    def routed(fn, n):
        M.init()
        ms, r = timed(fn, n)
        return ms, r, M.check_stats()["backend"]

    def device_only(fn, n):
        M.init(host_max_pmks=-1)
        try:
            ms, r = timed(fn, n)
            assert M.check_stats()["backend"] == L.DWPA_BACKEND_DEVICE
        finally:
            M.init()
        return ms, r

    for kind in ("pmkid", "eapol-kv2"):
        for k in (1, 16, 202):
            keys = [S.fast_psk(rng) for _ in range(k - 1)]
            psk = S.fast_psk(rng)
            keys.append(psk)
            line = (S.pmkid_line(psk, essid, ap, sta) if kind == "pmkid" else
                    S.eapol_line(psk, essid, ap, sta, an, sn, 2, -5, "BE", rng=rng))
            lib_ms, got, backend = routed(lambda: dwpa_amd.check_key_m22000(line, keys), reps)
            gpu_ms, got_dev = device_only(lambda: dwpa_amd.check_key_m22000(line, keys), reps)
            cpu_ms, exp = timed(lambda: O.c_check_key_m22000(line, keys), max(1, min(reps, 3 if k > 16 else reps)))
            rows.append({"call": f"check_key_m22000, {kind}, {k} key(s), nc=128", "keys": k,
                         "lib_ms_per_call": round(lib_ms, 3), "lib_backend": BACKENDS[backend],
                         "gpu_ms_per_call": round(gpu_ms, 3), "cpu_1core_ms_per_call": round(cpu_ms, 3),
                         "lib_over_cpu": round(lib_ms / cpu_ms, 3), "gpu_over_cpu": round(gpu_ms / cpu_ms, 3),
                         "same_result": got == exp and got_dev == exp})
    # the whole put_work request: 202 submitted PSKs, each against its net (one key per job), one batch call
    jobs = []
    for i in range(202):
        e2, a2, s2, an2, sn2 = S.random_net(rng)
        psk = S.fast_psk(rng)
        line = (S.pmkid_line(psk, e2, a2, s2) if i % 2 else S.eapol_line(psk, e2, a2, s2, an2, sn2, 2, i % 9 - 4, "LE",
                                                                         rng=rng))
        jobs.append((line, [psk if i % 3 else S.fast_psk(rng)], False, 128))
    batch = dwpa_amd.BatchJobs(jobs)
    lib_ms, _, backend = routed(lambda: batch.run(), reps)
    got_lib = batch.results()
    gpu_ms, _ = device_only(lambda: batch.run(), reps)
    got = batch.results()
    t0 = time.perf_counter()
    exp = [O.c_check_key_m22000(*j) for j in jobs]
    cpu_ms = (time.perf_counter() - t0) * 1e3
    rows.append({"call": "put_work request: 202 one-key jobs (PMKID + EAPOL keyver 2, nc=128) in one "
                         "dwpa_check_batch vs 202 check_key_m22000 calls", "keys": 202,
                 "lib_ms_per_call": round(lib_ms, 3), "lib_backend": BACKENDS[backend],
                 "gpu_ms_per_call": round(gpu_ms, 3), "cpu_1core_ms_per_call": round(cpu_ms, 3),
                 "lib_over_cpu": round(lib_ms / cpu_ms, 3), "gpu_over_cpu": round(gpu_ms / cpu_ms, 3),
                 "same_result": got == exp and got_lib == exp})
    # Caller-PMK checks (no PBKDF2: pure verify work), each once per sibling net of a crack:
    #   zero-PMK     check_key_m22000($struct, [''], $zpmk)                        common.php:592 (default nc=128)
    #   PMK reuse    check_key_m22000($struct, [$pass], $pmk, (|nc| << 1) + 1)      common.php:606 (nc up to 131)
    #   propagation  check_key_m22000($struct, [''], $pmk, |nc| * 2 + 128)          common.php:919 (nc up to 258)
    # A sibling is usually not the same network, so the miss (all 1 + 4 * ((nc >> 1) + 1) attempts run) is the
    # common case; the hit rows plant the correction near the middle of the window.
    zpmk = bytes(32)
    for site, nc, key, use_true, hit in (("zero-PMK (common.php:592)", 128, b"", False, False),
                                         ("PMK reuse (common.php:606)", 131, None, True, True),
                                         ("PMK propagation, hit (common.php:919)", 258, b"", True, True),
                                         ("PMK propagation, miss (common.php:919)", 258, b"", False, False)):
        for kind in ("pmkid", "eapol-kv2", "eapol-kv3"):
            psk = S.fast_psk(rng)
            e2, a2, s2, an2, sn2 = S.random_net(rng, essid_len=10)
            kv = {"eapol-kv2": 2, "eapol-kv3": 3}.get(kind)
            line = (S.pmkid_line(psk, e2, a2, s2) if kv is None else
                    S.eapol_line(psk, e2, a2, s2, an2, sn2, kv, 37 if hit else 0, "LE", rng=rng))
            pmk = S.pmk(psk, e2) if use_true else (zpmk if site.startswith("zero") else S.pmk(S.fast_psk(rng), e2))
            keys = [psk if key is None else key]
            lib_ms, got, backend = routed(lambda: dwpa_amd.check_key_m22000(line, keys, pmk, nc), reps)
            gpu_ms, got_dev = device_only(lambda: dwpa_amd.check_key_m22000(line, keys, pmk, nc), reps)
            cpu_ms, exp = timed(lambda: O.c_check_key_m22000(line, keys, pmk, nc), reps)
            rows.append({"call": f"{site}, {kind}, caller PMK, nc={nc}, {'hit' if hit else 'miss'}", "keys": 1,
                         "caller_pmk": True, "nc": nc, "hit": bool(got),
                         "lib_ms_per_call": round(lib_ms, 3), "lib_backend": BACKENDS[backend],
                         "gpu_ms_per_call": round(gpu_ms, 3), "cpu_1core_ms_per_call": round(cpu_ms, 3),
                         "lib_over_cpu": round(lib_ms / cpu_ms, 3), "gpu_over_cpu": round(gpu_ms / cpu_ms, 3),
                         "same_result": got == exp and got_dev == exp and bool(got) == hit})
    # one crack's propagation over 16 sibling nets as a single dwpa_check_batch (the batched snippet of INTEGRATION.md)
    jobs = []
    for i in range(16):
        psk = S.fast_psk(rng)
        e2, a2, s2, an2, sn2 = S.random_net(rng, essid_len=10)
        line = (S.pmkid_line(psk, e2, a2, s2) if i % 4 == 0 else
                S.eapol_line(psk, e2, a2, s2, an2, sn2, 2 + (i % 2), (i % 5) - 2, "BE", rng=rng))
        jobs.append((line, [b""], S.pmk(psk if i % 3 else S.fast_psk(rng), e2), 258))
    batch = dwpa_amd.BatchJobs(jobs)
    lib_ms, _, backend = routed(lambda: batch.run(), reps)
    got_lib = batch.results()
    gpu_ms, _ = device_only(lambda: batch.run(), reps)
    got = batch.results()
    t0 = time.perf_counter()
    exp = [O.c_check_key_m22000(*j) for j in jobs]
    cpu_ms = (time.perf_counter() - t0) * 1e3
    rows.append({"call": "PMK propagation to 16 sibling nets (PMKID + EAPOL keyver 2/3, nc=258) in one "
                         "dwpa_check_batch vs 16 check_key_m22000 calls", "keys": 16, "caller_pmk": True, "nc": 258,
                 "lib_ms_per_call": round(lib_ms, 3), "lib_backend": BACKENDS[backend],
                 "gpu_ms_per_call": round(gpu_ms, 3), "cpu_1core_ms_per_call": round(cpu_ms, 3),
                 "lib_over_cpu": round(lib_ms / cpu_ms, 3), "gpu_over_cpu": round(gpu_ms / cpu_ms, 3),
                 "same_result": got == exp and got_lib == exp})
    ok = all(r["same_result"] for r in rows)
    if rank == 0:
        emit({"metric": "ms per server check call (latency), m22000", "value": rows[0]["lib_ms_per_call"],
                          "unit": "ms", "n_gpus": world, "steps": reps, "warmup": 1, "higher_is_better": False,
                          "dtype": "u32", "data": "synthetic",
                          "config": {"workload": "C1 latency: FFI calls of 1/16/202 keys (put_work, common.php:902,"
                                                 "937) and caller-PMK checks (common.php:592,606,919) beside one "
                                                 "CPU core; value = one key, PMKID, as the library routes it",
                                     "parallelism": "none"},
                          "rows": rows, "cpu_model": host_cpu()["cpu_model"], "hits_verified": ok})
    if rank == 0 and not ok:
        sys.exit(3)


def _proc_status(key):
    try:
        with open("/proc/self/status") as f:
            return next((int(l.split()[1]) * 1024 for l in f if l.startswith(key + ":")), None)
    except OSError:
        return None


def _rss():
    """Resident memory in MiB: total, anonymous, file-backed, shared (the HIP runtime maps device files)."""
    return {k: round((_proc_status(k) or 0) / (1 << 20), 1) for k in ("VmRSS", "RssAnon", "RssFile", "RssShmem")}


def _hip_runtime():
    """The HIP runtime library this process already maps (the one libdwpa22000.so loaded), else ROCm's."""
    import ctypes
    try:
        with open("/proc/self/maps") as f:
            path = next((l.split()[-1] for l in f if "libamdhip64.so" in l), None)
    except OSError:
        path = None
    return ctypes.CDLL(path or os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libamdhip64.so"))


def _hip_mem_used(device=0):
    """Device-wide bytes in use (hipMemGetInfo: total - free) through the HIP runtime already in this process."""
    import ctypes
    hip = _hip_runtime()
    free, total = ctypes.c_size_t(0), ctypes.c_size_t(0)
    hip.hipSetDevice(device)
    if hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) != 0:
        return None
    return total.value - free.value


def cold_context(args):
    """c1cold child: a bare HIP context (hipInit + context creation, no library) and the device memory it holds --
    what every process that touches the GPU pays before any library buffer."""
    import ctypes
    t0 = time.perf_counter()
    hip = _hip_runtime()
    assert hip.hipInit(0) == 0 and hip.hipSetDevice(0) == 0
    assert hip.hipFree(None) == 0  # creates the context
    t1 = time.perf_counter()
    emit({"role": "context", "ms_runtime_and_context": round((t1 - t0) * 1e3, 2), "device_used_bytes": _hip_mem_used(),
          "rss_bytes": _proc_status("VmRSS"), "rss_mib": _rss(), "threads": len(os.listdir("/proc/self/task"))})


def cold_worker(args):
    """c1cold child: one PHP-FPM worker's life in a fresh process (common.php:849 -> :902 per request): load the
    library, make the first check call (HIP runtime + context, code-object load, the call context's buffers), the
    second, then args.steps calls alternating one key against a PMKID line (put_work, :902) and 202 keys against an
    EAPOL keyver-2 line at nc=128 (rkg.php:147 / a whole put_work candidate list).  Every result is checked."""
    import random
    from tests import synth as S
    rng = random.Random(1000 + args.cold_id)
    essid, ap, sta, an, sn = S.random_net(rng, essid_len=10)
    psk = S.fast_psk(rng)
    pmk = S.pmk(psk, essid)
    one = (S.pmkid_line(psk, essid, ap, sta), [psk])
    many = (S.eapol_line(psk, essid, ap, sta, an, sn, 2, -5, "BE", rng=rng), [S.fast_psk(rng) for _ in range(201)] + [psk])
    exp_one, exp_many = [psk, None, None, pmk], [psk, -5, "BE", pmk]
    t0 = time.perf_counter()
    import dwpa_amd
    from dwpa_amd import m22000 as M
    dwpa_amd.load()
    t_load = time.perf_counter() - t0
    rss = {"loaded": _rss()}
    if args.start_at:
        time.sleep(max(0.0, args.start_at - time.time()))
    t0 = time.perf_counter()
    if args.cold_warmup:
        ndev = dwpa_amd.device_count()  # the HIP runtime's initialisation, split out of the first call
    else:
        M.init(allow_cpu_fallback=1)  # what the PHP wrapper's ffi() does: the device is probed when a call needs it
        ndev = None
    t_init = time.perf_counter() - t0
    rss["runtime_init"] = _rss()
    calls, errors = [], []

    def call(kind):
        line, keys = one if kind == "one" else many
        t = time.perf_counter()
        backend = None
        try:
            r = dwpa_amd.check_key_m22000(line, keys)
            ok = r == (exp_one if kind == "one" else exp_many)
            backend = M.check_stats()["backend"]
        except Exception as e:  # noqa: BLE001 -- an allocation or device failure is what K workers may hit
            errors.append(repr(e)[:200])
            ok = False
        calls.append({"kind": kind, "ms": round((time.perf_counter() - t) * 1e3, 3), "ok": ok, "backend": backend})
    call("one")  # first call of the worker
    rss["first_call"] = _rss()
    call("one")  # second
    for i in range(args.steps):
        call("many" if i % 2 == 0 else "one")
    rss["end"] = _rss()
    res = M.resource_stats()
    emit({"role": "worker", "id": args.cold_id, "ms_import_and_load": round(t_load * 1e3, 2),
          "ms_runtime_init": round(t_init * 1e3, 2), "devices": ndev, "calls": calls,
          "errors": errors, "resources": res, "device_used_bytes": _hip_mem_used(), "rss_mib": rss,
          "rss_bytes": _proc_status("VmRSS"), "locked_bytes": _proc_status("VmLck"),
          "threads": len(os.listdir("/proc/self/task"))})


def main_cold(args):
    """--workload c1cold: the server path as PHP-FPM runs it.  Every PHP request reaches
    check_key_m22000 in a pool worker (put_work.php:14 -> common.php:849 -> :902), and each worker process loads the
    library and creates its own HIP context, call contexts and pinned staging.  This parent never touches the GPU;
    it starts fresh child processes (never a re-exec) and reports:
      * a bare context (runtime init + context, device memory it holds), 3 samples in turn;
      * one worker at a time, 3 samples: library load, the first call (everything a cold worker pays), the second,
        warm one-key and 202-key calls, and the worker's footprint (library device buffers and pinned memory by
        dwpa_resource_stats, device-wide use by hipMemGetInfo, RSS, threads);
      * K concurrent fresh workers (--cold-k, default 4 and 16; 16 also with DWPA_CALLS_PER_DEVICE=1 and
        DWPA_HOST_THREADS=2, the many-worker setting): every call's latency and any failed call."""
    import statistics
    import subprocess

    def spawn(role, i, env_extra=None, start_at=None, steps=None):
        cmd = [sys.executable, os.path.abspath(__file__), "--workload", "c1cold", "--cold-role", role,
               "--cold-id", str(i), "--steps", str(steps if steps is not None else args.steps)]
        if args.cold_warmup:
            cmd.append("--cold-warmup")
        if start_at:
            cmd += ["--start-at", repr(start_at)]
        env = dict(os.environ, **(env_extra or {}))
        return subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, text=True)

    def collect(p, timeout=240):
        out, err = p.communicate(timeout=timeout)
        if p.returncode != 0:
            raise SystemExit(f"c1cold child failed (rc {p.returncode}): {err[-2000:]}")
        return json.loads(out.strip().splitlines()[-1])

    def q(v, f):
        v = sorted(v)
        return round(v[min(len(v) - 1, int(f * len(v)))], 3) if v else None

    ctx = [collect(spawn("context", i)) for i in range(3)]
    seq = [collect(spawn("worker", i, steps=10)) for i in range(3)]
    mib = 1 << 20
    ctx_dev = statistics.median([c["device_used_bytes"] for c in ctx])
    rows = {"context_only": {"ms_runtime_and_context": [c["ms_runtime_and_context"] for c in ctx],
                             "device_used_mib": round(ctx_dev / mib, 1),
                             "rss_mib": round(statistics.median([c["rss_bytes"] for c in ctx]) / mib, 1),
                             "rss_mib_detail": ctx[0]["rss_mib"]},
            "one_worker_at_a_time": []}
    for w in seq:
        c = w["calls"]
        rows["one_worker_at_a_time"].append({
            "ms_import_and_load": w["ms_import_and_load"], "ms_runtime_init": w["ms_runtime_init"],
            "ms_first_call": c[0]["ms"], "ms_second_call": c[1]["ms"], "rss_mib_by_stage": w["rss_mib"],
            "backends": sorted({x["backend"] for x in c if x["backend"] is not None}),
            "devices_probed": w["resources"]["devices"],
            "ms_one_key_warm_median": q([x["ms"] for x in c[2:] if x["kind"] == "one"], 0.5),
            "ms_202_keys_warm_median": q([x["ms"] for x in c[2:] if x["kind"] == "many"], 0.5),
            "library_device_mib": round(w["resources"]["device_bytes"] / mib, 1),
            "library_pinned_host_mib": round(w["resources"]["pinned_host_bytes"] / mib, 1),
            "device_used_mib_whole_device": round(w["device_used_bytes"] / mib, 1),
            "device_used_mib_over_bare_context": round((w["device_used_bytes"] - ctx_dev) / mib, 1),
            "rss_mib": round(w["rss_bytes"] / mib, 1), "threads": w["threads"],
            "host_pool_threads": w["resources"]["host_pool_threads"],
            "call_contexts_used": w["resources"]["call_contexts_used"], "all_ok": all(x["ok"] for x in c)})
    conc = []
    many_env = {"DWPA_CALLS_PER_DEVICE": "1", "DWPA_HOST_THREADS": "2"}
    plans = [(int(k), {}) for k in args.cold_k.split(",") if k.strip()]
    for k, _ in list(plans):
        if k >= 8:  # the many-worker settings: one call context, two host threads, fewer HIP hardware queues
            plans += [(k, many_env), (k, dict(many_env, GPU_MAX_HW_QUEUES="2")),
                      (k, dict(many_env, GPU_MAX_HW_QUEUES="1"))]
    for k, env in plans:
        start = time.time() + 8.0  # every worker imported and loaded before the window opens
        ps = [spawn("worker", 100 + i, env, start_at=start, steps=args.steps) for i in range(k)]
        ws = [collect(p) for p in ps]
        calls = [c for w in ws for c in w["calls"]]
        first = [w["calls"][0]["ms"] for w in ws]
        conc.append({
            "workers": k, "env": env or "defaults",
            "ms_runtime_init_median": q([w["ms_runtime_init"] for w in ws], 0.5),
            "ms_first_call_median": q(first, 0.5), "ms_first_call_max": max(first),
            "ms_one_key_median": q([c["ms"] for w in ws for c in w["calls"][1:] if c["kind"] == "one"], 0.5),
            "ms_one_key_p95": q([c["ms"] for w in ws for c in w["calls"][1:] if c["kind"] == "one"], 0.95),
            "ms_202_keys_median": q([c["ms"] for c in calls if c["kind"] == "many"], 0.5),
            "ms_202_keys_p95": q([c["ms"] for c in calls if c["kind"] == "many"], 0.95),
            "calls": len(calls), "failed_calls": sum(1 for c in calls if not c["ok"]),
            "calls_by_backend": {str(b): sum(1 for c in calls if c["backend"] == b)
                                 for b in sorted({c["backend"] for c in calls if c["backend"] is not None})},
            "errors": sorted({e for w in ws for e in w["errors"]})[:5],
            "library_device_mib_per_worker": round(statistics.median([w["resources"]["device_bytes"] for w in ws]) / mib, 1),
            "library_pinned_host_mib_per_worker": round(
                statistics.median([w["resources"]["pinned_host_bytes"] for w in ws]) / mib, 1),
            "device_used_mib_whole_device_max": round(max(w["device_used_bytes"] for w in ws) / mib, 1),
            "rss_mib_per_worker": round(statistics.median([w["rss_bytes"] for w in ws]) / mib, 1),
            "threads_per_worker": statistics.median([w["threads"] for w in ws])})
    first = [r["ms_first_call"] for r in rows["one_worker_at_a_time"]]
    ok = all(r["all_ok"] for r in rows["one_worker_at_a_time"]) and all(c["failed_calls"] == 0 for c in conc)
    emit({"metric": "ms, first check_key_m22000 call of a fresh PHP-FPM worker process (cold)",
          "value": statistics.median(first), "unit": "ms", "n_gpus": 1, "steps": args.steps, "warmup": 0,
          "higher_is_better": False, "dtype": "u32", "data": "synthetic",
          "config": {"workload": "C1 cold: fresh worker processes (put_work.php:14 -> common.php:849,902), one key "
                                 "vs a PMKID line and 202 keys vs an EAPOL keyver-2 line at nc=128",
                     "worker_start": ("HIP runtime started before the first call (dwpa22000_warmup model)"
                                      if args.cold_warmup else "dwpa_init(allow_cpu_fallback=1), as the PHP "
                                      "wrapper's ffi(): the device is probed by the first call that needs it"),
                     "parallelism": "processes"},
          "rows": rows, "concurrent": conc, "cpu_model": host_cpu()["cpu_model"], "hits_verified": ok})
    if not ok:
        sys.exit(3)


def _c2_gz_dictionary(args, tmp):
    """The C2 dictionary as a gzip file on local disk: args.dict_words words (seed 2; lengths geometric around 10,
    ~30 % under 8 with --short-words), the planted PSK the 99,999,000th word.  Returns (path, psk, PMKs a pass
    derives up to the plant = words inside 8..63, gz bytes, seconds to write it)."""
    import gzip
    import numpy as np
    n = args.dict_words
    plant = min(PLANT_INDEX, n - 1)
    rng = np.random.default_rng(2)
    lens = np.clip(rng.geometric(0.3, n) + (6 if args.short_words else 7), 1, 63).astype(np.int64)
    lens[plant] = max(int(lens[plant]), 8)
    ends = np.cumsum(lens + 1)
    text = rng.integers(0x21, 0x7F, int(ends[-1]), dtype=np.uint8)
    text[ends - 1] = 0x0A
    psk = text[int(ends[plant - 1]) if plant else 0:int(ends[plant]) - 1].tobytes()
    path = os.path.join(tmp, "dict.txt.gz")
    t0 = time.perf_counter()
    with gzip.open(path, "wb", compresslevel=1) as f:
        step = 64 << 20
        for o in range(0, len(text), step):
            f.write(text[o:o + step].tobytes())
    return path, psk, int(np.count_nonzero(lens[:plant + 1] >= 8)), os.path.getsize(path), time.perf_counter() - t0


def _rule_pass_inputs(args, tmp, local):
    """The client's rule pass (help_crack.py:929-933, `-S -r <rules>`): a gzip dictionary of args.rule_words base
    words (6..16 printable bytes, seed 6) and a rules file (dwpa_amd/rulesets.py: the WPA set, 148 rules of
    bestWPA.rule's ops, or the server set), the planted PSK one rule's output of the 1000th-last word.  Candidates
    counted = those inside the 8..63 filter up to the plant: every rule of the WPA set changes a word's length as a
    function of that length only, so the count is sum over lengths of (words of that length) x (rules whose output
    length is in 8..63), from the library's own expansion of one word per length.  Returns a dict."""
    import gzip
    import numpy as np
    import dwpa_amd
    from dwpa_amd.rulesets import server_rules, wpa_rules
    n = max(2000, args.rule_words)
    rules = wpa_rules() if args.rules_set == "wpa" else server_rules()
    rules_text = "\n".join(rules)
    rng = np.random.default_rng(6)
    lens = rng.integers(6, 17, n).astype(np.int64)
    ends = np.cumsum(lens + 1)
    text = rng.integers(0x21, 0x7F, int(ends[-1]), dtype=np.uint8)
    text[text == ord("$")] = ord("%")  # no word starts a $HEX[] form
    text[ends - 1] = 0x0A
    plant_word = n - 1000
    word = text[int(ends[plant_word - 1]):int(ends[plant_word]) - 1].tobytes()
    row = dwpa_amd.rules_expand(rules_text, [word], device=local)[0]
    # the rules this pass loads: all of them (full), or those hashcat's -r loader keeps (no reject / memory function)
    loads = [args.rule_mode == "full" or dwpa_amd.rules_count_ex(r.encode("latin-1"))["loaded_hashcat"] == 1
             for r in rules]
    good = [r for r, c in enumerate(row) if c is not None and 8 <= len(c) <= 63 and loads[r]]
    # wpa: a rule in the middle of the set; server: the last kept one (of the added part: a memory / reject line
    # with --rule-mode full, a byte-arithmetic line under hashcat's loader)
    plant_rule = good[len(good) // 2] if args.rules_set == "wpa" else good[-1]
    reps = [bytes(b"abcdefghijklmnop"[:L]) for L in range(6, 17)]
    per_len = {L: sum(1 for c in r if c is not None and 8 <= len(c) <= 63)
               for L, r in zip(range(6, 17), dwpa_amd.rules_expand(rules_text, reps, device=local))}
    counts = np.bincount(lens[:plant_word + 1], minlength=17)
    dpath, rpath = os.path.join(tmp, "rules_dict.txt.gz"), os.path.join(tmp, "wpa.rule")
    with gzip.open(dpath, "wb", compresslevel=6) as f:
        f.write(text.tobytes())
    with open(rpath, "w") as f:
        f.write(rules_text + "\n")
    return {"dict": dpath, "rules_file": rpath, "rules": rules, "words": n, "psk": row[plant_rule],
            "plant": [plant_word, plant_rule], "cands": int(sum(int(counts[L]) * per_len[L] for L in range(6, 17)))}


def main_files(args, world, rank, local):
    """The client's own multi-GPU mode: ONE process runs dwpa_crack_files over a device mask of
    N GPUs, as help_crack's single hashcat process uses every device (help_crack.py:773) -- one host thread pair per
    device worker, one shared dictionary stream cut into work items by guided self-scheduling, no rank
    processes.  One step = the work unit's two passes (help_crack.py:923-933):
      1. the 100M-word C2 dictionary as a gzip file on local disk (streamed, inflated and $HEX[]-decoded on the
         host, uploaded item by item), one EAPOL keyver-2 line, --nonce-error-corrections=8, up to the planted word;
      2. the rule pass: a --rule-words gzip dictionary x the WPA rule set (rules file, amplified on the GPU).
    value = the PMKs of both passes / their wall time (the node figure); each pass is reported with its words,
    candidates and feed rate, and every device worker with its items, words, candidates, scan time and the time it
    waited for the shared feed.  hits_verified: each pass's outfile holds exactly the planted record.
    --gpus N: the mask covers devices 0..N-1 (n_gpus = N).  Under a launcher (WORLD_SIZE = N) rank 0 runs it and the
    other ranks exit without touching a GPU.  DWPA_CRACK_SHARDS_PER_DEVICE=k runs k workers per device: on a one-GPU
    box, k = 8 rehearses an 8-GPU node's worker count and feed (not its throughput).  The library's in-process
    dictionary cache is off for this leg (DWPA_DICT_CACHE_MB=0 unless set): every pass inflates its gzip file, as a
    client's first pass over a downloaded dictionary does."""
    import random
    import tempfile
    import dwpa_amd
    from dwpa_amd import _lib as L
    from dwpa_amd import m22000 as M
    from tests import synth as S

    ngpu = max(world, args.gpus or 1)
    if rank != 0:
        return
    ndev = dwpa_amd.device_count()
    if ngpu > ndev:
        raise SystemExit(f"bench.py --workload c2files: --gpus {ngpu} but {ndev} gfx950 device(s) visible")
    mask = (1 << ngpu) - 1
    spd = int(os.environ.get("DWPA_CRACK_SHARDS_PER_DEVICE", "1") or 1)
    tmp = tempfile.mkdtemp(prefix="dwpa_node_")
    d1, psk1, pmk1, gz_bytes, gz_s = _c2_gz_dictionary(args, tmp)
    rp = _rule_pass_inputs(args, tmp, local)
    rr = random.Random(1)
    essid, ap, sta, an, sn = S.random_net(rr, essid_len=10)
    h1, h2 = os.path.join(tmp, "c2.hash"), os.path.join(tmp, "rules.hash")
    with open(h1, "wb") as f:
        f.write(S.eapol_line(psk1, essid, ap, sta, an, sn, 2, 3, "LE", mp=0x80, rng=rr) + b"\n")
    rr2 = random.Random(2)
    e2, a2, s2, an2, sn2 = S.random_net(rr2, essid_len=10)
    with open(h2, "wb") as f:
        f.write(S.eapol_line(rp["psk"], e2, a2, s2, an2, sn2, 2, 3, "LE", mp=0x80, rng=rr2) + b"\n")
    reader = None
    tool = os.path.join(ROOT, "tools", "bin", "inflate_bench")
    if os.path.exists(tool):
        # the library's dictionary reader alone on this host (dict_reader.hpp): how many devices one gz stream feeds
        import subprocess
        r = subprocess.run([tool, d1], capture_output=True, text=True, timeout=300)
        if r.returncode == 0:
            reader = json.loads(r.stdout)
    passes = []
    ok = True
    for rep in range(args.warmup + args.steps):
        step = []
        for name, hpath, dpath, rules_file, psk, pmks in (("dictionary", h1, d1, None, psk1, pmk1),
                                                         ("rules", h2, rp["dict"], rp["rules_file"], rp["psk"],
                                                          rp["cands"])):
            opath = os.path.join(tmp, name + ".key")
            if os.path.exists(opath):
                os.remove(opath)
            t0 = time.perf_counter()
            rc = dwpa_amd.crack_files(hpath, [dpath], rules_file, 8, opath, device_mask=mask, batch=args.batch,
                                      rule_mode=L.DWPA_RULES_FULL if args.rule_mode == "full" else L.DWPA_RULES_HASHCAT)
            el = time.perf_counter() - t0
            st, workers = M.crack_stats(), M.crack_worker_stats()
            recs = open(opath, "rb").read().strip().split(b"\n") if os.path.exists(opath) else []
            good = rc == 0 and len(recs) == 1 and recs[0].endswith(b":" + psk)
            ok &= good
            step.append({"pass": name, "s": el, "pmks": pmks, "words": st["words"], "candidates": st["candidates"],
                         "cracked_record_ok": good, "workers": workers})
        passes.append(step)
    timed = passes[args.warmup:]
    t = sum(p["s"] for step in timed for p in step) / len(timed)
    pmks = pmk1 + rp["cands"]
    last = timed[-1]
    emit({
        "metric": METRIC, "value": round(pmks / t, 1), "unit": "PMK/s", "n_gpus": ngpu, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "client node mode: one process, dwpa_crack_files over a mask of the node's devices; "
                               "per step the C2 pass (100M-word gzip dictionary, one EAPOL keyver-2 line, hashcat NC 8) "
                               "then the rule pass (gzip dictionary x WPA rules file)",
                   "device_mask": mask, "shard_workers_per_device": spd, "workers": ngpu * spd,
                   "rehearsal": (f"{spd} shard workers on one device: an {spd}-GPU node's worker count and shared "
                                 "feed, not its throughput") if ngpu == 1 and spd > 1 else None,
                   "dict_words": args.dict_words, "gz_bytes": gz_bytes, "gz_write_s": round(gz_s, 2),
                   "rule_words": rp["words"], "rules": len(rp["rules"]), "rules_set": args.rules_set,
                   "rule_mode": args.rule_mode, "batch": args.batch,
                   "dict_cache": "off (every pass inflates)" if os.environ.get("DWPA_DICT_CACHE_MB") == "0" else "on",
                   "parallelism": f"one process, {ngpu} device(s) x {spd} worker(s), shared dictionary feed"},
        "passes": [{"pass": p["pass"], "s": round(p["s"], 3), "pmks": p["pmks"], "pmk_per_s": round(p["pmks"] / p["s"], 1),
                    "words": p["words"], "words_per_s_feed": round(p["words"] / p["s"], 1),
                    "candidates_reported_by_library": p["candidates"], "cracked_record_ok": p["cracked_record_ok"],
                    "workers": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in w.items()}
                                for w in p["workers"]]} for p in last],
        "pass_s": [[round(p["s"], 3) for p in step] for step in passes],
        "roofline": None, "cpu_baseline": None, "hits_verified": bool(ok), "reader": reader})
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    if not ok:
        sys.exit(3)


def main_files_rules(args, world, rank, local):
    """The client's rule pass through dwpa_crack_files (help_crack.py:929-933: `-S -r <rules>` over the work
    unit's dictionaries): a gzip dictionary of --rule-words base words (6..16
    printable bytes) on local disk x the WPA rule set (dwpa_amd/rulesets.py, 148 rules of bestWPA.rule's ops) in a
    rules file, amplified on the GPU, one EAPOL keyver-2 line in hashcat NC mode 8.  The planted PSK is one rule's
    output of the 1000th-last word, so a pass covers the dictionary up to there.  PMKs counted = candidates inside
    the 8..63 filter: every rule of the set changes a word's length as a function of that length only, so the
    count is sum over word lengths of (words of that length) x (rules whose output length is in 8..63), taken from
    the library's own rule expansion of one word per length.  One pass = one step; N>1 runs replicas."""
    import random
    import tempfile
    import torch.distributed as dist
    import dwpa_amd
    from tests import synth as S
    from dwpa_amd.shard import reduce_timing

    if world > 1:
        dist.init_process_group("gloo")
    tmp = tempfile.mkdtemp(prefix="dwpa_c3files_")
    rp = _rule_pass_inputs(args, tmp, local)
    n, rules, psk, cands = rp["words"], rp["rules"], rp["psk"], rp["cands"]
    dpath, rpath = rp["dict"], rp["rules_file"]
    plant_word, plant_rule = rp["plant"]
    rr = random.Random(1)
    essid, ap, sta, an, sn = S.random_net(rr, essid_len=10)
    line = S.eapol_line(psk, essid, ap, sta, an, sn, 2, 3, "LE", mp=0x80, rng=rr)
    hpath, opath = (os.path.join(tmp, x) for x in ("h.hash", "o.key"))
    with open(hpath, "wb") as f:
        f.write(line + b"\n")
    cracked = True
    times, all_passes = [], []
    for rep in range(args.warmup + args.steps):
        if os.path.exists(opath):
            os.remove(opath)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        from dwpa_amd import _lib as L
        rc = dwpa_amd.crack_files(hpath, [dpath], rpath, 8, opath, device_mask=1 << local, batch=args.batch,
                                  rule_mode=L.DWPA_RULES_FULL if args.rule_mode == "full" else L.DWPA_RULES_HASHCAT)
        el = time.perf_counter() - t0
        st = dwpa_amd.m22000.crack_stats()
        reported = st["candidates"]
        rules_loaded = (st["rules"], st["rules_skipped"], st["rules_rejmem"])
        all_passes.append(round(el, 3))
        if rep >= args.warmup:
            times.append(el)
        recs = open(opath, "rb").read().strip().split(b"\n") if os.path.exists(opath) else []
        cracked &= rc == 0 and len(recs) == 1 and recs[0].endswith(b":" + psk)
    elapsed = sum(times) / len(times)
    # content-dependent functions (reject, purge, memory) make the length-only count inexact: count what the library
    # derived for the server set
    counted = cands if args.rules_set == "wpa" else reported
    if world > 1:
        from dwpa_amd.shard import all_ranks
        cracked = all_ranks(dist, cracked)
        elapsed, total = reduce_timing(dist, elapsed, float(counted))
    else:
        total = float(counted)
    if rank == 0:
        emit({
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "PMK/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"client rule pass via dwpa_crack_files: {n}-word gzip dictionary x {len(rules)} "
                                   f"{args.rules_set} rules (rules file, amplified on the GPU, 8..63 filter), one "
                                   "EAPOL keyver-2 line, hashcat NC mode 8", "rule_words": n, "rules": len(rules),
                       "rules_set": args.rules_set, "rule_mode": args.rule_mode,
                       "rules_loaded_skipped_rejmem": list(rules_loaded),
                       "candidates_counted": "length-only count up to the plant" if args.rules_set == "wpa" else
                                             "the library's count of derived candidates (dwpa_crack_last_stats)",
                       "candidates_per_pass": cands, "candidates_reported_by_library": reported,
                       "batch": args.batch, "parallelism": f"replicas x{world}",
                       "plant": [plant_word, plant_rule]},
            "pass_s": all_passes,
            "roofline": None, "cpu_baseline": None, "hits_verified": bool(cracked)})
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not cracked:
        sys.exit(3)


def main_expand(args, world, rank, local):
    """help_crack's wordlist expansion `hashcat --stdout -r bestWPA.rule source.txt -o cracked.txt.gz`
    (help_crack.py:508, every 100th run over the site's cracked.txt + rkg.txt; :575 for prdict) through
    dwpa_rules_expand_file: --rule-words synthetic words (6..16 printable bytes) x the WPA rule set (148 rules),
    plain-text output like hashcat's.  A step = one expansion of the whole source; value = candidates written per
    second (the output rate; a candidate is not a PMK here).  The count is checked against the rule set's
    per-length counts and the first candidates against the library's in-memory expansion."""
    import tempfile
    import numpy as np
    import dwpa_amd
    from dwpa_amd.rulesets import wpa_rules
    n = max(2000, args.rule_words)
    rules = wpa_rules()
    rules_text = "\n".join(rules)
    rng = np.random.default_rng(9)
    lens = rng.integers(6, 17, n).astype(np.int64)
    ends = np.cumsum(lens + 1)
    text = rng.integers(0x21, 0x7F, int(ends[-1]), dtype=np.uint8)
    text[text == ord("$")] = ord("%")
    text[ends - 1] = 0x0A
    reps = [bytes(b"abcdefghijklmnop"[:L]) for L in range(6, 17)]
    per_len = {L: sum(1 for c in r if c is not None)
               for L, r in zip(range(6, 17), dwpa_amd.rules_expand(rules_text, reps, device=local))}
    expected = int(sum(int(c) * per_len[L] for L, c in enumerate(np.bincount(lens, minlength=17)) if L >= 6))
    tmp = tempfile.mkdtemp(prefix="dwpa_expand_")
    spath, rpath, opath = (os.path.join(tmp, x) for x in ("source.txt", "bestWPA.rule", "cracked.txt.gz"))
    with open(spath, "wb") as f:
        f.write(text.tobytes())
    with open(rpath, "w") as f:
        f.write(rules_text + "\n")
    first = [text[int(ends[i - 1]) if i else 0:int(ends[i]) - 1].tobytes() for i in range(8)]
    del text
    times, ok = [], True
    for rep in range(args.warmup + args.steps):
        t0 = time.perf_counter()
        words, cands = dwpa_amd.m22000.rules_expand_file(rpath, [spath], opath, 0, local)
        el = time.perf_counter() - t0
        if rep >= args.warmup:
            times.append(el)
        ok &= words == n and cands == expected
    out_bytes = os.path.getsize(opath)
    with open(opath, "rb") as f:
        head = f.read(1 << 16).split(b"\n")
    exp_head = [c for row in dwpa_amd.rules_expand(rules_text, first, device=local) for c in row if c is not None]
    ok &= head[:len(exp_head)] == exp_head
    for x in (spath, rpath, opath):
        os.remove(x)
    os.rmdir(tmp)
    el = sum(times) / len(times)
    if rank == 0:
        emit({"metric": "candidates/s written, hashcat --stdout -r replacement (wordlist expansion)",
              "value": round(expected / el, 1), "unit": "candidates/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "u8", "data": "synthetic",
              "config": {"workload": f"expandcracked: {n}-word source x {len(rules)} WPA rules -> plain-text wordlist "
                                     "(dwpa_rules_expand_file)", "rule_words": n, "rules": len(rules),
                         "candidates": expected, "output_bytes": out_bytes, "parallelism": f"replicas x{world}"},
              "roofline": None, "cpu_baseline": None, "hits_verified": bool(ok)})
    if rank == 0 and not ok:
        sys.exit(3)


def cpu_baseline_jobs(jobs, seconds):
    """The PHP path for the same jobs: check_key_m22000 per job on the OpenSSL restatement (oracle/), as PHP-FPM
    runs requests: one job per worker process at a time, min(16, affinity) single-threaded processes (oracle/
    php_pool.py; the box's CPU share per GPU), over a bounded prefix of the job list; the same with one process per
    physical core of the host (`all_host`); plus one process alone (one PHP request after another)."""
    from oracle.php_pool import PhpPool, _job_pmks
    hc = host_cpu()
    P = hc["threads_all"]
    if len(jobs) == 1:
        line, keys, pmk, nc = jobs[0]
        return cpu_baseline(line, lambda m: keys[-m:], seconds, "keys (ending at the true PSK)", nc=nc)

    def run_pool(p, budget):
        pool = PhpPool(p)
        try:
            return pool.job_pmks(jobs, budget)
        finally:
            pool.close()
    done, nkeys, dt = run_pool(P, seconds)
    done1, nkeys1 = 0, 0
    t1 = time.perf_counter()
    while done1 < len(jobs) and time.perf_counter() - t1 < seconds / 3:
        nkeys1 += _job_pmks(jobs[done1])
        done1 += 1
    dt1 = time.perf_counter() - t1
    def measure_all(PA):
        doneA, nkeysA, dtA = run_pool(PA, seconds / 2)
        return {"value": round(nkeysA / dtA, 1), "unit": "PMK/s",
                "sample": f"first {doneA} jobs ({nkeysA} PMKs derived), one job per free worker, {dtA:.1f} s",
                "scaling_vs_one_process": round(nkeysA / dtA / (nkeys1 / dt1), 2)}
    all_host = all_host_row(hc, P, measure_all, nkeys1 / dt1, nkeys / dt)
    return dict({"value": round(nkeys / dt, 1), "unit": "PMK/s", "cores": P, "kind": "port",
                 "workers": f"{P} single-threaded worker processes (PHP-FPM model, oracle/php_pool.py)",
                 "sample": f"first {done} jobs ({nkeys} PMKs derived: a job stops at its first matching key), "
                           f"check_key_m22000 per job, {dt:.1f} s",
                 "scaling_vs_one_process": round(nkeys / dt / (nkeys1 / dt1), 2),
                 "one_thread": {"value": round(nkeys1 / dt1, 1), "unit": "PMK/s", "cores": 1,
                                "sample": f"first {done1} jobs ({nkeys1} PMKs derived) in one process (one PHP "
                                          f"request after another), {dt1:.1f} s"},
                 "all_host": all_host},
                **hc)


def host_cpu():
    """CPU model and counts of the host the baseline runs on.  threads_all = min(16, affinity): a GPU box gives one
    GPU a 16-core share, and its nproc reports the whole machine.  physical_cores_affinity counts distinct cores of
    the affinity set (SMT siblings once); all_host_processes = that count, the whole-host PHP-FPM pool (one worker
    per physical core).  cgroup_cpu_max is the container's CPU quota (cgroup v2 cpu.max), if any."""
    from oracle.php_pool import physical_cores
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), model)
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota = f.read().strip()
    except OSError:
        pass
    quota_cpus = None
    if quota and quota.split()[0] != "max":
        q, per = quota.split()[:2]
        quota_cpus = int(q) / int(per)
    cpus = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else set(range(os.cpu_count() or 1))
    phys = physical_cores(cpus)
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": len(cpus),
            "physical_cores_affinity": phys, "threads_all": max(1, min(16, len(cpus))),
            "all_host_processes": max(1, min(len(cpus), phys)), "cgroup_cpu_max": quota, "cgroup_cpus": quota_cpus}


def all_host_row(hc, P, measure, one_rate, pool_rate):
    """cpu_baseline.all_host: the PHP-FPM pool of the whole host (one single-threaded worker per physical core),
    measured when the process may use that many CPUs.  Under a cgroup CPU quota smaller than that (the GPU box
    gives a job 16 CPUs: cpu.max 1600000 100000) 128 workers would only share 16 CPUs, so the row is then the
    extrapolation one-process rate x physical cores x the measured pool's per-process efficiency, marked as such."""
    PA = hc["all_host_processes"]
    if PA <= P:
        return None
    quota = hc.get("cgroup_cpus")
    if quota is None or quota >= PA:
        row = measure(PA)
        row.update({"cores": PA, "processes": PA, "kind": "measured"})
        return row
    eff = pool_rate / (P * one_rate)
    return {"value": round(one_rate * PA * eff, 1), "unit": "PMK/s", "cores": PA, "processes": PA,
            "kind": "extrapolated",
            "basis": f"one process {one_rate:.1f} PMK/s x {PA} physical cores x {eff:.3f} (the {P}-process pool's "
                     f"per-process efficiency); not measurable here: cgroup cpu.max {hc['cgroup_cpu_max']} = "
                     f"{quota:g} CPUs for this job"}


def cpu_baseline(line, keys_fn, seconds, what, nc=NC):
    """The PHP CPU path: check_key_m22000(line, [key]) once per key (one PHP request per key, as put_work does,
    common.php:902), restated in C on OpenSSL (oracle/; PKCS5_PBKDF2_HMAC is the call openssl_pbkdf2 makes,
    common.php:178-180,246-248).  Timed as PHP-FPM serves requests -- min(16, affinity) single-threaded worker
    processes (oracle/php_pool.py; the box's CPU share per GPU), and one worker per physical core of the whole host
    (`all_host`, the node comparison) -- and in one process (one PHP request), over bounded samples of the
    workload's own candidates that end at the planted PSK, which every run must find.  PHP nonce window nc=8 (21
    attempts per EAPOL key) unless the leg's jobs carry their own."""
    from oracle import oracle as O
    from oracle.php_pool import PhpPool
    hc = host_cpu()
    P = hc["threads_all"]

    def run_pool(p, budget):
        pool = PhpPool(p)
        try:
            probe = keys_fn(64 * p)
            pool.check_keys(line, probe, nc)  # first checks in each worker (OpenSSL's method caches, clocks)
            _, dtp = pool.check_keys(line, probe, nc)
            rate = len(probe) / dtp
            m = int(max(len(probe), min(400_000 * max(1, p // 16), rate * budget)))
            sample = keys_fn(m)
            idx, dt = pool.check_keys(line, sample, nc)
        finally:
            pool.close()
        return rate, sample, idx, dt
    rate, sample, idx, dt = run_pool(P, seconds)
    m = len(sample)
    one = keys_fn(int(max(16, min(m, rate / P * seconds / 3))))
    t1 = time.perf_counter()
    idx1, _ = O.c_check_many(line, one, nc, 1)
    dt1 = time.perf_counter() - t1
    found_all = [True]

    def measure_all(PA):
        _, sA, idxA, dtA = run_pool(PA, seconds / 2)
        found_all[0] = idxA == len(sA) - 1
        return {"value": round(len(sA) / dtA, 1), "unit": "PMK/s",
                "sample": f"{len(sA)} {what} ending at the planted PSK, one check per key, {dtA:.1f} s",
                "scaling_vs_one_process": round(len(sA) / dtA / (len(one) / dt1), 2)}
    all_host = all_host_row(hc, P, measure_all, len(one) / dt1, len(sample) / dt)
    return dict({"value": round(len(sample) / dt, 1), "unit": "PMK/s", "cores": P, "kind": "port",
                 "workers": f"{P} single-threaded worker processes (PHP-FPM model, oracle/php_pool.py)",
                 "sample": f"{len(sample)} {what} ending at the planted PSK, check_key_m22000(line, [key], False, "
                           f"{nc}) per key, {dt:.1f} s",
                 "found_planted": idx == len(sample) - 1 and idx1 == len(one) - 1 and found_all[0],
                 "scaling_vs_one_process": round(len(sample) / dt / (len(one) / dt1), 2),
                 "one_thread": {"value": round(len(one) / dt1, 1), "unit": "PMK/s", "cores": 1,
                                "sample": f"the last {len(one)} of them in one process (one PHP request), "
                                          f"{dt1:.1f} s"},
                 "all_host": all_host},
                **hc)


if __name__ == "__main__":
    main()
