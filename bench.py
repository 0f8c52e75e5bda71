"""bench.py -- PMK/s (PBKDF2-HMAC-SHA1 x4096) of the m22000 engine on MI355X, BASELINE.json configs[1] (C2).

Workload (per GPU): one ESSID, one EAPOL keyver-2 hashline (message_pair 0x80, planted nonce correction +3 LE,
PHP nonce window nc=8 -> 21 attempts), a 100M-word synthetic dictionary resident in HBM (uint64 offsets +
bytes, lengths geometric around 10 clipped to [8, 63]; the true PSK is word 99,999,000).  A step = one batch
of the dictionary through the hot path: candidates -> HMAC midstates -> PBKDF2 -> verify.  Rank r of N scans
batches r, r+N, ... (static keyspace shards, no collective on the data path): weak scaling.

The JSON line carries the PBKDF2 kernel's roofline (integer VALU bound) from HIP events recorded around each
launch on the stream it runs on, and the CPU baseline (the OpenSSL restatement of check_key_m22000 from
oracle/, timed on this host's cores on a bounded sample of the same workload).
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
NC = 8
# Roofline.  Work unit: 16,388 SHA-1 compressions per PMK (north_star).  Bound: integer
# VALU issue.  Measured on gfx950 (tools/valu_peak, profiles/r01/valu_issue_costs.json): xor/bitop3/add_u32 take
# 2 SIMD cycles per wave64 instruction, alignbit (rotate) and add3 take 4, so the cheapest HMAC inner-loop
# compression costs C_MIN = 1878.5 SIMD-cycles per wave (64 lanes; derivation in DESIGN.md section 4).
COMPRESSIONS_PER_PMK = 16388
C_MIN_CYCLES = 1878.5
SIMDS, CLOCK_HZ = 256 * 4, 2.4e9
PEAK_COMPRESSIONS = SIMDS * CLOCK_HZ * 64 / C_MIN_CYCLES
# HBM traffic of k_pbkdf2 per PMK, from the PMC passes of tools/profile_traffic.sh over this bench command
# (profiles/r01/traffic/traffic.json, per 4,194,304-PMK launch): FETCH_SIZE 167,954,944 B, doubled as
# MI355X_MICROARCH.md "HBM [CDNA4]" prescribes = 80 B/PMK (each of the two output-block lanes reads the 40-byte key
# midstate once), plus WRITE_SIZE 134,217,728 B = 32 B/PMK.  Algorithmic bytes are the same 80 + 32 = 112 B/PMK.
# PMC counters cannot be read inside a timed run, so the bench scales the measured per-PMK figure to its launches.
TRAFFIC_BYTES_PER_PMK = (2 * 167954944 + 134217728) / 4194304
ALGO_BYTES_PER_PMK = 80 + 32
# Nominal all-ops-full-rate view (128 int32 lane-ops/clk/CU, 576.5 ops/compression): reported, not attainable.
OPS_PER_COMPRESSION = 576.5
PEAK_LANE_OPS = 256 * 128 * CLOCK_HZ


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 22, help="candidates per step per GPU")
    ap.add_argument("--dict-words", type=int, default=DICT_WORDS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="batches in flight (c2/c3/c4), each on its own scan working set and HIP stream.  Measured "
                         "A/B (profiles/r01/pipeline/): 2 gains 0.2 %% -- the next batch's PBKDF2 waves hold the "
                         "SIMDs, so the verify runs starved beside it -- and blurs the per-kernel events; default 1")
    ap.add_argument("--workload", choices=["c1", "c2", "c3", "c4", "c5", "c2files"], default="c2",
                    help="c2 = BASELINE configs[1] (the bench line); c3/c4 = configs[2]/[3] legs; "
                         "c1/c5 = the FFI check path (host buffers, PCIe-inclusive); c2files = C2 through "
                         "dwpa_crack_files from a gz dictionary on disk (the help_crack client path)")
    ap.add_argument("--essids", type=int, default=1000, help="c3: number of ESSIDs (BASELINE: 1000)")
    ap.add_argument("--short-words", action="store_true",
                    help="c2files: lengths geometric(0.3)+6 so ~30 %% of the words are shorter than 8 and dropped "
                         "by the m22000 filter (as in real wordlists); PMK/s counts only 8..63-byte words")
    return ap.parse_args()


def make_dictionary(n, seed=2):
    """Host-side synthetic dictionary in the HBM layout (uint64 offsets + bytes), lengths geometric(0.3)+7 -> [8, 63]."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lens = np.clip(rng.geometric(0.3, n) + 7, 8, 63).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0x21, 0x7F, int(off[-1]) + 64, dtype=np.uint8)
    return off, data


class Workload:
    """One BASELINE.json config as a sequence of steps over HBM-resident candidates."""
    name = ""
    description = ""


def build_c2(args, local, S, Scan, Dictionary):
    """configs[1]: one ESSID, one EAPOL keyver-2 line, 100M-word dictionary."""
    import random
    w = Workload()
    n = args.dict_words
    w.plant = min(PLANT_INDEX, n - 1)
    w.off, w.data = make_dictionary(n)
    w.psk = w.data[int(w.off[w.plant]):int(w.off[w.plant + 1])].tobytes()
    rng = random.Random(1)
    w.essid, ap, sta, an, sn = S.random_net(rng, essid_len=10)
    w.line = S.eapol_line(w.psk, w.essid, ap, sta, an, sn, 2, 3, "LE", mp=0x80, rng=rng)
    w.dict = Dictionary(w.off, w.data, device=local)
    w.B = (args.batch + 63) & ~63
    w.nbatches = (n + w.B - 1) // w.B
    w.scans = [Scan([w.line], device=local, nc=NC, nc_mode=0, batch=w.B) for _ in range(args.pipeline)]
    w.groups = 1
    w.name = "C2"
    w.description = ("C2: one ESSID, one EAPOL keyver-2 line (mp 0x80, planted NC +3 LE), 100M-word synthetic "
                     "dictionary resident in HBM, PHP nonce window nc=8 (21 attempts)")
    w.extra = {"dict_words": n}

    def load(i, hs, sc):
        first = (i % w.nbatches) * w.B
        cnt = min(w.B, n - first)
        sc.load_dict(w.dict.off.ptr, w.dict.data.ptr, first, cnt, 8, 63, hs)
        return cnt

    def check(hits):
        return any(h["cand"] == w.plant and h["nc"] == 3 and h["endian"] == "LE" and h["pmk"] == S.pmk(w.psk, w.essid)
                   for h in hits)
    w.load, w.check, w.plant_batch = load, check, w.plant // w.B
    return w


def build_c4(args, local, S, Scan, Dictionary):
    """configs[3]: 8-digit numeric keyspace 00000000..99999999 generated in-kernel, one ESSID (PMKID line)."""
    import random
    w = Workload()
    n = 10 ** 8
    w.plant = 73019412
    rng = random.Random(3)
    w.essid, ap, sta, an, sn = S.random_net(rng, essid_len=8)
    w.line = S.pmkid_line(b"%08d" % w.plant, w.essid, ap, sta)
    w.B = (args.batch + 63) & ~63
    w.nbatches = (n + w.B - 1) // w.B
    w.scans = [Scan([w.line], device=local, nc=NC, nc_mode=0, batch=w.B) for _ in range(args.pipeline)]
    w.groups = 1
    w.name = "C4"
    w.description = "C4: 8-digit numeric keyspace (10^8) generated on the GPU, one ESSID, PMKID line"
    w.extra = {"keyspace": n}

    def load(i, hs, sc):
        first = (i % w.nbatches) * w.B
        cnt = min(w.B, n - first)
        sc.load_numeric(first, cnt, 8, hs)
        return cnt

    def check(hits):
        return any(h["cand"] == w.plant and h["pmk"] == S.pmk(b"%08d" % w.plant, w.essid) for h in hits)
    w.load, w.check, w.plant_batch = load, check, w.plant // w.B
    return w


def build_c3(args, local, S, Scan, Dictionary):
    """configs[2]: 10k-word dictionary x WPA rule set amplified on the GPU, across E ESSIDs with 1-4 lines each;
    each PMK is derived once per ESSID x candidate and tested against every line of that ESSID."""
    import random
    from dwpa_amd.rulesets import wpa_rules
    from dwpa_amd.device import dictionary_arrays
    import dwpa_amd
    w = Workload()
    rng = random.Random(4)
    base = [S.random_psk(rng, 6, 12) for _ in range(10000)]
    rules = wpa_rules()
    picks = [(rng.randrange(len(base)), rng.randrange(len(rules))) for _ in range(4 * args.essids)]
    expanded = dwpa_amd.rules_expand("\n".join(rules), [base[wi] for wi, _ in picks], device=local)
    w.off, w.data = dictionary_arrays(base)
    w.dict = Dictionary(w.off, w.data, device=local)
    lines, w.plants = [], []
    for e in range(args.essids):
        essid, ap, sta, an, sn = S.random_net(rng)
        for k in range(rng.randint(1, 4)):
            wi, ri = picks[4 * e + k]
            psk = expanded[4 * e + k][ri]
            if not psk or not 8 <= len(psk) <= 63:
                psk = b"not-in-keyspace-%d" % k
            elif e == 0 and k == 0:
                w.plants.append((len(lines), wi * len(rules) + ri, essid, psk))
            if k % 2:
                lines.append(S.pmkid_line(psk, essid, rng.randbytes(6), sta))
            else:
                lines.append(S.eapol_line(psk, essid, ap, sta, an, sn, 2, rng.randint(-3, 3), "LE", rng=rng))
    # one step = 4 x args.batch PMKs spread over every ESSID: 4*batch/E candidates x E ESSID groups, derived by
    # multi-group PBKDF2 launches (dwpa_scan_run).  Rule filtering makes the per-step count data-dependent, so the
    # last wave round of each launch is partial; 4x the C2 step keeps that tail near 2 %.
    w.B = max(len(rules) + 63, 4 * args.batch // max(1, args.essids)) // 64 * 64
    w.scans = [Scan(lines, device=local, nc=NC, nc_mode=0, batch=w.B) for _ in range(args.pipeline)]
    w.nrules = [sc.set_rules("\n".join(rules)) for sc in w.scans][0]
    w.words_per_step = max(1, w.B // w.nrules)
    w.nbatches = (len(base) + w.words_per_step - 1) // w.words_per_step
    w.groups = w.scans[0].groups
    w.name = "C3"
    w.description = (f"C3: 10k-word dictionary x {w.nrules} WPA rules amplified on the GPU (8..63 filter), "
                     f"{w.groups} ESSIDs x 1-4 lines, one PMK per ESSID x candidate")
    w.extra = {"essids": w.groups, "lines": len(lines), "rules": w.nrules}

    def load(i, hs, sc):
        first = (i % w.nbatches) * w.words_per_step
        nw = min(w.words_per_step, len(base) - first)
        sc.load_rules(w.dict.off.ptr, w.dict.data.ptr, first, nw, hs)
        return sc.loaded(hs) * w.groups

    def check(hits):
        return all(any(h["line"] == li and h["pmk"] == S.pmk(psk, essid) for h in hits)
                   for li, cand, essid, psk in w.plants)
    w.load, w.check = load, check
    w.plant_batch = (w.plants[0][1] // w.nrules) // w.words_per_step if w.plants else 0
    return w


def main():
    args = parse()
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DWPA_BENCH_ONE_DEVICE") == "1":
        local = 0  # rehearsal of the N>1 control path with every rank on one GPU (not a scaling measurement)
    if args.workload in ("c1", "c5"):
        return main_ffi(args, world, rank, local)
    if args.workload == "c2files":
        return main_files(args, world, rank, local)
    if world > 1:
        # control plane only (barrier, max-over-ranks time, sum of PMKs): the data path shards the keyspace and
        # never exchanges data, so there is no RCCL collective on the GPU.
        dist.init_process_group("gloo")

    import dwpa_amd
    from dwpa_amd import synth as S
    from dwpa_amd.device import Dictionary, Event, Stream
    from dwpa_amd.shard import batch_ids, reduce_timing

    build = {"c2": build_c2, "c3": build_c3, "c4": build_c4}[args.workload]
    w = build(args, local, S, dwpa_amd.Scan, Dictionary)
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
        if w.groups > 1:
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

    for s, b in enumerate(batch_ids(rank, world, 0, args.warmup, w.nbatches)):
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
    for s, b in enumerate(batch_ids(rank, world, args.warmup, args.steps, w.nbatches)):
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

    # correctness: the batch holding the planted PSK(s) must report them (untimed)
    for k in range(P):
        w.scans[k].hits(streams[k].handle)
    step(w.plant_batch, 0)
    verified = bool(w.check(w.scans[0].hits(streams[0].handle)))

    per_launch = list(counts) if w.groups > 1 else [c / w.groups for c in counts]
    pmk_per_launch = sum(per_launch) / len(per_launch)
    kernel_pmk_s = sum(per_launch) / (sum(kms) * 1e-3)
    achieved = kernel_pmk_s * COMPRESSIONS_PER_PMK
    if rank == 0:
        value = total / elapsed
        cpu = None
        if not args.no_cpu_baseline and args.workload == "c2" and world == 1:
            cpu = cpu_baseline(w.line, w.data, w.off, w.plant, args.cpu_seconds)
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
            "roofline": {
                "bound": "valu",
                "kernel": "k_pbkdf2" if w.groups == 1 else "k_pbkdf2_mg + k_verify (per dwpa_scan_run)",
                "achieved": round(achieved / 1e9, 3),
                "peak": round(PEAK_COMPRESSIONS / 1e9, 3),
                "unit": "G SHA-1 compressions/s",
                "frac": round(achieved / PEAK_COMPRESSIONS, 4),
                "traffic": round(TRAFFIC_BYTES_PER_PMK * pmk_per_launch),
                "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, profiles/r01/traffic)",
                "algorithmic_bytes": ALGO_BYTES_PER_PMK * pmk_per_launch,
                "hbm_gbs": round(TRAFFIC_BYTES_PER_PMK * pmk_per_launch / (kernel_ms * 1e-3) / 1e9, 3),
                "kernel_ms": round(kernel_ms, 3),
                "pmk_per_launch": pmk_per_launch,
                "kernel_pmk_per_s": round(kernel_pmk_s, 1),
                "roofline_pmk_per_s": round(PEAK_COMPRESSIONS / COMPRESSIONS_PER_PMK, 1),
                "peak_basis": f"{SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz x 64 lanes / {C_MIN_CYCLES} SIMD-cycles per "
                              "compression (measured gfx950 issue costs)",
                "frac_nominal_ops": round(kernel_pmk_s * COMPRESSIONS_PER_PMK * OPS_PER_COMPRESSION / PEAK_LANE_OPS, 4),
            },
            "cpu_baseline": cpu,
            "hits_verified": verified,
            "pbkdf2_kernel": "k_pbkdf2 (hipcc schedule)" if os.environ.get("DWPA_PBKDF2_PLAIN", "0") not in ("", "0")
                             else "k_pbkdf2_gfx950 (gfx950 VALU issue pass)",
            "rank0_local_s": round(elapsed_local, 4),
            "pipeline": P,
        }
        print(json.dumps(result), flush=True)
    for sc in w.scans:
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
    from dwpa_amd import synth as S
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
        jobs = S.c5_jobs()
        desc = ("C5: 250 PMKID + 250 x keyver 1/2/3 EAPOL lines (NC offsets 0..+-8, LE/BE) + 10 zero-PMK jobs, "
                "202 keys per job, nc=128 (261 attempts), dwpa_check_batch per step (FFI, host buffers)")
    batch = dwpa_amd.BatchJobs(jobs)
    for _ in range(args.warmup):
        batch.run()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.run()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        elapsed, total = reduce_timing(dist, time.perf_counter() - t0, float(batch.nkeys * args.steps))
    else:
        total = float(batch.nkeys * args.steps)
    got = batch.results()
    if args.workload == "c1":
        verified = bool(got[0]) and got[0][0] == psk and got[0][3] == S.pmk(psk, bytes.fromhex(line.split(b"*")[5].decode()))
    else:
        verified = sum(1 for g in got if g) >= 0.85 * len(jobs)
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline_jobs(jobs, args.cpu_seconds)
        print(json.dumps({
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "PMK/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": desc, "jobs": len(jobs), "keys_per_step": batch.nkeys,
                       "parallelism": f"replicas x{world}"},
            "roofline": None, "cpu_baseline": cpu, "hits_verified": verified,
            "hits": sum(1 for g in got if g)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not verified:
        sys.exit(3)


def main_files(args, world, rank, local):
    """C2 end to end through the client path (dwpa_crack_files, help_crack.py:765-802): the 100M-word dictionary
    as a gzip file on local disk, streamed, inflated and $HEX[]-decoded on the host, uploaded chunk by chunk and
    scanned against the C2 line (hashcat nonce mode, --nonce-error-corrections=8).  The planted PSK is the
    99,999,000th word, so the run covers the dictionary up to there.  One pass = one step; N>1 runs replicas."""
    import gzip
    import random
    import tempfile
    import numpy as np
    import torch.distributed as dist
    import dwpa_amd
    from dwpa_amd import synth as S
    from dwpa_amd.shard import reduce_timing

    if world > 1:
        dist.init_process_group("gloo")
    n = args.dict_words
    plant = min(PLANT_INDEX, n - 1)
    rng = np.random.default_rng(2)
    lens = np.clip(rng.geometric(0.3, n) + (6 if args.short_words else 7), 1, 63).astype(np.int64)
    lens[plant] = max(int(lens[plant]), 8)
    ends = np.cumsum(lens + 1)
    text = rng.integers(0x21, 0x7F, int(ends[-1]), dtype=np.uint8)
    text[ends - 1] = 0x0A
    psk = text[int(ends[plant - 1]) if plant else 0:int(ends[plant]) - 1].tobytes()
    rr = random.Random(1)
    essid, ap, sta, an, sn = S.random_net(rr, essid_len=10)
    line = S.eapol_line(psk, essid, ap, sta, an, sn, 2, 3, "LE", mp=0x80, rng=rr)
    tmp = tempfile.mkdtemp(prefix="dwpa_c2files_")
    dpath, hpath, opath = (os.path.join(tmp, x) for x in ("dict.txt.gz", "h.hash", "o.key"))
    t0 = time.perf_counter()
    with gzip.open(dpath, "wb", compresslevel=1) as f:
        step = 64 << 20
        for o in range(0, len(text), step):
            f.write(text[o:o + step].tobytes())
    gz_s = time.perf_counter() - t0
    gz_bytes = os.path.getsize(dpath)
    del text
    with open(hpath, "wb") as f:
        f.write(line + b"\n")
    cracked = True
    times = []
    for rep in range(args.warmup + args.steps):
        if os.path.exists(opath):
            os.remove(opath)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        rc = dwpa_amd.crack_files(hpath, [dpath], None, 8, opath, device_mask=1 << local, batch=args.batch)
        el = time.perf_counter() - t0
        if rep >= args.warmup:
            times.append(el)
        recs = open(opath, "rb").read().strip().split(b"\n") if os.path.exists(opath) else []
        cracked &= rc == 0 and len(recs) == 1 and recs[0].endswith(b":" + psk)
    elapsed = sum(times) / len(times)
    words = int(np.count_nonzero(lens[:plant + 1] >= 8))  # PMKs derived: words inside the 8..63 filter
    if world > 1:
        elapsed, total = reduce_timing(dist, elapsed, float(words))
    else:
        total = float(words)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "PMK/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "C2 via dwpa_crack_files: 100M-word gzip dictionary on local disk (streamed, "
                                   "inflated and uploaded per chunk), one EAPOL keyver-2 line, hashcat NC mode 8"
                                   + (", ~30 % of the words shorter than 8" if args.short_words else ""),
                       "dict_words": n, "gz_bytes": gz_bytes, "gz_write_s": round(gz_s, 2),
                       "words_scanned_per_pass": words, "batch": args.batch,
                       "parallelism": f"replicas x{world}"},
            "roofline": None, "cpu_baseline": None, "hits_verified": bool(cracked)}), flush=True)
    for x in (dpath, hpath, opath):
        if os.path.exists(x):
            os.remove(x)
    os.rmdir(tmp)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not cracked:
        sys.exit(3)


def cpu_baseline_jobs(jobs, seconds):
    """The PHP path for the same jobs: check_key_m22000 per job on the OpenSSL restatement (oracle/), jobs in
    parallel on up to 16 host threads, over a bounded prefix of the job list."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    if len(jobs) == 1:
        line, keys, pmk, nc = jobs[0]
        probe = keys[-threads * 32:]
        t0 = time.perf_counter()
        O.c_check_many(line, probe, nc, threads)
        rate = len(probe) / (time.perf_counter() - t0)
        sample = keys[-int(max(len(probe), min(len(keys), rate * seconds))):]
        t0 = time.perf_counter()
        idx, _ = O.c_check_many(line, sample, nc, threads)
        dt = time.perf_counter() - t0
        one = keys[-max(8, int(rate / threads * seconds / 4)):]
        t1 = time.perf_counter()
        O.c_check_many(line, one, nc, 1)
        dt1 = time.perf_counter() - t1
        return {"value": round(len(sample) / dt, 1), "unit": "PMK/s", "cores": threads, "kind": "port",
                "sample": f"last {len(sample)} keys (ending at the true PSK), one check per key, {dt:.1f} s",
                "found_planted": idx == len(sample) - 1,
                "one_php_request": {"value": round(len(one) / dt1, 1), "cores": 1,
                                    "sample": f"last {len(one)} keys on one thread, {dt1:.1f} s"}}
    done, nkeys = 0, 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while done < len(jobs) and time.perf_counter() - t0 < seconds:
            chunk = jobs[done:done + threads]
            list(ex.map(lambda j: O.c_check_key_m22000(*j), chunk))
            done += len(chunk)
            nkeys += sum(len(j[1]) for j in chunk)
    dt = time.perf_counter() - t0
    return {"value": round(nkeys / dt, 1), "unit": "PMK/s", "cores": threads, "kind": "port",
            "sample": f"first {done} jobs ({nkeys} keys), check_key_m22000 per job, {dt:.1f} s"}


def cpu_baseline(line, data, off, plant, seconds):
    """The PHP CPU path: check_key_m22000(line, [word]) per word (one PHP request per key, as put_work does,
    common.php:902), restated in C on OpenSSL (oracle/), on this host's cores; bounded sample ending at the
    planted PSK so the sample must also find it."""
    from oracle import oracle as O
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))

    def words(lo, hi):
        o = off[lo:hi + 1].astype("int64")
        raw = data[o[0]:o[-1]].tobytes()
        return [raw[o[i] - o[0]:o[i + 1] - o[0]] for i in range(hi - lo)]

    probe = words(plant - 64 * threads + 1, plant + 1)
    t0 = time.perf_counter()
    O.c_check_many(line, probe, NC, threads)
    rate = len(probe) / (time.perf_counter() - t0)
    m = int(max(len(probe), min(400_000, rate * seconds)))
    sample = words(plant - m + 1, plant + 1)
    t0 = time.perf_counter()
    idx, res = O.c_check_many(line, sample, NC, threads)
    dt = time.perf_counter() - t0
    return {"value": round(len(sample) / dt, 1), "unit": "PMK/s", "cores": threads, "kind": "port",
            "sample": f"{len(sample)} dictionary words ending at the planted PSK, check_key_m22000 per word "
                      f"(OpenSSL PKCS5_PBKDF2_HMAC + 21 NC attempts), {dt:.1f} s",
            "found_planted": idx == len(sample) - 1}


if __name__ == "__main__":
    main()
