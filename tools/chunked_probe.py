"""Diagnose the chunked derive (DWPA_CHECK_CHUNKS): one check_batch of 4 x 36,000 unique keys per setting, timed,
result compared with the head/tail split's.  Run each setting in its own process under a time limit:
    DWPA_CHECK_CHUNKS=K python3 tools/chunked_probe.py
"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dwpa_amd  # noqa: E402
from dwpa_amd import synth as S  # noqa: E402

rng = random.Random(91)
jobs = []
for e in range(4):
    essid, ap, sta, an, sn = S.random_net(rng, essid_len=9 + e)
    keys = [b"k%d-%06d-" % (e, i) + S.fast_psk(rng, 8, 20) for i in range(36000)]
    hit = [100, 20000, 1000, 30000][e]
    line = S.pmkid_line(keys[hit], essid, ap, sta)
    jobs.append((line, keys, False, 8))
t = time.time()
try:
    got = dwpa_amd.check_batch(jobs)
    ok = all(g and g[0] == j[1][h] for g, j, h in zip(got, jobs, [100, 20000, 1000, 30000]))
    err = None
except Exception as ex:  # noqa: BLE001
    ok, err = False, repr(ex)
t1 = time.time() - t
t = time.time()
if err is None:
    dwpa_amd.check_batch(jobs)
t2 = time.time() - t
print({"chunks": os.environ.get("DWPA_CHECK_CHUNKS"), "first_s": round(t1, 3), "second_s": round(t2, 3), "ok": ok,
       "err": err}, flush=True)
