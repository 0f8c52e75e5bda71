"""GPU parity at the full BASELINE.json sizes of the device-resident configs.

The full keyspaces are far beyond what the CPU oracle can re-derive, so these tests use the size-independent
property the domain offers: the exact hit set.  Hashlines are planted for PSKs at chosen positions of the
keyspace (first and last candidate, both sides of batch boundaries, random interior points); every other
candidate must miss.  Each reported hit is then re-derived on the CPU: the PMK with O.c_pbkdf2 (OpenSSL
PKCS5_PBKDF2_HMAC, the call PHP's openssl_pbkdf2 makes, web/common.php:178-180) and the nonce correction with
O.c_check_key_m22000 (the restatement of check_key_m22000, common.php:157-307).

* C4 -- the whole 8-digit numeric keyspace 00000000..99999999 generated in-kernel (10^8 PMKs, ~21 s).
* C2 -- a 100M-word dictionary resident in HBM against EAPOL keyver-2 lines of one ESSID in hashcat nonce mode
  (--nonce-error-corrections=8, help_crack.py:773), as the client runs it (~22 s).
* C3 -- one dwpa_scan_run over 1,024 ESSIDs of a word x rule batch amplified on the GPU (every group of the work
  unit in one PBKDF2 launch); the expected hits come from the rule oracle (oracle/rules.py).  And C3's base size:
  10,000 words x the rule set over 8 ESSIDs in 4,096-word batches (~11.8 M PMKs).
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import dwpa_amd  # noqa: E402
from tests import synth as S  # noqa: E402
from dwpa_amd.device import Dictionary  # noqa: E402
from dwpa_amd.rulesets import wpa_rules  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import rules as R  # noqa: E402

B = 1 << 22  # the bench's batch (candidates per launch)


def _check_hit(line, psk, essid, h, nc_php):
    """A hit's PMK and (nc, endian) against the CPU oracle."""
    assert h["pmk"] == O.c_pbkdf2(psk, essid), (line[:40], psk)
    exp = O.c_check_key_m22000(line, [psk], False, nc_php)
    assert exp and exp[3] == h["pmk"]
    assert [h["nc"], h["endian"]] == exp[1:3], (line[:40], h, exp)


def test_c4_full_numeric_keyspace():
    """BASELINE configs[3]: all 10^8 candidates of one ESSID; >= 16 planted lines spread over the range (the
    ends, batch boundaries, the bench's 73019412, random points), PMKID plus one EAPOL line per key version."""
    rng = random.Random(104)
    essid, ap, sta, an, sn = S.random_net(rng, essid_len=8)
    n = 10 ** 8
    plants = {0, 1, 99999999, 99999998, B - 1, B, 2 * B - 1, 2 * B, 12 * B - 1, 12 * B, 23 * B - 1, 23 * B,
              n - n % B - 1, n - n % B, 73019412, 12345678, 50000000}
    while len(plants) < 24:
        plants.add(rng.randrange(n))
    plants = sorted(plants)
    lines, want = [], {}
    for k, v in enumerate(plants):
        psk = b"%08d" % v
        if k % 8 == 3:  # EAPOL keyver 1/2/3 with a planted correction inside the PHP nc=8 window (+-5)
            kv = 1 + (k // 8) % 3
            lines.append(S.eapol_line(psk, essid, rng.randbytes(6), sta, rng.randbytes(32), rng.randbytes(32), kv,
                                      rng.randint(-5, 5), rng.choice(["LE", "BE"]), rng=rng))
        else:
            lines.append(S.pmkid_line(psk, essid, rng.randbytes(6), sta))
        want[len(lines) - 1] = v
    sc = dwpa_amd.Scan(lines, nc=8, nc_mode=0, batch=B)
    assert sc.groups == 1
    hits = []
    for first in range(0, n, B):
        sc.load_numeric(first, min(B, n - first), 8)
        sc.pbkdf2(0)
        sc.verify(0)
        hits += sc.hits()
    assert sorted((h["line"], h["cand"]) for h in hits) == sorted(want.items())
    for h in hits:
        _check_hit(lines[h["line"]], b"%08d" % h["cand"], essid, h, 8)
    sc.close()


def test_c2_full_dictionary_hashcat_nc():
    """BASELINE configs[1]: 100M synthetic words (lengths geometric(0.3)+7 clipped to [8, 63], as bench.py) in
    HBM, one ESSID, EAPOL keyver-2 lines whose PSKs sit at the first and last word, at a batch boundary and at
    the bench's plant index; hashcat nonce mode (+-8 both endians, message_pair 0x80 / 0x00)."""
    import bench
    n = bench.DICT_WORDS
    off, data = bench.make_dictionary(n)
    rng = random.Random(102)
    essid, ap, sta, an, sn = S.random_net(rng, essid_len=10)
    where = [0, B - 1, B, bench.PLANT_INDEX, n - 1]
    lines, want, psks = [], {}, {}
    for k, i in enumerate(where):
        a, b = int(off[i]), int(off[i + 1])
        tag = b"PLANTED%d" % k  # overwrite the word in place with a PSK no random word can equal
        data[a:b] = np.frombuffer((tag * 8)[:b - a], dtype=np.uint8)
        psk = data[a:b].tobytes()
        psks[i] = psk
        lines.append(S.eapol_line(psk, essid, rng.randbytes(6), sta, an, sn, 2, rng.randint(-8, 8),
                                  rng.choice(["LE", "BE"]), mp=(0x80, 0x00)[k % 2], rng=rng))
        want[len(lines) - 1] = i
    d = Dictionary(off, data)
    sc = dwpa_amd.Scan(lines, nc=8, nc_mode=1, batch=B)
    hits = []
    for first in range(0, n, B):
        sc.load_dict(d.off.ptr, d.data.ptr, first, min(B, n - first), 8, 63)
        sc.pbkdf2(0)
        sc.verify(0)
        hits += sc.hits()
    assert sorted((h["line"], h["cand"]) for h in hits) == sorted(want.items())
    for h in hits:
        # PHP nc=16 spans +-9 (halfnc = 9): the single matching correction is the same in both modes
        _check_hit(lines[h["line"]], psks[h["cand"]], essid, h, 16)
    sc.close()
    d.off.free()
    d.data.free()


def test_c3_scan_run_1024_essids_rules():
    """BASELINE configs[2] geometry: 1,024 ESSIDs x 1-3 lines, one batch of 64 words x the WPA rule set amplified
    on the GPU (8..63 filter), one dwpa_scan_run deriving every (ESSID, candidate) PMK once and verifying every
    line of its ESSID.  Hits are planted in the first, middle and last groups and every 37th one; the expected
    set is every (line, word * nrules + rule) whose oracle candidate equals the line's PSK (duplicate candidates
    from different rules included)."""
    rng = random.Random(103)
    rules = wpa_rules()
    nr = len(rules)
    words = [S.random_psk(rng, 6, 12) for _ in range(64)]
    words[5] = b"Password"   # rules that map two ways onto one string (': ' vs 'c') give duplicate candidates
    words[6] = b"a" * 60     # most appends overflow 63 and are filtered
    expanded = R.expand(rules, words)
    valid = {wi * nr + ri: c for wi, row in enumerate(expanded) for ri, c in enumerate(row)
             if c is not None and 8 <= len(c) <= 63}
    E = 1024
    planted = {0, E // 2, E - 1} | set(range(0, E, 37))
    lines, line_essid, line_psk = [], [], []
    for e in range(E):
        essid = b"n%04d-" % e + bytes(rng.choice(b"abcdefghij") for _ in range(rng.randint(0, 20)))
        _, ap, sta, an, sn = S.random_net(rng)
        for k in range(1 + e % 3):
            if e in planted:
                cand = rng.choice(sorted(valid))
                if e == 0 and k == 0:
                    cand = 5 * nr + rules.index("c")  # "Password": the ':' rule gives the same string
                psk = valid[cand]
            else:
                psk = b"not-in-keyspace-%d-%d" % (e, k)
            kind = (e + k) % 4
            if kind == 0:
                lines.append(S.pmkid_line(psk, essid, rng.randbytes(6), sta))
            else:
                lines.append(S.eapol_line(psk, essid, ap, sta, an, sn, kind, rng.randint(-5, 5),
                                          rng.choice(["LE", "BE"]), rng=rng))
            line_essid.append(essid)
            line_psk.append(psk)
    want = sorted((li, c) for li, psk in enumerate(line_psk) for c, v in valid.items() if v == psk)
    assert len({li for li, _ in want}) >= 30
    assert any(line_psk[li] == b"Password" for li, _ in want) and sum(line_psk[li] == b"Password" for li, _ in want) >= 2
    batch = (len(words) * nr + 63) // 64 * 64
    d = Dictionary.from_words(words)
    sc = dwpa_amd.Scan(lines, nc=8, nc_mode=0, batch=batch)
    assert sc.groups == E
    assert sc.set_rules("\n".join(rules)) == nr
    sc.load_rules(d.off.ptr, d.data.ptr, 0, len(words))
    assert sc.loaded() == len(valid)
    sc.run()
    hits = sc.hits()
    assert sorted((h["line"], h["cand"]) for h in hits) == want
    for h in hits:
        _check_hit(lines[h["line"]], valid[h["cand"]], line_essid[h["line"]], h, 8)
    sc.close()


def test_c3_full_base_dictionary_rules():
    """SURVEY.md 8(d) C3's base size: 10,000 words x the WPA rule set (~1.48 M candidates per ESSID, 8..63 filter on
    the GPU) against 8 ESSIDs of 2 lines each, in dwpa_scan_run batches of 4,096 words x every rule (the last batch
    partial), ~11.8 M PMKs.  PSKs are planted at (word, rule) positions across the keyspace -- the first and last
    word, both sides of the batch boundaries, the last rule -- each from the rule oracle's expansion of that one word;
    every planted (line, candidate) must be reported, and every reported hit must be the line's PSK by the oracle
    (another rule may produce the same string: such duplicates are genuine) with the oracle's PMK and correction."""
    rng = random.Random(105)
    rules = wpa_rules()
    parsed = [p for p in (R.parse(x) for x in rules) if p]
    nr = len(parsed)
    assert nr == len(rules)
    nw, per = 10000, 4096
    words = [S.random_psk(rng, 6, 12) for _ in range(nw)]
    spots = [(0, 0), (nw - 1, nr - 1), (per - 1, 3), (per, nr // 2), (2 * per - 1, nr - 1), (2 * per, 1),
             (rng.randrange(nw), rng.randrange(nr)), (rng.randrange(nw), rng.randrange(nr))]
    plants = []
    for w, r in spots:  # the next rule of the word whose candidate passes the 8..63 filter
        for k in range(nr):
            c = R.apply(parsed[(r + k) % nr], words[w])
            if c is not None and 8 <= len(c) <= 63:
                plants.append((w, (r + k) % nr, c))
                break
    assert len(plants) == len(spots)
    lines, line_essid, want = [], [], set()
    for e in range(8):
        essid = b"c3-%d-" % e + bytes(rng.choice(b"abcdef") for _ in range(rng.randint(1, 12)))
        _, ap, sta, an, sn = S.random_net(rng)
        for k in range(2):
            i = 2 * e + k
            if i < len(plants):
                w, r, psk = plants[i]
                want.add((len(lines), w * nr + r))
            else:
                psk = b"not-in-keyspace-%d" % i
            if (e + k) % 2 == 0:
                lines.append(S.pmkid_line(psk, essid, rng.randbytes(6), sta))
            else:
                lines.append(S.eapol_line(psk, essid, ap, sta, an, sn, 1 + (e % 3), rng.randint(-4, 4),
                                          rng.choice(["LE", "BE"]), rng=rng))
            line_essid.append(essid)
    d = Dictionary.from_words(words)
    sc = dwpa_amd.Scan(lines, nc=8, nc_mode=0, batch=(per * nr + 63) // 64 * 64)
    assert sc.groups == 8
    assert sc.set_rules("\n".join(rules)) == nr
    hits = []
    for w0 in range(0, nw, per):
        sc.load_rules(d.off.ptr, d.data.ptr, w0, min(per, nw - w0))
        sc.run()
        hits += sc.hits()
    sc.close()
    got = {(h["line"], h["cand"]) for h in hits}
    assert want <= got, sorted(want - got)
    psk_of = {li: (plants[li][2] if li < len(plants) else None) for li in range(len(lines))}
    for h in hits:
        w, r = divmod(h["cand"], nr)
        cand = R.apply(parsed[r], words[w])
        assert cand == psk_of[h["line"]], (h, cand)
        _check_hit(lines[h["line"]], cand, line_essid[h["line"]], h, 8)
