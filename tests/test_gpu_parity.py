"""GPU parity: the HIP path (through the C ABI) against the oracle, bit-exact on every result tuple.

Oracle = CPU restatement of web/common.php (oracle/), pinned by tests/test_oracle.py.  Fixtures under
tests/golden/ were produced by the oracle (tests/golden/make_golden.py).
"""
import gzip
import os
import random
from concurrent.futures import ThreadPoolExecutor

import pytest

pytestmark = pytest.mark.gpu

import dwpa_amd  # noqa: E402
from dwpa_amd import _lib as L  # noqa: E402
from tests import synth as S  # noqa: E402
from dwpa_amd.rulesets import wpa_rules  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import rules as R  # noqa: E402
from tests.conftest import dec, job_args  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert dwpa_amd.device_count() >= 1
    yield


def test_pbkdf2_vectors(kat):
    for v in kat["pbkdf2"]:
        p, s = bytes.fromhex(v["password"]), bytes.fromhex(v["salt"])
        assert dwpa_amd.pbkdf2_pmk([p], s)[0].hex() == v["pmk32"]


def test_pbkdf2_random_lengths():
    rng = random.Random(7)
    keys = [bytes(rng.randrange(256) for _ in range(n)) for n in list(range(0, 70)) + [100, 127, 128, 200, 300]]
    for essid_len in (1, 7, 32, 47, 51, 52, 60, 120):
        essid = bytes(rng.randrange(256) for _ in range(essid_len))
        got = dwpa_amd.pbkdf2_pmk(keys, essid)
        exp = O.c_pbkdf2_many(keys, essid, threads=16)
        assert b"".join(got) == exp, essid_len


def test_pbkdf2_long_keys():
    """hash_pbkdf2 takes a key of any length (common.php:178,246): keys longer than the 64-byte HMAC block are
    hashed first, on the GPU in k_prep_keys (sha1_long_key), up to tens of KB per lane."""
    rng = random.Random(8)
    keys = [bytes(rng.randrange(256) for _ in range(n)) for n in (1000, 4095, 4096, 4097, 65537)]
    keys += [b"A" * 64 * 1024]
    got = dwpa_amd.pbkdf2_pmk(keys, b"ThisIsASSID")
    assert b"".join(got) == O.c_pbkdf2_many(keys, b"ThisIsASSID", threads=8)
    # and through the check path, plain and as $HEX[], PMKID and EAPOL: the first long key that verifies
    ap, sta = bytes.fromhex("020000000001"), bytes.fromhex("020000000002")
    lines = [S.pmkid_line(keys[4], b"ThisIsASSID", ap, sta, got[4]),
             S.eapol_line(keys[4], b"ThisIsASSID", ap, sta, bytes(range(32)), bytes(range(32, 64)), 2, nc=2,
                          mp=0x80, the_pmk=got[4])]
    jobs = [(line, cand, False, 8) for line in lines
            for cand in ([b"x" * 9, keys[3], keys[4]], [keys[0], b"$HEX[" + keys[4].hex().encode() + b"]"])]
    exp = [O.c_check_key_m22000(*j) for j in jobs]
    assert all(e and e[0] == keys[4] for e in exp)
    assert [dwpa_amd.check_key_m22000(*j) for j in jobs] == exp
    assert dwpa_amd.check_batch(jobs) == exp


def test_essid_lengths_check_path():
    """ESSIDs of 0..1000 bytes through the check path (hex2bin takes any even-length field, common.php:165,233; an
    empty field fails valid_hex): the salt of 1, 2 and 16+ SHA-1 blocks (salt + INT(i) + padding crosses a block at 52
    and 116 bytes), PMKID and EAPOL, one call per job and one batch."""
    rng = random.Random(9)
    ap, sta = bytes.fromhex("020000000001"), bytes.fromhex("020000000002")
    jobs = []
    for n in (0, 1, 32, 33, 51, 52, 55, 56, 64, 115, 116, 255, 1000):
        essid = bytes(rng.randrange(256) for _ in range(n))
        psk = S.random_psk(rng)
        jobs.append((S.pmkid_line(psk, essid, ap, sta), [b"wrongpsk1", psk], False, 8))
        jobs.append((S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), 1 + n % 3, -1, "BE",
                                  rng=rng), [psk], False, 8))
    exp = [O.c_check_key_m22000(*j) for j in jobs]
    assert exp[0] is False and exp[1] is False and all(exp[2:])
    assert [dwpa_amd.check_key_m22000(*j) for j in jobs] == exp
    assert dwpa_amd.check_batch(jobs) == exp


def test_challenge_kat(kat):
    for c in kat["challenge"]:
        assert dwpa_amd.check_key_m22000(c["line"], [b"aaaa1234"]) == dec(c["expect"])
    # the outfile must carry both challenge records with the same PSK (help_crack.py:886-895)
    r = dwpa_amd.check_key_m22000(kat["challenge"][1]["line"], [b"x" * 8, b"aaaa1234"], False, 8)
    assert r[0] == b"aaaa1234" and r[1:3] == [4, "LE"]


def test_mixed_golden_single(mixed):
    for j in mixed:
        line, keys, pmk, nc = job_args(j)
        assert dwpa_amd.check_key_m22000(line, keys, pmk, nc) == dec(j["expect"]), j["tag"]


def test_mixed_golden_batch(mixed):
    jobs = [job_args(j) for j in mixed]
    got = dwpa_amd.check_batch(jobs)
    for j, g in zip(mixed, got):
        assert g == dec(j["expect"]), j["tag"]


def test_nc_windows_golden(nc_windows):
    """The call sites' windows (nc 258 = put_work PMK propagation :919, 131 = submission :606, odd, negative),
    hits at +-halfnc in both endians and one past, the first/last attempt of 521-attempt lists behind 300 keys
    (attempt-parallel verify), caller PMKs and growing short-ANONCE lists: one call per job, then one batch."""
    for j in nc_windows:
        line, keys, pmk, nc = job_args(j)
        assert dwpa_amd.check_key_m22000(line, keys, pmk, nc) == dec(j["expect"]), j["tag"]
    got = dwpa_amd.check_batch([job_args(j) for j in nc_windows])
    for j, g in zip(nc_windows, got):
        assert g == dec(j["expect"]), j["tag"]


def _oracle_many(jobs):
    with ThreadPoolExecutor(16) as ex:
        return list(ex.map(lambda a: O.c_check_key_m22000(*a), jobs))


def test_random_batch_vs_oracle():
    """C5-shaped: PMKID + keyver 1/2/3, planted corrections, decoys, shared ESSIDs, zero-PMK jobs."""
    rng = random.Random(2024)
    jobs = []
    nets = [S.random_net(rng) for _ in range(12)]
    for i in range(160):
        essid, ap, sta, an, sn = nets[rng.randrange(len(nets))]
        ap, sta = rng.randbytes(6), rng.randbytes(6)
        psk = S.random_psk(rng)
        kind = rng.choice(["pmkid", 1, 2, 3])
        if kind == "pmkid":
            line = S.pmkid_line(psk, essid, ap, sta)
        else:
            line = S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), kind, rng.randint(-9, 9),
                                rng.choice(["LE", "BE"]), rng=rng)
        keys = [S.random_psk(rng) for _ in range(rng.randint(0, 12))]
        if rng.random() < 0.8:
            keys.insert(rng.randint(0, len(keys)), psk)
        if rng.random() < 0.1:
            keys.insert(0, None)
        nc = rng.choice([0, 1, 8, 16, 128])
        jobs.append((line, keys, False, nc))
    exp = _oracle_many(jobs)
    got = dwpa_amd.check_batch(jobs)
    mism = [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not mism, mism[:3]
    assert sum(1 for e in exp if e) > 60


def test_binary_essids_and_keys_vs_oracle():
    """ESSIDs and PSKs of arbitrary bytes: NUL, 0x80-0xff, the hashline's own separators '*' and ':' (the ESSID field
    is hex, so hex2bin hands PHP any byte string, common.php:165,233), ESSIDs of 1..64 bytes sharing a batch, keys of
    0..80 bytes with embedded NULs (strings, not C strings, on both sides of the FFI) and $HEX[] forms of them."""
    rng = random.Random(4242)
    jobs = []
    for i in range(120):
        essid = bytes(rng.choice([0, 0x2a, 0x3a, 0xff, 0x80, rng.randrange(256)]) for _ in range(rng.choice(
            [1, 2, 13, 31, 32, 33, 47, 64])))
        ap, sta = rng.randbytes(6), rng.randbytes(6)
        psk = bytes(rng.choice([0, 0xff, 0x3a, rng.randrange(256)]) for _ in range(rng.choice([0, 1, 8, 31, 63, 64, 80])))
        kind = rng.choice(["pmkid", 1, 2, 3])
        if kind == "pmkid":
            line = S.pmkid_line(psk, essid, ap, sta)
        else:
            line = S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), kind, rng.randint(-5, 5),
                                rng.choice(["LE", "BE"]), rng=rng)
        keys = [bytes(rng.randrange(256) for _ in range(rng.randint(0, 20))) for _ in range(rng.randint(0, 6))]
        form = psk if i % 3 else b"$HEX[" + psk.hex().encode() + b"]"
        if rng.random() < 0.85:
            keys.insert(rng.randint(0, len(keys)), form)
        jobs.append((line, keys, False, rng.choice([0, 8, 128])))
    exp = _oracle_many(jobs)
    got = dwpa_amd.check_batch(jobs)
    mism = [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not mism, mism[:3]
    for i in range(0, len(jobs), 7):
        assert dwpa_amd.check_key_m22000(*jobs[i]) == exp[i]
    assert sum(1 for e in exp if e) > 70


def test_mutated_lines_vs_oracle():
    """Parse semantics by mutation (tests/mutate.py): 1,500 valid PMKID/keyver 1/2/3 lines with one or two random
    mutations each (type field spellings, dropped/inserted/replaced characters, upper-case fields, odd or short or
    long hex fields, extra/missing/empty fields, key-version bits, EAPOL frames around the 49-byte unpack), the
    planted key among decoys, nc in {0, 1, 8, -3, 6}.  One batch call and one call per job for the first 200 must
    equal the oracle exactly, whether the line was rejected, stopped matching or stayed valid."""
    from tests.mutate import mutated_jobs
    jobs = mutated_jobs(2, 1500)
    exp = _oracle_many(jobs)
    got = dwpa_amd.check_batch(jobs)
    mism = [(i, jobs[i][0], g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not mism, mism[:3]
    for i in range(200):
        assert dwpa_amd.check_key_m22000(*jobs[i]) == exp[i], jobs[i][0]
    assert sum(1 for e in exp if e) > 100


def test_long_eapol_frames_vs_oracle():
    """EAPOL frames up to the longest a hashline can carry: nets.struct is varchar(2000) (db/wpa.sql:162), so a
    frame has at most ~900 bytes -- 15 SHA-1/MD5 blocks, 57 CMAC blocks.  Keyver 1/2/3 at 99..900 bytes, hits at
    +-nc in both endians and decoys, through the key-parallel (nc 8) and attempt-parallel (nc 128) verifiers, in
    one batch and per job."""
    rng = random.Random(61)
    jobs = []
    for el in (99, 100, 111, 112, 119, 120, 128, 175, 176, 255, 256, 400, 512, 777, 900):
        for kv in (1, 2, 3):
            essid, ap, sta, an, sn = S.random_net(rng)
            psk = S.random_psk(rng)
            nc = rng.choice([8, 128])
            off = rng.choice([0, 1, -1, 4, -4]) if nc == 8 else rng.choice([0, 30, -65, 65])
            line = S.eapol_line(psk, essid, ap, sta, an, sn, kv, off, rng.choice(["LE", "BE"]), eapol_len=el, rng=rng)
            assert len(line) <= 2000 or el > 900
            jobs.append((line, [S.random_psk(rng), psk, S.random_psk(rng)], False, nc))
    exp = _oracle_many(jobs)
    assert all(exp)
    assert dwpa_amd.check_batch(jobs) == exp
    for j, e in zip(jobs, exp):
        assert dwpa_amd.check_key_m22000(*j) == e


def test_scan_dictionary_hbm():
    from dwpa_amd.device import Dictionary
    rng = random.Random(3)
    essid, ap, sta, an, sn = S.random_net(rng)
    words = [S.random_psk(rng, 8, 20) for _ in range(20000)]
    words[123] = b"short"          # dropped by the 8..63 filter
    words[124] = b"x" * 64         # dropped
    psk1, psk2 = words[7777], words[19999]
    lines = [S.eapol_line(psk1, essid, ap, sta, an, sn, 2, 3, "LE", mp=0x80, rng=rng),
             S.pmkid_line(psk2, essid, rng.randbytes(6), sta),
             S.eapol_line(words[5], b"other", ap, sta, an, sn, 3, -2, "BE", rng=rng)]
    d = Dictionary.from_words(words)
    sc = dwpa_amd.Scan(lines, nc=8, batch=8192)
    hits = []
    for first in range(0, len(words), 8192):
        cnt = min(8192, len(words) - first)
        sc.load_dict(d.off.ptr, d.data.ptr, first, cnt)
        for g in range(sc.groups):
            sc.pbkdf2(g)
            sc.verify(g)
        hits += sc.hits()
    got = sorted((h["line"], h["cand"], h["nc"], h["endian"]) for h in hits)
    assert got == [(0, 7777, 3, "LE"), (1, 19999, None, None), (2, 5, -2, "BE")]
    for h in hits:
        w = words[h["cand"]]
        assert h["pmk"] == S.pmk(w, essid if h["line"] < 2 else b"other")
    sc.close()


def test_scan_numeric_keyspace():
    rng = random.Random(4)
    essid, ap, sta, an, sn = S.random_net(rng)
    lines = [S.pmkid_line(b"00731941", essid, ap, sta),
             S.eapol_line(b"00999999", essid, ap, sta, an, sn, 1, -1, "BE", rng=rng)]
    sc = dwpa_amd.Scan(lines, nc=8, batch=1 << 16)
    hits = []
    for first in range(700000, 1000000, 1 << 16):
        sc.load_numeric(first, min(1 << 16, 1000000 - first), 8)
        sc.pbkdf2(0)
        sc.verify(0)
        hits += sc.hits()
    assert sorted((h["line"], h["cand"], h["nc"]) for h in hits) == [(0, 731941, None), (1, 999999, -1)]
    sc.close()


def test_rules_expand_vs_oracle():
    rng = random.Random(5)
    rules = wpa_rules() + ["C", "t", "q", "{", "}", "z2", "Z3", "@a", "sab", "p3", "D0", "'0", "T9", "$ ", "^ "]
    words = [S.random_psk(rng, 1, 30) for _ in range(300)] + [b"a", b"Password", b"x" * 130, b"y" * 255, b"z" * 256]
    got = dwpa_amd.rules_expand("\n".join(rules), words)
    exp = R.expand(rules, words)
    assert got == exp


@pytest.mark.parametrize("group", ["single", "memory", "combo"])
def test_rules_language_gpu_vs_oracle(group):
    """every function of hashcat's rule language (mangling, reject and memory functions) at edge
    arguments -- positions 0, len-1, len and beyond -- on words of 1..256 bytes (and the rejected empty and
    257-byte words), alone, after M, and in random combinations: the GPU rule engine equals oracle/rules.py."""
    from tests import rule_corpus as C
    rules = {"single": C.single_function_rules, "memory": C.memory_rules, "combo": C.combo_rules}[group]()
    words = C.words()
    got = dwpa_amd.rules_expand("\n".join(rules).encode("latin-1"), words)
    exp = R.expand(rules, words)
    bad = [(rules[j], w[:16], len(w), got[i][j], exp[i][j]) for i, w in enumerate(words) for j in range(len(rules))
           if got[i][j] != exp[i][j]]
    assert not bad, bad[:8]


def test_rules_fuzz_gpu_vs_oracle():
    """Random rule strings over the whole alphabet (tests/rule_corpus.py fuzz_rules): the GPU expands exactly the
    rules the oracle parses, in order, and every candidate equals the oracle's."""
    from tests import rule_corpus as C
    rules = C.fuzz_rules()
    words = C.fuzz_words()
    parsed = [r for r in rules if R.parse(r) is not None]
    got = dwpa_amd.rules_expand("\n".join(rules).encode("latin-1"), words)
    exp = R.expand(parsed, words)
    assert len(got[0]) == len(parsed)
    bad = [(parsed[j], w[:12], len(w)) for i, w in enumerate(words) for j in range(len(parsed)) if got[i][j] != exp[i][j]]
    assert not bad, bad[:8]


@pytest.mark.parametrize("mode", ["hashcat", "full"])
def test_crack_files_every_rule_family(tmp_path, mode):
    """A work unit whose server rule file (-S -r, help_crack.py:931-933) uses every family of the language beyond
    bestWPA.rule's ops -- insert/overwrite/extract/omit, swaps and byte arithmetic, block duplication, title case and
    toggle-after-separator, reject functions, memory functions -- plus lines that do not parse.  The skipped lines are
    counted in dwpa_crack_last_stats, not dropped silently.

    * hashcat (the default, DWPA_RULES_HASHCAT): hashcat's -r loader skips the lines using reject or memory
      functions (they work only with -j/-k), so exactly the PSKs behind the other families are found and the reject
      / memory lines count as skipped (rules_rejmem) -- the reference client's `-S -r` run tries the same candidates.
    * full (DWPA_RULES_FULL): every family runs and a PSK planted behind each one is found; a PSK only a rejected
      candidate would equal is not."""
    rng = random.Random(21)
    essid, _, sta, _, _ = S.random_net(rng)
    base = [S.random_psk(rng, 6, 14) for _ in range(3000)]
    base[700] = b"pass word-xyz"
    family = {"insert": "i4! o0P", "extract": "x15 $2 $0 $2 $4", "omit": "O23 ^#", "swap": "*03 k K",
              "arith": "+0 -1 L2 R3 .4 ,5", "dupe": "y3 Y2", "title": "E $!", "toggle_sep": "30  30-",
              "reject": ">9 /w !@ (p", "reject_eq": "=4  %1- $X", "memory": "M l 4", "memory_x": "u M X031 6",
              "memory_q": "M r Q $9"}
    invalid = ["I", "T", "X01", "3a-", "v12"]
    rules = list(family.values())
    rf = tmp_path / "help_crack.rules"
    rf.write_text("\n".join(rules[:5] + invalid + rules[5:]) + "\n")
    planted, lines = {}, []
    for k, (name, rule) in enumerate(family.items()):
        wi = 700 if name in ("title", "toggle_sep", "reject", "reject_eq") else 100 + 37 * k
        while not 8 <= len(R.apply(R.parse(rule), base[wi]) or b"") <= 63:  # the first word the rule keeps
            wi += 1
        psk = R.apply(R.parse(rule), base[wi])
        ap = bytes([2, 0, 0, 0, 0, k])
        planted[ap.hex()] = psk
        lines.append(S.pmkid_line(psk, essid, ap, sta))
    # only the rejected candidate of word 1500 under '<8 $!' (the word is longer than 8) would equal this PSK
    assert len(base[1500]) > 8
    never = base[1500] + b"!"
    rf.write_text(rf.read_text() + "<8 $!\n")
    lines.append(S.pmkid_line(never, essid, bytes([2, 0, 0, 0, 1, 0]), sta))
    hf = tmp_path / "h.hash"
    hf.write_bytes(b"\n".join(lines) + b"\n")
    d = tmp_path / "d.txt"
    d.write_bytes(b"\n".join(base) + b"\n")
    out = tmp_path / "o.key"
    rmode = {"hashcat": L.DWPA_RULES_HASHCAT, "full": L.DWPA_RULES_FULL}[mode]
    rc = dwpa_amd.crack_files(str(hf), [str(d)], str(rf), 8, str(out), batch=1 << 16, rule_mode=rmode)
    assert all(R.apply(R.parse(r), w) != never for r in rules + ["<8 $!"] for w in base)  # no candidate equals it
    assert rc == 1  # the never line stays uncracked
    got = {}
    for rec in out.read_bytes().strip().split(b"\n"):
        f = rec.split(b":", 4)
        v = f[4]
        if v.startswith(b"$HEX[") and v.endswith(b"]"):
            v = bytes.fromhex(v[5:-1].decode())
        got[f[1].decode()] = v
    rejmem = {"reject", "reject_eq", "memory", "memory_x", "memory_q"}
    kept = [n for n in family if mode == "full" or n not in rejmem]
    aps = list(planted)
    assert got == {aps[k]: planted[aps[k]] for k, n in enumerate(family) if n in kept}
    st = dwpa_amd.m22000.crack_stats()
    if mode == "full":
        assert (st["rules"], st["rules_skipped"], st["rules_rejmem"]) == (len(rules) + 1, len(invalid), 0)
    else:  # the five reject / memory families and the '<8 $!' line
        assert (st["rules"], st["rules_skipped"], st["rules_rejmem"]) == (len(kept), len(invalid) + 6, 6)
    counts = dwpa_amd.rules_count_ex(rf.read_bytes())
    assert (counts["parsed"], counts["loaded_hashcat"], counts["rejmem"], counts["invalid"]) == \
        (len(rules) + 1, len(rules) + 1 - 6, 6, len(invalid))


def test_crack_files_challenge(tmp_path):
    hf = tmp_path / "help_crack.hash"
    hf.write_bytes(b"\n".join(S.CHALLENGE_LINES) + b"\n")
    d1 = tmp_path / "d1.txt.gz"
    with gzip.open(d1, "wb") as f:
        f.write(b"\n".join([b"password%d" % i for i in range(5000)] + [b"aaaa1234"]) + b"\n")
    out = tmp_path / "help_crack.key"
    rc = dwpa_amd.crack_files(str(hf), [str(d1)], None, 8, str(out))
    assert rc == 0
    txt = out.read_text()
    recs = txt.strip().split("\n")
    assert len(recs) == 2
    for r in recs:
        assert "1c7ee5e2f2d0:0026c72e4900:dlink:aaaa1234" in r  # help_crack.py:858-860
    # help_crack's parser (get_key, :807-815) reads k = MAC_AP, v = hex(PSK)
    for r in recs:
        arr = r.split(":", 4)
        assert arr[1][:12] == "1c7ee5e2f2d0" and arr[4].encode().hex() == b"aaaa1234".hex()


def test_crack_files_rules_and_exhausted(tmp_path):
    rng = random.Random(6)
    essid, ap, sta, an, sn = S.random_net(rng)
    base = [S.random_psk(rng, 6, 12) for _ in range(3000)]
    rules = wpa_rules()
    target_word, target_rule = base[1234], rules.index("c $1 $2 $3")
    psk = R.apply(R.parse(rules[target_rule]), target_word)
    lines = [S.eapol_line(psk, essid, ap, sta, an, sn, 2, 2, "BE", rng=rng),
             S.pmkid_line(b"not-in-dict-!!", essid, ap, sta)]
    hf = tmp_path / "h.hash"
    hf.write_bytes(b"\n".join(lines) + b"\n")
    d = tmp_path / "d.txt"
    d.write_bytes(b"\n".join(base) + b"\n")
    rf = tmp_path / "r.rule"
    rf.write_text("\n".join(rules) + "\n")
    out = tmp_path / "o.key"
    rc = dwpa_amd.crack_files(str(hf), [str(d)], str(rf), 8, str(out), batch=1 << 16)
    assert rc == 1
    recs = out.read_bytes().strip().split(b"\n")
    assert len(recs) == 1
    plain = psk if all(0x20 <= c <= 0x7E and c != 0x3A for c in psk) else b"$HEX[" + psk.hex().encode() + b"]"
    assert recs[0].endswith(b":" + plain)


def test_scan_rules_device_resident():
    """configs[2] shape: words x rules amplified on the GPU, several ESSIDs, hits with word*nrules+rule ids."""
    from dwpa_amd.device import Dictionary
    rng = random.Random(8)
    base = [S.random_psk(rng, 5, 12) for _ in range(2000)]
    rules = wpa_rules()
    d = Dictionary.from_words(base)
    nets = [S.random_net(rng) for _ in range(3)]
    plants = [(17, rules.index("$2 $0 $2 $4")), (1999, rules.index("u $1")), (500, rules.index("^e ^h ^t"))]
    lines = []
    for (wi, ri), (essid, ap, sta, an, sn) in zip(plants, nets):
        psk = R.apply(R.parse(rules[ri]), base[wi])
        lines.append(S.eapol_line(psk, essid, ap, sta, an, sn, 2, -1, "BE", rng=rng))
    sc = dwpa_amd.Scan(lines, nc=8, batch=1 << 18)
    assert sc.set_rules("\n".join(rules)) == len(rules)
    per = (1 << 18) // len(rules)
    hits = []
    for first in range(0, len(base), per):
        sc.load_rules(d.off.ptr, d.data.ptr, first, min(per, len(base) - first))
        for g in range(sc.groups):
            sc.pbkdf2(g)
            sc.verify(g)
        hits += sc.hits()
    got = {(h["line"], h["nc"], h["endian"]) for h in hits}
    assert got == {(0, -1, "BE"), (1, -1, "BE"), (2, -1, "BE")}
    for h in hits:
        wi, ri = divmod(h["cand"], len(rules))
        essid = nets[h["line"]][0]
        assert h["pmk"] == S.pmk(R.apply(R.parse(rules[ri]), base[wi]), essid)
    sc.close()


def test_scan_run_many_essids_matches_per_group():
    """dwpa_scan_run: many ESSID groups per PBKDF2 launch (1- and 2-block salts in one launch, several launches
    when groups x batch exceeds 16M slots) gives exactly the per-group path's hits, and every hit's PMK is the
    oracle's."""
    from dwpa_amd.device import Dictionary
    rng = random.Random(12)
    words = [S.random_psk(rng, 8, 24) for _ in range(3000)]
    d = Dictionary.from_words(words)
    lines, plants = [], []
    for e in range(12):
        essid = bytes(rng.randrange(0x21, 0x7f) for _ in range((1, 9, 32, 52, 60)[e % 5]))
        _, ap, sta, an, sn = S.random_net(rng)
        for k in range(1 + e % 3):
            wi = rng.randrange(len(words))
            kind = (e + k) % 4
            if kind == 0:
                lines.append(S.pmkid_line(words[wi], essid, rng.randbytes(6), sta))
            else:
                lines.append(S.eapol_line(words[wi], essid, ap, sta, an, sn, kind, rng.randint(-5, 5),
                                          rng.choice(["LE", "BE"]), rng=rng))
            plants.append((len(lines) - 1, wi, essid))
    lines.append(S.pmkid_line(b"not-in-the-dictionary", b"lonely", rng.randbytes(6), rng.randbytes(6)))
    results = []
    for mode in ("run", "per_group"):
        sc = dwpa_amd.Scan(lines, nc=8, batch=1 << 22)  # 16M-slot launches hold 4 groups: 4+3+3+3 for 13 ESSIDs
        assert sc.groups == 13
        sc.load_dict(d.off.ptr, d.data.ptr, 0, len(words))
        if mode == "run":
            sc.run()
        else:
            for g in range(sc.groups):
                sc.pbkdf2(g)
                sc.verify(g)
        results.append(sorted((h["line"], h["cand"], h["nc"], h["endian"], h["pmk"]) for h in sc.hits()))
        sc.close()
    assert results[0] == results[1]
    found = {(h[0], h[1]) for h in results[0]}
    assert {(li, wi) for li, wi, _ in plants} <= found
    for li, cand, nc, endian, pmk in results[0]:
        essid = next(e for l, _, e in plants if l == li)
        assert pmk == O.c_pbkdf2(words[cand], essid)


def test_crack_files_hex_dictionary_and_outfile_escaping(tmp_path):
    """A13/A15: $HEX[] dictionary words are decoded before hashing (help_crack.py:520-552, maint.php:55-60), CRLF
    and empty lines are tolerated, and a PSK that is not printable ASCII or contains ':' is written back as
    $HEX[..] (help_crack.py:807-815 reads the outfile as UTF-8 and splits on ':'); plain PSKs stay plain."""
    rng = random.Random(21)
    essid, ap, sta, an, sn = S.random_net(rng)
    psk_colon = b"pa:ss\xe9word!"          # ':' and a non-ASCII byte -> $HEX[] both ways
    psk_plain = b"plain-psk-123"
    lines = [S.pmkid_line(psk_colon, essid, ap, sta),
             S.eapol_line(psk_plain, essid, ap, rng.randbytes(6), an, sn, 2, -2, "BE", rng=rng)]
    hf = tmp_path / "h.hash"
    hf.write_bytes(b"\n".join(lines) + b"\n")
    words = [b"filler%05d" % i for i in range(3000)]
    words[1000] = b"$HEX[" + psk_colon.hex().encode() + b"]"
    words[2000] = psk_plain
    d = tmp_path / "d.txt.gz"
    with gzip.open(d, "wb") as f:
        f.write(b"\r\n".join(words[:1500]) + b"\r\n\r\n" + b"\n".join(words[1500:]) + b"\n")
    out = tmp_path / "o.key"
    rc = dwpa_amd.crack_files(str(hf), [str(d)], None, 8, str(out))
    assert rc == 0
    recs = sorted(out.read_bytes().strip().split(b"\n"))
    assert len(recs) == 2
    assert sum(r.endswith(b":$HEX[" + psk_colon.hex().encode() + b"]") for r in recs) == 1
    assert sum(r.endswith(b":" + psk_plain) for r in recs) == 1
    # help_crack's get_key: split(":", 4) on the UTF-8 text recovers field 4 exactly
    for r in recs:
        arr = r.decode("utf-8").split(":", 4)
        assert len(arr) == 5 and arr[1] == ap.hex()


def _get_key(key_file):
    """help_crack.py:804-815 (get_key): outfile records -> {MAC_AP: hex(PSK)} (k = arr[1][:12], v from arr[4])."""
    res = {}
    with open(key_file, encoding="utf-8", errors="ignore") as f:
        for line in f:
            arr = line.rstrip("\n").split(":", 4)
            if len(arr) == 5:
                res[arr[1][:12]] = arr[4].encode("utf-8").hex()
    return res


def test_help_crack_two_pass_flow(tmp_path):
    """help_crack.py:923-933 through the ctypes drop-in: pass 1 without rules is exhausted (rc 1), pass 2 with the
    work unit's rules ("-S -r help_crack.rules") cracks the rest (rc 0); get_key parses the outfile unchanged."""
    from dwpa_amd.help_crack import run_cracker
    rng = random.Random(31)
    essid, ap, sta, an, sn = S.random_net(rng)
    alnum = b"abcdefghijklmnopqrstuvwxyz0123456789"  # outfile-safe PSKs: get_key returns them verbatim
    base = [bytes(rng.choice(alnum) for _ in range(rng.randint(8, 14))) for _ in range(2000)]
    rules = ["$1", "u", "c $2 $0 $2 $4"]
    direct, ruled = base[42], R.apply(R.parse(rules[2]), base[1500])
    ap2 = rng.randbytes(6)
    lines = [S.pmkid_line(direct, essid, ap, sta),
             S.eapol_line(ruled, essid, ap2, sta, an, sn, 2, 1, "LE", rng=rng)]
    conf = {"hash_file": str(tmp_path / "help_crack.hash"), "key_file": str(tmp_path / "help_crack.key"),
            "rules": "", "coptions": ""}
    (tmp_path / "help_crack.hash").write_bytes(b"\n".join(lines) + b"\n")
    d = tmp_path / "dict.txt.gz"
    with gzip.open(d, "wb") as f:
        f.write(b"\n".join(base) + b"\n")
    assert run_cracker(conf, [str(d)]) == 1
    assert _get_key(conf["key_file"]) == {ap.hex(): direct.hex()}
    (tmp_path / "help_crack.rules").write_text("\n".join(rules) + "\n")
    conf["rules"] = "-S -r " + str(tmp_path / "help_crack.rules")
    (tmp_path / "help_crack.hash").write_bytes(lines[1] + b"\n")  # prepare_work writes the uncracked lines
    assert run_cracker(conf, [str(d)]) == 0
    assert _get_key(conf["key_file"]) == {ap.hex(): direct.hex(), ap2.hex(): ruled.hex()}
    conf["hash_file"] = str(tmp_path / "missing.hash")
    with pytest.raises(FileNotFoundError):
        run_cracker(conf, [str(d)])


def test_help_crack_truncated_dictionary_no_livelock(tmp_path):
    """a cut .gz download.  run_cracker with max_tries=None (the reference's forever loop) and
    a sleepy() that fails the test: one attempt scans the words before the cut (a PSK there is found and written
    once), returns 1 like hashcat over gzread, and deletes the damaged file so prepare_dicts downloads it again.
    A PSK after the cut is not found."""
    from dwpa_amd.help_crack import run_cracker
    rng = random.Random(41)
    alnum = b"abcdefghijklmnopqrstuvwxyz0123456789"
    words = [bytes(rng.choice(alnum) for _ in range(rng.randint(8, 14))) for _ in range(300_000)]
    nets = [S.random_net(rng) for _ in range(3)]
    before, after = words[5000], words[290_000]
    lines = [S.pmkid_line(before, nets[0][0], nets[0][1], nets[0][2]),
             S.eapol_line(after, nets[1][0], nets[1][1], nets[1][2], nets[1][3], nets[1][4], 2, 2, "BE", rng=rng),
             S.pmkid_line(b"never-in-the-dictionary", nets[2][0], nets[2][1], nets[2][2])]
    conf = {"hash_file": str(tmp_path / "help_crack.hash"), "key_file": str(tmp_path / "help_crack.key"),
            "rules": "", "coptions": ""}
    (tmp_path / "help_crack.hash").write_bytes(b"\n".join(lines) + b"\n")
    blob = gzip.compress(b"\n".join(words) + b"\n", compresslevel=6)
    d = tmp_path / "cut.txt.gz"
    d.write_bytes(blob[:len(blob) * 2 // 3])

    def no_sleep():
        raise AssertionError("run_cracker retried a deterministic dictionary error")
    assert run_cracker(conf, [str(d)], sleepy=no_sleep, pprint=lambda *a: None, max_tries=None) == 1
    assert not d.exists()
    assert _get_key(conf["key_file"]) == {nets[0][1].hex(): before.hex()}
    assert open(conf["key_file"], "rb").read().count(b"\n") == 1


def _stdout_plain(c: bytes) -> bytes:
    """hashcat's --stdout form of a candidate: its raw bytes; one holding '\\n' or '\\r' (which would not stay one
    line) as $HEX[..]."""
    if b"\n" in c or b"\r" in c:
        return b"$HEX[" + c.hex().encode() + b"]"
    return c


@pytest.mark.parametrize("gzip_level", [0, 1])
def test_help_crack_expand_rules_file(tmp_path, gzip_level):
    """`hashcat --stdout -r bestWPA.rule source.txt -o cracked.txt.gz` (help_crack.py:508) via the GPU rule engine
    and the library's packing (dwpa_rules_expand_file): the output equals the rule oracle's expansion in word-major
    order with rejected candidates skipped, raw bytes as hashcat's --stdout writes them and $HEX[] only for a
    candidate holding a newline -- over 20k words x 148 rules (3M candidates: several sub-batches, both slot sets),
    $HEX[] source words decoded, a 300-byte word rejected.  Plain text (what hashcat writes) and gzip.  Parity with
    hashcat itself unpinned."""
    from dwpa_amd.help_crack import expand_rules
    rng = random.Random(32)
    words = [S.random_psk(rng, 1, 20) for _ in range(20000)] + [b"x" * 300]
    words[7] = b"\x00\xffAb"
    words[9] = b"ab\ncd\rxy"
    rules = wpa_rules()
    src = tmp_path / "source.txt"
    src.write_bytes(b"\n".join(b"$HEX[" + w.hex().encode() + b"]" if any(b < 0x20 or b > 0x7E for b in w) else w
                                for w in words) + b"\n")
    rf = tmp_path / "bestWPA.rule"
    rf.write_text("\n".join(rules) + "\n")
    out = tmp_path / "cracked.txt.gz"
    n = expand_rules(str(rf), str(src), str(out), gzip_level=gzip_level)
    exp = [_stdout_plain(c) for row in R.expand(rules, words) for c in row if c is not None]
    raw = out.read_bytes()
    if gzip_level:
        raw = gzip.decompress(raw)
    got = raw.split(b"\n")[:-1]
    assert n == len(exp) and len(got) == len(exp)
    assert got == exp
    assert any(g.startswith(b"\x00\xffAb") for g in got) and any(g.startswith(b"$HEX[61620a6364") for g in got)


def test_crack_files_several_dictionaries(tmp_path):
    """help_crack passes a dictionary list (help_crack.py:520-552): plain and gz files are read in parallel, a
    last line without '\\n' is still a word, and every planted PSK is found whichever file holds it."""
    rng = random.Random(41)
    essid, ap, sta, an, sn = S.random_net(rng)
    alnum = b"abcdefghijklmnopqrstuvwxyz0123456789"
    files, lines, psks = [], [], []
    for f in range(3):
        words = [bytes(rng.choice(alnum) for _ in range(rng.randint(8, 16))) for _ in range(20000 + 5000 * f)]
        psk = words[-1] if f == 2 else words[rng.randrange(len(words))]
        psks.append(psk)
        a = rng.randbytes(6)
        lines.append(S.pmkid_line(psk, essid, a, sta) if f != 1 else
                     S.eapol_line(psk, essid, a, sta, an, sn, 2, f, "LE", rng=rng))
        body = b"\n".join(words) + (b"" if f == 2 else b"\n")  # file 2 ends without a newline
        path = tmp_path / (f"d{f}.txt" if f == 0 else f"d{f}.txt.gz")
        if f == 0:
            path.write_bytes(body)
        else:
            with gzip.open(path, "wb") as fh:
                fh.write(body)
        files.append(str(path))
    hf = tmp_path / "h.hash"
    hf.write_bytes(b"\n".join(lines) + b"\n")
    out = tmp_path / "o.key"
    assert dwpa_amd.crack_files(str(hf), files, None, 8, str(out), batch=1 << 14) == 0
    recs = out.read_bytes().strip().split(b"\n")
    assert sorted(r.rsplit(b":", 1)[1] for r in recs) == sorted(psks)


def test_crack_files_several_shard_workers(tmp_path, capfd, monkeypatch):
    """The multi-device client path (hashcat uses every GPU, help_crack.py:773) rehearsed on one GPU: two shard
    workers on device 0 (DWPA_CRACK_SHARDS_PER_DEVICE=2) pull dictionary items from one queue, each with its own
    scan, stager and streams.  Hits are planted in several items (so both workers find some), one PSK appears in
    two items (its line must be written exactly once, then retired everywhere), and a line whose PMKID is shorter
    than 16 bytes (never matches; hashcat would not load it) must not keep rc at 1."""
    monkeypatch.setenv("DWPA_CRACK_SHARDS_PER_DEVICE", "2")
    monkeypatch.setenv("DWPA_TRACE", "1")
    rng = random.Random(51)
    essid, ap, sta, an, sn = S.random_net(rng)
    alnum = b"abcdefghijklmnopqrstuvwxyz0123456789"
    n = 600_000
    words = [b"w%07d" % i + bytes(rng.choice(alnum) for _ in range(3)) for i in range(n)]
    where = [100, 20_000, 60_000, 200_000, 500_000, n - 1]
    lines, psks = [], []
    for k, i in enumerate(where):
        psks.append(words[i])
        a = rng.randbytes(6)
        lines.append(S.pmkid_line(words[i], essid, a, sta) if k % 2 else
                     S.eapol_line(words[i], essid, a, sta, an, sn, 2, k - 3, "LE", rng=rng))
    words[30_000] = words[100]  # the first line's PSK again, in a later item
    short = S.pmkid_line(b"never", essid, ap, sta).split(b"*")
    short[2] = short[2][:16]    # 8-byte PMKID: strncmp over 16 bytes never matches (common.php:186)
    lines.append(b"*".join(short))
    hf = tmp_path / "h.hash"
    hf.write_bytes(b"\n".join(lines) + b"\n")
    d = tmp_path / "d.txt.gz"
    with gzip.open(d, "wb", compresslevel=1) as f:
        f.write(b"\n".join(words) + b"\n")
    out = tmp_path / "o.key"
    assert dwpa_amd.crack_files(str(hf), [str(d)], None, 8, str(out), batch=1 << 14) == 0
    recs = out.read_bytes().strip().split(b"\n")
    assert len(recs) == len(where)
    assert sorted(r.rsplit(b":", 1)[1] for r in recs) == sorted(psks)
    assert len({r.split(b":")[1] for r in recs}) == len(where)  # one record per line (MAC_AP differs per line)
    err = capfd.readouterr().err
    workers = [l for l in err.splitlines() if "crack worker" in l]
    assert len(workers) == 2, err[-2000:]
    assert all(int(l.split(": ")[1].split(" items")[0]) > 0 for l in workers), workers


def test_crack_files_dictionary_cache_next_work_unit(tmp_path, capfd, monkeypatch):
    """Two work units over the same gz dictionary (help_crack keeps its dictionaries between work units,
    help_crack.py:520-552): the first reads the file to its end (nothing cracks: rc 1) and leaves it decoded in the
    process-wide DictCache; the second, against other nets, replays it from memory (the trace counts one more
    replayed file) and finds its planted PSKs, including the file's last word."""
    monkeypatch.setenv("DWPA_TRACE", "1")
    rng = random.Random(53)
    alnum = b"abcdefghijklmnopqrstuvwxyz0123456789"
    words = [b"u%06d" % i + bytes(rng.choice(alnum) for _ in range(4)) for i in range(150_000)]
    d = tmp_path / "dict.txt.gz"
    with gzip.open(d, "wb", compresslevel=1) as f:
        f.write(b"\n".join(words) + b"\n")

    def unit(name, lines):
        hf = tmp_path / (name + ".hash")
        hf.write_bytes(b"\n".join(lines) + b"\n")
        out = tmp_path / (name + ".key")
        rc = dwpa_amd.crack_files(str(hf), [str(d)], None, 8, str(out), batch=1 << 14)
        recs = out.read_bytes().strip().split(b"\n") if out.exists() and out.stat().st_size else []
        err = capfd.readouterr().err
        replayed = [int(l.split("cache: ")[1].split()[0]) for l in err.splitlines() if "dictionary cache" in l]
        return rc, recs, replayed[-1]

    essid, ap, sta, an, sn = S.random_net(rng)
    rc, recs, before = unit("u1", [S.pmkid_line(b"not-in-the-dictionary", essid, ap, sta)])
    assert rc == 1 and recs == []
    essid2, ap2, sta2, an2, sn2 = S.random_net(rng)
    psks = [words[70_001], words[-1]]
    lines = [S.pmkid_line(psks[0], essid2, ap2, sta2),
             S.eapol_line(psks[1], essid2, rng.randbytes(6), sta2, an2, sn2, 2, -2, "BE", rng=rng)]
    rc, recs, after = unit("u2", lines)
    assert rc == 0 and sorted(r.rsplit(b":", 1)[1] for r in recs) == sorted(psks)
    assert after == before + 1


def test_crack_files_degenerate_inputs(tmp_path):
    """Empty and ragged inputs of the client path, with hashcat's outcomes (help_crack.py:776-786): an empty plain
    or gzip dictionary, a dictionary of words outside 8..63 only, and no dictionary at all exhaust the work unit
    (rc 1, nothing written); a hash file that is empty or holds no valid line is hashcat's "No hashes loaded" (rc
    -1); the 8- and 63-byte PSKs at the filter's edges are found and the 64-byte word beside them is not
    (m22000 keys are 8..63 bytes, INSTALL.md:83); the check path returns [] for no jobs and False for no keys."""
    rng = random.Random(71)
    essid, ap, sta, an, sn = S.random_net(rng)
    good = S.pmkid_line(b"edge-psk-1", essid, ap, sta)
    hf = tmp_path / "h.hash"
    hf.write_bytes(good + b"\n")
    out = tmp_path / "o.key"

    def run(dicts, hfile=hf):
        if out.exists():
            out.unlink()
        rc = dwpa_amd.crack_files(str(hfile), [str(d) for d in dicts], None, 8, str(out))
        recs = out.read_bytes().strip().split(b"\n") if out.exists() and out.stat().st_size else []
        return rc, recs

    empty = tmp_path / "empty.txt"
    empty.write_bytes(b"")
    empty_gz = tmp_path / "empty.txt.gz"
    empty_gz.write_bytes(gzip.compress(b""))
    ragged = tmp_path / "ragged.txt"
    ragged.write_bytes(b"\n".join([b"", b"short", b"x" * 64, b"y" * 100, b"\r", b"1234567"]) + b"\n\n")
    assert run([empty]) == (1, [])
    assert run([empty_gz]) == (1, [])
    assert run([ragged]) == (1, [])
    assert run([]) == (1, [])
    bad = tmp_path / "bad.hash"
    bad.write_bytes(b"WPA*01*zz*aa*bb*cc***\nnot a hashline\n\n")
    assert run([ragged], bad)[0] == -1
    none = tmp_path / "none.hash"
    none.write_bytes(b"")
    assert run([ragged], none)[0] == -1
    # the filter's edges: 8 and 63 bytes are candidates, 7 and 64 are not
    p8, p63 = b"e" * 7 + b"8", bytes(rng.choice(b"abcdef0123") for _ in range(63))
    e2, ap2, sta2, an2, sn2 = S.random_net(rng)
    lines = [S.pmkid_line(p8, e2, ap2, sta2), S.pmkid_line(p63, e2, rng.randbytes(6), sta2),
             S.pmkid_line(p63 + b"z", e2, rng.randbytes(6), sta2), S.pmkid_line(p8[:7], e2, rng.randbytes(6), sta2)]
    hf2 = tmp_path / "edges.hash"
    hf2.write_bytes(b"\n".join(lines) + b"\n")
    edges = tmp_path / "edges.txt"
    edges.write_bytes(b"\n".join([p8[:7], p8, p63, p63 + b"z"]) + b"\n")
    rc, recs = run([edges], hf2)
    assert rc == 1 and sorted(r.rsplit(b":", 1)[1] for r in recs) == sorted([p8, p63])
    assert dwpa_amd.check_batch([]) == []
    assert dwpa_amd.check_key_m22000(good, []) is False
    assert dwpa_amd.check_key_m22000(good, [None]) is False


def test_crack_last_stats(tmp_path, capsys):
    """dwpa_crack_last_stats after an exhausted pass and a rules pass: every dictionary word read, candidates =
    the words (or word x rule outputs) inside 8..63, valid hashlines loaded, lines cracked; the drop-in prints
    them as hashcat's end-of-run block."""
    from dwpa_amd import m22000 as M
    from dwpa_amd.help_crack import run_cracker
    rng = random.Random(73)
    words = [S.random_psk(rng, 4, 70) for _ in range(5000)]
    essid, ap, sta, an, sn = S.random_net(rng)
    psk = next(w for w in words[3000:] if 8 <= len(w) <= 63)
    hf = tmp_path / "h.hash"
    hf.write_bytes(S.pmkid_line(psk, essid, ap, sta) + b"\n" + S.pmkid_line(b"not-there!", essid, ap, sta) +
                   b"\nWPA*01*bad\n")
    d = tmp_path / "d.txt"
    d.write_bytes(b"\n".join(words) + b"\n")
    out = tmp_path / "o.key"
    assert dwpa_amd.crack_files(str(hf), [str(d)], None, 8, str(out)) == 1
    st = M.crack_stats()
    assert st["words"] == len(words) and st["candidates"] == sum(1 for w in words if 8 <= len(w) <= 63)
    assert st["hashes"] == 2 and st["cracked"] == 1 and st["seconds"] > 0
    rules = ["", ":", "$1", "]", "'7", "d"]
    rf = tmp_path / "r.rule"
    rf.write_text("\n".join(rules[1:]) + "\n")
    out.unlink()
    assert dwpa_amd.crack_files(str(hf), [str(d)], str(rf), 8, str(out)) == 1
    exp = dwpa_amd.rules_expand("\n".join(rules[1:]), words)
    st = M.crack_stats()
    assert st["candidates"] == sum(1 for row in exp for c in row if c is not None and 8 <= len(c) <= 63)
    conf = {"hash_file": str(hf), "key_file": str(out), "rules": "", "coptions": ""}
    capsys.readouterr()
    assert run_cracker(conf, [str(d)], sleepy=lambda: None, pprint=lambda *a: None) == 1
    text = capsys.readouterr().out
    assert "Status...........: Exhausted" in text and "Recovered........: 1/2 (50.00%) Digests" in text


@pytest.mark.skipif(os.environ.get("DWPA_PBKDF2_ISSUE") == "1", reason="already the forced issue-pass run")
def test_issue_pass_kernels_at_small_sizes():
    """Launches of at most one wave per SIMD take the plain-schedule PBKDF2 kernel (pbkdf2_module.cpp), so the
    small parity cases above run it.  Re-run the PBKDF2-bearing ones with the issue-pass kernels forced
    (DWPA_PBKDF2_ISSUE=1), in a child process because the switch is read once per process."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sel = ("pbkdf2_vectors or pbkdf2_random_lengths or challenge_kat or mixed_golden_batch or random_batch_vs_oracle"
           " or scan_dictionary_hbm or scan_numeric_keyspace or scan_run_many_essids")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(root, "tests", "test_gpu_parity.py"), "-k", sel],
                       cwd=root, env=dict(os.environ, DWPA_PBKDF2_ISSUE="1"), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout


@pytest.mark.parametrize("exit_on", ["1", "0"])
def test_first_key_exit_across_chunks(exit_on):
    """the first-key early exit of the attempt-parallel verify (first_hit) across chunks and segments.
    Jobs at nc=128 (keyver 2 and 3, 261 attempts: attempt-parallel) whose PSK appears several times -- in one
    segment, in several segments, and in later chunks of the call (dwpa_init batch = 128 slots, so 300-key jobs span
    three chunks) -- with null keys in between: key_index is the first copy, and every result equals the CPU
    oracle's, with the early exit on (default) and off (DWPA_FIRST_KEY_EXIT=0; one process each, the switch is read
    once)."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, DWPA_FIRST_KEY_EXIT=exit_on)
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "first_key_child.py")], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["exit"] == exit_on
    assert res["got"] == res["exp"] == res["single"]
    assert res["key_index"] == res["first_copy"]
    assert res["key_index"][:4] == [20, 140, 5, 299] and res["got"][4] is False


def test_expand_rules_file_long_candidates_grow_the_text_buffer(tmp_path):
    """The wordlist text is packed on the GPU into a buffer budgeted at 24 bytes per candidate; candidates of 100-256
    bytes overflow it, and the sub-batch is packed again into a bigger one.  Output = the rule oracle's expansion,
    in order, with a '\\r' inside some candidates written as $HEX[]."""
    from dwpa_amd.help_crack import expand_rules
    rng = random.Random(33)
    words = [S.random_psk(rng, 90, 120) for _ in range(40000)]
    words[5] = b"x" * 50 + b"\r" + b"y" * 50
    rules = [":", "d", "f", "p2", "$\r $!", "] ] ]"]
    src = tmp_path / "source.txt"
    src.write_bytes(b"\n".join(b"$HEX[" + w.hex().encode() + b"]" if b"\r" in w else w for w in words) + b"\n")
    rf = tmp_path / "long.rule"
    rf.write_bytes("\n".join(rules).encode() + b"\n")
    out = tmp_path / "out.txt"
    n = expand_rules(str(rf), str(src), str(out))
    exp = [_stdout_plain(c) for row in R.expand(rules, words) for c in row if c is not None]
    got = out.read_bytes().split(b"\n")[:-1]
    assert n == len(exp) and got == exp
    ncap = (1 << 20) // len(rules) * len(rules)  # the sub-batch's candidate slots (all words fit in one)
    assert sum(len(e) + 1 for e in exp) > 24 * ncap  # the 24-bytes-per-slot budget was exceeded
