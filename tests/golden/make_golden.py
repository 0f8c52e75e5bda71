"""Regenerates tests/golden/*.json (committed fixtures; run from the repo root: python tests/golden/make_golden.py).

Every expected value is produced by the C oracle (oracle/m22000_oracle.c, OpenSSL) and cross-checked against the
independent pure-Python oracle (oracle/oracle.py) before it is written.  Sources of the inputs:

* kat.json      -- the reference's only known-answer test: help_crack/help_crack.py:690-699 (challenge lines, PSK
                   "aaaa1234"), plus the public PBKDF2/802.11i/CMAC vectors (RFC 6070, IEEE 802.11i-2004 H.4,
                   RFC 4493), each asserted here against both oracles.
* mixed.json    -- seeded synthetic C5-shaped set (PMKID + EAPOL keyver 1/2/3 with planted nonce corrections in
                   both endians, zero-PMK and PMK-reuse jobs) and the PHP edge cases of web/common.php:3-307.
"""
from __future__ import annotations

import hashlib
import hmac
import json
import os
import random
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from tests import synth as S  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def enc(v):
    if isinstance(v, bytes):
        return {"hex": v.hex()}
    if isinstance(v, list):
        return [enc(x) for x in v]
    return v


def both(line, keys, pmk=False, nc=128):
    r1 = O.c_check_key_m22000(line, keys, pmk, nc)
    r2 = O.py_check_key_m22000(line, keys, pmk, nc)
    assert r1 == r2, (line, r1, r2)
    return r1


def kat():
    out = {"challenge": [], "pbkdf2": [], "cmac": []}
    for line in S.CHALLENGE_LINES:
        r = both(line, [S.CHALLENGE_PSK])
        assert r and r[0] == S.CHALLENGE_PSK
        out["challenge"].append({"line": line.decode(), "keys": [S.CHALLENGE_PSK.hex()], "nc": 128, "expect": enc(r)})
    # hashcat's default window (--nonce-error-corrections=8, help_crack.py:773) also finds the EAPOL line
    r = both(S.CHALLENGE_LINES[1], [S.CHALLENGE_PSK], False, 8)
    assert r[1:3] == [4, "LE"]
    # RFC 6070 (PBKDF2-HMAC-SHA1) at c = 4096 and IEEE 802.11i-2004 H.4.1 (PSK = PBKDF2(pass, SSID, 4096, 32))
    vec = [
        (b"password", b"salt", 4096, "4b007901b765489abead49d926f721d065a429c1"),
        (b"passwordPASSWORDpassword", b"saltSALTsaltSALTsaltSALTsaltSALTsalt", 4096,
         "3d2eec4fe41c849b80c8d83662c0e44a8b291a964cf2f07038"),
        (b"pass\0word", b"sa\0lt", 4096, "56fa6aa75548099dcc37d7f03425e0c3"),
        (b"password", b"IEEE", 4096, "f42c6fc52df0ebef9ebb4b90b38a5f902e83fe1b135a70e23aed762e9710a12e"),
        (b"ThisIsAPassword", b"ThisIsASSID", 4096, "0dc0d6eb90555ed6419756b9a15ec3e3209b63df707dd508d14581f8982721af"),
        (b"a" * 32, b"Z" * 32, 4096, "becb93866bb8c3832cb777c2f559807c8c59afcb6eae734885001300a981cc62"),
    ]
    for p, s, c, dk in vec:
        n = len(dk) // 2
        got_c = O.c_pbkdf2(p, s, c, n).hex()
        got_py = hashlib.pbkdf2_hmac("sha1", p, s, c, n).hex()
        if got_c != dk or got_py != dk:
            print("dropping unverified vector", p, s, dk, got_c, file=sys.stderr)
            continue
        out["pbkdf2"].append({"password": p.hex(), "salt": s.hex(), "iterations": c, "dk": dk,
                              "pmk32": O.c_pbkdf2(p, s, 4096, 32).hex()})
    key = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")
    msgs = [("", "bb1d6929e95937287fa37d129b756746"),
            ("6bc1bee22e409f96e93d7e117393172a", "070a16b46b4d4144f79bdd9dd04a287c"),
            ("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e5130c81c46a35ce411",
             "dfa66747de9ae63030ca32611497c827"),
            ("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e5130c81c46a35ce411"
             "e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710", "51f0bebf7e3b9d92fc49741779363cfe")]
    for m, t in msgs:
        mb = bytes.fromhex(m)
        assert O.c_omac1_aes_128(mb, key).hex() == t and O.omac1_aes_128(mb, key).hex() == t
        out["cmac"].append({"key": key.hex(), "msg": m, "tag": t})
    return out


def short_anonce_line(psk, essid, ap, sta, snonce, anonce_short, keyver, keys_before, attempt_index, nc):
    """EAPOL line with a < 32-byte ANONCE (PHP grows $n by substr_replace clamping, common.php:255-259):
    the MIC is computed for the PRF message PHP hashes at `attempt_index` of key ordinal `keys_before`."""
    eapol_len = 121
    rng = random.Random(99)
    body = bytearray(eapol_len)
    body[0], body[1] = 2, 3
    struct.pack_into(">H", body, 2, eapol_len - 4)
    body[4] = 2
    struct.pack_into(">H", body, 5, 0x0108 | keyver)
    body[17:49] = snonce
    body[99:] = rng.randbytes(eapol_len - 99)
    eapol = bytes(body)
    m = ap + sta if O.php_strncmp(ap, sta, 6) < 0 else sta + ap
    if O.php_strncmp(snonce, anonce_short, 6) < 0:
        n, swap = snonce + anonce_short, False
    else:
        n, swap = anonce_short + snonce, True
    halfnc = (nc >> 1) + 1
    order = [("N", 0)] + [x for k in range(1, halfnc + 1) for x in (("V", k), ("V", -k), ("N", k), ("N", -k))]
    msgs = []
    for _q in range(keys_before + 1):
        for e, off in order:
            raw = struct.pack(">I" if e == "N" else "<I", off & 0xFFFFFFFF)  # corr = 0 (unpack fails)
            n = O.substr_replace(n, raw, 28 if swap else 60, 4)
            msgs.append(n)
    nn = msgs[keys_before * len(order) + attempt_index]
    p = hashlib.pbkdf2_hmac("sha1", psk, essid, 4096, 32)
    ptk = hmac.new(p, b"Pairwise key expansion\0" + m + nn + b"\0", hashlib.sha1).digest()
    mic = hmac.new(ptk[:16], eapol, hashlib.md5 if keyver == 1 else hashlib.sha1).digest()[:16]
    return b"WPA*02*%s*%s*%s*%s*%s*%s*00" % (mic.hex().encode(), ap.hex().encode(), sta.hex().encode(),
                                             essid.hex().encode(), anonce_short.hex().encode(), eapol.hex().encode())


def mixed():
    rng = random.Random(5)
    jobs = []

    def add(line, keys, pmk=False, nc=128, tag=""):
        r = both(line, keys, pmk, nc)
        jobs.append({"tag": tag, "line": line.decode("latin-1"),
                     "keys": [None if k is None else k.hex() for k in keys],
                     "pmk": pmk.hex() if pmk else None, "nc": nc, "expect": enc(r)})

    # C5-shaped: PMKID + keyver 1/2/3, planted corrections in {0, +-1..+-8} x {LE, BE}
    for kind in ("pmkid", 1, 2, 3):
        for i in range(10):
            essid, ap, sta, an, sn = S.random_net(rng)
            psk = S.random_psk(rng)
            decoys = [S.random_psk(rng) for _ in range(rng.randint(0, 3))]
            keys = decoys + [psk] + [S.random_psk(rng)]
            if kind == "pmkid":
                line = S.pmkid_line(psk, essid, ap, sta)
            else:
                nc = rng.randint(-8, 8)
                line = S.eapol_line(psk, essid, ap, sta, an, sn, kind, nc, rng.choice(["LE", "BE"]), rng=rng)
            add(line, keys, tag=f"c5-{kind}")
    # a miss, and the PHP default window edge (+-65 found, +-66 not)
    essid, ap, sta, an, sn = S.random_net(rng)
    psk = S.random_psk(rng)
    add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 65, "BE", rng=rng), [psk], tag="nc-edge-65")
    add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, -66, "LE", rng=rng), [psk], tag="nc-edge-66-miss")
    add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 3, "LE", rng=rng), [psk], nc=4, tag="nc4-3")
    add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 4, "LE", rng=rng), [psk], nc=4, tag="nc4-4-miss")
    add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 0, "LE", rng=rng), [psk], nc=-2, tag="nc-neg")
    add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 1, "LE", rng=rng), [psk], nc=-2, tag="nc-neg-miss")
    # zero PMK (submission, common.php:592) and PMK reuse (:606, :919)
    zpmk = b"\0" * 32
    essid, ap, sta, an, sn = S.random_net(rng)
    add(S.pmkid_line(b"", essid, ap, sta, the_pmk=zpmk), [b""], zpmk, tag="zero-pmk-pmkid")
    add(S.eapol_line(b"", essid, ap, sta, an, sn, 2, 0, "LE", the_pmk=zpmk, rng=rng), [b""], zpmk, tag="zero-pmk-eapol")
    psk = S.random_psk(rng)
    real = S.pmk(psk, essid)
    line = S.eapol_line(psk, essid, ap, sta, an, sn, 3, -7, "BE", rng=rng)
    add(line, [b""], real, abs(-7) * 2 + 128, tag="pmk-propagate")
    add(line, [b"nope-nope", psk], real, 15, tag="pmk-first-key-only")  # PMK applies to the first key only
    add(line, [None, b"zzzzzzzz"], real, 15, tag="pmk-null-skipped")  # null keys keep the PMK for the next key
    # $HEX[] keys (common.php:3-25) and key lengths 0/64/65/100 (HMAC long-key path)
    for psk in [b"p\x00ss:w\xffrd!", b"x" * 64, b"y" * 65, bytes(range(1, 101)), b"", b"ab"]:
        essid, ap, sta, an, sn = S.random_net(rng)
        line = S.pmkid_line(psk, essid, ap, sta)
        add(line, [b"$HEX[" + psk.hex().encode() + b"]" if psk else b"$HEX[]", psk], tag="hexkey")
    essid, ap, sta, an, sn = S.random_net(rng)
    add(S.pmkid_line(b"$HEX[4142]", essid, ap, sta), [b"$HEX[4142]", b"AB"], tag="hex-decoded-not-literal")
    add(S.pmkid_line(b"$HEX[414]", essid, ap, sta), [b"$HEX[414]"], tag="hex-odd-literal")
    add(S.pmkid_line(b"$HEX[]", essid, ap, sta), [b"$HEX[]"], tag="hex-empty-literal")
    add(S.pmkid_line(b"$HEX[4G]", essid, ap, sta), [b"$HEX[4G]"], tag="hex-bad-literal")
    add(S.pmkid_line(b"\xab\xcd", essid, ap, sta), [b"$HEX[ABCD]"], tag="hex-upper")
    # parser edge cases (common.php:157-195)
    psk = b"edgecase1"
    essid, ap, sta, an, sn = S.random_net(rng)
    base = S.pmkid_line(psk, essid, ap, sta)
    f = base.split(b"*")
    for t in [b"1", b" 1", b"1 ", b"01.0", b"+1", b"1e0", b"0x1", b"001", b"1.", b".1e1", b"2", b"03", b""]:
        add(b"*".join([f[0], t] + f[2:]), [psk], tag=f"type-{t!r}")
    add(base.upper().replace(b"WPA", b"WPA", 1).replace(b"*01*", b"*01*"), [psk], tag="upper-hex-sig")
    add(b"WPA*01*" + f[2].upper() + b"*" + f[3].upper() + b"*" + f[4] + b"*" + f[5] + b"***", [psk], tag="upper-hex")
    add(b"WPA*01*" + f[2] + b"*" + f[3] + b"*" + f[4] + b"**" + b"**", [psk], tag="empty-essid")
    add(b"WPA*01*" + f[2][:30] + b"*" + f[3] + b"*" + f[4] + b"*" + f[5] + b"***", [psk], tag="short-pmkid")
    add(b"WPA*01*" + f[2] + b"00ff*" + f[3] + b"*" + f[4] + b"*" + f[5] + b"***", [psk], tag="long-pmkid")
    add(b"WPA*01*" + f[2] + b"*" + f[3] + b"*" + f[4] + b"*" + f[5] + b"*x*y*z*w", [psk], tag="explode-limit")
    add(b"WPA*01*" + f[2] + b"*" + f[3] + b"*" + f[4] + b"*" + f[5] + b"**", [psk], tag="8-fields")
    add(b"wpa*01*" + b"*".join(f[2:]), [psk], tag="bad-sig")
    add(b"WPA*01*" + f[2] + b"*" + f[3][:-1] + b"*" + f[4] + b"*" + f[5] + b"***", [psk], tag="odd-mac")
    # non-6-byte MACs and a 2-block ESSID salt
    for apl, stal, el in [(4, 8, 12), (6, 6, 60), (0 + 2, 6, 33), (7, 7, 52)]:
        essid, ap, sta, an, sn = S.random_net(rng, essid_len=min(el, 32))
        essid = (essid * 3)[:el]
        ap, sta = rng.randbytes(apl), rng.randbytes(stal)
        psk = S.random_psk(rng)
        add(S.pmkid_line(psk, essid, ap, sta), [psk], tag=f"macs-{apl}-{stal}-essid{el}")
        add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 2, "BE", rng=rng), [psk], nc=8, tag=f"eapol-macs-{apl}-{stal}-{el}")
    # EAPOL frame edge cases
    essid, ap, sta, an, sn = S.random_net(rng)
    psk = S.random_psk(rng)
    good = S.eapol_line(psk, essid, ap, sta, an, sn, 2, 0, "LE", rng=rng)
    g = good.split(b"*")
    add(b"*".join(g[:7] + [g[7][:96]] + g[8:]), [psk], tag="eapol-48-bytes")
    kv0 = bytearray(bytes.fromhex(g[7].decode()))
    kv0[6] &= 0xFC
    add(b"*".join(g[:7] + [kv0.hex().encode()] + g[8:]), [psk], tag="keyver0")
    add(b"*".join(g[:8] + [b"0"]), [psk], tag="bad-mp")
    add(b"*".join(g[:8] + [b"*"]), [psk], tag="star-mp")
    add(b"*".join(g[:2] + [g[2][:20]] + g[3:]), [psk], tag="short-mic")
    for el in (128, 129, 160, 250):  # CMAC complete / partial last block
        essid, ap, sta, an, sn = S.random_net(rng)
        psk = S.random_psk(rng)
        add(S.eapol_line(psk, essid, ap, sta, an, sn, 3, 1, "LE", eapol_len=el, rng=rng), [psk], nc=8, tag=f"kv3-len{el}")
        add(S.eapol_line(psk, essid, ap, sta, an, sn, 1, -1, "BE", eapol_len=el, rng=rng), [psk], nc=8, tag=f"kv1-len{el}")
    # swap/no-swap nonce order both ways and an ANONCE longer than 32 bytes
    for i in range(4):
        essid, ap, sta, an, sn = S.random_net(rng)
        psk = S.random_psk(rng)
        if i % 2:
            an, sn = bytes([0]) + an[1:], bytes([255]) + sn[1:]
        else:
            an, sn = bytes([255]) + an[1:], bytes([0]) + sn[1:]
        add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 1 + i, "LE", rng=rng), [psk], nc=16, tag=f"order-{i}")
    # short ANONCE: $n grows under substr_replace clamping, across attempts and keys (common.php:255-259)
    for (anlen, keys_before, att, nc) in [(20, 0, 0, 4), (20, 0, 3, 4), (20, 1, 2, 4), (20, 2, 0, 0), (29, 0, 1, 2),
                                          (29, 1, 0, 2), (10, 3, 0, -2)]:
        essid, ap, sta, an, sn = S.random_net(rng)
        sn = bytes([0]) + sn[1:]
        an = bytes([255]) + an[1:anlen]
        psk = S.random_psk(rng)
        line = short_anonce_line(psk, essid, ap, sta, sn, an, 2, keys_before, att, nc)
        keys = [S.random_psk(rng) for _ in range(keys_before)] + [psk]
        add(line, keys, nc=nc, tag=f"short-anonce-{anlen}-{keys_before}-{att}-{nc}")
        add(line, [None] + keys, nc=nc, tag=f"short-anonce-null-{anlen}-{keys_before}-{att}")
    # duplicated keys and matching key positions
    essid, ap, sta, an, sn = S.random_net(rng)
    psk = S.random_psk(rng)
    line = S.eapol_line(psk, essid, ap, sta, an, sn, 2, -3, "LE", rng=rng)
    add(line, [psk, psk], nc=8, tag="dup-keys")
    add(line, [], nc=8, tag="no-keys")
    add(line, [None, None], nc=8, tag="null-keys")
    # short ANONCE with wide windows (>= 64 attempts per list): the attempt-parallel verify with explicit per-key
    # lists, the winning attempt past the first 64 lanes and the key past the first list
    for (anlen, keys_before, att, nc, kv) in [(20, 2, 40, 32, 2), (29, 1, 100, 128, 2), (20, 3, 200, 128, 2),
                                              (20, 1, 70, 128, 1)]:
        essid, ap, sta, an, sn = S.random_net(rng)
        sn = bytes([0]) + sn[1:]
        an = bytes([255]) + an[1:anlen]
        psk = S.random_psk(rng)
        line = short_anonce_line(psk, essid, ap, sta, sn, an, kv, keys_before, att, nc)
        keys = [S.random_psk(rng) for _ in range(keys_before)] + [psk, S.random_psk(rng)]
        add(line, keys, nc=nc, tag=f"short-anonce-wide-{anlen}-{keys_before}-{att}-{nc}-kv{kv}")
    return {"jobs": jobs}


def nc_windows():
    """The nonce windows of check_key_m22000's real call sites (common.php:250-300, halfnc = (nc>>1)+1):
    put_work's PMK propagation nc = |nc|*2+128 (:919; |nc| = 65 -> 258, halfnc 130, 521 attempts), submission's
    (|nc|<<1)+1 (:606; 131, halfnc 66), odd and negative windows.  Hits are planted at +-halfnc in both endians
    (inside) and one past it (outside), at the first (N+0) and last (N-halfnc) attempt of a 521-attempt list, behind
    hundreds of keys (attempt-parallel verify, items past the first waves), with a caller PMK, and with short
    ANONCEs whose $n grows (explicit per-key lists at 521 attempts)."""
    rng = random.Random(258)
    jobs = []

    def add(line, keys, pmk=False, nc=128, tag=""):
        r = both(line, keys, pmk, nc)
        jobs.append({"tag": tag, "line": line.decode("latin-1"),
                     "keys": [None if k is None else k.hex() for k in keys],
                     "pmk": pmk.hex() if pmk else None, "nc": nc, "expect": enc(r)})
        return r

    for nc in (258, 131, 17, 1):
        half = (nc >> 1) + 1
        for kv in (1, 2, 3):
            for off, endian in ((half, "LE"), (-half, "LE"), (half, "BE"), (-half, "BE"), (half + 1, "LE"),
                                (-half - 1, "BE")):
                essid, ap, sta, an, sn = S.random_net(rng)
                psk = S.random_psk(rng)
                keys = [S.random_psk(rng) for _ in range(rng.randint(0, 2))] + [psk]
                r = add(S.eapol_line(psk, essid, ap, sta, an, sn, kv, off, endian, rng=rng), keys, nc=nc,
                        tag=f"nc{nc}-kv{kv}-{endian}{off:+d}")
                assert bool(r) == (abs(off) <= half), (nc, off, r)
    # first attempt (N+0) and last attempt (N-130) of a 521-attempt list, the key behind 300 (keyver 1/2) or
    # 40 (keyver 3: the pure-Python cross-check's AES is slow) other keys
    for kv, nkeys in ((1, 300), (2, 300), (3, 40)):
        for off, endian in ((0, "BE"), (-130, "BE"), (130, "LE")):
            essid, ap, sta, an, sn = S.random_net(rng)
            psk = S.random_psk(rng)
            keys = [S.random_psk(rng) for _ in range(nkeys)] + [psk]
            r = add(S.eapol_line(psk, essid, ap, sta, an, sn, kv, off, endian, rng=rng), keys, nc=258,
                    tag=f"nc258-last-key-kv{kv}-{endian}{off:+d}")
            assert r and r[0] == psk
    # negative windows: only N+0 is tried ((nc>>1)+1 <= 0)
    for nc in (-1, -3, -258):
        essid, ap, sta, an, sn = S.random_net(rng)
        psk = S.random_psk(rng)
        assert add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 0, "LE", rng=rng), [psk], nc=nc, tag=f"nc{nc}-0")
        assert not add(S.eapol_line(psk, essid, ap, sta, an, sn, 2, 1, "BE", rng=rng), [psk], nc=nc,
                       tag=f"nc{nc}-1-miss")
    # PMK propagation itself (:919): caller PMK, key '', nc = |-65|*2+128
    essid, ap, sta, an, sn = S.random_net(rng)
    psk = S.random_psk(rng)
    real = S.pmk(psk, essid)
    for kv in (1, 2, 3):
        line = S.eapol_line(psk, essid, rng.randbytes(6), sta, rng.randbytes(32), rng.randbytes(32), kv, -65, "BE",
                            rng=rng)
        assert add(line, [b""], real, abs(-65) * 2 + 128, tag=f"pmk-propagate-258-kv{kv}")
        assert not add(line, [b""], real, abs(-32) * 2 + 1, tag=f"pmk-submission-65-kv{kv}-miss")
    # short ANONCE at 521 attempts: $n grows, explicit lists; winning attempt late in the list, behind a key
    for (anlen, keys_before, att, kv) in [(20, 1, 520, 2), (29, 0, 259, 1), (20, 2, 300, 2), (10, 1, 0, 1)]:
        essid, ap, sta, an, sn = S.random_net(rng)
        sn = bytes([0]) + sn[1:]
        an = bytes([255]) + an[1:anlen]
        psk = S.random_psk(rng)
        line = short_anonce_line(psk, essid, ap, sta, sn, an, kv, keys_before, att, 258)
        keys = [S.random_psk(rng) for _ in range(keys_before)] + [psk, S.random_psk(rng)]
        assert add(line, keys, nc=258, tag=f"short-anonce-258-{anlen}-{keys_before}-{att}-kv{kv}")
    return {"jobs": jobs}


def main():
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat(), f, indent=1)
    with open(os.path.join(HERE, "mixed.json"), "w") as f:
        json.dump(mixed(), f, indent=0)
    with open(os.path.join(HERE, "nc_windows.json"), "w") as f:
        json.dump(nc_windows(), f, indent=0)
    print("ok")


if __name__ == "__main__":
    main()
