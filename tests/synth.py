"""Synthetic m22000 hashlines with a known PSK (the role hcxpcapngtool plays for real captures).

Builds PMKID (WPA*01) and EAPOL (WPA*02, keyver 1/2/3) lines whose stored ANONCE differs from the one that
produced the MIC by a planted nonce-error-correction offset, so a correct checker must report exactly
``[psk, nc, endian, pmk]`` (web/common.php:280-288).  Uses Python's hashlib/hmac and libcrypto's AES-128
(via ctypes) -- a data generator for tests and bench.py, not part of the GPU path.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import hashlib
import hmac
import random
import struct

_crypto = None


def _aes_ecb(key: bytes, block: bytes) -> bytes:
    global _crypto
    if _crypto is None:
        _crypto = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
        _crypto.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        _crypto.EVP_aes_128_ecb.restype = ctypes.c_void_p
        _crypto.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p] * 5
        _crypto.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _crypto.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                              ctypes.c_char_p, ctypes.c_int]
        _crypto.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
    ctx = _crypto.EVP_CIPHER_CTX_new()
    _crypto.EVP_EncryptInit_ex(ctx, _crypto.EVP_aes_128_ecb(), None, key, None)
    _crypto.EVP_CIPHER_CTX_set_padding(ctx, 0)
    out = ctypes.create_string_buffer(32)
    ol = ctypes.c_int(0)
    _crypto.EVP_EncryptUpdate(ctx, out, ctypes.byref(ol), block, 16)
    _crypto.EVP_CIPHER_CTX_free(ctx)
    return out.raw[:16]


def aes_cmac(key: bytes, msg: bytes) -> bytes:
    """RFC 4493."""
    def dbl(b):
        v = int.from_bytes(b, "big") << 1
        if v >> 128:
            v ^= 0x87
        return (v & ((1 << 128) - 1)).to_bytes(16, "big")
    L = _aes_ecb(key, b"\0" * 16)
    k1 = dbl(L)
    k2 = dbl(k1)
    blocks = [msg[i:i + 16] for i in range(0, len(msg), 16)] or [b""]
    last = blocks[-1]
    if len(last) == 16:
        last = bytes(a ^ b for a, b in zip(last, k1))
    else:
        last = bytes(a ^ b for a, b in zip(last + b"\x80" + b"\0" * (15 - len(last)), k2))
    blocks[-1] = last
    c = b"\0" * 16
    for b in blocks:
        c = _aes_ecb(key, bytes(x ^ y for x, y in zip(c, b)))
    return c


def pmk(psk: bytes, essid: bytes) -> bytes:
    return hashlib.pbkdf2_hmac("sha1", psk, essid, 4096, 32)


def pmkid_line(psk: bytes, essid: bytes, ap: bytes, sta: bytes, the_pmk: bytes | None = None) -> bytes:
    p = the_pmk or pmk(psk, essid)
    pid = hmac.new(p, b"PMK Name" + ap + sta, hashlib.sha1).digest()[:16]
    return b"WPA*01*%s*%s*%s*%s***" % (pid.hex().encode(), ap.hex().encode(), sta.hex().encode(), essid.hex().encode())


def _cmp6(a: bytes, b: bytes) -> int:
    x, y = a[:6], b[:6]
    return (x > y) - (x < y) if x != y else (min(6, len(a)) > min(6, len(b))) - (min(6, len(a)) < min(6, len(b)))


def eapol_line(psk: bytes, essid: bytes, ap: bytes, sta: bytes, anonce: bytes, snonce: bytes, keyver: int,
               nc: int = 0, endian: str = "LE", mp: int = 0x00, eapol_len: int = 121, the_pmk: bytes | None = None,
               rng: random.Random | None = None) -> bytes:
    """EAPOL line whose MIC verifies at correction `nc` (`endian` 'LE'=V / 'BE'=N) of the stored ANONCE."""
    rng = rng or random.Random(0)
    assert len(anonce) == 32 and len(snonce) == 32 and eapol_len >= 99
    key_info = (0x0100 | 0x0008 | keyver) & 0xFFFF
    body = bytearray(eapol_len)
    body[0], body[1] = 0x01 if keyver < 3 else 0x02, 0x03
    struct.pack_into(">H", body, 2, eapol_len - 4)
    body[4] = 0x02 if keyver != 1 else 0xFE
    struct.pack_into(">H", body, 5, key_info)
    struct.pack_into(">H", body, 7, 16 if keyver != 1 else 32)
    body[9:17] = rng.randbytes(8)
    body[17:49] = snonce
    # IV/RSC/ID stay zero, MIC (81..96) zero as stored in m22000, key data after 99
    struct.pack_into(">H", body, 97, eapol_len - 99)
    body[99:] = rng.randbytes(eapol_len - 99)
    eapol = bytes(body)
    p = the_pmk or pmk(psk, essid)
    m = ap + sta if _cmp6(ap, sta) < 0 else sta + ap
    fmt = "<I" if endian == "LE" else ">I"
    stored = struct.unpack(fmt, anonce[28:32])[0]
    true_anonce = anonce[:28] + struct.pack(fmt, (stored + nc) & 0xFFFFFFFF)
    n = snonce + true_anonce if _cmp6(snonce, anonce) < 0 else true_anonce + snonce
    if keyver in (1, 2):
        ptk = hmac.new(p, b"Pairwise key expansion\0" + m + n + b"\0", hashlib.sha1).digest()
        mic = hmac.new(ptk[:16], eapol, hashlib.md5 if keyver == 1 else hashlib.sha1).digest()[:16]
    else:
        ptk = hmac.new(p, b"\x01\x00Pairwise key expansion" + m + n + b"\x80\x01", hashlib.sha256).digest()
        mic = aes_cmac(ptk[:16], eapol)
    return b"WPA*02*%s*%s*%s*%s*%s*%s*%02x" % (mic.hex().encode(), ap.hex().encode(), sta.hex().encode(),
                                                essid.hex().encode(), anonce.hex().encode(), eapol.hex().encode(), mp)


def random_net(rng: random.Random, essid_len: int | None = None):
    essid_len = essid_len or rng.randint(1, 32)
    essid = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_ ") for _ in range(essid_len))
    return essid, rng.randbytes(6), rng.randbytes(6), rng.randbytes(32), rng.randbytes(32)


def random_psk(rng: random.Random, lo: int = 8, hi: int = 63) -> bytes:
    n = rng.randint(lo, hi)
    return bytes(rng.randint(0x20, 0x7E) for _ in range(n))


# The reference's own known-answer test (help_crack/help_crack.py:690-699): PSK "aaaa1234", ESSID "dlink".
CHALLENGE_PSK = b"aaaa1234"
CHALLENGE_LINES = [
    b"WPA*01*8ac36b891edca8eef49094b1afe061ac*1c7ee5e2f2d0*0026c72e4900*646c696e6b***",
    b"WPA*02*269a61ef25e135a4b423832ec4ecc7f4*1c7ee5e2f2d0*0026c72e4900*646c696e6b*"
    b"dbd249a3e9cec6ced3360fba3fae9ba4aa6ec6c76105796ff6b5a209d18782ca*"
    b"0103007702010a00000000000000000000645b1f684a2566e21266f123abc386"
    b"cc576f593e6dc5e3823a32fbd4af929f51000000000000000000000000000000"
    b"0000000000000000000000000000000000000000000000000000000000000000"
    b"00001830160100000fac020100000fac040100000fac023c000000*00",
]


def fast_psk(rng: random.Random, lo: int = 8, hi: int = 63) -> bytes:
    """Printable-ASCII PSK, length U[lo, hi] (same distribution family as random_psk, cheaper to draw in bulk)."""
    return bytes(0x20 + b % 95 for b in rng.randbytes(rng.randint(lo, hi)))


def c1_workload(seed: int = 0, n: int = 10_000):
    """BASELINE configs[0] / SURVEY.md 8(d) C1: n PSKs (length U[8,63], printable, ~1 % `$HEX[..]`) against one
    PMKID line (ESSID 10 B, random MACs, seed 1); the true PSK is the last key.  Returns (line, keys, psk)."""
    rng = random.Random(seed)
    keys = []
    for _ in range(n):
        k = fast_psk(rng)
        if rng.random() < 0.01:
            k = b"$HEX[" + k.hex().encode() + b"]"
        keys.append(k)
    net = random.Random(1)
    essid, ap, sta, _, _ = random_net(net, essid_len=10)
    psk = keys[-1]
    raw = bytes.fromhex(psk[5:-1].decode()) if psk.startswith(b"$HEX[") else psk
    return pmkid_line(raw, essid, ap, sta), keys, raw


def c5_jobs(seed: int = 5, per_kind: int = 250, keys_per_job: int = 202, essids: int = 200, nc: int = 128,
            hit_rate: float = 0.9, zero_pmk: int = 10):
    """The C5 batch (see c5_plan) without the planted indices."""
    return c5_plan(seed, per_kind, keys_per_job, essids, nc, hit_rate, zero_pmk)[0]


def c5_plan(seed: int = 5, per_kind: int = 250, keys_per_job: int = 202, essids: int = 200, nc: int = 128,
            hit_rate: float = 0.9, zero_pmk: int = 10):
    """per_kind PMKID + keyver 1/2/3 EAPOL lines (nonce offsets uniform in {0, +-1..+-8} x
    {LE, BE}) plus zero_pmk zero-PMK jobs (common.php:592), keys_per_job candidates per job (the put_work cap,
    common.php:937), the true PSK planted at a random index in hit_rate of the jobs.  ESSIDs are drawn from a
    pool of `essids` networks so the batch path groups lines.  Returns ([(line, keys, pmk, nc)], plants) where
    plants[i] is the index of job i's planted key (None: no key of the job was planted, the job must miss)."""
    rng = random.Random(seed)
    nets = [random_net(rng) for _ in range(essids)]
    jobs, plants = [], []
    for kind in ("pmkid", 1, 2, 3):
        for _ in range(per_kind):
            essid, ap, sta, an, sn = nets[rng.randrange(essids)]
            ap, sta = rng.randbytes(6), rng.randbytes(6)
            psk = fast_psk(rng)
            if kind == "pmkid":
                line = pmkid_line(psk, essid, ap, sta)
            else:
                line = eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), kind,
                                  rng.randint(-8, 8), rng.choice(["LE", "BE"]), mp=rng.choice([0, 0x80, 0x02]),
                                  eapol_len=rng.choice([121, 123, 151, 187]), rng=rng)
            keys = [fast_psk(rng) for _ in range(keys_per_job - 1)]
            if rng.random() < hit_rate:
                keys.insert(rng.randrange(keys_per_job), psk)
                plants.append(keys.index(psk))
            else:
                keys.append(fast_psk(rng))
                plants.append(None)
            jobs.append((line, keys, False, nc))
    zpmk = b"\0" * 32
    for i in range(zero_pmk):
        essid, ap, sta, an, sn = nets[rng.randrange(essids)]
        if i % 2:
            line = pmkid_line(b"", essid, ap, sta, the_pmk=zpmk)
        else:
            line = eapol_line(b"", essid, ap, sta, rng.randbytes(32), rng.randbytes(32), 2 + i % 4 // 2,
                              rng.randint(-8, 8), "BE", the_pmk=zpmk, rng=rng)
        jobs.append((line, [b""], zpmk, nc))
        plants.append(0)
    return jobs, plants
