"""TEST INFRASTRUCTURE ONLY -- the parity oracle.  Never imported by the product path.

Two independent CPU restatements of dwpa's PHP key check (/root/reference/web/common.php):

* ``C``: ctypes binding of ``oracle/build/liboracle22000.so`` (m22000_oracle.c: OpenSSL, same library
  PHP's openssl_pbkdf2/hash_hmac/openssl_encrypt use).
* ``py_check_key_m22000``: a pure-Python restatement (hashlib PBKDF2/HMAC + a from-scratch AES-128),
  written separately so the two cross-check each other.

Both return PHP's shape: ``False`` or ``[psk_bytes, nc, endian, pmk_bytes]`` where ``nc`` is ``None`` for
PMKID lines (common.php:186) and ``endian`` is ``None``/``'BE'``/``'LE'`` (common.php:280-288).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes
import hashlib
import hmac
import os
import re
import struct
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle22000.so")


# --------------------------------------------------------------------------------------------
# PHP helpers (common.php:3-36) -- pure Python
# --------------------------------------------------------------------------------------------
_XD = re.compile(rb"\A[0-9a-fA-F]+\Z")


def valid_hex(s: bytes) -> bool:
    """common.php:28-36 (ctype_xdigit('') is false)."""
    return len(s) % 2 == 0 and bool(_XD.match(s))


def hc_unhex(key: bytes) -> bytes:
    """common.php:3-25."""
    if len(key) <= 6:
        return key
    k = key[5:-1]
    if len(k) % 2 == 0 and key.startswith(b"$HEX[") and key.endswith(b"]") and _XD.match(k):
        return bytes.fromhex(k.decode())
    return key


_WS = b" \t\n\r\x0b\x0c"
_NUM = re.compile(rb"\A[ \t\n\r\x0b\x0c]*([+-]?(?:[0-9]+(?:\.[0-9]*)?|\.[0-9]+)(?:[eE][+-]?[0-9]+)?)[ \t\n\r\x0b\x0c]*\Z")


def php_eq_type(s: bytes, target: int) -> bool:
    """PHP 8 loose ``$s == '0N'`` (both strings; numeric strings compare numerically)."""
    m = _NUM.match(s)
    if m:
        try:
            return float(m.group(1)) == float(target)
        except OverflowError:  # pragma: no cover
            return False
    return s == b"0%d" % target


def php_strncmp(a: bytes, b: bytes, n: int) -> int:
    m = min(n, len(a), len(b))
    if a[:m] != b[:m]:
        return -1 if a[:m] < b[:m] else 1
    ma, mb = min(n, len(a)), min(n, len(b))
    return (ma > mb) - (ma < mb)


def substr_replace(s: bytes, r: bytes, off: int, ln: int) -> bytes:
    if off > len(s):
        off = len(s)
    if off + ln > len(s):
        ln = len(s) - off
    return s[:off] + r + s[off + ln:]


# --------------------------------------------------------------------------------------------
# AES-128 (FIPS-197) from scratch, for the CMAC restatement (common.php:56-112)
# --------------------------------------------------------------------------------------------
def _xt(a):
    a <<= 1
    return (a ^ 0x11B) & 0xFF if a & 0x100 else a


def _build_sbox():
    # multiplicative inverse via exp/log tables on generator 3, then the affine map
    exp, log = [0] * 256, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x ^= _xt(x)
    sbox = [0] * 256
    for a in range(256):
        inv = 0 if a == 0 else exp[(255 - log[a]) % 255]
        s = inv
        for k in range(1, 5):
            s ^= ((inv << k) | (inv >> (8 - k))) & 0xFF
        sbox[a] = s ^ 0x63
    return sbox


SBOX = _build_sbox()


def aes128_encrypt_block(key: bytes, block: bytes) -> bytes:
    rk = list(key)
    rcon = 1
    w = [list(key[i:i + 4]) for i in range(0, 16, 4)]
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = t[1:] + t[:1]
            t = [SBOX[b] for b in t]
            t[0] ^= rcon
            rcon = _xt(rcon)
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    rk = [sum(w[4 * r:4 * r + 4], []) for r in range(11)]
    s = [block[i] ^ rk[0][i] for i in range(16)]
    for r in range(1, 11):
        s = [SBOX[b] for b in s]
        # ShiftRows (state is column-major: s[4*c + row])
        s = [s[(4 * ((c + row) % 4)) + row] for c in range(4) for row in range(4)]
        if r != 10:
            ns = []
            for c in range(4):
                a0, a1, a2, a3 = s[4 * c:4 * c + 4]
                ns += [_xt(a0) ^ _xt(a1) ^ a1 ^ a2 ^ a3,
                       a0 ^ _xt(a1) ^ _xt(a2) ^ a2 ^ a3,
                       a0 ^ a1 ^ _xt(a2) ^ _xt(a3) ^ a3,
                       _xt(a0) ^ a0 ^ a1 ^ a2 ^ _xt(a3)]
            s = ns
        s = [s[i] ^ rk[r][i] for i in range(16)]
    return bytes(s)


def _lshift1(b: bytes) -> bytes:
    v = (int.from_bytes(b, "big") << 1) & ((1 << 128) - 1)
    return v.to_bytes(16, "big")


def omac1_aes_128(data: bytes, key: bytes) -> bytes:
    """common.php:72-112 (PHP str_split: '' -> [''] here, matching the C oracle)."""
    rval = b"\0" * 15 + b"\x87"
    lval = aes128_encrypt_block(key, b"\0" * 16)
    k0 = _lshift1(lval)
    if lval[0] > 127:
        k0 = bytes(x ^ y for x, y in zip(k0, rval))
    k1 = _lshift1(k0)
    if k0[0] > 127:
        k1 = bytes(x ^ y for x, y in zip(k1, rval))
    blocks = [data[i:i + 16] for i in range(0, len(data), 16)] or [b""]
    last = blocks[-1]
    if len(last) != 16:
        last = last + b"\x80" + b"\0" * (15 - len(last))
        last = bytes(x ^ y for x, y in zip(last, k1))
    else:
        last = bytes(x ^ y for x, y in zip(last, k0))
    blocks[-1] = last
    c = b"\0" * 16
    for blk in blocks:
        c = aes128_encrypt_block(key, bytes(x ^ y for x, y in zip(c, blk)))
    return c


def pbkdf2_pmk(key: bytes, essid: bytes) -> bytes:
    return hashlib.pbkdf2_hmac("sha1", key, essid, 4096, 32)


# --------------------------------------------------------------------------------------------
# check_key_m22000 (common.php:157-307), pure Python
# --------------------------------------------------------------------------------------------
def py_check_key_m22000(hashline: bytes, keys, pmk=False, nc: int = 128, pbkdf2=pbkdf2_pmk):
    if isinstance(hashline, str):
        hashline = hashline.encode()
    ahl = hashline.split(b"*", 8)
    if len(ahl) != 9:
        return False
    if ahl[0] != b"WPA":
        return False
    if not (valid_hex(ahl[3]) and valid_hex(ahl[4]) and valid_hex(ahl[5])):
        return False
    mac_ap, mac_sta, essid = (bytes.fromhex(ahl[i].decode()) for i in (3, 4, 5))
    if php_eq_type(ahl[1], 1):
        if not valid_hex(ahl[2]):
            return False
        pmkid = bytes.fromhex(ahl[2].decode())
        for key in keys:
            if key is None:
                continue
            if key.startswith(b"$HEX["):
                key = hc_unhex(key)
            if not pmk:
                pmk = pbkdf2(key, essid)
            test = hmac.new(pmk, b"PMK Name" + mac_ap + mac_sta, hashlib.sha1).digest()
            if php_strncmp(test, pmkid, 16) == 0:
                return [key, None, None, pmk]
            pmk = False
    elif php_eq_type(ahl[1], 2):
        for i in (2, 6, 7, 8):
            if not valid_hex(ahl[i]):
                return False
        keymic, nonce_ap, eapol = (bytes.fromhex(ahl[i].decode()) for i in (2, 6, 7))
        if len(eapol) >= 49:
            keyver = struct.unpack(">H", eapol[5:7])[0] & 3
            nonce_sta = eapol[17:49]
        else:
            keyver, nonce_sta = 0, b""
        m = mac_ap + mac_sta if php_strncmp(mac_ap, mac_sta, 6) < 0 else mac_sta + mac_ap
        if php_strncmp(nonce_sta, nonce_ap, 6) < 0:
            n, swap = nonce_sta + nonce_ap, False
        else:
            n, swap = nonce_ap + nonce_sta, True
        if len(nonce_ap) >= 32:
            corr = {"V": struct.unpack("<I", nonce_ap[28:32])[0], "N": struct.unpack(">I", nonce_ap[28:32])[0]}
        else:
            corr = {"V": 0, "N": 0}
        halfnc = (nc >> 1) + 1
        for key in keys:
            if key is None:
                continue
            if key.startswith(b"$HEX["):
                key = hc_unhex(key)
            if not pmk:
                pmk = pbkdf2(key, essid)
            ncarr = [["N", 0]]
            while True:
                for j in ncarr:
                    raw = struct.pack(">I" if j[0] == "N" else "<I", (corr[j[0]] + j[1]) & 0xFFFFFFFF)
                    n = substr_replace(n, raw, 28 if swap else 60, 4)
                    if keyver in (1, 2):
                        ptk = hmac.new(pmk, b"Pairwise key expansion\0" + m + n + b"\0", hashlib.sha1).digest()
                        test = hmac.new(ptk[:16], eapol, hashlib.md5 if keyver == 1 else hashlib.sha1).digest()
                    elif keyver == 3:
                        ptk = hmac.new(pmk, b"\1\0Pairwise key expansion" + m + n + b"\x80\1", hashlib.sha256).digest()
                        test = omac1_aes_128(eapol, ptk[:16])
                    else:
                        return False
                    if php_strncmp(test, keymic, 16) == 0:
                        if ncarr[0][1] == 0:
                            return [key, 0, None, pmk]
                        return [key, j[1], "BE" if j[0] == "N" else "LE", pmk]
                if ncarr[0][1] == 0:
                    ncarr = [["V", 1], ["V", -1], ["N", 1], ["N", -1]]
                else:
                    ncarr[0][1] += 1
                    ncarr[1][1] -= 1
                    ncarr[2][1] += 1
                    ncarr[3][1] -= 1
                if not ncarr[0][1] <= halfnc:
                    break
            pmk = False
    return False


def hash_m22000(hashline: bytes):
    """common.php:310-315."""
    ahl = hashline.split(b"*", 8)
    if len(ahl) != 9:
        return False
    return hashlib.md5(b"".join(ahl[1:8])).digest()


# --------------------------------------------------------------------------------------------
# C oracle (OpenSSL) via ctypes
# --------------------------------------------------------------------------------------------
class OKey(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("n", ctypes.c_size_t)]


class OResult(ctypes.Structure):
    _fields_ = [("key_index", ctypes.c_int32), ("nc", ctypes.c_int32), ("nc_is_null", ctypes.c_int32),
                ("endian", ctypes.c_int32), ("pmk", ctypes.c_uint8 * 32), ("key", ctypes.c_uint8 * 4096),
                ("key_len", ctypes.c_size_t)]


def build():
    """Compile the C oracle (gcc + libcrypto)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_check_m22000.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(OKey), ctypes.c_size_t,
                                          ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(OResult)]
        L.oracle_check_m22000.restype = ctypes.c_int
        L.oracle_check_many.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(OKey), ctypes.c_size_t,
                                        ctypes.c_int, ctypes.c_int, ctypes.POINTER(OResult)]
        L.oracle_check_many.restype = ctypes.c_int64
        L.oracle_pbkdf2_many.argtypes = [ctypes.POINTER(OKey), ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_int]
        L.oracle_pbkdf2_sha1.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_omac1_aes_128.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_void_p]
        L.oracle_hmac.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                  ctypes.c_void_p]
        L.oracle_hash_m22000.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_hash_m22000.restype = ctypes.c_int
        _lib = L
    return _lib


def _keys_array(keys):
    arr = (OKey * max(1, len(keys)))()
    keep = []
    for i, k in enumerate(keys):
        if k is None:
            arr[i].p, arr[i].n = None, 0
        else:
            b = ctypes.create_string_buffer(bytes(k), len(k) + 1)
            keep.append(b)
            arr[i].p, arr[i].n = ctypes.cast(b, ctypes.c_void_p), len(k)
    return arr, keep


def _result_to_php(r: OResult, src: bytes):
    # the C result holds the first len(r.key) bytes of the key; a longer one is the input key, decoded the same way
    key = bytes(r.key[:r.key_len]) if r.key_len <= len(r.key) else hc_unhex(bytes(src))
    pmk = bytes(r.pmk)
    if r.nc_is_null:
        return [key, None, None, pmk]
    return [key, r.nc, {0: None, 1: "BE", 2: "LE"}[r.endian], pmk]


def c_check_key_m22000(hashline, keys, pmk=False, nc: int = 128):
    if isinstance(hashline, str):
        hashline = hashline.encode()
    arr, keep = _keys_array(keys)
    res = OResult()
    rc = lib().oracle_check_m22000(hashline, len(hashline), arr, len(keys), bytes(pmk) if pmk else None, nc,
                                   ctypes.byref(res))
    if rc != 1:
        return False
    return _result_to_php(res, keys[res.key_index])


def c_check_many(hashline: bytes, keys, nc: int = 128, threads: int = 1):
    """One PHP request per key (put_work, common.php:902), on `threads` threads; returns (index, result)."""
    arr, keep = _keys_array(keys)
    res = OResult()
    idx = lib().oracle_check_many(hashline, len(hashline), arr, len(keys), nc, threads, ctypes.byref(res))
    return idx, (_result_to_php(res, keys[idx]) if idx >= 0 else False)


def c_pbkdf2_many(keys, essid: bytes, threads: int = 1) -> bytes:
    arr, keep = _keys_array(keys)
    out = ctypes.create_string_buffer(32 * len(keys))
    lib().oracle_pbkdf2_many(arr, len(keys), essid, len(essid), out, threads)
    return out.raw


def c_pbkdf2(key: bytes, salt: bytes, iters: int = 4096, dklen: int = 32) -> bytes:
    out = ctypes.create_string_buffer(dklen)
    lib().oracle_pbkdf2_sha1(key, len(key), salt, len(salt), iters, out, dklen)
    return out.raw


def c_omac1_aes_128(data: bytes, key: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().oracle_omac1_aes_128(data, len(data), key, out)
    return out.raw


def c_hash_m22000(line: bytes):
    out = ctypes.create_string_buffer(16)
    if not lib().oracle_hash_m22000(line, len(line), out):
        return False
    return out.raw
