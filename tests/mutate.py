"""Random hashline mutations for the parse-semantics fuzz tests (test_parse_fuzz.py on the CPU, test_gpu_parity.py
on the GPU).  check_key_m22000 (web/common.php:157-307) decides acceptance from explode('*', $line, 9), a loose
`==` on the type field, ctype_xdigit/even length on every hex field it reads, the EAPOL frame's length and key
version, and strncmp over 16 bytes of the PMKID/MIC.  The mutations below hit each of those decisions: most
mutated lines are rejected or stop matching, some stay valid (upper-case hex, extra fields past the ninth,
longer PMKIDs), and both kinds must come out exactly as the oracle says.
"""
from __future__ import annotations

import random

from tests import synth as S

TYPES = [b"01", b"02", b"1", b"2", b"001", b"002", b" 1", b"2 ", b"+1", b"1.0", b"2e0", b"0x1", b"", b"3", b"00",
         b"1 ", b" 02", b"02.", b".2e1", b"-1", b"1e", b"01\t", b"\n2"]
CHARS = b"0123456789abcdefABCDEF*gxz \t"


def _fields(line: bytes):
    return line.split(b"*")


def mutate(rng: random.Random, line: bytes) -> bytes:
    f = _fields(line)
    op = rng.randrange(11)
    if op == 0:  # type field (loose ==)
        f[1] = rng.choice(TYPES)
    elif op == 1:  # drop one character anywhere
        i = rng.randrange(len(line))
        return line[:i] + line[i + 1:]
    elif op == 2:  # insert one character
        i = rng.randrange(len(line) + 1)
        return line[:i] + bytes([rng.choice(CHARS)]) + line[i:]
    elif op == 3:  # replace one character
        i = rng.randrange(len(line))
        return line[:i] + bytes([rng.choice(CHARS)]) + line[i + 1:]
    elif op == 4:  # upper-case one field (ctype_xdigit accepts A-F)
        k = rng.randrange(len(f))
        f[k] = f[k].upper()
    elif op == 5:  # shorten a hex field by 1-4 nibbles (odd lengths, short MIC/PMKID/ANONCE/EAPOL)
        k = rng.randrange(2, len(f))
        f[k] = f[k][:max(0, len(f[k]) - rng.randint(1, 4))]
    elif op == 6:  # lengthen a hex field by 1-3 bytes
        k = rng.randrange(2, len(f))
        f[k] = f[k] + rng.randbytes(rng.randint(1, 3)).hex().encode()
    elif op == 7:  # duplicate a field (10 fields: the 9th keeps a '*')
        k = rng.randrange(len(f))
        f.insert(k, f[k])
    elif op == 8:  # drop a field
        del f[rng.randrange(len(f))]
    elif op == 9:  # empty a field
        f[rng.randrange(len(f))] = b""
    else:  # EAPOL key-information bits (key version 0..3) or frame shortened around the 49-byte unpack
        if len(f) > 7 and len(f[7]) >= 14:
            e = bytearray(f[7])
            if rng.random() < 0.5:
                e[13:14] = rng.choice(b"0123456789abcdef").to_bytes(1, "big")
                f[7] = bytes(e)
            else:
                f[7] = f[7][:2 * rng.choice([47, 48, 49, 50])]
        else:
            f[1] = rng.choice(TYPES)
    return b"*".join(f)


def base_jobs(rng: random.Random, n: int):
    """n valid (line, psk, keyver or 'pmkid') triples over a few shared ESSIDs."""
    nets = [S.random_net(rng) for _ in range(6)]
    out = []
    for _ in range(n):
        essid, ap, sta, an, sn = nets[rng.randrange(len(nets))]
        psk = S.random_psk(rng, 8, 20)
        kind = rng.choice(["pmkid", 1, 2, 3])
        if kind == "pmkid":
            line = S.pmkid_line(psk, essid, rng.randbytes(6), rng.randbytes(6))
        else:
            line = S.eapol_line(psk, essid, rng.randbytes(6), rng.randbytes(6), rng.randbytes(32), rng.randbytes(32),
                                kind, rng.randint(-3, 3), rng.choice(["LE", "BE"]), rng=rng)
        out.append((line, psk, kind))
    return out


def mutated_jobs(seed: int, n: int):
    """n check jobs (line, keys, pmk, nc): one or two mutations of a valid line, the right key among decoys."""
    rng = random.Random(seed)
    jobs = []
    for line, psk, _ in base_jobs(rng, n):
        for _ in range(rng.choice([1, 1, 2])):
            line = mutate(rng, line)
        keys = [S.random_psk(rng, 8, 12)] if rng.random() < 0.5 else []
        keys.insert(rng.randint(0, len(keys)), psk)
        jobs.append((line, keys, False, rng.choice([0, 1, 8, -3, 6])))
    return jobs
