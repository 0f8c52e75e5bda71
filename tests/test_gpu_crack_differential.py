"""The client path at scale: a random work unit through dwpa_crack_files (help_crack.py:765-802's hashcat -m22000
call) against a Python model of what it must crack.

The hash file holds PMKID and keyver 1/2/3 lines over shared ESSIDs, with planted nonce corrections of either
endianness and the message_pair bits the client honours (0x10 no NC, 0x20 LE only, 0x40 BE only, both or neither).
The PSKs are planted behind random rules of bestWPA.rule, as plain words or `$HEX[]` dictionary entries (some
CRLF). Decoys are a PSK in no candidate, a rule result outside 8..63 bytes, and a correction just outside the window.

The model:

* A line is cracked iff its PSK is a candidate (word x rule, 8..63 bytes; oracle/rules.py) and its planted
  correction lies in the window: 0 always; otherwise |nc| <= nonce_error_corrections and the endian allowed by mp.
* rc is 0 when every line is cracked, else 1.
* Every outfile record names a cracked line and its PSK (plain, or `$HEX[]` for a byte outside printable ASCII or a
  ':'), once per line.

The window's message_pair handling is this engine's reading of hashcat's (parity unpinned). The test
holds the GPU path to that reading and to the rule oracle at scale. DWPA_CRACK_DIFF_LINES sets the size (default
240 lines over 60 ESSIDs x 20,000 words x 24 rules; round 5 also ran 3 seeds x 1,200 lines over 300 ESSIDs,
profiles/r05/differential/), DWPA_CRACK_DIFF_SEED the seed."""
import gzip
import os
import random

import pytest

pytestmark = pytest.mark.gpu

import dwpa_amd  # noqa: E402
from tests import synth as S  # noqa: E402
from dwpa_amd.rulesets import wpa_rules  # noqa: E402
from oracle import rules as R  # noqa: E402


def _window_ok(kind, off, endian, mp, nec):
    if kind == "pmkid" or off == 0:
        return True
    if abs(off) > nec or mp & 0x10:
        return False
    le_only, be_only = (mp & 0x20) and not (mp & 0x40), (mp & 0x40) and not (mp & 0x20)
    return not ((le_only and endian == "BE") or (be_only and endian == "LE"))


def _plain(psk: bytes) -> bytes:
    return psk if all(0x20 <= c <= 0x7E and c != 0x3A for c in psk) else b"$HEX[" + psk.hex().encode() + b"]"


@pytest.mark.parametrize("nec", [8, 3])
def test_crack_files_differential(tmp_path, nec):
    n_lines = int(os.environ.get("DWPA_CRACK_DIFF_LINES", "240"))
    rng = random.Random(int(os.environ.get("DWPA_CRACK_DIFF_SEED", "77")) + nec)
    rules = [":"] + rng.sample(wpa_rules()[1:], 23)
    ops = [R.parse(r) for r in rules]
    words = [S.fast_psk(rng, 4, 20) for _ in range(20000)]
    hexed = set(rng.sample(range(len(words)), 400))  # written as $HEX[..] (decoded before the rules apply)
    for i in rng.sample(sorted(hexed), 40):
        words[i] = words[i][:3] + b":" + words[i][4:] if len(words[i]) > 4 else words[i]  # ':' forces $HEX out
    nets = [S.random_net(rng) for _ in range(max(60, n_lines // 4))]
    lines, expect = [], {}
    for li in range(n_lines):
        essid, _, _, an, sn = nets[rng.randrange(len(nets))]
        ap, sta = rng.randbytes(6), rng.randbytes(6)
        r = rng.random()
        if r < 0.75:  # a candidate: word x rule (possibly rejected or outside 8..63)
            psk = R.apply(ops[rng.randrange(len(ops))], words[rng.randrange(len(words))])
            crackable = psk is not None and 8 <= len(psk) <= 63
            psk = psk if psk is not None else b"rejected-by-rule"
        else:  # in no candidate
            psk, crackable = b"nowhere-" + rng.randbytes(6).hex().encode(), False
        kind = rng.choice(["pmkid", 1, 2, 3])
        off, endian, mp = rng.choice([0, 0, 1, -2, 3, -3, 4, 8, -8, 9, -12]), rng.choice(["LE", "BE"]), \
            rng.choice([0x00, 0x10, 0x20, 0x40, 0x60])
        if kind == "pmkid":
            line = S.pmkid_line(psk, essid, ap, sta)
        else:
            line = S.eapol_line(psk, essid, ap, sta, an, sn, kind, off, endian, mp=mp, rng=rng)
        lines.append(line)
        if crackable and _window_ok(kind, off, endian, mp, nec):
            expect[line.split(b"*")[2]] = psk
    hf = tmp_path / "w.hash"
    hf.write_bytes(b"\n".join(lines) + b"\n")
    dl = tmp_path / "d.txt.gz"
    with gzip.open(dl, "wb", compresslevel=1) as f:
        for i, w in enumerate(words):
            f.write((b"$HEX[" + w.hex().encode() + b"]" if i in hexed else w) + (b"\r\n" if i % 7 == 0 else b"\n"))
    rf = tmp_path / "r.rule"
    rf.write_text("\n".join(rules) + "\n")
    out = tmp_path / "w.key"
    rc = dwpa_amd.crack_files(str(hf), [str(dl)], str(rf), nec, str(out), batch=1 << 18)
    assert rc == (0 if len(expect) == n_lines else 1)
    got = {}
    for rec in out.read_bytes().splitlines():
        f = rec.split(b":", 4)
        assert f[0] not in got, rec  # one record per line
        got[f[0]] = f[4]
    assert got == {bytes.fromhex(k.decode()).hex().encode(): _plain(v) for k, v in expect.items()}
    print(f"crack differential nec={nec}: {n_lines} lines, {len(expect)} cracked")
    assert n_lines // 4 < len(expect) < n_lines
