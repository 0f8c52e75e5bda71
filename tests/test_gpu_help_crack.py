"""GPU: help_crack end to end through dwpa_amd.help_crack.install(), on a box with no hashcat or john (VERDICT r4
item 1).  The client is the reference's HelpCrack test double (tests/helpcrack_standin.py: the reference may not be
imported here); every step below is the reference's own call sequence:

* the challenge self-test of HelpCrack.run() (help_crack.py:883-895): check_tools -> prepare_challenge (a gzip
  dictionary holding "aaaa1234" with no newline) -> prepare_work -> run_cracker(disablestdout=True) -> get_key, and
  the acceptance rule of :893;
* expandcracked (:469-509): cracked.txt.gz + rkg.txt.gz -> source.txt -> `./hashcat.bin --stdout -o cracked.txt.gz
  -r bestWPA.rule source.txt`, answered on the GPU; the output equals the rule oracle's expansion;
* the prdict expansion of prepare_dicts (:557-585), the same way, then a crack over the expanded prdict.txt.gz.
"""
import gzip
import importlib
import random

import pytest

pytestmark = pytest.mark.gpu

from dwpa_amd import help_crack as H  # noqa: E402
from dwpa_amd.rulesets import wpa_rules  # noqa: E402
from oracle import rules as R  # noqa: E402
from tests import synth as S  # noqa: E402


@pytest.fixture
def client(monkeypatch, tmp_path):
    from tests import helpcrack_standin
    mod = importlib.reload(helpcrack_standin)
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("PATH", str(tmp_path / "nobin"))  # no hashcat, no john
    H.install(mod.HelpCrack)
    (tmp_path / "bestWPA.rule").write_text("\n".join(wpa_rules()) + "\n")
    return mod


def test_challenge_through_installed_methods(client):
    hc = client.HelpCrack()
    assert hc.challenge()
    assert hc.conf["format"] == "22000" and hc.conf["cracker"] == H.CRACKER
    assert not [m for c, m in hc.log if c == "FAIL"]


def test_challenge_fails_on_a_wrong_key(client):
    """The self-test is a real check: with the KAT's PSK changed, no record comes out and the rule of :893 fails."""
    hc = client.HelpCrack()
    client.CHALLENGE["key"] = "aaaa1235"
    assert not hc.challenge()


def _lines(raw: bytes):
    return raw.split(b"\n")[:-1]


def test_expandcracked_on_the_gpu(client, tmp_path):
    rng = random.Random(51)
    cracked = [S.random_psk(rng, 6, 16) for _ in range(4000)]
    rkg = [S.random_psk(rng, 8, 12) for _ in range(500)]
    with gzip.open("cracked.txt.gz", "wb") as f:
        f.write(b"\n".join(cracked) + b"\n")
    rkg_gz = gzip.compress(b"\n".join(rkg) + b"\n")
    hc = client.HelpCrack()
    hc.download = lambda url, fn: open(fn, "wb").write(rkg_gz)
    hc.check_tools()
    assert hc.expandcracked() == 0
    exp = [c for row in R.expand(wpa_rules(), cracked + rkg) for c in row if c is not None]
    assert _lines((tmp_path / "cracked.txt.gz").read_bytes()) == exp  # plain text, whatever its name (as hashcat)


def test_prdict_expansion_and_crack(client, tmp_path):
    rng = random.Random(52)
    words = [S.random_psk(rng, 6, 12) for _ in range(3000)]
    with gzip.open("prdict.txt.gz", "wb") as f:
        f.write(b"\n".join(words) + b"\n")
    hc = client.HelpCrack()
    hc.check_tools()
    dlist = hc.expand_prdict(["other.txt.gz"])
    assert dlist == ["prdict.txt.gz", "other.txt.gz"]
    rules = wpa_rules()
    exp = [c for row in R.expand(rules, words) for c in row if c is not None]
    assert _lines((tmp_path / "prdict.txt.gz").read_bytes()) == exp
    # a PSK only the expansion holds is then cracked from it (run_cracker over dictlist0's prdict, :924-929)
    psk = next(c for c in exp[len(exp) // 2:] if 8 <= len(c) <= 63 and b":" not in c)
    essid, ap, sta, an, sn = S.random_net(rng)
    hc.prepare_work({"hashes": [S.eapol_line(psk, essid, ap, sta, an, sn, 2, 3, "LE", rng=rng).decode()]})
    assert hc.run_cracker(["prdict.txt.gz"]) == 0
    assert hc.get_key() == [{"k": ap.hex(), "v": psk.hex()}]
