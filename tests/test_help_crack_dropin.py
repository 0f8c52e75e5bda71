"""CPU: help_crack's run_cracker drop-in keeps the reference's retry loop (help_crack/help_crack.py:776-786).

hashcat's error exits (-1, >= 2) are logged, followed by sleepy() and a retry; run() only ever sees 0 or 1.
Returning -1 instead would skip the rules pass (:930) and put_work would report an unsearched work unit as
searched.  The failure here is a dictionary that does not exist (DWPA_RC_ERROR with or without a GPU).
"""
import pytest

from dwpa_amd import _lib as L
from dwpa_amd import synth as S
from dwpa_amd.help_crack import run_cracker


def _conf(tmp_path):
    hf = tmp_path / "help_crack.hash"
    hf.write_bytes(S.CHALLENGE_LINES[0] + b"\n")
    return {"hash_file": str(hf), "key_file": str(tmp_path / "help_crack.key"), "rules": "", "coptions": ""}


def test_failure_is_retried_never_returned(tmp_path):
    conf = _conf(tmp_path)
    sleeps, logs = [], []
    with pytest.raises(L.DwpaError):
        run_cracker(conf, [str(tmp_path / "missing.txt.gz")], sleepy=lambda: sleeps.append(1),
                    pprint=lambda m, c="HEADER": logs.append((m, c)), max_tries=3)
    assert len(sleeps) == 2 and len(logs) == 3
    assert all(c == "FAIL" and "-1" in m for m, c in logs)


def test_run_flow_never_reaches_put_work_after_a_failure(tmp_path):
    """help_crack.py:923-933 shape: a cracker failure must not fall through to get_key/put_work."""
    conf = _conf(tmp_path)
    reached = []

    def run():
        rc = run_cracker(conf, [str(tmp_path / "missing.txt")], sleepy=lambda: None,
                         pprint=lambda *a: None, max_tries=2)
        if rc == 1:
            run_cracker(conf, [str(tmp_path / "missing.txt")], sleepy=lambda: None, pprint=lambda *a: None,
                        max_tries=2)
        reached.append("put_work")

    with pytest.raises(L.DwpaError):
        run()
    assert reached == []


def test_missing_hash_file_raises(tmp_path):
    conf = _conf(tmp_path)
    conf["hash_file"] = str(tmp_path / "nope.hash")
    with pytest.raises(FileNotFoundError):
        run_cracker(conf, [], max_tries=1)
