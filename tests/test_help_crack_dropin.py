"""CPU: help_crack's run_cracker drop-in (dwpa_amd/help_crack.py) and the reference's retry loop
(help_crack/help_crack.py:776-786).

* Device errors (hashcat's -1 / >= 2) are logged, followed by sleepy() and a retry; run() only ever sees 0 or 1.
  Returning -1 instead would skip the rules pass (:930) and put_work would report an unsearched work unit as
  searched.  Without a GPU the library fails every attempt with a device error, which is what these tests use.
* Dictionary errors are deterministic and never retried: an unreadable dictionary raises at
  once even with max_tries=None; a damaged gzip is scanned to the damage, returned as 0/1 and deleted so that
  prepare_dicts (:530-534) downloads it again (never the user's -ad dictionary).
* A failed attempt's key-file records are rolled back, so a retry never writes a hit twice.
"""
import gzip

import pytest

from dwpa_amd import _lib as L
from dwpa_amd import help_crack as H
from tests import synth as S
from dwpa_amd.help_crack import run_cracker


def _conf(tmp_path):
    hf = tmp_path / "help_crack.hash"
    hf.write_bytes(S.CHALLENGE_LINES[0] + b"\n")
    return {"hash_file": str(hf), "key_file": str(tmp_path / "help_crack.key"), "rules": "", "coptions": ""}


def _dict(tmp_path, name="d.txt.gz"):
    p = tmp_path / name
    with gzip.open(p, "wb") as f:
        f.write(b"password\naaaa1234\n")
    return str(p)


def test_device_failure_is_retried_never_returned(tmp_path):
    conf = _conf(tmp_path)
    sleeps, logs = [], []
    with pytest.raises(L.DwpaError):
        run_cracker(conf, [_dict(tmp_path)], sleepy=lambda: sleeps.append(1),
                    pprint=lambda m, c="HEADER": logs.append((m, c)), max_tries=3)
    assert len(sleeps) == 2 and len(logs) == 3
    assert all(c == "FAIL" and "-1" in m for m, c in logs)


def test_run_flow_never_reaches_put_work_after_a_failure(tmp_path):
    """help_crack.py:923-933 shape: a cracker failure must not fall through to get_key/put_work."""
    conf = _conf(tmp_path)
    reached = []
    d = _dict(tmp_path)

    def run():
        rc = run_cracker(conf, [d], sleepy=lambda: None, pprint=lambda *a: None, max_tries=2)
        if rc == 1:
            run_cracker(conf, [d], sleepy=lambda: None, pprint=lambda *a: None, max_tries=2)
        reached.append("put_work")

    with pytest.raises(L.DwpaError):
        run()
    assert reached == []


def test_unreadable_dictionary_raises_at_once(tmp_path):
    """max_tries=None (the reference's forever loop): a missing dictionary is reported by the library itself
    (before any device work, with or without a GPU) and raises on the first attempt, with no sleepy()."""
    conf = _conf(tmp_path)
    sleeps, logs = [], []
    with pytest.raises(L.DwpaError) as e:
        run_cracker(conf, [_dict(tmp_path), str(tmp_path / "missing.txt.gz")], sleepy=lambda: sleeps.append(1),
                    pprint=lambda m, c="HEADER": logs.append((m, c)), max_tries=None)
    assert e.value.code == L.DWPA_E_IO and sleeps == []
    assert any("missing.txt.gz" in m for m, _ in logs)


def test_library_reports_unreadable_dictionary_status(tmp_path):
    from dwpa_amd import m22000 as M
    conf = _conf(tmp_path)
    rc, st = M.crack_files_ex(conf["hash_file"], [_dict(tmp_path), str(tmp_path / "nope")], None, 8,
                              conf["key_file"])
    assert rc == L.DWPA_RC_ERROR and st == [L.DWPA_DICT_OK, L.DWPA_E_IO]


def test_damaged_dictionary_is_removed_and_rc_returned(tmp_path, monkeypatch):
    """Host logic of the drop-in with the library's answer stubbed: rc 1 with one damaged dictionary -> 1 is
    returned in one attempt, the damaged download is deleted, the user's -ad dictionary is kept."""
    conf = _conf(tmp_path)
    a, b, user = _dict(tmp_path, "a.txt.gz"), _dict(tmp_path, "b.txt.gz"), _dict(tmp_path, "mine.txt.gz")
    conf["additional"] = user
    calls = []

    def fake(hash_file, dicts, rules_file, nec, key_file, device_mask=0):
        calls.append(list(dicts))
        return 1, [L.DWPA_DICT_OK, L.DWPA_DICT_DAMAGED, L.DWPA_DICT_DAMAGED]
    monkeypatch.setattr(H.M, "crack_files_ex", fake)
    logs = []
    assert run_cracker(conf, [a, b, user], sleepy=lambda: None, pprint=lambda m, c="": logs.append((m, c))) == 1
    assert len(calls) == 1
    import os
    assert os.path.exists(a) and not os.path.exists(b) and os.path.exists(user)
    assert sum(1 for _, c in logs if c == "WARNING") == 2


def test_damaged_dictionary_kept_for_the_retry_of_a_failed_attempt(tmp_path, monkeypatch):
    """an attempt that read a damaged download and then failed with a device error (rc -1) is
    retried with the same dictionary list, so the file must still exist; it is removed only after the attempt that
    counts (rc 0/1).  Deleting it first made the retry fail the library's up-front open check (DWPA_E_IO) and
    broke the "device errors are retried, never returned" rule."""
    conf = _conf(tmp_path)
    a, b = _dict(tmp_path, "a.txt.gz"), _dict(tmp_path, "b.txt.gz")
    import os
    seen = []

    def fake(hash_file, dicts, rules_file, nec, key_file, device_mask=0):
        seen.append([os.path.exists(d) for d in dicts])
        if len(seen) == 1:
            return L.DWPA_RC_ERROR, [L.DWPA_DICT_OK, L.DWPA_DICT_DAMAGED]
        return L.DWPA_RC_EXHAUSTED, [L.DWPA_DICT_OK, L.DWPA_DICT_DAMAGED]
    monkeypatch.setattr(H.M, "crack_files_ex", fake)
    assert run_cracker(conf, [a, b], sleepy=lambda: None, pprint=lambda *a: None) == 1
    assert seen == [[True, True], [True, True]]
    assert os.path.exists(a) and not os.path.exists(b)


def test_failed_attempt_hits_are_rolled_back(tmp_path, monkeypatch):
    """An attempt that wrote a hit and then failed (device error) must not leave it behind: the retry writes it
    again, once."""
    conf = _conf(tmp_path)
    key = tmp_path / "help_crack.key"
    key.write_bytes(b"earlier-record\n")
    rec = b"8ac36b891edca8eef49094b1afe061ac:1c7ee5e2f2d0:0026c72e4900:dlink:aaaa1234\n"
    n = []

    def fake(hash_file, dicts, rules_file, nec, key_file, device_mask=0):
        n.append(1)
        with open(key_file, "ab") as f:
            f.write(rec)
        return (L.DWPA_RC_ERROR if len(n) == 1 else L.DWPA_RC_CRACKED), [L.DWPA_DICT_OK]
    monkeypatch.setattr(H.M, "crack_files_ex", fake)
    assert run_cracker(conf, [_dict(tmp_path)], sleepy=lambda: None, pprint=lambda *a: None) == 0
    assert len(n) == 2 and key.read_bytes() == b"earlier-record\n" + rec


def test_failed_first_attempt_without_key_file(tmp_path, monkeypatch):
    conf = _conf(tmp_path)
    n = []

    def fake(hash_file, dicts, rules_file, nec, key_file, device_mask=0):
        n.append(1)
        with open(key_file, "ab") as f:
            f.write(b"partial\n")
        return (L.DWPA_RC_ERROR if len(n) == 1 else L.DWPA_RC_EXHAUSTED), [L.DWPA_DICT_OK]
    monkeypatch.setattr(H.M, "crack_files_ex", fake)
    assert run_cracker(conf, [_dict(tmp_path)], sleepy=lambda: None, pprint=lambda *a: None) == 1
    assert (tmp_path / "help_crack.key").read_bytes() == b"partial\n"


def test_missing_hash_file_raises(tmp_path):
    conf = _conf(tmp_path)
    conf["hash_file"] = str(tmp_path / "nope.hash")
    with pytest.raises(FileNotFoundError):
        run_cracker(conf, [], max_tries=1)


def test_end_of_run_summary(tmp_path, monkeypatch, capsys):
    """Like hashcat, each finished attempt prints Status / Recovered / Progress / Speed on stdout (help_crack shows
    hashcat's output, help_crack.py:776), from dwpa_crack_last_stats; quiet (help_crack's disablestdout, the
    challenge run) prints nothing."""
    conf = _conf(tmp_path)
    monkeypatch.setattr(H.M, "crack_files_ex", lambda *a, **k: (1, [L.DWPA_DICT_OK]))
    monkeypatch.setattr(H.M, "crack_stats", lambda: {"words": 1000, "candidates": 9_790_000, "hashes": 4,
                                                     "cracked": 1, "seconds": 2.0, "rules": 148, "rules_skipped": 2})
    assert run_cracker(conf, [_dict(tmp_path)], sleepy=lambda: None, pprint=lambda *a: None) == 1
    out = capsys.readouterr().out
    assert "Rules............: 148 loaded, 2 skipped (invalid or unsupported)" in out
    assert "Status...........: Exhausted" in out and "Recovered........: 1/4 (25.00%) Digests" in out
    assert "Progress.........: 9790000 candidates from 1000 words" in out and "4.9 MH/s" in out
    assert run_cracker(conf, [_dict(tmp_path)], sleepy=lambda: None, pprint=lambda *a: None, quiet=True) == 1
    assert capsys.readouterr().out == ""
