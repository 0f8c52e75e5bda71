"""help_crack.py drop-in: run the m22000 attack in-process through libdwpa22000.so instead of a hashcat subprocess.

Replaces ``HelpCrack.run_cracker`` (help_crack/help_crack.py:765-802) and the ``hashcat --stdout -r`` rule
expansions (:508, :575) with the same inputs, outputs and return codes:

* inputs   -- ``conf["hash_file"]`` (one m22000 line per hash, written by prepare_work :439-442),
              ``conf["rules"]`` ("" or "-S -r <file>", :445-447 / :931-933), ``conf["key_file"]``, the dictionary
              list (plain or .gz), ``conf["coptions"]`` (``-d 1,2`` selects devices like hashcat's ``-d``);
* output   -- the ``-o`` key file in hashcat's m22000 outfile format, parsed unchanged by ``get_key`` (:804-879);
* rc       -- hashcat semantics: 0 all cracked, 1 exhausted (drives the second pass at :930); device errors are
              retried after ``sleepy()`` as the reference's loop does (:776-786), never returned; dictionary
              errors are not retried (see run_cracker).

Usage from help_crack.py (the one-line change INTEGRATION.md shows)::

    from dwpa_amd.help_crack import run_cracker as _gpu_run_cracker
    HelpCrack.run_cracker = lambda self, dictlist, disablestdout=False: _gpu_run_cracker(
        self.conf, dictlist, sleepy=self.sleepy, pprint=self.pprint, quiet=disablestdout)
"""
from __future__ import annotations

import gzip
import os
import shlex
import sys
import time

from . import m22000 as M
from . import _lib as L

NONCE_ERROR_CORRECTIONS = 8  # help_crack.py:773 passes --nonce-error-corrections=8


def _parse_options(rules: str, coptions: str):
    rules_file, devices = None, 0
    toks = shlex.split(rules or "") + shlex.split(coptions or "")
    i = 0
    while i < len(toks):
        t = toks[i]
        if t in ("-r", "--rules-file") and i + 1 < len(toks):
            rules_file = toks[i + 1]
            i += 2
            continue
        if t.startswith("--rules-file="):
            rules_file = t.split("=", 1)[1]
        elif t in ("-d", "--backend-devices") and i + 1 < len(toks):
            for d in toks[i + 1].split(","):
                if d.strip().isdigit() and int(d) >= 1:
                    devices |= 1 << (int(d) - 1)  # hashcat numbers devices from 1
            i += 2
            continue
        i += 1
    return rules_file, devices


def _sleepy(sec: int = 123) -> None:
    """HelpCrack.sleepy (help_crack.py:80-87): wait for things to calm down before the next attempt."""
    time.sleep(sec)


def _truncate(path: str, size) -> None:
    """Undo what a failed attempt appended to the key file (size None: the file did not exist)."""
    if size is None:
        if os.path.exists(path):
            os.unlink(path)
    elif os.path.exists(path) and os.path.getsize(path) > size:
        with open(path, "r+b") as f:
            f.truncate(size)


def _summary(rc: int) -> str:
    """hashcat's end-of-run block (Status / Recovered / Progress / Speed), from dwpa_crack_last_stats."""
    st = M.crack_stats()
    status = "Cracked" if rc == L.DWPA_RC_CRACKED else "Exhausted"
    speed = st["candidates"] / st["seconds"] if st["seconds"] > 0 else 0.0
    unit = next((u for u, f in (("MH/s", 1e6), ("kH/s", 1e3)) if speed >= f), "H/s")
    scale = {"MH/s": 1e6, "kH/s": 1e3, "H/s": 1.0}[unit]
    pct = 100.0 * st["cracked"] / st["hashes"] if st["hashes"] else 0.0
    lines = [
        "Session..........: help_crack (libdwpa22000, gfx950)",
        f"Status...........: {status}",
        "Hash.Mode........: 22000 (WPA-PBKDF2-PMKID+EAPOL)",
        f"Recovered........: {st['cracked']}/{st['hashes']} ({pct:.2f}%) Digests",
        f"Progress.........: {st['candidates']} candidates from {st['words']} words",
        f"Speed.#*.........: {speed / scale:8.1f} {unit}",
        f"Time.............: {st['seconds']:.2f} s",
    ]
    if st.get("rules") or st.get("rules_skipped"):
        lines.insert(4, f"Rules............: {st['rules']} loaded, {st['rules_skipped']} skipped (invalid or unsupported)")
    return "\n".join(lines)


def run_cracker(conf: dict, dictlist, nonce_error_corrections: int = NONCE_ERROR_CORRECTIONS, sleepy=None,
                pprint=None, max_tries: int | None = None, quiet: bool = False) -> int:
    """In-process equivalent of the hashcat command line at help_crack.py:773 with the reference's retry loop
    (:776-786): a failed attempt (library or GPU error -- hashcat's -1 / >= 2) is logged, followed by ``sleepy()``
    and retried, so only 0 (all cracked) or 1 (exhausted) ever reaches run(): returning -1 there would skip the
    rules pass (:930) and let put_work report an unsearched work unit as searched.  What a failed attempt appended
    to the key file is removed before the retry, so no hit is written twice.

    Dictionary errors are deterministic and are not retried:

    * a damaged gzip dictionary (truncated download, corrupt stream) is scanned up to the damage, exactly as
      hashcat's gzread reads it, and the call returns 0/1 like hashcat; the file is then deleted so that the next
      prepare_dicts (:520-552, which downloads only missing files and merely warns on an MD5 mismatch) fetches it
      again -- except the user's own ``conf["additional"]`` dictionary (-ad, :661-663), which is only reported;
    * a dictionary that cannot be opened makes the library fail before any device work; that raises DwpaError
      (DWPA_E_IO) at once instead of looping forever on the same work unit.

    ``sleepy``/``pprint`` are the HelpCrack methods when bound from help_crack.py.  ``max_tries`` (None = retry
    forever, as the reference does) ends the device-error loop with a DwpaError instead of a return value.  A
    missing hash file raises FileNotFoundError (the reference would fail on an unbound ``rc``).  Unless ``quiet``
    (help_crack's ``disablestdout``, the challenge run) a finished run prints hashcat's end-of-run block (Status,
    Recovered, Progress, Speed) on stdout, where help_crack shows hashcat's output (:776)."""
    if not os.path.exists(conf["hash_file"]):
        raise FileNotFoundError(conf["hash_file"])
    sleepy = sleepy or _sleepy
    pprint = pprint or (lambda mess, code="HEADER": print(mess, file=sys.stderr))
    rules_file, mask = _parse_options(conf.get("rules", ""), conf.get("coptions", ""))
    key_file = conf["key_file"]
    dictlist = list(dictlist)
    tries = 0
    while True:
        size0 = os.path.getsize(key_file) if os.path.exists(key_file) else None
        rc, status = M.crack_files_ex(conf["hash_file"], dictlist, rules_file, nonce_error_corrections, key_file,
                                      device_mask=mask)
        if rc in (L.DWPA_RC_CRACKED, L.DWPA_RC_EXHAUSTED):
            # a damaged download is removed only once the attempt has counted (its scan up to the damage is the
            # result); a failed attempt is retried below with the same dictionary list, which must still exist
            for d, st in zip(dictlist, status):
                if st != L.DWPA_DICT_DAMAGED:
                    continue
                if d == conf.get("additional"):
                    pprint(f"Dictionary {d} is damaged (truncated or corrupt gzip); scanned up to the damage",
                           "WARNING")
                else:
                    pprint(f"Dictionary {d} is damaged (truncated or corrupt gzip); scanned up to the damage, "
                           "removed so that it is downloaded again", "WARNING")
                    if os.path.exists(d):
                        os.unlink(d)
            if not quiet:
                try:
                    print(_summary(rc), flush=True)
                except L.DwpaError:  # no crack call ran in this thread (a stubbed library): nothing to summarise
                    pass
            return rc
        _truncate(key_file, size0)
        unreadable = [d for d, st in zip(dictlist, status) if st == L.DWPA_E_IO]
        if unreadable:
            pprint(f"Dictionary cannot be read: {', '.join(unreadable)}", "FAIL")
            raise L.DwpaError(L.DWPA_E_IO, f"dictionary cannot be read: {', '.join(unreadable)}")
        tries += 1
        pprint(f"libdwpa22000 crack_files failed with code {rc}", "FAIL")
        if max_tries is not None and tries >= max_tries:
            raise L.DwpaError(rc, f"crack_files failed {tries} times")
        sleepy()


def expand_rules(rules_file: str, source: str, out_path: str, gzip_level: int = 0, device: int = 0) -> int:
    """`hashcat --stdout -r rules_file source -o out_path` (help_crack.py:508 expandcracked, :575 prdict) with the
    rules applied on the GPU and the candidates packed and written by the library (dwpa_rules_expand_file): one per
    line, word-major, rejected candidates skipped, $HEX[] for non-printable ones.  Like hashcat, the output is plain
    text whatever its name (help_crack names it cracked.txt.gz; the dictionary readers take plain and gzip alike);
    gzip_level 1..9 compresses it.  Rule lines that do not parse are reported by the library on stderr ("skipping
    invalid or unsupported rule in <file> on line <n>"), and a file without a valid rule raises, as hashcat refuses
    to start.  Returns the number of candidates written."""
    _, cands = M.rules_expand_file(rules_file, [source], out_path, gzip_level, device)
    return cands
