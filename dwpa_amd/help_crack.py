"""help_crack.py drop-in: run the m22000 attack in-process through libdwpa22000.so instead of a hashcat subprocess.

Replaces, with the same inputs, outputs and return codes:

* ``HelpCrack.run_cracker`` (help_crack/help_crack.py:765-802, command line :773, rc handling :776-786):
  ``conf["hash_file"]`` (one m22000 line per hash, written by prepare_work :439-442), ``conf["rules"]`` ("" or
  "-S -r <file>", :445-447 / :931-933), ``conf["key_file"]``, the dictionary list (plain or .gz),
  ``conf["coptions"]`` (``-d 1,2`` selects devices like hashcat's ``-d``) -> the ``-o`` key file in hashcat's m22000
  outfile format, parsed unchanged by ``get_key`` (:804-879), and hashcat's rc (0 all cracked, 1 exhausted: drives
  the second pass at :930; device errors are retried after ``sleepy()`` as the reference's loop does, never
  returned; dictionary errors are not retried, see run_cracker);
* ``HelpCrack.check_tools`` (:191-307), which looks for a hashcat >= 6.2.6 or john binary and ``sys.exit(1)``s
  without one (:286-290): the replacement needs no binary, checks that a gfx950 device is usable, and sets
  ``conf["cracker"]`` and ``conf["format"] = "22000"`` (what ``set_format`` does for hashcat, :278-284), so that
  prepare_challenge (:705-708), prepare_work (:441) and prepare_dicts (:536, :571) take their m22000 branches;
* the two ``./hashcat.bin --stdout ... -r bestWPA.rule source.txt`` expansions -- ``expandcracked`` (:508-509) and
  the prdict expansion inline in ``prepare_dicts`` (:575-576) -- answered by the GPU rule engine
  (dwpa_rules_expand_file) through help_crack's module-level ``subprocess``: every other subprocess call
  (hcxpsktool :645, imeigen :684) goes to the real module unchanged.

Usage: two lines in help_crack.py's ``__main__`` block, before ``hc = HelpCrack(conf)`` (:995)::

    from dwpa_amd.help_crack import install
    install(HelpCrack)
"""
from __future__ import annotations

import os
import shlex
import shutil
import sys
import tempfile
import time

from . import m22000 as M
from . import _lib as L

NONCE_ERROR_CORRECTIONS = 8  # help_crack.py:773 passes --nonce-error-corrections=8
CRACKER = "libdwpa22000 (gfx950)"  # conf["cracker"] after the installed check_tools
HASHCAT_NAMES = ("hashcat", "hashcat.bin", "hashcat.exe")  # the binaries check_tools looks for (:244)


def _parse_options(rules: str, coptions: str):
    """The parts of help_crack's hashcat command line (:773) that change the work: ``conf["rules"]`` ("-S -r <file>")
    and the user's ``-co`` options -- the rules file, hashcat's ``-d`` device list (numbered from 1) and a
    ``--nonce-error-corrections`` that overrides the command line's 8 (hashcat takes the last one given).  Returns
    (rules file or None, device mask, nonce-error-corrections or None)."""
    rules_file, devices, nec = None, 0, None
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
        elif t == "--nonce-error-corrections" and i + 1 < len(toks) and toks[i + 1].isdigit():
            nec = int(toks[i + 1])
            i += 2
            continue
        elif t.startswith("--nonce-error-corrections=") and t.split("=", 1)[1].isdigit():
            nec = int(t.split("=", 1)[1])
        i += 1
    return rules_file, devices, nec


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
        rejmem = f", {st['rules_rejmem']} of them for reject / memory functions" if st.get("rules_rejmem") else ""
        lines.insert(4, f"Rules............: {st['rules']} loaded, {st['rules_skipped']} skipped (invalid or "
                        f"unsupported{rejmem})")
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
    rules_file, mask, nec = _parse_options(conf.get("rules", ""), conf.get("coptions", ""))
    if nec is not None:
        nonce_error_corrections = nec
    if nonce_error_corrections > L.DWPA_NC_MAX:  # deterministic: the library refuses it on every attempt
        pprint(f"--nonce-error-corrections={nonce_error_corrections} is above the supported {L.DWPA_NC_MAX}", "FAIL")
        raise L.DwpaError(L.DWPA_E_ARG, f"nonce_error_corrections {nonce_error_corrections} > {L.DWPA_NC_MAX}")
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
    line, word-major, rejected candidates skipped, raw bytes as hashcat writes them ($HEX[] only for a candidate
    holding '\\n' or '\\r', which would not stay one line).  Like hashcat, the output is plain
    text whatever its name (help_crack names it cracked.txt.gz; the dictionary readers take plain and gzip alike);
    gzip_level 1..9 compresses it.  Rule lines that do not parse are reported by the library on stderr ("skipping
    invalid or unsupported rule in <file> on line <n>"), and a file without a valid rule raises, as hashcat refuses
    to start.  Returns the number of candidates written."""
    _, cands = M.rules_expand_file(rules_file, [source], out_path, gzip_level, device)
    return cands


class HashcatArgError(ValueError):
    """A `hashcat --stdout` command line this replacement does not take (it names what)."""


def parse_hashcat_stdout(argv):
    """`hashcat --stdout` argv -> (rules files, wordlists, outfile or None).  Takes what help_crack.py:508,575 pass --
    ``--stdout --quiet -w 4 -o <out> -r <rules> <wordlist>`` -- in hashcat's spellings (``-oFILE``, ``--outfile=``,
    ``--rules-file``, ``-w4``, ``--workload-profile``); options that do not change the candidates (``--quiet``,
    ``-w``, ``--session``, ``--potfile-disable``, ...) are accepted and ignored.  Anything that would (masks,
    ``-a``, ``-j``/``-k``, ``-g`` random rules, ...) raises HashcatArgError."""
    rules, words, out = [], [], None
    ignore_flag = {"--stdout", "--quiet", "--potfile-disable", "--logfile-disable", "--advice-disable", "-O",
                   "--optimized-kernel-enable", "--force", "--status", "--machine-readable"}
    ignore_val = {"-w", "--workload-profile", "--session", "-d", "--backend-devices", "--status-timer",
                  "--outfile-format"}
    i, toks = 1, list(argv)
    while i < len(toks):
        t = toks[i]
        if t in ignore_flag or t.startswith("--session=") or t.startswith("--workload-profile="):
            i += 1
        elif t in ignore_val:
            i += 2
        elif t.startswith("-w") and t[2:].isdigit():
            i += 1
        elif t in ("-o", "--outfile"):
            out = toks[i + 1] if i + 1 < len(toks) else None
            i += 2
        elif t.startswith("--outfile="):
            out = t.split("=", 1)[1]
            i += 1
        elif t.startswith("-o") and len(t) > 2:
            out = t[2:]
            i += 1
        elif t in ("-r", "--rules-file"):
            if i + 1 >= len(toks):
                raise HashcatArgError(f"{t} needs a file")
            rules.append(toks[i + 1])
            i += 2
        elif t.startswith("--rules-file="):
            rules.append(t.split("=", 1)[1])
            i += 1
        elif t.startswith("-r") and len(t) > 2:
            rules.append(t[2:])
            i += 1
        elif t.startswith("-") and t != "-":
            raise HashcatArgError(f"option {t} is not supported by the GPU --stdout replacement")
        else:
            words.append(t)
            i += 1
    if not words:
        raise HashcatArgError("no wordlist")
    if len(rules) > 1:
        raise HashcatArgError("stacked -r rule files are not supported (help_crack passes one)")
    return rules, words, out


def is_hashcat_stdout(argv) -> bool:
    return bool(argv) and os.path.basename(str(argv[0])) in HASHCAT_NAMES and "--stdout" in argv


def hashcat_stdout(argv, device: int = 0, pprint=None) -> int:
    """Run a `hashcat --stdout [-r rules] [-o out] wordlists...` command line (help_crack.py:508, :575) on the GPU:
    every word x every rule, written word-major as hashcat writes it (expand_rules).  Without -r every word is
    written once (the ':' rule); without -o the candidates go to stdout.  Returns 0, or -1 with a message (a bad
    command line, an unreadable wordlist or rules file), as hashcat fails."""
    pprint = pprint or (lambda mess, code="HEADER": print(mess, file=sys.stderr))
    try:
        rules, words, out = parse_hashcat_stdout(argv)
    except HashcatArgError as e:
        pprint(f"hashcat --stdout replacement: {e}", "FAIL")
        return -1
    tmp = []
    try:
        if not rules:
            fd, noop = tempfile.mkstemp(suffix=".rule")
            os.write(fd, b":\n")
            os.close(fd)
            tmp.append(noop)
            rules = [noop]
        target = out
        if out is None:
            fd, target = tempfile.mkstemp(suffix=".txt")
            os.close(fd)
            tmp.append(target)
        M.rules_expand_file(rules[0], words, target, 0, device)
        if out is None:
            with open(target, "rb") as f:
                shutil.copyfileobj(f, sys.stdout.buffer)
            sys.stdout.flush()
        return 0
    except L.DwpaError as e:
        pprint(f"hashcat --stdout replacement failed: {e}", "FAIL")
        return -1
    finally:
        for t in tmp:
            if os.path.exists(t):
                os.unlink(t)


class SubprocessShim:
    """help_crack's module-level ``subprocess`` after install(): ``call`` answers a ``hashcat --stdout`` command line
    (help_crack.py:508-509 expandcracked, :575-576 prdict) with hashcat_stdout on the GPU; every other attribute and
    call is the real module's (hcxpsktool :645, imeigen :684 run as before)."""

    def __init__(self, real, device: int = 0):
        self._real = real
        self._device = device

    def __getattr__(self, name):
        return getattr(self._real, name)

    def call(self, args, *a, **kw):
        argv = shlex.split(args) if isinstance(args, str) else list(args)
        if is_hashcat_stdout(argv):
            return hashcat_stdout(argv, self._device)
        return self._real.call(args, *a, **kw)


def install(helpcrack_cls, device: int = 0):
    """Bind the GPU engine into help_crack's ``HelpCrack`` class (help_crack/help_crack.py:56) and module, so that
    ``HelpCrack.run()`` (:881-957) runs end to end on a box with no hashcat or john binary:

    * ``check_tools`` (:191-307): no binary search; exits like the original (:288-290) when no gfx950 device is
      usable, else sets ``conf["cracker"]`` and ``conf["format"] = "22000"`` and returns the cracker name;
    * ``run_cracker`` (:765-802): dwpa_amd.help_crack.run_cracker over ``self.conf``, with the instance's
      ``sleepy``/``pprint`` and ``disablestdout`` as ``quiet``;
    * the module's ``subprocess`` becomes a SubprocessShim, so the ``hashcat --stdout`` expansions of
      ``expandcracked`` (:508) and ``prepare_dicts`` (:575) run on the GPU (``device``) unchanged.

    Rule files (the server's ``rules``, :445-447, and the ``-r`` of both expansions) load as hashcat's ``-r`` does by
    default: a line using a reject function (``< > _ ! / ( ) = % Q``) or a memory function (``M 4 6 X``) is skipped
    and counted.  Which lines hashcat -r skips is third-party behaviour no reference file pins (parity unpinned);
    set ``DWPA_RULE_MODE=full`` in the environment (or ``rule_mode=DWPA_RULES_FULL``) if your rules rely on those
    functions and should run them.

    Idempotent.  Returns the class."""
    module = sys.modules.get(helpcrack_cls.__module__)

    def check_tools(self):
        try:
            ndev = M.device_count()
        except L.DwpaError:
            ndev = 0
        if ndev < 1:
            self.pprint("libdwpa22000: no usable gfx950 device (hashcat is not needed)", "FAIL")
            sys.exit(1)
        self.conf["cracker"] = CRACKER
        self.conf["format"] = "22000"
        return self.conf["cracker"]

    def run_cracker_method(self, dictlist, disablestdout=False):
        return run_cracker(self.conf, dictlist, sleepy=self.sleepy, pprint=self.pprint, quiet=disablestdout)

    check_tools.__doc__ = "help_crack.py:191-307 without a cracker binary (dwpa_amd.help_crack.install)"
    run_cracker_method.__doc__ = "help_crack.py:765-802 in-process on the GPU (dwpa_amd.help_crack.install)"
    helpcrack_cls.check_tools = check_tools
    helpcrack_cls.run_cracker = run_cracker_method
    if module is not None and hasattr(module, "subprocess") and not isinstance(module.subprocess, SubprocessShim):
        module.subprocess = SubprocessShim(module.subprocess, device)
    return helpcrack_cls
