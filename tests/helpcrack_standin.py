"""Test double of the reference client's ``HelpCrack`` (help_crack/help_crack.py:56), for the drop-in tests.

The reference itself may not be imported or run here (denied), so this module restates -- as a
behavioural model, not its text -- the methods dwpa_amd.help_crack.install() touches or relies on, with the same
names, ``conf`` keys, file names and subprocess command lines:

* ``check_tools``        :191-307  hashcat/john discovery; exits 1 when neither is on PATH (:286-290)
* ``prepare_challenge``  :690-725  the KAT work unit; the dictionary is gzip when conf["format"] == "22000"
* ``prepare_work``       :428-467  writes m22000 lines and the base64 rules only in format 22000
* ``run_cracker``        :765-802  shells out to conf["cracker"] (replaced by install())
* ``get_key``            :804-879  outfile -> [{"k": MAC_AP, "v": hex(PSK)}], then deletes the file
* ``expandcracked``      :469-509  cracked.txt.gz + rkg.txt.gz -> source.txt -> `hashcat.bin --stdout` (:508)
* ``expand_prdict``      :557-585  the prdict branch of prepare_dicts, `hashcat.bin --stdout` inline (:575)
* ``challenge``          :883-895  run()'s self-test and its acceptance rule (:893)

The module-level ``subprocess`` is what install() replaces, as in help_crack.py.
"""
from __future__ import annotations

import binascii
import gzip
import os
import shlex
import shutil
import subprocess
import sys

CHALLENGE = {
    "hashes": ["WPA*01*8ac36b891edca8eef49094b1afe061ac*1c7ee5e2f2d0*0026c72e4900*646c696e6b***",
               "WPA*02*269a61ef25e135a4b423832ec4ecc7f4*1c7ee5e2f2d0*0026c72e4900*646c696e6b*"
               "dbd249a3e9cec6ced3360fba3fae9ba4aa6ec6c76105796ff6b5a209d18782ca*"
               "0103007702010a00000000000000000000645b1f684a2566e21266f123abc386"
               "cc576f593e6dc5e3823a32fbd4af929f51000000000000000000000000000000"
               "0000000000000000000000000000000000000000000000000000000000000000"
               "00001830160100000fac020100000fac040100000fac023c000000*00"],
    "key": "aaaa1234",
    "dictname": "help_crack.challenge.dict",
}
# the two expansion command lines, verbatim (help_crack.py:508 and :575)
EXPAND_CRACKED = "./hashcat.bin --stdout --quiet -w 4 -o cracked.txt.gz -r bestWPA.rule source.txt"
EXPAND_PRDICT = "./hashcat.bin --stdout --quiet -o prdict.txt.gz -r bestWPA.rule source.txt"


def default_conf():
    return {"hash_file": "help_crack.hash", "key_file": "help_crack.key", "rules_file": "help_crack.rules",
            "additional": None, "format": None, "potfile": None, "cracker": "", "coptions": "", "rules": ""}


class HelpCrack:
    def __init__(self, conf=None):
        self.conf = conf if conf is not None else default_conf()
        self.log = []

    def pprint(self, mess, code="HEADER"):
        self.log.append((code, mess))

    def sleepy(self, sec=123):
        raise AssertionError("sleepy() called: a cracker attempt failed")

    def check_tools(self):
        found = [t for t in ("hashcat", "hashcat.bin") if shutil.which(t)] or \
                ([f"{shutil.which('john')} --format=wpapsk"] if shutil.which("john") else [])
        if not found:
            self.pprint("hashcat or john not found", "FAIL")
            sys.exit(1)
        self.conf["cracker"] = found[0]
        self.conf["format"] = "22000" if "hashcat" in found[0] else "wpapsk"
        return found[0]

    def prepare_challenge(self):
        netdata = dict(CHALLENGE, hashes=list(CHALLENGE["hashes"]))
        if self.conf["format"] == "22000":
            netdata["dictname"] += ".gz"
            with gzip.open(netdata["dictname"], "w") as fd:  # no trailing newline, as :708 writes it
                fd.write(netdata["key"].encode())
        else:
            with open(netdata["dictname"], "w", encoding="utf-8") as fd:
                fd.write(netdata["key"])
        if os.path.exists(self.conf["key_file"]):
            os.unlink(self.conf["key_file"])
        return netdata

    def prepare_work(self, netdata):
        with open(self.conf["hash_file"], "w", encoding="utf-8") as fd:
            for h in netdata["hashes"]:
                if self.conf["format"] != "22000":
                    raise AssertionError("the JtR conversion (m22000john, :441-451) would run")
                fd.write(f"{h}\n")
                if "rules" in netdata:
                    with open(self.conf["rules_file"], "wb") as fdr:
                        fdr.write(binascii.a2b_base64(netdata["rules"]))
                    self.conf["rules"] = f"-S -r {self.conf['rules_file']}"
                else:
                    self.conf["rules"] = ""
        return {"hkey": netdata.get("hkey")}

    def run_cracker(self, dictlist, disablestdout=False):
        cmd = (f"{self.conf['cracker']} -m22000 -w 4 --advice-disable --logfile-disable --potfile-disable "
               f"--nonce-error-corrections=8 --session help_crack {self.conf['rules']} {self.conf['coptions']} "
               f"-o{self.conf['key_file']} {self.conf['hash_file']} " + " ".join(dictlist))
        return subprocess.call(shlex.split(cmd))

    def get_key(self):
        res = []
        if os.path.exists(self.conf["key_file"]):
            with open(self.conf["key_file"], "r", encoding="utf-8", errors="ignore") as fd:
                for line in fd:
                    arr = line.split(":", 4)
                    if len(arr) == 5:
                        res.append({"k": arr[1][:12],
                                    "v": bytes(arr[4].rstrip("\r\n"), encoding="utf-8", errors="ignore").hex()})
        if res:
            os.unlink(self.conf["key_file"])
            return res
        return None

    def download(self, url, filename):  # tests replace it (there is no network)
        raise AssertionError(f"download({url}) not stubbed")

    def expandcracked(self):
        with gzip.open("cracked.txt.gz", "rb") as src, open("cracked.txt", "wb") as dst:
            shutil.copyfileobj(src, dst)
        self.download("https://wpa-sec.stanev.org/dict/rkg.txt.gz", "rkg.txt.gz")
        with gzip.open("rkg.txt.gz", "rb") as src, open("cracked.txt", "ab") as dst:
            shutil.copyfileobj(src, dst)
        if os.path.exists("source.txt"):
            os.unlink("source.txt")
        os.rename("cracked.txt", "source.txt")
        if os.path.exists("cracked.txt.gz"):
            os.unlink("cracked.txt.gz")
        return subprocess.call(shlex.split(EXPAND_CRACKED), stdout=None)

    def expand_prdict(self, dlist):
        """The prdict branch of prepare_dicts once prdict.txt.gz is downloaded (:560-585)."""
        with gzip.open("prdict.txt.gz", "rb") as src, open("source.txt", "wb") as dst:
            shutil.copyfileobj(src, dst)
        if self.conf["format"] == "22000":
            if os.path.exists("prdict.txt.gz"):
                os.unlink("prdict.txt.gz")
            subprocess.call(shlex.split(EXPAND_PRDICT), stdout=None)
            if os.path.exists("prdict.txt.gz"):
                dlist.insert(0, "prdict.txt.gz")
            else:
                self.pprint("Prdict not found", "FAIL")
        return dlist

    def challenge(self):
        """run()'s self-test (:883-895): True when the acceptance rule of :893 holds (its chained `!=` reduces to
        k0 != k1 because v is hex)."""
        self.check_tools()
        netdata = self.prepare_challenge()
        self.prepare_work(netdata)
        self.run_cracker([netdata["dictname"]], disablestdout=True)
        keypair = self.get_key()
        return bool(keypair) and len(keypair) == 2 and not (keypair[0]["v"] != keypair[1]["v"] != netdata["key"])
