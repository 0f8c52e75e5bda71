"""CPU: the host backend's check path (dwpa_amd/csrc/host_check.cpp + host_crypto.cpp) under AddressSanitizer +
UBSan.  The host backend answers put_work's checks on the server, so it sees users' hashlines and keys:
tools/host_check_fuzz.cpp sends batches of mutated PMKID / EAPOL keyver 1-3 lines with random, $HEX[], null, empty and
64 KiB keys, caller PMKs and nc from -9 to past DWPA_NC_MAX through host_cost, host_check_batch and host_pbkdf2; any
out-of-bounds access or undefined behaviour aborts the binary."""
import os
import random
import subprocess

from tests import synth as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_check_under_asan(tmp_path):
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/host_check_fuzz_asan"], check=True)
    rng = random.Random(3)
    rows = [(l, b"aaaa1234") for l in S.CHALLENGE_LINES]
    for kv in (1, 2, 3):
        for el in (99, 121, 200, 400):
            essid, ap, sta, _, _ = S.random_net(rng)
            psk = S.fast_psk(rng)
            rows.append((S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), kv,
                                      rng.randint(-3, 3), rng.choice(["LE", "BE"]), eapol_len=el, rng=rng), psk))
    for n in (1, 20, 32):
        essid, ap, sta, _, _ = S.random_net(rng, essid_len=n)
        psk = S.fast_psk(rng)
        rows.append((S.pmkid_line(psk, essid, ap, sta), psk))
    corpus = tmp_path / "corpus.txt"
    corpus.write_bytes(b"".join(l + b"\t" + p + b"\n" for l, p in rows))
    r = subprocess.run([os.path.join(ROOT, "tools", "bin", "host_check_fuzz_asan"), str(corpus), "600"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    f = r.stdout.split()
    assert int(f[3]) > 1500 and int(f[5]) > 50, r.stdout  # jobs run, hits found
