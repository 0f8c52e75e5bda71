"""CPU: randomly mutated hashlines (tests/mutate.py) through the library's host-side parse (dwpa_parse_m22000,
dwpa_hash_m22000) against the oracle's check_key_m22000 (web/common.php:157-315).  The parse runs without a
device, so this only checks consistency: a line the oracle verifies with its planted key must parse, a line the
parse rejects must never verify, and the dedupe key must equal the oracle's.  The exact results of the same
mutated jobs through the GPU path are in test_gpu_parity.py::test_mutated_lines_vs_oracle."""
from concurrent.futures import ThreadPoolExecutor

import dwpa_amd
from oracle import oracle as O
from tests.mutate import mutated_jobs


def test_mutated_lines_parse_vs_oracle():
    jobs = mutated_jobs(1, 600)
    with ThreadPoolExecutor(8) as ex:
        exp = list(ex.map(lambda a: O.c_check_key_m22000(*a), jobs))
    rejected = verified = 0
    for (line, keys, pmk, nc), e in zip(jobs, exp):
        p = dwpa_amd.parse_m22000(line, nc)
        if isinstance(p, int):
            rejected += 1
            assert not e, (line, p)
        if e:
            verified += 1
            assert isinstance(p, dict) and not p["never_matches"], (line, p)
            assert p["type"] == (1 if e[1] is None else 2), (line, p)
        assert dwpa_amd.hash_m22000(line) == O.c_hash_m22000(line), line
    # the mutations must exercise both outcomes
    assert rejected > 150 and verified > 30, (rejected, verified)


def test_parse_and_tables_under_asan(tmp_path):
    """The host code that sees untrusted hashlines (parse_m22000, the table builder at nc windows -7..258 in both
    modes, salt blocks, outfile fields, hc_unhex) over 20,000 mutated lines, built with AddressSanitizer + UBSan
    (tools/parse_fuzz.cpp; 600,000 lines ran clean in round 5): any out-of-bounds access or UB aborts the binary."""
    import os
    import random
    import subprocess
    from tests import synth as S
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", root, "tools/bin/parse_fuzz_asan"], check=True)
    rng = random.Random(1)
    lines = list(S.CHALLENGE_LINES)
    for kv in (1, 2, 3):
        for el in (99, 121, 200, 400):
            essid, ap, sta, _, _ = S.random_net(rng)
            lines.append(S.eapol_line(b"password1", essid, ap, sta, rng.randbytes(32), rng.randbytes(32), kv, 2, "LE",
                                      eapol_len=el, rng=rng))
    lines.append(S.pmkid_line(b"password1", b"E" * 32, b"\x01" * 6, b"\x02" * 6))
    corpus = tmp_path / "corpus.txt"
    corpus.write_bytes(b"\n".join(lines) + b"\n")
    r = subprocess.run([os.path.join(root, "tools", "bin", "parse_fuzz_asan"), str(corpus), "20000"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    accepted = int(r.stdout.split()[3])
    assert accepted > 3000, r.stdout
