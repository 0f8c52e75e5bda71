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
