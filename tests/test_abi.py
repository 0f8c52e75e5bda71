"""CPU: the C-ABI library loads, exports every symbol include/dwpa22000.h declares, its host-only helpers match
the oracle, and compute entry points fail loudly (no CPU fallback) when there is no GPU."""
import ctypes
import os
import re

import pytest

from dwpa_amd import _lib as L
from oracle import oracle as O
from dwpa_amd import synth as S


def declared_symbols():
    txt = open(L.HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dwpa_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_boundary():
    syms = declared_symbols()
    for s in ["dwpa_check_m22000", "dwpa_check_batch", "dwpa_pbkdf2_pmk", "dwpa_crack_files", "dwpa_scan_create",
              "dwpa_init", "dwpa_strerror", "dwpa_shutdown"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = L.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    for s in L.SIGNATURES:
        assert hasattr(lib, s), s


def test_abi_version_and_strerror():
    lib = L.load()
    assert lib.dwpa_abi_version() == 1
    for code in [0, 1, -1, -2, -3, -4, -10, -12, -13, -14, -15, -16, -999]:
        assert lib.dwpa_strerror(code)


def test_hc_unhex_matches_oracle():
    import dwpa_amd
    for k in [b"$HEX[414243]", b"$HEX[]", b"$HEX[41424]", b"$HEX[41zz]", b"$HEX[4142]x", b"plain", b"$HEX[00ff]",
              b"$HEX[AbCd]", b"$HEX[", b"1234567"]:
        assert dwpa_amd.hc_unhex(k) == O.hc_unhex(k), k


def test_hash_m22000_matches_oracle():
    import dwpa_amd
    for line in S.CHALLENGE_LINES + [b"WPA*01*a*b*c*d*e*f*g*h*i", b"WPA*01*x", b""]:
        assert dwpa_amd.hash_m22000(line) == O.c_hash_m22000(line)


def _gpu_present():
    return os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "0") != ""


@pytest.mark.skipif(_gpu_present(), reason="a GPU is visible: the no-device path is not reachable")
def test_compute_fails_loudly_without_gpu():
    import dwpa_amd
    from dwpa_amd import DwpaError
    with pytest.raises(DwpaError):
        dwpa_amd.check_key_m22000(S.CHALLENGE_LINES[0], [b"aaaa1234"])
    with pytest.raises(DwpaError):
        dwpa_amd.pbkdf2_pmk([b"password"], b"IEEE")
    lib = L.load()
    assert lib.dwpa_device_count() == L.DWPA_E_NODEV
