"""CPU: the C-ABI library loads, exports every symbol include/dwpa22000.h declares, and its host-only helpers match
the oracle.  What compute calls do without a GPU (DWPA_E_NODEV, or the host backend when asked for) is
tests/test_host_backend.py::test_routing_without_a_device."""
import ctypes
import os
import re

import pytest

from dwpa_amd import _lib as L
from oracle import oracle as O
from tests import synth as S


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
    assert lib.dwpa_abi_version() == 4  # 4: host backend (allow_cpu_fallback, host_max_pmks, check_stats.backend)
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


def test_line_info_long_essid_prefix_and_length():
    """dwpa_line_info.essid holds the first 32 bytes of a longer ESSID and essid_len the full length (PHP accepts
    any even-length hex ESSID, common.php:28-36; the check itself salts with all of it)."""
    import dwpa_amd
    essid = bytes(range(65, 65 + 52))
    line = S.pmkid_line(b"password", essid, bytes(6), bytes([1] * 6))
    info = L.LineInfo()
    assert L.load().dwpa_parse_m22000(line, len(line), 128, L.DWPA_NC_PHP, ctypes.byref(info)) == 0
    assert info.essid_len == 52
    assert bytes(info.essid) == essid[:32]
    d = dwpa_amd.parse_m22000(line)
    assert (d["essid"], d["essid_len"]) == (essid[:32], 52)


def _structs(txt):
    """typedef struct { fields } name;  ->  {name: [normalised field declarations]}"""
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for body, name in re.findall(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", txt, flags=re.S):
        out[name] = [" ".join(f.split()) for f in body.split(";") if f.strip()]
    return out


def test_php_ffi_cdef_matches_header():
    """php/dwpa22000.php declares the ABI again for FFI::cdef (the server binding, common.php:157-307); its structs
    and prototypes must stay identical to include/dwpa22000.h (PHP is not installed here, so this is the check)."""
    php = open(os.path.join(os.path.dirname(L.HEADER), "..", "php", "dwpa22000.php")).read()
    cdef = re.search(r"<<<'CDEF'(.*?)CDEF;", php, flags=re.S).group(1)
    hdr = open(L.HEADER).read()
    hs, ps = _structs(hdr), _structs(cdef)
    assert ps, "no structs in the PHP cdef"
    for name, fields in ps.items():
        assert hs.get(name) == fields, name
    def norm(s):
        s = " ".join(re.sub(r"/\*.*?\*/", "", s, flags=re.S).split())
        return re.sub(r"\s+([,);])", r"\1", s)
    for proto in re.findall(r"^\s*((?:int|const char \*)\s*dwpa_\w+\(.*?\);)", cdef, flags=re.M | re.S):
        assert norm(proto) in norm(hdr), proto


def test_nc_bound():
    """DWPA_NC_MAX: the header's bound, what it admits, and DWPA_E_ARG above it for EAPOL lines only (PHP ignores nc
    for PMKID lines); the PHP wrapper answers such a job with the original check_key_m22000 (codes <= -10)."""
    from dwpa_amd import m22000 as M
    hdr = open(L.HEADER).read()
    assert re.search(r"#define DWPA_NC_MAX (\d+)", hdr).group(1) == str(L.DWPA_NC_MAX)
    pmkid, eapol = S.CHALLENGE_LINES
    info = M.parse_m22000(eapol, L.DWPA_NC_MAX)
    assert info["attempts"] == 1 + 4 * ((L.DWPA_NC_MAX >> 1) + 1)
    assert M.parse_m22000(eapol, L.DWPA_NC_MAX, L.DWPA_NC_HASHCAT)["attempts"] == 1 + 4 * L.DWPA_NC_MAX
    assert M.parse_m22000(eapol, L.DWPA_NC_MAX + 1) == L.DWPA_E_ARG
    assert M.parse_m22000(eapol, 2**31 - 1, L.DWPA_NC_HASHCAT) == L.DWPA_E_ARG
    assert M.parse_m22000(eapol, -(2**31))["attempts"] == 1
    assert M.parse_m22000(pmkid, 2**31 - 1)["attempts"] == 1
    assert L.DWPA_E_ARG <= -10  # so php/dwpa22000.php falls back, never answers False


_NOMEM_CHILD = r"""
import ctypes, resource, sys
sys.path.insert(0, sys.argv[1])
from dwpa_amd import _lib as L
lib = L.load()
text = b":\n" * 20_000_000  # 40 MB of rules: the parsed set needs several times that
c = L.RulesCounts()
soft, hard = resource.getrlimit(resource.RLIMIT_AS)
vm = int([l for l in open("/proc/self/status") if l.startswith("VmSize")][0].split()[1]) * 1024
resource.setrlimit(resource.RLIMIT_AS, (vm + (64 << 20), hard))
rc = lib.dwpa_rules_count_ex(text, len(text), ctypes.byref(c))
print(rc)
"""


def test_no_exception_crosses_the_c_abi():
    """A host allocation that fails inside the library (std::bad_alloc) comes back as DWPA_E_NOMEM instead of
    aborting the caller's process (a PHP-FPM worker, help_crack): the child caps its address space, then asks the
    library to parse a rules text whose tables do not fit."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _NOMEM_CHILD, root], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == str(L.DWPA_E_NOMEM), (r.stdout, r.stderr[-2000:])


def test_python_nc_outside_int32_is_refused():
    """ctypes would wrap an nc outside int32 into a different window; the Python API refuses it before any call."""
    import dwpa_amd
    pmkid = S.CHALLENGE_LINES[0]
    for nc in (2**31, -2**31 - 1, 2**40 + 8):
        with pytest.raises(L.DwpaError) as e:
            dwpa_amd.check_key_m22000(pmkid, [b"aaaa1234"], False, nc)
        assert e.value.code == L.DWPA_E_ARG
        with pytest.raises(L.DwpaError):
            dwpa_amd.check_batch([(pmkid, [b"aaaa1234"], False, nc)])


def test_plain_c_client(tmp_path):
    """The header is plain C99 (what PHP FFI::cdef and any C caller consume): tools/abi_c_client.c compiles against it
    with -Wall -Wextra -Werror, links libdwpa22000.so and checks the reference's challenge (help_crack.py:692-699) with
    dwpa_check_m22000 and dwpa_check_batch, the host backend allowed (no GPU here: it answers)."""
    import subprocess
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "abi_c_client"
    lib = os.path.join(ROOT, "dwpa_amd", "lib")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tools", "abi_c_client.c"), "-L", lib, "-ldwpa22000",
                    "-Wl,-rpath," + lib, "-o", str(exe)], check=True)
    env = dict(os.environ, DWPA_HOST_MAX_PMKS="1000000000")
    r = subprocess.run([str(exe)] + [l.decode() for l in S.CHALLENGE_LINES], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "line 1: rc 1 key_index 1 nc_valid 1 nc 4 endian 2" in r.stdout and "batch: both hit" in r.stdout
