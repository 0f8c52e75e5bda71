"""CPU: the PHP FFI wrapper (php/dwpa22000.php) maps library return codes to check_key_m22000 behaviour.

There is no PHP interpreter in this image, so the wrapper's text is parsed and its decisions
are checked against include/dwpa22000.h:

* DWPA_HIT -> the [PSK, NC, endian, PMK] array; DWPA_MISS and the parse codes -1..-4 -> False, as
  check_key_m22000's own early returns (web/common.php:160-164,276,306);
* every runtime code (<= -10; since ABI 4 the library's host backend has already answered a call without a GPU) ->
  the original PHP check if kept (check_key_m22000_php) or an exception, never False: put_work (common.php:902,919)
  reads False as "wrong PSK" and would silently drop a genuine crack;
* a caller $pmk of any length other than 32 -> the original PHP check (PHP HMACs with the actual length,
  common.php:178-188); no padding or truncation.
"""
import os
import re

from dwpa_amd import _lib as L

PHP = os.path.join(os.path.dirname(L.HEADER), "..", "php", "dwpa22000.php")


def _src():
    txt = open(PHP).read()
    # strip comments so that the checks read code only
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return re.sub(r"//[^\n]*", "", txt)


def _header_codes():
    hdr = open(L.HEADER).read()
    return {name: int(v) for name, v in re.findall(r"#define\s+(DWPA_(?:E_\w+|MISS|HIT))\s+\(?(-?\d+)\)?", hdr)}


def _function(src, name):
    """Body of `function name(...) { ... }` (brace matched)."""
    m = re.search(r"function\s+%s\s*\([^)]*\)\s*\{" % re.escape(name), src)
    assert m, name
    depth, i = 1, m.end()
    while depth:
        depth += {"{": 1, "}": -1}.get(src[i], 0)
        i += 1
    return src[m.end():i - 1]


def _const(src, name):
    return int(re.search(r"const\s+%s\s*=\s*(-?\d+)\s*;" % name, src).group(1))


def test_code_classes_match_header():
    src, codes = _src(), _header_codes()
    assert _const(src, "HIT") == codes["DWPA_HIT"] == 1
    assert _const(src, "MISS") == codes["DWPA_MISS"] == 0
    first = _const(src, "FIRST_DEVICE_ERROR")
    assert first == codes["DWPA_E_NODEV"]
    assert "return $rc <= self::FIRST_DEVICE_ERROR;" in _function(src, "is_device_error")
    device = {n for n, v in codes.items() if v <= first}
    parse = {n for n, v in codes.items() if -10 < v < 0}
    assert device == {"DWPA_E_NODEV", "DWPA_E_HIP", "DWPA_E_ARG", "DWPA_E_NOMEM", "DWPA_E_IO", "DWPA_E_OVERFLOW",
                      "DWPA_E_RULE"}
    assert parse == {"DWPA_E_FORMAT", "DWPA_E_HEX", "DWPA_E_TYPE", "DWPA_E_KEYVER"}


def test_fallback_never_returns_false():
    body = _function(_src(), "fallback")
    assert "function_exists('check_key_m22000_php')" in body
    assert "return check_key_m22000_php($hashline, $keys, $pmk, $nc);" in body
    assert re.search(r"throw new Dwpa22000Error", body)
    assert "False" not in body


def _decide(body):
    """The single-call wrapper's decision chain, in order: [(condition, action)]."""
    steps = []
    for cond, act in re.findall(r"if\s*\((.*?)\)\s*\{\s*return\s+(.*?);\s*\}", body, flags=re.S):
        steps.append((" ".join(cond.split()), " ".join(act.split())))
    tail = re.findall(r"return\s+(False);\s*$", body.strip())
    return steps, tail


def test_single_check_code_map():
    body = _function(_src(), "check_key_m22000_gpu")
    steps, tail = _decide(body)
    assert steps == [
        ("!Dwpa22000::pmk_ok($pmk) || !Dwpa22000::nc_ok($nc)",
         "Dwpa22000::fallback(null, $hashline, $keys, $pmk, $nc)"),
        ("$rc == Dwpa22000::HIT", "Dwpa22000::result($vals, $res)"),
        ("Dwpa22000::is_device_error($rc)", "Dwpa22000::fallback($rc, $hashline, $keys, $pmk, $nc)"),
    ]
    assert tail == ["False"]  # reached only for 0 and -1..-4: everything <= -10 returned above


def test_batch_code_map():
    body = _function(_src(), "check_keys_m22000_gpu_batch")
    # no blanket False for a failed batch (round 1 returned array_fill(0, $n, False) on rc < 0)
    assert not re.search(r"return\s+array_fill", body)
    assert "$jrc = $rc < 0 ? $rc : $rcs[$s];" in body
    assert re.search(r"if \(\$jrc == Dwpa22000::HIT\) \{\s*\$res\[\$i\] = Dwpa22000::result", body)
    assert re.search(r"elseif \(\$rc < 0 \|\| Dwpa22000::is_device_error\(\$jrc\)\) \{.*?Dwpa22000::fallback\(\$jrc,",
                     body, flags=re.S)
    # jobs whose PMK or nc the ABI cannot take go to the PHP check, not to the library
    assert "if (Dwpa22000::pmk_ok($args[$i][2]) && Dwpa22000::nc_ok($args[$i][3])) {" in body
    assert re.search(r"if \(!Dwpa22000::pmk_ok\(\$a\[2\]\) \|\| !Dwpa22000::nc_ok\(\$a\[3\]\)\) \{\s*"
                     r"\$res\[\$i\] = Dwpa22000::fallback\(null,", body)


def test_pmk_is_never_padded_or_truncated():
    src = _src()
    pmk = _function(src, "pmk")
    assert "str_pad" not in pmk and "substr" not in pmk
    ok = _function(src, "pmk_ok")
    assert "return !$pmk || strlen((string) $pmk) == 32;" in ok


def test_library_routes_and_falls_back_itself():
    """ABI 4: ffi() turns the library's host backend on for a server without a usable GPU (allow_cpu_fallback), and
    check_key_m22000_routed no longer needs the reference's function: it is the library's own routing (small calls on
    the host backend, the rest on the GPU) under the name earlier deployments call.  dwpa22000_warmup() sends its one
    call to the GPU (host_max_pmks -1 for that call) and then restores the library's routing (0)."""
    src = _src()
    ffi = _function(src, "ffi")
    assert "$cfg->allow_cpu_fallback = self::CPU_FALLBACK;" in ffi and "$ffi->dwpa_init(FFI::addr($cfg));" in ffi
    assert "$cfg->struct_size = FFI::sizeof($cfg);" in ffi
    assert _const(src, "CPU_FALLBACK") == 1
    routed = _function(src, "check_key_m22000_routed")
    assert "check_key_m22000_php" not in routed
    assert routed.strip() == "return check_key_m22000_gpu($hashline, $keys, $pmk, $nc);"
    assert "$warm" not in src and "COLD_MIN_KEYS" not in src
    warm = _function(src, "dwpa22000_warmup")
    off, on = warm.index("$cfg->host_max_pmks = -1;"), warm.index("$cfg->host_max_pmks = 0;")
    call = warm.index("$ffi->dwpa_check_m22000(")
    assert off < call < on and warm.count("$ffi->dwpa_init(FFI::addr($cfg));") == 2
    line = "WPA*01*" + "0" * 32 + "*020000000001*020000000002*7761726d7570***"
    assert "$line = 'WPA*01*' . str_repeat('0', 32) . '*020000000001*020000000002*7761726d7570***';" in warm
    import dwpa_amd
    assert dwpa_amd.parse_m22000(line)["type"] == 1  # the warm-up line is a valid PMKID line


def test_nc_outside_the_abi_goes_to_php():
    """A PHP int outside int32 would be wrapped by FFI, and one above DWPA_NC_MAX is refused by the library: such an
    $nc goes to the original check (the result stays PHP's), for single and batch calls alike."""
    src = _src()
    hdr = open(L.HEADER).read()
    assert _const(src, "NC_MAX") == int(re.search(r"#define DWPA_NC_MAX (\d+)", hdr).group(1)) == L.DWPA_NC_MAX
    ok = _function(src, "nc_ok")
    assert "$v = (int) $nc;" in ok and "return $v >= -2147483648 && $v <= self::NC_MAX;" in ok
