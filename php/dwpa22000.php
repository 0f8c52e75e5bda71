<?php
/*
 * PHP FFI binding of libdwpa22000.so for dwpa's server (PHP >= 8.1 with ext/ffi, `ffi.enable=true` or preload).
 *
 * check_key_m22000_gpu() is a drop-in for check_key_m22000() (web/common.php:157-307): same arguments, same
 * return value (False or [PSK, NC, 'BE'|'LE'|Null, PMK]).  check_keys_m22000_gpu_batch() takes many
 * [hashline, keys, pmk, nc] jobs at once (put_work's loop, common.php:900-925; rkg.php:126,147) so every
 * (ESSID, key) PMK is derived once.  Needs hc_unhex() from common.php for the returned PSK.
 *
 * The library answers every call itself (ABI 4): on the GPU, or on its host backend -- its own SHA-1 / SHA-256 /
 * MD5 / AES-128 on the server's cores -- for small calls (one key, put_work's shape, common.php:902) and, because
 * ffi() turns allow_cpu_fallback on, on a server without a usable GPU or after a failed device call.  So the
 * reference's own function is not needed for correctness; kept under the name check_key_m22000_php it is only the
 * last resort below (INTEGRATION.md section 2).
 *
 * Library return code -> behaviour (pinned by tests/test_php_wrapper.py, which parses this file):
 *   DWPA_HIT (1)                                      -> [PSK, NC, endian, PMK]
 *   DWPA_MISS (0), parse codes -1..-4                 -> False, exactly as check_key_m22000's own early returns
 *                                                        (common.php:160-164,276,306)
 *   runtime codes <= -10 (the host backend failed     -> never False: put_work (common.php:902,919) reads False
 *   too: NOMEM, ...; ARG)                                as "this PSK is wrong" and would discard a genuine crack.
 *                                                        The job goes to check_key_m22000_php if it is defined,
 *                                                        else a Dwpa22000Error is thrown.
 *   a caller $pmk that is not 32 bytes                 -> the same last resort: PHP HMACs with the PMK's actual
 *                                                        length (common.php:178-188), the ABI takes 32 bytes
 *                                                        (nets.pmk is binary(32), db/wpa.sql, so no call site has one).
 *
 * Not exercised by a PHP interpreter here: the build image has none (SURVEY.md section 8c); the same C entry
 * points are exercised through ctypes by tests/test_gpu_parity.py and tests/test_host_backend.py.
 */

final class Dwpa22000Error extends RuntimeException
{
}

final class Dwpa22000
{
    const HIT = 1;
    const MISS = 0;
    const FIRST_DEVICE_ERROR = -10;  /* DWPA_E_NODEV; every code <= this is a device/runtime failure */

    private static $ffi = null;
    /* DWPA_NC_MAX: the largest nc the library takes (every reference call site fits); the ABI's nc is an int32 */
    const NC_MAX = 65664;
    /* dwpa_config.allow_cpu_fallback for this worker: 1 = the host backend answers without a usable GPU */
    const CPU_FALLBACK = 1;

    public static function ffi()
    {
        if (self::$ffi === null) {
            $cdef = <<<'CDEF'
typedef struct { const uint8_t *ptr; size_t len; } dwpa_bytes;
typedef struct { int32_t key_index; int32_t nc; int8_t endian; uint8_t nc_valid; uint8_t reserved[2]; uint8_t pmk[32]; } dwpa_result;
typedef struct { const char *line; size_t line_len; const dwpa_bytes *keys; size_t nkeys; const uint8_t *pmk; int32_t nc; } dwpa_job;
typedef struct { uint32_t struct_size; uint32_t device_mask; uint32_t batch; int32_t nc_mode; int32_t rule_mode; int32_t allow_cpu_fallback; int32_t host_max_pmks; int32_t reserved[1]; } dwpa_config;
int dwpa_init(const dwpa_config *cfg);
int dwpa_check_m22000(const char *line, size_t line_len, const dwpa_bytes *keys, size_t nkeys, const uint8_t *pmk, int nc, dwpa_result *out);
int dwpa_check_batch(const dwpa_job *jobs, size_t njobs, dwpa_result *out, int *rcs);
int dwpa_device_count(void);
const char *dwpa_strerror(int code);
CDEF;
            $lib = getenv('DWPA_LIB') ?: (defined('DWPA_LIB') ? DWPA_LIB : '/opt/dwpa/libdwpa22000.so');
            $ffi = FFI::cdef($cdef, $lib);
            // the host backend answers when this server has no usable GPU (host_max_pmks 0: the library default)
            $cfg = $ffi->new('dwpa_config');
            $cfg->struct_size = FFI::sizeof($cfg);
            $cfg->allow_cpu_fallback = self::CPU_FALLBACK;
            $ffi->dwpa_init(FFI::addr($cfg));
            self::$ffi = $ffi;
        }
        return self::$ffi;
    }

    /* rc <= -10: the library could not decide (its host backend failed too, or an argument it cannot take) -- the
     * answer is not "wrong key" */
    public static function is_device_error($rc)
    {
        return $rc <= self::FIRST_DEVICE_ERROR;
    }

    /* last resort: the original PHP check_key_m22000 if kept (renamed check_key_m22000_php), or an exception --
     * never False */
    public static function fallback($rc, $hashline, $keys, $pmk, $nc)
    {
        if (function_exists('check_key_m22000_php')) {
            return check_key_m22000_php($hashline, $keys, $pmk, $nc);
        }
        $msg = $rc === null ? 'caller PMK is not 32 bytes, or nc is out of range'
                            : FFI::string(self::ffi()->dwpa_strerror($rc));
        throw new Dwpa22000Error("libdwpa22000: $msg (rc $rc)");
    }

    /* an $nc the library reads as PHP does: FFI would wrap a PHP int outside int32, and the library refuses one
     * above DWPA_NC_MAX (an EAPOL job; PHP ignores $nc for PMKID lines, but such calls are left to PHP as well) */
    public static function nc_ok($nc)
    {
        $v = (int) $nc;
        return $v >= -2147483648 && $v <= self::NC_MAX;
    }

    /* a caller PMK the ABI can take: `if (!$pmk)` (common.php:178) means derive; otherwise exactly 32 bytes */
    public static function pmk_ok($pmk)
    {
        return !$pmk || strlen((string) $pmk) == 32;
    }

    /* PHP array of keys -> [dwpa_bytes[], keep-alive buffers, values] */
    public static function keys($keys)
    {
        $ffi = self::ffi();
        $vals = array_values($keys);
        $n = count($vals);
        $arr = $ffi->new('dwpa_bytes[' . max(1, $n) . ']');
        $keep = [];
        foreach ($vals as $i => $k) {
            if (is_null($k)) {                       // common.php:172 -- null keys are skipped
                $arr[$i]->ptr = null;
                $arr[$i]->len = 0;
                continue;
            }
            $k = (string) $k;
            $len = strlen($k);
            $buf = $ffi->new('uint8_t[' . max(1, $len) . ']');
            if ($len) {
                FFI::memcpy($buf, $k, $len);
            }
            $keep[] = $buf;
            $arr[$i]->ptr = FFI::addr($buf[0]);
            $arr[$i]->len = $len;
        }
        return [$arr, $keep, $vals];
    }

    /* 32-byte caller PMK -> uint8_t[32], or null (derive); callers check pmk_ok() first */
    public static function pmk($pmk)
    {
        if (!$pmk) {                                 // common.php:178 -- `if (!$pmk)`
            return null;
        }
        $b = self::ffi()->new('uint8_t[32]');
        FFI::memcpy($b, (string) $pmk, 32);
        return $b;
    }

    public static function result($vals, $res)
    {
        $key = $vals[$res->key_index];
        if (str_starts_with($key, '$HEX[')) {
            $key = hc_unhex($key);
        }
        $pmk = FFI::string($res->pmk, 32);
        if (!$res->nc_valid) {
            return [$key, Null, Null, $pmk];
        }
        $endian = [0 => Null, 1 => 'BE', 2 => 'LE'][$res->endian];
        return [$key, $res->nc, $endian, $pmk];
    }
}

function check_key_m22000_gpu($hashline, $keys, $pmk = False, $nc = 128)
{
    if (!Dwpa22000::pmk_ok($pmk) || !Dwpa22000::nc_ok($nc)) {
        return Dwpa22000::fallback(null, $hashline, $keys, $pmk, $nc);
    }
    $ffi = Dwpa22000::ffi();
    [$arr, $keep, $vals] = Dwpa22000::keys($keys);
    $pm = Dwpa22000::pmk($pmk);
    $res = $ffi->new('dwpa_result');
    $rc = $ffi->dwpa_check_m22000($hashline, strlen($hashline), $arr, count($vals),
                                  $pm === null ? null : FFI::addr($pm[0]), (int) $nc, FFI::addr($res));
    if ($rc == Dwpa22000::HIT) {
        return Dwpa22000::result($vals, $res);
    }
    if (Dwpa22000::is_device_error($rc)) {
        return Dwpa22000::fallback($rc, $hashline, $keys, $pmk, $nc);
    }
    return False;                                    // DWPA_MISS or a parse code (-1..-4)
}

/* $jobs: list of [hashline, keys, pmk (False for none), nc]; returns a list of check_key_m22000 results */
function check_keys_m22000_gpu_batch($jobs)
{
    $jobs = array_values($jobs);
    $n = count($jobs);
    if ($n == 0) {
        return [];
    }
    $ffi = Dwpa22000::ffi();
    $args = [];
    $gpu = [];                                       // indices of the jobs the library checks
    foreach ($jobs as $i => $job) {
        $args[$i] = $job + [null, [], False, 128];
        if (Dwpa22000::pmk_ok($args[$i][2]) && Dwpa22000::nc_ok($args[$i][3])) {
            $gpu[] = $i;
        }
    }
    $res = array_fill(0, $n, False);
    $m = count($gpu);
    $rc = 0;
    if ($m) {
        $cj = $ffi->new("dwpa_job[$m]");
        $keep = [];
        $vals = [];
        foreach ($gpu as $s => $i) {
            [$line, $keys, $pmk, $nc] = $args[$i];
            [$arr, $k, $v] = Dwpa22000::keys($keys);
            $pm = Dwpa22000::pmk($pmk);
            $lb = $ffi->new('char[' . max(1, strlen($line)) . ']');
            FFI::memcpy($lb, $line, strlen($line));
            $keep[] = [$arr, $k, $pm, $lb];
            $vals[$s] = $v;
            $cj[$s]->line = FFI::addr($lb[0]);
            $cj[$s]->line_len = strlen($line);
            $cj[$s]->keys = FFI::addr($arr[0]);
            $cj[$s]->nkeys = count($v);
            $cj[$s]->pmk = $pm === null ? null : FFI::addr($pm[0]);
            $cj[$s]->nc = (int) $nc;
        }
        $out = $ffi->new("dwpa_result[$m]");
        $rcs = $ffi->new("int[$m]");
        $rc = $ffi->dwpa_check_batch($cj, $m, $out, $rcs);
        foreach ($gpu as $s => $i) {
            // the whole batch failed (rc < 0), or this job did: the PHP check decides, never a silent False
            $jrc = $rc < 0 ? $rc : $rcs[$s];
            if ($jrc == Dwpa22000::HIT) {
                $res[$i] = Dwpa22000::result($vals[$s], $out[$s]);
            } elseif ($rc < 0 || Dwpa22000::is_device_error($jrc)) {
                [$line, $keys, $pmk, $nc] = $args[$i];
                $res[$i] = Dwpa22000::fallback($jrc, $line, $keys, $pmk, $nc);
            }                                        // else DWPA_MISS / parse code: False
        }
    }
    foreach ($args as $i => $a) {
        if (!Dwpa22000::pmk_ok($a[2]) || !Dwpa22000::nc_ok($a[3])) {
            $res[$i] = Dwpa22000::fallback(null, $a[0], $a[1], $a[2], $a[3]);
        }
    }
    return $res;
}

/* Since ABI 4 the library routes by call shape itself: a call whose PBKDF2 work the host backend finishes in about
 * 2 ms on this server's cores (one key: 0.24 ms, against PHP's 1.1 ms) runs there, the rest and every caller-PMK
 * check on the GPU.  A worker that has not made a GPU call yet keeps calls of up to 8x that on the host and does not
 * start the HIP runtime until a call needs it (INTEGRATION.md section 2).  check_key_m22000_routed stays as the name
 * earlier deployments call. */
function check_key_m22000_routed($hashline, $keys, $pmk = False, $nc = 128)
{
    return check_key_m22000_gpu($hashline, $keys, $pmk, $nc);
}

/* Optional, for pools whose workers make large calls (pm = static, pm.max_requests = 0): pay the GPU start-up in this
 * worker now -- the runtime, the code objects and the call context, through one 512-key check of a fixed PMKID line
 * (a miss) forced onto the GPU -- e.g. from an auto_prepend_file on the worker's first request.  Workers that only
 * make put_work's small calls need no warm-up: the host backend answers them.  Returns the number of usable gfx950
 * devices (0: none -- every check then runs on the library's host backend). */
function dwpa22000_warmup()
{
    $ffi = Dwpa22000::ffi();
    $n = $ffi->dwpa_device_count();
    if ($n > 0) {
        // this one call on the GPU whatever its size (host_max_pmks -1), then the library's routing again (0)
        $cfg = $ffi->new('dwpa_config');
        $cfg->struct_size = FFI::sizeof($cfg);
        $cfg->allow_cpu_fallback = Dwpa22000::CPU_FALLBACK;
        $cfg->host_max_pmks = -1;
        $ffi->dwpa_init(FFI::addr($cfg));
        $line = 'WPA*01*' . str_repeat('0', 32) . '*020000000001*020000000002*7761726d7570***';
        $keys = [];
        for ($i = 0; $i < 512; $i++) {
            $keys[] = sprintf('warmup-key-%04d', $i);
        }
        [$arr, $keep, $vals] = Dwpa22000::keys($keys);
        $res = $ffi->new('dwpa_result');
        $ffi->dwpa_check_m22000($line, strlen($line), $arr, count($vals), null, 128, FFI::addr($res));
        $cfg->host_max_pmks = 0;
        $ffi->dwpa_init(FFI::addr($cfg));
    }
    return max(0, $n);
}
