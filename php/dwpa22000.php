<?php
/*
 * PHP FFI binding of libdwpa22000.so for dwpa's server (PHP >= 8.1 with ext/ffi, `ffi.enable=true` or preload).
 *
 * check_key_m22000_gpu() is a drop-in for check_key_m22000() (web/common.php:157-307): same arguments, same
 * return value (False or [PSK, NC, 'BE'|'LE'|Null, PMK]).  check_keys_m22000_gpu_batch() takes many
 * [hashline, keys, pmk, nc] jobs at once (put_work's loop, common.php:900-925; rkg.php:126,147) so every
 * (ESSID, key) PMK is derived once on the GPU.  Needs hc_unhex() from common.php for the returned PSK.
 *
 * Library return code -> behaviour (pinned by tests/test_php_wrapper.py, which parses this file):
 *   DWPA_HIT (1)                                      -> [PSK, NC, endian, PMK]
 *   DWPA_MISS (0), parse codes -1..-4                 -> False, exactly as check_key_m22000's own early returns
 *                                                        (common.php:160-164,276,306)
 *   device / runtime codes <= -10 (NODEV, HIP, ARG,   -> never False: put_work (common.php:902,919) reads False
 *   NOMEM, IO, OVERFLOW, RULE)                           as "this PSK is wrong" and would discard a genuine crack.
 *                                                        The job goes to the original PHP check, kept under the
 *                                                        name check_key_m22000_php (INTEGRATION.md section 2), or,
 *                                                        if that is not defined, a Dwpa22000Error is thrown.
 *   a caller $pmk that is not 32 bytes                 -> the original PHP check as well: PHP HMACs with the PMK's
 *                                                        actual length (common.php:178-188), the ABI takes 32 bytes.
 *
 * Not exercised by a PHP interpreter here: the build image has none (SURVEY.md section 8c); the same C entry
 * points are exercised through ctypes by tests/test_gpu_parity.py.
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
    /* whether this worker process has made a library call yet: its first one also initialises the HIP runtime, loads
     * the code objects and creates the call context (bench.py --workload c1cold, INTEGRATION.md section 2) */
    public static $warm = false;
    /* a cold worker sends a derive to the GPU only from this many keys on: PHP's ~1.1 ms per key then costs about what
     * the first call does (~0.2-0.3 s for a worker started alone, up to ~0.7 s in a start-up storm of 16) */
    const COLD_MIN_KEYS = 256;
    /* DWPA_NC_MAX: the largest nc the library takes; the ABI's nc is an int32 */
    const NC_MAX = 65536;

    public static function ffi()
    {
        if (self::$ffi === null) {
            $cdef = <<<'CDEF'
typedef struct { const uint8_t *ptr; size_t len; } dwpa_bytes;
typedef struct { int32_t key_index; int32_t nc; int8_t endian; uint8_t nc_valid; uint8_t reserved[2]; uint8_t pmk[32]; } dwpa_result;
typedef struct { const char *line; size_t line_len; const dwpa_bytes *keys; size_t nkeys; const uint8_t *pmk; int32_t nc; } dwpa_job;
int dwpa_check_m22000(const char *line, size_t line_len, const dwpa_bytes *keys, size_t nkeys, const uint8_t *pmk, int nc, dwpa_result *out);
int dwpa_check_batch(const dwpa_job *jobs, size_t njobs, dwpa_result *out, int *rcs);
int dwpa_device_count(void);
const char *dwpa_strerror(int code);
CDEF;
            $lib = getenv('DWPA_LIB') ?: (defined('DWPA_LIB') ? DWPA_LIB : '/opt/dwpa/libdwpa22000.so');
            self::$ffi = FFI::cdef($cdef, $lib);
        }
        return self::$ffi;
    }

    /* rc <= -10: the library could not decide (no device, runtime error, ...) -- the answer is not "wrong key" */
    public static function is_device_error($rc)
    {
        return $rc <= self::FIRST_DEVICE_ERROR;
    }

    /* the original PHP check_key_m22000 (renamed check_key_m22000_php), or an exception -- never False */
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
    Dwpa22000::$warm = true;
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
        Dwpa22000::$warm = true;
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

/* Routing by call shape (INTEGRATION.md §2, round-4 latencies in profiles/r04/c1lat.json): a one-key check and a
 * caller-PMK check of a PMKID line stay in PHP (one PBKDF2 on one core, 1.1 ms, against 8.5 ms for the GPU's single
 * PBKDF2 chain; one HMAC, 4 us, against a GPU call's ~0.08 ms); a check of several keys and a caller-PMK check of an
 * EAPOL line (up to 521 PRF + MIC attempts, 2-12x faster on the GPU) go to the library.  Needs
 * check_key_m22000_php, the reference's function renamed; without it everything goes to the library. */
function check_key_m22000_routed($hashline, $keys, $pmk = False, $nc = 128)
{
    if (function_exists('check_key_m22000_php')) {
        $pmkid = strncmp($hashline, 'WPA*01*', 7) === 0;
        if ($pmk ? $pmkid : count($keys) < 2) {
            return check_key_m22000_php($hashline, $keys, $pmk, $nc);
        }
        // a worker's first library call pays the runtime start-up (round 5, profiles/r05/c1cold/): until then only
        // a derive big enough to cost PHP as much goes to the GPU; caller-PMK checks (<= 1.8 ms in PHP) stay in PHP
        if (!Dwpa22000::$warm && ($pmk || count($keys) < Dwpa22000::COLD_MIN_KEYS)) {
            return check_key_m22000_php($hashline, $keys, $pmk, $nc);
        }
    }
    return check_key_m22000_gpu($hashline, $keys, $pmk, $nc);
}

/* Optional, for pools that keep their workers (pm = static, pm.max_requests = 0): pay the start-up in this worker
 * now -- the runtime, the code objects and the call context, through one one-key check of a fixed PMKID line (a
 * miss) -- e.g. from an auto_prepend_file on the worker's first request, so that its later calls are all warm.
 * Returns the number of usable gfx950 devices (0: none -- every check then goes to check_key_m22000_php). */
function dwpa22000_warmup()
{
    $ffi = Dwpa22000::ffi();
    $n = $ffi->dwpa_device_count();
    if ($n > 0) {
        $line = 'WPA*01*' . str_repeat('0', 32) . '*020000000001*020000000002*7761726d7570***';
        [$arr, $keep, $vals] = Dwpa22000::keys(['warmup-key']);
        $res = $ffi->new('dwpa_result');
        $rc = $ffi->dwpa_check_m22000($line, strlen($line), $arr, 1, null, 128, FFI::addr($res));
        Dwpa22000::$warm = $rc >= 0;
    }
    return max(0, $n);
}
