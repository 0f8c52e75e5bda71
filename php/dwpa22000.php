<?php
/*
 * PHP FFI binding of libdwpa22000.so for dwpa's server (PHP >= 8.1 with ext/ffi, `ffi.enable=true` or preload).
 *
 * check_key_m22000_gpu() is a drop-in for check_key_m22000() (web/common.php:157-307): same arguments, same
 * return value (False or [PSK, NC, 'BE'|'LE'|Null, PMK]).  check_keys_m22000_gpu_batch() takes many
 * [hashline, keys, pmk, nc] jobs at once (put_work's loop, common.php:900-925; rkg.php:126,147) so every
 * (ESSID, key) PMK is derived once on the GPU.  Every negative library code maps to False, as the PHP
 * function's own early returns do.  Needs hc_unhex() from common.php for the returned PSK.
 *
 * Not exercised in this repository's CI: the build image has no PHP interpreter (SURVEY.md §8c); the same
 * C entry points are exercised through ctypes by tests/test_gpu_parity.py.
 */

final class Dwpa22000
{
    private static $ffi = null;

    public static function ffi()
    {
        if (self::$ffi === null) {
            $cdef = <<<'CDEF'
typedef struct { const uint8_t *ptr; size_t len; } dwpa_bytes;
typedef struct { int32_t key_index; int32_t nc; int8_t endian; uint8_t nc_valid; uint8_t reserved[2]; uint8_t pmk[32]; } dwpa_result;
typedef struct { const char *line; size_t line_len; const dwpa_bytes *keys; size_t nkeys; const uint8_t *pmk; int32_t nc; } dwpa_job;
int dwpa_check_m22000(const char *line, size_t line_len, const dwpa_bytes *keys, size_t nkeys, const uint8_t *pmk, int nc, dwpa_result *out);
int dwpa_check_batch(const dwpa_job *jobs, size_t njobs, dwpa_result *out, int *rcs);
const char *dwpa_strerror(int code);
CDEF;
            $lib = getenv('DWPA_LIB') ?: (defined('DWPA_LIB') ? DWPA_LIB : '/opt/dwpa/libdwpa22000.so');
            self::$ffi = FFI::cdef($cdef, $lib);
        }
        return self::$ffi;
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

    public static function pmk($pmk)
    {
        if (!$pmk) {                                 // common.php:178 -- `if (!$pmk)`
            return null;
        }
        $b = self::ffi()->new('uint8_t[32]');
        FFI::memcpy($b, substr(str_pad((string) $pmk, 32, "\0"), 0, 32), 32);
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
    $ffi = Dwpa22000::ffi();
    [$arr, $keep, $vals] = Dwpa22000::keys($keys);
    $pm = Dwpa22000::pmk($pmk);
    $res = $ffi->new('dwpa_result');
    $rc = $ffi->dwpa_check_m22000($hashline, strlen($hashline), $arr, count($vals),
                                  $pm === null ? null : FFI::addr($pm[0]), (int) $nc, FFI::addr($res));
    if ($rc != 1) {
        return False;
    }
    return Dwpa22000::result($vals, $res);
}

/* $jobs: list of [hashline, keys, pmk (False for none), nc]; returns a list of check_key_m22000 results */
function check_keys_m22000_gpu_batch($jobs)
{
    $ffi = Dwpa22000::ffi();
    $n = count($jobs);
    if ($n == 0) {
        return [];
    }
    $cj = $ffi->new("dwpa_job[$n]");
    $keep = [];
    $vals = [];
    foreach (array_values($jobs) as $i => $job) {
        [$line, $keys, $pmk, $nc] = $job + [null, [], False, 128];
        [$arr, $k, $v] = Dwpa22000::keys($keys);
        $pm = Dwpa22000::pmk($pmk);
        $lb = $ffi->new('char[' . max(1, strlen($line)) . ']');
        FFI::memcpy($lb, $line, strlen($line));
        $keep[] = [$arr, $k, $pm, $lb];
        $vals[] = $v;
        $cj[$i]->line = FFI::addr($lb[0]);
        $cj[$i]->line_len = strlen($line);
        $cj[$i]->keys = FFI::addr($arr[0]);
        $cj[$i]->nkeys = count($v);
        $cj[$i]->pmk = $pm === null ? null : FFI::addr($pm[0]);
        $cj[$i]->nc = (int) $nc;
    }
    $out = $ffi->new("dwpa_result[$n]");
    $rcs = $ffi->new("int[$n]");
    if ($ffi->dwpa_check_batch($cj, $n, $out, $rcs) < 0) {
        return array_fill(0, $n, False);
    }
    $res = [];
    for ($i = 0; $i < $n; $i++) {
        $res[] = $rcs[$i] == 1 ? Dwpa22000::result($vals[$i], $out[$i]) : False;
    }
    return $res;
}
