"""ctypes binding of libdwpa22000.so (include/dwpa22000.h).

Importing works anywhere.  The check path and PBKDF2 run on the gfx950 device, or on the library's own host backend
for small calls and -- only when asked for (dwpa_config.allow_cpu_fallback, DWPA_CPU_FALLBACK=1) -- without a device;
otherwise a call without a device returns DWPA_E_NODEV and the wrappers raise ``DwpaError``, loudly.  The client
path (crack_files, scans, rule expansion) is device-only.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DWPA_LIB", os.path.join(HERE, "lib", "libdwpa22000.so"))
HEADER = os.path.join(os.path.dirname(HERE), "include", "dwpa22000.h")

DWPA_MISS, DWPA_HIT = 0, 1
DWPA_E_FORMAT, DWPA_E_HEX, DWPA_E_TYPE, DWPA_E_KEYVER = -1, -2, -3, -4
DWPA_E_NODEV, DWPA_E_HIP, DWPA_E_ARG, DWPA_E_NOMEM, DWPA_E_IO, DWPA_E_OVERFLOW, DWPA_E_RULE = -10, -11, -12, -13, -14, -15, -16
DWPA_RC_CRACKED, DWPA_RC_EXHAUSTED, DWPA_RC_ERROR = 0, 1, -1
DWPA_NC_PHP, DWPA_NC_HASHCAT = 0, 1
DWPA_NC_MAX = 65664  # the largest nc / nonce_error_corrections taken (include/dwpa22000.h)
DWPA_DICT_OK, DWPA_DICT_DAMAGED = 0, 1  # dwpa_crack_files_ex per-dictionary status (or DWPA_E_IO)
DWPA_RULES_DEFAULT, DWPA_RULES_HASHCAT, DWPA_RULES_FULL = 0, 1, 2  # dwpa_config.rule_mode
DWPA_BACKEND_DEVICE, DWPA_BACKEND_HOST_SMALL, DWPA_BACKEND_HOST_FALLBACK = 0, 1, 2  # dwpa_check_stats.backend


class DwpaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"dwpa error {code}: {msg}")
        self.code = code


class Bytes(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class Result(ctypes.Structure):
    _fields_ = [("key_index", ctypes.c_int32), ("nc", ctypes.c_int32), ("endian", ctypes.c_int8),
                ("nc_valid", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 2), ("pmk", ctypes.c_uint8 * 32)]


class Job(ctypes.Structure):
    _fields_ = [("line", ctypes.c_char_p), ("line_len", ctypes.c_size_t), ("keys", ctypes.POINTER(Bytes)),
                ("nkeys", ctypes.c_size_t), ("pmk", ctypes.c_char_p), ("nc", ctypes.c_int32)]


class Config(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device_mask", ctypes.c_uint32), ("batch", ctypes.c_uint32),
                ("nc_mode", ctypes.c_int32), ("rule_mode", ctypes.c_int32), ("allow_cpu_fallback", ctypes.c_int32),
                ("host_max_pmks", ctypes.c_int32), ("reserved", ctypes.c_int32 * 1)]


class CrackStats(ctypes.Structure):
    _fields_ = [("words", ctypes.c_uint64), ("candidates", ctypes.c_uint64), ("hashes", ctypes.c_uint32),
                ("cracked", ctypes.c_uint32), ("seconds", ctypes.c_double), ("rules", ctypes.c_uint32),
                ("rules_skipped", ctypes.c_uint32), ("rules_rejmem", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class CrackWorker(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("items", ctypes.c_uint32), ("words", ctypes.c_uint64),
                ("candidates", ctypes.c_uint64), ("wait_s", ctypes.c_double), ("scan_s", ctypes.c_double)]


class CheckStats(ctypes.Structure):
    _fields_ = [("jobs", ctypes.c_uint32), ("slots", ctypes.c_uint32), ("pmks", ctypes.c_uint32),
                ("tail_pmks", ctypes.c_uint32), ("tail_waves", ctypes.c_uint32), ("tail_waves_raised", ctypes.c_uint32),
                ("hits", ctypes.c_uint32), ("backend", ctypes.c_uint32), ("seconds", ctypes.c_double)]


class Resources(ctypes.Structure):
    _fields_ = [("device_bytes", ctypes.c_uint64), ("pinned_host_bytes", ctypes.c_uint64),
                ("host_pool_threads", ctypes.c_uint32), ("devices", ctypes.c_uint32), ("call_contexts", ctypes.c_uint32),
                ("call_contexts_used", ctypes.c_uint32)]


class RulesCounts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("present", "parsed", "loaded_hashcat", "rejmem", "invalid",
                                               "first_invalid_line", "first_rejmem_line", "reserved")]


class LineInfo(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("keyver", ctypes.c_int32), ("essid_len", ctypes.c_uint32),
                ("mac_ap_len", ctypes.c_uint32), ("mac_sta_len", ctypes.c_uint32), ("target_len", ctypes.c_uint32),
                ("attempts", ctypes.c_uint32), ("lists", ctypes.c_uint32), ("never_matches", ctypes.c_uint32),
                ("essid", ctypes.c_uint8 * 32), ("mac_ap", ctypes.c_uint8 * 16), ("mac_sta", ctypes.c_uint8 * 16),
                ("hash_m22000", ctypes.c_uint8 * 16)]


class Hit(ctypes.Structure):
    _fields_ = [("cand", ctypes.c_uint64), ("line", ctypes.c_uint32), ("nc", ctypes.c_int32), ("endian", ctypes.c_int8),
                ("nc_valid", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 2), ("pmk", ctypes.c_uint8 * 32)]


_P = ctypes.c_void_p
SIGNATURES = {
    "dwpa_abi_version": ([], ctypes.c_int),
    "dwpa_init": ([ctypes.POINTER(Config)], ctypes.c_int),
    "dwpa_device_count": ([], ctypes.c_int),
    "dwpa_strerror": ([ctypes.c_int], ctypes.c_char_p),
    "dwpa_shutdown": ([], None),
    "dwpa_check_m22000": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(Bytes), ctypes.c_size_t, ctypes.c_char_p,
                           ctypes.c_int, ctypes.POINTER(Result)], ctypes.c_int),
    "dwpa_check_batch": ([ctypes.POINTER(Job), ctypes.c_size_t, ctypes.POINTER(Result), ctypes.POINTER(ctypes.c_int)],
                         ctypes.c_int),
    "dwpa_check_last_stats": ([ctypes.POINTER(CheckStats)], ctypes.c_int),
    "dwpa_resource_stats": ([ctypes.POINTER(Resources)], ctypes.c_int),
    "dwpa_pbkdf2_pmk": ([ctypes.POINTER(Bytes), ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, _P], ctypes.c_int),
    "dwpa_hc_unhex": ([ctypes.c_char_p, ctypes.c_size_t, _P, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "dwpa_hash_m22000": ([ctypes.c_char_p, ctypes.c_size_t, _P], ctypes.c_int),
    "dwpa_parse_m22000": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    "dwpa_crack_files": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, ctypes.c_char_p, ctypes.c_int,
                          ctypes.c_char_p, ctypes.POINTER(Config)], ctypes.c_int),
    "dwpa_crack_last_stats": ([ctypes.POINTER(CrackStats)], ctypes.c_int),
    "dwpa_crack_worker_stats": ([ctypes.POINTER(CrackWorker), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)],
                                ctypes.c_int),
    "dwpa_crack_files_ex": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t, ctypes.c_char_p,
                             ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(Config), ctypes.POINTER(ctypes.c_int32)],
                            ctypes.c_int),
    "dwpa_rules_expand": ([ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(Bytes), ctypes.c_size_t, _P, _P,
                           ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "dwpa_rules_expand_file": ([ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t,
                                ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "dwpa_rules_count": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32),
                          ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "dwpa_rules_count_ex": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(RulesCounts)], ctypes.c_int),
    "dwpa_rules_apply_host": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t, _P,
                               ctypes.POINTER(ctypes.c_uint32)], ctypes.c_int),
    "dwpa_scan_create": ([ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
                          ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(_P)], ctypes.c_int),
    "dwpa_scan_num_groups": ([_P], ctypes.c_int),
    "dwpa_scan_line_status": ([_P, ctypes.c_size_t], ctypes.c_int),
    "dwpa_scan_load_dict": ([_P, _P, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _P],
                            ctypes.c_int),
    "dwpa_scan_set_rules": ([_P, ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "dwpa_scan_load_rules": ([_P, _P, _P, ctypes.c_uint64, ctypes.c_uint32, _P], ctypes.c_int),
    "dwpa_scan_load_numeric": ([_P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _P], ctypes.c_int),
    "dwpa_scan_pbkdf2": ([_P, ctypes.c_int, _P], ctypes.c_int),
    "dwpa_scan_verify": ([_P, ctypes.c_int, _P], ctypes.c_int),
    "dwpa_scan_run": ([_P, _P], ctypes.c_int),
    "dwpa_scan_hits": ([_P, ctypes.POINTER(Hit), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), _P], ctypes.c_int),
    "dwpa_scan_loaded": ([_P, ctypes.POINTER(ctypes.c_uint32), _P], ctypes.c_int),
    "dwpa_scan_destroy": ([_P], None),
    "dwpa_dev_alloc": ([ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(_P)], ctypes.c_int),
    "dwpa_dev_free": ([ctypes.c_int, _P], ctypes.c_int),
    "dwpa_dev_upload": ([ctypes.c_int, _P, _P, ctypes.c_size_t], ctypes.c_int),
    "dwpa_dev_download": ([ctypes.c_int, _P, _P, ctypes.c_size_t], ctypes.c_int),
    "dwpa_stream_create": ([ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "dwpa_stream_sync": ([_P], ctypes.c_int),
    "dwpa_stream_destroy": ([_P], ctypes.c_int),
    "dwpa_event_create": ([ctypes.c_int, ctypes.POINTER(_P)], ctypes.c_int),
    "dwpa_event_record": ([_P, _P], ctypes.c_int),
    "dwpa_event_elapsed_ms": ([_P, _P, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "dwpa_event_destroy": ([_P], ctypes.c_int),
}

_lib = None


def load():
    """Load the shared library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DwpaError(DWPA_E_NODEV, f"{LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
    return _lib


def check(rc: int, what: str = "") -> int:
    if rc < 0 and rc not in (DWPA_E_FORMAT, DWPA_E_HEX, DWPA_E_TYPE, DWPA_E_KEYVER):
        raise DwpaError(rc, (what + ": " if what else "") + load().dwpa_strerror(rc).decode(errors="replace"))
    return rc


def bytes_array(items):
    """Python sequence of bytes/None -> (ctypes array of Bytes, keep-alive list)."""
    arr = (Bytes * max(1, len(items)))()
    keep = []
    for i, k in enumerate(items):
        if k is None:
            arr[i].ptr, arr[i].len = None, 0
        else:
            k = bytes(k)
            b = ctypes.create_string_buffer(k, len(k) + 1)
            keep.append(b)
            arr[i].ptr, arr[i].len = ctypes.cast(b, ctypes.c_void_p), len(k)
    return arr, keep
