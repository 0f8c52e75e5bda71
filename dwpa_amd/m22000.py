"""Python host side of libdwpa22000.so, mirroring dwpa's own interfaces for the m22000 path.

``check_key_m22000`` keeps the exact call signature and return shape of the PHP function it replaces
(web/common.php:157-307): ``False`` or ``[PSK, NC, endian, PMK]`` with ``NC``/``endian`` ``None`` for PMKID
lines, ``endian`` in ``{None, 'BE', 'LE'}``, ``PSK`` after ``$HEX[]`` decoding and ``PMK`` as 32 raw bytes.
The arithmetic runs in libdwpa22000.so: on the GPU, or on the library's host backend for small calls and (only when
asked for, ``init(allow_cpu_fallback=1)``) without a device; otherwise a call without a device raises ``DwpaError``.
"""
from __future__ import annotations

import ctypes

from . import _lib as L

_ENDIAN = {0: None, 1: "BE", 2: "LE"}


def _b(x) -> bytes:
    if isinstance(x, str):
        return x.encode("utf-8", "surrogateescape")
    return bytes(x)


def device_count() -> int:
    return L.check(L.load().dwpa_device_count(), "device_count")


def init(device_mask: int = 0, batch: int = 0, rule_mode: int = L.DWPA_RULES_DEFAULT, allow_cpu_fallback: int = 0,
         host_max_pmks: int = 0) -> int:
    """dwpa_init: the process's device selection, check batch, rule-file mode and host backend switches
    (allow_cpu_fallback 1/-1/0 = on/off/DWPA_CPU_FALLBACK; host_max_pmks n/-1/0 = small-call threshold/never/
    DWPA_HOST_MAX_PMKS or the PMKs the host pool derives in 2 ms).  Returns 0 or raises (DWPA_E_NODEV without a device unless the
    fallback is on)."""
    cfg = L.Config(ctypes.sizeof(L.Config), int(device_mask), int(batch), 0, int(rule_mode), int(allow_cpu_fallback),
                   int(host_max_pmks))
    return L.check(L.load().dwpa_init(ctypes.byref(cfg)), "init")


def hc_unhex(key) -> bytes:
    """common.php:3-25 ($HEX[...] decoding), executed by the library's host code."""
    k = _b(key)
    out = ctypes.create_string_buffer(max(1, len(k)))
    n = ctypes.c_size_t(0)
    L.check(L.load().dwpa_hc_unhex(k, len(k), out, ctypes.byref(n)), "hc_unhex")
    return out.raw[:n.value]


def hash_m22000(hashline):
    """common.php:310-315: raw md5 over fields 1..7, or False."""
    h = _b(hashline)
    out = ctypes.create_string_buffer(16)
    if L.load().dwpa_hash_m22000(h, len(h), out) < 0:
        return False
    return out.raw


def parse_m22000(hashline, nc: int = 128, nc_mode: int = L.DWPA_NC_PHP):
    """Host-side parse (common.php:157-237 acceptance rules): dict of fields, or the negative parse code."""
    h = _b(hashline)
    info = L.LineInfo()
    rc = L.load().dwpa_parse_m22000(h, len(h), int(nc), int(nc_mode), ctypes.byref(info))
    if rc < 0:
        return rc
    return {"type": info.type, "keyver": info.keyver, "essid": bytes(info.essid[:min(32, info.essid_len)]),
            "essid_len": info.essid_len, "mac_ap": bytes(info.mac_ap[:min(16, info.mac_ap_len)]),
            "mac_sta": bytes(info.mac_sta[:min(16, info.mac_sta_len)]), "target_len": info.target_len,
            "attempts": info.attempts, "lists": info.lists, "never_matches": bool(info.never_matches),
            "hash_m22000": bytes(info.hash_m22000)}


def group_by_essid(hashlines):
    """Per-ESSID grouping of a work unit (get_work hands out one ESSID, web/content/get_work.php:96-109);
    duplicate lines (same hash_m22000 key, common.php:310-315) are dropped.  Returns {essid: [lines]}."""
    groups, seen = {}, set()
    for line in hashlines:
        p = parse_m22000(line)
        if isinstance(p, int) or p["hash_m22000"] in seen:
            continue
        seen.add(p["hash_m22000"])
        groups.setdefault(p["essid"] if p["essid_len"] <= 32 else _b(line).split(b"*")[5], []).append(_b(line))
    return groups


def _result(keys, r: L.Result):
    key = keys[r.key_index]
    key = _b(key)
    if key.startswith(b"$HEX["):
        key = hc_unhex(key)
    pmk = bytes(r.pmk)
    if not r.nc_valid:
        return [key, None, None, pmk]
    return [key, int(r.nc), _ENDIAN[int(r.endian)], pmk]


def _nc(nc) -> int:
    """The ABI's nc is an int32: a value outside it would be wrapped by ctypes into a different window."""
    v = int(nc)
    if not -2**31 <= v < 2**31:
        raise L.DwpaError(L.DWPA_E_ARG, f"nc {v} is outside int32")
    return v


def check_key_m22000(hashline, keys, pmk=False, nc: int = 128):
    """Drop-in for PHP check_key_m22000($hashline, $keys, $pmk=False, $nc=128)."""
    h = _b(hashline)
    keys = list(keys)
    arr, keep = L.bytes_array([None if k is None else _b(k) for k in keys])
    res = L.Result()
    pm = bytes(pmk) if pmk else None  # PHP: `if (!$pmk)` -- False/''/None all mean "derive"
    if pm is not None and len(pm) != 32:
        raise ValueError("pmk must be 32 bytes")
    rc = L.check(L.load().dwpa_check_m22000(h, len(h), arr, len(keys), pm, _nc(nc), ctypes.byref(res)),
                 "check_m22000")
    if rc != L.DWPA_HIT:
        return False
    return _result(keys, res)


class BatchJobs:
    """A dwpa_check_batch argument block built once (ctypes job/key arrays) and run any number of times."""

    def __init__(self, jobs):
        jobs = list(jobs)
        self.n = n = len(jobs)
        self.carr = (L.Job * max(1, n))()
        self._keep = []
        self.key_lists = []
        for i, (line, keys, pmk, nc) in enumerate(jobs):
            h = _b(line)
            keys = list(keys)
            arr, k = L.bytes_array([None if x is None else _b(x) for x in keys])
            pm = bytes(pmk) if pmk else None
            self._keep += [h, arr, k, pm]
            self.key_lists.append(keys)
            c = self.carr[i]
            c.line, c.line_len = h, len(h)
            c.keys, c.nkeys = ctypes.cast(arr, ctypes.POINTER(L.Bytes)), len(keys)
            c.pmk, c.nc = pm, _nc(nc)
        self.nkeys = sum(len(k) for k in self.key_lists)
        self.out = (L.Result * max(1, n))()
        self.rcs = (ctypes.c_int * max(1, n))()

    def run(self) -> None:
        L.check(L.load().dwpa_check_batch(self.carr, self.n, self.out, self.rcs), "check_batch")

    def results(self) -> list:
        res = []
        for i in range(self.n):
            if self.rcs[i] == L.DWPA_HIT:
                res.append(_result(self.key_lists[i], self.out[i]))
            else:
                L.check(self.rcs[i], "check_batch job")
                res.append(False)
        return res


def check_stats():
    """dwpa_check_last_stats: {jobs, slots, pmks, tail_pmks, tail_waves, tail_waves_raised, hits, backend, seconds}
    of this thread's last check call (backend: DWPA_BACKEND_DEVICE / _HOST_SMALL / _HOST_FALLBACK)."""
    st = L.CheckStats()
    L.check(L.load().dwpa_check_last_stats(ctypes.byref(st)), "check_last_stats")
    return {k: getattr(st, k) for k, _ in L.CheckStats._fields_ if k != "reserved"}


def resource_stats():
    """dwpa_resource_stats: {device_bytes, pinned_host_bytes, host_pool_threads, devices, call_contexts,
    call_contexts_used} this process's library holds now (host only)."""
    st = L.Resources()
    L.check(L.load().dwpa_resource_stats(ctypes.byref(st)), "resource_stats")
    return {k: getattr(st, k) for k, _ in L.Resources._fields_}


def check_batch(jobs):
    """jobs: iterable of (hashline, keys, pmk_or_False, nc).  Returns a list of check_key_m22000 results."""
    b = BatchJobs(jobs)
    b.run()
    return b.results()


def pbkdf2_pmk(keys, essid) -> list:
    """PMK = PBKDF2-HMAC-SHA1(key, essid, 4096, 32) for every key (raw bytes): on the GPU, or on the host backend for
    at most host_max_pmks keys."""
    keys = [_b(k) for k in keys]
    e = _b(essid)
    arr, keep = L.bytes_array(keys)
    out = ctypes.create_string_buffer(32 * max(1, len(keys)))
    L.check(L.load().dwpa_pbkdf2_pmk(arr, len(keys), e, len(e), out), "pbkdf2_pmk")
    raw = out.raw
    return [raw[32 * i:32 * i + 32] for i in range(len(keys))]


def rules_count(rules_text):
    """(rule lines present, rules that parse, 1-based line of the first that does not or 0) -- host only."""
    rt = _b(rules_text)
    present, parsed, first = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_uint32(0)
    L.check(L.load().dwpa_rules_count(rt, len(rt), ctypes.byref(present), ctypes.byref(parsed), ctypes.byref(first)),
            "rules_count")
    return present.value, parsed.value, first.value


def rules_count_ex(rules_text) -> dict:
    """Both loaders' counts (host only): {present, parsed (DWPA_RULES_FULL loads these), loaded_hashcat (hashcat's
    -r loader keeps these), rejmem, invalid, first_invalid_line, first_rejmem_line}."""
    rt = _b(rules_text)
    c = L.RulesCounts()
    L.check(L.load().dwpa_rules_count_ex(rt, len(rt), ctypes.byref(c)), "rules_count_ex")
    return {k: getattr(c, k) for k, _ in L.RulesCounts._fields_ if k != "reserved"}


def rules_apply_host(rules_text, rule_index: int, word):
    """Rule `rule_index` of rules_text applied to `word` on the host by the GPU's interpreter: bytes or None."""
    rt, w = _b(rules_text), _b(word)
    out = ctypes.create_string_buffer(256)
    n = ctypes.c_uint32(0)
    L.check(L.load().dwpa_rules_apply_host(rt, len(rt), int(rule_index), w, len(w), out, ctypes.byref(n)),
            "rules_apply_host")
    return None if n.value == 0xFFFFFFFF else out.raw[:n.value]


def rules_expand_file(rules_file, sources, out_path, gzip_level: int = 0, device: int = 0):
    """`hashcat --stdout -r rules_file sources -o out_path` on the GPU: returns (words read, candidates written)."""
    src = [_b(x) for x in sources]
    arr = (ctypes.c_char_p * max(1, len(src)))(*src)
    w, c = ctypes.c_uint64(0), ctypes.c_uint64(0)
    L.check(L.load().dwpa_rules_expand_file(device, _b(rules_file), arr, len(src), _b(out_path), int(gzip_level),
                                            ctypes.byref(w), ctypes.byref(c)), "rules_expand_file")
    return w.value, c.value


def rules_expand(rules_text, words, device: int = 0):
    """GPU rule application (hashcat --stdout -r): returns [[candidate or None (rejected)] per rule] per word."""
    rt = _b(rules_text)
    words = [_b(w) for w in words]
    nr = ctypes.c_uint32(0)
    lib = L.load()
    L.check(lib.dwpa_rules_expand(device, rt, len(rt), None, 0, None, None, ctypes.byref(nr)), "rules_expand")
    nrules = nr.value
    if not words or not nrules:
        return [[] for _ in words]
    arr, keep = L.bytes_array(words)
    out = ctypes.create_string_buffer(len(words) * nrules * 256)
    lens = (ctypes.c_uint32 * (len(words) * nrules))()
    L.check(lib.dwpa_rules_expand(device, rt, len(rt), arr, len(words), out, lens, ctypes.byref(nr)), "rules_expand")
    raw = out.raw
    res = []
    for i in range(len(words)):
        row = []
        for r in range(nrules):
            c = i * nrules + r
            n = lens[c]
            row.append(None if n == 0xFFFFFFFF else raw[c * 256:c * 256 + n])
        res.append(row)
    return res


def crack_files(hash_file, dicts, rules_file=None, nonce_error_corrections: int = 8, out_file="help_crack.key",
                device_mask: int = 0, batch: int = 0, nc_mode: int = L.DWPA_NC_HASHCAT,
                rule_mode: int = L.DWPA_RULES_DEFAULT) -> int:
    """In-process hashcat -m22000 replacement; returns a hashcat exit code (0 cracked, 1 exhausted, -1 error).
    rule_mode: DWPA_RULES_DEFAULT (the process's: hashcat's -r loader unless DWPA_RULE_MODE=full), _HASHCAT or _FULL
    (reject / memory lines run too)."""
    return crack_files_ex(hash_file, dicts, rules_file, nonce_error_corrections, out_file, device_mask, batch,
                          nc_mode, rule_mode)[0]


def crack_files_ex(hash_file, dicts, rules_file=None, nonce_error_corrections: int = 8, out_file="help_crack.key",
                   device_mask: int = 0, batch: int = 0, nc_mode: int = L.DWPA_NC_HASHCAT,
                   rule_mode: int = L.DWPA_RULES_DEFAULT):
    """crack_files plus one status per dictionary: (rc, [DWPA_DICT_OK | DWPA_DICT_DAMAGED | DWPA_E_IO])."""
    cfg = L.Config(ctypes.sizeof(L.Config), device_mask, batch, nc_mode, rule_mode)
    dl = [_b(d) for d in dicts]
    darr = (ctypes.c_char_p * max(1, len(dl)))(*dl)
    st = (ctypes.c_int32 * max(1, len(dl)))()
    rc = L.load().dwpa_crack_files_ex(_b(hash_file), darr, len(dl), _b(rules_file) if rules_file else None,
                                      _nc(nonce_error_corrections), _b(out_file), ctypes.byref(cfg), st)
    return rc, [int(st[i]) for i in range(len(dl))]


def crack_stats():
    """dwpa_crack_last_stats: {words, candidates, hashes, cracked, seconds, rules, rules_skipped, rules_rejmem} of
    this thread's last crack call."""
    st = L.CrackStats()
    L.check(L.load().dwpa_crack_last_stats(ctypes.byref(st)), "crack_last_stats")
    return {"words": st.words, "candidates": st.candidates, "hashes": st.hashes, "cracked": st.cracked,
            "seconds": st.seconds, "rules": st.rules, "rules_skipped": st.rules_skipped,
            "rules_rejmem": st.rules_rejmem}


def crack_worker_stats():
    """dwpa_crack_worker_stats: per shard worker of this thread's last crack call, [{device, items, words,
    candidates, wait_s, scan_s}] (wait_s: time its scanner waited for the shared dictionary feed)."""
    lib = L.load()
    n = ctypes.c_size_t(0)
    L.check(lib.dwpa_crack_worker_stats(None, 0, ctypes.byref(n)), "crack_worker_stats")
    arr = (L.CrackWorker * max(1, n.value))()
    L.check(lib.dwpa_crack_worker_stats(arr, n.value, ctypes.byref(n)), "crack_worker_stats")
    return [{k: getattr(arr[i], k) for k, _ in L.CrackWorker._fields_} for i in range(n.value)]


class Scan:
    """Device-resident scan of one work unit (hashlines grouped by ESSID) -- the client hot loop.

    Pointers are raw device addresses (e.g. ``tensor.data_ptr()``), streams raw ``hipStream_t`` handles
    (e.g. ``torch.cuda.Stream.cuda_stream``); 0 = the null stream.
    """

    def __init__(self, lines, device: int = 0, nc: int = 8, nc_mode: int = L.DWPA_NC_PHP, batch: int = 1 << 22):
        self.lines = [_b(x) for x in lines]
        self._lib = L.load()
        n = len(self.lines)
        lp = (ctypes.c_char_p * max(1, n))(*self.lines)
        ll = (ctypes.c_size_t * max(1, n))(*[len(x) for x in self.lines])
        h = ctypes.c_void_p()
        L.check(self._lib.dwpa_scan_create(device, lp, ll, n, _nc(nc), int(nc_mode), int(batch), ctypes.byref(h)),
                "scan_create")
        self._h = h
        self.batch = (int(batch) + 63) & ~63
        self.groups = self._lib.dwpa_scan_num_groups(h)

    def line_status(self, i: int) -> int:
        return self._lib.dwpa_scan_line_status(self._h, i)

    def load_dict(self, d_offsets: int, d_bytes: int, first: int, count: int, minlen=8, maxlen=63, stream: int = 0):
        L.check(self._lib.dwpa_scan_load_dict(self._h, d_offsets, d_bytes, first, count, minlen, maxlen, stream),
                "scan_load_dict")

    def set_rules(self, rules_text) -> int:
        t = _b(rules_text)
        self.nrules = L.check(self._lib.dwpa_scan_set_rules(self._h, t, len(t)), "scan_set_rules")
        return self.nrules

    def load_rules(self, d_offsets: int, d_bytes: int, first_word: int, nwords: int, stream: int = 0):
        L.check(self._lib.dwpa_scan_load_rules(self._h, d_offsets, d_bytes, first_word, nwords, stream),
                "scan_load_rules")

    def load_numeric(self, first: int, count: int, digits: int = 8, stream: int = 0):
        L.check(self._lib.dwpa_scan_load_numeric(self._h, first, count, digits, stream), "scan_load_numeric")

    def pbkdf2(self, group: int = 0, stream: int = 0):
        L.check(self._lib.dwpa_scan_pbkdf2(self._h, group, stream), "scan_pbkdf2")

    def verify(self, group: int = 0, stream: int = 0):
        L.check(self._lib.dwpa_scan_verify(self._h, group, stream), "scan_verify")

    def run(self, stream: int = 0):
        """PBKDF2 + verify of the loaded batch for every ESSID group with an uncracked line, many groups per
        launch (dwpa_scan_run)."""
        L.check(self._lib.dwpa_scan_run(self._h, stream), "scan_run")

    def loaded(self, stream: int = 0) -> int:
        c = ctypes.c_uint32(0)
        L.check(self._lib.dwpa_scan_loaded(self._h, ctypes.byref(c), stream), "scan_loaded")
        return c.value

    def hits(self, stream: int = 0, cap: int = 1 << 16):
        buf = (L.Hit * cap)()
        n = ctypes.c_size_t(0)
        L.check(self._lib.dwpa_scan_hits(self._h, buf, cap, ctypes.byref(n), stream), "scan_hits")
        out = []
        for i in range(min(n.value, cap)):
            h = buf[i]
            out.append({"cand": int(h.cand), "line": int(h.line),
                        "nc": int(h.nc) if h.nc_valid else None,
                        "endian": _ENDIAN[int(h.endian)] if h.nc_valid else None,
                        "pmk": bytes(h.pmk)})
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._lib.dwpa_scan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
