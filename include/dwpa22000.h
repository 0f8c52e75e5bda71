/*
 * dwpa22000.h -- C ABI of libdwpa22000.so, the MI355X (gfx950) m22000 PMK derivation + verification engine.
 *
 * Drop-in boundary for dwpa's one data-parallel hot path (PBKDF2-HMAC-SHA1 x4096 over an ESSID salt, then
 * PMKID / EAPOL keyver 1,2,3 checks with nonce-error-correction).  Two callers bind it:
 *
 *   (1) PHP FFI on the server, in place of check_key_m22000()      web/common.php:157-307
 *       call sites common.php:592 (zero PMK), :606 (PMK reuse), :902 (put_work), :919 (PMK propagation),
 *       web/rkg.php:126,147 (router-keygen / single-mode bulk checks)
 *   (2) Python ctypes in help_crack.py, in place of run_cracker()'s hashcat subprocess
 *       help_crack/help_crack.py:765-802 (command line :773, rc handling :776-786, outfile parsed by get_key :804-879)
 *
 * Plain C types only.  The caller owns every buffer; the library keeps no caller pointer after a call returns and
 * returns no heap memory.  All entry points are thread-safe.
 *
 * Two backends answer the check path (dwpa_check_m22000, dwpa_check_batch) and dwpa_pbkdf2_pmk:
 *   - the gfx950 device (the hot path: PBKDF2 and the verifiers as hand-written HIP kernels);
 *   - the library's host backend (its own SHA-1 / SHA-256 / MD5 / AES-128, with SHA-NI / AES-NI where the CPU has
 *     them, over the host pool's threads), the same semantics and the same results, which answers
 *       (a) small calls -- at least one PBKDF2 derive and at most dwpa_config.host_max_pmks PMK-equivalents (put_work
 *           checks one key per call, common.php:902, and one PBKDF2 chain on a lone GPU wave takes ~8 ms), and
 *       (b) every call, when no usable gfx950 device exists or a device call failed, if allow_cpu_fallback is on.
 *   dwpa_check_last_stats().backend says which one answered a call.  The client path (dwpa_crack_files, dwpa_scan_*,
 *   dwpa_rules_expand*) is device-only: without a device it returns DWPA_E_NODEV / DWPA_RC_ERROR.
 *
 * Concurrent check calls (dwpa_check_m22000 / dwpa_check_batch / dwpa_pbkdf2_pmk from several threads) run on up to
 * DWPA_CALLS_PER_DEVICE (default 2) call contexts per device at once and overlap on the GPU; more callers wait for
 * a free context.  Separate processes (PHP-FPM workers) each hold their own contexts.
 */
#ifndef DWPA22000_H
#define DWPA22000_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DWPA_ABI_VERSION 4   /* 2: dwpa_crack_stats.rules / rules_skipped, dwpa_rules_count; 3: dwpa_check_last_stats,
                                dwpa_config.rule_mode, dwpa_rules_count_ex, dwpa_crack_stats.rules_rejmem; 4: the host
                                backend -- dwpa_config.allow_cpu_fallback / host_max_pmks, dwpa_check_stats.backend */

/* ---- return codes ------------------------------------------------------------------------------------------ */
#define DWPA_MISS 0            /* no key matched (PHP: False)                                                 */
#define DWPA_HIT 1             /* a key matched; the result struct is filled (PHP: [PSK, NC, endian, PMK])   */
#define DWPA_E_FORMAT (-1)     /* not 9 '*'-separated fields or signature != "WPA"   (common.php:159-161)     */
#define DWPA_E_HEX (-2)        /* a required field is not valid even-length hex       (common.php:28-36,162-195) */
#define DWPA_E_TYPE (-3)       /* type field is neither 01 nor 02                     (common.php:167,190,306) */
#define DWPA_E_KEYVER (-4)     /* EAPOL key version not 1/2/3 or EAPOL < 49 bytes     (common.php:274-276)     */
#define DWPA_E_NODEV (-10)     /* no usable gfx950 device (and allow_cpu_fallback off)                         */
#define DWPA_E_HIP (-11)       /* HIP runtime error                                                            */
#define DWPA_E_ARG (-12)       /* invalid argument                                                             */
#define DWPA_E_NOMEM (-13)     /* host or device allocation failed                                             */
#define DWPA_E_IO (-14)        /* file could not be read or written                                            */
#define DWPA_E_OVERFLOW (-15)  /* hit buffer overflow                                                          */
#define DWPA_E_RULE (-16)      /* unsupported or malformed rule                                                */
/* -1..-4 are check_key_m22000's own False returns (malformed line).  Codes <= -10 are device/runtime failures:
 * the result is unknown, so wrappers must not turn them into False (put_work, common.php:902,919, would read
 * "wrong PSK"); php/dwpa22000.php hands such jobs to the original PHP check or throws. */

/* hashcat exit codes returned by dwpa_crack_files (help_crack.py:776-786,930 interpret them) */
#define DWPA_RC_CRACKED 0      /* every hashline cracked                                                       */
#define DWPA_RC_EXHAUSTED 1    /* keyspace exhausted, not every hashline cracked                               */
#define DWPA_RC_ERROR (-1)

/* rule-file loading (dwpa_config.rule_mode; dwpa_crack_files' -r rules and dwpa_rules_expand_file) */
#define DWPA_RULES_DEFAULT 0   /* the process's mode: dwpa_init's rule_mode, else DWPA_RULE_MODE=full|hashcat from the
                                  environment, else DWPA_RULES_HASHCAT                                            */
#define DWPA_RULES_HASHCAT 1   /* hashcat's -r loader: a line using a reject function (< > _ ! / ( ) = % Q) or a memory
                                  function (M 4 6 X) is skipped and counted like an invalid one -- those work only
                                  with -j/-k -- so the candidates are the ones hashcat -r tries (default).  Parity
                                  unpinned: hashcat is not in the reference, no reference file shows which lines -r
                                  skips; this follows hashcat's documentation (oracle/rules.py).  Rules relying on
                                  those functions: DWPA_RULES_FULL / DWPA_RULE_MODE=full                          */
#define DWPA_RULES_FULL 2      /* every line of the whole rule language runs, reject and memory functions included (a
                                  superset of hashcat -r's candidates)                                             */

/* nonce-error-correction semantics */
#define DWPA_NC_PHP 0          /* common.php:250-300: N+0, then V+k,V-k,N+k,N-k for k = 1..(nc>>1)+1, $n mutated */
#define DWPA_NC_HASHCAT 1      /* hashcat --nonce-error-corrections=N: N+0, then +-k, k = 1..N, message_pair bits
                                  0x10 (no NC), 0x20 (LE only), 0x40 (BE only) honoured (third-party semantics)   */
#define DWPA_NC_MAX 65664      /* the largest nc / nonce_error_corrections taken (PHP mode: 131,333 attempts per key).
                                  Every reference call site fits, nets.nc being a smallint (db/wpa.sql:165):
                                  common.php:919 passes |nc| * 2 + 128 <= 65,664, :606 (|nc| << 1) + 1 <= 65,537.  A
                                  larger one on an EAPOL line is DWPA_E_ARG for that job (the PHP wrapper then runs
                                  the original check_key_m22000 if it is kept, else throws); dwpa_scan_create /
                                  dwpa_crack_files refuse it.                                                      */

typedef struct {
    const uint8_t *ptr;        /* NULL = PHP null key (skipped, common.php:172,240) */
    size_t len;
} dwpa_bytes;

typedef struct {
    int32_t key_index;         /* index into keys[] of the first matching key (input order), -1 if none    */
    int32_t nc;                /* nonce correction (DB column nets.nc); valid when nc_valid                */
    int8_t endian;             /* 0 = Null, 1 = 'BE', 2 = 'LE'  (DB column nets.endian)                    */
    uint8_t nc_valid;          /* 0 = PHP Null (PMKID lines), 1 = integer                                  */
    uint8_t reserved[2];
    uint8_t pmk[32];           /* PMK used for the hit (DB column nets.pmk)                                */
} dwpa_result;

typedef struct {
    const char *line;          /* one m22000 hashline (WPA*01*... / WPA*02*...), not NUL-terminated needed  */
    size_t line_len;
    const dwpa_bytes *keys;
    size_t nkeys;
    const uint8_t *pmk;        /* NULL, or 32 bytes used for the first non-null key (common.php:157,178)    */
    int32_t nc;                /* PHP $nc (default 128)                                                    */
} dwpa_job;

typedef struct {
    uint32_t struct_size;      /* sizeof(dwpa_config) */
    uint32_t device_mask;      /* bit d = use device d; 0 = all visible devices */
    uint32_t batch;            /* candidate slots per device per launch; 0 = auto */
    int32_t nc_mode;           /* DWPA_NC_PHP or DWPA_NC_HASHCAT (crack_files default: HASHCAT) */
    int32_t rule_mode;         /* DWPA_RULES_DEFAULT (0) / _HASHCAT / _FULL (ABI 3; was reserved[0]) */
    int32_t allow_cpu_fallback; /* ABI 4 (was reserved[1]), dwpa_init only: 1 = without a usable device, or after a
                                  device call failed (DWPA_E_NODEV / _HIP / _NOMEM / _OVERFLOW), check and PBKDF2
                                  calls run on the host backend; -1 = never; 0 = DWPA_CPU_FALLBACK=1 from the
                                  environment, else never.  With it on, dwpa_init returns 0 without probing for a
                                  device: the first call that needs one probes (a process whose calls all stay on the
                                  host backend never starts the HIP runtime) */
    int32_t host_max_pmks;     /* ABI 4 (was reserved[2]), dwpa_init only: a check call with at least one PBKDF2 derive
                                  and at most this many PMK-equivalents (derives + nonce-correction verify work /
                                  16,388 compressions) runs on the host backend, a dwpa_pbkdf2_pmk call of at most this
                                  many keys too; -1 = never (every call on the device); 0 = DWPA_HOST_MAX_PMKS from
                                  the environment (<= 0: never), else the PMKs the library's host pool derives in
                                  2 ms on this CPU (measured at first use; ~460 on 16 threads of an EPYC 9575F, at
                                  least 8).  Until the process's first device call
                                  completes the threshold is 8x this: that call also starts the HIP runtime (0.2-0.7 s
                                  in a fresh PHP-FPM worker) */
    int32_t reserved[1];
} dwpa_config;

typedef struct {
    uint64_t cand;             /* candidate id: dictionary word index, numeric value, or word*nrules+rule */
    uint32_t line;             /* index of the hashline in the scan's line array */
    int32_t nc;
    int8_t endian;
    uint8_t nc_valid;
    uint8_t reserved[2];
    uint8_t pmk[32];
} dwpa_hit;

/* ---- library ------------------------------------------------------------------------------------------------ */
int dwpa_abi_version(void);
/* Optional: select devices / batch size for the whole process (check path, PBKDF2 and scan calls that follow).
 * Lazy and idempotent; every entry point initialises on first use.  dwpa_crack_files' own cfg applies to that call
 * only and leaves this selection unchanged. */
int dwpa_init(const dwpa_config *cfg);
int dwpa_device_count(void);
const char *dwpa_strerror(int code);
void dwpa_shutdown(void);

/* ---- server-side check: PHP FFI replacement of check_key_m22000 (web/common.php:157-307) -------------------- */
/* Returns DWPA_HIT and fills *out, DWPA_MISS, or a negative code (php/dwpa22000.php: MISS and -1..-4 -> False,
 * codes <= -10 -> the original PHP check_key_m22000, never False). */
int dwpa_check_m22000(const char *line, size_t line_len, const dwpa_bytes *keys, size_t nkeys,
                      const uint8_t *pmk /* nullable, 32 bytes */, int nc, dwpa_result *out);
/* Bulk form (put_work's per-candidate loop, rkg.php's per-net loop): jobs grouped by ESSID internally so
 * each (ESSID, key) PMK is derived once.  rcs[i] / out[i] as for dwpa_check_m22000.  Returns 0 or a
 * negative code if the whole batch failed (device error). */
int dwpa_check_batch(const dwpa_job *jobs, size_t njobs, dwpa_result *out, int *rcs);
/* What the calling thread's last dwpa_check_m22000 / dwpa_check_batch call did (ABI 3): which backend answered it
 * (ABI 4), its jobs, the non-null keys of usable lines (slots), the (ESSID, key) PMKs derived after deduplication (on
 * the host backend: by it; the tail fields below stay 0 there), how many of those formed the device call's tail
 * (the remainder under one wave per SIMD: derived by the host backend beside the head when it fits the head's time,
 * tail_waves 0; else by a tail launch beside the head at low wave priority), the tail launch's waves and how many of
 * them saw the head end and raised their priority, the hits, and the call's wall time.
 * Returns 0, or DWPA_E_ARG before any check call in this thread. */
typedef struct {
    uint32_t jobs;
    uint32_t slots;
    uint32_t pmks;
    uint32_t tail_pmks;
    uint32_t tail_waves;
    uint32_t tail_waves_raised;
    uint32_t hits;
    uint32_t backend;          /* ABI 4: DWPA_BACKEND_* -- who answered the call */
    double seconds;
} dwpa_check_stats;
#define DWPA_BACKEND_DEVICE 0         /* the gfx950 device                                                    */
#define DWPA_BACKEND_HOST_SMALL 1     /* the host backend: a small call (dwpa_config.host_max_pmks)           */
#define DWPA_BACKEND_HOST_FALLBACK 2  /* the host backend: no usable device / a failed device call, with
                                         allow_cpu_fallback on                                               */
int dwpa_check_last_stats(dwpa_check_stats *out);
/* What this process's copy of the library holds right now (ABI 3; host only, never initialises a device): device
 * buffers and pinned host memory of every call context, scan and crack call, the host pool's worker threads (grown
 * on demand up to DWPA_HOST_THREADS - 1), and the call contexts (devices x DWPA_CALLS_PER_DEVICE) and how many of them
 * have run a call.  For sizing PHP-FPM pools, where every worker process loads its own copy. */
typedef struct {
    uint64_t device_bytes;
    uint64_t pinned_host_bytes;
    uint32_t host_pool_threads;
    uint32_t devices;
    uint32_t call_contexts;
    uint32_t call_contexts_used;
} dwpa_resources;
int dwpa_resource_stats(dwpa_resources *out);

/* ---- primitives exposed for parity tests and wrappers ------------------------------------------------------ */
/* PMK = PBKDF2-HMAC-SHA1(key, essid, 4096, 32) for every key (raw bytes, no $HEX[] decoding; a NULL key derives as
 * the empty key).  At most host_max_pmks keys: on the host backend, as the check path routes. */
int dwpa_pbkdf2_pmk(const dwpa_bytes *keys, size_t nkeys, const uint8_t *essid, size_t essid_len,
                    uint8_t *pmks_out /* nkeys * 32 */);
/* hashcat $HEX[...] decoding as web/common.php:3-25; *out_len <= in_len. */
int dwpa_hc_unhex(const uint8_t *in, size_t in_len, uint8_t *out, size_t *out_len);
/* Parse one hashline with check_key_m22000's acceptance rules (common.php:157-237) and describe the nonce-
 * correction attempt lists the verifier would run for `nc` (host only, no device needed).  Returns 0 or the
 * negative parse code.  essid holds the first min(essid_len, 32) bytes of the decoded ESSID and essid_len its full
 * length: PHP accepts longer ESSIDs (any even-length hex, common.php:28-36) and the check uses all of them; only
 * this description is cut.  mac_ap / mac_sta likewise hold the first 16 bytes. */
typedef struct {
    int32_t type;              /* 1 PMKID, 2 EAPOL */
    int32_t keyver;            /* EAPOL key version (0 if unknown) */
    uint32_t essid_len, mac_ap_len, mac_sta_len, target_len;
    uint32_t attempts;         /* attempts per key (1 + 4*((nc>>1)+1) in PHP mode) */
    uint32_t lists;            /* distinct attempt lists (> 1 only when PHP's $n grows, short ANONCE) */
    uint32_t never_matches;    /* PMKID/MIC shorter than 16 bytes */
    uint8_t essid[32];
    uint8_t mac_ap[16], mac_sta[16];
    uint8_t hash_m22000[16];   /* common.php:310-315 dedupe key */
} dwpa_line_info;
int dwpa_parse_m22000(const char *line, size_t line_len, int nc, int nc_mode, dwpa_line_info *out);
/* md5 over fields 1..7 (common.php:310-315); DWPA_E_FORMAT if the line has != 9 fields. */
int dwpa_hash_m22000(const char *line, size_t line_len, uint8_t out[16]);

/* ---- client-side: ctypes replacement of run_cracker() (help_crack.py:765-802) ------------------------------ */
/* Reads hash_file (one m22000 line per line), the dictionaries (plain text or .gz, one word per line, $HEX[]
 * decoded), applies rules_file (hashcat rule syntax, may be NULL) and writes one outfile record per cracked line:
 *   <PMKID|MIC hex>:<MAC_AP hex>:<MAC_STA hex>:<ESSID>:<PSK>   (ESSID/PSK as $HEX[..] when not printable)
 * Returns a hashcat exit code (DWPA_RC_*).  nonce_error_corrections as --nonce-error-corrections.  cfg (nullable):
 * device_mask / batch / nc_mode for this call only (device_mask 0 = the dwpa_init selection, default all devices);
 * a field beyond cfg->struct_size keeps its default (0 = the whole current struct).
 * Lines that can never match (PMKID or MIC shorter than 16 bytes, which hashcat does not load) do not count
 * towards "every hashline cracked".  DWPA_CRACK_SHARDS_PER_DEVICE=k runs k shard workers per device. */
int dwpa_crack_files(const char *hash_file, const char *const *dicts, size_t ndicts, const char *rules_file,
                     int nonce_error_corrections, const char *out_file, const dwpa_config *cfg);
/* dwpa_crack_files plus one outcome per dictionary (dict_status[ndicts], nullable):
 *   DWPA_DICT_OK       read to its end (or not needed: every line cracked first)
 *   DWPA_DICT_DAMAGED  corrupt or truncated gzip stream, by zlib's own verdict: scanned up to the damage, and the
 *                      call still returns 0/1 (hashcat reads wordlists through gzread and does the same).  For a
 *                      truncated stream the words are exactly those of the bytes gzread delivers; for a corrupt body
 *                      or CRC they are at least those (the parallel decoder may deliver the bytes before the failing
 *                      check, and how much gzread drops depends on its buffer and read sizes).  The file should be
 *                      fetched again (help_crack.py:530-534 only downloads a missing file)
 *   DWPA_E_IO          cannot be opened or read: the call returns DWPA_RC_ERROR (before any device work when the
 *                      file cannot be opened, as hashcat refuses to start) */
#define DWPA_DICT_OK 0
#define DWPA_DICT_DAMAGED 1
int dwpa_crack_files_ex(const char *hash_file, const char *const *dicts, size_t ndicts, const char *rules_file,
                        int nonce_error_corrections, const char *out_file, const dwpa_config *cfg,
                        int32_t *dict_status);
/* What the calling thread's last dwpa_crack_files(_ex) call did, for a hashcat-style end-of-run summary
 * (help_crack shows hashcat's output, help_crack.py:776): dictionary words read, candidates derived (inside the
 * 8..63 filter, after the rules), hashlines loaded and cracked, wall time, and the rules file's rules loaded and
 * skipped (a line that does not parse is skipped with a stderr message, as hashcat's "Skipping invalid or
 * unsupported rule"; 0 / 0 without a rules file).  Returns 0, or DWPA_E_ARG before any call in this thread. */
typedef struct {
    uint64_t words;
    uint64_t candidates;
    uint32_t hashes;
    uint32_t cracked;
    double seconds;
    uint32_t rules;            /* rules loaded from rules_file (ABI 2) */
    uint32_t rules_skipped;    /* rule lines of rules_file skipped: not parsing, or (DWPA_RULES_HASHCAT) using reject /
                                  memory functions (ABI 2) */
    uint32_t rules_rejmem;     /* of rules_skipped, the lines skipped for reject / memory functions (ABI 3) */
    uint32_t reserved;
} dwpa_crack_stats;
int dwpa_crack_last_stats(dwpa_crack_stats *out);
/* Per shard worker of the calling thread's last dwpa_crack_files(_ex) call (ABI 4): one worker per selected device
 * (DWPA_CRACK_SHARDS_PER_DEVICE per device), each a stager thread uploading work items and a scanner thread running
 * them.  wait_s is the scanner's time waiting for a staged item (the shared dictionary feed not keeping up), scan_s its
 * time scanning.  Copies min(cap, workers) entries, sets *n = workers; returns 0, or DWPA_E_ARG before any call. */
typedef struct {
    int32_t device;
    uint32_t items;            /* work items (contiguous word ranges of the shared feed) scanned */
    uint64_t words;            /* dictionary words of those items */
    uint64_t candidates;       /* candidates derived (after the rules, inside the 8..63 filter) */
    double wait_s;
    double scan_s;
} dwpa_crack_worker;
int dwpa_crack_worker_stats(dwpa_crack_worker *out, size_t cap, size_t *n);

/* hashcat rules (the whole rule language of hashcat >= 6.2.6: every mangling, reject and memory function; one
 * rule per line, '#' comments; semantics in dwpa_amd/csrc/rules.hpp and oracle/rules.py).  The text entry points
 * below (dwpa_rules_expand, dwpa_rules_apply_host, dwpa_rules_count, dwpa_scan_set_rules) are the interpreter and
 * take every function; the rules *files* of dwpa_crack_files and dwpa_rules_expand_file go through hashcat's -r
 * loader rule unless DWPA_RULES_FULL (dwpa_config.rule_mode / dwpa_init / DWPA_RULE_MODE=full) is selected.
 * GPU rule application (replaces `hashcat --stdout -r rules words`, help_crack.py:508,575): out holds
 * nwords*nrules candidates of 256 bytes (word-major), out_len their lengths (0xFFFFFFFF = the input word or a
 * reject / memory function rejected it).  With out == NULL only *nrules_out is set (number of rules that parse).
 * Rule lines that do not parse are skipped with a stderr message each (out != NULL). */
int dwpa_rules_expand(int device, const char *rules_text, size_t rules_len, const dwpa_bytes *words, size_t nwords,
                      uint8_t *out, uint32_t *out_len, uint32_t *nrules_out);
/* `hashcat --stdout -r rules_file sources... -o out_path` (help_crack.py:508 expandcracked, :575 prdict): every word of
 * the sources (plain or gzip, one per line, $HEX[] decoded) x every rule of rules_file (loaded under the process's
 * rule mode, DWPA_RULES_HASHCAT unless dwpa_init / DWPA_RULE_MODE chose full), expanded on `device`, written to
 * out_path one candidate per line in word-major order, rejected candidates skipped, raw bytes as hashcat's --stdout
 * writes them -- except a candidate holding '\n' or '\r', which would not survive as one line and is written as
 * $HEX[..] (the dictionary readers decode it; hashcat would have split it); gzip_level 0 = plain text (what hashcat
 * writes), 1..9 = gzip.
 * Counts the words read and the candidates written.  Returns 0 or a negative code (DWPA_E_IO: a source cannot be
 * opened or the output cannot be written; DWPA_E_RULE: no valid rule). */
int dwpa_rules_expand_file(int device, const char *rules_file, const char *const *sources, size_t nsources,
                           const char *out_path, int gzip_level, uint64_t *words_out, uint64_t *cands_out);
/* Host only: rule `rule_index` (0-based among the rules that parse) applied to one word by the same interpreter the
 * GPU runs, compiled for the host; *out_len = 0xFFFFFFFF when rejected.  out holds 256 bytes. */
int dwpa_rules_apply_host(const char *rules_text, size_t rules_len, uint32_t rule_index, const uint8_t *word,
                          size_t word_len, uint8_t *out, uint32_t *out_len);
/* Host only: rule lines present (neither empty nor '#' comments), how many of them parse, and the 1-based line
 * number of the first one that does not (0 = none). */
int dwpa_rules_count(const char *rules_text, size_t rules_len, uint32_t *nrules_present, uint32_t *nrules_parsed,
                     uint32_t *first_skipped_line);
/* Host only (ABI 3): both loaders' counts for one rules text -- what DWPA_RULES_FULL loads (parsed) and what
 * hashcat's -r loader (DWPA_RULES_HASHCAT) keeps (loaded_hashcat = parsed - rejmem). */
typedef struct {
    uint32_t present;             /* rule lines (neither empty nor '#' comments)                               */
    uint32_t parsed;              /* lines that parse in the whole language: DWPA_RULES_FULL loads these        */
    uint32_t loaded_hashcat;      /* parsed lines free of reject / memory functions: DWPA_RULES_HASHCAT loads these */
    uint32_t rejmem;              /* parsed lines using a reject or memory function                            */
    uint32_t invalid;             /* lines that do not parse (skipped in both modes)                           */
    uint32_t first_invalid_line;  /* 1-based line numbers, 0 = none                                            */
    uint32_t first_rejmem_line;
    uint32_t reserved;
} dwpa_rules_counts;
int dwpa_rules_count_ex(const char *rules_text, size_t rules_len, dwpa_rules_counts *out);

/* ---- device-resident scan API (inputs already in HBM; used by the client loop and bench.py) --------------- */
typedef struct dwpa_scan dwpa_scan;
/* Upload a work unit's hashlines (any number of ESSIDs) to `device` with a batch of `batch` candidate slots. */
int dwpa_scan_create(int device, const char *const *lines, const size_t *line_lens, size_t nlines, int nc,
                     int nc_mode, uint32_t batch, dwpa_scan **out);
int dwpa_scan_num_groups(const dwpa_scan *scan);              /* number of distinct ESSIDs */
int dwpa_scan_line_status(const dwpa_scan *scan, size_t line); /* 0 usable, or the negative parse code */
/* Stage 1: candidates into the batch.  Dictionary words [first, first+count) of an HBM-resident dictionary
 * (d_offsets: count+1 uint64 byte offsets into d_bytes).  Words outside [minlen, maxlen] are dropped
 * (hashcat m22000 accepts 8..63).  count <= batch. */
int dwpa_scan_load_dict(dwpa_scan *scan, const uint64_t *d_offsets, const uint8_t *d_bytes, uint64_t first,
                        uint32_t count, uint32_t minlen, uint32_t maxlen, void *hip_stream);
/* Rule amplification on the GPU: set the scan's rules once (hashcat rule syntax, one per line), then load
 * words [first_word, first_word+nwords) x every rule; candidate id = word * nrules + rule, 8..63 filter applied.
 * nwords * nrules must be <= batch.  Returns the number of rules that parsed (set) or 0 (load). */
int dwpa_scan_set_rules(dwpa_scan *scan, const char *rules_text, size_t rules_len);
int dwpa_scan_load_rules(dwpa_scan *scan, const uint64_t *d_offsets, const uint8_t *d_bytes, uint64_t first_word,
                         uint32_t nwords, void *hip_stream);
/* Decimal keyspace first..first+count-1, zero-padded to `digits` characters. */
int dwpa_scan_load_numeric(dwpa_scan *scan, uint64_t first, uint32_t count, uint32_t digits, void *hip_stream);
/* Stages 2 and 3 for ESSID group g (PMKs of the loaded batch, then every uncracked line of that ESSID). */
int dwpa_scan_pbkdf2(dwpa_scan *scan, int group, void *hip_stream);
int dwpa_scan_verify(dwpa_scan *scan, int group, void *hip_stream);
/* Stages 2 and 3 for every ESSID group that still has an uncracked line: one PBKDF2 launch covers as many groups
 * x the loaded batch as fit 16M candidate slots (the ESSID salt is wave-uniform), followed by one verify launch
 * over all of their uncracked lines.  Hits are the same as the per-group calls'.  batch must be a multiple of
 * 64 (dwpa_scan_create rounds it up). */
int dwpa_scan_run(dwpa_scan *scan, void *hip_stream);
/* Synchronises the stream and copies the hits found since the last call into out[0..min(*nhits, cap)).  *nhits is
 * the number found, which can exceed cap; the hits beyond cap are lost, because the call also clears the device's
 * hit buffer.  A cap of at least the scan's batch size always suffices: a batch yields at most one hit per
 * candidate slot and line. */
int dwpa_scan_hits(dwpa_scan *scan, dwpa_hit *out, size_t cap, size_t *nhits, void *hip_stream);
/* Candidate slots filled by the last load (synchronises). */
int dwpa_scan_loaded(dwpa_scan *scan, uint32_t *count, void *hip_stream);
void dwpa_scan_destroy(dwpa_scan *scan);

/* ---- device plumbing for callers without their own HIP runtime (ctypes/PHP) ---------------------------------
 * Buffers, streams and events of the runtime the kernels run on.  Callers that already hold HIP objects from a
 * different HIP runtime instance (e.g. a framework bundling its own libamdhip64) must not pass them here. */
int dwpa_dev_alloc(int device, size_t bytes, void **out);
int dwpa_dev_free(int device, void *p);
int dwpa_dev_upload(int device, void *dst, const void *src, size_t bytes);
int dwpa_dev_download(int device, void *dst, const void *src, size_t bytes);
int dwpa_stream_create(int device, void **out);
int dwpa_stream_sync(void *stream);
int dwpa_stream_destroy(void *stream);
int dwpa_event_create(int device, void **out);
int dwpa_event_record(void *event, void *stream);
int dwpa_event_elapsed_ms(void *start, void *stop, float *ms); /* synchronises on stop */
int dwpa_event_destroy(void *event);

#ifdef __cplusplus
}
#endif
#endif /* DWPA22000_H */
