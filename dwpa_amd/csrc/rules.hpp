// rules.hpp -- hashcat rule engine: the whole rule language of hashcat >= 6.2.6 (help_crack.py:46), as help_crack
// uses it through `hashcat --stdout -r` (help_crack.py:508,575) and `-S -r` with the server's merged per-dictionary
// rules (help_crack.py:445-447,931-933; get_work.php:86-92; db/wpa.sql:48).  Parsing on the host, application on
// the GPU (rules_dev.hip); RuleSet::apply_host re-applies a rule on the host to report a hit's PSK.
//
// Functions (N, M, I = position/length 0-9 then A-Z; X, Y = any byte):
//   no argument   :  l  u  c  C  t  r  d  f  {  }  [  ]  k  K  q  E  M  4  6  Q
//   N             TN pN DN zN ZN 'N yN YN LN RN +N -N .N ,N <N >N _N
//   X             $X ^X @X eX !X /X (X )X
//   N X           iNX oNX =NX %NX 3NX
//   X Y           sXY
//   N M           xNM ONM *NM
//   N M I         XNMI
// Work buffer = hashcat's RP_PASSWORD_SIZE (256).  Semantics (bounds, reject and memory functions) are stated in
// oracle/rules.py, the test oracle all three implementations are held to; hashcat itself is third party, so they
// are parity unpinned by the reference.  A rule line that does not parse is skipped and reported (stderr, hashcat's
// "Skipping invalid or unsupported rule", and the counts below), never dropped silently.
//
// Loader modes (RuleSet::mode): rules *files* (dwpa_crack_files' -r, dwpa_rules_expand_file) load as hashcat's -r
// loader does by default (DWPA_RULES_HASHCAT): reject functions (< > _ ! / ( ) = % Q) and memory functions (M 4 6 X)
// work only with -j/-k, so a line using one is skipped and counted like an invalid line and the candidate set is
// exactly hashcat -r's; DWPA_RULES_FULL runs them (a superset).  The text entry points are the interpreter and load
// every function.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "dwpa22000.h"

namespace dwpa {

constexpr int RP_PASSWORD_SIZE = 256;

// One rule function: op byte + up to three arguments (positions already converted to 0..35).  The device image
// stores each as one u32 word {op, p1, p2, p3} (little-endian bytes).
struct RuleOp {
    uint8_t op, p1, p2, p3;
};

// True when the rule uses a reject or a memory function (hashcat's -r loader skips such lines).
bool rule_uses_rejmem(const std::vector<RuleOp>& ops);

struct RuleSet {
    std::vector<std::vector<RuleOp>> rules;
    std::vector<std::string> text;
    int mode = DWPA_RULES_FULL;           // DWPA_RULES_HASHCAT: skip reject / memory lines (files set it)
    uint32_t present = 0;                 // rule lines seen (not empty, not a '#' comment)
    std::vector<std::string> skipped;     // lines skipped: not parsing, or (HASHCAT mode) reject / memory
    std::vector<uint32_t> skipped_lines;  // their 1-based line numbers
    uint32_t rejmem = 0;                  // of skipped, the reject / memory lines (HASHCAT mode)
    std::string source = "rules";         // file name for the messages
    bool quiet = false;                   // no stderr message per skipped line
    size_t size() const { return rules.size(); }
    int load_file(const char* path);
    void load_text(const char* text, size_t len);
    int add_line(const std::string& line, uint32_t lineno = 0);  // 1 added, 0 not a rule, -1 skipped
    bool all_noop() const;
    // the candidate, or false when the input or a reject / memory function rejects it
    bool apply_host(size_t rule, const std::string& word, std::string* out) const;
    // flat device image: offsets[nrules+1] (in ops) into u32 op words
    void flatten(std::vector<uint32_t>& offs, std::vector<uint32_t>& code) const;
};

// Parse one rule line; returns false if it is not a complete rule.  *ops empty for a comment / empty line.
bool parse_rule(const std::string& line, std::vector<RuleOp>* ops, bool* is_rule);

struct DevRules {
    int device = -1;
    uint32_t nrules = 0;
    void* offs = nullptr;
    void* code = nullptr;
};

int rules_upload(int device, const RuleSet& rs, DevRules* out);
void rules_release(DevRules* r);
// Stage 1 for word x rule candidates: words [first, first+nwords) of an HBM dictionary, every rule; candidates
// outside 8..63 bytes (or rejected by a rule) are dropped; candidate id = word * nrules + rule.
int rules_load(dwpa_scan* scan, const DevRules* r, const uint64_t* off, const uint8_t* bytes, uint64_t first,
               uint32_t nwords, hipStream_t s, bool fill = false);

// out: nwords x nrules 256-byte slots, out_len their lengths (0xFFFFFFFF = rejected); text_len (nullable): each
// candidate's bytes in --stdout text (raw + '\n', or $HEX[..] + '\n' when it holds '\n' / '\r'; 0 = rejected).
hipError_t launch_rules_expand(const uint64_t* off, const uint8_t* bytes, uint32_t nwords, const uint32_t* roffs,
                               const uint32_t* rcode, uint32_t nrules, uint8_t* out, uint32_t* out_len,
                               hipStream_t s, uint32_t* text_len = nullptr);
// The --stdout text of candidates [0, n) of a launch_rules_expand with text_len, packed on the GPU in candidate
// order into text: bsum / bcnt scratch of text_pack_blocks(n) words each; tot[0] = text bytes, tot[1] = kept
// candidates (both on the device).  Only candidates whose text ends within `cap` bytes are written: when tot[0] >
// cap, grow text and pack again (the slots are unchanged).
uint32_t text_pack_blocks(uint32_t n);
hipError_t launch_text_pack(const uint8_t* out, const uint32_t* out_len, const uint32_t* text_len, uint32_t n,
                            uint32_t* bsum, uint32_t* bcnt, uint32_t* tot, uint8_t* text, uint64_t cap,
                            hipStream_t s);
hipError_t launch_rules_prep(const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t nwords,
                             const uint32_t* roffs, const uint32_t* rcode, uint32_t nrules, uint32_t minlen,
                             uint32_t maxlen, uint32_t* mid, uint64_t* ids, uint32_t* counter, uint32_t cap,
                             hipStream_t s);

}  // namespace dwpa
