// rules.hpp -- hashcat rule engine (CPU rule-processor semantics, as used by help_crack's `hashcat --stdout -r`
// (help_crack.py:508,575) and `-S -r` (:445-447,931-933)).  Parsing on the host, application on the GPU.
//
// Supported ops: the 16 used by help_crack/bestWPA.rule plus a few neighbours from the same family:
//   :  l  u  c  C  t  r  d  f  {  }  [  ]  q  TN  pN  DN  'N  zN  ZN  $X  ^X  sXY  @X
// Positions N are 0-9 then A-Z (10-35).  Work buffer = hashcat's RP_PASSWORD_SIZE (256): an op whose result
// would not fit leaves the word unchanged.  Rules that fail to parse are skipped (hashcat: "Skipping invalid
// or unsupported rule").  Semantics of the third-party engine are unpinned by the reference's tests.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "dwpa22000.h"

namespace dwpa {

constexpr int RP_PASSWORD_SIZE = 256;

struct RuleOp {
    uint8_t op, p1, p2;
};

struct RuleSet {
    std::vector<std::vector<RuleOp>> rules;
    std::vector<std::string> text;
    size_t size() const { return rules.size(); }
    int load_file(const char* path);
    int add_line(const std::string& line);  // 1 added, 0 skipped (comment/empty/invalid)
    bool all_noop() const;
    std::string apply_host(size_t rule, const std::string& word) const;
    // flat device image: offsets[nrules+1] into a byte code of (op,p1,p2) triples
    void flatten(std::vector<uint32_t>& offs, std::vector<uint8_t>& code) const;
};

struct DevRules {
    int device = -1;
    uint32_t nrules = 0;
    void* offs = nullptr;
    void* code = nullptr;
};

int rules_upload(int device, const RuleSet& rs, DevRules* out);
void rules_release(DevRules* r);
// Stage 1 for word x rule candidates: words [first, first+nwords) of an HBM dictionary, every rule; candidates
// outside 8..63 bytes are dropped; candidate id = word * nrules + rule.
int rules_load(dwpa_scan* scan, const DevRules* r, const uint64_t* off, const uint8_t* bytes, uint64_t first,
               uint32_t nwords, hipStream_t s, bool fill = false);

hipError_t launch_rules_expand(const uint64_t* off, const uint8_t* bytes, uint32_t nwords, const uint32_t* roffs,
                               const uint8_t* rcode, uint32_t nrules, uint8_t* out, uint32_t* out_len,
                               hipStream_t s);
hipError_t launch_rules_prep(const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t nwords,
                             const uint32_t* roffs, const uint8_t* rcode, uint32_t nrules, uint32_t minlen,
                             uint32_t maxlen, uint32_t* mid, uint64_t* ids, uint32_t* counter, uint32_t cap,
                             hipStream_t s);

}  // namespace dwpa
