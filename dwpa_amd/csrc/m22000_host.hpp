// m22000_host.hpp -- hashline parsing (PHP semantics) and device-table building (internal).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "tables.hpp"

namespace dwpa {

// A hashline parsed with the exact acceptance rules of web/common.php:157-195.
struct ParsedLine {
    int status = 0;          // 0 ok, else DWPA_E_*
    int kind = 0;            // LINE_PMKID / LINE_EAPOL
    std::string mac_ap, mac_sta, essid, pmkid, keymic, nonce_ap, eapol, mp;
    int keyver = 0;          // EAPOL key_information & 3 (0 if the frame is < 49 bytes)
    std::string field2_hex;  // PMKID/MIC exactly as written (outfile)
};

ParsedLine parse_m22000(const char* s, size_t n);
void parse_m22000_into(const char* s, size_t n, ParsedLine& p);  // reuses p's string capacity
// False when the line's PMKID / MIC is shorter than 16 bytes: strncmp over 16 bytes never matches
// (common.php:186,280); TableBuilder marks such lines `never`.
inline bool line_can_match(const ParsedLine& p) {
    return (p.kind == LINE_PMKID ? p.pmkid.size() : p.keymic.size()) >= 16;
}

// hashcat $HEX[] decoding as web/common.php:3-25 (only applied to keys starting with "$HEX[")
std::string hc_unhex(const std::string& k);
bool starts_hex(const uint8_t* p, size_t n);

// Host image of the device tables of one work unit.
struct TableBuilder {
    std::vector<LineDev> lines;
    std::vector<AttDev> atts;
    std::vector<uint32_t> pool;  // pre-padded hash blocks (16 words each) and CMAC blocks (4 words each)
    std::vector<uint8_t> never;  // per line: 1 if the line can never match (target shorter than 16 bytes)

    // KW blocks of every attempt's PRF blocks for the key-parallel verifier: always (att_kw_all, scan API), else
    // only for lines with fewer than ATT_PARALLEL_MIN attempts (the check path verifies the others attempt-parallel).
    bool att_kw_all = false;
    // Host backend (host_check.cpp): every block stays a raw 16-word block -- the PMKID message, the PRF prefix and
    // the MIC blocks are not expanded to KW form, and no attempt gets KW blocks.
    bool raw = false;

    // Adds a parsed (status 0) line; returns its index.
    uint32_t add_line(const ParsedLine& p, int nc, int nc_mode, int nec);
};

// PBKDF2 salt blocks for an ESSID: [2][nblk][16] big-endian words of ESSID || INT(i) || SHA1 padding
// (inner hash after the 64-byte ipad block).  Returns nblk.
uint32_t build_salt_blocks(const std::string& essid, std::vector<uint32_t>& out);

// outfile helpers (hashcat outfile-format 1 for -m 22000 as parsed by help_crack.py:807-815)
std::string hex_lower(const std::string& s);
std::string hashcat_plain(const std::string& s);  // printable ASCII without ':' as-is, else $HEX[..]

}  // namespace dwpa
