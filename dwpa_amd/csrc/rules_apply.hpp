// rules_apply.hpp -- the rule interpreter, compiled twice: for the GPU (rules_dev.hip: every lane runs it on its own
// candidate, the rule being wave-uniform) and for the host (rules.cpp: re-application of a hit's rule for the
// outfile).  One source, so the PSK written for a hit is by construction the candidate the GPU derived; both are
// held to oracle/rules.py (the restatement of hashcat's rule functions, whose docstring states every bound).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dwpa {

constexpr int RULE_RP = 256;  // hashcat RP_PASSWORD_SIZE
constexpr int RULE_REJECT = -1;

__host__ __device__ __forceinline__ bool rc_lower(uint32_t c) { return c - 'a' < 26u; }
__host__ __device__ __forceinline__ bool rc_upper(uint32_t c) { return c - 'A' < 26u; }
__host__ __device__ __forceinline__ uint8_t rc_tolower(uint8_t c) { return rc_upper(c) ? (uint8_t)(c | 0x20) : c; }
__host__ __device__ __forceinline__ uint8_t rc_toupper(uint8_t c) { return rc_lower(c) ? (uint8_t)(c & 0xdf) : c; }
__host__ __device__ __forceinline__ uint8_t rc_toggle(uint8_t c) {
    return (rc_lower(c) || rc_upper(c)) ? (uint8_t)(c ^ 0x20) : c;
}

// Applies the rule (nops u32 words {op, p1, p2, p3}) to w[0..len) in place.  w and mem hold RULE_RP + 4 bytes.
// orig/orig_len = the input word (the memory until M saves another).  Returns the new length or RULE_REJECT.
__host__ __device__ inline int rule_apply(uint8_t* w, int len, uint8_t* mem, const uint8_t* orig, int orig_len,
                                          const uint32_t* code, uint32_t nops) {
    constexpr int RP = RULE_RP;
    if (len < 1 || len > RP) return RULE_REJECT;
    const uint8_t* mp = orig;  // memory: the input word until M
    int mlen = orig_len;
    for (uint32_t k = 0; k < nops; k++) {
        const uint32_t word = code[k];
        const uint32_t op = word & 0xff, p1 = (word >> 8) & 0xff, p2 = (word >> 16) & 0xff, p3 = word >> 24;
        const int a = (int)p1, b = (int)p2;
        switch (op) {
        case 'l':
            for (int i = 0; i < len; i++) w[i] = rc_tolower(w[i]);
            break;
        case 'u':
            for (int i = 0; i < len; i++) w[i] = rc_toupper(w[i]);
            break;
        case 'c':
            for (int i = 0; i < len; i++) w[i] = rc_tolower(w[i]);
            if (len) w[0] = rc_toupper(w[0]);
            break;
        case 'C':
            for (int i = 0; i < len; i++) w[i] = rc_toupper(w[i]);
            if (len) w[0] = rc_tolower(w[0]);
            break;
        case 't':
            for (int i = 0; i < len; i++) w[i] = rc_toggle(w[i]);
            break;
        case 'T':
            if (a < len) w[a] = rc_toggle(w[a]);
            break;
        case 'r':
            for (int i = 0, j = len - 1; i < j; i++, j--) { uint8_t t = w[i]; w[i] = w[j]; w[j] = t; }
            break;
        case 'd':
            if (2 * len < RP) { for (int i = 0; i < len; i++) w[len + i] = w[i]; len *= 2; }
            break;
        case 'p':
            if (len * a + len < RP) {
                for (int t = 1; t <= a; t++)
                    for (int i = 0; i < len; i++) w[t * len + i] = w[i];
                len += len * a;
            }
            break;
        case 'f':
            if (2 * len < RP) { for (int i = 0; i < len; i++) w[len + i] = w[len - 1 - i]; len *= 2; }
            break;
        case '{':
            if (len) { uint8_t c = w[0]; for (int i = 0; i + 1 < len; i++) w[i] = w[i + 1]; w[len - 1] = c; }
            break;
        case '}':
            if (len) { uint8_t c = w[len - 1]; for (int i = len - 1; i > 0; i--) w[i] = w[i - 1]; w[0] = c; }
            break;
        case '[':
            if (len) { for (int i = 0; i + 1 < len; i++) w[i] = w[i + 1]; len--; }
            break;
        case ']':
            if (len) len--;
            break;
        case 'q':
            if (2 * len < RP) {
                for (int i = len - 1; i >= 0; i--) { w[2 * i + 1] = w[i]; w[2 * i] = w[i]; }
                len *= 2;
            }
            break;
        case 'D':
            if (a < len) { for (int i = a; i + 1 < len; i++) w[i] = w[i + 1]; len--; }
            break;
        case '\'':
            if (a < len) len = a;
            break;
        case 'z':
            if (len && len + a < RP) {
                for (int i = len - 1; i >= 0; i--) w[i + a] = w[i];
                for (int i = 1; i <= a; i++) w[i] = w[0];
                len += a;
            }
            break;
        case 'Z':
            if (len && len + a < RP) { for (int i = 0; i < a; i++) w[len + i] = w[len - 1]; len += a; }
            break;
        case '$':
            if (len + 1 < RP) w[len++] = (uint8_t)p1;
            break;
        case '^':
            if (len + 1 < RP) { for (int i = len; i > 0; i--) w[i] = w[i - 1]; w[0] = (uint8_t)p1; len++; }
            break;
        case 's':
            for (int i = 0; i < len; i++) if (w[i] == p1) w[i] = (uint8_t)p2;
            break;
        case '@': {
            int o = 0;
            for (int i = 0; i < len; i++) if (w[i] != p1) w[o++] = w[i];
            len = o;
            break;
        }
        case 'x':  // extract: w = w[a : a+b]
            if (a < len && a + b <= len) { for (int i = 0; i < b; i++) w[i] = w[a + i]; len = b; }
            break;
        case 'O':  // omit b bytes at a
            if (a < len && a + b <= len) { for (int i = a; i + b < len; i++) w[i] = w[i + b]; len -= b; }
            break;
        case 'i':  // insert byte p2 at a
            if (a <= len && len + 1 < RP) { for (int i = len; i > a; i--) w[i] = w[i - 1]; w[a] = (uint8_t)p2; len++; }
            break;
        case 'o':  // overwrite at a
            if (a < len) w[a] = (uint8_t)p2;
            break;
        case '*':
            if (a < len && b < len) { uint8_t t = w[a]; w[a] = w[b]; w[b] = t; }
            break;
        case 'k':
            if (len >= 2) { uint8_t t = w[0]; w[0] = w[1]; w[1] = t; }
            break;
        case 'K':
            if (len >= 2) { uint8_t t = w[len - 1]; w[len - 1] = w[len - 2]; w[len - 2] = t; }
            break;
        case 'L':
            if (a < len) w[a] = (uint8_t)(w[a] << 1);
            break;
        case 'R':
            if (a < len) w[a] = (uint8_t)(w[a] >> 1);
            break;
        case '+':
            if (a < len) w[a] = (uint8_t)(w[a] + 1);
            break;
        case '-':
            if (a < len) w[a] = (uint8_t)(w[a] - 1);
            break;
        case '.':
            if (a + 1 < len) w[a] = w[a + 1];
            break;
        case ',':
            if (a >= 1 && a < len) w[a] = w[a - 1];
            break;
        case 'y':  // duplicate the first a bytes in front
            if (a <= len && len + a < RP) {
                for (int i = len - 1; i >= 0; i--) w[i + a] = w[i];
                len += a;
            }
            break;
        case 'Y':  // duplicate the last a bytes at the end
            if (a <= len && len + a < RP) { for (int i = 0; i < a; i++) w[len + i] = w[len - a + i]; len += a; }
            break;
        case 'E':
        case 'e': {  // lower-case, then upper-case the first byte and every byte after a separator (in the lowered word)
            const uint8_t sep = op == 'E' ? (uint8_t)' ' : (uint8_t)p1;
            for (int i = 0; i < len; i++) w[i] = rc_tolower(w[i]);
            bool up = true;  // the previous (lowered) byte was a separator, or this is the first byte
            for (int i = 0; i < len; i++) {
                const bool is_sep = w[i] == sep;
                if (up) w[i] = rc_toupper(w[i]);
                up = is_sep;
            }
            break;
        }
        case '3': {  // toggle the byte after the a-th (0-based) occurrence of p2
            int seen = 0;
            for (int i = 0; i < len; i++)
                if (w[i] == p2) {
                    if (seen == a) {
                        if (i + 1 < len) w[i + 1] = rc_toggle(w[i + 1]);
                        break;
                    }
                    seen++;
                }
            break;
        }
        case 'M':
            for (int i = 0; i < len; i++) mem[i] = w[i];
            mp = mem;
            mlen = len;
            break;
        case '4':
            if (len + mlen >= RP) return RULE_REJECT;
            for (int i = 0; i < mlen; i++) w[len + i] = mp[i];
            len += mlen;
            break;
        case '6':
            if (len + mlen >= RP) return RULE_REJECT;
            for (int i = len - 1; i >= 0; i--) w[i + mlen] = w[i];
            for (int i = 0; i < mlen; i++) w[i] = mp[i];
            len += mlen;
            break;
        case 'X': {  // insert mem[a : a+b] at p3
            const int at = (int)p3;
            if (b < 1 || a + b > mlen || at > len || len + b > RP) return RULE_REJECT;
            for (int i = len - 1; i >= at; i--) w[i + b] = w[i];
            for (int i = 0; i < b; i++) w[at + i] = mp[a + i];
            len += b;
            break;
        }
        case '<':
            if (len > a) return RULE_REJECT;
            break;
        case '>':
            if (len < a) return RULE_REJECT;
            break;
        case '_':
            if (len != a) return RULE_REJECT;
            break;
        case '!':
            for (int i = 0; i < len; i++) if (w[i] == p1) return RULE_REJECT;
            break;
        case '/': {
            bool found = false;
            for (int i = 0; i < len; i++) found |= w[i] == p1;
            if (!found) return RULE_REJECT;
            break;
        }
        case '(':
            if (!len || w[0] != p1) return RULE_REJECT;
            break;
        case ')':
            if (!len || w[len - 1] != p1) return RULE_REJECT;
            break;
        case '=':
            if (a >= len || w[a] != p2) return RULE_REJECT;
            break;
        case '%': {
            int cnt = 0;
            for (int i = 0; i < len; i++) cnt += w[i] == p2;
            if (cnt < a) return RULE_REJECT;
            break;
        }
        case 'Q': {
            bool same = len == mlen;
            for (int i = 0; same && i < len; i++) same = w[i] == mp[i];
            if (same) return RULE_REJECT;
            break;
        }
        default:
            break;  // ':' (the parser admits no other op)
        }
    }
    return len;
}

}  // namespace dwpa
