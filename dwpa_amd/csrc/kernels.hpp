// kernels.hpp -- host-side launchers for kernels.hip (internal to libdwpa22000.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tables.hpp"

namespace dwpa {

hipError_t launch_prep_dict(const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t count, uint32_t minlen,
                            uint32_t maxlen, uint32_t* mid, uint64_t* ids, uint32_t* counter, uint32_t cap,
                            bool compact, hipStream_t s);
// check path: unique key u = slot uslot[u] of the call's key bytes (koff/klen per slot) -> mid row u
hipError_t launch_prep_keys(const uint64_t* koff, const uint32_t* klen, const uint8_t* kbytes, const uint32_t* uslot,
                            uint32_t count, uint32_t* mid, uint32_t cap, hipStream_t s);
hipError_t launch_prep_numeric(uint64_t first, uint32_t count, uint32_t digits, uint32_t* mid, uint64_t* ids,
                               uint32_t cap, hipStream_t s);
// product launch: issue-pass code object (pbkdf2_module.cpp); DWPA_PBKDF2_PLAIN=1 -> launch_pbkdf2_plain
// work (nullable): a 4-byte device counter the work-queue kernel may use (zeroed here before the launch)
hipError_t launch_pbkdf2(const uint32_t* mid, uint32_t cap, uint32_t base, uint32_t count, const uint32_t* counter,
                         const uint32_t* salt, uint32_t nsalt, uint32_t* pmk, hipStream_t s, uint32_t* work = nullptr);
hipError_t launch_pbkdf2_plain(const uint32_t* mid, uint32_t cap, uint32_t base, uint32_t count,
                               const uint32_t* counter, const uint32_t* salt, uint32_t nsalt, uint32_t* pmk,
                               hipStream_t s);
const char* pbkdf2_variant();
// PMKs that give every SIMD of the current device one PBKDF2 wave (two output-block lanes per PMK); 0 on error
uint32_t pbkdf2_wave_unit();
// many ESSIDs per launch: slot s uses the salt entry pool + sref[s] = {nsalt, [2][nsalt][16] words}
hipError_t launch_pbkdf2_ms(const uint32_t* mid, uint32_t cap, uint32_t count, const uint32_t* pool,
                            const uint32_t* sref, uint32_t* pmk, hipStream_t s);
hipError_t launch_pbkdf2_ms_plain(const uint32_t* mid, uint32_t cap, uint32_t count, const uint32_t* pool,
                                  const uint32_t* sref, uint32_t* pmk, hipStream_t s);
// attempt-parallel verification of EAPOL lists with >= ATT_PARALLEL_MIN attempts: lane = (key, attempt) item,
// segs[i].pad = first wave of segment i (ceil(count * natt / 64) waves each, nwaves in all), segs[i].count <= segk
// (1..64); keys = scratch of eapol_key_words(vc) x kstride words, kstride >= segk * nsegs
uint32_t eapol_key_words(uint32_t vc);
// first_hit (nullable): per line, the smallest key ordinal (ids[slot]: a job's keys numbered in input order, across
// all chunks of the call) with a hit so far (~0u: none); waves whose keys all come after it exit at once, and hits
// lower it (the check wants only the first key in input order).  Reset it once per call, not per chunk.
hipError_t launch_verify_att(const uint32_t* pmk, uint32_t cap, const uint64_t* ids, const SegDev* segs,
                             uint32_t nsegs, uint32_t nwaves, uint32_t* keys, uint32_t kstride, uint32_t segk,
                             const LineDev* lines, const uint32_t* pool, const AttDev* atts, HitDev* hits,
                             uint32_t* hitcnt, uint32_t hitcap, uint32_t* first_hit, uint32_t vc, hipStream_t s);
// many ESSID groups x one batch per launch (cap % 64 == 0): gsalt[c] = {salt word offset, nsalt} of chunk group c,
// PMK word k of (c, slot) at pmk[k * pstride + c * cap + slot]
hipError_t launch_pbkdf2_mg(const uint32_t* mid, uint32_t cap, const uint32_t* counter, uint32_t ngroups,
                            const uint32_t* salt, const uint32_t* gsalt, uint32_t* pmk, uint32_t pstride,
                            hipStream_t s, uint32_t* work = nullptr);
hipError_t launch_pbkdf2_mg_plain(const uint32_t* mid, uint32_t cap, const uint32_t* counter, uint32_t ngroups,
                                  const uint32_t* salt, const uint32_t* gsalt, uint32_t* pmk, uint32_t pstride,
                                  hipStream_t s);
// Check-path tail: PBKDF2 of slots [0, count) like launch_pbkdf2_ms_plain, at wave priority 0 until *flag != 0,
// then at `prio` (0 = never raised); every wave that raises itself adds 1 to *raised.  launch_set_flag sets the
// flag (queue it after the head).
hipError_t launch_pbkdf2_ms_tail(const uint32_t* mid, uint32_t cap, uint32_t count, const uint32_t* pool,
                                 const uint32_t* sref, uint32_t* pmk, uint32_t* flag, uint32_t prio,
                                 uint32_t* raised, hipStream_t s);
hipError_t launch_set_flag(uint32_t* flag, hipStream_t s);
constexpr uint32_t GATHER_CALLER = 0x80000000u;
hipError_t launch_gather_pmk(const uint32_t* upmk, uint32_t ucap, const uint32_t* cpmk, const uint32_t* src,
                             uint32_t n, uint32_t* pmk, uint32_t cap, hipStream_t s);
// out: host-mapped, >= 16 + hitcap * sizeof(HitDev) bytes (word 0 = hit count, word 1 = *raised or 0, HitDev
// records from byte 16)
hipError_t launch_hits_out(const uint32_t* hitcnt, const HitDev* hits, uint32_t hitcap, uint32_t* out,
                           const uint32_t* raised, hipStream_t s);
hipError_t launch_set_pmk(uint32_t* pmk, uint32_t cap, uint32_t slot, const uint32_t w[8], hipStream_t s);
hipError_t launch_verify(const uint32_t* pmk, uint32_t cap, const uint64_t* ids, const uint32_t* counter,
                         const SegDev* segs, uint32_t nsegs, uint32_t line_base, uint32_t nlines, const LineDev* lines,
                         const uint32_t* pool, const AttDev* atts, HitDev* hits, uint32_t* hitcnt, uint32_t hitcap,
                         uint32_t vc, hipStream_t s, const uint32_t* line_list = nullptr,
                         const uint32_t* line_poff = nullptr, uint32_t pstride = 0);

}  // namespace dwpa
