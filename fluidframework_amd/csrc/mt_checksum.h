// mt_checksum.h -- per-document 64-bit checksum of the canonical state (DESIGN.md "Checksum").
// Host+device statement; the oracle (oracle/mtcpu.cpp) and oracle/canon.py restate it
// independently and tests/ check all three agree.
#pragma once
#include <stdint.h>
#include "mt_synth.h"  // mt_mix64, MT_HD

MT_HD static inline uint64_t mt_fnv1a_step(uint64_t h, uint8_t c) { return (h ^ c) * 0x100000001B3ull; }
#define MT_FNV_INIT 0xCBF29CE484222325ull
// a Marker's "text hash": the fnv1a of its one ReferenceType byte, xor this tag
#define MT_MARKER_TAG 0x4D41524B45520000ull

MT_HD static inline uint64_t mt_seg_hash(uint64_t idx, uint64_t text_hash, int32_t seq, int32_t client, int32_t rseq,
                                         int32_t rclient, uint64_t overlap, uint64_t props_lo, uint32_t props_defined) {
    uint64_t b = (uint64_t)(uint32_t)seq | ((uint64_t)(uint32_t)client << 32);
    uint64_t c = (uint64_t)(uint32_t)rseq | ((uint64_t)(uint32_t)rclient << 32);
    uint64_t h = mt_mix64(text_hash ^ (idx * 0xD6E8FEB86659FD93ull));
    h = mt_mix64(h ^ b);
    h = mt_mix64(h ^ c);
    h = mt_mix64(h ^ overlap);
    h = mt_mix64(h ^ props_lo ^ ((uint64_t)props_defined << 63));
    return h;
}
// canonical client id of a stored short id: NonCollabClient (snapshot loads) is -2
MT_HD static inline int32_t mt_canon_client(uint32_t c) { return c == 0xFEu ? -2 : (int32_t)c; }
MT_HD static inline uint64_t mt_tree_term(uint64_t count, uint64_t b, uint64_t depth) {
    return mt_mix64(count ^ (b << 8) ^ (depth << 56));
}
MT_HD static inline uint64_t mt_finish_checksum(uint64_t seg_sum, uint64_t tree_sum, int32_t cur_seq, int32_t min_seq,
                                                uint32_t nsegs) {
    uint64_t s = mt_mix64(seg_sum) ^ mt_mix64(tree_sum ^ 0x5851F42D4C957F2Dull);
    s ^= mt_mix64((uint64_t)(uint32_t)cur_seq | ((uint64_t)(uint32_t)min_seq << 32));
    return mt_mix64(s ^ nsegs);
}
