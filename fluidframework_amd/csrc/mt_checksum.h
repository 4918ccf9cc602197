// mt_checksum.h -- per-document 64-bit checksum of the canonical state (DESIGN.md "Checksum").
// Host+device statement; the oracle (oracle/mtcpu.cpp) and oracle/canon.py restate it
// independently and tests/ check all three agree.
#pragma once
#include <stdint.h>
#include "mt_synth.h"  // mt_mix64, MT_HD
#include "mt_state.h"

// fnv1a over the text's UTF-16 code units (h ^= unit): for text up to U+00FF it is the fnv1a of
// the Latin-1 bytes, so narrow and wide documents of the same state hash alike
MT_HD static inline uint64_t mt_fnv1a_step(uint64_t h, uint32_t c) { return (h ^ c) * 0x100000001B3ull; }
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
// The overlap term: the ids < 64 as a bitmask; a wide document's ids >= 64 hashed in (mt_ovx_hash:
// up to eight ids below 256 as their ascending byte list -- round 3's form, so earlier fixtures keep
// their checksums -- any other list folded id by id).  The props term: the low bytes of the value ids of keys 0..7 (the
// narrow u64); a wide document's high bytes (hi) and keys 8..15 (xlo, xhi) hashed in, then keys
// 16..31 (the four pxx words) when any is set.  Both are the narrow word itself whenever the wide
// part is empty, and a document without keys >= 16 keeps its round-4 checksum.
MT_HD static inline uint64_t mt_ovl_term(uint64_t mask, uint64_t ovx) {
    return ovx ? mask ^ mt_mix64(ovx ^ 0x4F56584944530000ull) : mask;
}
MT_HD static inline uint64_t mt_props_term(uint64_t lo, uint64_t hi, uint64_t xlo, uint64_t xhi,
                                           const uint64_t* y = nullptr) {
    uint64_t t = lo;
    if (hi | xlo | xhi)
        t ^= mt_mix64(mt_mix64(hi ^ 0x1111111111111111ull) ^ mt_mix64(xlo ^ 0x2222222222222222ull) ^
                      mt_mix64(xhi ^ 0x3333333333333333ull));
    if (y && (y[0] | y[1] | y[2] | y[3]))
        t ^= mt_mix64(mt_mix64(y[0] ^ 0x4444444444444444ull) ^ mt_mix64(y[1] ^ 0x5555555555555555ull) ^
                      mt_mix64(y[2] ^ 0x6666666666666666ull) ^ mt_mix64(y[3] ^ 0x7777777777777777ull));
    return t;
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

// ---- readers of a document's HBM state, narrow or wide (mt_state.h) ------------------------------
// form: 0 narrow; a wide document: 1, plus 2 when its stored keys 16..31 are valid (MT_WIDE_XKV) and
// 4 when its stored overlap ids past the 16th are (MT_WIDE_XOV); a reader never looks at words a
// document has not stored
MT_HD static inline int mt_form(bool wide, uint32_t wbits) {
    return wide ? 1 | ((wbits & MT_WIDE_XKV) ? 2 : 0) | ((wbits & MT_WIDE_XOV) ? 4 : 0) : 0;
}
// the two words (low bytes, high bytes) holding key k's value id of a wide segment at HBM index i
// (k >= 16: forms with stored keys 16..31 only)
MT_HD static inline void mt_gpwords(const mt_gstate& g, size_t i, int k, uint64_t& lo, uint64_t& hi) {
    if (k < 8) {
        lo = g.props[i];
        hi = g.ph[i];
    } else if (k < 16) {
        lo = g.pxl[i];
        hi = g.pxh[i];
    } else {
        const uint64_t* y = g.pxx + 4 * i + 2 * ((k - 16) >> 3);
        lo = y[0];
        hi = y[1];
    }
}
// segment at HBM index i (= doc * segcap + position): value id of key k
MT_HD static inline uint32_t mt_gprop(const mt_gstate& g, int form, size_t i, int k) {
    const int sh = 8 * (k & 7);
    if (!form) return k < 8 ? (uint32_t)((g.props[i] >> sh) & 0xFFu) : 0u;
    if (k >= 16 && !(form & 2)) return 0u;
    uint64_t lo, hi;
    mt_gpwords(g, i, k, lo, hi);
    return (uint32_t)((lo >> sh) & 0xFFu) | ((uint32_t)((hi >> sh) & 0xFFu) << 8);
}
// matchProperties' value comparison of two segments (properties.ts:62-93)
MT_HD static inline bool mt_gprops_eq(const mt_gstate& g, int form, size_t a, size_t b) {
    if (g.props[a] != g.props[b]) return false;
    if (!form) return true;
    if (g.ph[a] != g.ph[b] || g.pxl[a] != g.pxl[b] || g.pxh[a] != g.pxh[b]) return false;
    if (form & 2)
        for (int q = 0; q < 4; q++)
            if (g.pxx[4 * a + q] != g.pxx[4 * b + q]) return false;
    return true;
}
MT_HD static inline uint64_t mt_gprops_term(const mt_gstate& g, int form, size_t i) {
    return form ? mt_props_term(g.props[i], g.ph[i], g.pxl[i], g.pxh[i], (form & 2) ? g.pxx + 4 * i : nullptr)
                : g.props[i];
}
// A wide segment's overlapping removers >= 64: up to MT_OVX_IDS (32) u16 ids, ascending from the low
// half-word of lo[0]: ids 0..15 in the four words `lo`, ids 16..31 in the four words `hi` (null: none,
// a document without its extension in use); 0 = none.  At rest both are one row of MT_OVX_WORDS words
// per segment (mt_state.h ovx); the LDS engine stages them as two arrays (mt_apply.hip Lds).
#define MT_OVX_WORDS 8
MT_HD static inline uint32_t mt_ovx_id2(const uint64_t* lo, const uint64_t* hi, int q) {
    const uint64_t* x = q < 16 ? lo : hi;
    q &= 15;
    return x ? (uint32_t)(x[q >> 2] >> (16 * (q & 3))) & 0xFFFFu : 0u;
}
MT_HD static inline bool mt_ovx_has2(const uint64_t* lo, const uint64_t* hi, uint32_t c) {
    for (int q = 0; q < MT_OVX_IDS; q++) {
        const uint32_t v = mt_ovx_id2(lo, hi, q);
        if (!v) return false;
        if (v == c) return true;
    }
    return false;
}
MT_HD static inline uint64_t mt_ovx_hash2(const uint64_t* lo, const uint64_t* hi) {
    uint64_t packed = 0, h = 0x9E3779B97F4A7C15ull;
    bool small = true;
    int n = 0;
    for (; n < MT_OVX_IDS; n++) {
        const uint32_t v = mt_ovx_id2(lo, hi, n);
        if (!v) break;
        if (v > 255u || n >= 8) small = false;
        else packed |= (uint64_t)v << (8 * n);
        h = mt_mix64(h ^ v);
    }
    if (!n) return 0;
    return small ? packed : (h ? h : 1ull);
}
// the at-rest list of the segment at HBM index i
MT_HD static inline const uint64_t* mt_govx_lo(const mt_gstate& g, size_t i) { return g.ovx + MT_OVX_WORDS * i; }
MT_HD static inline const uint64_t* mt_govx_hi(const mt_gstate& g, int form, size_t i) {
    return (form & 4) ? g.ovx + MT_OVX_WORDS * i + 4 : nullptr;
}
// the short client ids of the segment at HBM index i (a wide document's ids >= 256 via chi)
MT_HD static inline uint32_t mt_gclient(const mt_gstate& g, bool wide, size_t i) {
    return (uint32_t)g.client[i] | (wide && g.chi ? (uint32_t)(g.chi[i] & 0xFFu) << 8 : 0u);
}
MT_HD static inline uint32_t mt_grclient(const mt_gstate& g, bool wide, size_t i) {
    return (uint32_t)g.rclient[i] | (wide && g.chi ? (uint32_t)(g.chi[i] >> 8) << 8 : 0u);
}
MT_HD static inline uint64_t mt_govl_term(const mt_gstate& g, int form, size_t i) {
    return form ? mt_ovl_term(g.ovl[i], mt_ovx_hash2(mt_govx_lo(g, i), mt_govx_hi(g, form, i))) : g.ovl[i];
}
// code unit q of the text at arena unit offset `off` of document d (its current half)
MT_HD static inline uint32_t mt_gtext(const mt_gstate& g, uint32_t d, const mt_doc_scalars& sc, uint32_t off) {
    const uint8_t* a = g.text + ((size_t)d * 2 + sc.text_half) * g.textcap;
    return (sc.wide & MT_WIDE_DOC) ? (uint32_t)reinterpret_cast<const uint16_t*>(a)[off] : (uint32_t)a[off];
}
