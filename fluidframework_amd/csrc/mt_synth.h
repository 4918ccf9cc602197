// mt_synth.h -- synthetic multi-client op-log model shared by the device generator (bench.py's
// workload source, generated straight into HBM) and the oracle's host generator (tests), so
// both produce bit-identical logs.  Spec: DESIGN.md "Synthetic workloads" (after SURVEY.md §8d):
// observer-driven, every op picks (client C, refSeq R) and positions inside what C had seen.
//
// Every random draw is r(doc, op, slot) = mix64(key(seed, doc) ^ op << 20 ^ slot): a counter
// RNG, so any lane can draw any value without shared generator state.
#ifndef MT_SYNTH_H
#define MT_SYNTH_H

#include <stdint.h>

#include "../../include/mtgpu.h"

#if defined(__HIPCC__)
#define MT_HD __host__ __device__
#else
#define MT_HD
#endif

/* mt_synth_cfg is declared in include/mtgpu.h (it is part of the bench-tooling C-ABI). */

/* slot numbers of the per-op draws */
enum {
    MT_R_CLIENT = 0, MT_R_LAG = 1, MT_R_STALL = 2, MT_R_TYPE = 3, MT_R_POS1 = 4, MT_R_BIGLEN = 5,
    MT_R_LEN = 6, MT_R_AIM = 7, MT_R_AIMPICK = 8, MT_R_AIMPRE = 9, MT_R_AIMPOST = 10, MT_R_NKEYS = 11,
    MT_R_KEY0 = 12, MT_R_VAL0 = 13, MT_R_NULL0 = 14, MT_R_VAL1 = 15, MT_R_NULL1 = 16, MT_R_REWRITE = 17,
    MT_R_IPROPS = 18, MT_R_IKEY = 19, MT_R_IVAL = 20, MT_R_TBIG = 21, MT_R_TLEN = 22, MT_R_MARKER = 23,
    MT_R_MREF = 24, MT_R_CHAR0 = 64
};

MT_HD static inline uint64_t mt_mix64(uint64_t z) {  /* splitmix64 */
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
MT_HD static inline uint64_t mto_rng_key(uint32_t seed, uint32_t doc) {
    return mt_mix64(((uint64_t)seed << 32) ^ mt_mix64((uint64_t)doc + 0x632BE59BD9B4E019ull));
}
MT_HD static inline uint64_t mto_rng(uint64_t key, uint32_t op, uint32_t slot) {
    return mt_mix64(key ^ ((uint64_t)op << 20) ^ (uint64_t)slot);
}
MT_HD static inline uint32_t mt_ru(uint64_t key, uint32_t op, uint32_t slot, uint32_t lo, uint32_t hi) {
    return lo + (uint32_t)(((mto_rng(key, op, slot) >> 32) * (uint64_t)(hi - lo + 1)) >> 32);
}
MT_HD static inline int mt_rp(uint64_t key, uint32_t op, uint32_t slot, uint32_t p32) {
    return (uint32_t)mto_rng(key, op, slot) < p32;
}
/* text of an insert: length 1..16 (300 with p = 1/256); chars [a-z0-9], '\n' with p = 1/64 */
MT_HD static inline uint32_t mt_gen_text_len(uint64_t key, uint32_t op) {
    return (mto_rng(key, op, MT_R_TBIG) & 255) == 0 ? 300u : mt_ru(key, op, MT_R_TLEN, 1, 16);
}
/* a marker insert (p_marker): its ReferenceType, Tile / NestBegin / NestEnd (ops.ts:6-16) */
MT_HD static inline int mt_gen_is_marker(const mt_synth_cfg& cfg, uint64_t key, uint32_t op) {
    return cfg.p_marker && (uint32_t)mto_rng(key, op, MT_R_MARKER) < cfg.p_marker;
}
MT_HD static inline uint8_t mt_gen_ref_type(uint64_t key, uint32_t op) {
    const uint32_t k = (uint32_t)(mto_rng(key, op, MT_R_MREF) >> 40) % 3u;
    return (uint8_t)(k == 0 ? 1u : (k == 1 ? 2u : 4u));
}
MT_HD static inline uint8_t mt_gen_char(uint64_t key, uint32_t op, uint32_t t) {
    uint64_t r = mto_rng(key, op, MT_R_CHAR0 + t);
    if ((r & 63) == 0) return (uint8_t)'\n';
    uint32_t c = (uint32_t)((r >> 8) % 36);
    return (uint8_t)(c < 26 ? 'a' + c : '0' + (c - 26));
}

#ifdef __cplusplus
/* The per-op decision procedure (host form).  `len(R, C)` = getLength in C's view at R;
 * `pick(R, C, k, &pos, &len)` finds the k-th segment visible to (R, C) whose removal C has not
 * seen (rseq > R) and returns how many there are (k = UINT32_MAX: count only).  Writes `rec`
 * (payload_off left 0) and the payload into `buf`; returns the payload length. */
template <class LenF, class PickF>
static inline uint32_t mto_gen_op(const mt_synth_cfg& cfg, uint64_t key, uint32_t i, int32_t seq,
                                  int32_t* cref, int32_t* stall_until, mt_op_rec& rec, uint8_t* buf,
                                  LenF&& len_of, PickF&& pick) {
    const uint32_t C = cfg.n_clients;
    int32_t c = (int32_t)mt_ru(key, i, MT_R_CLIENT, 1, C);
    int32_t lag = (int32_t)mt_ru(key, i, MT_R_LAG, 0, cfg.max_lag);
    int32_t want = seq - lag > 0 ? seq - lag : 0;
    if (cfg.stall_ops && c == 1) {
        if (seq < *stall_until) want = cref[1];
        else if (mt_ru(key, i, MT_R_STALL, 1, cfg.stall_ops) == 1) *stall_until = seq + (int32_t)cfg.stall_ops;
    }
    int32_t R = cref[c] > want ? cref[c] : want;
    if (R > seq) R = seq;
    cref[c] = R;
    int32_t msn = R;
    for (uint32_t k = 1; k <= C; k++) msn = cref[k] < msn ? cref[k] : msn;
    const int32_t S = seq + 1;
    const int32_t L = len_of(R, c);
    const uint32_t rt = (uint32_t)mto_rng(key, i, MT_R_TYPE);
    uint8_t type = (L == 0 || rt < cfg.p_insert) ? 0 : (rt - cfg.p_insert < cfg.p_remove ? 1 : 2);
    rec = mt_op_rec{};
    rec.seq = S;
    rec.ref_seq = R;
    rec.msn = msn;
    rec.client = (uint16_t)c;
    rec.type = type;
    uint32_t n = 0, np = 0;
    if (type == 0) {
        rec.pos1 = (int32_t)mt_ru(key, i, MT_R_POS1, 0, (uint32_t)L);
        if (mt_gen_is_marker(cfg, key, i)) {
            rec.flags |= MT_F_MARKER;
            buf[n++] = mt_gen_ref_type(key, i);
        } else {
            uint32_t tl = mt_gen_text_len(key, i);
            for (uint32_t t = 0; t < tl; t++) buf[n++] = mt_gen_char(key, i, t);
        }
        if (cfg.n_keys && mt_rp(key, i, MT_R_IPROPS, cfg.p_insert_props)) {
            rec.flags |= 2; /* MT_F_PROPS */
            buf[n++] = (uint8_t)mt_ru(key, i, MT_R_IKEY, 0, cfg.n_keys - 1);
            buf[n++] = (uint8_t)mt_ru(key, i, MT_R_IVAL, 1, cfg.n_values);
            np = 1;
        }
    } else {
        int32_t a = (int32_t)mt_ru(key, i, MT_R_POS1, 0, (uint32_t)L - 1), b = 0;
        int aimed = 0;
        if (type == 1 && cfg.p_overlap && mt_rp(key, i, MT_R_AIM, cfg.p_overlap)) {
            int32_t ppos = 0, plen = 0;
            uint32_t cnt = pick(R, c, 0xFFFFFFFFu, &ppos, &plen);
            if (cnt) {
                pick(R, c, mt_ru(key, i, MT_R_AIMPICK, 0, cnt - 1), &ppos, &plen);
                int32_t pre = (int32_t)mt_ru(key, i, MT_R_AIMPRE, 0, 2), post = (int32_t)mt_ru(key, i, MT_R_AIMPOST, 0, 2);
                a = ppos - pre > 0 ? ppos - pre : 0;
                b = ppos + plen + post < L ? ppos + plen + post : L;
                aimed = 1;
            }
        }
        if (!aimed) {
            int32_t big = (int32_t)((mto_rng(key, i, MT_R_BIGLEN) & 15) == 0);
            int32_t q = L / 4 > 1 ? L / 4 : 1;
            int32_t ln = big ? (int32_t)mt_ru(key, i, MT_R_LEN, 1, (uint32_t)q) : (int32_t)mt_ru(key, i, MT_R_LEN, 1, 16);
            b = a + ln < L ? a + ln : L;
        }
        rec.pos1 = a;
        rec.pos2 = b;
        if (type == 2) {
            if (mt_rp(key, i, MT_R_REWRITE, cfg.p_rewrite)) rec.flags |= 1; /* MT_F_REWRITE */
            uint32_t nk = mt_ru(key, i, MT_R_NKEYS, 1, 2);
            uint32_t k0 = mt_ru(key, i, MT_R_KEY0, 0, cfg.n_keys - 1);
            uint32_t k1 = (k0 + 3) % cfg.n_keys;
            buf[n++] = (uint8_t)k0;
            buf[n++] = mt_rp(key, i, MT_R_NULL0, cfg.p_null) ? 0 : (uint8_t)mt_ru(key, i, MT_R_VAL0, 1, cfg.n_values);
            np = 1;
            if (nk == 2 && k1 != k0) {
                buf[n++] = (uint8_t)k1;
                buf[n++] = mt_rp(key, i, MT_R_NULL1, cfg.p_null) ? 0 : (uint8_t)mt_ru(key, i, MT_R_VAL1, 1, cfg.n_values);
                np = 2;
            }
        }
    }
    rec.flags |= (uint8_t)(np << 3);
    rec.payload_len = n;
    return n;
}
#endif

#endif /* MT_SYNTH_H */
