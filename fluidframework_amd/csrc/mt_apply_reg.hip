// mt_apply_reg.hip -- register-resident merge-tree apply engine for gfx950 (CDNA4).
//
// Same semantics as mt_apply.hip (the observer Client.applyMsg of the reference,
// client.ts:797-828, bit-exact); a different home for the document state:
//
//   * every per-segment field the op path touches lives in VGPRs, BLOCKED by lane: slot i of
//     the document is register j = i % K of lane i / K (K = CAP / 64).  The visibility of every
//     segment for an op's (refSeq, client) view (mergeTree.ts:1667-1697) is K per-lane
//     evaluations plus one wave-wide DPP scan: the PartialSequenceLengths query
//     (partialLengths.ts:433-487) without any memory traffic;
//   * the leaf level of the B-tree is a set of per-lane K-bit masks over the same slots: block
//     starts (bsm), the starting slot's needsScour state (sc0 / sc1), live slots (lvm); so
//     "which leaf block holds slot k", "where does block b start" and "how many children has it"
//     are ballot / popcount / DPP questions, not LDS walks, and block edits touch one register.
//     Interior levels (touched only by leaf splits and packs) are child-count arrays in LDS, as
//     in mt_apply.hip;
//   * a zamboni unlink (mergeTree.ts:1289-1365) only clears its slot's live bit (a dead slot has
//     no length in any view and is no child of any block); dead slots are squeezed out when the
//     document is written back, so nothing moves on an unlink.  An insert or a split moves the later slots one register to the right
//     (K predicated moves per field per lane, DPP wave_shr:1 across lanes);
//   * cold fields (property set, text offset) stay in LDS indexed by a segment id that never
//     changes while the segment is linked; the zamboni heap holds those ids.
// Capacity classes K = 2 ... 16 (128..1024 slots in steps of 64).  Bigger documents, documents that ever
// see a client id above 32 (the register overlap set is 32 bits wide), and a launch that carries
// snapshot body appends (MT_OP_LOAD, once in a document's life) run on mt_apply.hip's LDS engine;
// both engines share the HBM layout of mt_state.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtgpu.h"
#include "mt_state.h"
#include "mt_wave.h"

namespace mtr {

constexpr int kMaxNodes = 8;           // MaxNodesInBlock, mergeTree.ts:334
constexpr int kTextGranularity = 256;  // MergeTree.TextSegmentGranularity, mergeTree.ts:1059
constexpr int kNarrowClients = 32;     // register overlap set: clients 1..32 at bit C-1 of ov
constexpr int kC64Clients = 63;        // ... and 33..63 at bit C-33 of oh (the C64 instantiation)
constexpr uint32_t kLenBits = 17;      // li = len | id << 17  (len <= textcap <= 65536)
constexpr uint32_t kLenMask = (1u << kLenBits) - 1;
constexpr uint32_t kNoId = 0x7FFFu;    // id of a padding slot
constexpr uint32_t kEmptyLi = kNoId << kLenBits;
// cf = client (bits 0-7) | removedClientId (8-15) | segment flags (16-23)
constexpr uint32_t F_RM = (uint32_t)MT_SF_REMOVED << 16;
constexpr uint32_t F_PDEF = (uint32_t)MT_SF_PDEF << 16;
constexpr uint32_t F_NL = (uint32_t)MT_SF_NL << 16;
constexpr uint32_t F_HASNL = (uint32_t)MT_SF_HASNL << 16;
constexpr uint32_t F_MARKER = (uint32_t)MT_SF_MARKER << 16;
// register-only flag: ENDS_WITH_NEWLINE not yet known.  A boundary split leaves the left part's last
// character unread (the text is in HBM: one dependent global load per split); the flag is resolved
// where it is read -- scour's append decisions (the block's children at once) and the store.
constexpr uint32_t F_NLQ = 1u << 21;
constexpr uint32_t kEmptyCf = 0xFFu;     // padding: client 255 never matches (and the slot is dead)
constexpr uint16_t kDead = 0xFFFFu;

// The document arrays are read and written through global-address-space pointers (global_load /
// global_store: vmcnt only), not generic ones (flat_*: both counters, so every wait drains LDS too)
#define MT_GLOB __attribute__((address_space(1)))
#define MT_KARG __attribute__((address_space(4)))
template <class T>
MT_DEV MT_GLOB T* gp(T* p) { return (MT_GLOB T*)p; }
typedef const MT_KARG mt_gstate KGState;
typedef uint32_t EvWords __attribute__((ext_vector_type(4)));
// One 96-byte event row (mt_event, include/mtgpu.h) through a global pointer, six 16-byte stores
// built from the field values: a row assembled as an mt_event first costs the 24 registers of the
// struct at every call site (the event kernels' register peak and scratch came from exactly that).
// pv01..pv67: pvals[0..7] two to a word (the register engine's eight keys; pvals[8..31] are zero).
MT_DEV void put_event(MT_GLOB mt_event* p, int32_t seq, int op, unsigned flags, int leaf, int pos, uint32_t len,
                      uint32_t pmask = 0, uint32_t pv01 = 0, uint32_t pv23 = 0, uint32_t pv45 = 0, uint32_t pv67 = 0) {
    static_assert(sizeof(mt_event) == 96 && offsetof(mt_event, pvals) == 24, "mt_event");
    MT_GLOB EvWords* q = reinterpret_cast<MT_GLOB EvWords*>(p);
    const EvWords z = {0u, 0u, 0u, 0u};
    q[0] = EvWords{(uint32_t)seq, ((uint32_t)op & 0xFFu) | ((flags & 0xFFu) << 8), (uint32_t)leaf, (uint32_t)pos};
    q[1] = EvWords{len, pmask, pv01, pv23};
    q[2] = EvWords{pv45, pv67, 0u, 0u};
    q[3] = z;
    q[4] = z;
    q[5] = z;
}

MT_DEV int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
MT_DEV uint32_t uniu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// lane l <- lane l-1 (lane 0 <- fill)
MT_DEV int shr1(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false); }
// lane l <- lane l+1 (lane 63 <- fill)
MT_DEV int shl1(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, 0x130, 0xf, 0xf, false); }
MT_DEV int wave_total(int v) { return wave_last(wave_incl_scan(v)); }

// ---- optional per-phase cycle accounting (diagnostic build: -DMT_PROF; never in the product)
enum { P_LOAD, P_SCAN, P_BOUND, P_INSERT, P_RANGE, P_ZAMBONI, P_SCOUR, P_STORE, P_OPS, P_ZPOP, P_REPACK,
       P_B_GET, P_B_BLK, P_B_TXT, P_B_INS, P_N_SCOUR, P_N_UNLINK, P_N_APPEND, P_N_SPLIT,
       P_COMPACT, P_N_COMPACT, P_N_APPBYTES, P_B_SRCH, P_B_LEAF, P_OP, P_NSLOT };
[[maybe_unused]] constexpr int kProfStride = 32;  // slots per class in mt_prof_acc
#ifdef MT_PROF
__device__ unsigned long long mt_prof_acc[16 * kProfStride];  // [K - 1 = 0..15][slot]
MT_DEV uint64_t prof_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
// -DMT_PROF_ONLY=<slot>: only that phase's stamps run (one stamp pair per phase execution, so its
// overhead is a constant that the P_OP-only build calibrates); default: every stamp
#ifndef MT_PROF_ONLY
#define MT_PROF_ONLY -1
#endif
#define PROF_ON(s) (MT_PROF_ONLY < 0 || MT_PROF_ONLY == (s))
#define PROF_BEGIN(v, s) const uint64_t v = PROF_ON(s) ? prof_now() : 0
#define PROF_BEGIN2(v, s1, s2) const uint64_t v = (PROF_ON(s1) || PROF_ON(s2)) ? prof_now() : 0
#define PROF_END(arr, slot, v) \
    do {                       \
        if (PROF_ON(slot)) arr[slot] += prof_now() - (v); \
    } while (0)
#define PROF_CNT(slot, v) prof[slot] += (v)
#else
#define PROF_BEGIN(v, s)
#define PROF_BEGIN2(v, s1, s2)
#define PROF_END(arr, slot, v)
#define PROF_CNT(slot, v)
#endif

template <int K>
struct RLds {
    static constexpr int CAP = 64 * K;
    // leaf blocks, blocks per interior level, heap entries (1-based): the class limits of mt::Lds at
    // CAP, and at least those of the 256 class -- the launch's worst-case growth (mt_bin_kernel: 2 leaf
    // blocks, 1 interior block and 4 heap entries per op) needs them for a b = 32 launch to fit the
    // 192 class at all (mt_engine.cpp kClassParams)
    static constexpr int LB = CAP / 2 > 128 ? CAP / 2 : 128;
    static constexpr int IB = CAP / 8 + 8 > 40 ? CAP / 8 + 8 : 40;
    static constexpr int H = CAP / 2 + 64 > 192 ? CAP / 2 + 64 : 192;
    uint64_t props[CAP];    // by segment id: 8 keys x u8 value id
    // scr: scratch by slot / position / leaf block (load, store); tln: by segment id, the text length
    // while linked, 0 once unlinked (the op loop's compaction).  They share their words, as neither
    // is live while the other is (load writes tln after its last scr read; store runs after the op
    // loop): 4 B per slot less LDS, which lifts the waves per CU that LDS allows at K = 7, 9, 10
    // and 14-16 to what the registers allow (K = 9: 11 -> 12, K = 10: 11 -> 12)
    union {
        int32_t scr[CAP + 1];
        uint32_t tln[CAP + 1];
    };
    int32_t hseq[H];
    uint16_t toff[CAP];     // by segment id: text view offset (at store: id -> position)
    uint16_t hslot[H];      // heap entry -> segment id
    uint8_t ibcnt[MT_MAXLEV - 1][IB];  // interior levels: level L's child counts in ibcnt[L - 1]
    uint8_t lbsc[LB + 1];   // store staging: needsScour per leaf block
    int32_t nb[MT_MAXLEV];  // blocks per interior level (leaf blocks are counted by BS bits)
    // scour scratch: the live children by rank, one array per field (separate 4-byte stores: no
    // 4-register tuple built per slot, which cost ~20 VGPRs at the scour's register peak)
    // zr[q]: the removal seq of a removed child q, else its seq; zr[8 + q] its li, zr[16 + q] its cf,
    // zr[24 + q] its slot
    uint32_t zr[4 * kMaxNodes];
    // the lanes' discard words of the branch-free LDS stores (a lane with nothing to store writes
    // here; never read)
    uint64_t dum[64];
};

struct Elem {
    int32_t seq, rseq;
    uint32_t li, cf, ov, oh;
    int32_t cum;
};
// A boundary split of the segment at slot k: the two parts' lengths / ids (li), the left part's
// flags and cumulative end (insert_at applies it: the right part enters at k + 1)
struct Cut {
    uint32_t lli, lcf, rli;
    int32_t pos;
};

// W: documents with client ids above 32 (any up to 63): the overlap set takes a second register
// per slot (oh), otherwise the same engine.  EV: delta / maintenance events are recorded
// (mt_events_enable): the reference's callbacks in firing order, as mt_event rows
template <int K, bool W = false, bool EV = false>
struct RWave {
    using L = RLds<K>;
    static constexpr int CAP = L::CAP;
    static constexpr uint32_t kAll = (1u << K) - 1u;
    // clang ext vectors: SSA values end to end, never a private-memory array
    typedef int32_t VI __attribute__((ext_vector_type(K)));
    typedef uint32_t VU __attribute__((ext_vector_type(K)));
    typedef uint32_t U4 __attribute__((ext_vector_type(4)));
    typedef uint32_t U2 __attribute__((ext_vector_type(2)));
    L& s;
    const int lane;
    uint8_t* const abase;
    const uint32_t textcap;

    // ---- document state in registers (blocked: slot i = lane * K + j).  ext vectors: SSA values
    // end to end, and a wave-uniform dynamic index becomes s_set_gpr_idx register indexing.
    VI seq, rseq;
    VU li, cf, ov;
    VU oh;   // (W only) overlap clients 33..63
    VI cum;  // per-op scratch: inclusive visible prefix for the op's view
    // ---- uniform document scalars
    int ns, nlive, nb0, nlev, heap_n, cur_seq, min_seq, err, err_seq, next_id;
    uint32_t text_top, text_half;
    bool dirty;  // arena stores issued and not yet waited for
    uint32_t pb; // the current op's payload, prefetched: lane i holds byte i (i < 64)
    // per-lane K-bit masks over this lane's slots: starts a leaf block (bsm), live (lvm), and the
    // needsScour state (MT_SC_*) of the block a start slot begins: bit 0 in sc0, bit 1 in sc1
    uint32_t bsm, lvm, sc0, sc1;
    // (EV) the document's event rows, their capacity, the rows recorded so far, the op's seq
    MT_GLOB mt_event* evp = nullptr;
    uint32_t evcap = 0;
    int evn = 0;
    int32_t evseq = 0;
#ifdef MT_PROF
    uint64_t prof[P_NSLOT] = {};
#endif

    MT_DEV RWave(L& lds, uint8_t* a, uint32_t tc)
        : s(lds), lane(lane_id()), abase(a), textcap(tc), dirty(false) {}
    // the current arena half
    MT_DEV uint8_t* arena() const { return abase + (size_t)text_half * textcap; }

    MT_DEV int idx(int j) const { return lane * K + j; }

    MT_DEV void fail(int code, int32_t sq) {
        if (err == 0) {
            err = code;
            err_seq = sq;
        }
    }
    MT_DEV static uint32_t len_of(uint32_t l) { return l & kLenMask; }
    MT_DEV static uint32_t id_of(uint32_t l) { return l >> kLenBits; }

    // ------------------------------------------------------------ slot masks
    MT_DEV uint32_t bs_bits() const { return bsm; }
    MT_DEV uint32_t live_bits() const { return lvm; }
    // this lane's bit of uniform slot k (0 if another lane holds it)
    MT_DEV uint32_t kbit(int k) const {
        const int r = k - lane * K;
        return (r >= 0 && r < K) ? (1u << r) : 0u;
    }
    // needsScour state of the block starting at uniform slot a; set it / the block-start bit
    MT_DEV int sc_of(int a) const {
        const int r = uni(a % K);
        return __builtin_amdgcn_readlane((int)(((sc0 >> r) & 1u) | (((sc1 >> r) & 1u) << 1)), a / K);
    }
    MT_DEV void set_sc(int a, int v) {
        const uint32_t b = kbit(a);
        sc0 = (v & 1) ? (sc0 | b) : (sc0 & ~b);
        sc1 = (v & 2) ? (sc1 | b) : (sc1 & ~b);
    }
    MT_DEV void set_bs(int a, bool on) {
        const uint32_t b = kbit(a);
        bsm = on ? (bsm | b) : (bsm & ~b);
    }
    // the masks after shift_in(p, ..): slots >= p move up one, slot p gets (bs, scv, live)
    MT_DEV static uint32_t shift_mask(uint32_t m, uint32_t lo, bool at, bool above, int r, bool bit) {
        const uint32_t c = (uint32_t)shr1((int)((m >> (K - 1)) & 1u), 0);
        return (m & lo) | (((m & ~lo) << 1) & kAll) | ((at && bit) ? (1u << r) : 0u) | (above ? c : 0u);
    }
    MT_DEV void mask_shift(int p, bool bs, int scv, bool live) {
        const uint32_t lo = below(p);
        const int r = p - lane * K;
        const bool at = r >= 0 && r < K, above = r < 0;
        bsm = shift_mask(bsm, lo, at, above, r, bs);
        lvm = shift_mask(lvm, lo, at, above, r, live);
        sc0 = shift_mask(sc0, lo, at, above, r, (scv & 1) != 0);
        sc1 = shift_mask(sc1, lo, at, above, r, (scv & 2) != 0);
    }
    // this lane's slots with index < k
    MT_DEV uint32_t below(int k) const {
        const int r = k - lane * K;
        return r <= 0 ? 0u : (r >= K ? kAll : ((1u << r) - 1u));
    }
    // slot of the r-th (0-based) set bit of the lanes' masks m; -1 if there is none
    MT_DEV int nth_slot(uint32_t m, int r) const {
        const int c = __popc(m);
        const int incl = wave_incl_scan(c);
        const uint64_t hit = wave_ballot(r >= incl - c && r < incl);
        if (!hit) return -1;
        const int lk = first_lane(hit);
        uint32_t mm = (uint32_t)__builtin_amdgcn_readlane((int)m, lk);
        for (int q = r - __builtin_amdgcn_readlane(incl - c, lk); q > 0; q--) mm &= mm - 1;
        return uni(lk * K + (int)__builtin_ctz(mm));
    }
    // minimum over the lanes of a per-lane slot index (0x7fffffff = none): lane l's slots all
    // precede lane l + 1's, so it is the value of the first lane that has one
    MT_DEV static int first_hit(int v) {
        const uint64_t m = wave_ballot(v != 0x7fffffff);
        return uni(m ? __builtin_amdgcn_readlane(v, first_lane(m)) : 0x7fffffff);
    }
    // first slot >= from whose bit is set in m; ns if none
    MT_DEV int first_from(uint32_t m, int from) const {
        const uint32_t x = m & ~below(from);
        const uint64_t hit = wave_ballot(x != 0);
        if (!hit) return ns;
        const int lk = first_lane(hit);
        return uni(lk * K + (int)__builtin_ctz((uint32_t)__builtin_amdgcn_readlane((int)x, lk)));
    }
    // ------------------------------------------------------------ leaf blocks
    MT_DEV int leaf_of(int k) const { return uni(wave_total(__popc(bs_bits() & below(k + 1))) - 1); }
    MT_DEV int bs_slot(int b) const { return b >= nb0 ? ns : nth_slot(bs_bits(), b); }
    // ---- navigation by slot: a ballot and a readlane or two, no wave-wide scan.  A leaf block
    // is the slot range from its start mark to the next one (or ns); slot 0 always starts block 0.
    MT_DEV int block_start(int k) const {  // start of the leaf block holding slot k
        const uint32_t m = bsm & below(k + 1);
        const int l = 63 - __builtin_clzll(wave_ballot(m != 0));
        return uni(l * K + (31 - __builtin_clz((uint32_t)__builtin_amdgcn_readlane((int)m, l))));
    }
    MT_DEV int next_start(int k) const { return first_from(bsm, k + 1); }  // end of the block holding k
    // set bits of the lanes' masks m inside slots [a, e) (a block spans one or two lanes almost always)
    MT_DEV int count_in(uint32_t m, int a, int e) const {
        a = uni(a);
        e = uni(e);
        if (e <= a) return 0;
        const uint32_t x = m & below(e) & ~below(a);
        const int la = a / K, lb = (e - 1) / K;
        if (lb - la > 1) return uni(wave_total(__popc(x)));
        int c = __popc((uint32_t)__builtin_amdgcn_readlane((int)x, la));
        if (lb != la) c += __popc((uint32_t)__builtin_amdgcn_readlane((int)x, lb));
        return uni(c);
    }
    MT_DEV int live_in(int a, int e) const { return count_in(lvm, a, e); }
    // slot of the r-th (0-based) set bit of m inside [a, e); -1 if there is none
    MT_DEV int nth_in(uint32_t m, int a, int e, int r) const {
        const uint32_t x = m & below(e) & ~below(a);
        for (int l = a / K; l <= (e - 1) / K; l++) {
            uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)x, l);
            const int c = __popc(w);
            if (r < c) {
                for (; r > 0; r--) w &= w - 1;
                return l * K + __builtin_ctz(w);
            }
            r -= c;
        }
        return -1;
    }

    // ------------------------------------------------------------ delta events (EV)
    // One callback record (mt_event, include/mtgpu.h) written by lane 0 in firing order (the
    // reference's mergeTreeDeltaCallback / mergeTreeMaintenanceCallback, mergeTreeDeltaCallback.ts).
    // Segments are named by their leaf ordinal among the linked segments (live slots) and, for op
    // callbacks, their local-view position; rows past the capacity are counted, not written (the
    // document then halts with MT_DERR_EVENTS after the op).
    MT_DEV void emit(int op, unsigned flags, int leaf, int pos, uint32_t len) {
        if (lane == 0 && evn < (int)evcap) {
            put_event(evp + evn, evseq, op, flags, leaf, pos, len);
        }
        evn = evn + 1;
    }
    MT_DEV int live_before(int k) const { return uni(wave_total(__popc(lvm & below(k)))); }
    // characters of the unremoved linked segments before slot k: the local view's position
    MT_DEV int local_before(int k) const {
        const uint32_t m = lvm & below(k);
        int t = 0;
#pragma unroll
        for (int j = 0; j < K; j++) t += (((m >> j) & 1u) && !(cf[j] & F_RM)) ? (int)len_of(li[j]) : 0;
        return uni(wave_total(t));
    }
    // The REMOVE / ANNOTATE callback (mergeTree.ts:2705-2712 / 2592-2600): its delta segments in
    // document order, lane-parallel (each lane writes the rows of its own slots, placed by a prefix
    // count).  REMOVE runs after the edits (the segments this op removed: rseq == S by C; positions
    // with the removal applied), ANNOTATE before them (propertyDeltas need the previous values:
    // SegmentPropertiesManager.addProperties' deltas, segmentPropertiesManager.ts:60-108 -- a
    // rewrite records each key it deletes with its old value, every key of the op the value before
    // it is set, null for a rewrite's null-valued key).  tm: the op's touched slots.
    MT_DEV void emit_range(bool is_remove, int32_t S, int C, uint32_t tm, uint64_t pclr, uint64_t pset, bool rewrite) {
        uint32_t hm = 0;
#pragma unroll
        for (int j = 0; j < K; j++) {
            const uint32_t f = cf[j];
            const bool hit = ((tm >> j) & 1u) &&
                             (!is_remove || ((f & F_RM) && rseq[j] == S && ((f >> 8) & 0xFFu) == (uint32_t)C));
            hm |= hit ? (1u << j) : 0u;
        }
        const int hc = __popc(hm);
        const int hinc = wave_incl_scan(hc);
        const int total = wave_last(hinc);
        if (total == 0) return emit(is_remove ? MT_EV_REMOVE : MT_EV_ANNOTATE, MT_EVF_FIRST | MT_EVF_EMPTY, -1, -1, 0);
        int ll = 0, lc = 0;
#pragma unroll
        for (int j = 0; j < K; j++) {
            ll += (((lvm >> j) & 1u) && !(cf[j] & F_RM)) ? (int)len_of(li[j]) : 0;
            lc += (lvm >> j) & 1u;
        }
        int pos = wave_incl_scan(ll) - ll, leaf = wave_incl_scan(lc) - lc, idx = evn + hinc - hc;
        // the op's keys (bit k), and those it sets to a value (not null)
        uint32_t okeys = 0, onz = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            okeys |= ((pclr >> (8 * k)) & 0xFFu) ? (1u << k) : 0u;
            onz |= ((pset >> (8 * k)) & 0xFFu) ? (1u << k) : 0u;
        }
#pragma unroll
        for (int j = 0; j < K; j++) {
            const bool live = (lvm >> j) & 1u;
            if ((hm >> j) & 1u) {
                if (idx < (int)evcap) {
                    const int eop = is_remove ? MT_EV_REMOVE : MT_EV_ANNOTATE;
                    const unsigned efl = idx == evn ? MT_EVF_FIRST : 0u;
                    if (is_remove) {
                        put_event(evp + idx, evseq, eop, efl, leaf, pos, len_of(li[j]));
                    } else {
                        const uint64_t old = (cf[j] & F_PDEF) ? s.props[id_of(li[j])] : 0ull;
                        uint32_t oldnz = 0;
#pragma unroll
                        for (int k = 0; k < 8; k++) oldnz |= ((old >> (8 * k)) & 0xFFu) ? (1u << k) : 0u;
                        const uint32_t pm = okeys | (rewrite ? (oldnz & ~onz) : 0u);
                        // the reported values: the old value of each reported key, null (0) where a
                        // rewrite nulls a key the op names without a value
                        const uint32_t rep = pm & ~(rewrite ? (okeys & ~onz) : 0u);
                        uint32_t pw[4];
#pragma unroll
                        for (int h = 0; h < 4; h++) {
                            const uint32_t v0 = ((rep >> (2 * h)) & 1u) ? (uint32_t)(old >> (16 * h)) & 0xFFu : 0u;
                            const uint32_t v1 = ((rep >> (2 * h + 1)) & 1u) ? (uint32_t)(old >> (16 * h + 8)) & 0xFFu : 0u;
                            pw[h] = v0 | (v1 << 16);
                        }
                        put_event(evp + idx, evseq, eop, efl, leaf, pos, len_of(li[j]), pm, pw[0], pw[1], pw[2], pw[3]);
                    }
                }
                idx++;
            }
            pos += (live && !(cf[j] & F_RM)) ? (int)len_of(li[j]) : 0;
            leaf += live ? 1 : 0;
        }
        evn = evn + total;
    }

    // ------------------------------------------------------------ element access
    MT_DEV Elem get(int k) const {  // all fields of the slot at uniform position k
        const int lk = k / K, jk = uni(k % K);
        Elem r;
        r.seq = __builtin_amdgcn_readlane(seq[jk], lk);
        r.rseq = __builtin_amdgcn_readlane(rseq[jk], lk);
        r.li = (uint32_t)__builtin_amdgcn_readlane((int)li[jk], lk);
        r.cf = (uint32_t)__builtin_amdgcn_readlane((int)cf[jk], lk);
        r.ov = (uint32_t)__builtin_amdgcn_readlane((int)ov[jk], lk);
        if constexpr (W) r.oh = (uint32_t)__builtin_amdgcn_readlane((int)oh[jk], lk);
        r.cum = __builtin_amdgcn_readlane(cum[jk], lk);
        return r;
    }
    MT_DEV uint32_t get_li(int k) const {
        const int jk = uni(k % K);
        return (uint32_t)__builtin_amdgcn_readlane((int)li[jk], k / K);
    }
    // (per-register selects, not a uniform dynamic-index write: that is an s_set_gpr_idx move into a
    // fresh copy of the whole register tuple, which the enclosing loops then copy back at their joins)
    MT_DEV void set_li_cf(int k, uint32_t lv, uint32_t cv) {
        const int r = k - lane * K;
#pragma unroll
        for (int j = 0; j < K; j++) {
            li[j] = j == r ? lv : li[j];
            cf[j] = j == r ? cv : cf[j];
        }
    }
    // insert e at slot p: slots >= p move one register right.  dup (a boundary split of the segment
    // at slot p - 1): slots >= p - 1 move right instead, so slot p receives a copy of the cut segment
    // (patch_cut then gives the two parts their li / cf / cum).  Both forms are this one pass from one
    // call site (insert_at): two call sites -- or a dynamic-index patch of slot p - 1 before the
    // shift -- left the state in different registers on the two paths and the insert loop's join
    // copied all of it (ISA: ~110 v_mov per join at K = 9)
    template <bool CUM>
    MT_DEV void shift_in(int p, const Elem& e, bool bs, int scv, bool live, bool dup = false) {
        mask_shift(p, bs, scv, live);
        const int32_t c_seq = shr1(seq[K - 1], 0), c_rseq = shr1(rseq[K - 1], 0);
        const uint32_t c_li = (uint32_t)shr1((int)li[K - 1], 0), c_cf = (uint32_t)shr1((int)cf[K - 1], 0);
        const uint32_t c_ov = (uint32_t)shr1((int)ov[K - 1], 0);
        const uint32_t c_oh = W ? (uint32_t)shr1((int)oh[K - 1], 0) : 0u;
        const int32_t c_cum = CUM ? shr1(cum[K - 1], 0) : 0;
        // per lane: the register index of slot p in this lane, less one for dup (registers above it
        // take their left neighbour), and the register taking e (none for dup)
        const int r = p - lane * K;
        const int rq = dup ? r - 1 : r;
        const int ra = dup ? -K - 2 : r;
#pragma unroll
        for (int j = K - 1; j >= 0; j--) {
            const bool mv = j > rq, at = j == ra;
            const int32_t pseq = j ? seq[j - 1] : c_seq, prseq = j ? rseq[j - 1] : c_rseq;
            const uint32_t pli = j ? li[j - 1] : c_li, pcf = j ? cf[j - 1] : c_cf, pov = j ? ov[j - 1] : c_ov;
            seq[j] = mv ? pseq : (at ? e.seq : seq[j]);
            rseq[j] = mv ? prseq : (at ? e.rseq : rseq[j]);
            li[j] = mv ? pli : (at ? e.li : li[j]);
            cf[j] = mv ? pcf : (at ? e.cf : cf[j]);
            ov[j] = mv ? pov : (at ? e.ov : ov[j]);
            if constexpr (W) {
                const uint32_t poh = j ? oh[j - 1] : c_oh;
                oh[j] = mv ? poh : (at ? e.oh : oh[j]);
            }
            if (CUM) {
                const int32_t pcm = j ? cum[j - 1] : c_cum;
                cum[j] = mv ? pcm : (at ? e.cum : cum[j]);
            }
            // register j is rewritten only after register j + 1 (its last reader): the new value can
            // take the old one's register, so the state keeps its registers through the shift and
            // the joins after it need no copies
            __builtin_amdgcn_sched_barrier(0);
        }
        ns = ns + 1;
    }
    // after shift_in(p, .., dup): slot p - 1 becomes the cut's left part, slot p's li the right part's
    // (in-place per-register selects: the state keeps its registers)
    MT_DEV void patch_cut(int p, const Cut& c) {
        const int r = p - lane * K;
#pragma unroll
        for (int j = 0; j < K; j++) {
            const bool lp = j == r - 1, rp = j == r;
            li[j] = lp ? c.lli : (rp ? c.rli : li[j]);
            cf[j] = lp ? c.lcf : cf[j];
            cum[j] = lp ? c.pos : cum[j];
        }
    }

    // ------------------------------------------------------------ visibility
    // nodeLength leaf branch for a remote client (mergeTree.ts:1667-1697); dead slots have length 0
    MT_DEV int vis(int j, int32_t R, int C) const {
        // bitwise, not short-circuit: no branch per slot
        const uint32_t f = cf[j];
        const bool seen = ((f & 0xFFu) == (uint32_t)C) | (seq[j] <= R);
        const uint32_t ovw = (W && C > kNarrowClients) ? oh[j] : ov[j];
        const bool hid = ((f & F_RM) != 0) & ((((f >> 8) & 0xFFu) == (uint32_t)C) | (((ovw >> ((C - 1) & 31)) & 1u) != 0) |
                                              (rseq[j] <= R));
        return (seen & !hid & (((lvm >> j) & 1u) != 0)) ? (int)len_of(li[j]) : 0;
    }
    // cum = inclusive prefix of vis over the slots; returns getLength(R, C)
    MT_DEV int scan(int32_t R, int C) {
        int acc = 0;
#pragma unroll
        for (int j = 0; j < K; j++) {
            acc += vis(j, R, C);
            cum[j] = acc;
        }
        const int incl = wave_incl_scan(acc);
        const int excl = incl - acc;
#pragma unroll
        for (int j = 0; j < K; j++) cum[j] += excl;
        return wave_last(incl);
    }
    MT_DEV int cs0() const { return shr1(cum[K - 1], 0); }  // visible start of this lane's first slot

    // ----------------------------------------------------------------- interior levels (LDS)
    MT_DEV uint8_t* lvl(int Lv) { return s.ibcnt[Lv - 1]; }  // Lv >= 1
    MT_DEV int nbl(int Lv) const { return uni(s.nb[Lv]); }

    template <class T>
    MT_DEV void lshift_right(T* a, int from, int count_end) {  // a[from..end) -> a[from+1..end+1)
        for (int hi = count_end; hi > from; hi -= 64) {
            const int i = hi - 1 - lane;
            T v{};
            const bool ok = i >= from;
            if (ok) v = a[i];
            wave_sync();
            if (ok) a[i + 1] = v;
            wave_sync();
        }
    }
    template <class T>
    MT_DEV void lshift_left(T* a, int from, int count_end, int by) {  // a[from..end) -> a[from-by..)
        for (int lo = from; lo < count_end; lo += 64) {
            const int i = lo + lane;
            T v{};
            const bool ok = i < count_end;
            if (ok) v = a[i];
            wave_sync();
            if (ok) a[i - by] = v;
            wave_sync();
        }
    }
    // parent (at level Lv+1) of block b at level Lv, and that parent's first child
    MT_DEV int parent_of(int Lv, int b, int* first_child) {
        const uint8_t* pc = lvl(Lv + 1);
        const int np = nbl(Lv + 1);
        int carry = 0;
        for (int base = 0; base < np; base += 64) {
            const int p = base + lane;
            const int c = p < np ? (int)pc[p] : 0;
            const int incl = wave_incl_scan(c) + carry;
            const uint64_t m = wave_ballot(p < np && incl - c <= b && b < incl);
            if (m) {
                const int fl = first_lane(m);
                if (first_child) *first_child = __builtin_amdgcn_readlane(incl - c, fl);
                return base + fl;
            }
            carry = wave_last(incl);
        }
        return -1;
    }
    // an interior block b at level Lv >= 1 reached kMaxNodes children: split 4/4 upward and
    // grow a new root (mergeTree.ts:2446-2489, 1876-1887)
    MT_DEV bool split_up(int Lv, int b, int32_t sq) {
        for (;;) {
            const int half = kMaxNodes / 2;
            int parent = -1;
            if (Lv < nlev - 1) parent = parent_of(Lv, b, nullptr);
            const int nb = nbl(Lv);
            if (nb + 1 > L::IB) return fail(MT_DERR_CAPACITY, sq), false;
            uint8_t* a = lvl(Lv);
            lshift_right(a, b + 1, nb);
            if (lane == 0) {
                a[b] = (uint8_t)half;
                a[b + 1] = (uint8_t)half;
                s.nb[Lv] = nb + 1;
            }
            wave_sync();
            if (Lv == nlev - 1) {
                if (nlev + 1 > MT_MAXLEV) return fail(MT_DERR_CAPACITY, sq), false;
                const int nl = nlev;
                if (lane == 0) {
                    lvl(nl)[0] = 2;
                    s.nb[nl] = 1;
                }
                nlev = nl + 1;
                wave_sync();
                return true;
            }
            uint8_t* pc = lvl(Lv + 1);
            const int c = uni(pc[parent]) + 1;
            if (lane == 0) pc[parent] = (uint8_t)c;
            wave_sync();
            if (c < kMaxNodes) return true;
            Lv = Lv + 1;
            b = parent;
        }
    }

    // the leaf block of slots [a, e) reached kMaxNodes live children: its child of rank 4 starts
    // the next block (split, mergeTree.ts:2476-2489)
    MT_DEV bool split_leaf(int a, int e, int32_t sq) {
        if (nb0 + 1 > L::LB) return fail(MT_DERR_CAPACITY, sq), false;
        const int s4 = nth_in(lvm, a, e, kMaxNodes / 2);
        int parent = -1;
        if (nlev > 1) parent = parent_of(0, leaf_of(a), nullptr);
        set_bs(s4, true);  // new block, needsScour undefined
        set_sc(s4, MT_SC_UNDEF);
        nb0 += 1;
        if (nlev == 1) {  // the root was the only leaf block: new root with 2 children
            if (lane == 0) {
                s.ibcnt[0][0] = 2;
                s.nb[1] = 1;
            }
            nlev = 2;
            wave_sync();
            return true;
        }
        const int c = uni(s.ibcnt[0][parent]) + 1;
        if (lane == 0) s.ibcnt[0][parent] = (uint8_t)c;
        wave_sync();
        if (c < kMaxNodes) return true;
        return split_up(1, parent, sq);
    }

    // insert e at slot k (a <= k <= en) of the leaf block of slots [a, en) (insertingWalk's child
    // insert, mergeTree.ts:2446-2470)
    // (cut: a boundary split's right part, a copy of slot k - 1 patched after the shift; k > a)
    MT_DEV bool insert_at(int k, int a, int en, const Elem& e, int32_t sq, const Cut& cut, bool dup) {
        if (ns + 1 > CAP) return fail(MT_DERR_CAPACITY, sq), false;
        const bool front = !dup && k == a;  // new first child: it takes over the block's marks
        PROF_BEGIN(ti0, P_B_INS);
        // (a split's right part is the cut slot shifted one register right with its li replaced, in
        // the same pass that writes the left part: no readlane of the slot, no dynamic-index patch)
        const int scv = front ? sc_of(a) : 0;
        shift_in<true>(k, e, front, scv, true, dup);
        if (dup) patch_cut(k, cut);
        if (front) {
            set_bs(k + 1, false);
            set_sc(k + 1, MT_SC_UNDEF);
        }
        PROF_END(prof, P_B_INS, ti0);
        nlive += 1;
        PROF_BEGIN(ti1, P_B_LEAF);
        const bool over = live_in(a, en + 1) >= kMaxNodes;
        PROF_END(prof, P_B_LEAF, ti1);
        if (!over) return true;
        PROF_BEGIN(ti2, P_COMPACT);
        PROF_CNT(P_N_COMPACT, 1);
        const bool r = split_leaf(a, en + 1, sq);
        PROF_END(prof, P_COMPACT, ti2);
        return r;
    }
    MT_DEV int alloc_id(int32_t sq) {
        if (next_id >= CAP) {
            fail(MT_DERR_CAPACITY, sq);
            return -1;
        }
        return next_id++;
    }

    // ------------------------------------------------------------------- text
    // The arena is global memory; arena stores stay in flight until the next arena read.
    MT_DEV void arena_sync() {
        if (dirty) {
            __threadfence_block();
            dirty = false;
        }
    }
    MT_DEV void arena_copy(uint32_t dst, uint32_t src, uint32_t cnt) {
        arena_sync();
        for (uint32_t base = 0; base < cnt; base += 64) {
            const uint32_t i = base + lane;
            if (i < cnt) arena()[dst + i] = arena()[src + i];
        }
        dirty = true;
    }
    // relocate every linked segment's text into the other arena half, in segment-id order: from the
    // per-id lengths and offsets in LDS alone, so no register state is live in here (the content of
    // every segment is what counts; its place in the arena is free)
    MT_DEV void compact_text(int nid) {  // ids [0, nid) are the segments
        PROF_BEGIN(tc, P_COMPACT);
        PROF_CNT(P_N_COMPACT, 1);
        arena_sync();
        const uint8_t* src0 = arena();
        uint8_t* dst = abase + (size_t)(text_half ^ 1u) * textcap;
        uint32_t carry = 0;
        for (int base = 0; base < nid; base += 64) {
            const int i = base + lane;
            const uint32_t l = i < nid ? s.tln[i] : 0u;
            const uint32_t incl = (uint32_t)wave_incl_scan((int)l);
            const uint32_t at = carry + incl - l;
            if (l) {
                const uint8_t* src = src0 + s.toff[i];
#pragma clang loop unroll(disable) vectorize(disable)
                for (uint32_t q = 0; q < l; q++) dst[at + q] = src[q];
                s.toff[i] = (uint16_t)at;
            }
            carry += (uint32_t)wave_last((int)incl);
        }
        dirty = true;
        wave_sync();
        text_half ^= 1u;
        text_top = carry;
        PROF_END(prof, P_COMPACT, tc);
    }
    MT_DEV bool arena_reserve(uint32_t need, int32_t sq, int nid) {
        if (text_top + need <= textcap) return true;
        compact_text(nid);
        if (text_top + need <= textcap) return true;
        fail(MT_DERR_TEXT_ARENA, sq);
        return false;
    }

    // ensureIntervalBoundary(pos) (mergeTree.ts:2241-2245), first half: find the segment visible to
    // the op's view that strictly contains pos and describe its cut (left part in place, cum kept
    // valid for the view; right part entering at slot k1 of the leaf block [ba, be)).  Nothing in
    // the registers changes here: insert_at applies the cut.
    MT_DEV bool split_prep(int pos, int32_t sq, Cut& c, int& k1, int& ba, int& be) {
        PROF_BEGIN(ts0, P_B_SRCH);
        int cs = cs0();
        int hitj = -1;
#pragma unroll
        for (int j = 0; j < K; j++) {
            if (cs < pos && pos < cum[j]) hitj = j;
            cs = cum[j];
        }
        const uint64_t m = wave_ballot(hitj >= 0);
        PROF_END(prof, P_B_SRCH, ts0);
        if (!m) return false;
        PROF_CNT(P_N_SPLIT, 1);
        PROF_BEGIN(tb0, P_B_GET);
        const int lk = first_lane(m);
        const int jk = uni(__builtin_amdgcn_readlane(hitj, lk));
        const int k = lk * K + jk;
        const uint32_t eli = (uint32_t)__builtin_amdgcn_readlane((int)li[jk], lk);
        const uint32_t ecf = (uint32_t)__builtin_amdgcn_readlane((int)cf[jk], lk);
        const int32_t ecum = __builtin_amdgcn_readlane(cum[jk], lk);
        PROF_END(prof, P_B_GET, tb0);
        const uint32_t len = len_of(eli);
        const int off = pos - (ecum - (int)len);
        const int t = alloc_id(sq);
        if (t < 0) return false;
        PROF_BEGIN(tb1, P_B_BLK);
        ba = block_start(k);
        be = next_start(k);
        PROF_END(prof, P_B_BLK, tb1);
        PROF_BEGIN(tb2, P_B_TXT);
        // BaseSegment.splitAt + TextSegment.createSplitSegmentAt (mergeTree.ts:524-568)
        const uint32_t id = id_of(eli);
        const uint64_t pid = s.props[id];  // (issued with the toff read: one LDS round trip)
        const uint32_t to = uniu(s.toff[id]);
        if (lane == 0) {
            s.props[t] = pid;
            s.toff[t] = (uint16_t)(to + (uint32_t)off);
            s.tln[id] = (uint32_t)off;
            s.tln[t] = len - (uint32_t)off;
        }
        c.lli = (uint32_t)off | (id << kLenBits);
        // the left part ends in "\n" only if the segment has one: otherwise known now (F_NLQ: the
        // character is read where the flag is needed -- scour, store)
        c.lcf = (ecf & F_HASNL) ? ((ecf & ~F_NL) | F_NLQ) : (ecf & ~(F_NL | F_NLQ));
        c.rli = (len - (uint32_t)off) | ((uint32_t)t << kLenBits);
        c.pos = pos;
        wave_sync();
        PROF_END(prof, P_B_TXT, tb2);
        if constexpr (EV) {  // MergeTreeMaintenanceType.SPLIT (mergeTree.ts:2231-2236): the right part is not linked yet
            const int lf = live_before(k);
            emit(MT_EV_SPLIT, MT_EVF_FIRST, lf, -1, (uint32_t)off);
            emit(MT_EV_SPLIT, 0u, lf + 1, -1, len - (uint32_t)off);
        }
        k1 = k + 1;
        return true;
    }

    // ------------------------------------------------------------------- heap
    // Heap<LRUSegment> (collections.ts:213-265), comparer maxSeq (mergeTree.ts:923-926)
    // Both sifts are lane-parallel with one LDS round trip per five levels: the path a sift takes
    // depends only on the heap's values before it (the moving key is compared with them, never
    // stored on the way), so the lanes read the candidates first and the walk runs on registers.
    // Push: lane i holds the key's ancestor i + 1 levels up; the key rises past the ancestors
    // while `parent - key > 0` (the exact comparison of collections.ts:228-236).
    MT_DEV bool heap_push(int32_t key, int id, int32_t sq) {
        if (heap_n + 1 >= L::H) return fail(MT_DERR_CAPACITY, sq), false;
        const int k0 = heap_n + 1;
        const int anc = lane < 31 ? (k0 >> (lane + 1)) : 0;
        const bool has = anc >= 1;
        const int32_t av = has ? s.hseq[anc] : 0;
        const uint16_t as = has ? s.hslot[anc] : (uint16_t)0;
        const int up = first_lane(wave_ballot(!has || av - key <= 0));  // levels the key rises
        wave_sync();
        if (lane < up) {  // ancestor `lane` moves one level down, into its child on the path
            const int child = k0 >> lane;
            s.hseq[child] = av;
            s.hslot[child] = as;
        }
        if (lane == 0) {
            s.hseq[k0 >> up] = key;
            s.hslot[k0 >> up] = (uint16_t)id;
        }
        heap_n = heap_n + 1;
        wave_sync();
        return true;
    }
    // Pop (collections.ts:240-263): the last entry x replaces the root and sinks along the
    // smaller-child path (the left child unless the right one is strictly smaller) while
    // `x - child > 0`.  Lane t < 62 holds the node t + 2 of the five-level subtree below k in
    // heap order (relative index r at lane r - 2); the path is decided from two ballots -- "the
    // right sibling is strictly smaller" at every left child, "x - node <= 0" at every node -- by
    // bit walks on the scalar unit, with no readlane per level, and the path's nodes move up one
    // level in one masked LDS store.  (The first window's read also fetches the root's segment and
    // the last entry, in lanes 62 and 63: one LDS round trip per window.)
    MT_DEV int heap_pop() {
        const int cnt = heap_n - 1;
        int k = 1, id = 0;
        int32_t x = 0;
        uint32_t xs = 0;
        const int r = lane + 2;
        const int dep = 31 - __builtin_clz((uint32_t)r);
        for (bool first = true, more = true; more; first = false) {
            const int node = (k << dep) + (r - (1 << dep));
            const bool ok = lane < 62 && node <= cnt;
            const int at = lane < 62 ? (ok ? node : 0) : (lane == 62 ? heap_n : 1);
            const int32_t v = (ok || (first && lane >= 62)) ? s.hseq[at] : 0;
            const uint32_t sl = (ok || (first && lane >= 62)) ? (uint32_t)s.hslot[at] : 0u;
            if (first) {
                id = uni(__builtin_amdgcn_readlane((int)sl, 63));
                x = uni(__builtin_amdgcn_readlane(v, 62));
                xs = uniu((uint32_t)__builtin_amdgcn_readlane((int)sl, 62));
            }
            const int32_t vr = shl1(v, 0);
            const bool rok = shl1(ok ? 1 : 0, 0) != 0;  // the right sibling exists
            const uint64_t pick = wave_ballot((r & 1) == 0 && ok && rok && v - vr > 0);
            const uint64_t stop = wave_ballot(ok && x - v <= 0);
            wave_sync();
            uint64_t path = 0;
            int rr = 1;
            more = false;
            for (int lv = 0; lv < 5; lv++) {
                if ((k << 1) > cnt) break;
                const int jr = (rr << 1) + (int)((pick >> ((rr << 1) - 2)) & 1u);
                if ((stop >> (jr - 2)) & 1u) break;
                path |= 1ull << (jr - 2);
                k = (k << 1) + (jr & 1);
                rr = jr;
                more = lv == 4 && (k << 1) <= cnt;
            }
            if ((path >> lane) & 1u) {  // the path's children move up into their parents
                s.hseq[node >> 1] = v;
                s.hslot[node >> 1] = (uint16_t)sl;
            }
            wave_sync();
        }
        if (lane == 0) {
            s.hseq[k] = x;
            s.hslot[k] = (uint16_t)xs;
        }
        heap_n = heap_n - 1;
        wave_sync();
        return id;
    }
    // addToLRUSet (mergeTree.ts:1273-1283) for segment `id` in the leaf block starting at slot a
    MT_DEV bool add_lru(int a, int id, int32_t sq) {
        if (sc_of(a) != MT_SC_TRUE && sq > cur_seq) {
            set_sc(a, MT_SC_TRUE);
            return heap_push(sq, id, sq);
        }
        return true;
    }

    // ---------------------------------------------------------------- zamboni
    MT_DEV int slot_of_id(int id) const {  // -1 once unlinked (segment.parent === undefined)
        int hit = -1;
#pragma unroll
        for (int j = 0; j < K; j++)
            if ((int)id_of(li[j]) == id && ((lvm >> j) & 1u)) hit = idx(j);
        const uint64_t m = wave_ballot(hit >= 0);
        if (!m) return -1;
        return __builtin_amdgcn_readlane(hit, first_lane(m));
    }

    // TextSegment.append (textSegment.ts:76-85) of a whole run: the live child of rank p absorbs
    // the following children whose bits are set in runm.  Only the text content is state, so
    // the run is made contiguous once (or found contiguous) instead of pair by pair.  Lane q of
    // (vli, vcf, vslot) holds the block's live child of rank q.
    // The head's new li / cf are returned (hli, hcf), not written to the register state here: scour
    // writes every head back after its run loop, so the loop carries no register state.
    MT_DEV void append_run(int p, uint32_t runm, uint32_t vli, uint32_t vcf, uint32_t& hli, uint32_t& hcf) {
        const uint32_t pli = (uint32_t)__builtin_amdgcn_readlane((int)vli, p);
        const uint32_t pid_ = id_of(pli);
        const uint32_t lastq = 31u - (uint32_t)__builtin_clz(runm);
        // per-lane piece: lane q of the run holds (offset, length); exclusive prefix = its place
        const bool in_run = lane == p || (lane < 32 && ((runm >> lane) & 1u));
        const uint32_t myl = in_run ? len_of(vli) : 0u;
        const uint32_t incl = (uint32_t)wave_incl_scan((int)myl);
        const uint32_t total = (uint32_t)wave_last((int)incl);
        for (int pass = 0; pass < 2; pass++) {
            // adjacent views: every piece starts where the run's text so far would end
            const uint32_t myt = in_run ? (uint32_t)s.toff[id_of(vli)] : 0u;
            const uint32_t pt = uniu((uint32_t)__builtin_amdgcn_readlane((int)myt, p));
            const bool adj = __ballot(in_run && myt != pt + (incl - myl)) == 0;
            if (adj) break;  // nothing to copy
            if (pass == 0) {
                if (!arena_reserve(total, cur_seq, next_id)) return;
                continue;    // a compaction lays the run out contiguously
            }
            const uint32_t top = text_top;
            PROF_CNT(P_N_APPBYTES, total);
            uint64_t pieces = __ballot(in_run);
            while (pieces) {
                const int q = first_lane(pieces);
                pieces &= pieces - 1;
                const uint32_t ql = (uint32_t)__builtin_amdgcn_readlane((int)myl, q);
                const uint32_t qt = (uint32_t)__builtin_amdgcn_readlane((int)myt, q);
                const uint32_t at = top + (uint32_t)__builtin_amdgcn_readlane((int)(incl - myl), q);
                arena_copy(at, qt, ql);
            }
            if (lane == 0) s.toff[pid_] = (uint16_t)top;
            text_top = top + total;
            wave_sync();
        }
        if (lane == 0) s.tln[pid_] = total;
        const uint32_t pcf = (uint32_t)__builtin_amdgcn_readlane((int)vcf, p);
        const uint32_t lcf = (uint32_t)__builtin_amdgcn_readlane((int)vcf, (int)lastq);
        const uint32_t anynl = __ballot(in_run && (vcf & F_HASNL)) ? F_HASNL : 0u;
        hli = total | (pid_ << kLenBits);
        hcf = (pcf & ~F_NL) | (lcf & F_NL) | anynl;
    }

    // scourNode on the leaf block whose slots are [a, e) (mergeTree.ts:1289-1365); returns the
    // block's new child count.  Unlinked children become DEAD slots in place.
    MT_DEV int scour(int a, int e) {
        const uint32_t lb = live_bits() & below(e) & ~below(a);
        const int c = __popc(lb);
        const int incl = wave_incl_scan(c);
        const int rbase = incl - c;
        const int cnt = wave_last(incl);
        if (cnt > kMaxNodes) return fail(MT_DERR_CAPACITY, cur_seq), cnt;
        // the live children, rank by rank, through LDS scratch (one 16-byte record each: the
        // removal seq of a removed child, else its seq -- the only one the decisions read)
        // (every lane stores every slot: a slot that is no live child of the block goes to the
        // lane's discard words -- no per-slot branch)
        uint32_t* const dum = reinterpret_cast<uint32_t*>(s.dum) + lane;  // (z[0 .. 3 kMaxNodes])
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int q = rbase + __popc(lb & ((1u << j) - 1u));
            uint32_t* const z = ((lb >> j) & 1u) ? &s.zr[q] : dum;
            z[0] = (uint32_t)((cf[j] & F_RM) ? rseq[j] : seq[j]);
            z[kMaxNodes] = li[j];
            z[2 * kMaxNodes] = cf[j];
            z[3 * kMaxNodes] = (uint32_t)idx(j);
        }
        wave_sync();
        const bool mine = lane < cnt;
        // (every lane reads -- lane q < 8 its child's words, the others words of the scratch area
        // behind them -- and the values are selected after: no exec-masked branch per read)
        const int zq = lane & (kMaxNodes - 1);
        const uint32_t r0 = s.zr[zq], r1 = s.zr[kMaxNodes + zq], r2 = s.zr[2 * kMaxNodes + zq],
                       r3 = s.zr[3 * kMaxNodes + zq];
        const int32_t vsq = mine ? (int32_t)r0 : 0;
        const uint32_t vli = mine ? r1 : 0u;
        uint32_t vcf = mine ? r2 : 0u;
        const int vslot = mine ? (int)r3 : 0;
        const uint64_t pr = s.props[mine ? id_of(vli) : 0u];
        const uint64_t vpr = mine ? pr : 0ull;
        if (__ballot(mine && (vcf & F_NLQ))) {  // the children's pending ENDS_WITH_NEWLINE, in one load
            arena_sync();
            if (mine && (vcf & F_NLQ)) {
                const uint8_t c = arena()[(uint32_t)s.toff[id_of(vli)] + len_of(vli) - 1];
                vcf = (vcf & ~(F_NL | F_NLQ)) | (c == '\n' ? F_NL : 0u);
            }
        }
        // scourNode's decisions (mergeTree.ts:1289-1365), lane-parallel: child q is unlinked if it
        // is a tombstone at or below the MSN; it is appended to the run before it if both are live,
        // acked at or below the MSN and non-empty, the run does not end in "\n", the props match
        // (canAppend textSegment.ts:63-68, matchProperties properties.ts:62-93) -- the run's
        // newline and props are those of child q-1 -- and the run or q is within
        // TextSegmentGranularity; only that last clause depends on earlier decisions
        const int32_t minSeq = min_seq;
        const bool rm = mine && (vcf & F_RM) != 0;
        const uint32_t ql = len_of(vli);
        const bool elig = mine && !rm && vsq <= minSeq && ql > 0;
        const bool pelig = shr1(elig ? 1 : 0, 0) != 0;
        const uint32_t pcf = (uint32_t)shr1((int)vcf, 0);
        const uint32_t pprl = (uint32_t)shr1((int)(uint32_t)vpr, 0);
        const uint32_t pprh = (uint32_t)shr1((int)(uint32_t)(vpr >> 32), 0);
        // (canAppend needs two text segments: a Marker neither appends nor is appended to,
        // mergeTree.ts:793, textSegment.ts:63-68)
        const bool a0 = elig && pelig && !((pcf | vcf) & F_MARKER) && !(pcf & F_NL) && ((pcf ^ vcf) & F_PDEF) == 0 && pprl == (uint32_t)vpr &&
                        pprh == (uint32_t)(vpr >> 32);
        const uint32_t a0m = (uint32_t)__ballot(a0);
        uint32_t appm = a0m;
        if (__ballot(a0 && ql > (uint32_t)kTextGranularity)) {
            // a long child joins only a run still within the granularity: walk the runs in order
            const uint32_t em = (uint32_t)__ballot(elig);
            uint32_t plen = 0;
            appm = 0;
            for (int q = 0; q < cnt; q++) {
                const uint32_t lq = (uint32_t)__builtin_amdgcn_readlane((int)ql, q);
                if (((a0m >> q) & 1u) && (plen <= (uint32_t)kTextGranularity || lq <= (uint32_t)kTextGranularity)) {
                    appm |= 1u << q;
                    plen += lq;
                } else {
                    plen = ((em >> q) & 1u) ? lq : 0u;
                }
            }
        }
        const uint32_t unlink = (uint32_t)__ballot(rm && vsq <= minSeq) | appm;
        const int kept = cnt - __popc(unlink);
        // lane q appended: the child of the run's head, the last child before q not appended
        const uint32_t heads = ~appm & ((1u << (lane & 31)) - 1u);
        const int vtgt = (lane < 32 && ((appm >> lane) & 1u)) ? 31 - __builtin_clz(heads) : -1;
        if constexpr (EV) {
            // UNLINK (mergeTree.ts:1310-1315) and APPEND (:1335-1340) callbacks in child order: child q
            // is named by the block's first ordinal plus the children kept before it (the earlier ones
            // are gone by then); an APPEND pair names the run's head with its grown length, then q
            const bool app = vtgt >= 0;
            const bool tomb = mine && ((unlink >> lane) & 1u) && !app;
            const int kb = lane - __popc(unlink & (lane < 32 ? ((1u << lane) - 1u) : 0xFFFFFFFFu));
            const int nrec = tomb ? 1 : (app ? 2 : 0);
            const int rinc = wave_incl_scan(nrec);
            const int rtot = wave_last(rinc);
            if (rtot) {
                const int st = live_before(a);
                const int ainc = wave_incl_scan(app ? (int)ql : 0);
                const int hp = app ? vtgt : lane;
                const int kbp = __shfl(kb, hp, 64), aincp = __shfl(ainc, hp, 64);
                const uint32_t lenp = (uint32_t)__shfl((int)ql, hp, 64);
                const int o = evn + rinc - nrec;
                if (tomb && o < (int)evcap) put_event(evp + o, evseq, MT_EV_UNLINK, MT_EVF_FIRST, st + kb, -1, ql);
                if (app) {
                    if (o < (int)evcap)
                        put_event(evp + o, evseq, MT_EV_APPEND, MT_EVF_FIRST, st + kbp, -1, lenp + (uint32_t)(ainc - aincp));
                    if (o + 1 < (int)evcap) put_event(evp + o + 1, evseq, MT_EV_APPEND, 0u, st + kb, -1, ql);
                }
                evn = evn + rtot;
            }
        }
        PROF_CNT(P_N_UNLINK, __popc(unlink));
        uint64_t runs = __ballot(vtgt >= 0);
        if (runs) {
            // the runs' text work; each head's new li / cf parked in its child lane (nli / ncf) ...
            uint32_t nli = vli, ncf = vcf, heads = 0;
            while (runs) {
                const int p = __builtin_amdgcn_readlane(vtgt, first_lane(runs));
                const uint64_t runm = __ballot(vtgt == p);
                runs &= ~runm;
                PROF_CNT(P_N_APPEND, __popcll(runm));
                uint32_t hli = 0, hcf = 0;
                append_run(p, (uint32_t)runm, vli, vcf, hli, hcf);
                if (err) return cnt;
                nli = lane == p ? hli : nli;
                ncf = lane == p ? hcf : ncf;
                heads |= 1u << p;
            }
            // ... and written back in one pass: register j of a lane holds the block's child of rank
            // q (its prefix count), which reads its new values from lane q (no state in the loop above)
#pragma unroll
            for (int j = 0; j < K; j++) {
                const int q = rbase + __popc(lb & ((1u << j) - 1u));
                const bool hit = ((lb >> j) & 1u) && q < 32 && ((heads >> q) & 1u);
                const uint32_t xl = (uint32_t)__builtin_amdgcn_ds_bpermute(q << 2, (int)nli);
                const uint32_t xc = (uint32_t)__builtin_amdgcn_ds_bpermute(q << 2, (int)ncf);
                li[j] = hit ? xl : li[j];
                cf[j] = hit ? xc : cf[j];
            }
        }
        // unlink: the slots become dead in place (their block marks stay)
        const bool gone = mine && ((unlink >> lane) & 1u);
        if (gone) s.tln[id_of(vli)] = 0u;
        uint64_t gm = __ballot(gone);
        uint32_t kill = 0;
        while (gm) {
            const int sl = __builtin_amdgcn_readlane(vslot, first_lane(gm));
            gm &= gm - 1;
            if (sl / K == lane) kill |= 1u << (sl % K);
        }
        lvm &= ~kill;
        nlive -= __popc(unlink);
        return kept;
    }

    // The block-count half of pack (mergeTree.ts:1368-1420) for interior levels Lv >= 1: the m
    // children of block P at level Lv+1 (`total` grandchildren) are repacked evenly, recursing up.
    MT_DEV void repack(int Lv, int P, int first_child, int m, int total) {
        for (;;) {
            const int half = kMaxNodes / 2;
            int cc = min(kMaxNodes - 1, total / half);
            if (cc < 1) cc = 1;
            const int base = total / cc, extra = total % cc;
            uint8_t* a = lvl(Lv);
            const int nb = nbl(Lv);
            wave_sync();
            if (cc < m) {
                lshift_left(a, first_child + m, nb, m - cc);
            } else if (cc > m) {
                for (int q = 0; q < cc - m; q++) lshift_right(a, first_child + m, nb + q);
            }
            if (lane < cc) a[first_child + lane] = (uint8_t)(base + (lane < extra ? 1 : 0));
            wave_sync();
            if (lane == 0) {
                s.nb[Lv] = nb + cc - m;
                lvl(Lv + 1)[P] = (uint8_t)cc;
            }
            wave_sync();
            if (!(cc < kMaxNodes / 2 && (Lv + 1) < nlev - 1)) return;  // underflow(parent) && parent.parent
            int fc = 0;
            const int PP = parent_of(Lv + 1, P, &fc);
            Lv = Lv + 1;
            P = PP;
            first_child = fc;
            m = uni(lvl(Lv + 1)[P]);
            total = 0;
            const uint8_t* c = lvl(Lv);
            for (int j = first_child; j < first_child + m; j++) total += uni(c[j]);
        }
    }
    // pack at the leaf level: the m leaf blocks under level-1 block P (first fc; `total` live
    // children after scouring) become cc evenly filled blocks -- only block marks change
    MT_DEV void repack_leaf(int P, int fc, int m, int total, int A, int E) {
        const int half = kMaxNodes / 2;
        int cc = min(kMaxNodes - 1, total / half);
        if (cc < 1) cc = 1;
        const int base = total / cc, extra = total % cc;
        // the new block starts: slot A, then the live children of ranks t * base + min(t, extra)
        // (one uniform lookup per new block, not a compare network per register); every new block:
        // needsScour undefined
        const uint32_t rng = below(E) & ~below(A);
        bsm &= ~rng;
        sc0 &= ~rng;
        sc1 &= ~rng;
        set_bs(A, true);
#pragma clang loop unroll(disable)
        for (int t = 1; t < cc; t++) set_bs(nth_in(lvm, A, E, t * base + min(t, extra)), true);
        nb0 += cc - m;
        if (lane == 0) s.ibcnt[0][P] = (uint8_t)cc;
        wave_sync();
        if (cc < kMaxNodes / 2 && 1 < nlev - 1) {  // underflow(parent) && parent.parent
            int fc2 = 0;
            const int PP = parent_of(1, P, &fc2);
            const int m2 = uni(lvl(2)[PP]);
            int total2 = 0;
            for (int j = fc2; j < fc2 + m2; j++) total2 += uni(lvl(1)[j]);
            repack(1, PP, fc2, m2, total2);
        }
    }

    // zamboniSegments (mergeTree.ts:1422-1478), zamboniSegmentsMaxCount = 2.  One scour call
    // site: step 0 scours the popped segment's block; on underflow steps 1..m scour every
    // sibling under its parent (pack's scourNode loop), then repack.
    MT_DEV void zamboni() {
        // (continues and returns folded into conditions: one exit per loop, see apply)
#pragma unroll
        for (int it = 0; it < 2 && !err; it++) {
            if (heap_n == 0 || uni(s.hseq[1]) > min_seq) break;
            PROF_BEGIN(tz, P_ZPOP);
            const int id = heap_pop();
            const int k = id == (int)kDead ? -1 : slot_of_id(id);
            if (k < 0) continue;
            const int a = block_start(k), e = next_start(k);
            PROF_END(prof, P_ZPOP, tz);
            if (sc_of(a) == MT_SC_FALSE) continue;
            const int cnt = live_in(a, e);
            int P = -1, fc = 0, m = 0, total = 0;
            int A = 0, ee = e;  // pack: the first sibling's start, and the end of the last scoured one
            for (int step = 0;; step++) {
                int aa = a;
                if (step > 0) {  // the siblings under the parent, left to right
                    aa = step == 1 ? A : ee;
                    ee = next_start(aa);
                }
                PROF_BEGIN(ts, P_SCOUR);
                PROF_CNT(P_N_SCOUR, 1);
                const int kept = scour(aa, ee);
                PROF_END(prof, P_SCOUR, ts);
                bool more = !err;
                if (more) {
                    if (step == 0) {
                        set_sc(a, MT_SC_FALSE);
                        more = kept < cnt && kept < kMaxNodes / 2 && nlev > 1;
                        if (more) {
                            P = parent_of(0, leaf_of(a), &fc);
                            m = uni(s.ibcnt[0][P]);
                            A = bs_slot(fc);
                        }
                    } else {
                        total += kept;
                    }
                }
                if (!more || step == m) break;
            }
            PROF_BEGIN(tr, P_REPACK);
            if (P >= 0 && !err) repack_leaf(P, fc, m, total, A, ee);
            PROF_END(prof, P_REPACK, tr);
        }
    }

    // -------------------------------------------------------------------- ops
    // byte i of the current op's payload (uniform i): from the prefetch register when it can
    MT_DEV uint32_t pbyte(const uint8_t* pay, int i) const {
        return i < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)pb, i) : (uint32_t)pay[i];
    }
    // props: apply the op's (key, value) pairs at payload offset off; value 0 = null = delete
    // (properties.ts:95-116)
    MT_DEV uint64_t apply_pairs(uint64_t p, const uint8_t* pay, int off, int np) const {
        for (int q = 0; q < np; q++) {
            const int k = (int)pbyte(pay, off + 2 * q);
            const uint64_t v = pbyte(pay, off + 2 * q + 1);
            p = (p & ~(0xFFull << (8 * k))) | (v << (8 * k));
        }
        return p;
    }

    // blockInsert (mergeTree.ts:2141-2224) of a text segment at pos, after the boundary split:
    // choose its slot k in leaf block b, write its text and cold fields, build its element.
    // Returns its id (< 0 on error) and its child index inside block b before a possible split.
    // kl >= 0: the boundary split at pos just cut the segment at slot kl (its right part is at kl + 1).
    // Then the walk needs no search: the first block whose cumulative end >= pos is kl's block (every
    // earlier block ends at or before kl's start, < pos), and in it the first child with pos < end is
    // the right part -- or, when the split's leaf split moved the right part into the next block,
    // kl's block ends at kl and the segment goes at its end: slot kl + 1 either way.
    MT_DEV int place_prep(const mt_op_rec op, const uint8_t* pay, int tlen, int np, Elem& en,
                          int& k, int& ba, int& be, int kl) {
        const int32_t S = op.seq, R = op.ref_seq;
        const int C = op.client, pos = op.pos1;
        if (kl >= 0) {
            k = kl + 1;
            ba = block_start(kl);
            be = next_start(kl);
        } else {
        // insertingWalk descends into the first block whose cumulative visible end >= pos
        // (breakTie is true for blocks, :2248-2277).  cum is monotone over the slots, so that is the
        // block holding the first slot with cum >= pos: every block before it ends at a slot before
        // that one, at a cumulative end < pos
        // (bitwise, not short-circuit, here and below: no exec-masked branch per register)
        int first = 0x7fffffff;
#pragma unroll
        for (int j = K - 1; j >= 0; j--) {
            const int i = idx(j);
            first = ((i < ns) & (cum[j] >= pos)) ? i : first;
        }
        first = first_hit(first);  // slots are blocked by lane: the first lane with a hit has the minimum
        if (first == 0x7fffffff) return fail(MT_DERR_INSERT_FAILED, S), -1;
        const int a = block_start(first), e = next_start(first);
        ba = a;
        be = e;
        // leaf placement: first child with pos < len, or pos == len == 0 and breakTie; else the
        // end of the block (:2431-2444)
        int best = 0x7fffffff;
        {
            const int cs = cs0();
#pragma unroll
            for (int j = K - 1; j >= 0; j--) {
                const int i = idx(j);
                const int ce = cum[j];
                const int csj = j ? cum[j - 1] : cs;
                const bool rm_before = ((cf[j] & F_RM) != 0) & (rseq[j] <= R);
                const bool h = (((lvm >> j) & 1u) != 0) & (i >= a) & (i < e) &
                               ((ce > pos) | ((ce == pos) & (csj == pos) & !rm_before));
                best = h ? i : best;
            }
        }
        best = first_hit(best);
        k = best != 0x7fffffff ? best : e;
        }
        const int t = alloc_id(S);
        if (t < 0) return -1;
        if (!arena_reserve((uint32_t)tlen, S, t)) return -1;  // (t's text is not written yet)
        const uint32_t top = text_top;
        bool hasnl = false;
        uint8_t* const ar = arena();
        for (int base = 0; base < tlen; base += 64) {
            const int i = base + lane;
            const uint8_t c = i < tlen ? (uint8_t)(base == 0 ? pb : pay[i]) : 0;
            if (i < tlen) ar[top + i] = c;
            hasnl = hasnl || __ballot(i < tlen && c == '\n') != 0;
        }
        dirty = true;
        // a Marker (MT_F_MARKER): length 1, its one arena byte is its ReferenceType, no newline
        uint32_t fl = (op.flags & MT_F_MARKER) ? F_MARKER
                                               : ((pbyte(pay, tlen - 1) == '\n' ? F_NL : 0u) | (hasnl ? F_HASNL : 0u));
        uint64_t p = 0;
        if (op.flags & MT_F_PROPS) {  // TextSegment.make -> addProperties
            fl |= F_PDEF;
            p = apply_pairs(0, pay, tlen, np);
        }
        if (lane == 0) {
            s.props[t] = p;
            s.toff[t] = (uint16_t)top;
            s.tln[t] = (uint32_t)tlen;
        }
        text_top = top + (uint32_t)tlen;
        wave_sync();
        en.seq = S;
        en.rseq = 0;
        en.li = (uint32_t)tlen | ((uint32_t)t << kLenBits);
        en.cf = (uint32_t)C | fl;
        en.ov = 0;
        en.oh = 0;
        en.cum = pos + tlen;
        return t;
    }

    // markRangeRemoved / annotateRange leaf actions over mapRange (mergeTree.ts:2607-2719,
    // 2565-2605, 2903-2965) after the two boundary splits
    MT_DEV void range_action(const mt_op_rec op, const uint8_t* pay, int tlen, int np) {
        const int32_t S = op.seq;
        const int C = op.client, start = op.pos1, end = op.pos2;
        const bool is_remove = op.type == MT_OP_REMOVE;
        const bool rewrite = op.flags & MT_F_REWRITE;
        const uint32_t cbit = 1u << ((C - 1) & 31);
        const bool hic = W && C > kNarrowClients;  // (W) the client's bit is in oh
        // the op's (key, value) pairs as one uniform clear mask and set value: later pairs win, as
        // applied in order (properties.ts:95-116)
        uint64_t pclr = 0, pset = 0;
        if (!is_remove) {
            for (int q = 0; q < np; q++) {
                const int k = (int)pbyte(pay, tlen + 2 * q);
                const uint64_t m = 0xFFull << (8 * k);
                pclr |= m;
                pset = (pset & ~m) | ((uint64_t)pbyte(pay, tlen + 2 * q + 1) << (8 * k));
            }
        }
        uint32_t tm = 0;  // touched slots of this lane
        {
            int cs = cs0();
#pragma unroll
            for (int j = 0; j < K; j++) {
                const int ce = cum[j];
                tm |= (ce > cs && cs < end && ce > start) ? (1u << j) : 0u;
                cs = ce;
            }
        }
        if (EV && !is_remove) emit_range(false, S, C, tm, pclr, pset, rewrite);
        if (is_remove) {
            // branch-free register updates (a store per branch would merge into a pointer phi and
            // push the state arrays to scratch)
#pragma unroll
            for (int j = 0; j < K; j++) {
                const bool touched = (tm >> j) & 1u;
                const uint32_t f = cf[j];
                const bool was_rm = (f & F_RM) != 0;
                const bool mark = touched && !was_rm;    // first remover wins
                const bool overlap = touched && was_rm;  // addOverlappingClient
                ov[j] = (overlap && !hic) ? (ov[j] | cbit) : ov[j];
                if constexpr (W) oh[j] = (overlap && hic) ? (oh[j] | cbit) : oh[j];
                rseq[j] = mark ? S : rseq[j];
                cf[j] = mark ? ((f & ~0xFF00u) | F_RM | ((uint32_t)C << 8)) : f;
            }
        } else {
            // SegmentPropertiesManager.addProperties (remote, no combining op) on the touched slots'
            // property sets, four slots per LDS round trip: every lane reads and writes
            // unconditionally, an untouched slot through the lane's discard word, so there is no
            // per-slot branch and no per-slot wait
            uint64_t* const dum = s.dum + lane;
            constexpr int Q = 4;
#pragma unroll
            for (int j0 = 0; j0 < K; j0 += Q) {
                uint64_t* pa[Q];
                uint64_t pv[Q];
#pragma unroll
                for (int q = 0; q < Q; q++) {
                    if (j0 + q < K) {
                        pa[q] = ((tm >> (j0 + q)) & 1u) ? &s.props[id_of(li[j0 + q])] : dum;
                        pv[q] = *pa[q];
                    }
                }
#pragma unroll
                for (int q = 0; q < Q; q++) {
                    if (j0 + q < K) {
                        const uint64_t p = ((cf[j0 + q] & F_PDEF) && !rewrite) ? pv[q] : 0ull;
                        *pa[q] = (p & ~pclr) | pset;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < K; j++) cf[j] = ((tm >> j) & 1u) ? (cf[j] | F_PDEF) : cf[j];
        }
        if (EV && is_remove) emit_range(true, S, C, tm, 0, 0, false);
        // addToLRUSet for the touched segments in document order: one push per leaf block
        // (its first touched child) whose needsScour is not already true
        int from = 0;
        for (;;) {
            const int k = first_from(tm, from);
            if (k >= ns) break;
            if (!add_lru(block_start(k), (int)id_of(get_li(k)), S)) return;
            from = next_start(k);
        }
    }

    // Client.applyMsg for the observer (client.ts:797-828): the op, then updateSeqNumbers
    // (client.ts:821-828, MergeTree.setMinSeq mergeTree.ts:1718-1736).  Every register-heavy
    // routine has exactly one call site.
    MT_DEV void apply(const mt_op_rec op, const uint8_t* payload) {
        const int np = MT_OP_NPAIRS(op);
        const int32_t S = op.seq;
        if (op.type > MT_OP_NOOP) return fail(MT_DERR_BAD_OP, S);  // (err: the op loop stops)
        const uint8_t* pay = payload + op.payload_off;
        const int tlen = (int)op.payload_len - 2 * np;
        const bool noop = MT_OP_IS_NOOP(op);  // incl. an empty-string insert (client.ts:403-407)
        if constexpr (EV) evseq = S;
        // (the checks set a code instead of returning: apply runs inlined in the op loop, and every
        // early exit is one more edge the CFG structurizer routes the register state along)
        int bad = 0;
        const bool ins = op.type == MT_OP_INSERT;
        if (!noop) {
            uint32_t kmax = 0;
            if (op.payload_len >= (uint32_t)(2 * np))
                for (int q = 0; q < np; q++) kmax = max(kmax, pbyte(pay, tlen + 2 * q));
            // the window asserts (completeAndLogOp client.ts:461-464, updateSeqNumbers :826) are
            // decided before any edit: the document halts before the failing message.  (The
            // reference runs them after the op, so a failing insert outranks them: mt_fixup_kernel,
            // after the apply, from the halted state.)
            bad = (op.client == 0 || op.client > (W ? kC64Clients : kNarrowClients)) ? MT_DERR_LIMITS
                  : (op.payload_len < (uint32_t)(2 * np) || !MT_OP_NO_TEXT_OK(op)) ? MT_DERR_BAD_OP
                  : (np > 0 && kmax >= MT_MAX_KEYS) ? MT_DERR_LIMITS
                  : (op.pos1 < 0 || (!ins && op.pos2 < 0)) ? MT_DERR_BAD_OP
                  : !(cur_seq < S) ? MT_DERR_SEQ_ORDER
                  : (!(min_seq <= op.msn) || !(op.msn <= S)) ? MT_DERR_MSN_ORDER : 0;
            if (bad) fail(bad, S);
        }
        if (!noop && !bad) {
            PROF_BEGIN(t0, P_SCAN);
            scan(op.ref_seq, op.client);
            PROF_END(prof, P_SCAN, t0);
            // insertion steps: the boundary splits (ensureIntervalBoundary), then for an insert
            // the new segment; every step ends in the one insert_at call site
            const int nsteps = ins ? (tlen > 0 ? 2 : 1) : 2;
            int kl = -1;  // (an insert) the slot of the segment the boundary split at pos cut
            // (one exit: every failing step has set err -- a return or continue from inside the loop
            // is a multi-exit region that the CFG structurizer lowers with a flow variable and
            // copies of the register state on its edges)
            // nsteps <= 2: unrolled, the two steps keep their own register assignment instead of
            // joining the whole state at a loop back edge (C3 +4.0%, C4 +3.8%, C5 +5.7%:
            // profiles/r06_ab/ab6_step_unroll_*)
#pragma unroll
            for (int step = 0; step < 2 && step < nsteps; step++) {
                PROF_BEGIN2(t1, P_BOUND, P_INSERT);
                const bool placing = ins && step == 1;
                Elem e{};
                Cut cut{};
                int k = 0, ba = 0, be = 0, t = -1;
                bool go;
                if (!placing) {
                    go = split_prep(step == 0 ? op.pos1 : op.pos2, S, cut, k, ba, be);
                    if (go) kl = k - 1;
                } else {
                    t = place_prep(op, pay, tlen, np, e, k, ba, be, uni(kl));
                    go = t >= 0;
                }
                if (go) {
                    // (uniform by construction; the phi that merges the two prep paths is not
                    // provably so, and its users would run on the VALU)
                    k = uni(k);
                    ba = uni(ba);
                    be = uni(be);
                    t = uni(t);
#ifdef MT_UNI_ELEM
                    // (the inserted element and the cut as scalars: 4-8 B less scratch in most classes)
                    e.seq = uni(e.seq);
                    e.rseq = uni(e.rseq);
                    e.li = uniu(e.li);
                    e.cf = uniu(e.cf);
                    e.ov = uniu(e.ov);
                    e.oh = uniu(e.oh);
                    e.cum = uni(e.cum);
                    cut.lli = uniu(cut.lli);
                    cut.lcf = uniu(cut.lcf);
                    cut.rli = uniu(cut.rli);
                    cut.pos = uni(cut.pos);
#endif
                    const bool ok = insert_at(k, ba, be, e, S, cut, !placing);
                    if (placing) {
                        PROF_END(prof, P_INSERT, t1);
                    } else {
                        PROF_END(prof, P_BOUND, t1);
                    }
                    if (ok && placing) {
                        // saveIfLocal -> addToLRUSet (mergeTree.ts:2164-2179): the new segment's block
                        // after a possible split, the one holding slot k
                        const bool lru = S > min_seq ? add_lru(block_start(k), t, S) : true;
                        if (EV && lru)  // MergeTreeDeltaType.INSERT (mergeTree.ts:1981-1988)
                            emit(MT_EV_INSERT, MT_EVF_FIRST, live_before(k), local_before(k), (uint32_t)tlen);
                    }
                }
                if (err) break;
            }
            if (!err) {
                if (EV && ins && tlen == 0) emit(MT_EV_INSERT, MT_EVF_FIRST, -1, -1, 0);  // an empty text with props: never linked
                if (!ins) {
                    PROF_BEGIN(t2, P_RANGE);
                    range_action(op, pay, tlen, np);
                    PROF_END(prof, P_RANGE, t2);
                }
            }
        }
        const int32_t msn = op.msn;
        // zamboni after the op, then updateSeqNumbers and zamboni again when the msn moved: one call
        // site, one exit (err)
        // (unrolled, as the zamboni passes and the steps: C3 +2.2 %, C5 +3.1 %, profiles/r06_ab/ab7_*)
#pragma unroll
        for (int ph = 0; ph < 2 && !err; ph++) {
            bool run = !noop;
            if (ph == 1) {
                run = false;
                if (!(op.flags & MT_F_GROUP_MORE)) {
                    // (a non-op message's asserts, all before its edits: the document halts before it)
                    if (!(cur_seq <= S)) {
                        fail(MT_DERR_SEQ_ORDER, S);  // client.ts:824
                    } else if (!(msn <= S) || !(min_seq <= msn)) {
                        fail(MT_DERR_MSN_ORDER, S);  // :826, mergeTree.ts:1722
                    } else {
                        cur_seq = S;
                        run = msn > min_seq;
                        if (run) min_seq = msn;
                    }
                }
            }
            if (run) {
                PROF_BEGIN(t3, P_ZAMBONI);
                zamboni();
                PROF_END(prof, P_ZAMBONI, t3);
            }
        }
        if (EV && evn > (int)evcap) fail(MT_DERR_EVENTS, S);  // halt rather than drop callbacks
    }

    // ------------------------------------------------------------ load / store
    // K consecutive u32 of one lane (16-byte aligned when K % 4 == 0, 8-byte when K is even)
    MT_DEV VU ld_u32(const MT_GLOB uint32_t* p) const {
        VU v;
        if constexpr (K % 2 == 1) {
#pragma unroll
            for (int j = 0; j < K; j++) v[j] = p[j];
        } else if constexpr (K % 4 == 0) {
#pragma unroll
            for (int c = 0; c < K / 4; c++) {
                const U4 x = reinterpret_cast<const MT_GLOB U4*>(p)[c];
                v[4 * c] = x[0];
                v[4 * c + 1] = x[1];
                v[4 * c + 2] = x[2];
                v[4 * c + 3] = x[3];
            }
        } else {
#pragma unroll
            for (int c = 0; c < K / 2; c++) {
                const U2 x = reinterpret_cast<const MT_GLOB U2*>(p)[c];
                v[2 * c] = x[0];
                v[2 * c + 1] = x[1];
            }
        }
        return v;
    }
    MT_DEV VU ld_u8(const uint8_t* p) const {  // K consecutive bytes of one lane
        VU v;
        if constexpr (K % 2 == 1) {
#pragma unroll
            for (int j = 0; j < K; j++) v[j] = p[j];
        } else if constexpr (K % 4 == 0) {
#pragma unroll
            for (int c = 0; c < K / 4; c++) {
                const uint32_t w = reinterpret_cast<const uint32_t*>(p)[c];
#pragma unroll
                for (int q = 0; q < 4; q++) v[4 * c + q] = (w >> (8 * q)) & 0xFFu;
            }
        } else {
#pragma unroll
            for (int c = 0; c < K / 2; c++) {
                const uint32_t w = reinterpret_cast<const uint16_t*>(p)[c];
                v[2 * c] = w & 0xFFu;
                v[2 * c + 1] = w >> 8;
            }
        }
        return v;
    }

    // ---- raw rows of the load: every global read of a launch is issued before any of it is used
    static constexpr int BW = (K % 2 == 1) ? K : (K % 4 == 0 ? K / 4 : K / 2);  // words per byte row
    MT_DEV void ld8_raw(const MT_GLOB uint8_t* p, uint32_t (&w)[BW]) const {  // K consecutive bytes of one lane
#pragma unroll
        for (int c = 0; c < BW; c++) {
            if constexpr (K % 2 == 1)
                w[c] = p[c];
            else if constexpr (K % 4 == 0)
                w[c] = reinterpret_cast<const MT_GLOB uint32_t*>(p)[c];
            else
                w[c] = reinterpret_cast<const MT_GLOB uint16_t*>(p)[c];
        }
    }
    MT_DEV static uint32_t byte_at(const uint32_t (&w)[BW], int j) {
        if constexpr (K % 2 == 1) return w[j] & 0xFFu;
        else if constexpr (K % 4 == 0) return (w[j / 4] >> (8 * (j % 4))) & 0xFFu;
        else return (w[j / 2] >> (8 * (j % 2))) & 0xFFu;
    }
    MT_DEV void ld64_raw(const MT_GLOB uint64_t* p, uint32_t (&w)[2 * K]) const {  // K consecutive u64: (lo, hi) pairs
        if constexpr (K % 2 == 1) {
#pragma unroll
            for (int j = 0; j < K; j++) {
                const U2 x = reinterpret_cast<const MT_GLOB U2*>(p)[j];
                w[2 * j] = x[0];
                w[2 * j + 1] = x[1];
            }
        } else {
#pragma unroll
            for (int c = 0; c < K / 2; c++) {
                const U4 x = reinterpret_cast<const MT_GLOB U4*>(p)[c];
                w[4 * c] = x[0];
                w[4 * c + 1] = x[1];
                w[4 * c + 2] = x[2];
                w[4 * c + 3] = x[3];
            }
        }
    }

    // The document's state into the wave: every global read is issued first (the per-segment rows
    // blocked by lane, K consecutive entries each, like the register state; the leaf-block, heap and
    // interior-level rows by chunks of 64) and waited for once, then the LDS images and the register
    // state are built from the registers.  (Before: a loop per array with a dependent load per
    // iteration, ~20 serialized memory round trips per launch.)
    MT_DEV void load(KGState& g, uint32_t d) {
        const MT_GLOB mt_doc_scalars& sc = gp(g.sc)[d];
        const int n = uni(sc.nseg);
        nlev = uni(sc.nlev);
        heap_n = uni(sc.heap_n);
        cur_seq = uni(sc.cur_seq);
        min_seq = uni(sc.min_seq);
        err = uni(sc.err);
        err_seq = uni(sc.err_seq);
        text_top = uniu(sc.text_top);
        text_half = uniu(sc.text_half);
        nb0 = uni(sc.nb[0]);
        next_id = n;
        nlive = n;
        ns = n;
        if constexpr (EV) {
            evp = gp(g.ev) + (size_t)d * g.evcap;
            evcap = g.evcap;
            evn = uni((int)gp(g.evn)[d]);
            evseq = cur_seq;
        }
        const size_t so = (size_t)d * g.segcap;
        const size_t lo = (size_t)d * g.lbcap;
        const size_t ho = (size_t)d * g.hcap;
        const int i0 = lane * K;
        const bool mine = i0 < n;
        // ---- 1. the reads, straight-line (no branch, so nothing is waited for before the last is
        // issued): rows are read whole (segcap >= CAP keeps them inside the document); a lane past
        // the document's n segments, and a chunk past its blocks or heap, re-reads the first one
        // (the same lines: no extra traffic) and its values are never used
        const int ir = mine ? i0 : 0;
        VU vsq, vrs, vln, vto;
        uint32_t pw[2 * K], ow[2 * K], bcw[BW], brw[BW], bfw[BW];
        vsq = ld_u32(reinterpret_cast<const MT_GLOB uint32_t*>(gp(g.seq) + so + ir));
        vrs = ld_u32(reinterpret_cast<const MT_GLOB uint32_t*>(gp(g.rseq) + so + ir));
        vln = ld_u32(gp(g.len) + so + ir);
        vto = ld_u32(gp(g.toff) + so + ir);
        ld64_raw(gp(g.props) + so + ir, pw);
        ld64_raw(gp(g.ovl) + so + ir, ow);
        ld8_raw(gp(g.client) + so + ir, bcw);
        ld8_raw(gp(g.rclient) + so + ir, brw);
        ld8_raw(gp(g.flags) + so + ir, bfw);
        constexpr int LBC = (L::LB + 63) / 64;  // leaf-block chunks (nb0 <= LB <= lbcap)
        uint32_t lbc_[LBC], lbs_[LBC];
#pragma unroll
        for (int c = 0; c < LBC; c++) {
            const size_t b = lo + (c * 64 < nb0 ? c * 64 + lane : 0);
            lbc_[c] = gp(g.lbcnt)[b];
            lbs_[c] = gp(g.lbscour)[b];
        }
        constexpr int HC = (L::H + 63) / 64;  // heap chunks (entries 1..heap_n, hcap >= H)
        int32_t hq[HC];
        uint32_t hs[HC];
#pragma unroll
        for (int c = 0; c < HC; c++) {
            const size_t i = ho + 1 + (c * 64 < heap_n ? c * 64 + lane : 0);
            hq[c] = gp(g.hseq)[i];
            hs[c] = gp(g.hslot)[i];  // position at store == id at load
        }
        constexpr int IBL = MT_MAXLEV - 1;  // interior levels, two chunks each (the rest: below)
        uint32_t ibw[IBL][2];
#pragma unroll
        for (int Lv = 1; Lv <= IBL; Lv++) {
            const size_t io = ((size_t)d * (MT_MAXLEV - 1) + (Lv < nlev ? Lv - 1 : 0)) * g.ibcap;
#pragma unroll
            for (int c = 0; c < 2; c++) ibw[Lv - 1][c] = gp(g.ibcnt)[io + c * 64 + lane];  // (ibcap >= 264)
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- 2. the LDS images: cold fields by segment id (= position at load; ids >= n get
        // garbage here and are written when allocated), leaf marks cleared, heap, interior levels
#pragma unroll
        for (int j = 0; j < K; j++) {
            s.props[i0 + j] = (uint64_t)pw[2 * j] | ((uint64_t)pw[2 * j + 1] << 32);
            s.toff[i0 + j] = (uint16_t)vto[j];
            s.scr[i0 + j] = 0;
        }
#pragma unroll
        for (int c = 0; c < HC; c++) {
            const int i = 1 + c * 64 + lane;
            if (c * 64 < heap_n && i <= heap_n) {
                s.hseq[i] = hq[c];
                s.hslot[i] = (uint16_t)hs[c];
            }
        }
#pragma unroll
        for (int Lv = 1; Lv <= IBL; Lv++) {
            if (Lv < nlev) {
                const int nbl_ = uni(sc.nb[Lv]);
#pragma unroll
                for (int c = 0; c < 2; c++)
                    if (c * 64 + lane < nbl_) s.ibcnt[Lv - 1][c * 64 + lane] = (uint8_t)ibw[Lv - 1][c];
                if (nbl_ > 128) {  // (documents far past the register classes' typical shape)
                    const size_t io = ((size_t)d * (MT_MAXLEV - 1) + (Lv - 1)) * g.ibcap;
#pragma clang loop unroll(disable) vectorize(disable)
                    for (int i = 128 + lane; i < nbl_; i += 64) s.ibcnt[Lv - 1][i] = gp(g.ibcnt)[io + i];
                }
            }
        }
        if (lane < MT_MAXLEV) s.nb[lane] = sc.nb[lane];
        wave_sync();
        // leaf blocks -> a mark (1 | needsScour << 1) at the first position of every non-empty block
        int nempty = 0;
        {
            int carry = 0;
#pragma unroll
            for (int cc = 0; cc < LBC; cc++) {
                if (cc * 64 < nb0) {
                    const int b = cc * 64 + lane;
                    const int c = b < nb0 ? (int)lbc_[cc] : 0;
                    const int scv = (int)lbs_[cc];
                    const int incl = wave_incl_scan(c) + carry;
                    if (b < nb0 && c > 0) s.scr[incl - c] = 1 | (scv << 1);
                    nempty += __popcll(wave_ballot(b < nb0 && c == 0));
                    carry = wave_last(incl);
                }
            }
        }
        wave_sync();
        // ---- 3. the register state (padding past n: dead, length 0, client 255)
        bsm = lvm = sc0 = sc1 = 0u;
#pragma unroll
        for (int j = 0; j < K; j++) {
            const bool in = i0 + j < n;
            const int mk = s.scr[i0 + j];  // scr[i] for i >= n is harmless (selected away)
            seq[j] = in ? (int32_t)vsq[j] : 0x7fffffff;
            rseq[j] = in ? (int32_t)vrs[j] : 0;
            li[j] = in ? (vln[j] | ((uint32_t)(i0 + j) << kLenBits)) : kEmptyLi;
            ov[j] = in ? ((ow[2 * j] >> 1) | (ow[2 * j + 1] << 31)) : 0u;
            if constexpr (W) oh[j] = in ? (ow[2 * j + 1] >> 1) : 0u;
            cf[j] = in ? (byte_at(bcw, j) | (byte_at(brw, j) << 8) | ((byte_at(bfw, j) & 0x1Fu) << 16)) : kEmptyCf;
            cum[j] = 0;
            const uint32_t bit = in ? (1u << j) : 0u;
            lvm |= bit;
            bsm |= (mk & 1) ? bit : 0u;
            sc0 |= (mk & 2) ? bit : 0u;
            sc1 |= (mk & 4) ? bit : 0u;
        }
        wave_sync();  // (tln shares scr's words: the marks are read)
#pragma unroll
        for (int j = 0; j < K; j++) s.tln[i0 + j] = vln[j];
        // empty leaf blocks (rare): a dead slot holds each one's place and marks
        if (nempty) {
            if (ns + nempty > CAP) {
                fail(MT_DERR_CAPACITY, cur_seq);
            } else {
                int carry = 0, placed = 0;
                for (int base = 0; base < nb0; base += 64) {
                    const int b = base + lane;
                    const int c = b < nb0 ? (int)gp(g.lbcnt)[lo + b] : 0;
                    const int scv = b < nb0 ? (int)gp(g.lbscour)[lo + b] : 0;
                    const int incl = wave_incl_scan(c) + carry;
                    uint64_t em = wave_ballot(b < nb0 && c == 0);
                    while (em) {
                        const int fl = first_lane(em);
                        em &= em - 1;
                        Elem ph;
                        ph.seq = 0x7fffffff;
                        ph.rseq = 0;
                        ph.li = kEmptyLi;
                        ph.cf = kEmptyCf;
                        ph.ov = 0;
                        ph.oh = 0;
                        ph.cum = 0;
                        shift_in<false>(__builtin_amdgcn_readlane(incl - c, fl) + placed, ph, true,
                                        __builtin_amdgcn_readlane(scv, fl), false);
                        placed++;
                    }
                    carry = wave_last(incl);
                }
            }
        }
    }

    // one register field -> HBM in position order, staged through LDS (scattered LDS writes,
    // coalesced HBM stores; no per-slot 64-bit addresses kept live)
    template <class T, class F>
    MT_DEV void store_field(const T& v, uint32_t lb, int pbase, int nn, F&& put) {
        // (a dead slot goes to the lane's discard word: no per-slot branch)
        int32_t* const dum = reinterpret_cast<int32_t*>(s.dum) + lane;
#pragma unroll
        for (int j = 0; j < K; j++)
            *(((lb >> j) & 1u) ? &s.scr[pbase + __popc(lb & ((1u << j) - 1u))] : dum) = (int32_t)v[j];
        wave_sync();
        // four rows per LDS round trip (scr holds CAP + 1 entries: the reads past nn are clamped)
#pragma clang loop unroll(disable) vectorize(disable)
        for (int base = 0; base < nn; base += 256) {
            uint32_t v[4];
#pragma unroll
            for (int q = 0; q < 4; q++) v[q] = (uint32_t)s.scr[min(base + 64 * q + lane, CAP)];
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (base + 64 * q + lane < nn) put(base + 64 * q + lane, v[q]);
        }
        wave_sync();
    }

    MT_DEV void store(KGState& g, uint32_t d) {
        const size_t so = (size_t)d * g.segcap;
        // live slots -> positions (dead slots are squeezed out here)
        const uint32_t lb = live_bits();
        const int c = __popc(lb);
        const int incl = wave_incl_scan(c);
        const int pbase = incl - c;
        const int nn = wave_last(incl);
        {  // pending ENDS_WITH_NEWLINE flags (F_NLQ) from the text
            uint32_t q = 0;
#pragma unroll
            for (int j = 0; j < K; j++) q |= ((cf[j] & F_NLQ) && ((lb >> j) & 1u)) ? (1u << j) : 0u;
            if (__ballot(q != 0)) {
                arena_sync();
                // every slot's offset, then every slot's byte: one LDS and one memory round trip
                uint32_t at[K];
#pragma unroll
                for (int j = 0; j < K; j++) {
                    const bool on = (q >> j) & 1u;
                    const uint32_t to = s.toff[on ? id_of(li[j]) : 0u];
                    at[j] = on ? to + len_of(li[j]) - 1 : 0u;
                }
                uint32_t ch[K];
#pragma unroll
                for (int j = 0; j < K; j++) ch[j] = arena()[at[j]];
#pragma unroll
                for (int j = 0; j < K; j++)
                    if ((q >> j) & 1u) cf[j] = (cf[j] & ~(F_NL | F_NLQ)) | (ch[j] == '\n' ? F_NL : 0u);
            }
        }
        store_field(seq, lb, pbase, nn, [&](int i, uint32_t v) { gp(g.seq)[so + i] = (int32_t)v; });
        store_field(rseq, lb, pbase, nn, [&](int i, uint32_t v) { gp(g.rseq)[so + i] = (int32_t)v; });
        store_field(ov, lb, pbase, nn, [&](int i, uint32_t v) { gp(g.ovl)[so + i] = (uint64_t)v << 1; });
        if constexpr (W)  // (after the low half: the same rows, read back and completed)
            store_field(oh, lb, pbase, nn, [&](int i, uint32_t v) { gp(g.ovl)[so + i] |= (uint64_t)v << 33; });
        store_field(cf, lb, pbase, nn, [&](int i, uint32_t v) {
            gp(g.client)[so + i] = (uint8_t)(v & 0xFFu);
            gp(g.rclient)[so + i] = (uint8_t)((v >> 8) & 0xFFu);
            gp(g.flags)[so + i] = (uint8_t)((v >> 16) & 0x1Fu);
        });
        store_field(li, lb, pbase, nn, [&](int i, uint32_t v) {
            const uint32_t id = id_of(v);
            gp(g.len)[so + i] = len_of(v);
            gp(g.toff)[so + i] = s.toff[id];
            gp(g.props)[so + i] = s.props[id];
        });
        // leaf blocks: live children and needsScour, in block order
        const uint32_t bm = bs_bits();
        const int bc = __popc(bm);
        const int bbase = wave_incl_scan(bc) - bc;
#pragma unroll
        for (int j = 0; j < K; j++) {
            if ((bm >> j) & 1u) {
                const int b = bbase + __popc(bm & ((1u << j) - 1u));
                s.scr[b] = pbase + __popc(lb & ((1u << j) - 1u));
                s.lbsc[b] = (uint8_t)(((sc0 >> j) & 1u) | (((sc1 >> j) & 1u) << 1));
            }
        }
        if (lane == 0) s.scr[nb0] = nn;
        wave_sync();
        const size_t lo = (size_t)d * g.lbcap;
        int nempty = 0;
#pragma clang loop unroll(disable) vectorize(disable)
        for (int b = lane; b < nb0; b += 64) {
            const int cnt = s.scr[b + 1] - s.scr[b];
            gp(g.lbcnt)[lo + b] = (uint8_t)cnt;
            gp(g.lbscour)[lo + b] = s.lbsc[b];
            nempty += cnt == 0 ? 1 : 0;
        }
        nempty = wave_total(nempty);
        // id -> position for the heap remap (toff is dead now)
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = lane; i < next_id; i += 64) s.toff[i] = kDead;
        wave_sync();
#pragma unroll
        for (int j = 0; j < K; j++)
            if ((lb >> j) & 1u) s.toff[id_of(li[j])] = (uint16_t)(pbase + __popc(lb & ((1u << j) - 1u)));
        wave_sync();
        for (int Lv = 1; Lv < nlev; Lv++) {
            const size_t io = ((size_t)d * (MT_MAXLEV - 1) + (Lv - 1)) * g.ibcap;
            const int nbl_ = min(nbl(Lv), (int)g.ibcap);
#pragma clang loop unroll(disable) vectorize(disable)
            for (int i = lane; i < nbl_; i += 64) gp(g.ibcnt)[io + i] = s.ibcnt[Lv - 1][i];
        }
        if (heap_n >= (int)g.hcap) fail(MT_DERR_CAPACITY, cur_seq);
        const size_t ho = (size_t)d * g.hcap;
        const int hn = min(heap_n, (int)g.hcap - 1);
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = 1 + lane; i <= hn; i += 64) {
            gp(g.hseq)[ho + i] = s.hseq[i];
            const uint16_t id = s.hslot[i];
            gp(g.hslot)[ho + i] = id == kDead ? kDead : s.toff[id];
        }
        if (lane == 0) {
            MT_GLOB mt_doc_scalars& sc = gp(g.sc)[d];
            sc.nseg = nn;
            sc.nlev = nlev;
            sc.heap_n = heap_n;
            sc.cur_seq = cur_seq;
            sc.min_seq = min_seq;
            sc.err = err;
            sc.err_seq = err_seq;
            sc.text_top = text_top;
            sc.text_half = text_half;
            sc.n_empty = (uint32_t)nempty;
            sc.nb[0] = nb0;
        }
        if (lane >= 1 && lane < MT_MAXLEV) gp(g.sc)[d].nb[lane] = s.nb[lane];
        if constexpr (EV)
            if (lane == 0) gp(g.evn)[d] = (uint32_t)evn;
    }
};

// Op records in blocks of 8 (256 B: lane l holds dword l % 8 of record base + l / 8), double-
// buffered: a record's fields are readlanes of a register loaded 1..15 ops earlier.  Both loads are
// unconditional (the record index and the payload byte are clamped into the batch), so no exec-masked
// branch hides their position from the compiler's vmcnt bookkeeping.
MT_DEV uint32_t load_op_block(const mt_op_rec* ops, uint32_t base, uint32_t end, int lane) {
    const uint32_t r = min(base + (uint32_t)(lane >> 3), end - 1u);  // (end > base's first record)
    return reinterpret_cast<const uint32_t*>(ops + r)[lane & 7];
}
// lane i <- payload byte i of a record (i < 64; lanes past the payload hold a copy of its last byte,
// never read); the payload buffer holds at least one byte
MT_DEV uint32_t load_payload(const uint8_t* payload, uint32_t poff, uint32_t plen, int lane) {
    return payload[plen ? poff + min((uint32_t)lane, plen - 1u) : 0u];
}
MT_DEV mt_op_rec op_from_block(uint32_t blk, uint32_t j) {
    const int l = (int)(j * 8);
    mt_op_rec r;
    r.seq = __builtin_amdgcn_readlane((int)blk, l + 0);
    r.ref_seq = __builtin_amdgcn_readlane((int)blk, l + 1);
    r.msn = __builtin_amdgcn_readlane((int)blk, l + 2);
    const uint32_t w3 = (uint32_t)__builtin_amdgcn_readlane((int)blk, l + 3);
    r.client = (uint16_t)(w3 & 0xFFFFu);
    r.type = (uint8_t)((w3 >> 16) & 0xFFu);
    r.flags = (uint8_t)(w3 >> 24);
    r.pos1 = __builtin_amdgcn_readlane((int)blk, l + 4);
    r.pos2 = __builtin_amdgcn_readlane((int)blk, l + 5);
    r.payload_off = (uint32_t)__builtin_amdgcn_readlane((int)blk, l + 6);
    r.payload_len = (uint32_t)__builtin_amdgcn_readlane((int)blk, l + 7);
    return r;
}

// The document arrays of mt_gstate are only needed by load() and store().  Both read them
// through a pointer to the kernel's own argument block that the compiler cannot see through, so
// the ~40 SGPRs of pointers are not held live across the op loop (where they were spilled into
// VGPR lanes and reloaded in the hot phases).  g is the kernel's first argument: offset 0.
MT_DEV KGState& kernarg_gstate() {
    KGState* p = (KGState*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}

// Waves per SIMD by class.  The register state is 6 K VGPRs per lane and the op path needs ~110
// more (text compaction reads no register state: compact_text).  The kernels are issue-latency
// bound, so a class takes the highest occupancy whose spill stays small.  Round 3 measured K = 4 at
// 5 waves, K = 6 and 7 at 4 and K = 10 at 3, each with a few bytes of scratch, faster than one wave
// fewer without it, while 200+ B of scratch (K = 8 at 4, K = 11 / 12 at 3) measured 1.2-2.6x slower
// (profiles/r03_ab_occupancy.log); the scratch each class keeps at HEAD is in
// profiles/r05_resource_usage_reg.txt (tools/resource_usage.py).  The small classes
// (documents up to ~125 segments, C5's) run at K = 2: 7 and K = 3: 6 waves, +3.3 % on C5 against 5 / 5
// and +2.5 % against 8 / 7 (profiles/r04_ab_small_occupancy*_C5.log).
// Round 5 re-picked three classes with the PMC traffic in the A/B (profiles/r05_ab_occupancy/): K = 7
// at 3 waves is spill-free (158 VGPRs; 176 B of scratch at 4) and faster (C3's 448 class 50.6 -> 43.9 ms,
// its traffic 13.3x -> 1.19x its algorithmic bytes); K = 2 at 6 and K = 3 at 5 waves keep 24 / 28 B of
// scratch instead of 60 / 104 B (C5 traffic 3.9x -> 2.6x and 12.0x -> 2.0x) for 1 % of C5's rate.
// Round 6 (after the one-pass shift cut the register peaks: K = 7 at four waves 64 B of scratch, K = 2
// at seven 24 B, K = 3 at six 40 B): K = 7 at four +0.8 % on C3, K = 2 / 3 at seven / six +2.8 % on C5;
// K = 8 / 9 at four (124 / 144 B) -3.2 % on C3 (profiles/r06_ab/ab4_*).  With the step loop unrolled:
// K = 11 at three (120 B) +2.9 % on C3 (its 704 class 54.2 -> 47.3 ms); K = 7 at three (spill-free)
// -3.3 % on C4 (profiles/r06_ab/ab6_*); K = 12 at three would take 356 B.  With the zamboni passes
// unrolled too: K = 8 at four (60 B) +0.6 % C3 (its 512 class 45.7 -> 44.0 ms), K = 12 at three (116 B)
// -1.1 % (profiles/r06_ab/ab8_*); K = 3 at seven (48 B) +1.8 % on C5, K = 2 at eight +0.9 % (both: +1.1 %),
// K = 2 / 3 at six / five (spill-free) -3.1 % (profiles/r06_ab/ab11_*); K = 5 at five (68 B) its C4 class
// 65.0 -> 60.9 ms, K = 4 at six neutral (profiles/r06_ab/ab12_*)
constexpr int wpe_default(int K) {
    return K <= 3 ? 7 : K <= 5 ? 5 : K <= 8 ? 4 : K <= 11 ? 3 : 2;
}
// MT_WPE_OV={w0,w1,...,w16} overrides classes one by one (0 = the default), for A/B builds.
#ifndef MT_WPE_OV
#define MT_WPE_OV {0}
#endif
constexpr int wpe_ov[17] = MT_WPE_OV;
constexpr int wpe(int K) { return K < 17 && wpe_ov[K] > 0 ? wpe_ov[K] : wpe_default(K); }
template <int K, bool W, bool EV>
MT_DEV void reg_apply(uint8_t* text, uint32_t textcap, const mt_op_rec* __restrict__ ops,
                      const uint8_t* __restrict__ payload, const uint32_t* __restrict__ row_ptr,
                      const uint32_t* __restrict__ doc_ids, uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t w = blockIdx.x;
    if (w >= n_docs) return;
    const uint32_t d = doc_ids ? doc_ids[w] : w;
    RLds<K>& lds = *reinterpret_cast<RLds<K>*>(smem);
    RWave<K, W, EV> wv(lds, text + (size_t)d * 2 * textcap, textcap);
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    const uint32_t a = min(r1, r0 + op_lo);
    const uint32_t b = op_cnt ? min(r1, a + op_cnt) : r1;
    if (a >= b) return;
    PROF_BEGIN(tl, P_LOAD);
    wv.load(kernarg_gstate(), d);
    PROF_END(wv.prof, P_LOAD, tl);
    // software pipeline: op i's payload was loaded at the end of op i-1's apply and op i+1's is
    // issued at the end of op i's, so every wait for a prefetch finds it a whole op old (a prefetch
    // issued at the top of the loop was waited for at once: the copy into the current-op register,
    // and any arena read of the op, drain vmcnt to 0).  (Round 6 tried both an explicit vmcnt(0) at
    // the end of each op and requesting op i+1's payload in the middle of op i, where its last
    // reader is done: neutral, and 0.90x -- the mid-op request raised K = 9's scratch from 24 to
    // 212 B; profiles/r06_ab/ab4_*.)
    uint32_t blk0 = load_op_block(ops, a, b, wv.lane);
    uint32_t blk1 = load_op_block(ops, a + 8, b, wv.lane);
    uint32_t pb = load_payload(payload, (uint32_t)__builtin_amdgcn_readlane((int)blk0, 6),
                               (uint32_t)__builtin_amdgcn_readlane((int)blk0, 7), wv.lane);
    uint32_t pbn = 0;
    if (a + 1 < b)
        pbn = load_payload(payload, (uint32_t)__builtin_amdgcn_readlane((int)blk0, 14),
                           (uint32_t)__builtin_amdgcn_readlane((int)blk0, 15), wv.lane);
    for (uint32_t i = a; i < b; i++) {
        if (wv.err) break;
        // op i's fields are taken from its block here (not carried over from the previous
        // iteration: ten fewer scalars live across the apply)
        const mt_op_rec op = op_from_block(blk0, (i - a) & 7u);
        wv.pb = pb;
        PROF_BEGIN(top, P_OP);
        wv.apply(op, payload);
        PROF_END(wv.prof, P_OP, top);
#ifdef MT_PROF
        wv.prof[P_OPS]++;
#endif
        pb = pbn;
        const uint32_t jn = (i + 1 - a) & 7u;  // op i+1's record in its block
        if (jn == 0) {
            blk0 = blk1;
            blk1 = load_op_block(ops, i + 9, b, wv.lane);
        }
        if (i + 2 < b) {  // op i+2's payload: in blk1 when it starts the next block
            const uint32_t j2 = (i + 2 - a) & 7u;
            uint32_t poff, plen;
            if (j2 == 0) {
                poff = (uint32_t)__builtin_amdgcn_readlane((int)blk1, 6);
                plen = (uint32_t)__builtin_amdgcn_readlane((int)blk1, 7);
            } else {
                poff = (uint32_t)__builtin_amdgcn_readlane((int)blk0, (int)(j2 * 8 + 6));
                plen = (uint32_t)__builtin_amdgcn_readlane((int)blk0, (int)(j2 * 8 + 7));
            }
            pbn = load_payload(payload, poff, plen, wv.lane);
        }
    }
    PROF_BEGIN(tt, P_STORE);
    wv.store(kernarg_gstate(), d);
    PROF_END(wv.prof, P_STORE, tt);
#ifdef MT_PROF
    if (wv.lane == 0)
        for (int q = 0; q < P_NSLOT; q++)
            atomicAdd(&mt_prof_acc[(K - 1) * kProfStride + q],
                      (unsigned long long)wv.prof[q]);
#endif
}

// the narrow register engine (client ids <= 32) and its C64 form (client ids <= 63: a second overlap
// register per slot, one occupancy step lower where the state no longer fits)
#ifndef MT_WPE_C64_OV
#define MT_WPE_C64_OV {0}
#endif
constexpr int wpe_c64_ov[17] = MT_WPE_C64_OV;
// The C64 form carries K more VGPRs of state; same rule (A/B on C3W in profiles/r03_ab_occupancy.log:
// K = 3..6 one wave up, K = 8, 9 at 3 with <= 100 B of scratch; K = 7 at 4 would spill ~200 B).
// K >= 13 runs one wave per SIMD: at two it spilled 590-660 B per lane in round 4's code, at one the
// excess lives in AGPRs (C3W 137.3 -> 184.5 M ops/s, profiles/r04_ab_c64_occupancy_C3W.log).  (The
// event kernels measured the other way: one wave at K >= 11 0.89x, r04_ab_events_onewave_C3.jsonl.)
// Round 6, after the unrolled op path cut the register peaks: K >= 13 at two waves takes 60 B, K = 10
// at three 60 B -- C3W 223.5 -> 258.7 M ops/s (profiles/r06_ab/ab13_side_occupancy/).
constexpr int wpe_c64_default(int K) { return K <= 4 ? 5 : K <= 6 ? 4 : K <= 10 ? 3 : 2; }
constexpr int wpe_c64(int K) { return K < 17 && wpe_c64_ov[K] > 0 ? wpe_c64_ov[K] : wpe_c64_default(K); }
template <int K>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(wpe(K)))) void reg_apply_kernel(
    mt_gstate g, const mt_op_rec* __restrict__ ops, const uint8_t* __restrict__ payload,
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ doc_ids, uint32_t n_docs, uint32_t op_lo,
    uint32_t op_cnt) {
    reg_apply<K, false, false>(g.text, g.textcap, ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt);
}
// ... and with delta / maintenance events recorded (mt_events_enable): the same engine, its event
// rows written from the split, insert, range and scour steps (the kernel without EV carries no event
// code; C64 documents record on the LDS engine)
// The event-recording kernels need ~35 VGPRs more (the event rows' placement and property deltas):
// at the plain kernels' occupancy they would spill 180-560 B per lane from K = 2 on, so they run one
// or two waves lower, spill-free up to K = 9 (K = 10 / 11: 100 / 180 B at two waves).
// MT_WPE_EV_OV overrides them like MT_WPE_OV.  Round 6 (the unrolled op path): K = 6..8 three waves
// spill-free, K = 9 / 10 / 11 at three 64 / 72 / 144 B -- C3 with events 231.7 -> 260.8 M ops/s (K <= 10),
// 258.7 -> 269.9 M (K = 11; K = 12 at three loses its class, 37.5 -> 42.7 ms)
// (profiles/r06_ab/ab13_side_occupancy/).
constexpr int wpe_ev_default(int K) { return K <= 2 ? 4 : K <= 11 ? 3 : 2; }
#ifndef MT_WPE_EV_OV
#define MT_WPE_EV_OV {0}
#endif
constexpr int wpe_ev_ov[17] = MT_WPE_EV_OV;
constexpr int wpe_ev(int K) { return K < 17 && wpe_ev_ov[K] > 0 ? wpe_ev_ov[K] : wpe_ev_default(K); }
template <int K>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(wpe_ev(K)))) void reg_apply_kernel_ev(
    mt_gstate g, const mt_op_rec* __restrict__ ops, const uint8_t* __restrict__ payload,
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ doc_ids, uint32_t n_docs, uint32_t op_lo,
    uint32_t op_cnt) {
    reg_apply<K, false, true>(g.text, g.textcap, ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt);
}
template <int K>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(wpe_c64(K)))) void reg_apply_kernel_c64(
    mt_gstate g, const mt_op_rec* __restrict__ ops, const uint8_t* __restrict__ payload,
    const uint32_t* __restrict__ row_ptr, const uint32_t* __restrict__ doc_ids, uint32_t n_docs, uint32_t op_lo,
    uint32_t op_cnt) {
    reg_apply<K, true, false>(g.text, g.textcap, ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt);
}

}  // namespace mtr

// form: 0 = the narrow register engine, 1 = its C64 form, 2 = the narrow form recording events
extern "C" hipError_t mt_launch_apply_reg(int cap_class, int form, const mt_gstate* g, const mt_op_rec* ops,
                                          const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                          uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    dim3 grid(n_docs), block(64);
#define MTR_LAUNCH(CAPV)                                                                                     \
    case CAPV: {                                                                                             \
        constexpr int K = CAPV / 64;                                                                         \
        if (form == 1)                                                                                       \
            hipLaunchKernelGGL((mtr::reg_apply_kernel_c64<K>), grid, block, sizeof(mtr::RLds<K>), stream, *g, \
                               ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt);                       \
        else if (form == 2)                                                                                  \
            hipLaunchKernelGGL((mtr::reg_apply_kernel_ev<K>), grid, block, sizeof(mtr::RLds<K>), stream, *g,  \
                               ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt);                       \
        else                                                                                                 \
            hipLaunchKernelGGL((mtr::reg_apply_kernel<K>), grid, block, sizeof(mtr::RLds<K>), stream, *g,     \
                               ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt);                       \
        return hipGetLastError();                                                                            \
    }
#ifdef MT_REG_ONLY_K  // (diagnostic builds: one class instantiated, for fast resource-usage / ISA looks)
    switch (cap_class) {
        MTR_LAUNCH(64 * MT_REG_ONLY_K)
        default:
            return hipErrorInvalidValue;
    }
#else
    switch (cap_class) {
        MTR_LAUNCH(128)
        MTR_LAUNCH(192)
        MTR_LAUNCH(256)
        MTR_LAUNCH(320)
        MTR_LAUNCH(384)
        MTR_LAUNCH(448)
        MTR_LAUNCH(512)
        MTR_LAUNCH(576)
        MTR_LAUNCH(640)
        MTR_LAUNCH(704)
        MTR_LAUNCH(768)
        MTR_LAUNCH(832)
        MTR_LAUNCH(896)
        MTR_LAUNCH(960)
        MTR_LAUNCH(1024)
        default:
            return hipErrorInvalidValue;
    }
#endif
#undef MTR_LAUNCH
}

// diagnostic: read (and clear) the per-phase cycle totals of a -DMT_PROF build (zeros otherwise)
extern "C" int mt_prof_read(unsigned long long* out, int n) {
#ifdef MT_PROF
    if (n > 16 * mtr::kProfStride) n = 16 * mtr::kProfStride;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mtr::mt_prof_acc), n * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    unsigned long long z[16 * mtr::kProfStride] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mtr::mt_prof_acc), z, sizeof z) != hipSuccess) return -1;
    return n;
#else
    for (int i = 0; i < n; i++) out[i] = 0;
    return 0;
#endif
}
