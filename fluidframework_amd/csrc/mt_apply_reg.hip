// mt_apply_reg.hip -- register-resident merge-tree apply engine for gfx950 (CDNA4).
//
// Same semantics as mt_apply.hip (the observer Client.applyMsg of the reference,
// client.ts:797-828, bit-exact) with a different placement of the document state:
//
//   * the hot per-segment fields live in VGPRs, BLOCKED by lane: segment i of the document is
//     register slot j = i % K of lane i / K (K = CAP / 64).  Visibility for an op's (refSeq,
//     client) view (mergeTree.ts:1667-1697) is then K independent per-lane evaluations plus ONE
//     wave-wide DPP scan -- the whole PartialSequenceLengths query (partialLengths.ts:433-487)
//     costs ~K VALU ops per lane and no LDS traffic;
//   * inserting a segment at document position p (a split, an insert) moves every later segment
//     one slot: K predicated moves per field per lane, with the lane-crossing element carried
//     by DPP wave_shr:1 (wave_shl:1 for an unlink);
//   * cold per-segment fields (property set, text offset) stay in LDS indexed by a segment id
//     that never changes while the segment is linked, so they never move; the B-tree shape
//     (leaf/interior child counts, needsScour), the zamboni heap and small scratch are in LDS
//     exactly as in mt_apply.hip.
// Register budget sets the capacity classes: K = 2, 4, 8, 16 (128..1024 segments).  Documents
// beyond 1024 segments run on mt_apply.hip's LDS engine (CAP 2048).  HBM layout (mt_state.h)
// is shared by both engines, so documents move freely between classes from launch to launch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtgpu.h"
#include "mt_state.h"
#include "mt_wave.h"

namespace mtr {

constexpr int kMaxNodes = 8;           // MaxNodesInBlock, mergeTree.ts:334
constexpr int kTextGranularity = 256;  // MergeTree.TextSegmentGranularity, mergeTree.ts:1059
constexpr uint32_t kLenBits = 17;      // li = len | id << 17  (len <= textcap <= 65536)
constexpr uint32_t kLenMask = (1u << kLenBits) - 1;
constexpr uint32_t kNoId = 0x7FFFu;    // id of an unused register slot
constexpr uint32_t kEmptyLi = kNoId << kLenBits;
constexpr uint32_t kEmptyCf = 0xFFu;   // client 255: never an op's client, len 0 -> invisible
constexpr uint32_t F_RM = (uint32_t)MT_SF_REMOVED << 16;
constexpr uint32_t F_PDEF = (uint32_t)MT_SF_PDEF << 16;
constexpr uint32_t F_NL = (uint32_t)MT_SF_NL << 16;
constexpr uint16_t kDead = 0xFFFFu;

MT_DEV int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
MT_DEV uint32_t uniu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// lane l <- lane l-1 (lane 0 <- fill)
MT_DEV int shr1(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false); }
// lane l <- lane l+1 (lane 63 <- fill)
MT_DEV int shl1(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, 0x130, 0xf, 0xf, false); }

// ---- optional per-phase cycle accounting (diagnostic build: -DMT_PROF; never in the product)
#ifdef MT_PROF
__device__ unsigned long long mt_prof_acc[96];  // [class 0..3][24 slots]
MT_DEV uint64_t prof_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PROF_BEGIN(v) const uint64_t v = prof_now()
#define PROF_END(arr, slot, v) arr[slot] += prof_now() - (v)
#else
#define PROF_BEGIN(v)
#define PROF_END(arr, slot, v)
#endif
enum { P_LOAD, P_SCAN, P_BOUND, P_INSERT, P_RANGE, P_ZAMBONI, P_SCOUR, P_STORE, P_OPS, P_ZPOP, P_REPACK,
       P_B_GET, P_B_BLK, P_B_TXT, P_B_INS, P_N_SCOUR, P_N_UNLINK, P_N_APPEND, P_N_SPLIT, P_NSLOT };
#ifdef MT_PROF
#define PROF_CNT(slot, v) prof[slot] += (v)
#else
#define PROF_CNT(slot, v)
#endif

template <int K>
struct RLds {
    static constexpr int CAP = 64 * K;
    static constexpr int LB = CAP / 2;      // leaf blocks        (same class limits as mt::Lds)
    static constexpr int IB = CAP / 8 + 8;  // blocks per interior level
    static constexpr int H = CAP / 2 + 64;  // heap entries (1-based)
    uint64_t props[CAP];    // by segment id: 8 keys x u8 value id
    int32_t pcum[CAP];      // by position: spilled inclusive visible prefix (scratch)
    int32_t bst[LB + 1];    // scratch: leaf-block start positions
    int32_t hseq[H];
    uint16_t toff[CAP];     // by segment id: text view offset (at store: id -> position)
    uint16_t pid[CAP];      // by position: spilled segment ids (scratch)
    uint16_t hslot[H];      // heap entry -> segment id (kDead once unlinked)
    uint8_t lbcnt[LB];
    uint8_t lbscour[LB];
    uint8_t ibcnt[MT_MAXLEV - 1][IB];
    int32_t nb[MT_MAXLEV];
    int32_t zseq[kMaxNodes + 1], zrseq[kMaxNodes + 1];   // scour scratch: one leaf block
    uint32_t zli[kMaxNodes + 1], zcf[kMaxNodes + 1];
};

struct Elem {
    int32_t seq, rseq;
    uint32_t li, cf, o0, o1;
    int32_t cum;
};

template <int K>
struct RWave {
    using L = RLds<K>;
    static constexpr int CAP = L::CAP;
    L& s;
    const int lane;
    uint8_t* const abase;
    uint8_t* arena;
    const uint32_t textcap;

    // ---- document state in registers (blocked: element i = lane * K + j)
    // (clang ext vectors: SSA values end to end, never a private-memory array)
    typedef int32_t VI __attribute__((ext_vector_type(K)));
    typedef uint32_t VU __attribute__((ext_vector_type(K)));
    VI seq, rseq;
    VU li, cf, o0, o1;
    VI cum;   // per-op scratch: inclusive visible prefix for the op's view
    // ---- uniform document scalars
    int n, nlev, heap_n, cur_seq, min_seq, err, err_seq, next_id;
    uint32_t text_top, text_half;
#ifdef MT_PROF
    uint64_t prof[P_NSLOT] = {};
#endif

    MT_DEV RWave(L& lds, uint8_t* a, uint32_t tc) : s(lds), lane(lane_id()), abase(a), arena(a), textcap(tc) {}

    MT_DEV int idx(int j) const { return lane * K + j; }

    MT_DEV void fail(int code, int32_t sq) {
        if (err == 0) {
            err = code;
            err_seq = sq;
        }
    }

    // ------------------------------------------------------------ element access
    MT_DEV static uint32_t len_of(uint32_t l) { return l & kLenMask; }
    MT_DEV static uint32_t id_of(uint32_t l) { return l >> kLenBits; }

    // all fields of the element at uniform position k
    MT_DEV Elem get(int k) const {
        const int lk = k / K, jk = k % K;
        int32_t a = seq[0], b = rseq[0], g = cum[0];
        uint32_t c = li[0], d = cf[0], e = o0[0], f = o1[0];
#pragma unroll
        for (int j = 1; j < K; j++) {
            if (jk == j) {
                a = seq[j];
                b = rseq[j];
                c = li[j];
                d = cf[j];
                e = o0[j];
                f = o1[j];
                g = cum[j];
            }
        }
        Elem r;
        r.seq = __builtin_amdgcn_readlane(a, lk);
        r.rseq = __builtin_amdgcn_readlane(b, lk);
        r.li = (uint32_t)__builtin_amdgcn_readlane((int)c, lk);
        r.cf = (uint32_t)__builtin_amdgcn_readlane((int)d, lk);
        r.o0 = (uint32_t)__builtin_amdgcn_readlane((int)e, lk);
        r.o1 = (uint32_t)__builtin_amdgcn_readlane((int)f, lk);
        r.cum = __builtin_amdgcn_readlane(g, lk);
        return r;
    }
    MT_DEV uint32_t get_li(int k) const {
        const int lk = k / K, jk = k % K;
        uint32_t c = li[0];
#pragma unroll
        for (int j = 1; j < K; j++)
            if (jk == j) c = li[j];
        return (uint32_t)__builtin_amdgcn_readlane((int)c, lk);
    }
    // overwrite li / cf / cum of the element at uniform position k
    MT_DEV void set_li_cf(int k, uint32_t lv, uint32_t cv) {
        const int lk = k / K, jk = k % K;
#pragma unroll
        for (int j = 0; j < K; j++) {
            if (jk == j && lane == lk) {
                li[j] = lv;
                cf[j] = cv;
            }
        }
    }
    MT_DEV void set_cum(int k, int32_t v) {
        const int lk = k / K, jk = k % K;
#pragma unroll
        for (int j = 0; j < K; j++)
            if (jk == j && lane == lk) cum[j] = v;
    }

    // insert element e at position p: positions >= p move one slot right
    template <bool CUM>
    MT_DEV void shift_in(int p, const Elem& e) {
        const int32_t c_seq = shr1(seq[K - 1], 0), c_rseq = shr1(rseq[K - 1], 0);
        const uint32_t c_li = (uint32_t)shr1((int)li[K - 1], 0), c_cf = (uint32_t)shr1((int)cf[K - 1], 0);
        const uint32_t c_o0 = (uint32_t)shr1((int)o0[K - 1], 0), c_o1 = (uint32_t)shr1((int)o1[K - 1], 0);
        const int32_t c_cum = CUM ? shr1(cum[K - 1], 0) : 0;
#pragma unroll
        for (int j = K - 1; j >= 0; j--) {
            const int i = idx(j);
            const bool mv = i > p, at = i == p;
            const int32_t pseq = j ? seq[j - 1] : c_seq, prseq = j ? rseq[j - 1] : c_rseq;
            const uint32_t pli = j ? li[j - 1] : c_li, pcf = j ? cf[j - 1] : c_cf;
            const uint32_t po0 = j ? o0[j - 1] : c_o0, po1 = j ? o1[j - 1] : c_o1;
            seq[j] = mv ? pseq : (at ? e.seq : seq[j]);
            rseq[j] = mv ? prseq : (at ? e.rseq : rseq[j]);
            li[j] = mv ? pli : (at ? e.li : li[j]);
            cf[j] = mv ? pcf : (at ? e.cf : cf[j]);
            o0[j] = mv ? po0 : (at ? e.o0 : o0[j]);
            o1[j] = mv ? po1 : (at ? e.o1 : o1[j]);
            if (CUM) {
                const int32_t pcm = j ? cum[j - 1] : c_cum;
                cum[j] = mv ? pcm : (at ? e.cum : cum[j]);
            }
        }
        n = n + 1;
    }

    // remove the element at position p: positions > p move one slot left
    MT_DEV void shift_out(int p) {
        const int32_t c_seq = shl1(seq[0], 0x7fffffff), c_rseq = shl1(rseq[0], 0);
        const uint32_t c_li = (uint32_t)shl1((int)li[0], (int)kEmptyLi), c_cf = (uint32_t)shl1((int)cf[0], (int)kEmptyCf);
        const uint32_t c_o0 = (uint32_t)shl1((int)o0[0], 0), c_o1 = (uint32_t)shl1((int)o1[0], 0);
#pragma unroll
        for (int j = 0; j < K; j++) {
            const bool mv = idx(j) >= p;
            const bool last = j == K - 1;
            seq[j] = mv ? (last ? c_seq : seq[j + (last ? 0 : 1)]) : seq[j];
            rseq[j] = mv ? (last ? c_rseq : rseq[j + (last ? 0 : 1)]) : rseq[j];
            li[j] = mv ? (last ? c_li : li[j + (last ? 0 : 1)]) : li[j];
            cf[j] = mv ? (last ? c_cf : cf[j + (last ? 0 : 1)]) : cf[j];
            o0[j] = mv ? (last ? c_o0 : o0[j + (last ? 0 : 1)]) : o0[j];
            o1[j] = mv ? (last ? c_o1 : o1[j + (last ? 0 : 1)]) : o1[j];
        }
        n = n - 1;
    }

    // ------------------------------------------------------------ visibility
    // nodeLength leaf branch for a remote client (mergeTree.ts:1667-1697)
    MT_DEV int vis(int j, int32_t R, int C) const {
        const uint32_t f = cf[j];
        const bool seen = ((int)(f & 0xFFu) == C) || (seq[j] <= R);
        const uint32_t ob = C < 32 ? (o0[j] >> (C & 31)) : (o1[j] >> (C & 31));
        const bool hid = (f & F_RM) && ((int)((f >> 8) & 0xFFu) == C || (ob & 1u) || rseq[j] <= R);
        return (seen && !hid) ? (int)len_of(li[j]) : 0;
    }

    // cum[] = inclusive prefix of vis over document order; returns getLength(R, C)
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
    // visible start of this lane's first element
    MT_DEV int cs0() const { return shr1(cum[K - 1], 0); }

    // spill cum (and ids) to LDS by position for the block-level logic
    MT_DEV void spill(bool ids) {
#pragma unroll
        for (int j = 0; j < K; j++) s.pcum[idx(j)] = cum[j];
        if (ids) {
#pragma unroll
            for (int j = 0; j < K; j++) s.pid[idx(j)] = (uint16_t)id_of(li[j]);
        }
        wave_sync();
    }
    MT_DEV int pcstart(int k) const { return k > 0 ? s.pcum[k - 1] : 0; }

    // ----------------------------------------------------------------- blocks
    MT_DEV uint8_t* lvl(int Lv) { return Lv == 0 ? s.lbcnt : s.ibcnt[Lv - 1]; }
    MT_DEV int lvlcap(int Lv) const { return Lv == 0 ? L::LB : L::IB; }
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

    // bst[b] = first position of leaf block b (bst[nb0] = n)
    MT_DEV void block_starts() {
        const int nb = nbl(0);
        int carry = 0;
        for (int base = 0; base < nb; base += 64) {
            const int b = base + lane;
            const int c = b < nb ? (int)s.lbcnt[b] : 0;
            const int incl = wave_incl_scan(c) + carry;
            if (b < nb) s.bst[b] = incl - c;
            carry = wave_last(incl);
        }
        if (lane == 0) s.bst[nb] = carry;
        wave_sync();
    }
    // leaf block holding position k (the first block whose end is past k); needs bst
    MT_DEV int block_of_pos(int k) {
        const int nb = nbl(0);
        for (int base = 0; base < nb; base += 64) {
            const int b = base + lane;
            const bool hit = b < nb && s.bst[b] <= k && k < s.bst[b] + (int)s.lbcnt[b];
            const uint64_t m = wave_ballot(hit);
            if (m) return base + first_lane(m);
        }
        return -1;
    }
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
                if (first_child) *first_child = wave_bcast(incl - c, fl);
                return base + fl;
            }
            carry = wave_last(incl);
        }
        return -1;
    }
    MT_DEV bool insert_block_after(int Lv, int b, int cnt) {
        const int nb = nbl(Lv);
        if (nb + 1 > lvlcap(Lv)) return false;
        uint8_t* a = lvl(Lv);
        lshift_right(a, b + 1, nb);
        if (Lv == 0) lshift_right(s.lbscour, b + 1, nb);
        if (lane == 0) {
            a[b + 1] = (uint8_t)cnt;
            if (Lv == 0) s.lbscour[b + 1] = MT_SC_UNDEF;
            s.nb[Lv] = nb + 1;
        }
        wave_sync();
        return true;
    }
    // split 4/4 upward + new root (mergeTree.ts:2446-2489, 1876-1887)
    MT_DEV bool split_up(int Lv, int b, int32_t sq) {
        for (;;) {
            const int half = kMaxNodes / 2;
            int parent = -1;
            if (Lv < nlev - 1) parent = parent_of(Lv, b, nullptr);
            if (lane == 0) lvl(Lv)[b] = (uint8_t)half;
            wave_sync();
            if (!insert_block_after(Lv, b, half)) return fail(MT_DERR_CAPACITY, sq), false;
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

    // insert element e at position k of leaf block b (blockInsert/insertChildNode)
    template <bool CUM>
    MT_DEV bool insert_at(int k, int b, const Elem& e, int32_t sq) {
        if (n + 1 > CAP) return fail(MT_DERR_CAPACITY, sq), false;
        shift_in<CUM>(k, e);
        const int c = uni(s.lbcnt[b]) + 1;
        if (lane == 0) s.lbcnt[b] = (uint8_t)c;
        wave_sync();
        if (c >= kMaxNodes) return split_up(0, b, sq);
        return true;
    }
    MT_DEV int alloc_id(int32_t sq) {
        if (next_id >= CAP) {
            fail(MT_DERR_CAPACITY, sq);
            return -1;
        }
        return next_id++;
    }

    // ------------------------------------------------------------------- text
    MT_DEV void arena_copy(uint32_t dst, uint32_t src, uint32_t cnt) {
        for (uint32_t base = 0; base < cnt; base += 64) {
            const uint32_t i = base + lane;
            uint8_t v = 0;
            if (i < cnt) v = arena[src + i];
            __threadfence_block();
            if (i < cnt) arena[dst + i] = v;
        }
        __threadfence_block();
    }
    // relocate every linked segment's text, in document order, into the other arena half.
    // (len, id) go through the pcum/pid scratch so the copy loop is not unrolled K times;
    // callers never need pcum/pid after a reserve.
    MT_DEV void compact_text() {
#pragma unroll
        for (int j = 0; j < K; j++) {
            s.pcum[idx(j)] = (int32_t)len_of(li[j]);
            s.pid[idx(j)] = (uint16_t)id_of(li[j]);
        }
        wave_sync();
        uint8_t* dst = abase + (size_t)(text_half ^ 1u) * textcap;
        uint32_t carry = 0;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            const uint32_t l = i < n ? (uint32_t)s.pcum[i] : 0u;
            const uint32_t incl = (uint32_t)wave_incl_scan((int)l);
            const uint32_t at = carry + incl - l;
            if (l) {
                const uint32_t id = s.pid[i];
                const uint8_t* src = arena + s.toff[id];
                for (uint32_t q = 0; q < l; q++) dst[at + q] = src[q];
                s.toff[id] = (uint16_t)at;
            }
            carry += (uint32_t)wave_last((int)incl);
        }
        __threadfence_block();
        wave_sync();
        text_half ^= 1u;
        text_top = carry;
        arena = dst;
    }
    MT_DEV bool arena_reserve(uint32_t need, int32_t sq) {
        if (text_top + need <= textcap) return true;
        compact_text();
        if (text_top + need <= textcap) return true;
        fail(MT_DERR_TEXT_ARENA, sq);
        return false;
    }

    // ensureIntervalBoundary(pos) (mergeTree.ts:2241-2245): split the segment visible to the
    // op's view that strictly contains pos; keeps cum valid for that view.
    MT_DEV bool boundary(int pos, int32_t sq) {
        int cs = cs0();
        int hitj = -1;
#pragma unroll
        for (int j = 0; j < K; j++) {
            if (cs < pos && pos < cum[j]) hitj = j;
            cs = cum[j];
        }
        const uint64_t m = wave_ballot(hitj >= 0);
        if (!m) return true;
        PROF_CNT(P_N_SPLIT, 1);
        PROF_BEGIN(tb0);
        const int lk = first_lane(m);
        const int k = lk * K + __builtin_amdgcn_readlane(hitj, lk);
        const Elem e = get(k);
        PROF_END(prof, P_B_GET, tb0);
        const uint32_t len = len_of(e.li);
        const int off = pos - (e.cum - (int)len);
        const int t = alloc_id(sq);
        if (t < 0) return false;
        PROF_BEGIN(tb1);
        block_starts();
        const int b = block_of_pos(k);
        PROF_END(prof, P_B_BLK, tb1);
        PROF_BEGIN(tb2);
        // BaseSegment.splitAt + TextSegment.createSplitSegmentAt (mergeTree.ts:524-568)
        const uint32_t id = id_of(e.li);
        const uint32_t to = uniu(s.toff[id]);
        const uint8_t last = arena[to + (uint32_t)off - 1];
        if (lane == 0) {
            s.props[t] = s.props[id];
            s.toff[t] = (uint16_t)(to + (uint32_t)off);
        }
        Elem r = e;
        r.li = (len - (uint32_t)off) | ((uint32_t)t << kLenBits);
        set_li_cf(k, (uint32_t)off | (id << kLenBits), (e.cf & ~F_NL) | (last == '\n' ? F_NL : 0u));
        set_cum(k, pos);
        wave_sync();
        PROF_END(prof, P_B_TXT, tb2);
        PROF_BEGIN(tb3);
        const bool ok = insert_at<true>(k + 1, b, r, sq);
        PROF_END(prof, P_B_INS, tb3);
        return ok;
    }

    // ------------------------------------------------------------------- heap
    // Heap<LRUSegment> (collections.ts:213-265), comparer maxSeq (mergeTree.ts:923-926)
    MT_DEV bool heap_push(int32_t key, int id, int32_t sq) {
        if (heap_n + 1 >= L::H) return fail(MT_DERR_CAPACITY, sq), false;
        if (lane == 0) {
            int k = heap_n + 1;
            s.hseq[k] = key;
            s.hslot[k] = (uint16_t)id;
            while (k > 1 && s.hseq[k >> 1] - s.hseq[k] > 0) {
                const int32_t ts = s.hseq[k >> 1];
                const uint16_t tl = s.hslot[k >> 1];
                s.hseq[k >> 1] = s.hseq[k];
                s.hslot[k >> 1] = s.hslot[k];
                s.hseq[k] = ts;
                s.hslot[k] = tl;
                k >>= 1;
            }
        }
        heap_n = heap_n + 1;
        wave_sync();
        return true;
    }
    MT_DEV int heap_pop() {
        int id = 0;
        if (lane == 0) {
            id = s.hslot[1];
            const int cnt = heap_n - 1;
            s.hseq[1] = s.hseq[heap_n];
            s.hslot[1] = s.hslot[heap_n];
            int k = 1;
            while ((k << 1) <= cnt) {
                int j = k << 1;
                if (j < cnt && s.hseq[j] - s.hseq[j + 1] > 0) j++;
                if (s.hseq[k] - s.hseq[j] <= 0) break;
                const int32_t ts = s.hseq[k];
                const uint16_t tl = s.hslot[k];
                s.hseq[k] = s.hseq[j];
                s.hslot[k] = s.hslot[j];
                s.hseq[j] = ts;
                s.hslot[j] = tl;
                k = j;
            }
        }
        id = __builtin_amdgcn_readlane(id, 0);
        heap_n = heap_n - 1;
        wave_sync();
        return id;
    }
    // addToLRUSet (mergeTree.ts:1273-1283) for segment `id` in leaf block b
    MT_DEV bool add_lru(int b, int id, int32_t sq) {
        if (uni(s.lbscour[b]) != MT_SC_TRUE && sq > cur_seq) {
            if (lane == 0) s.lbscour[b] = MT_SC_TRUE;
            wave_sync();
            return heap_push(sq, id, sq);
        }
        return true;
    }

    // ---------------------------------------------------------------- zamboni
    MT_DEV int pos_of_id(int id) const {
        int hit = -1;
#pragma unroll
        for (int j = 0; j < K; j++)
            if ((int)id_of(li[j]) == id) hit = idx(j);
        const uint64_t m = wave_ballot(hit >= 0);
        if (!m) return -1;
        return __builtin_amdgcn_readlane(hit, first_lane(m));
    }

    // TextSegment.append (textSegment.ts:76-85): prev.text += seg.text.  prev/q index the
    // scour scratch (block positions st + prev / st + q).
    MT_DEV void append_text(int st, int prev, int q) {
        const uint32_t pid_ = id_of(uniu(s.zli[prev])), qid = id_of(uniu(s.zli[q]));
        const uint32_t pl = len_of(uniu(s.zli[prev])), ql = len_of(uniu(s.zli[q]));
        {
            const uint32_t pt = uniu(s.toff[pid_]), qt = uniu(s.toff[qid]);
            uint32_t need = 0;
            if (pt + pl != qt && pt + pl != text_top) need = pl + ql;
            else if (pt + pl != qt) need = ql;
            if (need && !arena_reserve(need, cur_seq)) return;
        }
        const uint32_t pt = uniu(s.toff[pid_]), qt = uniu(s.toff[qid]);
        uint32_t top = text_top;
        if (pt + pl == qt) {
            // adjacent views: nothing to copy
        } else if (pt + pl == top) {
            arena_copy(top, qt, ql);
            top += ql;
        } else {
            arena_copy(top, pt, pl);
            arena_copy(top + pl, qt, ql);
            if (lane == 0) s.toff[pid_] = (uint16_t)top;
            top += pl + ql;
        }
        const uint32_t nli = (pl + ql) | (pid_ << kLenBits);
        const uint32_t ncf = (uniu(s.zcf[prev]) & ~F_NL) | (uniu(s.zcf[q]) & F_NL);
        wave_sync();
        if (lane == 0) {
            s.zli[prev] = nli;
            s.zcf[prev] = ncf;
        }
        set_li_cf(st + prev, nli, ncf);  // registers stay current (a compaction may follow)
        text_top = top;
        wave_sync();
    }

    // scourNode on leaf block b (mergeTree.ts:1289-1365); returns the new child count
    MT_DEV int scour(int b) {
        const int st = uni(s.bst[b]);
        const int cnt = uni(s.lbcnt[b]);
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int i = idx(j);
            if (i >= st && i < st + cnt) {
                const int q = i - st;
                s.zseq[q] = seq[j];
                s.zrseq[q] = rseq[j];
                s.zli[q] = li[j];
                s.zcf[q] = cf[j];
            }
        }
        wave_sync();
        const int32_t minSeq = min_seq;
        int kept = 0, prev = -1;
        uint32_t unlink = 0;
        for (int q = 0; q < cnt; q++) {
            const uint32_t f = uniu(s.zcf[q]);
            if (f & F_RM) {
                if (uni(s.zrseq[q]) > minSeq) kept++;
                else unlink |= 1u << q;  // UNLINK
                prev = -1;
            } else if (uni(s.zseq[q]) <= minSeq) {
                bool app = false;
                const uint32_t ql = len_of(uniu(s.zli[q]));
                if (prev >= 0) {
                    const uint32_t pf = uniu(s.zcf[prev]);
                    const uint32_t pl = len_of(uniu(s.zli[prev]));
                    const bool pm = ((pf ^ f) & F_PDEF) == 0 &&
                                    s.props[id_of(uniu(s.zli[prev]))] == s.props[id_of(uniu(s.zli[q]))];
                    // canAppend + matchProperties (textSegment.ts:63-68, properties.ts:62-93)
                    app = !(pf & F_NL) && (pl <= (uint32_t)kTextGranularity || ql <= (uint32_t)kTextGranularity) &&
                          pm && ql > 0;
                }
                if (uni(app ? 1 : 0)) {
                    append_text(st, prev, q);
                    PROF_CNT(P_N_APPEND, 1);
                    if (err) return cnt;
                    unlink |= 1u << q;  // APPEND: segment.parent = undefined
                } else {
                    kept++;
                    prev = ql > 0 ? q : -1;
                }
            } else {
                kept++;
                prev = -1;
            }
        }
        if (kept < cnt) {
            for (int q = cnt - 1; q >= 0; q--)
                if (unlink & (1u << q)) shift_out(st + q);
            PROF_CNT(P_N_UNLINK, __popc(unlink));
            const int d = cnt - kept;
            if (lane == 0) s.lbcnt[b] = (uint8_t)kept;
            const int nb = nbl(0);
            for (int base = b + 1; base <= nb; base += 64) {
                const int jb = base + lane;
                if (jb <= nb) s.bst[jb] -= d;
            }
            wave_sync();
        }
        return kept;
    }

    // The block-count half of pack (mergeTree.ts:1368-1420): the m children of block P at
    // level Lv+1 (first child first_child, `total` grandchildren after scouring) are repacked
    // evenly, recursing upward on underflow.
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
                if (Lv == 0) lshift_left(s.lbscour, first_child + m, nb, m - cc);
            } else if (cc > m) {
                for (int q = 0; q < cc - m; q++) {
                    lshift_right(a, first_child + m, nb + q);
                    if (Lv == 0) lshift_right(s.lbscour, first_child + m, nb + q);
                }
            }
            if (lane < cc) {
                a[first_child + lane] = (uint8_t)(base + (lane < extra ? 1 : 0));
                if (Lv == 0) s.lbscour[first_child + lane] = MT_SC_UNDEF;
            }
            wave_sync();
            if (lane == 0) {
                s.nb[Lv] = nb + cc - m;
                lvl(Lv + 1)[P] = (uint8_t)cc;
            }
            wave_sync();
            if (Lv == 0) block_starts();
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

    // zamboniSegments (mergeTree.ts:1422-1478), zamboniSegmentsMaxCount = 2.  One scour call
    // site: step 0 scours the popped segment's block; on underflow steps 1..m scour every
    // sibling under its parent (pack's scourNode loop), then repack.
    MT_DEV void zamboni() {
        for (int it = 0; it < 2; it++) {
            if (heap_n == 0 || uni(s.hseq[1]) > min_seq) break;
            PROF_BEGIN(tz);
            const int id = heap_pop();
            if (id == (int)kDead) continue;
            const int k = pos_of_id(id);
            if (k < 0) continue;  // segment.parent === undefined
            block_starts();
            const int b = block_of_pos(k);
            PROF_END(prof, P_ZPOP, tz);
            if (uni(s.lbscour[b]) == MT_SC_FALSE) continue;
            const int cnt = uni(s.lbcnt[b]);
            int P = -1, fc = 0, m = 0, total = 0;
            for (int step = 0;; step++) {
                const int blk = step == 0 ? b : fc + step - 1;
                PROF_BEGIN(ts);
                PROF_CNT(P_N_SCOUR, 1);
                const int kept = scour(blk);
                PROF_END(prof, P_SCOUR, ts);
                if (err) return;
                if (step == 0) {
                    if (lane == 0) s.lbscour[b] = MT_SC_FALSE;
                    wave_sync();
                    if (!(kept < cnt && kept < kMaxNodes / 2 && nlev > 1)) break;
                    P = parent_of(0, b, &fc);
                    m = uni(s.ibcnt[0][P]);
                } else {
                    total += kept;
                }
                if (step == m) break;
            }
            PROF_BEGIN(tr);
            if (P >= 0) repack(0, P, fc, m, total);
            PROF_END(prof, P_REPACK, tr);
            if (err) return;
        }
    }

    // -------------------------------------------------------------------- ops
    static MT_DEV uint64_t apply_pairs(uint64_t p, const uint8_t* pairs, int np) {
        for (int q = 0; q < np; q++) {
            const int k = pairs[2 * q];
            const uint64_t v = pairs[2 * q + 1];
            p = (p & ~(0xFFull << (8 * k))) | (v << (8 * k));
        }
        return p;
    }

    // blockInsert (mergeTree.ts:2141-2224) of a text segment at pos, after the boundary split
    MT_DEV void place_insert(const mt_op_rec& op, const uint8_t* pay, int tlen, const uint8_t* pairs, int np) {
        const int32_t S = op.seq, R = op.ref_seq;
        const int C = op.client, pos = op.pos1;
        spill(false);
        block_starts();
        const int nb = nbl(0);
        // first leaf block whose cumulative visible end >= pos (insertingWalk descent)
        int b = -1;
        for (int base = 0; base < nb; base += 64) {
            const int jb = base + lane;
            bool hit = false;
            if (jb < nb) {
                const int st = s.bst[jb], c = s.lbcnt[jb];
                const int bend = c > 0 ? s.pcum[st + c - 1] : pcstart(st);
                hit = bend >= pos;
            }
            const uint64_t m = wave_ballot(hit);
            if (m) {
                b = base + first_lane(m);
                break;
            }
        }
        if (b < 0) return fail(MT_DERR_INSERT_FAILED, S);
        const int st = uni(s.bst[b]), c = uni(s.lbcnt[b]);
        // leaf placement: first child with pos < len, or pos == len == 0 and breakTie
        // (mergeTree.ts:2248-2277); else the end of block b (:2431-2444)
        int best = 0x7fffffff;
        {
            const int cs = cs0();
#pragma unroll
            for (int j = K - 1; j >= 0; j--) {
                const int i = idx(j);
                const int ce = cum[j];
                const int csj = j ? cum[j - 1] : cs;
                const bool rm_before = (cf[j] & F_RM) && rseq[j] <= R;
                const bool h = i >= st && i < st + c && (ce > pos || (ce == pos && csj == pos && !rm_before));
                if (h) best = i;
            }
        }
        best = wave_min(best);
        const int k = best != 0x7fffffff ? best : st + c;
        const int t = alloc_id(S);
        if (t < 0) return;
        if (!arena_reserve((uint32_t)tlen, S)) return;
        const uint32_t top = text_top;
        for (int base = 0; base < tlen; base += 64) {
            const int i = base + lane;
            if (i < tlen) arena[top + i] = pay[i];
        }
        __threadfence_block();
        uint32_t fl = pay[tlen - 1] == '\n' ? F_NL : 0u;
        uint64_t p = 0;
        if (op.flags & MT_F_PROPS) {  // TextSegment.make -> addProperties
            fl |= F_PDEF;
            p = apply_pairs(0, pairs, np);
        }
        if (lane == 0) {
            s.props[t] = p;
            s.toff[t] = (uint16_t)top;
        }
        text_top = top + (uint32_t)tlen;
        wave_sync();
        Elem e;
        e.seq = S;
        e.rseq = 0;
        e.li = (uint32_t)tlen | ((uint32_t)t << kLenBits);
        e.cf = (uint32_t)C | fl;
        e.o0 = 0;
        e.o1 = 0;
        e.cum = 0;
        const int idx_in = k - st;  // index inside block b before a possible split
        const int before_nb = nbl(0);
        if (!insert_at<false>(k, b, e, S)) return;
        const int bb = (nbl(0) > before_nb && idx_in >= kMaxNodes / 2) ? b + 1 : b;
        if (S > min_seq) add_lru(bb, t, S);  // saveIfLocal -> addToLRUSet (mergeTree.ts:2164-2179)
    }

    // markRangeRemoved / annotateRange leaf actions over mapRange (mergeTree.ts:2607-2719,
    // 2565-2605, 2903-2965) after the two boundary splits
    MT_DEV void range_action(const mt_op_rec& op, const uint8_t* pairs, int np) {
        const int32_t S = op.seq;
        const int C = op.client, start = op.pos1, end = op.pos2;
        const bool is_remove = op.type == MT_OP_REMOVE;
        const bool rewrite = op.flags & MT_F_REWRITE;
        const uint32_t cb0 = C < 32 ? (1u << C) : 0u, cb1 = C < 32 ? 0u : (1u << (C - 32));
        {
            int cs = cs0();
#pragma unroll
            for (int j = 0; j < K; j++) {
                const int ce = cum[j];
                if (ce > cs && cs < end && ce > start) {
                    if (is_remove) {
                        if (cf[j] & F_RM) {  // addOverlappingClient (first remover wins)
                            o0[j] |= cb0;
                            o1[j] |= cb1;
                        } else {
                            cf[j] = (cf[j] & ~0xFF00u) | F_RM | ((uint32_t)C << 8);
                            rseq[j] = S;
                        }
                    } else {  // SegmentPropertiesManager.addProperties (remote, no combining op)
                        const uint32_t id = id_of(li[j]);
                        uint64_t p = (cf[j] & F_PDEF) ? s.props[id] : 0;
                        if (rewrite) p = 0;
                        s.props[id] = apply_pairs(p, pairs, np);
                        cf[j] |= F_PDEF;
                    }
                }
                cs = ce;
            }
        }
        spill(true);
        // addToLRUSet for touched segments in document order: one heap push per leaf block
        // whose needsScour is not already true, for its first touched segment
        block_starts();
        const int nb = nbl(0);
        for (int base = 0; base < nb; base += 64) {
            const int jb = base + lane;
            int first = -1;
            if (jb < nb) {
                const int st = s.bst[jb], c = s.lbcnt[jb];
                for (int q = 0; q < c; q++) {
                    const int k = st + q;
                    const int ce = s.pcum[k], cs = pcstart(k);
                    if (ce > cs && cs < end && ce > start) {
                        first = k;
                        break;
                    }
                }
            }
            uint64_t m = wave_ballot(first >= 0);
            while (m) {
                const int fl = first_lane(m);
                m &= m - 1;
                const int k = __builtin_amdgcn_readlane(first, fl);
                if (!add_lru(base + fl, uni(s.pid[k]), S)) return;
            }
        }
    }

    // Client.applyMsg for the observer (client.ts:797-828): the op, then updateSeqNumbers
    // (client.ts:821-828, MergeTree.setMinSeq mergeTree.ts:1718-1736).  Written so every
    // register-heavy routine has exactly one call site.
    MT_DEV void apply(const mt_op_rec& op, const uint8_t* payload) {
        const int np = op.flags >> MT_F_NPAIRS_SHIFT;
        const int32_t S = op.seq;
        if (op.type > MT_OP_NOOP) return fail(MT_DERR_BAD_OP, S);
        const uint8_t* pay = payload + op.payload_off;
        const int tlen = (int)op.payload_len - 2 * np;
        const uint8_t* pairs = pay + tlen;
        if (op.type != MT_OP_NOOP) {
            if (op.client == 0 || op.client >= MT_MAX_CLIENTS) return fail(MT_DERR_LIMITS, S);
            if (op.payload_len < (uint32_t)(2 * np)) return fail(MT_DERR_BAD_OP, S);
            if (!(cur_seq < S)) return fail(MT_DERR_SEQ_ORDER, S);      // client.ts:461-462
            if (!(min_seq <= op.msn)) return fail(MT_DERR_MSN_ORDER, S);  // client.ts:463-464
            for (int q = 0; q < np; q++)
                if (pairs[2 * q] >= MT_MAX_KEYS) return fail(MT_DERR_LIMITS, S);
            const bool ins = op.type == MT_OP_INSERT;
            if (op.pos1 < 0 || (!ins && op.pos2 < 0)) return fail(MT_DERR_BAD_OP, S);
            PROF_BEGIN(t0);
            scan(op.ref_seq, op.client);
            PROF_END(prof, P_SCAN, t0);
            PROF_BEGIN(t1);
            const int nbd = ins ? 1 : 2;
            for (int bi = 0; bi < nbd; bi++)
                if (!boundary(bi == 0 ? op.pos1 : op.pos2, S)) return;
            PROF_END(prof, P_BOUND, t1);
            PROF_BEGIN(t2);
            if (ins) {
                if (tlen > 0) place_insert(op, pay, tlen, pairs, np);
                PROF_END(prof, P_INSERT, t2);
            } else {
                range_action(op, pairs, np);
                PROF_END(prof, P_RANGE, t2);
            }
            if (err) return;
        }
        const int32_t msn = op.msn;
        for (int ph = 0; ph < 2; ph++) {
            if (ph == 0) {
                if (op.type == MT_OP_NOOP) continue;
            } else {
                if (op.flags & MT_F_GROUP_MORE) break;
                if (!(cur_seq <= S)) return fail(MT_DERR_SEQ_ORDER, S);
                cur_seq = S;
                if (!(msn <= S) || !(min_seq <= msn)) return fail(MT_DERR_MSN_ORDER, S);
                if (!(msn > min_seq)) break;
                min_seq = msn;
            }
            PROF_BEGIN(t3);
            zamboni();
            PROF_END(prof, P_ZAMBONI, t3);
            if (err) return;
        }
    }

    // ------------------------------------------------------------ load / store
    MT_DEV void load(const mt_gstate& g, uint32_t d) {
        const mt_doc_scalars& sc = g.sc[d];
        n = uni(sc.nseg);
        nlev = uni(sc.nlev);
        heap_n = uni(sc.heap_n);
        cur_seq = uni(sc.cur_seq);
        min_seq = uni(sc.min_seq);
        err = uni(sc.err);
        err_seq = uni(sc.err_seq);
        text_top = uniu(sc.text_top);
        text_half = uniu(sc.text_half);
        next_id = n;
        const size_t so = (size_t)d * g.segcap;
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = lane; i < n; i += 64) {
            s.props[i] = g.props[so + i];
            s.toff[i] = (uint16_t)g.toff[so + i];
        }
        const size_t lo = (size_t)d * g.lbcap;
        const int nb0 = uni(sc.nb[0]);
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = lane; i < nb0; i += 64) {
            s.lbcnt[i] = g.lbcnt[lo + i];
            s.lbscour[i] = g.lbscour[lo + i];
        }
        for (int Lv = 1; Lv < nlev; Lv++) {
            const size_t io = ((size_t)d * (MT_MAXLEV - 1) + (Lv - 1)) * g.ibcap;
            const int nbl_ = uni(sc.nb[Lv]);
#pragma clang loop unroll(disable) vectorize(disable)
            for (int i = lane; i < nbl_; i += 64) s.ibcnt[Lv - 1][i] = g.ibcnt[io + i];
        }
        const size_t ho = (size_t)d * g.hcap;
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = 1 + lane; i <= heap_n; i += 64) {
            s.hseq[i] = g.hseq[ho + i];
            s.hslot[i] = g.hslot[ho + i];  // position at store == id at load
        }
        if (lane < MT_MAXLEV) s.nb[lane] = sc.nb[lane];
        // whole-lane vector loads (segcap >= CAP, so reading past n stays inside the document's
        // rows); lanes past the last segment skip HBM entirely
        typedef uint32_t V2U __attribute__((ext_vector_type(2 * K)));
        typedef uint8_t VB __attribute__((ext_vector_type(K)));
        const int i0 = lane * K;
        // field by field, with scheduling barriers: the loaded rows never coexist with the state
        seq = 0x7fffffff;
        rseq = 0;
        li = kEmptyLi;
        cf = kEmptyCf;
        o0 = 0;
        o1 = 0;
        if (i0 < n) {
            VI live;
#pragma unroll
            for (int j = 0; j < K; j++) live[j] = i0 + j < n ? -1 : 0;
            {
                const VI v = *reinterpret_cast<const VI*>(g.seq + so + i0);
                seq = (v & live) | (0x7fffffff & ~live);
            }
            __builtin_amdgcn_sched_barrier(0);
            rseq = *reinterpret_cast<const VI*>(g.rseq + so + i0) & live;
            __builtin_amdgcn_sched_barrier(0);
            {
                const VU v = *reinterpret_cast<const VU*>(g.len + so + i0);
#pragma unroll
                for (int j = 0; j < K; j++) li[j] = live[j] ? (v[j] | ((uint32_t)(i0 + j) << kLenBits)) : kEmptyLi;
            }
            __builtin_amdgcn_sched_barrier(0);
            {
                const V2U ov = *reinterpret_cast<const V2U*>(g.ovl + so + i0);
#pragma unroll
                for (int j = 0; j < K; j++) {
                    o0[j] = live[j] ? ov[2 * j] : 0u;
                    o1[j] = live[j] ? ov[2 * j + 1] : 0u;
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            {
                const VB bc = *reinterpret_cast<const VB*>(g.client + so + i0);
                const VB br = *reinterpret_cast<const VB*>(g.rclient + so + i0);
                const VB bf = *reinterpret_cast<const VB*>(g.flags + so + i0);
#pragma unroll
                for (int j = 0; j < K; j++)
                    cf[j] = live[j] ? ((uint32_t)bc[j] | ((uint32_t)br[j] << 8) | ((uint32_t)bf[j] << 16)) : kEmptyCf;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        cum = 0;
        wave_sync();
        arena = abase + (size_t)text_half * textcap;
    }

    MT_DEV void store(const mt_gstate& g, uint32_t d) {
        const size_t so = (size_t)d * g.segcap;
        if ((uint32_t)n > g.segcap || nbl(0) > (int)g.lbcap || heap_n >= (int)g.hcap) fail(MT_DERR_CAPACITY, cur_seq);
        const int nn = min(n, (int)g.segcap);
        typedef uint32_t V2U __attribute__((ext_vector_type(2 * K)));
        typedef uint8_t VB __attribute__((ext_vector_type(K)));
        typedef uint64_t V64 __attribute__((ext_vector_type(K)));
        const int i0 = lane * K;
        if (i0 < nn) {  // whole-lane vector stores, field by field; slots past nn carry filler
            *reinterpret_cast<VI*>(g.seq + so + i0) = seq;
            *reinterpret_cast<VI*>(g.rseq + so + i0) = rseq;
            __builtin_amdgcn_sched_barrier(0);
            {
                V2U ov;
#pragma unroll
                for (int j = 0; j < K; j++) {
                    ov[2 * j] = o0[j];
                    ov[2 * j + 1] = o1[j];
                }
                *reinterpret_cast<V2U*>(g.ovl + so + i0) = ov;
            }
            __builtin_amdgcn_sched_barrier(0);
            {
                VB bc, br, bf;
#pragma unroll
                for (int j = 0; j < K; j++) {
                    bc[j] = (uint8_t)(cf[j] & 0xFFu);
                    br[j] = (uint8_t)((cf[j] >> 8) & 0xFFu);
                    bf[j] = (uint8_t)((cf[j] >> 16) & 0xFFu);
                }
                *reinterpret_cast<VB*>(g.client + so + i0) = bc;
                *reinterpret_cast<VB*>(g.rclient + so + i0) = br;
                *reinterpret_cast<VB*>(g.flags + so + i0) = bf;
            }
            __builtin_amdgcn_sched_barrier(0);
            {
                VU ln;
#pragma unroll
                for (int j = 0; j < K; j++) ln[j] = len_of(li[j]);
                *reinterpret_cast<VU*>(g.len + so + i0) = ln;
            }
            __builtin_amdgcn_sched_barrier(0);
            {
                VU to;
#pragma unroll
                for (int j = 0; j < K; j++) to[j] = s.toff[min(id_of(li[j]), (uint32_t)(CAP - 1))];
                *reinterpret_cast<VU*>(g.toff + so + i0) = to;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < K; j++) g.props[so + i0 + j] = s.props[min(id_of(li[j]), (uint32_t)(CAP - 1))];
        }
        wave_sync();
        // id -> position for the heap remap (toff is dead now)
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = lane; i < next_id; i += 64) s.toff[i] = kDead;
        wave_sync();
#pragma unroll
        for (int j = 0; j < K; j++) {
            const int i = idx(j);
            if (i < nn) s.toff[id_of(li[j])] = (uint16_t)i;
        }
        wave_sync();
        const size_t lo = (size_t)d * g.lbcap;
        const int nb0 = min(nbl(0), (int)g.lbcap);
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = lane; i < nb0; i += 64) {
            g.lbcnt[lo + i] = s.lbcnt[i];
            g.lbscour[lo + i] = s.lbscour[i];
        }
        for (int Lv = 1; Lv < nlev; Lv++) {
            const size_t io = ((size_t)d * (MT_MAXLEV - 1) + (Lv - 1)) * g.ibcap;
            const int nbl_ = min(nbl(Lv), (int)g.ibcap);
#pragma clang loop unroll(disable) vectorize(disable)
            for (int i = lane; i < nbl_; i += 64) g.ibcnt[io + i] = s.ibcnt[Lv - 1][i];
        }
        const size_t ho = (size_t)d * g.hcap;
        const int hn = min(heap_n, (int)g.hcap - 1);
#pragma clang loop unroll(disable) vectorize(disable)
        for (int i = 1 + lane; i <= hn; i += 64) {
            g.hseq[ho + i] = s.hseq[i];
            const uint16_t id = s.hslot[i];
            g.hslot[ho + i] = id == kDead ? kDead : s.toff[id];
        }
        if (lane == 0) {
            mt_doc_scalars& sc = g.sc[d];
            sc.nseg = nn;
            sc.nlev = nlev;
            sc.heap_n = heap_n;
            sc.cur_seq = cur_seq;
            sc.min_seq = min_seq;
            sc.err = err;
            sc.err_seq = err_seq;
            sc.text_top = text_top;
            sc.text_half = text_half;
        }
        if (lane < MT_MAXLEV) g.sc[d].nb[lane] = s.nb[lane];
    }
};

template <int K>
__global__ __launch_bounds__(64) void reg_apply_kernel(mt_gstate g, const mt_op_rec* __restrict__ ops,
                                                       const uint8_t* __restrict__ payload,
                                                       const uint32_t* __restrict__ row_ptr,
                                                       const uint32_t* __restrict__ doc_ids, uint32_t n_docs,
                                                       uint32_t op_lo, uint32_t op_cnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t w = blockIdx.x;
    if (w >= n_docs) return;
    const uint32_t d = doc_ids ? doc_ids[w] : w;
    RLds<K>& lds = *reinterpret_cast<RLds<K>*>(smem);
    RWave<K> wv(lds, g.text + (size_t)d * 2 * g.textcap, g.textcap);
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    const uint32_t a = min(r1, r0 + op_lo);
    const uint32_t b = op_cnt ? min(r1, a + op_cnt) : r1;
    if (a >= b) return;
    PROF_BEGIN(tl);
    wv.load(g, d);
    PROF_END(wv.prof, P_LOAD, tl);
    for (uint32_t i = a; i < b; i++) {
        if (wv.err) break;
        const mt_op_rec op = ops[i];
        wv.apply(op, payload);
#ifdef MT_PROF
        wv.prof[P_OPS]++;
#endif
    }
    PROF_BEGIN(tt);
    wv.store(g, d);
    PROF_END(wv.prof, P_STORE, tt);
#ifdef MT_PROF
    if (wv.lane == 0)
        for (int q = 0; q < P_NSLOT; q++) atomicAdd(&mt_prof_acc[(K == 2 ? 0 : K == 4 ? 24 : K == 8 ? 48 : 72) + q], (unsigned long long)wv.prof[q]);
#endif
}

}  // namespace mtr

extern "C" hipError_t mt_launch_apply_reg(int cap_class, const mt_gstate* g, const mt_op_rec* ops,
                                          const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                          uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    dim3 grid(n_docs), block(64);
#define MTR_LAUNCH(CAPV)                                                                                     \
    case CAPV: {                                                                                             \
        constexpr int K = CAPV / 64;                                                                         \
        hipLaunchKernelGGL((mtr::reg_apply_kernel<K>), grid, block, sizeof(mtr::RLds<K>), stream, *g, ops,    \
                           payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt);                                \
        return hipGetLastError();                                                                            \
    }
    switch (cap_class) {
        MTR_LAUNCH(128)
        MTR_LAUNCH(256)
        MTR_LAUNCH(512)
        MTR_LAUNCH(1024)
        default:
            return hipErrorInvalidValue;
    }
#undef MTR_LAUNCH
}

// diagnostic: read (and clear) the per-phase cycle totals of a -DMT_PROF build (zeros otherwise)
extern "C" int mt_prof_read(unsigned long long* out, int n) {
#ifdef MT_PROF
    if (n > 96) n = 96;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mtr::mt_prof_acc), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    unsigned long long z[96] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mtr::mt_prof_acc), z, sizeof z) != hipSuccess) return -1;
    return n;
#else
    for (int i = 0; i < n; i++) out[i] = 0;
    return 0;
#endif
}
