// mt_apply.hip -- the MI355X batched merge-tree apply engine (gfx950 / CDNA4).
//
// One wave64 per document.  A launch stages each document's compact state (HBM, document
// order, structure-of-arrays; mt_state.h) into the wave's slice of LDS, applies that
// document's next ops in seq order -- the observer Client.applyMsg of the reference
// (client.ts:797-828) -- and writes the state back compacted.  Per op, lanes cooperate:
//   * visibility of every segment for (refSeq R, client C) and the position prefix sums are
//     lane-parallel over the document order (DPP scan, mt_wave.h): this is what
//     PartialSequenceLengths caches on the CPU (partialLengths.ts:433-487);
//   * the B-tree shape (arity 8, split 4/4, pack, needsScour) is kept as per-level child-count
//     arrays beside the ordered segment array, so the shape-dependent placement and zamboni
//     rules (mergeTree.ts:2248-2277, 2345-2489, 1273-1478) are reproduced exactly;
//   * split / insert / remove / annotate become shifts of the order array plus per-slot
//     field writes; zamboni scour/pack are compactions of the order array + count edits.
// Nothing here is a dense contraction: no MFMA.  The wave's LDS footprint sets occupancy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mtgpu.h"
#include "mt_checksum.h"
#include "mt_state.h"
#include "mt_synth.h"
#include "mt_wave.h"

namespace mt {

constexpr int kMaxNodes = 8;           // MaxNodesInBlock, mergeTree.ts:334
constexpr int kTextGranularity = 256;  // MergeTree.TextSegmentGranularity, mergeTree.ts:1059

// An op's property pairs in its payload: narrow (key u8, value u8) or wide (MT_OP_WIDE: key u8,
// value u16 LE); value 0 = null = delete
struct Pairs {
    const uint8_t* p;
    int np;
    bool wide;
    MT_DEV int key(int q) const { return p[wide ? 3 * q : 2 * q]; }
    MT_DEV uint32_t val(int q) const { return wide ? (uint32_t)p[3 * q + 1] | ((uint32_t)p[3 * q + 2] << 8) : p[2 * q + 1]; }
    MT_DEV int key_limit() const { return wide ? MT_MAX_KEYS_WIDE : MT_MAX_KEYS; }
};

// The editing form's per-document pending-group state with GN group slots (mt_loc's fields; GN = 64
// is mt_loc itself)
template <int GN>
struct LocState {
    int32_t own;
    uint32_t glo, ghi;
    uint32_t stamp;
    uint32_t gt[GN];
    uint32_t lseq;
    uint32_t gls[GN];
    uint32_t rgn, rgpn;
};
// mt_loc's scalars: the editing forms with 64 group slots keep the groups' stamps and localSeqs
// (mt_loc.gt / gls) in HBM, in the document's own mt_loc (Wave::gtp / glsp)
struct LocLite {
    int32_t own;
    uint32_t glo, ghi;
    uint32_t stamp;
    uint32_t lseq;
    uint32_t rgn, rgpn;
};

// An editing document's per-segment rows in HBM: its big-pool row once it has one, else its
// MT_LOC_CAP-slot row (mt_state.h)
struct LocRow {
    uint64_t* gm;
    uint64_t* pk;
    uint32_t* ct;
    uint64_t* lsq;
    int cap;
};
MT_DEV LocRow loc_row(const mt_gstate& g, uint32_t d) {
    const uint32_t r = g.locbig[d];
    if (r != MT_NO_ROW) {
        const size_t o = (size_t)r * MT_LOC_BIGCAP;
        return {g.gmb + o, g.pkb + o, g.ctb + o, g.lsqb + o, MT_LOC_BIGCAP};
    }
    const size_t o = (size_t)d * MT_LOC_CAP;
    return {g.gm + o, g.pk + o, g.ct + o, g.lsq + o, MT_LOC_CAP};
}

// W: a wide document (include/mtgpu.h "limits"): per slot also the overlap ids >= 64 (ovx) and the
// property words ph / pxl / pxh / pxx (u16 value ids, keys 8..31); UTF-16 text.  GW: (LOC) group-mask
// words per slot, 64 GW pending edits at most (GW > 1: MT_WIDE_GROUPS documents, HBM workspace only)
template <int CAP, bool LOC = false, bool W = false, int GW = 1>
struct Lds {
    static constexpr int LB = CAP / 2;      // leaf blocks
    static constexpr int IB = CAP / 8 + 8;  // blocks per interior level
    static constexpr int H = CAP / 2 + 64;  // heap entries (1-based)
    uint64_t ovl[CAP];
    uint64_t props[CAP];
    int32_t seq[CAP];
    int32_t rseq[CAP];
    uint32_t len[CAP];
    uint32_t toff[CAP];
    int32_t cum[CAP];       // scratch: inclusive prefix of visible length per position
    uint16_t bst[LB + 1];   // scratch: leaf-block start positions
    int32_t hseq[H];
    uint16_t hslot[H];
    uint16_t order[CAP];    // document order -> slot
    uint16_t freel[CAP];
    // short client ids: u8 in the narrow form, u16 in the wide one (ids up to 65534)
    typename std::conditional<W, uint16_t, uint8_t>::type client[CAP];
    typename std::conditional<W, uint16_t, uint8_t>::type rclient[CAP];
    uint8_t flags[CAP];
    uint8_t lbcnt[LB];
    uint8_t lbscour[LB];
    uint8_t ibcnt[MT_MAXLEV - 1][IB];
    int32_t n, nlev, heap_n, cur_seq, min_seq, err, err_seq, nfree, next_slot;
    int32_t evn, evseq;     // delta events recorded (mt_events_enable) / seq of the message applying
    int32_t nb[MT_MAXLEV];
    uint32_t text_top, text_half;
    int32_t gcref[LOC ? 1 : 64];  // generator: latest refSeq per client (deli clientSeqManager)
    int32_t gstall;         // generator: client 1 holds its refSeq until this seq
    uint32_t gpay;          // generator: payload bytes used in this document's region
    // an editing client's document (LOC, mt_loc): per slot the pending group mask, the pending
    // property counts (MT_PK_*) and the creation stamp
    typename std::conditional<(GW > 1), LocState<64 * GW>, LocLite>::type lc;
    uint64_t ovx[W ? 4 * CAP : 1];  // (W) overlapping removers >= 64: ids 0..15 of the u16 lists (mt_checksum.h)
    uint64_t ph[W ? CAP : 1];
    uint64_t pxl[W ? CAP : 1];
    uint64_t pxh[W ? CAP : 1];
    uint32_t wide;                // the document's mt_doc_scalars.wide bits
    uint32_t lkeys;               // its declared label keys (mt_doc_scalars.label_keys)
    // a stale marker's cached label value ids (mt_gstate.slab), by slot; the editing form keeps them
    // in HBM (mt_gstate.slabx): its LDS is at the two-waves-per-CU limit without them
    uint32_t slab[LOC ? 1 : CAP];
    // (LOC) the creation stamps, the localSeq pairs, the pending property counts and the pending-group
    // masks by slot: the HBM-workspace forms keep them here, the LDS-staged ones launch without this
    // tail (loc_lds_bytes) and keep them in HBM (mt_gstate.ctx / lsqx / pkx / gmxs; Wave::ctp / lsqp
    // / pkp / gmp) -- read at annotates, acks, reconnects and zamboni's pending test (one load per
    // block), and 7 KB less LDS per document at 256 slots is the eighth to twelfth wave per CU
    uint32_t ct[LOC ? CAP : 1];
    uint64_t lsq[LOC ? CAP : 1];  // localSeq (low 32) / localRemovedSeq (high 32), 0: undefined
    uint64_t pk[LOC ? CAP : 1];   // pending property counts (MT_PK_*)
    uint64_t gm[LOC ? CAP * GW : 1];  // pending-group masks (GW words per slot)
    // (W) the extension (mt_state.h MT_WIDE_XK / MT_WIDE_XO), last: ids 16..31 of the overlap lists
    // and keys 16..31 ([slot][4] each, mt_state.h pxx).  The HBM-workspace form keeps it here; the
    // LDS-staged form launches without these members (kExtBytes less LDS) and stages the extension
    // of the documents that use it in an HBM region of the same layout (Wave::ext)
    uint64_t ovh[W ? 4 * CAP : 1];
    uint64_t pxx[W ? 4 * CAP : 1];
    static constexpr size_t kExtBytes = W ? 2 * 4 * CAP * sizeof(uint64_t) : 0;
};
// (the extension is the struct's tail: a launch may leave it out of its LDS)
// the LDS of the editing form staged in LDS: Lds without the stamps' tail (Lds::ct and after)
template <int CAP>
constexpr size_t loc_lds_bytes() {
    using L = Lds<CAP, true>;
    return offsetof(L, ct);
}
// the LDS of the wide form staged in LDS: Lds without the extension
template <int CAP>
constexpr size_t wl_lds_bytes() { return sizeof(Lds<CAP, false, true>) - Lds<CAP, false, true>::kExtBytes; }
using LdsW256 = Lds<256, false, true>;
using LdsW512 = Lds<512, false, true>;
static_assert(offsetof(LdsW256, ovh) + LdsW256::kExtBytes == sizeof(LdsW256), "the wide extension ends Lds");
static_assert(offsetof(LdsW512, ovh) + LdsW512::kExtBytes == sizeof(LdsW512), "the wide extension ends Lds");

// G = false: the document is staged in the wave's LDS.  G = true (documents above 2048 segments,
// SURVEY.md §8 a9 "unbounded B-tree"): the same structure lives in a per-wave workspace in HBM
// (mt_launch_apply_big); lanes exchange it through the vector L1 / L2, so a pass boundary also
// waits for the wave's outstanding stores (workgroup scope = the wave's CU).
template <int CAP, bool G = false, bool LOC = false, bool W = false, int GW = 1>
struct Wave {
    using L = Lds<CAP, LOC, W, GW>;
    using CT = typename std::conditional<W, uint16_t, uint8_t>::type;  // a short client id (Lds::client)
    // (LOC) pending-group masks: GW words per slot; pending edit ordinal N is bit N % GN
    static constexpr uint32_t GN = 64u * GW;
    MT_DEV uint64_t& gmw(int sl, uint32_t N) { return gmp[sl * GW + (int)((N % GN) >> 6)]; }
    MT_DEV bool gm_has(int sl, uint32_t N) { return (gmw(sl, N) >> (N & 63u)) & 1ull; }
    MT_DEV void gm_set(int sl, uint32_t N) { gmw(sl, N) |= 1ull << (N & 63u); }
    MT_DEV void gm_clr(int sl, uint32_t N) { gmw(sl, N) &= ~(1ull << (N & 63u)); }
    MT_DEV bool gm_any(int sl) {
        uint64_t v = 0;
        for (int w = 0; w < GW; w++) v |= gmp[sl * GW + w];
        return v != 0;
    }
    MT_DEV void gm_copy(int t, int sl) {
        for (int w = 0; w < GW; w++) gmp[t * GW + w] = gmp[sl * GW + w];
    }
    MT_DEV void gm_zero(int t) {
        for (int w = 0; w < GW; w++) gmp[t * GW + w] = 0ull;
    }
    using TC = typename std::conditional<W, uint16_t, uint8_t>::type;  // a text code unit in the arena
    MT_DEV static void sync() {
        if (G) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        } else {
            wave_sync();
        }
    }
    L& s;
    const int lane;
    TC* const abase;        // document's double-buffered arena: [2][textcap]
    TC* arena;              // current half
    const uint32_t textcap; // code units per half
    mt_event* const ev;     // the document's delta-event records (null: not recording)
    const uint32_t evcap;
    // (W) the extension's region ([ovh][pxx] as in Lds), and its parts this launch stages (null: not
    // staged -- mt_state.h MT_WIDE_XO / MT_WIDE_XK, decided by binning)
    uint64_t* ext = nullptr;
    uint64_t* xo_p = nullptr;
    uint64_t* xk_p = nullptr;
    uint32_t* ctp = nullptr;  // (LOC) the creation stamps by slot (Lds::ct, or HBM: mt_gstate.ctx)
    uint64_t* lsqp = nullptr;  // (LOC) the localSeq pairs by slot (Lds::lsq, or HBM: mt_gstate.lsqx)
    uint64_t* pkp = nullptr;   // (LOC) the pending property counts by slot (Lds::pk, or HBM: mt_gstate.pkx)
    uint64_t* gmp = nullptr;   // (LOC) the pending-group masks by slot (Lds::gm, or HBM: mt_gstate.gmxs)
    uint32_t* gtp = nullptr;   // (LOC) the groups' creation stamps and localSeqs (LocState, or the
    uint32_t* glsp = nullptr;  // document's mt_loc in HBM)
    // (LOC) their writes are read by other lanes: through HBM in the LDS-staged forms
    MT_DEV static void ct_publish() {
        if (!G) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    }
    uint32_t rix = 0;       // index of the record being applied within its document
    mt_op_rec* rg = nullptr;  // (LOC) the document's regenerated-op buffer and its payload
    uint8_t* rgp = nullptr;

    uint32_t* xslab = nullptr;  // (LOC) this document's slot-indexed slab in HBM while it tracks labels
    MT_DEV Wave(L& lds, uint8_t* a, uint32_t tc_bytes, mt_event* e = nullptr, uint32_t ec = 0)
        : s(lds), lane(lane_id()), abase(reinterpret_cast<TC*>(a)), arena(reinterpret_cast<TC*>(a)),
          textcap(tc_bytes / (uint32_t)sizeof(TC)), ev(e), evcap(ec) {}

    // ------------------------------------------------------------ wide state
    // removedClientOverlap holds client C (ids < 64: the bitmask; a wide document's others: ovx, and
    // ovh with the extension)
    MT_DEV const uint64_t* ovx_hi(int slot) const { return xo_p ? xo_p + 4 * slot : nullptr; }
    MT_DEV bool ovl_has(int slot, int C) const {
        if (C < 64) return C >= 0 && ((s.ovl[slot] >> C) & 1ull);
        if constexpr (W) return mt_ovx_has2(&s.ovx[4 * slot], ovx_hi(slot), (uint32_t)C);
        return false;
    }
    // addOverlappingClient (mergeTree.ts:2544-2552); false: a wide segment's list is full (16 ids
    // without the extension -- binning gives a document that could get there the extension first)
    MT_DEV bool ovl_add(int slot, int C) {
        if (C < 64) {
            s.ovl[slot] |= 1ull << C;
            return true;
        }
        if constexpr (W) {
            uint64_t* lo = &s.ovx[4 * slot];
            const uint64_t* hi = ovx_hi(slot);
            if (mt_ovx_has2(lo, hi, (uint32_t)C)) return true;
            if (mt_ovx_id2(lo, hi, xo_p ? MT_OVX_IDS - 1 : 15)) return false;  // full: MT_DERR_LIMITS
            uint64_t out[8] = {};  // insert C into the ascending u16 list
            int j = 0;
            bool done = false;
            auto put = [&](uint32_t v) {
                out[j >> 2] |= (uint64_t)v << (16 * (j & 3));
                j++;
            };
            for (int q = 0; q < MT_OVX_IDS; q++) {
                const uint32_t v = mt_ovx_id2(lo, hi, q);
                if (!v) break;
                if (!done && (uint32_t)C < v) {
                    put((uint32_t)C);
                    done = true;
                }
                put(v);
            }
            if (!done) put((uint32_t)C);
            for (int w = 0; w < 4; w++) lo[w] = out[w];
            if (xo_p)
                for (int w = 0; w < 4; w++) xo_p[4 * slot + w] = out[4 + w];
            return true;
        }
        return false;
    }
    // a slot's overlap list ids >= 64: copied from another slot / cleared
    MT_DEV void ovx_copy(int t, int sl) {
        for (int q = 0; q < 4; q++) s.ovx[4 * t + q] = s.ovx[4 * sl + q];
        if (xo_p)
            for (int q = 0; q < 4; q++) xo_p[4 * t + q] = xo_p[4 * sl + q];
    }
    MT_DEV void ovx_zero(int t) {
        for (int q = 0; q < 4; q++) s.ovx[4 * t + q] = 0ull;
        if (xo_p)
            for (int q = 0; q < 4; q++) xo_p[4 * t + q] = 0ull;
    }
    // (W) the words holding key k of a slot: its low-byte and high-byte words
    MT_DEV uint64_t* plo(int sl, int k) {
        return k < 8 ? &s.props[sl] : k < 16 ? &s.pxl[sl] : xk_p + 4 * sl + 2 * ((k - 16) >> 3);
    }
    MT_DEV uint64_t* phi(int sl, int k) {
        return k < 8 ? &s.ph[sl] : k < 16 ? &s.pxh[sl] : xk_p + 4 * sl + 2 * ((k - 16) >> 3) + 1;
    }
    // value id of key k of a slot (0 = absent)
    MT_DEV uint32_t pval(int sl, int k) {
        const int sh = 8 * (k & 7);
        if constexpr (W) {
            if (k >= 16 && !xk_p) return 0u;
            return (uint32_t)((*plo(sl, k) >> sh) & 0xFFu) | ((uint32_t)((*phi(sl, k) >> sh) & 0xFFu) << 8);
        }
        return k < 8 ? (uint32_t)((s.props[sl] >> sh) & 0xFFu) : 0u;
    }
    MT_DEV void pset(int sl, int k, uint32_t v) {
        const int sh = 8 * (k & 7);
        const uint64_t m = ~(0xFFull << sh);
        if constexpr (W) {
            uint64_t* lo = plo(sl, k);
            uint64_t* hi = phi(sl, k);
            *lo = (*lo & m) | ((uint64_t)(v & 0xFFu) << sh);
            *hi = (*hi & m) | ((uint64_t)(v >> 8) << sh);
        } else if (k < 8) {
            s.props[sl] = (s.props[sl] & m) | ((uint64_t)(v & 0xFFu) << sh);
        }
    }
    MT_DEV void pclear(int sl) {
        s.props[sl] = 0;
        if constexpr (W) {
            s.ph[sl] = s.pxl[sl] = s.pxh[sl] = 0;
            if (xk_p)
                for (int q = 0; q < 4; q++) xk_p[4 * sl + q] = 0;
        }
    }
    MT_DEV void pcopy(int dst, int src) {
        s.props[dst] = s.props[src];
        if constexpr (W) {
            s.ph[dst] = s.ph[src];
            s.pxl[dst] = s.pxl[src];
            s.pxh[dst] = s.pxh[src];
            if (xk_p)
                for (int q = 0; q < 4; q++) xk_p[4 * dst + q] = xk_p[4 * src + q];
        }
    }
    MT_DEV bool peq(int a, int b) const {
        if (s.props[a] != s.props[b]) return false;
        if constexpr (W) {
            if (s.ph[a] != s.ph[b] || s.pxl[a] != s.pxl[b] || s.pxh[a] != s.pxh[b]) return false;
            if (xk_p)
                for (int q = 0; q < 4; q++)
                    if (xk_p[4 * a + q] != xk_p[4 * b + q]) return false;
        }
        return true;
    }
    // the op's (key, value) pairs onto a slot's props (properties.ts:95-116)
    MT_DEV void papply(int sl, const Pairs& pr) {
        for (int q = 0; q < pr.np; q++) pset(sl, pr.key(q), pr.val(q));
    }
    static constexpr int kKeys = W ? MT_MAX_KEYS_WIDE : MT_MAX_KEYS;

    // ------------------------------------------------------------ block caches
    // The HierMergeBlock label caches (rightmostTiles / leftmostTiles / rangeStacks, mergeTree.ts:
    // 263-318) of a document with declared label keys (mt_set_label_keys): blockUpdate rebuilds a
    // leaf block's from its live markers' labels; annotateRange changes labels without one
    // (mergeTree.ts:2565-2605).  A marker annotated since its leaf block's last rebuild is "stale":
    // its flags carry MT_SF_STALE and slab the tile / range label value ids the caches still hold.
    MT_DEV bool track() const { return s.lkeys != MT_NO_LABEL_KEYS; }
    // (lane-parallel, before an annotate changes the slot's props)
    MT_DEV void mark_stale(int sl) {
        const uint8_t f = s.flags[sl];
        if ((f & MT_SF_MARKER) && !(f & MT_SF_STALE)) {
            const uint32_t kt = s.lkeys & 0xFFu, kr = (s.lkeys >> 8) & 0xFFu;
            const bool def = (f & MT_SF_PDEF) != 0;
            const uint32_t vt = def && kt < (uint32_t)kKeys ? pval(sl, (int)kt) : 0u;
            const uint32_t vr = def && kr < (uint32_t)kKeys ? pval(sl, (int)kr) : 0u;
            if constexpr (LOC)
                xslab[sl] = vt | (vr << 16);
            else
                s.slab[sl] = vt | (vr << 16);
            s.flags[sl] = (uint8_t)(f | MT_SF_STALE);
        }
    }
    // blockUpdate of the leaf block(s) holding positions [k0, k1): their caches are current again
    MT_DEV void refresh(int k0, int k1) {
        if (!track()) return;
        sync();
        for (int i = k0 + lane; i < k1; i += 64) s.flags[s.order[i]] &= (uint8_t)~MT_SF_STALE;
        sync();
    }

    // ------------------------------------------------------------ delta events
    // One callback record (mt_event, include/mtgpu.h), written by lane 0 in firing order: the
    // reference's mergeTreeDeltaCallback / mergeTreeMaintenanceCallback (mergeTreeDeltaCallback.ts).
    MT_DEV void emit(int op, unsigned flags, int leaf, int pos, uint32_t len) {
        if (!ev) return;
        const int n = s.evn;
        if (lane == 0 && n < (int)evcap) {
            mt_event e{};
            e.seq = s.evseq;
            e.op = (int8_t)op;
            e.flags = (uint8_t)flags;
            e.leaf = leaf;
            e.pos = pos;
            e.len = len;
            ev[n] = e;
        }
        sync();
        s.evn = n + 1;
        sync();
    }
    // characters of unremoved segments before document position k (the local view's position)
    MT_DEV int local_prefix(int k) {
        int t = 0;
        for (int base = 0; base < k; base += 64) {
            const int i = base + lane;
            if (i < k) {
                const int sl = s.order[i];
                t += (s.flags[sl] & MT_SF_REMOVED) ? 0 : (int)s.len[sl];
            }
        }
        return wave_sum(t);
    }
    // The REMOVE / ANNOTATE callback (mergeTree.ts:2705-2712 / 2592-2600): its delta segments in
    // document order, lane-parallel.  REMOVE runs after the edits (segments this op removed: rseq
    // == S by C; their local position with the removal applied), ANNOTATE before them (the
    // propertyDeltas need the previous values; annotate does not move the local view).
    MT_DEV void emit_range(bool is_remove, int32_t S, int C, int start, int end, const Pairs& pr, bool rewrite) {
        if (!ev) return;
        const int n = s.n, e0 = s.evn;
        int cnt = 0, lpos = 0;
        const uint64_t below = (1ull << lane) - 1ull;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            bool hit = false;
            int ll = 0;
            uint32_t ln = 0;
            uint32_t pm = 0;
            uint8_t xf = 0;
            uint16_t pv[kKeys] = {0};
            int sl = 0;
            if (i < n) {
                sl = s.order[i];
                const uint8_t f = s.flags[sl];
                ln = s.len[sl];
                uint64_t pk = 0;  // (LOC, a remote annotate: keys with pending local changes are skipped)
                if constexpr (LOC) pk = (S != -1 && (f & MT_SF_PDEF)) ? pkp[sl] : 0ull;
                ll = (f & MT_SF_REMOVED) ? 0 : (int)ln;
                const int ce = s.cum[i], cs = cstart(i);
                hit = ce > cs && cs < end && ce > start;
                if (is_remove) {
                    hit = hit && (f & MT_SF_REMOVED) && !(f & MT_SF_OVW) && s.rseq[sl] == S && s.rclient[sl] == C;
                } else if (hit) {
                    // SegmentPropertiesManager.addProperties' deltas (segmentPropertiesManager.ts:60-108):
                    // a rewrite records each key it deletes with its old value; every key of the op
                    // records the value before it is set (null when absent, and null for a rewrite's
                    // null-valued key, deleted a moment earlier)
                    const bool pdef = (f & MT_SF_PDEF) != 0;
                    if (MT_PK_RW(pk) > 0) {
                        xf = MT_EVF_NOPD;  // dropped while a local rewrite is pending: propertyDeltas undefined
                    } else {
                        if (rewrite) {
                            for (int k = 0; k < kKeys; k++) {
                                const uint32_t old = pdef ? pval(sl, k) : 0u;
                                if (old && (k >= 8 || MT_PK_KEY(pk, k) == 0)) {
                                    bool keep = false;  // a key the rewrite sets again keeps its value here
                                    for (int q = 0; q < pr.np; q++) keep = keep || (pr.key(q) == k && pr.val(q) != 0);
                                    if (!keep) pm |= 1u << k;
                                }
                                pv[k] = (uint16_t)old;
                            }
                        }
                        for (int q = 0; q < pr.np; q++) {
                            const int k = pr.key(q);
                            if (k < 8 && MT_PK_KEY(pk, k) > 0) continue;
                            const uint32_t prev = (rewrite && pr.val(q) == 0) ? 0u : (pdef ? pval(sl, k) : 0u);
                            pm |= 1u << k;
                            pv[k] = (uint16_t)prev;
                        }
                    }
                }
            }
            const int incl = wave_incl_scan(ll);
            const uint64_t m = wave_ballot(hit);
            const int idx = cnt + __popcll(m & below);
            if (hit && e0 + idx < (int)evcap) {
                mt_event e{};
                e.seq = s.evseq;
                e.op = (int8_t)(is_remove ? MT_EV_REMOVE : MT_EV_ANNOTATE);
                e.flags = (uint8_t)((idx == 0 ? MT_EVF_FIRST : 0) | xf);
                e.pmask = pm;
                e.leaf = i;
                e.pos = lpos + incl - ll;
                e.len = ln;
                for (int k = 0; k < kKeys; k++) e.pvals[k] = (pm >> k) & 1u ? pv[k] : (uint16_t)0;
                ev[e0 + idx] = e;
            }
            cnt += __popcll(m);
            lpos += wave_last(incl);
        }
        sync();
        if (cnt == 0) return emit(is_remove ? MT_EV_REMOVE : MT_EV_ANNOTATE, MT_EVF_FIRST | MT_EVF_EMPTY, -1, -1, 0);
        s.evn = e0 + cnt;
        sync();
    }

    MT_DEV void fail(int code, int32_t seq) {
        if (s.err == 0) {
            s.err = code;
            s.err_seq = seq;
        }
        sync();
    }

    // -------------------------------------------------------------- visibility
    // nodeLength leaf branch for a remote client (mergeTree.ts:1667-1697)
    MT_DEV int vis(int slot, int32_t R, int C) const {
        if constexpr (LOC) {
            // the editing client sees its local view (nodeLength :1660-1665, localNetLength
            // :1161-1172); others never see a pending insert (seq -1) and see through a pending
            // removal (removedSeq -1) (:1675-1686)
            if (C == s.lc.own) return (s.flags[slot] & MT_SF_REMOVED) ? 0 : (int)s.len[slot];
            const bool seen = (s.client[slot] == C) || (s.seq[slot] != -1 && s.seq[slot] <= R);
            if (!seen) return 0;
            if ((s.flags[slot] & MT_SF_REMOVED) &&
                (s.rclient[slot] == C || ovl_has(slot, C) || (s.rseq[slot] != -1 && s.rseq[slot] <= R)))
                return 0;
            return (int)s.len[slot];
        }
        const bool seen = (s.client[slot] == C) || (s.seq[slot] <= R);
        if (!seen) return 0;
        if (s.flags[slot] & MT_SF_REMOVED) {
            // (C = NonCollabClient for a snapshot body append: no overlap bit, MT_OP_LOAD)
            if (s.rclient[slot] == C || ovl_has(slot, C) || s.rseq[slot] <= R) return 0;
        }
        return (int)s.len[slot];
    }

    // cum[i] = sum of vis over positions 0..i; returns the total (getLength(R, C))
    MT_DEV int scan(int32_t R, int C) {
        const int n = s.n;
        int carry = 0;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            const int v = i < n ? vis(s.order[i], R, C) : 0;
            const int incl = wave_incl_scan(v) + carry;
            if (i < n) s.cum[i] = incl;
            carry = wave_last(incl);
        }
        sync();
        return carry;
    }
    MT_DEV int cstart(int k) const { return k > 0 ? s.cum[k - 1] : 0; }

    // ------------------------------------------------------------- array shifts
    template <class T>
    MT_DEV void shift_right(T* a, int from, int count_end) {  // a[from..end) -> a[from+1..end+1)
        for (int hi = count_end; hi > from; hi -= 64) {
            const int i = hi - 1 - lane;
            T v{};
            const bool ok = i >= from;
            if (ok) v = a[i];
            sync();
            if (ok) a[i + 1] = v;
            sync();
        }
    }
    template <class T>
    MT_DEV void shift_left(T* a, int from, int count_end, int by) {  // a[from..end) -> a[from-by..)
        for (int lo = from; lo < count_end; lo += 64) {
            const int i = lo + lane;
            T v{};
            const bool ok = i < count_end;
            if (ok) v = a[i];
            sync();
            if (ok) a[i - by] = v;
            sync();
        }
    }

    // ----------------------------------------------------------------- blocks
    MT_DEV uint8_t* lvl(int L) { return L == 0 ? s.lbcnt : s.ibcnt[L - 1]; }
    MT_DEV int lvlcap(int Lv) const { return Lv == 0 ? L::LB : L::IB; }

    // bst[b] = first position of leaf block b (bst[nb0] = n)
    MT_DEV void block_starts() {
        const int nb = s.nb[0];
        int carry = 0;
        for (int base = 0; base < nb; base += 64) {
            const int b = base + lane;
            const int c = b < nb ? (int)s.lbcnt[b] : 0;
            const int incl = wave_incl_scan(c) + carry;
            if (b < nb) s.bst[b] = incl - c;
            carry = wave_last(incl);
        }
        if (lane == 0) s.bst[nb] = carry;
        sync();
    }

    // leaf block containing position k (first non-empty block whose range holds k); needs bst
    MT_DEV int block_of_pos(int k) {
        const int nb = s.nb[0];
        for (int base = 0; base < nb; base += 64) {
            const int b = base + lane;
            const bool hit = b < nb && s.bst[b] <= k && k < s.bst[b] + (int)s.lbcnt[b];
            const uint64_t m = wave_ballot(hit);
            if (m) return base + first_lane(m);
        }
        return -1;
    }

    // parent index (level L+1) of block b at level L, and the first child index of that parent
    MT_DEV int parent_of(int L, int b, int* first_child) {
        const uint8_t* pc = lvl(L + 1);
        const int np = s.nb[L + 1];
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

    // insert a new block with `cnt` children right after block b at level L
    MT_DEV bool insert_block_after(int L, int b, int cnt) {
        const int nb = s.nb[L];
        if (nb + 1 > lvlcap(L)) return false;
        uint8_t* a = lvl(L);
        shift_right(a, b + 1, nb);
        if (L == 0) shift_right(s.lbscour, b + 1, nb);
        if (lane == 0) {
            a[b + 1] = (uint8_t)cnt;
            if (L == 0) s.lbscour[b + 1] = MT_SC_UNDEF;
        }
        s.nb[L] = nb + 1;
        sync();
        return true;
    }

    // block b at level L has reached kMaxNodes children: split 4/4 upward (split +
    // insertingWalk's parent insert + updateRoot, mergeTree.ts:2446-2489, 1876-1887)
    MT_DEV bool split_up(int L, int b, int32_t seq) {
        for (;;) {
            const int half = kMaxNodes / 2;
            int parent = -1;
            if (L < s.nlev - 1) parent = parent_of(L, b, nullptr);
            if (lane == 0) lvl(L)[b] = (uint8_t)half;
            sync();
            if (!insert_block_after(L, b, half)) return fail(MT_DERR_CAPACITY, seq), false;
            if (L == s.nlev - 1) {  // split the root: new root with 2 children
                if (s.nlev + 1 > MT_MAXLEV) return fail(MT_DERR_CAPACITY, seq), false;
                const int nl = s.nlev;
                if (lane == 0) lvl(nl)[0] = 2;
                s.nb[nl] = 1;
                s.nlev = nl + 1;
                sync();
                return true;
            }
            uint8_t* pc = lvl(L + 1);
            const int c = (int)pc[parent] + 1;
            if (lane == 0) pc[parent] = (uint8_t)c;
            sync();
            if (c < kMaxNodes) return true;
            L = L + 1;
            b = parent;
        }
    }

    // ------------------------------------------------------------------ slots
    MT_DEV int alloc_slot(int32_t seq) {
        int sl;
        if (s.nfree > 0) {
            sl = s.freel[s.nfree - 1];
            sync();
            s.nfree = s.nfree - 1;
        } else {
            sl = s.next_slot;
            if (sl >= CAP) {
                fail(MT_DERR_CAPACITY, seq);
                return -1;
            }
            s.next_slot = sl + 1;
        }
        sync();
        return sl;
    }
    // unlink: free the slot and kill heap entries that still point at it
    MT_DEV void free_slot(int sl) {
        const int hn = s.heap_n;
        for (int base = 1; base <= hn; base += 64) {
            const int i = base + lane;
            if (i <= hn && s.hslot[i] == sl) s.hslot[i] = MT_DEAD_SLOT;
        }
        if (lane == 0) s.freel[s.nfree] = (uint16_t)sl;
        sync();
        s.nfree = s.nfree + 1;
        sync();
    }

    // insert slot `sl` at document position k of leaf block b; splits blocks as needed.
    // `cum_val` >= 0 also keeps the cum[] scratch aligned (for a second boundary split).
    MT_DEV bool insert_at(int k, int b, int sl, int cum_val, int32_t seq) {
        const int n = s.n;
        if (n + 1 > CAP) return fail(MT_DERR_CAPACITY, seq), false;
        shift_right(s.order, k, n);
        if (cum_val >= 0) shift_right(s.cum, k, n);
        if (lane == 0) {
            s.order[k] = (uint16_t)sl;
            if (cum_val >= 0) s.cum[k] = cum_val;
        }
        s.n = n + 1;
        const int c = (int)s.lbcnt[b] + 1;
        sync();
        if (lane == 0) s.lbcnt[b] = (uint8_t)c;
        sync();
        if (c >= kMaxNodes) return split_up(0, b, seq);
        return true;
    }

    // ------------------------------------------------------------------- text
    MT_DEV void arena_copy(uint32_t dst, uint32_t src, uint32_t n) {
        for (uint32_t base = 0; base < n; base += 64) {
            const uint32_t i = base + lane;
            TC v = 0;
            if (i < n) v = arena[src + i];
            __threadfence_block();
            if (i < n) arena[dst + i] = v;
        }
        __threadfence_block();
    }

    // Copy every linked segment's text, in document order, into the other half of the arena
    // (TextSegment text has no identity; only its content is state).  Afterwards adjacent
    // segments are adjacent in the arena, so later appends are free.
    MT_DEV void compact_text() {
        TC* dst = abase + (size_t)(s.text_half ^ 1u) * textcap;
        const int n = s.n;
        uint32_t carry = 0;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            const int sl = i < n ? s.order[i] : 0;
            const int l = i < n ? (int)s.len[sl] : 0;
            const int incl = wave_incl_scan(l);
            const uint32_t at = carry + (uint32_t)(incl - l);
            if (i < n) {
                const TC* src = arena + s.toff[sl];
                for (int q = 0; q < l; q++) dst[at + q] = src[q];
            }
            sync();
            if (i < n) s.toff[sl] = at;
            carry += (uint32_t)wave_last(incl);
        }
        __threadfence_block();
        s.text_half = s.text_half ^ 1u;
        s.text_top = carry;
        arena = dst;
        sync();
    }
    MT_DEV bool arena_reserve(uint32_t need, int32_t seq) {
        if (s.text_top + need <= textcap) return true;
        compact_text();
        if (s.text_top + need <= textcap) return true;
        fail(MT_DERR_TEXT_ARENA, seq);
        return false;
    }

    // ensureIntervalBoundary(pos) (mergeTree.ts:2241-2245): split the segment visible to
    // (R, C) that strictly contains pos.  Keeps cum[] valid for the same view.
    MT_DEV bool boundary(int pos, int32_t R, int C, int32_t seq) {
        const int n = s.n;
        int k = -1;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            const bool hit = i < n && cstart(i) < pos && pos < s.cum[i];
            const uint64_t m = wave_ballot(hit);
            if (m) {
                k = base + first_lane(m);
                break;
            }
        }
        if (k < 0) return true;
        const int sl = s.order[k];
        const int off = pos - cstart(k);
        const int t = alloc_slot(seq);
        if (t < 0) return false;
        block_starts();
        const int b = block_of_pos(k);
        // BaseSegment.splitAt + TextSegment.createSplitSegmentAt (mergeTree.ts:524-568)
        if (lane == 0) {
            s.seq[t] = s.seq[sl];
            s.client[t] = s.client[sl];
            s.rseq[t] = s.rseq[sl];
            s.rclient[t] = s.rclient[sl];
            s.ovl[t] = s.ovl[sl];
            if constexpr (W)
                ovx_copy(t, sl);
            pcopy(t, sl);
            s.flags[t] = s.flags[sl];
            s.len[t] = s.len[sl] - (uint32_t)off;
            s.toff[t] = s.toff[sl] + (uint32_t)off;
            s.len[sl] = (uint32_t)off;
            if constexpr (LOC) {  // segmentGroups.copyTo + the property manager's counts (mergeTree.ts:555-560)
                gm_copy(t, sl);
                pkp[t] = pkp[sl];
                lsqp[t] = lsqp[sl];
                s.lc.stamp = s.lc.stamp + 1;  // stamps start at 1: segments from before editing have 0
                ctp[t] = s.lc.stamp;
                ct_publish();
            }
            const TC last = arena[s.toff[sl] + (uint32_t)off - 1];
            s.flags[sl] = (uint8_t)((s.flags[sl] & ~MT_SF_NL) | (last == '\n' ? MT_SF_NL : 0));
        }
        const int old_end = s.cum[k];
        sync();
        if (lane == 0) s.cum[k] = pos;
        sync();
        // MergeTreeMaintenanceType.SPLIT (mergeTree.ts:2231-2236): [segment, next-to-be-linked]
        emit(MT_EV_SPLIT, MT_EVF_FIRST, k, -1, (uint32_t)off);
        emit(MT_EV_SPLIT, 0, k + 1, -1, s.len[t]);
        const int bs = s.bst[b], bc = s.lbcnt[b];
        if (!insert_at(k + 1, b, t, old_end, seq)) return false;
        refresh(bs, bs + bc + 1);  // insertingWalk: blockUpdateLength of the split's block (or both halves)
        return true;
    }

    // ------------------------------------------------------------------- heap
    // Heap<LRUSegment> (collections.ts:213-265), comparer maxSeq (mergeTree.ts:923-926)
    MT_DEV bool heap_push(int32_t key, int sl, int32_t seq) {
        if (s.heap_n + 1 >= L::H) return fail(MT_DERR_CAPACITY, seq), false;
        if (lane == 0) {
            int k = s.heap_n + 1;
            s.hseq[k] = key;
            s.hslot[k] = (uint16_t)sl;
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
        const int hn = s.heap_n + 1;
        sync();
        s.heap_n = hn;
        sync();
        return true;
    }
    MT_DEV int heap_pop() {
        int sl = 0;
        if (lane == 0) {
            sl = s.hslot[1];
            const int cnt = s.heap_n - 1;
            s.hseq[1] = s.hseq[s.heap_n];
            s.hslot[1] = s.hslot[s.heap_n];
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
        sl = wave_bcast(sl, 0);
        sync();
        s.heap_n = s.heap_n - 1;
        sync();
        return sl;
    }

    // addToLRUSet (mergeTree.ts:1273-1283) for a segment in leaf block b
    MT_DEV bool add_lru(int b, int sl, int32_t seq) {
        if (s.lbscour[b] != MT_SC_TRUE && seq > s.cur_seq) {
            sync();
            if (lane == 0) s.lbscour[b] = MT_SC_TRUE;
            sync();
            return heap_push(seq, sl, seq);
        }
        return true;
    }

    // ---------------------------------------------------------------- zamboni
    MT_DEV bool props_match(int a, int b) const {  // matchProperties, properties.ts:62-93
        return ((s.flags[a] ^ s.flags[b]) & MT_SF_PDEF) == 0 && peq(a, b);
    }

    // scourNode on leaf block b (mergeTree.ts:1289-1365).  Unlinks removed segments at or
    // below minSeq, appends acked segments into their predecessor, compacts the order array.
    // Returns the block's new child count.  Two passes: the decisions first, child by child on
    // scalars (the run's grown length and trailing newline are tracked, no text moves), then the
    // appends, unlinks and callbacks in child order -- the text copies run with little else live
    // (inlined into the decision loop, they set the editing form's register peak)
    MT_DEV int scour(int b) {
        const int st = s.bst[b];
        const int cnt = s.lbcnt[b];
        const int32_t minSeq = s.min_seq;
        uint32_t unl = 0, app = 0;  // children unlinked / appended to the run before them (bit q)
        // (LOC) the children with a pending group (segmentGroups not empty: held, mergeTree.ts:1295),
        // one lane per child: the masks may live in HBM
        uint32_t pendm = 0;
        if constexpr (LOC) pendm = (uint32_t)wave_ballot(lane < cnt && gm_any(s.order[st + lane]));
        int prev = -1;              // the run's head
        uint32_t plen = 0;          // its length with the appends so far
        bool pnl = false;           // its ENDS_WITH_NEWLINE after them
        for (int q = 0; q < cnt; q++) {
            const int sl = s.order[st + q];
            const uint8_t f = s.flags[sl];
            if ((pendm >> q) & 1u) {
                prev = -1;
            } else if (f & MT_SF_REMOVED) {
                if (!(s.rseq[sl] > minSeq)) unl |= 1u << q;
                prev = -1;
            } else if (s.seq[sl] <= minSeq) {
                const uint32_t ql = s.len[sl];
                // TextSegment.canAppend: two text segments (a Marker never appends, nor is appended
                // to: Marker.canAppend, TextSegment.is, mergeTree.ts:793; textSegment.ts:63-68)
                const bool a = prev >= 0 && !((s.flags[prev] | f) & MT_SF_MARKER) && !pnl &&
                               (plen <= (uint32_t)kTextGranularity || ql <= (uint32_t)kTextGranularity) &&
                               props_match(prev, sl) && ql > 0;
                if (a) {
                    app |= 1u << q;
                    plen += ql;
                } else {
                    prev = ql > 0 ? sl : -1;
                    plen = ql;
                }
                pnl = (f & MT_SF_NL) != 0;
            } else {
                prev = -1;
            }
        }
        if (!(unl | app)) return cnt;
        int kept = 0, hd = -1;  // children kept so far; the last of them (an append's head)
        for (int q = 0; q < cnt; q++) {
            const int sl = s.order[st + q];
            if ((unl >> q) & 1u) {
                emit(MT_EV_UNLINK, MT_EVF_FIRST, st + kept, -1, s.len[sl]);  // mergeTree.ts:1310-1315
                free_slot(sl);  // UNLINK
            } else if ((app >> q) & 1u) {
                append_text(hd, sl);
                emit(MT_EV_APPEND, MT_EVF_FIRST, st + kept - 1, -1, s.len[hd]);  // mergeTree.ts:1335-1340
                emit(MT_EV_APPEND, 0, st + kept, -1, s.len[sl]);
                free_slot(sl);  // APPEND: segment.parent = undefined
            } else {
                hd = sl;
                kept++;
            }
        }
        // the kept children close ranks (lane q: child q)
        const uint32_t keepm = ((1u << cnt) - 1u) & ~(unl | app);
        const bool mine = lane < cnt && ((keepm >> lane) & 1u);
        const uint16_t v = mine ? s.order[st + lane] : (uint16_t)0;
        sync();
        if (mine) s.order[st + __popc(keepm & ((1u << lane) - 1u))] = v;
        sync();
        shift_left(s.order, st + cnt, s.n, cnt - kept);
        s.n = s.n - (cnt - kept);
        sync();
        if (lane == 0) s.lbcnt[b] = (uint8_t)kept;
        // later block starts move left
        const int nb = s.nb[0];
        for (int base = b + 1; base <= nb; base += 64) {
            const int j = base + lane;
            if (j <= nb) s.bst[j] -= (cnt - kept);
        }
        sync();
        return kept;
    }

    // TextSegment.append (textSegment.ts:76-85): prev.text += seg.text
    MT_DEV void append_text(int prev, int sl) {
        if (s.toff[prev] + s.len[prev] != s.toff[sl] && s.toff[prev] + s.len[prev] != s.text_top) {
            if (!arena_reserve(s.len[prev] + s.len[sl], s.cur_seq)) return;
        } else if (s.toff[prev] + s.len[prev] != s.toff[sl]) {
            if (!arena_reserve(s.len[sl], s.cur_seq)) return;
        }
        const uint32_t pt = s.toff[prev], pl = s.len[prev], qt = s.toff[sl], ql = s.len[sl];
        uint32_t top = s.text_top;
        if (pt + pl == qt) {
            // views are adjacent in the arena: nothing to copy
        } else if (pt + pl == top) {
            arena_copy(top, qt, ql);
            top += ql;
        } else {
            arena_copy(top, pt, pl);
            arena_copy(top + pl, qt, ql);
            if (lane == 0) s.toff[prev] = top;
            top += pl + ql;
        }
        sync();
        if (lane == 0) {
            s.len[prev] = pl + ql;
            s.flags[prev] = (uint8_t)((s.flags[prev] & ~MT_SF_NL) | (s.flags[sl] & (MT_SF_NL | MT_SF_HASNL)));
        }
        s.text_top = top;
        sync();
    }

    // pack (mergeTree.ts:1368-1420): repack the children of block P at level L+1, recursing up
    MT_DEV void pack(int L, int P, int first_child) {
        for (;;) {
            const int m = lvl(L + 1)[P];
            int total = 0;
            if (L == 0) {
                for (int j = first_child; j < first_child + m; j++) total += scour(j);
            } else {
                const uint8_t* c = lvl(L);
                for (int j = first_child; j < first_child + m; j++) total += c[j];
            }
            const int half = kMaxNodes / 2;
            int cc = min(kMaxNodes - 1, total / half);
            if (cc < 1) cc = 1;
            const int base = total / cc, extra = total % cc;
            uint8_t* a = lvl(L);
            const int nb = s.nb[L];
            sync();
            if (cc < m) {
                shift_left(a, first_child + m, nb, m - cc);
                if (L == 0) shift_left(s.lbscour, first_child + m, nb, m - cc);
            } else if (cc > m) {
                for (int q = 0; q < cc - m; q++) {
                    shift_right(a, first_child + m, nb + q);
                    if (L == 0) shift_right(s.lbscour, first_child + m, nb + q);
                }
            }
            if (lane < cc) {
                a[first_child + lane] = (uint8_t)(base + (lane < extra ? 1 : 0));
                if (L == 0) s.lbscour[first_child + lane] = MT_SC_UNDEF;
            }
            s.nb[L] = nb + cc - m;
            sync();
            if (lane == 0) lvl(L + 1)[P] = (uint8_t)cc;
            sync();
            if (L == 0) {
                block_starts();
                refresh(s.bst[first_child], s.bst[first_child + cc]);  // every packed block is new
            }
            // underflow(parent) && parent.parent
            if (cc < kMaxNodes / 2 && (L + 1) < s.nlev - 1) {
                int fc = 0;
                const int PP = parent_of(L + 1, P, &fc);
                L = L + 1;
                P = PP;
                first_child = fc;
                continue;
            }
            return;
        }
    }

    // find the current position of slot sl (segment identity of a heap entry)
    MT_DEV int pos_of_slot(int sl) {
        const int n = s.n;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            const uint64_t m = wave_ballot(i < n && s.order[i] == sl);
            if (m) return base + first_lane(m);
        }
        return -1;
    }

    // zamboniSegments (mergeTree.ts:1422-1478), zamboniSegmentsMaxCount = 2
    MT_DEV void zamboni() {
        for (int it = 0; it < 2; it++) {
            if (s.heap_n == 0 || s.hseq[1] > s.min_seq) break;
            sync();
            const int sl = heap_pop();
            if (sl == (int)MT_DEAD_SLOT) continue;
            const int k = pos_of_slot(sl);
            if (k < 0) continue;
            block_starts();
            const int b = block_of_pos(k);
            if (s.lbscour[b] == MT_SC_FALSE) continue;
            const int cnt = s.lbcnt[b];
            const int kept = scour(b);
            sync();
            if (lane == 0) s.lbscour[b] = MT_SC_FALSE;
            sync();
            if (kept < cnt && kept < kMaxNodes / 2 && s.nlev > 1) {
                int fc = 0;
                const int P = parent_of(0, b, &fc);
                pack(0, P, fc);
            } else if (kept < cnt) {
                refresh(s.bst[b], s.bst[b] + kept);  // blockUpdatePathLengths(block)
            }
            if (s.err) return;
        }
    }

    // -------------------------------------------------------------------- ops
    MT_DEV void op_insert(const mt_op_rec& op, const uint8_t* pay, int tlen, const Pairs& pr) {
        const int32_t S = op.seq, R = op.ref_seq;
        const bool ld = MT_OP_TYPE(op) == MT_OP_LOAD;
        const int C = ld ? (int)MT_LOAD_CLIENT(op) : (int)op.client, pos = op.pos1;
        if (!boundary(pos, R, C, S)) return;  // cum: apply() scanned for (R, C)
        if (tlen > 0) {  // blockInsert (mergeTree.ts:2141-2224)
            block_starts();
            const int nb = s.nb[0];
            // first leaf block whose cumulative visible end >= pos (insertingWalk descent)
            int b = -1;
            for (int base = 0; base < nb; base += 64) {
                const int j = base + lane;
                bool hit = false;
                if (j < nb) {
                    const int st = s.bst[j], c = s.lbcnt[j];
                    const int bend = c > 0 ? s.cum[st + c - 1] : cstart(st);
                    hit = bend >= pos;
                }
                const uint64_t m = wave_ballot(hit);
                if (m) {
                    b = base + first_lane(m);
                    break;
                }
            }
            if (b < 0) return fail(MT_DERR_INSERT_FAILED, S);
            int st = s.bst[b], c = s.lbcnt[b];
            uint64_t m;
            for (;;) {
                // leaf placement: first child with pos < len, or pos == len == 0 and breakTie
                bool hit = false;
                if (lane < c) {
                    const int k = st + lane;
                    const int ce = s.cum[k], cs = cstart(k);
                    const int sl = s.order[k];
                    bool rm_before = (s.flags[sl] & MT_SF_REMOVED) && s.rseq[sl] <= R;
                    bool tie = true;
                    if constexpr (LOC) {  // breakTie (mergeTree.ts:2248-2277) with pending segments
                        rm_before = rm_before && s.rseq[sl] != -1;
                        tie = C == s.lc.own || s.seq[sl] != -1;
                    }
                    hit = ce > pos || (ce == pos && cs == pos && !rm_before && tie);
                }
                m = wave_ballot(hit);
                if constexpr (LOC) {
                    // blockInsert's continuePredicate (mergeTree.ts:2143-2160, 2431-2436): a sequenced
                    // insert that runs off block b goes on into the next block when the first leaf
                    // after b in the local view is a pending local insert
                    if (!m && S != -1 && b + 1 < nb) {
                        const int e0 = st + c, n = s.n;
                        int f = -1;
                        for (int base = e0; base < n && f < 0; base += 64) {
                            const int k = base + lane;
                            const bool lv = k < n && !(s.flags[s.order[k]] & MT_SF_REMOVED) && s.len[s.order[k]] > 0;
                            const uint64_t lm = wave_ballot(lv);
                            if (lm) f = base + first_lane(lm);
                        }
                        if (f >= 0 && s.seq[s.order[f]] == -1) {
                            b = b + 1;
                            st = s.bst[b];
                            c = s.lbcnt[b];
                            continue;
                        }
                    }
                }
                break;
            }
            // not found: append at the end of block b (pos_rem == 0 there, mergeTree.ts:2431-2444)
            const int k = m ? st + first_lane(m) : st + c;
            const int t = alloc_slot(S);
            if (t < 0) return;
            if (!arena_reserve((uint32_t)tlen, S)) return;
            const uint32_t top = s.text_top;
            bool hasnl = false;
            const bool wop = (op.type & MT_OP_WIDE) != 0;  // the payload text is UTF-16 code units
            auto unit = [&](int i) -> uint32_t {
                return wop ? (uint32_t)pay[2 * i] | ((uint32_t)pay[2 * i + 1] << 8) : (uint32_t)pay[i];
            };
            for (int base = 0; base < tlen; base += 64) {
                const int i = base + lane;
                uint32_t c = 0;
                if (i < tlen) {
                    c = unit(i);
                    arena[top + i] = (TC)c;
                }
                hasnl = hasnl || wave_ballot(i < tlen && c == '\n') != 0;
            }
            __threadfence_block();
            if (lane == 0) {
                // a snapshot body segment may arrive removed (SnapshotLoader.specToSegment,
                // snapshotLoader.ts:101-106): MT_OP_LOAD carries removedSeq in pos2
                const bool lrm = MT_OP_TYPE(op) == MT_OP_LOAD && op.pos2 >= 0;
                s.seq[t] = S;
                s.client[t] = (CT)C;
                s.rseq[t] = lrm ? op.pos2 : 0;
                s.rclient[t] = lrm ? (CT)MT_LOAD_RCLIENT(op) : 0;
                s.ovl[t] = 0;
                if constexpr (W)
                    ovx_zero(t);
                s.len[t] = (uint32_t)tlen;
                s.toff[t] = top;
                // a Marker (MT_F_MARKER): length 1, its arena byte is its ReferenceType
                uint8_t f = (op.flags & MT_F_MARKER) ? MT_SF_MARKER
                                                     : ((unit(tlen - 1) == '\n' ? MT_SF_NL : 0) | (hasnl ? MT_SF_HASNL : 0));
                f |= lrm ? MT_SF_REMOVED : 0;
                pclear(t);
                if (op.flags & MT_F_PROPS) {  // TextSegment.make -> addProperties
                    f |= MT_SF_PDEF;
                    papply(t, pr);
                }
                s.flags[t] = f;
                if constexpr (LOC) {  // a local insert is its edit's one pending segment (saveIfLocal)
                    gm_zero(t);
                    if (S == -1) gm_set(t, s.lc.ghi);
                    pkp[t] = 0;
                    lsqp[t] = S == -1 ? (uint64_t)s.lc.lseq : 0ull;
                    s.lc.stamp = s.lc.stamp + 1;
                    const uint32_t stamp = s.lc.stamp;
                    ctp[t] = stamp;
                    ct_publish();
                    if (S == -1) {
                        gtp[s.lc.ghi % GN] = stamp;
                        glsp[s.lc.ghi % GN] = s.lc.lseq;
                        ct_publish();
                        s.lc.ghi = s.lc.ghi + 1;
                    }
                }
            }
            s.text_top = top + (uint32_t)tlen;
            sync();
            const int idx = k - st;  // index inside block b before a possible split
            const int before_nb = s.nb[0];
            if (!insert_at(k, b, t, -1, S)) return;
            refresh(st, st + c + 1);  // insertingWalk: blockUpdateLength of the insert's block (or both halves)
            const int bb = (s.nb[0] > before_nb && idx >= kMaxNodes / 2) ? b + 1 : b;
            if (S > s.min_seq) {  // saveIfLocal -> addToLRUSet (mergeTree.ts:2164-2179)
                if (!add_lru(bb, t, S)) return;
            }
            // MergeTreeDeltaType.INSERT (mergeTree.ts:1981-1988); a snapshot body append has no opArgs
            if (ev && MT_OP_TYPE(op) != MT_OP_LOAD) emit(MT_EV_INSERT, MT_EVF_FIRST, k, local_prefix(k), (uint32_t)tlen);
        } else if (MT_OP_TYPE(op) != MT_OP_LOAD) {
            emit(MT_EV_INSERT, MT_EVF_FIRST, -1, -1, 0);  // an empty text with props: never linked
        }
        if (S != -1) zamboni();  // (a local edit runs no zamboni, mergeTree.ts:1994-1997)
    }

    MT_DEV void op_range(const mt_op_rec& op, const Pairs& pr) {
        const int32_t S = op.seq, R = op.ref_seq;
        const int C = op.client, start = op.pos1, end = op.pos2;
        const bool is_remove = MT_OP_TYPE(op) == MT_OP_REMOVE;
        if (!boundary(start, R, C, S)) return;  // cum: apply() scanned for (R, C)
        if (!boundary(end, R, C, S)) return;
        // markRangeRemoved / annotateRange leaf actions over mapRange (mergeTree.ts:2903-2965)
        const int n = s.n;
        const bool rewrite = op.flags & MT_F_REWRITE;
        const bool local = S == -1;
        uint32_t gN = 0;
        if constexpr (LOC) {
            if (local) {  // this edit's pending group (addToPendingList, mergeTree.ts:1922-1929)
                gN = s.lc.ghi;
                sync();
                if (lane == 0) {
                    gtp[gN % GN] = s.lc.stamp + 1;  // every member existed before it
                    glsp[gN % GN] = s.lc.lseq;
                }
                ct_publish();
                sync();
                s.lc.ghi = s.lc.ghi + 1;
                sync();
            }
        }
        if (!is_remove) emit_range(false, S, C, start, end, pr, rewrite);
        bool over = false;  // (a wide segment's overlap list full)
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            if (i < n) {
                const int ce = s.cum[i], cs = cstart(i);
                if (ce > cs && cs < end && ce > start) {
                    const int sl = s.order[i];
                    if constexpr (LOC) {
                        if (local) gm_set(sl, gN);
                    }
                    if (!is_remove && track()) mark_stale(sl);
                    if (LOC && !is_remove) {
                        annotate_loc(sl, pr.p, pr.np, rewrite, local);
                    } else if (is_remove) {
                        bool pend_rm = false;
                        if constexpr (LOC) pend_rm = (s.flags[sl] & MT_SF_REMOVED) && s.rseq[sl] == -1;
                        if (pend_rm) {  // a pending local removal: this one replaces it (mergeTree.ts:2621-2627)
                            s.rseq[sl] = S;
                            s.rclient[sl] = (CT)C;
                            s.flags[sl] |= MT_SF_OVW;  // (not among this op's removedSegments)
                            if constexpr (LOC) lsqp[sl] &= 0xFFFFFFFFull;  // localRemovedSeq = undefined
                        } else if (s.flags[sl] & MT_SF_REMOVED) {
                            over = !ovl_add(sl, C) || over;  // addOverlappingClient (first remover wins)
                        } else {
                            s.flags[sl] |= MT_SF_REMOVED;
                            s.rseq[sl] = S;
                            s.rclient[sl] = (CT)C;
                            if constexpr (LOC) {  // localRemovedSeq (mergeTree.ts:2637)
                                lsqp[sl] = (lsqp[sl] & 0xFFFFFFFFull) | ((uint64_t)(local ? s.lc.lseq : 0u) << 32);
                            }
                        }
                    } else {  // SegmentPropertiesManager.addProperties (remote, no combining op)
                        if (rewrite || !(s.flags[sl] & MT_SF_PDEF)) pclear(sl);
                        papply(sl, pr);
                        s.flags[sl] |= MT_SF_PDEF;
                    }
                }
            }
        }
        if (wave_ballot(over)) return fail(MT_DERR_LIMITS, S);
        if constexpr (LOC) ct_publish();  // (the localRemovedSeq writes, read by other lanes later)
        sync();
        if (is_remove && track()) {  // markRangeRemoved's post action: blockUpdate of every block mapRange enters
            block_starts();
            const int nb = s.nb[0];
            for (int base = 0; base < nb; base += 64) {
                const int j = base + lane;
                if (j < nb) {
                    const int st = s.bst[j], c = s.lbcnt[j];
                    bool any = false;
                    for (int q = 0; q < c; q++) {
                        const int ce = s.cum[st + q], cs = cstart(st + q);
                        any = any || (ce > cs && cs < end && ce > start);
                    }
                    if (any)
                        for (int q = 0; q < c; q++) s.flags[s.order[st + q]] &= (uint8_t)~MT_SF_STALE;
                }
            }
            sync();
        }
        if (is_remove) emit_range(true, S, C, start, end, pr, rewrite);
        if constexpr (LOC) {
            if (is_remove) {
                for (int i = lane; i < n; i += 64) s.flags[s.order[i]] &= (uint8_t)~MT_SF_OVW;
                sync();
            }
        }
        if (local) return;  // pending segments join no LRU set and a local edit runs no zamboni
        // addToLRUSet for touched segments in document order: one heap push per leaf block
        // whose needsScour is not already true, for its first touched segment
        block_starts();
        const int nb = s.nb[0];
        for (int base = 0; base < nb; base += 64) {
            const int j = base + lane;
            int first = -1;
            if (j < nb) {
                const int st = s.bst[j], c = s.lbcnt[j];
                for (int q = 0; q < c; q++) {
                    const int k = st + q;
                    const int ce = s.cum[k], cs = cstart(k);
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
                const int k = wave_bcast(first, fl);
                if (!add_lru(base + fl, s.order[k], S)) return;
            }
        }
        zamboni();
    }

    // SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111) for an editing
    // client's document: a local change counts its keys pending (and a rewrite), a remote one skips
    // keys with pending local changes and is dropped whole while a local rewrite is pending
    MT_DEV void annotate_loc(int sl, const uint8_t* pairs, int np, bool rewrite, bool local) {
        if constexpr (LOC) {
            uint64_t p = (s.flags[sl] & MT_SF_PDEF) ? s.props[sl] : 0;
            uint64_t pk = (s.flags[sl] & MT_SF_PDEF) ? pkp[sl] : 0;
            s.flags[sl] |= MT_SF_PDEF;
            if (!local && MT_PK_RW(pk) > 0) {
                s.props[sl] = p;
                pkp[sl] = pk;
                return;
            }
            if (rewrite) {
                if (local) pk += 1ull << 56;
                for (int k = 0; k < 8; k++) {
                    bool keep = false;  // newProps[key] truthy
                    for (int q = 0; q < np; q++) keep = keep || (pairs[2 * q] == k && pairs[2 * q + 1] != 0);
                    if (((p >> (8 * k)) & 0xFFu) && !keep && (local || MT_PK_KEY(pk, k) == 0)) p &= ~(0xFFull << (8 * k));
                }
            }
            for (int q = 0; q < np; q++) {
                const int k = pairs[2 * q];
                if (local) {
                    if (MT_PK_KEY(pk, k) < 127) pk += 1ull << (7 * k);
                } else if (MT_PK_KEY(pk, k) > 0) {
                    continue;
                }
                p = (p & ~(0xFFull << (8 * k))) | ((uint64_t)pairs[2 * q + 1] << (8 * k));
            }
            s.props[sl] = p;
            pkp[sl] = pk;
        }
    }

    // ackPendingSegment (client.ts:588-625 -> mergeTree.ts:1893-1920, BaseSegment.ack :487-522): the
    // editing client's own sequenced message settles its oldest pending edit.  Its group's list
    // order (which the heap pushes follow) is rebuilt: the members that existed when the edit was
    // made (stamp < gt) in document order, then the parts split off later, by stamp.
    MT_DEV void ack_one(int k, int32_t S, uint32_t N, uint8_t type, const uint8_t* pairs, int np, bool rewrite) {
        if constexpr (LOC) {
            const int sl = s.order[k];
            sync();
            if (lane == 0) {
                gm_clr(sl, N);
                if (type == MT_OP_INSERT) {
                    s.seq[sl] = S;
                    lsqp[sl] &= ~0xFFFFFFFFull;
                } else if (type == MT_OP_REMOVE) {
                    lsqp[sl] &= 0xFFFFFFFFull;
                    if (s.rseq[sl] == -1) s.rseq[sl] = S;  // else a remote removal overwrote it
                } else {  // ackPendingProperties (segmentPropertiesManager.ts:15-28)
                    uint64_t pk = pkp[sl];
                    if (rewrite && MT_PK_RW(pk) > 0) pk -= 1ull << 56;
                    for (int q = 0; q < np; q++)
                        if (MT_PK_KEY(pk, pairs[2 * q]) > 0) pk -= 1ull << (7 * pairs[2 * q]);
                    pkp[sl] = pk;
                }
            }
            ct_publish();
            sync();
            const int b = block_of_pos(k);
            add_lru(b, sl, S);
            refresh(s.bst[b], s.bst[b] + s.lbcnt[b]);  // ackPendingSegment: blockUpdatePathLengths(parent)
        }
    }
    MT_DEV void op_ack(const mt_op_rec& op, const uint8_t* pairs, int np) {
        if constexpr (LOC) {
            const int32_t S = op.seq;
            if (s.lc.glo < s.lc.ghi) {
                const uint32_t Lo = s.lc.glo;
                const uint32_t gt = gtp[Lo % GN];
                const bool rewrite = op.flags & MT_F_REWRITE;
                block_starts();
                const int n = s.n;
                for (int base = 0; base < n; base += 64) {  // the original members, in document order
                    const int i = base + lane;
                    bool mem = false;
                    if (i < n) {
                        const int sl = s.order[i];
                        mem = gm_has(sl, Lo) && ctp[sl] < gt;
                    }
                    uint64_t m = wave_ballot(mem);
                    while (m) {
                        const int fl = first_lane(m);
                        m &= m - 1;
                        ack_one(base + fl, S, Lo, op.type, pairs, np, rewrite);
                        if (s.err) return;
                    }
                }
                for (;;) {  // the parts split off later, by creation stamp
                    uint32_t best = 0xFFFFFFFFu;
                    for (int base = 0; base < n; base += 64) {
                        const int i = base + lane;
                        uint32_t v = 0xFFFFFFFFu;
                        if (i < n) {
                            const int sl = s.order[i];
                            if (gm_has(sl, Lo)) v = ctp[sl];
                        }
                        uint32_t mv = v;
                        for (int o = 32; o; o >>= 1) mv = min(mv, (uint32_t)__shfl_xor((int)mv, o, 64));
                        best = min(best, mv);
                    }
                    if (best == 0xFFFFFFFFu) break;
                    int k = -1;
                    for (int base = 0; base < n && k < 0; base += 64) {
                        const int i = base + lane;
                        const uint64_t hm = wave_ballot(i < n && gm_has(s.order[i], Lo) && ctp[s.order[i]] == best);
                        if (hm) k = base + first_lane(hm);
                    }
                    if (k < 0) break;
                    ack_one(k, S, Lo, op.type, pairs, np, rewrite);
                    if (s.err) return;
                }
                sync();
                s.lc.glo = Lo + 1;
                sync();
            }
            zamboni();
        }
    }

    // Client.regeneratePendingOp -> resetPendingDeltaToOps (client.ts:708-766, 855-893) for the
    // oldest pending edit, whose op is `op`: its segments in document order, each at its
    // findReconnectionPostition (:674-706: the segments before it inserted and not removed as of the
    // edit's localSeq), become one new op each (a removal only while still locally removed), each
    // with a new pending group of the same localSeq at the queue's tail.  The new ops go to the
    // document's regenerated-op buffer after a header record (type MT_OP_NOOP) carrying rix.
    MT_DEV void op_regen(const mt_op_rec& op, const uint8_t* payload) {
        if constexpr (LOC) {
            const int32_t S = MT_SEQ_REGEN;
            if (s.lc.own < 0 || (int)op.client != s.lc.own || op.type > MT_OP_ANNOTATE) return fail(MT_DERR_BAD_OP, S);
            if (s.lc.glo == s.lc.ghi) return fail(MT_DERR_BAD_OP, S);
            const int np = MT_OP_NPAIRS(op);
            const uint8_t* opairs = payload + op.payload_off + (op.payload_len - 2 * np);
            const uint32_t Lo = s.lc.glo;
            const uint32_t Ls = glsp[Lo % GN];
            auto emit_rec = [&](const mt_op_rec& r) -> bool {
                if (s.lc.rgn >= MT_RG_RECS || s.lc.rgpn + r.payload_len > MT_RG_BYTES) return fail(MT_DERR_CAPACITY, S), false;
                if (lane == 0) rg[s.lc.rgn] = r;
                sync();
                s.lc.rgn = s.lc.rgn + 1;
                s.lc.rgpn = s.lc.rgpn + r.payload_len;
                sync();
                return true;
            };
            mt_op_rec h{};
            h.seq = (int32_t)rix;
            h.type = MT_OP_NOOP;
            if (!emit_rec(h)) return;
            const int n = s.n;
            for (int base = 0; base < n; base += 64) {
                const int i = base + lane;
                const bool mem = i < n && gm_has(s.order[i], Lo);
                uint64_t m = wave_ballot(mem);
                while (m) {
                    const int k = base + first_lane(m);
                    m &= m - 1;
                    const int sl = s.order[k];
                    int pos = 0;  // findReconnectionPostition
                    for (int b2 = 0; b2 < k; b2 += 64) {
                        const int j = b2 + lane;
                        int v = 0;
                        if (j < k) {
                            const int sj = s.order[j];
                            const uint32_t lo = (uint32_t)lsqp[sj], hi = (uint32_t)(lsqp[sj] >> 32);
                            if ((lo == 0 || lo <= Ls) && (!(s.flags[sj] & MT_SF_REMOVED) || (hi != 0 && hi > Ls))) v = (int)s.len[sj];
                        }
                        pos += wave_sum(v);
                    }
                    sync();
                    if (lane == 0) gm_clr(sl, Lo);
                    ct_publish();
                    sync();
                    const uint32_t len = s.len[sl];
                    mt_op_rec r{};
                    r.seq = (int32_t)rix;
                    r.type = op.type;
                    r.client = (uint16_t)s.lc.own;
                    r.pos1 = pos;
                    r.pos2 = op.type == MT_OP_INSERT ? 0 : pos + (int32_t)len;
                    r.payload_off = s.lc.rgpn;
                    bool keep = true;
                    uint8_t kv[16];
                    int nkv = 0;
                    if (op.type == MT_OP_INSERT) {  // the segment's spec: its text (or refType) and props
                        const uint8_t f = s.flags[sl];
                        r.flags = (f & MT_SF_MARKER) ? MT_F_MARKER : 0;
                        if (f & MT_SF_PDEF) {
                            r.flags |= MT_F_PROPS;
                            for (int q = 0; q < 8; q++) {
                                const uint8_t v = (uint8_t)(s.props[sl] >> (8 * q));
                                if (v) {
                                    kv[2 * nkv] = (uint8_t)q;
                                    kv[2 * nkv + 1] = v;
                                    nkv++;
                                }
                            }
                        }
                        r.payload_len = len + 2u * (uint32_t)nkv;
                    } else if (op.type == MT_OP_REMOVE) {
                        keep = (lsqp[sl] >> 32) != 0;  // still locally removed
                        r.payload_len = 0;
                    } else {
                        r.flags = op.flags & MT_F_REWRITE;
                        nkv = np < 8 ? np : 8;
                        for (int q = 0; q < 2 * nkv; q++) kv[q] = opairs[q];
                        r.payload_len = 2u * (uint32_t)nkv;
                    }
                    if (!keep) continue;
                    r.flags |= (uint8_t)(nkv << MT_F_NPAIRS_SHIFT);
                    if (s.lc.rgpn + r.payload_len > MT_RG_BYTES) return fail(MT_DERR_CAPACITY, S);
                    if (op.type == MT_OP_INSERT) {
                        for (uint32_t t = lane; t < len; t += 64) rgp[s.lc.rgpn + t] = arena[s.toff[sl] + t];
                    }
                    if (lane == 0)
                        for (int q = 0; q < 2 * nkv; q++) rgp[s.lc.rgpn + (op.type == MT_OP_INSERT ? len : 0) + q] = kv[q];
                    if (!emit_rec(r)) return;
                    // its own pending group, same localSeq, at the queue's tail
                    if (s.lc.ghi - s.lc.glo >= GN) return fail(MT_DERR_CAPACITY, S);
                    sync();
                    if (lane == 0) {
                        const uint32_t N = s.lc.ghi;
                        gm_set(sl, N);
                        glsp[N % GN] = Ls;
                        gtp[N % GN] = ctp[sl];
                    }
                    ct_publish();
                    sync();
                    s.lc.ghi = s.lc.ghi + 1;
                    sync();
                }
            }
            sync();
            s.lc.glo = Lo + 1;
            sync();
        }
    }

    // Client.updateSeqNumbers + MergeTree.setMinSeq (client.ts:821-828, mergeTree.ts:1718-1736)
    MT_DEV void update_seq(int32_t msn, int32_t seq) {
        if (!(s.cur_seq <= seq)) return fail(MT_DERR_SEQ_ORDER, seq);
        sync();
        s.cur_seq = seq;
        sync();
        if (!(msn <= seq) || !(s.min_seq <= msn)) return fail(MT_DERR_MSN_ORDER, seq);
        if (msn > s.min_seq) {
            sync();
            s.min_seq = msn;
            sync();
            zamboni();
        }
    }

    // A local edit of the editing client (client.ts:163-214 -> applyInsertOp / applyRemoveRangeOp /
    // applyAnnotateRangeOp): refSeq = currentSeq, seq = UnassignedSequenceNumber, the local view; no
    // window asserts, no seq update.  The first one names the document's editing client.
    MT_DEV void apply_local(const mt_op_rec& op, const uint8_t* payload) {
        const int np = MT_OP_NPAIRS(op);
        const int C = op.client;
        if (s.lc.own < 0) {
            sync();
            s.lc.own = C;
            sync();
        }
        // (the editing client may be short id 0, the reference's own id, client.ts:1057-1062; its
        // document stays narrow: the editing form has no wide state)
        if (C != s.lc.own || C >= MT_MAX_CLIENTS || (op.type & MT_OP_WIDE)) return fail(MT_DERR_LIMITS, -1);
        if (op.payload_len < (uint32_t)(2 * np) || !MT_OP_NO_TEXT_OK(op)) return fail(MT_DERR_BAD_OP, -1);
        if (s.lc.ghi - s.lc.glo >= GN) return fail(MT_DERR_CAPACITY, -1);
        const uint8_t* pay = payload + op.payload_off;
        const int tlen = (int)op.payload_len - 2 * np;
        const Pairs pr{pay + tlen, np, false};
        for (int q = 0; q < np; q++)
            if (pr.key(q) >= MT_MAX_KEYS) return fail(MT_DERR_LIMITS, -1);
        mt_op_rec o = op;
        o.ref_seq = s.cur_seq;
        s.evseq = -1;  // (a local edit's callbacks: seq -1)
        const int L = scan(o.ref_seq, C);
        if (op.type == MT_OP_INSERT && tlen <= 0) return;  // insertSegmentLocal: nothing for an empty segment
        sync();
        s.lc.lseq = s.lc.lseq + 1;  // ++collabWindow.localSeq (mergeTree.ts:1976, 2571, 2613)
        sync();
        if (op.type == MT_OP_INSERT) {
            if (o.pos1 < 0 || o.pos1 > L) return fail(MT_DERR_INSERT_FAILED, -1);
            op_insert(o, pay, tlen, pr);
        } else {
            if (o.pos1 < 0 || o.pos2 > L || o.pos1 >= o.pos2) return fail(MT_DERR_BAD_OP, -1);  // getValidOpRange
            op_range(o, pr);
        }
        if (ev && s.evn > (int)evcap) fail(MT_DERR_EVENTS, -1);
    }
    MT_DEV void apply_ack(const mt_op_rec& op, const uint8_t* payload) {
        const int np = MT_OP_NPAIRS(op);
        const int32_t S = op.seq;
        s.evseq = S;
        if (!(s.cur_seq <= S)) return fail(MT_DERR_SEQ_ORDER, S);                                  // client.ts:824
        if (!(op.msn <= S) || !(s.min_seq <= op.msn)) return fail(MT_DERR_MSN_ORDER, S);           // :826
        if (op.type & MT_OP_WIDE) return fail(MT_DERR_LIMITS, S);
        if (op.payload_len < (uint32_t)(2 * np) || !MT_OP_NO_TEXT_OK(op)) return fail(MT_DERR_BAD_OP, S);
        op_ack(op, payload + op.payload_off + (op.payload_len - 2 * np), np);
        if (s.err) return;
        if (!(op.flags & MT_F_GROUP_MORE)) update_seq(op.msn, S);
        if (ev && s.evn > (int)evcap) fail(MT_DERR_EVENTS, S);
    }

    MT_DEV void apply(const mt_op_rec& op, const uint8_t* payload) {
        const int np = MT_OP_NPAIRS(op);
        const int32_t S = op.seq;
        const int type = MT_OP_TYPE(op);
        const bool wop = (op.type & MT_OP_WIDE) != 0;
        if constexpr (LOC) {
            if (S == MT_SEQ_REGEN) return op_regen(op, payload);
            if (type <= MT_OP_ANNOTATE && S == -1) return apply_local(op, payload);
            if (s.lc.own >= 0 && (int)op.client == s.lc.own && type <= MT_OP_ANNOTATE && !MT_OP_IS_NOOP(op))
                return apply_ack(op, payload);
        }
        if (type > MT_OP_LOAD) return fail(MT_DERR_BAD_OP, S);
        // (a wide op reaches only the wide form: mt_bin_kernel routes its document there)
        if (wop && !W) return fail(MT_DERR_LIMITS, S);
        constexpr int kClients = W ? MT_MAX_CLIENTS_WIDE : MT_MAX_CLIENTS;
        // MT_OP_LOAD: MergeTree.insertSegments from SnapshotLoader.loadBody (snapshotLoader.ts:192-224),
        // no Client around it: no window asserts and no updateSeqNumbers
        const bool load = type == MT_OP_LOAD;
        const bool noop = MT_OP_IS_NOOP(op);  // incl. an empty-string insert (client.ts:403-407)
        // (a short id >= 256 only in the wide form; 254 is NonCollabClient's, never a remote client's)
        const int C = load ? (int)MT_LOAD_CLIENT(op) : (int)op.client;
        const uint32_t plen = MT_OP_PAIRS_LEN(op);
        s.evseq = S;
        if (load) {
            const int RC = (int)MT_LOAD_RCLIENT(op);
            const bool ok = (C == MT_CLIENT_NONCOLLAB || (C >= 1 && C < kClients)) &&
                            (op.pos2 < 0 || (RC >= 1 && RC < kClients && RC != MT_CLIENT_NONCOLLAB));
            if (!ok) return fail(MT_DERR_LIMITS, S);
            if (op.payload_len < plen || (wop && ((op.payload_len - plen) & 1u))) return fail(MT_DERR_BAD_OP, S);
        } else if (!noop) {
            if (op.client == 0 || op.client >= kClients || op.client == MT_CLIENT_NONCOLLAB)
                return fail(MT_DERR_LIMITS, S);
            if (op.payload_len < plen || (wop && ((op.payload_len - plen) & 1u)) || !MT_OP_NO_TEXT_OK(op))
                return fail(MT_DERR_BAD_OP, S);
        } else {  // every assert of the message before any edit: the document halts before it
            if (!(s.cur_seq <= S)) return fail(MT_DERR_SEQ_ORDER, S);  // client.ts:824
            if (!(op.msn <= S) || !(s.min_seq <= op.msn)) return fail(MT_DERR_MSN_ORDER, S);  // :826, mergeTree.ts:1722
        }
        const uint8_t* pay = payload + op.payload_off;
        const int tlen = (int)((op.payload_len - plen) >> (wop ? 1 : 0));  // text code units
        const Pairs pr{pay + (op.payload_len - plen), np, wop};
        for (int q = 0; q < np; q++)
            if (pr.key(q) >= pr.key_limit() || (W && pr.key(q) >= 16 && !xk_p)) return fail(MT_DERR_LIMITS, S);
        if (!noop) {
            if (op.pos1 < 0 || (type != MT_OP_INSERT && !load && op.pos2 < 0)) return fail(MT_DERR_BAD_OP, S);
            const int L = scan(op.ref_seq, C);  // cum for the op's view (no edit yet)
            // the window asserts run after the op in the reference (completeAndLogOp, client.ts:461-464;
            // updateSeqNumbers :826), so a failing insert (mergeTree.ts:2210) is reported first; all of
            // them are decided here, before any edit: the document halts before the failing message
            int wc = 0;
            if (load) wc = 0;
            else if (!(s.cur_seq < S)) wc = MT_DERR_SEQ_ORDER;
            else if (!(s.min_seq <= op.msn) || !(op.msn <= S)) wc = MT_DERR_MSN_ORDER;
            if ((type == MT_OP_INSERT || load) && tlen > 0 && op.pos1 > L) wc = MT_DERR_INSERT_FAILED;
            if (wc) return fail(wc, S);
            if (type == MT_OP_INSERT || load) op_insert(op, pay, tlen, pr);
            else op_range(op, pr);
        }
        if (s.err) return;
        if (!load && !(op.flags & MT_F_GROUP_MORE)) update_seq(op.msn, S);
        if (ev && s.evn > (int)evcap) fail(MT_DERR_EVENTS, S);  // halt rather than drop callbacks
    }

    // ---------------------------------------------------------------- generator
    // Device form of mto_gen_op (mt_synth.h): synthesise op i of this document from the
    // observer state, write its record + payload, and return it.  Must match the host form
    // draw for draw (tests/test_gpu_parity.py compares the logs byte for byte).
    MT_DEV mt_op_rec gen_op(const mt_synth_cfg& cfg, uint64_t key, uint32_t i, uint8_t* pay, uint32_t pay_off,
                            uint32_t paycap) {
        const int32_t seq = s.cur_seq;
        const uint32_t C = cfg.n_clients;
        const int c = (int)mt_ru(key, i, MT_R_CLIENT, 1, C);
        const int32_t lag = (int32_t)mt_ru(key, i, MT_R_LAG, 0, cfg.max_lag);
        int32_t want = seq - lag > 0 ? seq - lag : 0;
        if (cfg.stall_ops && c == 1) {
            if (seq < s.gstall) {
                want = s.gcref[1];
            } else if (mt_ru(key, i, MT_R_STALL, 1, cfg.stall_ops) == 1) {
                sync();
                s.gstall = seq + (int32_t)cfg.stall_ops;
            }
        }
        int32_t R = s.gcref[c] > want ? s.gcref[c] : want;
        if (R > seq) R = seq;
        sync();
        if (lane == 0) s.gcref[c] = R;
        sync();
        const int32_t mine = (lane >= 1 && lane <= (int)C) ? s.gcref[lane] : 0x7fffffff;
        const int32_t msn = min(R, wave_min(mine));
        const int L = scan(R, c);
        const uint32_t rt = (uint32_t)mto_rng(key, i, MT_R_TYPE);
        const uint8_t type = (L == 0 || rt < cfg.p_insert) ? 0 : (rt - cfg.p_insert < cfg.p_remove ? 1 : 2);
        mt_op_rec rec{};
        rec.seq = seq + 1;
        rec.ref_seq = R;
        rec.msn = msn;
        rec.client = (uint16_t)c;
        rec.type = type;
        uint32_t n = 0, np = 0;
        uint8_t pr[4] = {0, 0, 0, 0};
        if (type == 0) {
            rec.pos1 = (int32_t)mt_ru(key, i, MT_R_POS1, 0, (uint32_t)L);
            const bool mk = mt_gen_is_marker(cfg, key, i);
            const uint32_t tl = mk ? 1u : mt_gen_text_len(key, i);
            if (pay_off + tl + 2 <= paycap) {
                if (mk) {
                    if (lane == 0) pay[0] = mt_gen_ref_type(key, i);
                } else {
                    for (uint32_t t = lane; t < tl; t += 64) pay[t] = mt_gen_char(key, i, t);
                }
            }
            if (mk) rec.flags |= MT_F_MARKER;
            n = tl;
            if (cfg.n_keys && mt_rp(key, i, MT_R_IPROPS, cfg.p_insert_props)) {
                rec.flags |= MT_F_PROPS;
                pr[0] = (uint8_t)mt_ru(key, i, MT_R_IKEY, 0, cfg.n_keys - 1);
                pr[1] = (uint8_t)mt_ru(key, i, MT_R_IVAL, 1, cfg.n_values);
                np = 1;
            }
        } else {
            int32_t a = (int32_t)mt_ru(key, i, MT_R_POS1, 0, (uint32_t)L - 1), b = 0;
            bool aimed = false;
            if (type == 1 && cfg.p_overlap && mt_rp(key, i, MT_R_AIM, cfg.p_overlap)) {
                // segments visible to (R, c) whose removal c has not seen: count, then pick one
                const int nn = s.n;
                uint32_t cnt = 0;
                for (int base = 0; base < nn; base += 64) {
                    const int k = base + lane;
                    bool hit = false;
                    if (k < nn) {
                        const int sl = s.order[k];
                        hit = s.cum[k] > cstart(k) && (s.flags[sl] & MT_SF_REMOVED) && s.rseq[sl] > R;
                    }
                    cnt += (uint32_t)__popcll(wave_ballot(hit));
                }
                if (cnt) {
                    const uint32_t pick = mt_ru(key, i, MT_R_AIMPICK, 0, cnt - 1);
                    uint32_t seen = 0;
                    int kk = -1;
                    for (int base = 0; base < nn && kk < 0; base += 64) {
                        const int k = base + lane;
                        bool hit = false;
                        if (k < nn) {
                            const int sl = s.order[k];
                            hit = s.cum[k] > cstart(k) && (s.flags[sl] & MT_SF_REMOVED) && s.rseq[sl] > R;
                        }
                        const uint64_t m = wave_ballot(hit);
                        const uint32_t pc = (uint32_t)__popcll(m);
                        if (pick < seen + pc) {
                            uint64_t mm = m;
                            for (uint32_t q = seen; q < pick; q++) mm &= mm - 1;
                            kk = base + first_lane(mm);
                        }
                        seen += pc;
                    }
                    const int32_t ppos = cstart(kk), plen = s.cum[kk] - cstart(kk);
                    const int32_t pre = (int32_t)mt_ru(key, i, MT_R_AIMPRE, 0, 2);
                    const int32_t post = (int32_t)mt_ru(key, i, MT_R_AIMPOST, 0, 2);
                    a = ppos - pre > 0 ? ppos - pre : 0;
                    b = ppos + plen + post < L ? ppos + plen + post : L;
                    aimed = true;
                }
            }
            if (!aimed) {
                const int32_t big = (int32_t)((mto_rng(key, i, MT_R_BIGLEN) & 15) == 0);
                const int32_t q = L / 4 > 1 ? L / 4 : 1;
                const int32_t ln = big ? (int32_t)mt_ru(key, i, MT_R_LEN, 1, (uint32_t)q)
                                       : (int32_t)mt_ru(key, i, MT_R_LEN, 1, 16);
                b = a + ln < L ? a + ln : L;
            }
            rec.pos1 = a;
            rec.pos2 = b;
            if (type == 2) {
                if (mt_rp(key, i, MT_R_REWRITE, cfg.p_rewrite)) rec.flags |= MT_F_REWRITE;
                const uint32_t nk = mt_ru(key, i, MT_R_NKEYS, 1, 2);
                const uint32_t k0 = mt_ru(key, i, MT_R_KEY0, 0, cfg.n_keys - 1);
                const uint32_t k1 = (k0 + 3) % cfg.n_keys;
                pr[0] = (uint8_t)k0;
                pr[1] = mt_rp(key, i, MT_R_NULL0, cfg.p_null) ? 0 : (uint8_t)mt_ru(key, i, MT_R_VAL0, 1, cfg.n_values);
                np = 1;
                if (nk == 2 && k1 != k0) {
                    pr[2] = (uint8_t)k1;
                    pr[3] = mt_rp(key, i, MT_R_NULL1, cfg.p_null) ? 0 : (uint8_t)mt_ru(key, i, MT_R_VAL1, 1, cfg.n_values);
                    np = 2;
                }
            }
        }
        if (pay_off + n + 2 * np > paycap) {
            fail(MT_DERR_TEXT_ARENA, rec.seq);
            n = 0;
            np = 0;
        } else if (lane == 0) {
            for (uint32_t q = 0; q < 2 * np; q++) pay[n + q] = pr[q];
        }
        __threadfence_block();
        rec.flags |= (uint8_t)(np << MT_F_NPAIRS_SHIFT);
        rec.payload_len = n + 2 * np;
        rec.payload_off = 0;  // caller rebases
        sync();
        return rec;
    }

    // ------------------------------------------------------------ load / store
    MT_DEV void load(const mt_gstate& g, uint32_t d) {
        const mt_doc_scalars& sc = g.sc[d];
        const int n = sc.nseg;
        const size_t so = (size_t)d * g.segcap;
        for (int i = lane; i < n; i += 64) {
            s.seq[i] = g.seq[so + i];
            s.rseq[i] = g.rseq[so + i];
            s.len[i] = g.len[so + i];
            s.toff[i] = g.toff[so + i];
            s.ovl[i] = g.ovl[so + i];
            s.props[i] = g.props[so + i];
            s.client[i] = g.client[so + i];
            s.rclient[i] = g.rclient[so + i];
            s.flags[i] = g.flags[so + i];
            s.order[i] = (uint16_t)i;
        }
        const bool trk = sc.label_keys != MT_NO_LABEL_KEYS && g.slab;
        if constexpr (LOC) {
            xslab = trk ? g.slabx + so : nullptr;
            if (trk) {
                for (int i = lane; i < n; i += 64) xslab[i] = g.slab[so + i];
                __threadfence_block();  // (lanes write and later read each other's slots)
            }
        } else {
            for (int i = lane; i < n; i += 64) s.slab[i] = trk ? g.slab[so + i] : 0u;
        }
        const size_t lo = (size_t)d * g.lbcap;
        for (int i = lane; i < sc.nb[0]; i += 64) {
            s.lbcnt[i] = g.lbcnt[lo + i];
            s.lbscour[i] = g.lbscour[lo + i];
        }
        for (int L = 1; L < sc.nlev; L++) {
            const size_t io = ((size_t)d * (MT_MAXLEV - 1) + (L - 1)) * g.ibcap;
            for (int i = lane; i < sc.nb[L]; i += 64) s.ibcnt[L - 1][i] = g.ibcnt[io + i];
        }
        const size_t ho = (size_t)d * g.hcap;
        for (int i = 1 + lane; i <= sc.heap_n; i += 64) {
            s.hseq[i] = g.hseq[ho + i];
            s.hslot[i] = g.hslot[ho + i];
        }
        const bool was_wide = (sc.wide & MT_WIDE_DOC) != 0;
        if constexpr (W) {
            // the extension: staged when binning asks for it (every slot of the region: stored words
            // for the document's segments, zeros for the rest)
            xo_p = (sc.wide & MT_WIDE_XO) ? ext : nullptr;
            xk_p = (sc.wide & MT_WIDE_XK) && ext ? ext + 4 * CAP : nullptr;
            if (((sc.wide & MT_WIDE_XO) || (sc.wide & MT_WIDE_XK)) && !ext && lane == 0) s.err = MT_DERR_LIMITS;
            const bool ov = was_wide && (sc.wide & MT_WIDE_XOV), kv = was_wide && (sc.wide & MT_WIDE_XKV);
            for (int i = lane; i < CAP && (xo_p || xk_p); i += 64) {
                for (int q = 0; q < 4 && xo_p; q++) xo_p[4 * i + q] = ov && i < n ? g.ovx[MT_OVX_WORDS * (so + i) + 4 + q] : 0ull;
                for (int q = 0; q < 4 && xk_p; q++) xk_p[4 * i + q] = kv && i < n ? g.pxx[4 * (so + i) + q] : 0ull;
            }
            for (int i = lane; i < n; i += 64) {
                for (int q = 0; q < 4; q++) s.ovx[4 * i + q] = was_wide ? g.ovx[MT_OVX_WORDS * (so + i) + q] : 0ull;
                // (the short ids' high bytes; a narrow document's ids are below 64)
                const uint32_t hi = was_wide ? g.chi[so + i] : 0u;
                s.client[i] = (CT)(s.client[i] | ((hi & 0xFFu) << 8));
                s.rclient[i] = (CT)(s.rclient[i] | ((hi >> 8) << 8));
                s.ph[i] = was_wide ? g.ph[so + i] : 0ull;
                s.pxl[i] = was_wide ? g.pxl[so + i] : 0ull;
                s.pxh[i] = was_wide ? g.pxh[so + i] : 0ull;
            }
        }
        if (lane == 0) {
            s.wide = sc.wide;
            s.lkeys = trk ? sc.label_keys : MT_NO_LABEL_KEYS;
            s.n = n;
            s.nlev = sc.nlev;
            for (int L = 0; L < MT_MAXLEV; L++) s.nb[L] = sc.nb[L];
            s.heap_n = sc.heap_n;
            s.cur_seq = sc.cur_seq;
            s.min_seq = sc.min_seq;
            s.err = sc.err;
            s.err_seq = sc.err_seq;
            s.nfree = 0;
            s.next_slot = n;
            s.text_top = sc.text_top;
            s.text_half = sc.text_half;
            s.evn = g.evn ? (int32_t)g.evn[d] : 0;
            s.evseq = sc.cur_seq;
        }
        if constexpr (LOC) {
            if (lane == 0) {
                s.lc.own = g.loc[d].own;
                s.lc.glo = g.loc[d].glo;
                s.lc.ghi = g.loc[d].ghi;
                s.lc.stamp = g.loc[d].stamp;
                s.lc.lseq = g.loc[d].lseq;
                s.lc.rgn = g.loc[d].rgn;
                s.lc.rgpn = g.loc[d].rgpn;
            }
            // (a document that has not edited yet has never stored these arrays)
            const bool has = g.loc[d].own >= 0;
            const LocRow lr = loc_row(g, d);
            if constexpr (GW == 1) {
                // (the groups' stamps and localSeqs stay in the document's mt_loc: gtp / glsp)
                for (int i = lane; i < n; i += 64) gmp[i] = has ? lr.gm[i] : 0ull;
            } else if (g.sc[d].wide & MT_WIDE_GROUPS) {
                const uint32_t gx = g.locgx[d];
                for (uint32_t j = lane; j < GN; j += 64) {
                    gtp[j] = g.locx[gx].gt[j];
                    glsp[j] = g.locx[gx].gls[j];
                }
                const uint64_t* gmx = g.gmx + (size_t)gx * MT_LOC_BIGCAP * GW;
                for (int i = lane; i < n * GW; i += 64) gmp[i] = gmx[i];
            } else {
                // entering the wide-group form: ordinal N moves from bit / index N % 64 to N % GN
                // (at most 64 pending, so N % 64 names one ordinal of [glo, ghi))
                const uint32_t glo = g.loc[d].glo, np = g.loc[d].ghi - glo;
                for (uint32_t j = lane; j < GN; j += 64) gtp[j] = glsp[j] = 0u;
                sync();
                if ((uint32_t)lane < np) {
                    const uint32_t N = glo + (uint32_t)lane;
                    gtp[N % GN] = g.loc[d].gt[N & 63u];
                    glsp[N % GN] = g.loc[d].gls[N & 63u];
                }
                for (int i = lane; i < n; i += 64) {
                    for (int w = 0; w < GW; w++) gmp[i * GW + w] = 0ull;
                    uint64_t m = has ? lr.gm[i] : 0ull;
                    while (m) {
                        const uint32_t b = (uint32_t)__builtin_ctzll(m);
                        m &= m - 1;
                        gm_set(i, glo + ((b - glo) & 63u));
                    }
                }
            }
            for (int i = lane; i < n; i += 64) {
                pkp[i] = has ? lr.pk[i] : 0ull;
                ctp[i] = has ? lr.ct[i] : 0u;
                lsqp[i] = has ? lr.lsq[i] : 0ull;
            }
            ct_publish();
        }
        sync();
        arena = abase + (size_t)s.text_half * textcap;
        if constexpr (W) {
            if (!was_wide) promote();
        }
    }

    // A narrow document enters the wide form (include/mtgpu.h "limits"): its Latin-1 text becomes
    // UTF-16 code units in the other arena half (compacted, in document order; a half holds
    // textcap units); the overlap ids >= 64 and the wide property words start empty (load).  When the
    // text does not fit, the document halts with MT_DERR_TEXT_ARENA and stays narrow.
    MT_DEV void promote() {
        if constexpr (W) {
            const int n = s.n;
            const uint32_t tcb = textcap * (uint32_t)sizeof(TC);  // bytes per half
            const uint8_t* src = reinterpret_cast<const uint8_t*>(abase) + (size_t)s.text_half * tcb;
            int total = 0;
            for (int base = 0; base < n; base += 64) total += wave_sum(base + lane < n ? (int)s.len[base + lane] : 0);
            if ((uint32_t)total > textcap) return fail(MT_DERR_TEXT_ARENA, s.cur_seq);
            TC* dst = abase + (size_t)(s.text_half ^ 1u) * textcap;
            uint32_t carry = 0;
            for (int base = 0; base < n; base += 64) {
                const int i = base + lane;
                const int l = i < n ? (int)s.len[i] : 0;
                const int incl = wave_incl_scan(l);
                const uint32_t at = carry + (uint32_t)(incl - l);
                if (i < n) {
                    const uint8_t* t = src + s.toff[i];
                    for (int q = 0; q < l; q++) dst[at + q] = (TC)t[q];
                }
                sync();
                if (i < n) s.toff[i] = at;
                carry += (uint32_t)wave_last(incl);
            }
            __threadfence_block();
            sync();
            if (lane == 0) {
                s.text_half = s.text_half ^ 1u;
                s.text_top = carry;
                s.wide = s.wide | MT_WIDE_DOC | MT_WIDE_LDS;
            }
            sync();
            arena = dst;
        }
    }

    MT_DEV void store(const mt_gstate& g, uint32_t d) {
        const int n = s.n;
        const size_t so = (size_t)d * g.segcap;
        if ((uint32_t)n > g.segcap || s.nb[0] > (int)g.lbcap || s.heap_n >= (int)g.hcap) fail(MT_DERR_CAPACITY, s.cur_seq);
        const int nn = min(n, (int)g.segcap);
        if constexpr (LOC)
            if (xslab) __threadfence_block();  // mark_stale's HBM writes, read below by other lanes
        for (int i = lane; i < nn; i += 64) {
            const int sl = s.order[i];
            g.seq[so + i] = s.seq[sl];
            g.rseq[so + i] = s.rseq[sl];
            g.len[so + i] = s.len[sl];
            g.toff[so + i] = s.toff[sl];
            g.ovl[so + i] = s.ovl[sl];
            g.props[so + i] = s.props[sl];
            g.client[so + i] = (uint8_t)s.client[sl];
            g.rclient[so + i] = (uint8_t)s.rclient[sl];
            g.flags[so + i] = s.flags[sl];
            if (track()) g.slab[so + i] = LOC ? xslab[sl] : s.slab[sl];
            s.cum[sl] = i;  // slot -> position for the heap remap
        }
        sync();
        const size_t lo = (size_t)d * g.lbcap;
        int nempty = 0;
        for (int i = lane; i < min(s.nb[0], (int)g.lbcap); i += 64) {
            g.lbcnt[lo + i] = s.lbcnt[i];
            g.lbscour[lo + i] = s.lbscour[i];
            nempty += s.lbcnt[i] == 0 ? 1 : 0;
        }
        nempty = wave_sum(nempty);
        for (int L = 1; L < s.nlev; L++) {
            const size_t io = ((size_t)d * (MT_MAXLEV - 1) + (L - 1)) * g.ibcap;
            for (int i = lane; i < min(s.nb[L], (int)g.ibcap); i += 64) g.ibcnt[io + i] = s.ibcnt[L - 1][i];
        }
        const size_t ho = (size_t)d * g.hcap;
        for (int i = 1 + lane; i <= min(s.heap_n, (int)g.hcap - 1); i += 64) {
            g.hseq[ho + i] = s.hseq[i];
            const uint16_t sl = s.hslot[i];
            g.hslot[ho + i] = sl == MT_DEAD_SLOT ? MT_DEAD_SLOT : (uint16_t)s.cum[sl];
        }
        if (lane == 0) {
            mt_doc_scalars& sc = g.sc[d];
            sc.nseg = nn;
            sc.nlev = s.nlev;
            for (int L = 0; L < MT_MAXLEV; L++) sc.nb[L] = s.nb[L];
            sc.heap_n = s.heap_n;
            sc.cur_seq = s.cur_seq;
            sc.min_seq = s.min_seq;
            sc.err = s.err;
            sc.err_seq = s.err_seq;
            sc.text_top = s.text_top;
            sc.text_half = s.text_half;
            sc.n_empty = (uint32_t)nempty;
            if (g.evn) g.evn[d] = (uint32_t)s.evn;
            if (W) sc.wide = s.wide;
            if (GW > 1 && s.lc.own >= 0) sc.wide = sc.wide | MT_WIDE_GROUPS;
        }
        if constexpr (W) {
            int ovn = 0;  // the longest overlap list of ids >= 64 (binning's bound, mt_state.h MT_WIDE_OVN)
            for (int i = lane; i < nn; i += 64) {
                const int sl = s.order[i];
                for (int q = 0; q < 4; q++) g.ovx[MT_OVX_WORDS * (so + i) + q] = s.ovx[4 * sl + q];
                g.chi[so + i] = (uint16_t)(((uint32_t)s.client[sl] >> 8) | (((uint32_t)s.rclient[sl] >> 8) << 8));
                g.ph[so + i] = s.ph[sl];
                g.pxl[so + i] = s.pxl[sl];
                g.pxh[so + i] = s.pxh[sl];
                for (int q = 0; q < 4 && xo_p; q++) g.ovx[MT_OVX_WORDS * (so + i) + 4 + q] = xo_p[4 * sl + q];
                for (int q = 0; q < 4 && xk_p; q++) g.pxx[4 * (so + i) + q] = xk_p[4 * sl + q];
                int m = 0;
                while (m < MT_OVX_IDS && mt_ovx_id2(&s.ovx[4 * sl], ovx_hi(sl), m)) m++;
                ovn = max(ovn, m);
            }
            ovn = wave_max(ovn);
            if (lane == 0) {
                const uint32_t keep = s.wide & ~((0xFFu << MT_WIDE_OVN_SHIFT) | MT_WIDE_XOV);
                g.sc[d].wide = keep | (xk_p ? MT_WIDE_XKV : 0u) | (xo_p && ovn > 16 ? MT_WIDE_XOV : 0u) |
                               ((uint32_t)ovn << MT_WIDE_OVN_SHIFT);
            }
        }
        if constexpr (LOC) {
            if (s.lc.own >= 0) {
                const LocRow lr = loc_row(g, d);  // (loc_admit: nn <= CAP <= lr.cap)
                uint64_t* gmx = GW > 1 ? g.gmx + (size_t)g.locgx[d] * MT_LOC_BIGCAP * GW : nullptr;
                for (int i = lane; i < min(nn, lr.cap); i += 64) {
                    const int sl = s.order[i];
                    if constexpr (GW == 1) {
                        lr.gm[i] = gmp[sl];
                    } else {
                        for (int w = 0; w < GW; w++) gmx[i * GW + w] = gmp[sl * GW + w];
                    }
                    lr.pk[i] = pkp[sl];
                    lr.ct[i] = ctp[sl];
                    lr.lsq[i] = lsqp[sl];
                }
                if (lane == 0) {
                    g.loc[d].own = s.lc.own;
                    g.loc[d].glo = s.lc.glo;
                    g.loc[d].ghi = s.lc.ghi;
                    g.loc[d].stamp = s.lc.stamp;
                    g.loc[d].lseq = s.lc.lseq;
                    g.loc[d].rgn = s.lc.rgn;
                    g.loc[d].rgpn = s.lc.rgpn;
                }
                if constexpr (GW > 1) {
                    const uint32_t gx = g.locgx[d];
                    for (uint32_t j = lane; j < GN; j += 64) {
                        g.locx[gx].gt[j] = gtp[j];
                        g.locx[gx].gls[j] = glsp[j];
                    }
                }
            }
        }
    }
};

struct GenArgs {
    mt_synth_cfg cfg;
    int32_t* cref;      // [doc][64]
    int32_t* stall;     // [doc]
    uint32_t* pay_used; // [doc]
    uint32_t paycap;    // payload bytes per document region
    uint32_t doc_id_base; // global id of local document 0 (the RNG stream is per global doc id)
    const uint32_t* gids; // or the global id of every local document (a hash-routed shard)
};

// An editing document enters the editing form at CAP slots only if this launch's ops cannot outgrow
// it (the form cannot move a document between capacities mid-launch); otherwise it halts with
// MT_DERR_CAPACITY, and a wide document with MT_DERR_LIMITS (no local edits in the wide form).
// MT_DERR_CAPACITY too when the engine could not give the document the pool rows its form needs.
template <int CAP, int GW = 1>
MT_DEV bool loc_admit(const mt_gstate& g, const mt_op_rec* ops, uint32_t d, uint32_t a, uint32_t b) {
    using LS = Lds<CAP, true>;
    const mt_doc_scalars& sc = g.sc[d];
    if (sc.wide & MT_WIDE_DOC) {
        if (threadIdx.x == 0 && !sc.err) {
            g.sc[d].err = MT_DERR_LIMITS;
            g.sc[d].err_seq = ops[a].seq;
        }
        return false;
    }
    const int nops = (int)(b - a);
    int ib_need = 0;
    for (int L = 1; L < sc.nlev; L++) ib_need = max(ib_need, sc.nb[L]);
    if (!(sc.nseg + 2 * nops + (int)sc.n_empty + 1 <= CAP && sc.nb[0] + 2 * nops + 1 <= LS::LB &&
          ib_need + nops + 1 <= LS::IB && sc.heap_n + 4 * nops + 16 <= LS::H && CAP <= loc_row(g, d).cap &&
          (GW == 1 || g.locgx[d] != MT_NO_ROW))) {
        if (threadIdx.x == 0 && !sc.err) {
            g.sc[d].err = MT_DERR_CAPACITY;
            g.sc[d].err_seq = ops[a].seq;
        }
        return false;
    }
    return true;
}

// The op records of a document in blocks of 8, double-buffered in two registers (lane l holds dword
// l % 8 of record base + l / 8; the register engine's mtr::load_op_block): a record's fields are
// readlanes of a register loaded up to 15 records earlier, so no record waits for its own load
MT_DEV uint32_t op_block(const mt_op_rec* ops, uint32_t base, uint32_t end, int lane) {
    const uint32_t r = min(base + (uint32_t)(lane >> 3), end - 1u);  // (end > base's first record)
    return reinterpret_cast<const uint32_t*>(ops + r)[lane & 7];
}
MT_DEV mt_op_rec op_of_block(uint32_t blk, uint32_t j) {
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
// The records [a, b) of a document through op_block's two buffers: f(op, i) per record until it
// returns false
template <typename F>
MT_DEV void for_each_op(const mt_op_rec* ops, uint32_t a, uint32_t b, int lane, F&& f) {
    uint32_t blk0 = op_block(ops, a, b, lane);
    uint32_t blk1 = op_block(ops, a + 8, b, lane);
    for (uint32_t i = a; i < b; i++) {
        const mt_op_rec op = op_of_block(blk0, (i - a) & 7u);
        if (((i + 1 - a) & 7u) == 0) {
            blk0 = blk1;
            blk1 = op_block(ops, i + 9, b, lane);
        }
        if (!f(op, i)) break;
    }
}

// The document arrays of mt_gstate are needed by load() and store() only.  Both get them as a copy
// read through a pointer to the kernel's own argument block (g: the first argument, offset 0) that
// the compiler cannot see through, so the pointers are loaded at those two sites and are not held
// live across the op loop (where ~50 SGPR pairs were spilled into VGPR lanes: mt_apply_reg.hip
// kernarg_gstate, the same remedy)
MT_DEV mt_gstate kernarg_g() {
    const char* p = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    mt_gstate g;
    __builtin_memcpy(&g, p, sizeof g);
    return g;
}
// (MT_LOC_WPE: the editing form's waves per SIMD at 256 slots, for A/B builds; 0 = the compiler's)
#ifndef MT_LOC_WPE
#define MT_LOC_WPE 0
#endif
constexpr int loc_wpe(int CAP, bool LOC) { return LOC && CAP <= 256 && MT_LOC_WPE > 0 ? MT_LOC_WPE : 1; }
template <int CAP, bool GEN, bool LOC = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(loc_wpe(CAP, LOC))))
void apply_kernel(mt_gstate g, mt_op_rec* __restrict__ ops,
                                                   uint8_t* __restrict__ payload,
                                                   const uint32_t* __restrict__ row_ptr,
                                                   const uint32_t* __restrict__ doc_ids, uint32_t n_docs,
                                                   uint32_t op_lo, uint32_t op_cnt, GenArgs gen) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t w = blockIdx.x;
    if (w >= n_docs) return;
    const uint32_t d = doc_ids ? doc_ids[w] : w;
    Lds<CAP, LOC>& lds = *reinterpret_cast<Lds<CAP, LOC>*>(smem);
    Wave<CAP, false, LOC> wv(lds, g.text + (size_t)d * 2 * g.textcap, g.textcap,
                             GEN || !g.ev ? nullptr : g.ev + (size_t)d * g.evcap, g.evcap);
    if constexpr (LOC) {  // (launched without Lds::ct / lsq)
        wv.ctp = g.ctx + (size_t)d * MT_LOC_CAP;
        wv.lsqp = g.lsqx + (size_t)d * MT_LOC_CAP;
        wv.pkp = g.pkx + (size_t)d * MT_LOC_CAP;
        wv.gmp = g.gmxs + (size_t)d * MT_LOC_CAP;
        wv.gtp = g.loc[d].gt;
        wv.glsp = g.loc[d].gls;
    }
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    const uint32_t a = min(r1, r0 + op_lo);
    const uint32_t b = op_cnt ? min(r1, a + op_cnt) : r1;
    if (a >= b) return;
    if (LOC && !loc_admit<CAP>(g, ops, d, a, b)) return;
    wv.load(kernarg_g(), d);
    if (LOC) {
        wv.rg = g.rg + (size_t)d * MT_RG_RECS;
        wv.rgp = g.rgp + (size_t)d * MT_RG_BYTES;
    }
    if constexpr (GEN) {
        lds.gcref[wv.lane] = gen.cref[(size_t)d * 64 + wv.lane];
        if (wv.lane == 0) {
            lds.gstall = gen.stall[d];
            lds.gpay = gen.pay_used[d];
        }
        wave_sync();
        const uint64_t key = mto_rng_key(gen.cfg.seed, gen.gids ? gen.gids[d] : gen.doc_id_base + d);
        const size_t pbase = (size_t)d * gen.paycap;
        for (uint32_t i = a; i < b; i++) {
            if (lds.err) break;
            const uint32_t off = lds.gpay;
            mt_op_rec op = wv.gen_op(gen.cfg, key, i - r0, payload + pbase + off, off, gen.paycap);
            if (lds.err) break;
            op.payload_off = (uint32_t)(pbase + off);
            if (wv.lane == 0) ops[i] = op;
            lds.gpay = off + op.payload_len;
            wave_sync();
            wv.apply(op, payload);
        }
        gen.cref[(size_t)d * 64 + wv.lane] = lds.gcref[wv.lane];
        if (wv.lane == 0) {
            gen.stall[d] = lds.gstall;
            gen.pay_used[d] = lds.gpay;
        }
    } else {
        for_each_op(ops, a, b, wv.lane, [&](const mt_op_rec& op, uint32_t i) {
            if (lds.err) return false;
            wv.rix = i - r0;
            wv.apply(op, payload);
            return true;
        });
    }
    wv.store(kernarg_g(), d);
}

// Documents above 2048 segments: the same engine with the document's structure in a per-wave
// HBM workspace (ws + w * sizeof(Lds<CAP>)) instead of LDS.  Latency-bound like the LDS form but
// without its 160 KiB-per-CU ceiling; such documents are rare, so a handful of waves serve them.
// W: wide documents (include/mtgpu.h "limits"), every capacity class from 2048 segments up.
// LOC: the editing form above MT_LOC_CAP segments or past 64 pending edits (GW = 4: MT_WIDE_GROUPS
// documents; mt_launch_apply_loc_big).
template <int CAP, bool W = false, bool LOC = false, int GW = 1>
__global__ __launch_bounds__(64) void apply_kernel_g(mt_gstate g, const mt_op_rec* __restrict__ ops,
                                                     const uint8_t* __restrict__ payload,
                                                     const uint32_t* __restrict__ row_ptr,
                                                     const uint32_t* __restrict__ doc_ids, uint32_t n_docs,
                                                     uint32_t op_lo, uint32_t op_cnt, uint8_t* __restrict__ ws) {
    const uint32_t w = blockIdx.x;
    if (w >= n_docs) return;
    const uint32_t d = doc_ids ? doc_ids[w] : w;
    using LS = Lds<CAP, LOC, W, GW>;
    LS& st = *reinterpret_cast<LS*>(ws + (size_t)w * sizeof(LS));
    Wave<CAP, true, LOC, W, GW> wv(st, g.text + (size_t)d * 2 * g.textcap, g.textcap,
                                   g.ev ? g.ev + (size_t)d * g.evcap : nullptr, g.evcap);
    if constexpr (W) wv.ext = st.ovh;  // (the extension: the workspace's own tail)
    if constexpr (LOC) {
        wv.ctp = st.ct;
        wv.lsqp = st.lsq;
        wv.pkp = st.pk;
        wv.gmp = st.gm;
        if constexpr (GW > 1) {
            wv.gtp = st.lc.gt;
            wv.glsp = st.lc.gls;
        } else {
            wv.gtp = g.loc[d].gt;
            wv.glsp = g.loc[d].gls;
        }
    }
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    const uint32_t a = min(r1, r0 + op_lo);
    const uint32_t b = op_cnt ? min(r1, a + op_cnt) : r1;
    if (a >= b) return;
    if (LOC && !loc_admit<CAP, GW>(g, ops, d, a, b)) return;
    wv.load(kernarg_g(), d);
    if (LOC) {
        wv.rg = g.rg + (size_t)d * MT_RG_RECS;
        wv.rgp = g.rgp + (size_t)d * MT_RG_BYTES;
    }
    for_each_op(ops, a, b, wv.lane, [&](const mt_op_rec& op, uint32_t i) {
        if (st.err) return false;
        if (LOC) wv.rix = i - r0;
        wv.apply(op, payload);
        return true;
    });
    wv.store(kernarg_g(), d);
}

// The wide form with the document staged in LDS (small wide documents: CAP <= 512, where its
// ~112 B per slot still lets two or more waves share a CU); the extension (keys 16..31, overlap
// ids past the 16th) of the documents that use it in an HBM region (wsx)
template <int CAP>
__global__ __launch_bounds__(64) void apply_kernel_wl(mt_gstate g, const mt_op_rec* __restrict__ ops,
                                                      const uint8_t* __restrict__ payload,
                                                      const uint32_t* __restrict__ row_ptr,
                                                      const uint32_t* __restrict__ doc_ids, uint32_t n_docs,
                                                      uint32_t op_lo, uint32_t op_cnt, uint64_t* __restrict__ wsx) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t w = blockIdx.x;
    if (w >= n_docs) return;
    const uint32_t d = doc_ids ? doc_ids[w] : w;
    using LS = Lds<CAP, false, true>;
    LS& st = *reinterpret_cast<LS*>(smem);  // (launched without its extension members: LS::kExtBytes)
    Wave<CAP, false, false, true> wv(st, g.text + (size_t)d * 2 * g.textcap, g.textcap,
                                     g.ev ? g.ev + (size_t)d * g.evcap : nullptr, g.evcap);
    // the extension of the documents that stage it: an HBM region per wave, laid out as LS's tail
    wv.ext = wsx ? wsx + (size_t)w * (LS::kExtBytes / sizeof(uint64_t)) : nullptr;
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    const uint32_t a = min(r1, r0 + op_lo);
    const uint32_t b = op_cnt ? min(r1, a + op_cnt) : r1;
    if (a >= b) return;
    wv.load(kernarg_g(), d);
    for_each_op(ops, a, b, wv.lane, [&](const mt_op_rec& op, uint32_t) {
        if (st.err) return false;
        wv.apply(op, payload);
        return true;
    });
    wv.store(kernarg_g(), d);
}

}  // namespace mt

// ------------------------------------------------------------------------------------------
// host-side launchers (called from mt_engine.cpp)
static hipError_t launch_any(int cap_class, bool gen, const mt_gstate* g, mt_op_rec* ops, uint8_t* payload,
                             const uint32_t* row_ptr, const uint32_t* doc_ids, uint32_t n_docs, uint32_t op_lo,
                             uint32_t op_cnt, const mt::GenArgs& ga, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    dim3 grid(n_docs), block(64);
#define MT_LAUNCH(CAPV)                                                                                      \
    case CAPV: {                                                                                             \
        const size_t lds = sizeof(mt::Lds<CAPV>);                                                            \
        if (gen)                                                                                             \
            hipLaunchKernelGGL((mt::apply_kernel<CAPV, true>), grid, block, lds, stream, *g, ops, payload,    \
                               row_ptr, doc_ids, n_docs, op_lo, op_cnt, ga);                                 \
        else                                                                                                 \
            hipLaunchKernelGGL((mt::apply_kernel<CAPV, false>), grid, block, lds, stream, *g, ops, payload,   \
                               row_ptr, doc_ids, n_docs, op_lo, op_cnt, ga);                                 \
        return hipGetLastError();                                                                            \
    }
    switch (cap_class) {
        MT_LAUNCH(128)
        MT_LAUNCH(256)
        MT_LAUNCH(384)
        MT_LAUNCH(512)
        MT_LAUNCH(640)
        MT_LAUNCH(768)
        MT_LAUNCH(896)
        MT_LAUNCH(1024)
        MT_LAUNCH(2048)
        default:
            return hipErrorInvalidValue;
    }
#undef MT_LAUNCH
}

extern "C" hipError_t mt_launch_apply(int cap_class, const mt_gstate* g, const mt_op_rec* ops, const uint8_t* payload,
                                      const uint32_t* row_ptr, const uint32_t* doc_ids, uint32_t n_docs,
                                      uint32_t op_lo, uint32_t op_cnt, hipStream_t stream) {
    mt::GenArgs ga{};
    return launch_any(cap_class, false, g, const_cast<mt_op_rec*>(ops), const_cast<uint8_t*>(payload), row_ptr,
                      doc_ids, n_docs, op_lo, op_cnt, ga, stream);
}

extern "C" hipError_t mt_launch_gen(int cap_class, const mt_gstate* g, const mt_synth_cfg* cfg, uint32_t doc_id_base,
                                    const uint32_t* gids, int32_t* cref, int32_t* stall, uint32_t* pay_used, uint32_t paycap, mt_op_rec* ops,
                                    uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                    uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, hipStream_t stream) {
    mt::GenArgs ga{*cfg, cref, stall, pay_used, paycap, doc_id_base, gids};
    return launch_any(cap_class, true, g, ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt, ga, stream);
}

// classes above 2048 segments (workspace: n_docs * mt_lds_bytes(cap_class) bytes of HBM)
extern "C" hipError_t mt_launch_apply_big(int cap_class, const mt_gstate* g, const mt_op_rec* ops,
                                          const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                          uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, uint8_t* ws,
                                          hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    dim3 grid(n_docs), block(64);
#define MT_LAUNCH_BIG(CAPV)                                                                                  \
    case CAPV:                                                                                               \
        hipLaunchKernelGGL((mt::apply_kernel_g<CAPV>), grid, block, 0, stream, *g, ops, payload, row_ptr,     \
                           doc_ids, n_docs, op_lo, op_cnt, ws);                                              \
        return hipGetLastError();
    switch (cap_class) {
        MT_LAUNCH_BIG(4096)
        MT_LAUNCH_BIG(8192)
        MT_LAUNCH_BIG(16384)
        MT_LAUNCH_BIG(32768)
        MT_LAUNCH_BIG(65472)
        default:
            return hipErrorInvalidValue;
    }
#undef MT_LAUNCH_BIG
}

// wide documents (mt_bin_kernel's wide buckets; workspace: n_docs * mt_lds_bytes_wide(cap_class)):
// up to 512 segments staged in LDS, above that in the HBM workspace (1024 for the classes up to it)
extern "C" hipError_t mt_launch_apply_wide(int cap_class, const mt_gstate* g, const mt_op_rec* ops,
                                           const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                           uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, uint8_t* ws,
                                           int xl, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    dim3 grid(n_docs), block(64);
    if (cap_class <= 512) {
        // (the extension never takes LDS: with xl, ws holds it for the documents that stage it,
        // mt_lds_bytes_wide per document)
#define MT_LAUNCH_WL(CAPV)                                                                                   \
        hipLaunchKernelGGL((mt::apply_kernel_wl<CAPV>), grid, block,                                         \
                           mt::wl_lds_bytes<CAPV>(), stream,                                         \
                           *g, ops, payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt,                        \
                           xl ? reinterpret_cast<uint64_t*>(ws) : nullptr);                                  \
        return hipGetLastError();
        if (cap_class <= 256) {
            MT_LAUNCH_WL(256)
        }
        MT_LAUNCH_WL(512)
#undef MT_LAUNCH_WL
    }
    if (cap_class <= 1024) cap_class = 1024;
#define MT_LAUNCH_WIDE(CAPV)                                                                                 \
    case CAPV:                                                                                               \
        hipLaunchKernelGGL((mt::apply_kernel_g<CAPV, true>), grid, block, 0, stream, *g, ops, payload, row_ptr, \
                           doc_ids, n_docs, op_lo, op_cnt, ws);                                              \
        return hipGetLastError();
    switch (cap_class) {
        MT_LAUNCH_WIDE(1024)
        MT_LAUNCH_WIDE(2048)
        MT_LAUNCH_WIDE(4096)
        MT_LAUNCH_WIDE(8192)
        MT_LAUNCH_WIDE(16384)
        MT_LAUNCH_WIDE(32768)
        MT_LAUNCH_WIDE(65472)
        default:
            return hipErrorInvalidValue;
    }
#undef MT_LAUNCH_WIDE
}

extern "C" size_t mt_lds_bytes_wide(int cap_class) {
    // (staged in LDS: the workspace holds only the extension, for launches that stage it)
    if (cap_class <= 256) return mt::Lds<256, false, true>::kExtBytes;
    if (cap_class <= 512) return mt::Lds<512, false, true>::kExtBytes;
    if (cap_class <= 1024) return sizeof(mt::Lds<1024, false, true>);
    switch (cap_class) {
        case 2048: return sizeof(mt::Lds<2048, false, true>);
        case 4096: return sizeof(mt::Lds<4096, false, true>);
        case 8192: return sizeof(mt::Lds<8192, false, true>);
        case 16384: return sizeof(mt::Lds<16384, false, true>);
        case 32768: return sizeof(mt::Lds<32768, false, true>);
        case 65472: return sizeof(mt::Lds<65472, false, true>);
        default: return 0;
    }
}

// documents with an editing client (mt_bin_kernel's last bucket): the LDS engine's editing form
extern "C" hipError_t mt_launch_apply_loc(int cap_class, const mt_gstate* g, const mt_op_rec* ops,
                                          const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                          uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    mt::GenArgs ga{};
    // the editing form at 256 / 512 / 1024 slots: its LDS (~78 B per slot, without the stamps'
    // tail: loc_lds_bytes) allows 8 / 3 / 2 waves per CU
#define MT_LAUNCH_LOC(CAPV)                                                                                  \
    case CAPV:                                                                                               \
        hipLaunchKernelGGL((mt::apply_kernel<CAPV, false, true>), dim3(n_docs), dim3(64),                     \
                           mt::loc_lds_bytes<CAPV>(), stream, *g, const_cast<mt_op_rec*>(ops),               \
                           const_cast<uint8_t*>(payload), row_ptr, doc_ids, n_docs, op_lo, op_cnt, ga);     \
        return hipGetLastError();
    switch (cap_class) {
        MT_LAUNCH_LOC(256)
        MT_LAUNCH_LOC(512)
        MT_LAUNCH_LOC(MT_LOC_CAP)
        default:
            return hipErrorInvalidValue;
    }
#undef MT_LAUNCH_LOC
}

// editing documents above MT_LOC_CAP segments (mt_bin_kernel's last editing buckets): the editing
// form with its structure in the HBM workspace (n_docs * mt_lds_bytes_loc(cap_class) bytes)
// (gw = MT_LOC_GW: the MT_WIDE_GROUPS documents' form, MT_LOC_GROUPS_WIDE pending edits, at 1024 / 4096 /
// 8192 slots)
extern "C" hipError_t mt_launch_apply_loc_big(int cap_class, int gw, const mt_gstate* g, const mt_op_rec* ops,
                                              const uint8_t* payload, const uint32_t* row_ptr,
                                              const uint32_t* doc_ids, uint32_t n_docs, uint32_t op_lo,
                                              uint32_t op_cnt, uint8_t* ws, hipStream_t stream) {
    if (n_docs == 0) return hipSuccess;
    dim3 grid(n_docs), block(64);
#define MT_LAUNCH_LOCB(CAPV, GWV)                                                                            \
    if (cap_class == CAPV && gw == GWV) {                                                                    \
        hipLaunchKernelGGL((mt::apply_kernel_g<CAPV, false, true, GWV>), grid, block, 0, stream, *g, ops,     \
                           payload, row_ptr, doc_ids, n_docs, op_lo, op_cnt, ws);                            \
        return hipGetLastError();                                                                            \
    }
    MT_LAUNCH_LOCB(2048, 1)
    MT_LAUNCH_LOCB(4096, 1)
    MT_LAUNCH_LOCB(1024, MT_LOC_GW)
    MT_LAUNCH_LOCB(4096, MT_LOC_GW)
    MT_LAUNCH_LOCB(8192, 1)
    MT_LAUNCH_LOCB(8192, MT_LOC_GW)
#undef MT_LAUNCH_LOCB
    return hipErrorInvalidValue;
}

extern "C" size_t mt_lds_bytes_loc(int cap_class, int gw) {
    if (gw == 1 && cap_class == 2048) return sizeof(mt::Lds<2048, true>);
    if (gw == 1 && cap_class == 4096) return sizeof(mt::Lds<4096, true>);
    if (gw == MT_LOC_GW && cap_class == 1024) return sizeof(mt::Lds<1024, true, false, MT_LOC_GW>);
    if (gw == MT_LOC_GW && cap_class == 4096) return sizeof(mt::Lds<4096, true, false, MT_LOC_GW>);
    if (gw == 1 && cap_class == 8192) return sizeof(mt::Lds<8192, true>);
    if (gw == MT_LOC_GW && cap_class == 8192) return sizeof(mt::Lds<8192, true, false, MT_LOC_GW>);
    return 0;
}

extern "C" size_t mt_lds_bytes(int cap_class) {
    switch (cap_class) {
        case 4096: return sizeof(mt::Lds<4096>);
        case 8192: return sizeof(mt::Lds<8192>);
        case 16384: return sizeof(mt::Lds<16384>);
        case 32768: return sizeof(mt::Lds<32768>);
        case 65472: return sizeof(mt::Lds<65472>);
        case 128: return sizeof(mt::Lds<128>);
        case 256: return sizeof(mt::Lds<256>);
        case 512: return sizeof(mt::Lds<512>);
        case 1024: return sizeof(mt::Lds<1024>);
        case 2048: return sizeof(mt::Lds<2048>);
        default: return 0;
    }
}
