// mt_service.hip -- small device kernels around the apply engine: document init, per-launch
// capacity binning, canonical-state checksums.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtgpu.h"
#include "mt_checksum.h"
#include "mt_state.h"
#include "mt_wave.h"

// Client + startOrUpdateCollaboration: an empty root block, collab window (0, 0)
// (mergeTree.ts:1125-1129, 1254-1271)
__global__ void mt_init_kernel(mt_gstate g, uint32_t n_docs) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n_docs) return;
    mt_doc_scalars sc{};
    sc.nseg = 0;
    sc.nlev = 1;
    sc.nb[0] = 1;
    sc.n_empty = 1;  // the root leaf block starts empty
    sc.win_op = -1;
    sc.label_keys = MT_NO_LABEL_KEYS;
    g.sc[d] = sc;
    g.loc[d].own = -1;  // an observer until its first local edit
    g.loc[d].glo = g.loc[d].ghi = g.loc[d].stamp = g.loc[d].lseq = g.loc[d].rgn = g.loc[d].rgpn = 0;
    g.lbcnt[(size_t)d * g.lbcap] = 0;
    g.lbscour[(size_t)d * g.lbcap] = MT_SC_UNDEF;
}

// mt_set_label_keys: documents [d0, d1) track the block caches of their tile / range labels and run
// on the LDS engine from now on
__global__ void mt_label_keys_kernel(mt_gstate g, uint32_t d0, uint32_t d1, uint32_t keys) {
    const uint32_t d = d0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= d1) return;
    const uint32_t old = g.sc[d].label_keys;  // (a key left undeclared, 0xFF, keeps its value; the host
    uint32_t nk = 0;                         // refused conflicting declarations)
    for (int h = 0; h < 16; h += 8) nk |= (((keys >> h) & 0xFFu) != 0xFFu ? (keys >> h) & 0xFFu : (old >> h) & 0xFFu) << h;
    g.sc[d].label_keys = nk;
    g.sc[d].wide |= MT_WIDE_LDS;
}
extern "C" hipError_t mt_launch_label_keys(const mt_gstate* g, uint32_t d0, uint32_t d1, uint32_t keys, hipStream_t st) {
    if (d1 <= d0) return hipSuccess;
    hipLaunchKernelGGL(mt_label_keys_kernel, dim3((d1 - d0 + 255) / 256), dim3(256), 0, st, *g, d0, d1, keys);
    return hipGetLastError();
}

// SnapshotLoader.loadHeader (snapshotLoader.ts:119-157) for a batch of documents, one wave per
// document: the header chunk's segments become the document in order (specToSegment, :85-117:
// NonCollabClient / UniversalSequenceNumber without merge info), texts packed into the arena's
// first half; MergeTree.reloadFromSegments (mergeTree.ts:1195-1251) shapes the tree bottom-up with
// MaxNodesInBlock - 1 = 7 children per block (the last block of a level takes the rest) until one
// block is left; startOrUpdateCollaboration (client.ts:1051-1071, mergeTree.ts:1254-1271) sets the
// window and an empty LRU heap.  Every block's needsScour is undefined.
__global__ __launch_bounds__(64) void mt_load_kernel(mt_gstate g, uint32_t n, const uint32_t* __restrict__ doc_ids,
                                                     const uint32_t* __restrict__ row_ptr,
                                                     const mt_load_seg* __restrict__ segs,
                                                     const uint8_t* __restrict__ text,
                                                     const int32_t* __restrict__ min_seq,
                                                     const int32_t* __restrict__ cur_seq) {
    const uint32_t w = blockIdx.x;
    if (w >= n) return;
    const uint32_t d = doc_ids[w];
    const int lane = lane_id();
    const uint32_t r0 = row_ptr[w];
    const int ns = (int)(row_ptr[w + 1] - r0);
    constexpr int kPerBlock = 7;  // MaxNodesInBlock - 1
    int nb[MT_MAXLEV] = {0};
    int nlev = 0;
    int err = 0;
    {
        int m = ns;
        do {
            const int blocks = m == 0 ? 1 : (m + kPerBlock - 1) / kPerBlock;
            if (nlev >= MT_MAXLEV || blocks > (int)(nlev == 0 ? g.lbcap : g.ibcap)) {
                err = MT_DERR_CAPACITY;
                break;
            }
            nb[nlev++] = blocks;
            m = blocks;
        } while (m > 1);
    }
    if (ns > (int)g.segcap) err = MT_DERR_CAPACITY;
    const size_t so = (size_t)d * g.segcap;
    uint8_t* arena = g.text + (size_t)d * 2 * g.textcap;  // half 0
    // a document with any segment beyond the narrow limits loads in the wide form (UTF-16 text,
    // u16 value ids, keys < 32, client ids >= 64; include/mtgpu.h "limits")
    bool wdoc = false, lds = false;
    for (int base = 0; base < ns; base += 64) {
        const int i = base + lane;
        bool w = false, l32 = false;
        if (i < ns) {
            const mt_load_seg& sg = segs[r0 + i];
            const bool pdef = sg.flags & MT_SF_PDEF;
            const uint32_t c = sg.client | ((uint32_t)sg.client_hi << 8), rc = sg.rclient | ((uint32_t)sg.rclient_hi << 8);
            w = (sg.flags & MT_LSF_U16) || (c >= MT_MAX_CLIENTS && c != MT_CLIENT_NONCOLLAB) ||
                (sg.rseq >= 0 && rc >= MT_MAX_CLIENTS);
            for (int k = 0; k < MT_MAX_KEYS_WIDE; k++)
                w = w || (pdef && (k >= MT_MAX_KEYS ? sg.props[k] != 0 : sg.props[k] > 255));
            l32 = (c > 32 && c != MT_CLIENT_NONCOLLAB) || (sg.rseq >= 0 && rc > 32);
        }
        wdoc = wdoc || wave_ballot(w) != 0;
        lds = lds || wave_ballot(l32) != 0;
    }
    if (wdoc && !g.ovx) err = MT_DERR_LIMITS;  // (the engine allocates the wide state before it loads)
    const uint32_t ucap = wdoc ? g.textcap / 2 : g.textcap;  // code units per arena half
    uint16_t* arena16 = reinterpret_cast<uint16_t*>(arena);
    uint32_t carry = 0;
    bool key16 = false;  // a segment with a key >= 16: keys 16..31 in use (mt_state.h MT_WIDE_XK)
    for (int base = 0; base < ns && !err; base += 64) {
        const int i = base + lane;
        mt_load_seg sg{};
        if (i < ns) sg = segs[r0 + i];
        const uint32_t l = i < ns ? sg.text_len : 0u;
        const uint32_t incl = (uint32_t)wave_incl_scan((int)l);
        const uint32_t at = carry + incl - l;
        carry += (uint32_t)wave_last((int)incl);
        if (carry > ucap) {
            err = MT_DERR_TEXT_ARENA;
            break;
        }
        if (i < ns) {
            const bool u16 = sg.flags & MT_LSF_U16;
            const uint8_t* t = text + sg.text_off;
            auto unit = [&](uint32_t q) -> uint32_t { return u16 ? (uint32_t)t[2 * q] | ((uint32_t)t[2 * q + 1] << 8) : t[q]; };
            bool nl = false;
            for (uint32_t q = 0; q < l; q++) {
                const uint32_t c = unit(q);
                if (wdoc) arena16[at + q] = (uint16_t)c;
                else arena[at + q] = (uint8_t)c;
                nl = nl || c == '\n';
            }
            const bool rm = sg.rseq >= 0;
            const bool mk = sg.flags & MT_SF_MARKER;  // a Marker spec: one unit, its ReferenceType
            uint8_t fl = (uint8_t)((rm ? MT_SF_REMOVED : 0u) | (sg.flags & (MT_SF_PDEF | MT_SF_MARKER)) |
                                   (nl && !mk ? MT_SF_HASNL : 0u));
            if (!mk && l && unit(l - 1) == '\n') fl |= MT_SF_NL;
            uint64_t w4[8] = {};  // props as the narrow word + the wide words (keys 0..31: lo, hi per 8)
            for (int k = 0; k < MT_MAX_KEYS_WIDE; k++) {
                w4[(k >> 3) * 2] |= (uint64_t)(sg.props[k] & 0xFFu) << (8 * (k & 7));
                w4[(k >> 3) * 2 + 1] |= (uint64_t)(sg.props[k] >> 8) << (8 * (k & 7));
            }
            g.seq[so + i] = sg.seq;
            g.rseq[so + i] = rm ? sg.rseq : 0;
            g.len[so + i] = l;
            g.toff[so + i] = at;
            g.ovl[so + i] = 0;  // removedClientOverlap is not part of a snapshot
            g.props[so + i] = w4[0];
            if (wdoc) {
                for (int q = 0; q < MT_OVX_WORDS; q++) g.ovx[(so + i) * MT_OVX_WORDS + q] = 0;
                g.chi[so + i] = (uint16_t)(sg.client_hi | ((rm ? sg.rclient_hi : 0u) << 8));
                g.ph[so + i] = w4[1];
                g.pxl[so + i] = w4[2];
                g.pxh[so + i] = w4[3];
                for (int q = 0; q < 4; q++) g.pxx[4 * (so + i) + q] = w4[4 + q];
                key16 = key16 || (w4[4] | w4[5] | w4[6] | w4[7]) != 0;
            }
            g.client[so + i] = sg.client;
            g.rclient[so + i] = rm ? sg.rclient : 0;
            g.flags[so + i] = fl;
        }
    }
    if (!err) {
        // block shape, level by level: block b of a level has min(7, m - 7b) children
        int m = ns;
        for (int L = 0; L < nlev; L++) {
            uint8_t* cnt = L == 0 ? g.lbcnt + (size_t)d * g.lbcap
                                  : g.ibcnt + ((size_t)d * (MT_MAXLEV - 1) + (L - 1)) * g.ibcap;
            for (int b = lane; b < nb[L]; b += 64) {
                cnt[b] = (uint8_t)min(kPerBlock, m - kPerBlock * b);
                if (L == 0) g.lbscour[(size_t)d * g.lbcap + b] = MT_SC_UNDEF;
            }
            m = nb[L];
        }
    }
    const uint32_t lkeys = g.sc[d].label_keys;  // (declared keys outlive a load)
    const bool xl = wave_ballot(key16) != 0;
    if (lane == 0) {
        mt_doc_scalars sc{};
        sc.win_op = -1;
        sc.label_keys = lkeys;
        if (err) {  // the document keeps an empty tree and reports the error
            sc.nlev = 1;
            sc.nb[0] = 1;
            sc.n_empty = 1;
            sc.err = err;
            sc.err_seq = cur_seq[w];
            g.lbcnt[(size_t)d * g.lbcap] = 0;
            g.lbscour[(size_t)d * g.lbcap] = MT_SC_UNDEF;
        } else {
            sc.nseg = ns;
            sc.nlev = nlev;
            for (int L = 0; L < nlev; L++) sc.nb[L] = nb[L];
            sc.n_empty = ns == 0 ? 1u : 0u;
            sc.text_top = carry;
            sc.wide = (wdoc || lkeys != MT_NO_LABEL_KEYS ? MT_WIDE_LDS : 0u) | (lds ? MT_WIDE_C64 : 0u) |
                      (wdoc ? MT_WIDE_DOC : 0u) | (xl ? MT_WIDE_XK | MT_WIDE_XKV : 0u);
        }
        sc.cur_seq = cur_seq[w];
        sc.min_seq = min_seq[w];
        g.sc[d] = sc;
        g.loc[d].own = -1;
        g.loc[d].glo = g.loc[d].ghi = g.loc[d].stamp = g.loc[d].lseq = g.loc[d].rgn = g.loc[d].rgpn = 0;
    }
}

// Bin the documents that have ops in this launch by the capacity class they need.  Each op
// adds at most 2 segments (a boundary split + an insert, or two boundary splits), at most 2 leaf
// blocks, and a handful of heap entries; the register engine also pads one slot per empty leaf
// block.  classes[k] = {CAP, LB, IB, H}.  Buckets: 0 .. n_classes-1 the capacity classes,
// n_classes the editing documents, then one per class from first_wide on for the wide documents
// (include/mtgpu.h "limits"; promoted here by their first wide op or client id >= 64), then -- when
// the register engine serves classes 0 .. first_lds-1 -- one per such class for the documents that
// need the LDS engine there (declared label keys):
// the LDS engine at that class's capacity, not at first_lds's; then one per such class for the
// documents that only need 64-bit overlap sets (a client id above 32): the register engine's C64 form;
// then the editing documents' 256 / 512-slot forms, their 2048 / 4096-slot HBM-workspace forms and
// the wide-group forms (MT_WIDE_GROUPS: 256 pending edits) at 1024 / 4096 slots, then both at 8192.
// Binning is wave-aggregated: one atomic per (wave, bucket).
__global__ void mt_bin_kernel(mt_gstate g, const uint32_t* __restrict__ row_ptr, uint32_t n_docs, uint32_t op_lo,
                              uint32_t op_cnt, const int32_t* __restrict__ classes, int n_classes, int first_lds,
                              int first_wide, uint32_t* __restrict__ counts, uint32_t* __restrict__ ids,
                              const mt_op_rec* __restrict__ ops, const uint8_t* __restrict__ payload,
                              unsigned long long* __restrict__ acc) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    const int n_buckets = n_classes + 1 + (n_classes > first_wide ? n_classes - first_wide : 0) + 2 * first_lds + 8;
    int c = -1;
    unsigned long long bytes = 0;
    if (d < n_docs) {
        const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
        const uint32_t a = min(r1, r0 + op_lo);
        const uint32_t b = op_cnt ? min(r1, a + op_cnt) : r1;
        const mt_doc_scalars sc = g.sc[d];
        if (a < b && !sc.err) {
            const int nops = (int)(b - a);
            int32_t own = g.loc[d].own;
            const bool needs_lds = (sc.wide & MT_WIDE_LDS) != 0;
            bool c64 = (sc.wide & MT_WIDE_C64) != 0;
            bool wdoc = (sc.wide & MT_WIDE_DOC) != 0;
            const bool wdoc0 = wdoc;
            // snapshot body appends (MT_OP_LOAD, SnapshotLoader.loadBody) are applied by the LDS
            // engine only: the register engine's hot loop stays free of them
            bool lds_only = false, editing = own >= 0;
            const uint32_t pend = own >= 0 ? g.loc[d].ghi - g.loc[d].glo : 0u;  // pending edits
            uint32_t nloc = 0, nregen = 0;  // (an editing document: its local edits / reconnects here)
            // the wide form's extension (mt_state.h MT_WIDE_XK / MT_WIDE_XO): a property key >= 16 in
            // this launch, and removes by ids >= 64 that could grow an overlap list past 16
            bool key16 = false;
            uint32_t nrem_hi = 0;
            unsigned long long ob = 0;
            // one pass over this launch's records (each is read once: the loops below were separate)
            // (only a document with no recorded failure and no sticky error: -2 marks a record the
            // fixup consumed, and a halted document's window is never replayed again)
            bool win = ops && sc.win_op == -1 && sc.err == 0;
            int32_t cur = sc.cur_seq, mn = sc.min_seq;
            for (uint32_t i = a; ops && i < b; i++) {
                const mt_op_rec o = ops[i];
                const uint32_t ty = MT_OP_TYPE(o);
                lds_only = lds_only || ty == MT_OP_LOAD;
                editing = editing || (o.seq == -1 && o.type != MT_OP_LOAD);
                nloc += o.seq == -1 ? 1u : 0u;
                nregen += o.seq == MT_SEQ_REGEN ? 1u : 0u;
                ob += 32ull + o.payload_len;
                nrem_hi += (ty == MT_OP_REMOVE && o.client >= MT_MAX_CLIENTS) ? 1u : 0u;
                if (o.type & MT_OP_WIDE) {
                    const uint32_t np = MT_OP_NPAIRS(o);
                    if (np && (!payload || o.payload_len < 3u * np)) {
                        key16 = true;  // (unread pairs: the extension, to be safe)
                    } else {
                        const uint8_t* pp = payload + o.payload_off + (o.payload_len - 3u * np);
                        for (uint32_t q = 0; q < np; q++) key16 = key16 || pp[3 * q] >= 16;
                    }
                }
                if (!wdoc0) {
                    const uint32_t c = o.client;
                    const bool load = ty == MT_OP_LOAD;
                    const uint32_t c0 = load ? MT_LOAD_CLIENT(o) : c, c1 = load ? MT_LOAD_RCLIENT(o) : 0u;
                    const bool has0 = !load || c0 != MT_CLIENT_NONCOLLAB, has1 = load && o.pos2 >= 0;
                    c64 = c64 || (has0 && c0 > 32) || (has1 && c1 > 32);
                    wdoc = wdoc || (o.type & MT_OP_WIDE) ||
                           (load ? ((has0 && c0 >= MT_MAX_CLIENTS) || (has1 && c1 >= MT_MAX_CLIENTS))
                                 : (!MT_OP_IS_NOOP(o) && c >= MT_MAX_CLIENTS));
                }
                // replay the collab window over this launch's ops (client.ts:461-464, 821-828;
                // mergeTree.ts:1718-1722) to find the first op the apply will halt on for a window
                // assert; mt_fixup_kernel decides after the apply whether "insert failed" outranks it.
                // An editing client's local edits (seq -1) touch no window; its acks assert only in
                // updateSeqNumbers (client.ts:804-806, 821-828)
                if (!win || ty == MT_OP_LOAD) continue;  // snapshot body append: no window update
                if (ty > MT_OP_LOAD) {
                    win = false;
                    continue;
                }
                if (o.seq == -1) {
                    if (own < 0) own = o.client;
                    continue;
                }
                if (o.seq == MT_SEQ_REGEN) continue;  // reconnect: no window update
                const bool ack = (int32_t)o.client == own;
                const bool bad = (MT_OP_IS_NOOP(o) || ack) ? (!(cur <= o.seq) || !(o.msn <= o.seq) || !(mn <= o.msn))
                                                          : (!(cur < o.seq) || !(mn <= o.msn) || !(o.msn <= o.seq));
                if (bad) {
                    g.sc[d].win_op = (int32_t)i;
                    win = false;
                    continue;
                }
                if (!(o.flags & MT_F_GROUP_MORE)) {
                    cur = o.seq;
                    mn = o.msn > mn ? o.msn : mn;
                }
            }
            if (!wdoc0 && ops && c64 && !(sc.wide & MT_WIDE_C64)) g.sc[d].wide = sc.wide | MT_WIDE_C64;
            int ib_need = 0;
            for (int L = 1; L < sc.nlev; L++) ib_need = max(ib_need, sc.nb[L]);
            c = n_classes - 1;
            // (snapshot appends start at the first class the LDS engine serves)
            for (int k = lds_only ? first_lds : 0; k < n_classes; k++) {
                const int cap = classes[4 * k], lb = classes[4 * k + 1], ib = classes[4 * k + 2],
                          h = classes[4 * k + 3];
                if (sc.nseg + 2 * nops + (int)sc.n_empty + 1 <= cap && sc.nb[0] + 2 * nops + 1 <= lb &&
                    ib_need + nops + 1 <= ib && sc.heap_n + 4 * nops + 16 <= h) {
                    c = k;
                    break;
                }
            }
            const int cls = c;  // the capacity class (before the bucket remaps below)
            if (wdoc && !editing) {
                // the wide form, from the 2048 class up (the wide state is the engine's to allocate:
                // without it the document halts)
                if (!g.ovx) {
                    g.sc[d].err = MT_DERR_LIMITS;
                    g.sc[d].err_seq = ops ? ops[a].seq : 0;
                    c = -1;
                } else {
                    c = n_classes - 1;
                    for (int k = first_wide; k < n_classes; k++) {
                        const int cap = classes[4 * k], lb = classes[4 * k + 1], ib = classes[4 * k + 2],
                                  h = classes[4 * k + 3];
                        if (sc.nseg + 2 * nops + (int)sc.n_empty + 1 <= cap && sc.nb[0] + 2 * nops + 1 <= lb &&
                            ib_need + nops + 1 <= ib && sc.heap_n + 4 * nops + 16 <= h) {
                            c = k;
                            break;
                        }
                    }
                    c = n_classes + 1 + (c - first_wide);
                    const bool xk = (sc.wide & MT_WIDE_XK) || key16;
                    const bool xo = MT_WIDE_OVN(sc.wide) + nrem_hi > 16u;
                    const uint32_t w0 = g.sc[d].wide;
                    const uint32_t w1 = (w0 & ~MT_WIDE_XO) | (xk ? MT_WIDE_XK : 0u) | (xo ? MT_WIDE_XO : 0u);
                    if (w1 != w0) g.sc[d].wide = w1;
                    // (per wide bucket: how many of its documents stage the extension)
                    if (xk || xo) atomicAdd(&counts[n_buckets + (c - (n_classes + 1))], 1u);
                }
            }
            if (!wdoc && c < first_lds && (needs_lds || c64)) {
                // the LDS engine at a register class's capacity, or the register engine's C64 form
                const int lds_base = n_classes + 1 + (n_classes > first_wide ? n_classes - first_wide : 0);
                c = (needs_lds ? lds_base : lds_base + first_lds) + c;
            }
            if (editing) {
                // the editing documents' buckets (mt_launch_apply_loc): the 1024-slot form at n_classes,
                // the 256 / 512-slot forms after the C64 buckets (when the chosen class fits them), then
                // the HBM-workspace forms at 2048 / 4096 / 8192 slots (mt_launch_apply_loc_big)
                const int cap = classes[4 * cls];
                const int ebase = n_classes + 1 + (n_classes > first_wide ? n_classes - first_wide : 0) + 2 * first_lds;
                c = cap <= 256    ? ebase
                    : cap <= 512  ? ebase + 1
                    : cap <= 1024 ? n_classes
                    : cap <= 2048 ? ebase + 2
                    : cap <= 4096 ? ebase + 3
                                  : ebase + 6;
                // past 64 pending edits (or close: each local edit and each reconnect's op adds a
                // group): the form with 256 group slots, at 1024 / 4096 / 8192 slots, for good
                if ((sc.wide & MT_WIDE_GROUPS) || pend + nloc + 4u * nregen > 48u)
                    c = cap <= 1024 ? ebase + 4 : cap <= 4096 ? ebase + 5 : ebase + 7;
            }
            if (acc) {
                // algorithmic bytes of this document's share of the launch (DESIGN.md "Roofline
                // accounting"): persistent state in + out, op records, payload
                unsigned long long st = (unsigned long long)MT_SEG_STATE_BYTES * sc.nseg + 2ull * sc.nb[0] +
                                        6ull * sc.heap_n + sizeof(mt_doc_scalars);
                // an editing document's per-segment rows (group mask words, pending property counts,
                // creation stamp, localSeq pair: mt_gstate gm / pk / ct / lsq), which its form reads and
                // writes by slot during the launch: counted as state in + out like the rest
                if (editing)
                    st += (unsigned long long)(20u + 8u * ((sc.wide & MT_WIDE_GROUPS) ? MT_LOC_GW : 1u)) * sc.nseg;
                for (int L = 1; L < sc.nlev; L++) st += (unsigned long long)sc.nb[L];
                if (!ops) ob = 32ull * (b - a);  // (with records: summed in the pass above)
                bytes = 2ull * st + ob;
            }
        }
    }
    const int lane = (int)(threadIdx.x & 63u);
    for (int k = 0; k < n_buckets; k++) {
        const uint64_t m = wave_ballot(c == k);
        if (!m) continue;
        const int leader = first_lane(m);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&counts[k], (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, leader, 64);
        if (c == k) ids[(size_t)k * n_docs + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = d;
        if (acc) {
            unsigned long long v = c == k ? bytes : 0ull;
            for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
            if (lane == leader) atomicAdd(&acc[k], v);
        }
    }
}

// After an apply: a document halted on a window assert by an insert with text reports "MergeTree
// insert failed" instead when the insert was also past the end of its view -- the reference
// applies the op (mergeTree.ts:2210-2216 throws) before completeAndLogOp's and updateSeqNumbers'
// asserts (client.ts:461-464, 826).  The halted state is the state before that op, so
// getLength(refSeq, client) is read from HBM.  One thread per document; the loop runs only for
// such (rare) documents.
__global__ void mt_fixup_kernel(mt_gstate g, const mt_op_rec* __restrict__ ops, uint32_t n_docs) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n_docs) return;
    const mt_doc_scalars sc = g.sc[d];
    if (sc.win_op < 0) return;
    // consumed: the index names a record of this batch only, which a later batch's fixup must not read
    g.sc[d].win_op = -2;
    if (sc.err != MT_DERR_SEQ_ORDER && sc.err != MT_DERR_MSN_ORDER) return;
    const mt_op_rec o = ops[sc.win_op];
    if (o.seq != sc.err_seq || MT_OP_TYPE(o) != MT_OP_INSERT || o.payload_len <= MT_OP_PAIRS_LEN(o)) return;
    const size_t so = (size_t)d * g.segcap;
    const int32_t R = o.ref_seq;
    const uint32_t C = o.client;
    const bool wdoc = (sc.wide & MT_WIDE_DOC) != 0;
    const int form = mt_form(wdoc, sc.wide);
    int64_t len = 0;
    for (int i = 0; i < sc.nseg; i++) {  // nodeLength leaf branch (mergeTree.ts:1667-1697)
        // (an editing client's pending local edits carry seq / removedSeq -1, UnassignedSequenceNumber,
        // which no refSeq has seen)
        const bool seen = mt_gclient(g, wdoc, so + i) == C || (g.seq[so + i] != -1 && g.seq[so + i] <= R);
        const bool ov = C < 64 ? ((g.ovl[so + i] >> C) & 1ull) != 0
                               : (wdoc && mt_ovx_has2(mt_govx_lo(g, so + i), mt_govx_hi(g, form, so + i), C));
        const bool hid = (g.flags[so + i] & MT_SF_REMOVED) &&
                         (mt_grclient(g, wdoc, so + i) == C || ov || (g.rseq[so + i] != -1 && g.rseq[so + i] <= R));
        if (seen && !hid) len += g.len[so + i];
    }
    if ((int64_t)o.pos1 > len) g.sc[d].err = MT_DERR_INSERT_FAILED;
}

// checksum of the canonical state (mt_checksum.h), one wave per document
__global__ __launch_bounds__(64) void mt_checksum_kernel(mt_gstate g, uint32_t n_docs, uint64_t* __restrict__ out) {
    const uint32_t d = blockIdx.x;
    if (d >= n_docs) return;
    const int lane = lane_id();
    const mt_doc_scalars sc = g.sc[d];
    const size_t so = (size_t)d * g.segcap;
    const bool wdoc = (sc.wide & MT_WIDE_DOC) != 0;
    const int form = mt_form(wdoc, sc.wide);
    uint64_t seg_sum = 0;
    for (int i = lane; i < sc.nseg; i += 64) {
        uint64_t h = MT_FNV_INIT;
        const uint32_t t0 = g.toff[so + i], tl = g.len[so + i];
        for (uint32_t q = 0; q < tl; q++) h = mt_fnv1a_step(h, mt_gtext(g, d, sc, t0 + q));
        const uint8_t f = g.flags[so + i];
        if (f & MT_SF_MARKER) h ^= MT_MARKER_TAG;  // a Marker: its ReferenceType byte, tagged
        const bool rm = f & MT_SF_REMOVED;
        seg_sum += mt_seg_hash((uint64_t)i, h, g.seq[so + i], mt_canon_client(mt_gclient(g, wdoc, so + i)),
                               rm ? g.rseq[so + i] : -1, rm ? (int32_t)mt_grclient(g, wdoc, so + i) : -1,
                               mt_govl_term(g, form, so + i),
                               mt_gprops_term(g, form, so + i), (f & MT_SF_PDEF) ? 1u : 0u);
    }
    uint64_t tree_sum = 0;
    for (int L = 0; L < sc.nlev; L++) {
        const uint64_t depth = (uint64_t)(sc.nlev - 1 - L);
        const uint8_t* cnt = L == 0 ? g.lbcnt + (size_t)d * g.lbcap
                                    : g.ibcnt + ((size_t)d * (MT_MAXLEV - 1) + (L - 1)) * g.ibcap;
        for (int b = lane; b < sc.nb[L]; b += 64) tree_sum += mt_tree_term(cnt[b], (uint64_t)b, depth);
    }
    // wave sums of 64-bit values
    for (int o = 1; o < 64; o <<= 1) {
        seg_sum += (uint64_t)__shfl_xor((unsigned long long)seg_sum, o, 64);
        tree_sum += (uint64_t)__shfl_xor((unsigned long long)tree_sum, o, 64);
    }
    if (lane == 0) out[d] = mt_finish_checksum(seg_sum, tree_sum, sc.cur_seq, sc.min_seq, (uint32_t)sc.nseg);
}

extern "C" hipError_t mt_launch_init(const mt_gstate* g, uint32_t n_docs, hipStream_t st) {
    hipLaunchKernelGGL(mt_init_kernel, dim3((n_docs + 255) / 256), dim3(256), 0, st, *g, n_docs);
    return hipGetLastError();
}
extern "C" hipError_t mt_launch_load(const mt_gstate* g, uint32_t n, const uint32_t* doc_ids, const uint32_t* row_ptr,
                                     const mt_load_seg* segs, const uint8_t* text, const int32_t* min_seq,
                                     const int32_t* cur_seq, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_load_kernel, dim3(n), dim3(64), 0, st, *g, n, doc_ids, row_ptr, segs, text, min_seq,
                       cur_seq);
    return hipGetLastError();
}
extern "C" hipError_t mt_launch_bin(const mt_gstate* g, const uint32_t* row_ptr, uint32_t n_docs, uint32_t op_lo,
                                    uint32_t op_cnt, const int32_t* classes, int n_classes, int first_lds,
                                    int first_wide, uint32_t* counts, uint32_t* ids, const mt_op_rec* ops,
                                    const uint8_t* payload, unsigned long long* acc, hipStream_t st) {
    hipLaunchKernelGGL(mt_bin_kernel, dim3((n_docs + 255) / 256), dim3(256), 0, st, *g, row_ptr, n_docs, op_lo, op_cnt,
                       classes, n_classes, first_lds, first_wide, counts, ids, ops, payload, acc);
    return hipGetLastError();
}
// The host's record check (mt_engine.cpp scan_records) on the device, for a feed's first tick, whose
// host check would otherwise sit between the start and the first copy: bit 0 of *flags a payload
// out of bounds, bit 1 a record that needs the wide document form (wide_rec).  Reads the records
// only (no payload, no document state): a refused tick leaves every document as it was.
__global__ __launch_bounds__(256) void mt_scan_records_kernel(const mt_op_rec* __restrict__ ops, uint64_t n_ops,
                                                              uint64_t payload_bytes, uint32_t* __restrict__ flags) {
    uint32_t f = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_ops; i += (uint64_t)gridDim.x * blockDim.x) {
        const mt_op_rec o = ops[i];
        if ((uint64_t)o.payload_off + o.payload_len > payload_bytes) f |= 1u;
        bool wide = (o.type & MT_OP_WIDE) != 0;
        if (MT_OP_TYPE(o) == MT_OP_LOAD) {
            const uint32_t c0 = MT_LOAD_CLIENT(o), c1 = MT_LOAD_RCLIENT(o);
            wide = wide || (c0 != MT_CLIENT_NONCOLLAB && c0 >= MT_MAX_CLIENTS) || (o.pos2 >= 0 && c1 >= MT_MAX_CLIENTS);
        } else {
            wide = wide || (!MT_OP_IS_NOOP(o) && o.client >= MT_MAX_CLIENTS);
        }
        if (wide) f |= 2u;
    }
    // one atomic per wave (vector memory atomics)
    const uint64_t bad = __ballot(f & 1u), wide = __ballot(f & 2u);
    if ((threadIdx.x & 63) == 0 && (bad || wide)) atomicOr(flags, (bad ? 1u : 0u) | (wide ? 2u : 0u));
}
extern "C" hipError_t mt_launch_scan_records(const mt_op_rec* ops, uint64_t n_ops, uint64_t payload_bytes,
                                             uint32_t* flags, hipStream_t st) {
    hipError_t r = hipMemsetAsync(flags, 0, sizeof(uint32_t), st);
    if (r != hipSuccess || n_ops == 0) return r;
    const uint64_t blocks = (n_ops + 255) / 256 < 4096 ? (n_ops + 255) / 256 : 4096;
    hipLaunchKernelGGL(mt_scan_records_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, ops, n_ops, payload_bytes, flags);
    return hipGetLastError();
}
extern "C" hipError_t mt_launch_fixup(const mt_gstate* g, const mt_op_rec* ops, uint32_t n_docs, hipStream_t st) {
    if (n_docs == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_fixup_kernel, dim3((n_docs + 255) / 256), dim3(256), 0, st, *g, ops, n_docs);
    return hipGetLastError();
}
// The leaf block holding segment ib, as its position range [*lo, *hi) ([n, n) for ib < 0)
MT_DEV void mt_leaf_block_of(const mt_gstate& g, uint32_t d, const mt_doc_scalars& sc, int ib, int* lo, int* hi) {
    *lo = *hi = sc.nseg;
    if (ib < 0) return;
    const uint8_t* cnt = g.lbcnt + (size_t)d * g.lbcap;
    const int nb = sc.nb[0];
    int carry = 0;
    for (int base = 0; base < nb; base += 64) {
        const int b = base + lane_id();
        const int c = b < nb ? (int)cnt[b] : 0;
        const int incl = wave_incl_scan(c) + carry;
        const uint64_t m = wave_ballot(b < nb && c > 0 && incl - c <= ib && ib < incl);
        if (m) {
            const int l = first_lane(m);
            *lo = __builtin_amdgcn_readlane(incl - c, l);
            *hi = __builtin_amdgcn_readlane(incl, l);
            return;
        }
        carry = wave_last(incl);
    }
}
// The value id of label key `key` of segment i as the query sees it: a stale marker (MT_SF_STALE) outside
// the search path's leaf block [blo, bhi) answers with the labels its block's caches still hold
// (HierMergeBlock rightmostTiles / leftmostTiles / rangeStacks, rebuilt by blockUpdate only)
MT_DEV uint32_t mt_label_vid(const mt_gstate& g, int form, size_t so, int i, uint32_t key, uint32_t lkeys, int blo,
                             int bhi) {
    uint32_t v = mt_gprop(g, form, so + i, key);
    if (lkeys != MT_NO_LABEL_KEYS && g.slab && (i < blo || i >= bhi) && (g.flags[so + i] & MT_SF_STALE)) {
        const uint32_t sl = g.slab[so + i];
        if (key == (lkeys & 0xFFu)) v = sl & 0xFFFFu;
        else if (key == ((lkeys >> 8) & 0xFFu)) v = sl >> 16;
    }
    return v;
}
// the segment whose local-view range holds pos (the leaf search() stops on), -1 past the end
MT_DEV int mt_containing(const mt_gstate& g, size_t so, int n, int pos) {
    int carry = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane_id();
        const int ll = (i < n && !(g.flags[so + i] & MT_SF_REMOVED)) ? (int)g.len[so + i] : 0;
        const int incl = wave_incl_scan(ll) + carry;
        const uint64_t m = wave_ballot(i < n && ll > 0 && incl - ll <= pos && pos < incl);
        if (m) return base + first_lane(m);
        carry = wave_last(incl);
    }
    return -1;
}

// mt_find_tiles: Client.findTile for a batch of queries, one wave per query, over the document's
// compact HBM state in the local view (include/mtgpu.h; mergeTree.ts:1763-1870, 996-1035)
__global__ __launch_bounds__(64) void mt_tiles_kernel(mt_gstate g, const mt_tile_query* __restrict__ q, uint32_t nq,
                                                      mt_tile_result* __restrict__ out) {
    const uint32_t w = blockIdx.x;
    if (w >= nq) return;
    const int lane = lane_id();
    const mt_tile_query qq = q[w];
    const uint32_t d = qq.doc;
    const mt_doc_scalars sc = g.sc[d];
    const int n = sc.nseg;
    const size_t so = (size_t)d * g.segcap;
    const bool wdoc = (sc.wide & MT_WIDE_DOC) != 0;
    const int pos = qq.pos;
    int blo = n, bhi = n;  // the search path's leaf block (its tiles answer with their current labels)
    auto labeled = [&](int i) -> bool {  // refHasTileLabel (mergeTree.ts:581-597)
        if (qq.key >= MT_MAX_KEYS_WIDE || !(g.flags[so + i] & MT_SF_MARKER) || !(mt_gtext(g, d, sc, g.toff[so + i]) & 1u))
            return false;
        const uint32_t v = mt_label_vid(g, mt_form(wdoc, sc.wide), so, i, qq.key, sc.label_keys, blo, bhi);
        return v != 0 && v < 256 && ((qq.vmask[v >> 5] >> (v & 31)) & 1u);
    };
    auto local_len = [&](int i) -> int { return (g.flags[so + i] & MT_SF_REMOVED) ? 0 : (int)g.len[so + i]; };
    int res = -1, rpos = -1;
    if (qq.preceding) {
        // search: the last live tile at a position <= pos (shifted children's rightmostTiles, then
        // the leaf holding pos)
        if (sc.label_keys != MT_NO_LABEL_KEYS) mt_leaf_block_of(g, d, sc, mt_containing(g, so, n, pos), &blo, &bhi);
        int carry = 0;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            const int ll = i < n ? local_len(i) : 0;
            const int incl = wave_incl_scan(ll);
            const int start = carry + incl - ll;
            const bool cand = i < n && ll > 0 && start <= pos && labeled(i);
            const uint64_t m = wave_ballot(cand);
            if (m) {
                const int l = 63 - __builtin_clzll(m);
                res = base + l;
                rpos = __builtin_amdgcn_readlane(start, l);
            }
            if (__builtin_amdgcn_readfirstlane(start) > pos) break;
            carry += wave_last(incl);
        }
    } else {
        int total = 0;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            total += wave_sum(i < n ? local_len(i) : 0);
        }
        if (pos <= total && n > 0) {
            // the leaf backwardSearch stops on: the last segment starting at or before pos
            int carry = 0, is = -1, istart = 0, base = 0;
            for (; base < n; base += 64) {
                const int i = base + lane;
                const int ll = i < n ? local_len(i) : 0;
                const int incl = wave_incl_scan(ll);
                const int start = carry + incl - ll;
                const uint64_t m = wave_ballot(i < n && start <= pos);
                if (m) {
                    const int l = 63 - __builtin_clzll(m);
                    is = base + l;
                    istart = __builtin_amdgcn_readlane(start, l);
                }
                if (m != ~0ull) break;
                carry += wave_last(incl);
            }
            // ... unless a trailing empty leaf block comes after it at that same position
            const bool trailing_empty = is == n - 1 && pos == total && sc.nb[0] > 0 &&
                                        g.lbcnt[(size_t)d * g.lbcap + sc.nb[0] - 1] == 0;
            if (sc.label_keys != MT_NO_LABEL_KEYS) mt_leaf_block_of(g, d, sc, is, &blo, &bhi);
            if (!trailing_empty) {
                if (labeled(is)) {  // recordTileStart: removed or not
                    res = is;
                    rpos = istart;
                } else {
                    // the first live tile after it (shifted children's leftmostTiles)
                    int c2 = istart + local_len(is);
                    for (int b2 = is + 1; b2 < n && res < 0; b2 += 64) {
                        const int i = b2 + lane;
                        const int ll = i < n ? local_len(i) : 0;
                        const int incl = wave_incl_scan(ll);
                        const uint64_t m = wave_ballot(i < n && ll > 0 && labeled(i));
                        if (m) {
                            const int l = __builtin_ctzll(m);
                            res = b2 + l;
                            rpos = c2 + __builtin_amdgcn_readlane(incl - ll, l);
                        }
                        c2 += wave_last(incl);
                    }
                }
            }
        }
    }
    if (lane == 0) {
        out[w].pos = res >= 0 ? rpos : -1;
        out[w].ordinal = res;
    }
}

extern "C" hipError_t mt_launch_tiles(const mt_gstate* g, const mt_tile_query* q, uint32_t n, mt_tile_result* out,
                                      hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_tiles_kernel, dim3(n), dim3(64), 0, st, *g, q, n, out);
    return hipGetLastError();
}

// mt_resolve_positions: MergeTree.getContainingSegment / getPosition for a batch of queries, one wave
// per query over the document's compact state in HBM (include/mtgpu.h).  The B-tree walk of
// searchBlock (mergeTree.ts:1797-1829) descends into the first child whose length in the view exceeds
// what is left of pos; over the leaves in order that is the first leaf whose inclusive view prefix
// exceeds pos -- a wave prefix sum per 64 leaves, stopping at the chunk that holds it.  getPosition
// (mergeTree.ts:1585-1602) sums the local view's lengths before the leaf.
__global__ __launch_bounds__(64) void mt_resolve_kernel(mt_gstate g, const mt_pos_query* __restrict__ q, uint32_t nq,
                                                        uint32_t n_docs, mt_pos_result* __restrict__ out) {
    const uint32_t w = blockIdx.x;
    if (w >= nq) return;
    const int lane = lane_id();
    const mt_pos_query qq = q[w];
    const uint32_t d = qq.doc;
    if (d >= n_docs || qq.kind > MT_POS_OF_ORDINAL) {  // (device-resident queries are not checked on the host)
        if (lane == 0) out[w] = mt_pos_result{MT_POS_BAD_QUERY, 0, 0, 0};
        return;
    }
    const mt_doc_scalars sc = g.sc[d];
    const int n = sc.nseg;
    const size_t so = (size_t)d * g.segcap;
    const bool wdoc = (sc.wide & MT_WIDE_DOC) != 0;
    const int form = mt_form(wdoc, sc.wide);
    const bool local = qq.ref_seq == MT_POS_LOCAL;
    const int32_t R = qq.ref_seq;
    const uint32_t C = qq.client;
    auto view_len = [&](int i) -> int {  // nodeLength's leaf branch (mergeTree.ts:1659-1697)
        const bool rm = (g.flags[so + i] & MT_SF_REMOVED) != 0;
        if (local) return rm ? 0 : (int)g.len[so + i];
        // (pending local edits: seq / removedSeq -1, UnassignedSequenceNumber, seen by no refSeq)
        const bool seen = mt_gclient(g, wdoc, so + i) == C || (g.seq[so + i] != -1 && g.seq[so + i] <= R);
        const bool ov = C < 64 ? ((g.ovl[so + i] >> C) & 1ull) != 0
                               : (wdoc && mt_ovx_has2(mt_govx_lo(g, so + i), mt_govx_hi(g, form, so + i), C));
        const bool hid = rm && (mt_grclient(g, wdoc, so + i) == C || ov || (g.rseq[so + i] != -1 && g.rseq[so + i] <= R));
        return (seen && !hid) ? (int)g.len[so + i] : 0;
    };
    mt_pos_result r{-1, 0, 0, 0};
    int vcarry = 0, lcarry = 0;
    const bool by_ord = qq.kind == MT_POS_OF_ORDINAL;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const int vl = i < n ? view_len(i) : 0;
        const int ll = (i < n && !(g.flags[so + i] & MT_SF_REMOVED)) ? (int)g.len[so + i] : 0;
        const int vincl = vcarry + wave_incl_scan(vl);
        const int lincl = lcarry + wave_incl_scan(ll);
        const uint64_t m = wave_ballot(i < n && (by_ord ? i == qq.pos : qq.pos < vincl));
        if (m) {
            const int l = first_lane(m);
            r.ordinal = base + l;
            r.offset = qq.pos - __builtin_amdgcn_readlane(vincl - vl, l);
            r.position = __builtin_amdgcn_readlane(lincl - ll, l);
            r.length = g.len[so + base + l];
            if (by_ord) r.offset = 0;
            break;
        }
        vcarry = __builtin_amdgcn_readlane(vincl, 63);
        lcarry = __builtin_amdgcn_readlane(lincl, 63);
    }
    if (r.ordinal < 0) {  // none: offset = pos minus the view's length, position = the local length
        r.offset = qq.pos - vcarry;
        r.position = lcarry;
    }
    if (lane == 0) out[w] = r;
}

// mt_segment_infos: one thread per (document, ordinal) pair gathers the segment's fields
__global__ void mt_seginfo_kernel(mt_gstate g, const uint32_t* __restrict__ docs, const int32_t* __restrict__ ords,
                                  uint32_t n, mt_seg_info* __restrict__ out) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n) return;
    const uint32_t d = docs[w];
    const int32_t i = ords[w];
    const mt_doc_scalars sc = g.sc[d];
    mt_seg_info r{};
    r.seq = INT32_MIN;
    if (i >= 0 && i < sc.nseg) {
        const size_t so = (size_t)d * g.segcap + i;
        const bool wdoc = (sc.wide & MT_WIDE_DOC) != 0 && g.ovx;
        const uint8_t f = g.flags[so];
        const bool rm = (f & MT_SF_REMOVED) != 0;
        r.seq = g.seq[so];
        r.rseq = rm ? g.rseq[so] : -1;
        r.client = mt_canon_client(mt_gclient(g, wdoc, so));
        r.rclient = rm ? (int32_t)mt_grclient(g, wdoc, so) : -1;
        r.len = g.len[so];
        r.flags = f & (MT_SF_REMOVED | MT_SF_PDEF | MT_SF_MARKER);
        r.toff = g.toff[so];
        r.wide = wdoc ? 1u : 0u;
        r.overlap = g.ovl[so];
        const int form = mt_form(wdoc, sc.wide);
        for (int q = 0; q < MT_OVX_IDS; q++)
            r.overlap_hi[q] = wdoc ? (uint16_t)mt_ovx_id2(mt_govx_lo(g, so), mt_govx_hi(g, form, so), q) : 0;
        for (int k = 0; k < MT_MAX_KEYS_WIDE; k++) r.props[k] = (uint16_t)mt_gprop(g, form, so, k);
    }
    out[w] = r;
}

// mt_range_stacks: Client.getStackContext for a batch of (document, position, label) queries, one wave
// per query (include/mtgpu.h; mergeTree.ts:1750-1760, 953-994, 246-261).  The stack is always its
// unmatched ends followed by its unmatched begins (an end is pushed only when the top is not a
// begin), so the fold needs only the two lengths: ends `a`, depth `t`; the top is a begin iff t > a.
__global__ __launch_bounds__(64) void mt_stacks_kernel(mt_gstate g, const mt_tile_query* __restrict__ q, uint32_t nq,
                                                       uint32_t cap, mt_stack_item* __restrict__ items,
                                                       uint32_t* __restrict__ depth) {
    const uint32_t w = blockIdx.x;
    if (w >= nq) return;
    const int lane = lane_id();
    const mt_tile_query qq = q[w];
    const uint32_t d = qq.doc;
    const mt_doc_scalars sc = g.sc[d];
    const int n = sc.nseg;
    const size_t so = (size_t)d * g.segcap;
    const bool wdoc = (sc.wide & MT_WIDE_DOC) != 0;
    const int pos = qq.pos;
    mt_stack_item* out = items + (size_t)w * cap;
    int a = 0, t = 0, carry = 0;
    bool touched = false;
    int blo = n, bhi = n;  // the search path's leaf block (its markers fold with their current labels)
    if (sc.label_keys != MT_NO_LABEL_KEYS) mt_leaf_block_of(g, d, sc, mt_containing(g, so, n, pos), &blo, &bhi);
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const int ll = (i < n && !(g.flags[so + i] & MT_SF_REMOVED)) ? (int)g.len[so + i] : 0;
        const int incl = wave_incl_scan(ll);
        const int start = carry + incl - ll;
        uint32_t rt = 0;
        bool cand = false;
        if (i < n && ll > 0 && start <= pos && qq.key < MT_MAX_KEYS_WIDE && (g.flags[so + i] & MT_SF_MARKER)) {
            rt = mt_gtext(g, d, sc, g.toff[so + i]);
            const uint32_t v = mt_label_vid(g, mt_form(wdoc, sc.wide), so, i, qq.key, sc.label_keys, blo, bhi);
            cand = (rt & 6u) && v != 0 && v < 256 && ((qq.vmask[v >> 5] >> (v & 31)) & 1u);
        }
        uint64_t m = wave_ballot(cand);
        touched |= m != 0;
        while (m) {  // applyRangeReference for each, in document order
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t r = __builtin_amdgcn_readlane(rt, l);
            int slot = -1;
            if (r & 2u) {
                slot = t++;
            } else if (t > a) {
                t--;
            } else {
                slot = t++;
                a = t;
            }
            if (slot >= 0 && slot < (int)cap && lane == l) out[slot] = mt_stack_item{start, i, r};
        }
        if (__builtin_amdgcn_readfirstlane(start) > pos) break;
        carry += wave_last(incl);
    }
    if (lane == 0) depth[w] = (uint32_t)t | (touched ? MT_STACK_TOUCHED : 0u);
}

extern "C" hipError_t mt_launch_stacks(const mt_gstate* g, const mt_tile_query* q, uint32_t n, uint32_t cap,
                                       mt_stack_item* items, uint32_t* depth, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_stacks_kernel, dim3(n), dim3(64), 0, st, *g, q, n, cap, items, depth);
    return hipGetLastError();
}

// mt_events_drain: document d's recorded events (at most evcap) to out + off[d], one wave per document
__global__ __launch_bounds__(64) void mt_events_pack_kernel(mt_gstate g, uint32_t n_docs, const uint64_t* __restrict__ off,
                                                           mt_event* __restrict__ out) {
    const uint32_t d = blockIdx.x;
    if (d >= n_docs) return;
    const uint32_t n = min(g.evn[d], g.evcap);
    const mt_event* src = g.ev + (size_t)d * g.evcap;
    mt_event* dst = out + off[d];
    for (uint32_t i = threadIdx.x; i < n; i += 64) dst[i] = src[i];
}

extern "C" hipError_t mt_launch_events_pack(const mt_gstate* g, uint32_t n_docs, const uint64_t* off, mt_event* out,
                                            hipStream_t st) {
    if (n_docs == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_events_pack_kernel, dim3(n_docs), dim3(64), 0, st, *g, n_docs, off, out);
    return hipGetLastError();
}

extern "C" hipError_t mt_launch_checksum(const mt_gstate* g, uint32_t n_docs, uint64_t* out, hipStream_t st) {
    hipLaunchKernelGGL(mt_checksum_kernel, dim3(n_docs), dim3(64), 0, st, *g, n_docs, out);
    return hipGetLastError();
}

// SnapshotV1.extractSync (packages/dds/merge-tree/src/snapshotV1.ts:151-247) for every document
// of [d0, d0 + n_docs), one wave per document: each segment is classified lane-parallel (elided:
// removed at or below the MSN; coalescable: acked below the MSN and live; else it keeps its merge
// info), then the coalescing decisions (canAppend textSegment.ts:63-68 on the run so far,
// matchProperties properties.ts:62-93) run in order over the lanes with readlane.  Output per
// document: specs of 3 u32 {first segment position, span << 1 | has_merge_info, text length},
// at most nseg of them, and their count.  A coalesced run spans the positions from its first to its
// last segment; the elided segments inside it (removed at or below the MSN) are not part of it.
__global__ __launch_bounds__(64) void mt_snapshot_kernel(mt_gstate g, uint32_t d0, uint32_t n_docs, uint32_t cap,
                                                         uint32_t* __restrict__ specs, uint32_t* __restrict__ counts) {
    const uint32_t w = blockIdx.x;
    if (w >= n_docs) return;
    const uint32_t d = d0 + w;
    const int lane = lane_id();
    const mt_doc_scalars sc = g.sc[d];
    const int n = sc.nseg;
    const int32_t msn = sc.min_seq;
    const size_t so = (size_t)d * g.segcap;
    const bool wdoc = (sc.wide & MT_WIDE_DOC) != 0;
    const int form = mt_form(wdoc, sc.wide);
    uint32_t* out = specs + (size_t)w * cap * 3;
    int k = 0;
    bool have = false;
    int ps = 0, pc = 0;
    uint32_t plen = 0, pfl = 0;
    uint64_t pprops = 0;  // the run's props (narrow word; a wide document compares all words in HBM)
    auto emit = [&](int pos, int cnt, bool meta, uint32_t len) {
        if (lane == 0 && k < (int)cap) {
            out[3 * k] = (uint32_t)pos;
            out[3 * k + 1] = ((uint32_t)cnt << 1) | (meta ? 1u : 0u);
            out[3 * k + 2] = len;
        }
        k++;
    };
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        int cls = 0;  // 0 elided, 1 coalescable, 2 merge info
        uint32_t len = 0, fl = 0;
        uint64_t pr = 0;
        if (i < n) {
            fl = g.flags[so + i];
            len = g.len[so + i];
            pr = g.props[so + i];
            const bool rm = fl & MT_SF_REMOVED;
            const int32_t s = g.seq[so + i];
            if (s == -1 || (rm && g.rseq[so + i] <= msn)) cls = 0;  // pending insert / removal (snapshotV1.ts:184)
            else if (s <= msn && !rm) cls = 1;
            else cls = 2;
        }
        const int m = min(64, n - base);
        for (int j = 0; j < m; j++) {
            const int c = __builtin_amdgcn_readlane(cls, j);
            if (c == 0) continue;
            const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)len, j);
            if (c == 2) {
                if (have) emit(ps, pc, false, plen);
                have = false;
                emit(base + j, 1, true, lj);
                continue;
            }
            const uint32_t fj = (uint32_t)__builtin_amdgcn_readlane((int)fl, j);
            const uint64_t pj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pr, j) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pr >> 32), j) << 32);
            if (have && !((pfl | fj) & MT_SF_MARKER) && !(pfl & MT_SF_NL) && (plen <= 256u || lj <= 256u) &&
                ((pfl ^ fj) & MT_SF_PDEF) == 0 &&
                pprops == pj && (!wdoc || mt_gprops_eq(g, form, so + ps, so + base + j))) {
                pc = base + j - ps + 1;  // span from the run's first segment (elided ones inside it skipped by the reader)
                plen += lj;
                pfl = (pfl & ~MT_SF_NL) | (fj & MT_SF_NL);
            } else {
                if (have) emit(ps, pc, false, plen);
                have = true;
                ps = base + j;
                pc = 1;
                plen = lj;
                pfl = fj;
                pprops = pj;
            }
        }
    }
    if (have) emit(ps, pc, false, plen);
    if (lane == 0) counts[w] = (uint32_t)k;
}

extern "C" hipError_t mt_launch_snapshot(const mt_gstate* g, uint32_t d0, uint32_t n_docs, uint32_t cap,
                                         uint32_t* specs, uint32_t* counts, hipStream_t st) {
    if (n_docs == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_snapshot_kernel, dim3(n_docs), dim3(64), 0, st, *g, d0, n_docs, cap, specs, counts);
    return hipGetLastError();
}

extern "C" hipError_t mt_launch_resolve(const mt_gstate* g, const mt_pos_query* q, uint32_t n, uint32_t n_docs, mt_pos_result* out,
                                        hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_resolve_kernel, dim3(n), dim3(64), 0, st, *g, q, n, n_docs, out);
    return hipGetLastError();
}
extern "C" hipError_t mt_launch_seginfo(const mt_gstate* g, const uint32_t* docs, const int32_t* ords, uint32_t n,
                                        mt_seg_info* out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mt_seginfo_kernel, dim3((n + 255) / 256), dim3(256), 0, st, *g, docs, ords, n, out);
    return hipGetLastError();
}
