// mt_deli.hip -- deli ticketing for many documents at once and its C-ABI
// (include/mtgpu.h, "deli" section).
//
// The reference sequences one document per DeliLambda: every raw message goes through
// ticket() (server/routerlicious/packages/lambdas/src/deli/lambda.ts:255-544), which checks the
// client's sequence order, tracks joined clients in a ClientSequenceNumberManager
// (deli/clientSeqManager.ts:70-143, a binary heap on referenceSequenceNumber) and assigns
// sequenceNumber / minimumSequenceNumber.  Messages of one document are strictly sequential,
// documents are independent.
//
// Device mapping: eight documents per wave64, eight lanes per document, each lane owning eight
// client records in VGPRs, so the heap becomes a group-wide min (no data-dependent memory
// traffic) and the per-message decision tree runs as VALU selects on all four SIMDs of a CU
// (see deli_kernel).  HBM traffic is the algorithmic minimum: 16 B in + 16 B out per message,
// plus 9 B per client slot and 20 B of scalars in and out per document.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/mtgpu.h"
#include "mt_wave.h"

namespace mtd {

enum : int { CL_JOINED = 1, CL_NACK = 2 };

// per-document state in HBM (structure of arrays; client arrays are [doc * 64 + client]); a
// document that ever sees a client id >= 64 is promoted, for good, to a row of the big pool
// ([row * MT_DELI_MAX_CLIENTS + client]) and ticketed by the wide form (one document per wave)
struct DeliState {
    int4* sc;         // {sequenceNumber, minimumSequenceNumber, lastSentMSN, err}
    int32_t* err_at;  // message index (inside the document's stream) of the sticky error
    int32_t* csn;
    int32_t* ref;
    uint8_t* fl;      // CL_JOINED | CL_NACK
    uint32_t* big;    // per document: its row of the big pool, or kNoRow
    int32_t* bcsn;    // big pool: [row][MT_DELI_MAX_CLIENTS]
    int32_t* bref;
    uint8_t* bfl;
    uint32_t big_cap; // rows in the big pool
    // [0] rows handed out fresh (a count that may pass big_cap: the attempts), [1] documents queued
    // for the wide form in this call, [2] rows on the free list (as int: the kernel's pops may take it
    // below zero, which reads as empty; the host repairs it before it pushes)
    uint32_t* ctl;
    uint32_t* free_rows;  // [big_cap]: rows given back by restored documents, a stack of ctl[2]
    uint32_t* queue;  // [max_docs]: those documents
    int32_t* resume;  // per queued document: its first message the wide form tickets
};
constexpr uint32_t kNoRow = 0xFFFFFFFFu;

constexpr int kPerLane = 8;                           // client slots per lane
typedef int32_t V8 __attribute__((ext_vector_type(kPerLane)));

// min over the G lanes of a document's group, in every lane of the group: G = 8 with quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], then row_half_mirror (lane i <-> 7-i inside each half-row); G = 64
// the whole wave
template <int G>
MT_DEV int group_min(int v) {
    if constexpr (G == 64) {
        return wave_min(v);
    } else {
        v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0xB1, 0xf, 0xf, false));
        v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x4E, 0xf, 0xf, false));
        v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x141, 0xf, 0xf, false));
        return v;
    }
}
// slot k of a lane's 8 client slots (k differs between groups: a select chain, not an index)
MT_DEV int pick(const V8& a, int k) {
    int r = a[0];
#pragma unroll
    for (int i = 1; i < kPerLane; i++) r = k == i ? a[i] : r;
    return r;
}

// One document per group of G lanes, lane q of the group owning the document's clients
// 8q..8q+7 (csn, refSeq in VGPRs; joined / nacked as 2-bit fields of one VGPR): G = 8, eight
// documents per wave, 64 clients each (the common form); G = 64, one document per wave with 512
// (the wide form, for documents past client 63).  Every branch of ticket() is evaluated as per-lane
// selects, so the CU's four SIMDs do the work in parallel (a wave-per-document form runs the
// decision tree on the CU's single scalar unit).  A client lookup is one ds_bpermute from its owner
// lane; the heap minimum is 8 local mins and a group reduction.  Messages are staged through LDS G
// per document at a time (one coalesced 16-byte load per lane, prefetched a chunk ahead); tickets
// go back the same way.  Messages [m0, len) of the document's stream are ticketed; in the G = 8 form
// a message from a client >= 64 stops the document there and queues it for the wide form
// (`stop`), which promotes it and tickets the rest.
template <int G>
MT_DEV void deli_group(DeliState& g, const int4* __restrict__ msgs, uint32_t d, bool live, uint32_t r0, int len,
                       int m0, int32_t* ccsn_p, int32_t* cref_p, uint8_t* cfl_p, int4* __restrict__ out,
                       mt_op_rec* __restrict__ ops, uint64_t n_ops, int4 (&stage)[64]) {
    constexpr int NC = G * kPerLane;  // clients this form holds
    const int lane = lane_id();
    const int li = lane & (G - 1), gbase = lane & ~(G - 1);
    int4 s0 = make_int4(0, 0, 0, 0);
    int err_at = -1;
    V8 csn = 0, ref = 0;
    uint32_t fl = 0;
    if (live) {
        s0 = g.sc[d];
        err_at = g.err_at[d];
        const int4 c0 = *reinterpret_cast<const int4*>(ccsn_p), c1 = *reinterpret_cast<const int4*>(ccsn_p + 4);
        const int4 f0 = *reinterpret_cast<const int4*>(cref_p), f1 = *reinterpret_cast<const int4*>(cref_p + 4);
        csn = V8{c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        ref = V8{f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
        const uint2 fb = *reinterpret_cast<const uint2*>(cfl_p);
#pragma unroll
        for (int i = 0; i < kPerLane; i++) fl |= (((i < 4 ? fb.x >> (8 * i) : fb.y >> (8 * (i - 4)))) & 3u) << (2 * i);
    }
    int seq = s0.x, msn = s0.y, last = s0.z, err = s0.w;
    int stop = -1;  // (G = 8) the message from a client >= 64 this document stops at
    const int maxlen = -wave_min(live ? -len : 0);  // wave-uniform trip count
    int4 nxt = make_int4(0, 0, 0, 0);
    if (live && m0 + li < len) nxt = msgs[r0 + m0 + li];
    for (int jb = m0; jb < maxlen; jb += G) {
        const int4 cur = nxt;
        if (live && jb + G + li < len) nxt = msgs[r0 + jb + G + li];  // next chunk in flight
        wave_sync();
        stage[lane] = cur;
        wave_sync();
        int4 t = make_int4(0, 0, 0, 0);
        const int steps = min(G, maxlen - jb);
        for (int jj = 0; jj < steps; jj++) {
            const int4 mm = stage[gbase + jj];
            const int mc = mm.x, mr = mm.y;
            const int c = mm.z & 0xFFFF, kind = (mm.z >> 16) & 0xFF;
            if (G == 8 && live && jb + jj < len && !err && stop < 0 && c >= NC && c < MT_DELI_MAX_CLIENTS &&
                kind <= MT_RAW_CONTROL)
                stop = jb + jj;  // (group-uniform: every lane of the group reads the same message)
            const bool act = live && jb + jj < len && stop < 0;
            const bool bad = c >= NC || kind > MT_RAW_CONTROL;
            const int cq = c & (kPerLane - 1), owner = gbase + ((c / kPerLane) & (G - 1));
            // client c's record, from its owner lane
            const int ccsn = __builtin_amdgcn_ds_bpermute(owner << 2, pick(csn, cq));
            const int cfl = __builtin_amdgcn_ds_bpermute(owner << 2, (int)((fl >> (2 * cq)) & 3u));
            const bool joined = (cfl & CL_JOINED) != 0, nacked = (cfl & CL_NACK) != 0;
            const bool go = act && !err && !bad;
            // checkOrder + the client / system branches of ticket() (lambda.ts:265-347)
            const bool isc = kind <= MT_RAW_NOOP_DATA;
            const bool gap = isc && joined && mc > ccsn + 1;
            const bool dup = isc && joined && mc < ccsn + 1;
            const bool nackc = isc && !gap && !dup && (!joined || nacked);
            const bool nackr = isc && !gap && !dup && !nackc && mr != -1 && mr < msn;
            const bool clok = isc && !gap && !dup && !nackc && !nackr;
            const bool rev_op = clok && kind == MT_RAW_OP;          // client no-ops do not rev (:414-425)
            const int s1 = seq + (rev_op ? 1 : 0);
            const int tr0 = (rev_op && mr == -1) ? s1 : mr;          // REST op (:422-424)
            const bool afail = clok && tr0 < msn;                   // assert (:426-428)
            const bool leave_ok = kind == MT_RAW_LEAVE && joined;
            const bool join_new = kind == MT_RAW_JOIN && !joined;
            const bool drop = dup || (kind == MT_RAW_LEAVE && !joined) || (kind == MT_RAW_JOIN && joined);
            const bool nack = gap || nackc || nackr;
            // ClientSequenceNumberManager updates, by the owner lane
            const bool ups = go && ((clok && !afail) || nackr || kind == MT_RAW_JOIN);
            const bool rem = go && leave_ok;
            if ((ups || rem) && lane == owner) {
                const int ucsn = kind == MT_RAW_JOIN ? 0 : mc;
                const int uref = (nackr || kind == MT_RAW_JOIN) ? msn : tr0;
#pragma unroll
                for (int i = 0; i < kPerLane; i++) {
                    csn[i] = (ups && cq == i) ? ucsn : csn[i];
                    ref[i] = (ups && cq == i) ? uref : ref[i];
                }
                const uint32_t ufl = ups ? (uint32_t)(CL_JOINED | (nackr ? CL_NACK : 0)) : 0u;
                fl = (fl & ~(3u << (2 * cq))) | (ufl << (2 * cq));
            }
            const int s2 = s1 + ((leave_ok || join_new) ? 1 : 0);  // join / leave rev (:437-442)
            // getMinimumSequenceNumber (:446-455)
            int mv = INT_MAX;
#pragma unroll
            for (int i = 0; i < kPerLane; i++) mv = min(mv, ((fl >> (2 * i)) & 1u) ? ref[i] : INT_MAX);
            mv = group_min<G>(mv);
            const bool none = mv == INT_MAX;
            int msn2 = none ? s2 : mv;
            // send type (:457-517)
            int st = MT_TK_SENT, s3 = s2, tr = tr0;
            if (kind == MT_RAW_NOOP) {
                st = MT_TK_LATER;
            } else if (kind == MT_RAW_NOOP_DATA || kind == MT_RAW_SERVER_NOOP) {
                if (msn2 <= last) st = kind == MT_RAW_NOOP_DATA ? MT_TK_LATER : MT_TK_NEVER;
                else s3 = s2 + 1;
            } else if (kind == MT_RAW_NOCLIENT) {
                if (none) {
                    s3 = s2 + 1;
                    tr = s3;
                    msn2 = s3;
                } else {
                    st = MT_TK_NEVER;
                }
            } else if (kind == MT_RAW_CONTROL) {
                st = MT_TK_NEVER;
            }
            // outcome
            int ts = seq, tm = msn, to = mr, tst = MT_TK_HALTED;
            if (go) {
                if (drop) {
                    tst = MT_TK_DROPPED;
                } else if (nack) {                                 // createNackMessage (:683-712)
                    tst = gap ? MT_TK_NACK_GAP : (nackc ? MT_TK_NACK_CLIENT : MT_TK_NACK_REFSEQ);
                    ts = msn;
                    last = msn;
                } else if (afail) {
                    err = MT_DELI_ERR_ASSERT;
                    err_at = jb + jj;
                    seq = s1;
                    ts = s1;
                    to = tr0;
                } else {
                    seq = s3;
                    msn = msn2;
                    if (st == MT_TK_SENT) last = msn2;             // handler (:217-218)
                    ts = s3;
                    tm = msn2;
                    to = tr;
                    tst = st;
                }
            } else if (act && !err) {
                err = c >= NC ? MT_DELI_ERR_CLIENT : MT_DELI_ERR_KIND;
                err_at = jb + jj;
            }
            if (li == jj) t = make_int4(ts, tm, to, tst);
        }
        if (live && jb + li < len && (stop < 0 || jb + li < stop)) {
            out[r0 + jb + li] = t;
            // my message of this chunk is still staged: its op_index links the op record
            const uint32_t opi = (uint32_t)stage[lane].w;
            if (ops && opi && opi <= n_ops) {
                mt_op_rec* o = ops + (opi - 1u);
                o->seq = t.w == MT_TK_SENT ? t.x : MT_SEQ_NACK;  // never MT_SEQ_LOCAL
                o->msn = t.y;
                o->ref_seq = t.z;
            }
        }
    }
    if (!live) return;
    if (li == 0) {
        g.sc[d] = make_int4(seq, msn, last, err);
        g.err_at[d] = err_at;
        if (G == 8 && stop >= 0) {  // the rest of the stream goes to the wide form
            const uint32_t q = atomicAdd(&g.ctl[1], 1u);
            g.queue[q] = d;
            g.resume[d] = stop;
        }
    }
    *reinterpret_cast<int4*>(ccsn_p) = make_int4(csn[0], csn[1], csn[2], csn[3]);
    *reinterpret_cast<int4*>(ccsn_p + 4) = make_int4(csn[4], csn[5], csn[6], csn[7]);
    *reinterpret_cast<int4*>(cref_p) = make_int4(ref[0], ref[1], ref[2], ref[3]);
    *reinterpret_cast<int4*>(cref_p + 4) = make_int4(ref[4], ref[5], ref[6], ref[7]);
    uint2 fb = make_uint2(0u, 0u);
#pragma unroll
    for (int i = 0; i < kPerLane; i++) {
        const uint32_t v = (fl >> (2 * i)) & 3u;
        if (i < 4) fb.x |= v << (8 * i);
        else fb.y |= v << (8 * (i - 4));
    }
    *reinterpret_cast<uint2*>(cfl_p) = fb;
}

// eight documents per wave (the common form); a document already promoted to the big pool is
// queued for the wide form whole
__global__ __launch_bounds__(64) void deli_kernel(DeliState g, const int4* __restrict__ msgs,
                                                  const uint32_t* __restrict__ row_ptr, uint32_t n_docs,
                                                  int4* __restrict__ out, mt_op_rec* __restrict__ ops,
                                                  uint64_t n_ops) {
    __shared__ int4 stage[64];
    const int lane = lane_id();
    const int li = lane & 7;
    const uint32_t d = blockIdx.x * 8 + (uint32_t)(lane / 8);
    bool live = d < n_docs;
    uint32_t r0 = 0;
    int len = 0;
    if (live) {
        r0 = row_ptr[d];
        len = (int)(row_ptr[d + 1] - r0);
        if (g.big[d] != kNoRow) {  // promoted earlier: the wide form tickets it
            if (len > 0 && li == 0) {
                const uint32_t q = atomicAdd(&g.ctl[1], 1u);
                g.queue[q] = d;
                g.resume[d] = 0;
            }
            live = false;
        }
    }
    if (wave_ballot(live && len > 0) == 0) return;
    const size_t cb = (size_t)(live ? d : 0) * MT_MAX_CLIENTS + (size_t)li * kPerLane;
    deli_group<8>(g, msgs, d, live, r0, len, 0, g.csn + cb, g.ref + cb, g.fl + cb, out, ops, n_ops, stage);
}

// the wide form: the queued documents, one per wave (persistent over the queue); a document's first
// visit promotes it -- a row of the big pool, its 64 clients' state copied in
__global__ __launch_bounds__(64) void deli_wide_kernel(DeliState g, const int4* __restrict__ msgs,
                                                       const uint32_t* __restrict__ row_ptr, int4* __restrict__ out,
                                                       mt_op_rec* __restrict__ ops, uint64_t n_ops) {
    __shared__ int4 stage[64];
    const int lane = lane_id();
    const uint32_t nq = g.ctl[1];
    for (uint32_t i = blockIdx.x; i < nq; i += gridDim.x) {
        const uint32_t d = g.queue[i];
        const uint32_t r0 = row_ptr[d];
        const int len = (int)(row_ptr[d + 1] - r0);
        const int m0 = g.resume[d];
        uint32_t row = g.big[d];
        if (row == kNoRow) {
            // a row from the free list (each pop that finds it non-empty takes a distinct entry: only
            // pops run during the kernel), else a fresh one
            uint32_t r = 0;
            if (lane == 0) {
                const int fr = atomicSub(reinterpret_cast<int*>(&g.ctl[2]), 1);
                r = fr > 0 ? g.free_rows[fr - 1] : atomicAdd(&g.ctl[0], 1u);
            }
            r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
            if (r >= g.big_cap) {  // no row left: the document halts at the message that needed one
                if (lane == 0) {
                    int4 sc = g.sc[d];
                    if (!sc.w) {
                        sc.w = MT_DELI_ERR_CAPACITY;
                        g.err_at[d] = m0;
                    }
                    g.sc[d] = sc;
                }
                wave_sync();
                const int4 sc = g.sc[d];
                for (int j = m0 + lane; j < len; j += 64) {
                    const int4 m = msgs[r0 + j];
                    out[r0 + j] = make_int4(sc.x, sc.y, m.y, MT_TK_HALTED);
                    const uint32_t opi = (uint32_t)m.w;
                    if (ops && opi && opi <= n_ops) {
                        mt_op_rec* o = ops + (opi - 1u);
                        o->seq = MT_SEQ_NACK;
                        o->msn = sc.y;
                        o->ref_seq = m.y;
                    }
                }
                continue;
            }
            row = r;
            const size_t src = (size_t)d * MT_MAX_CLIENTS, dst = (size_t)row * MT_DELI_MAX_CLIENTS;
            for (int c = lane; c < MT_DELI_MAX_CLIENTS; c += 64) {
                const bool in = c < MT_MAX_CLIENTS;
                g.bcsn[dst + c] = in ? g.csn[src + c] : 0;
                g.bref[dst + c] = in ? g.ref[src + c] : 0;
                g.bfl[dst + c] = in ? g.fl[src + c] : (uint8_t)0;
            }
            __threadfence_block();
            if (lane == 0) g.big[d] = row;
        }
        const size_t cb = (size_t)row * MT_DELI_MAX_CLIENTS + (size_t)lane * kPerLane;
        deli_group<64>(g, msgs, d, true, r0, len, m0, g.bcsn + cb, g.bref + cb, g.bfl + cb, out, ops, n_ops, stage);
    }
}

// every document from one checkpoint (bench tooling)
__global__ void restore_all_kernel(DeliState g, uint32_t n_docs, mt_deli_checkpoint ck) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_docs * MT_MAX_CLIENTS) return;
    const uint32_t d = i / MT_MAX_CLIENTS, c = i % MT_MAX_CLIENTS;
    const mt_deli_client& cl = ck.clients[c];
    g.csn[i] = cl.csn;
    g.ref[i] = cl.ref_seq;
    g.fl[i] = (uint8_t)((cl.joined ? CL_JOINED : 0) | (cl.nack ? CL_NACK : 0));
    if (c == 0) {
        g.sc[d] = make_int4(ck.seq, ck.msn, ck.last_sent_msn, 0);
        g.err_at[d] = -1;
        g.big[d] = kNoRow;  // (every document restored: the big pool starts over)
        if (d == 0) {
            g.ctl[0] = 0u;
            g.ctl[2] = 0u;
        }
    }
}

// raw op messages behind a device op log: csn counted per client (lane c counts client c)
__global__ __launch_bounds__(64) void raw_from_ops_kernel(const mt_op_rec* __restrict__ ops,
                                                          const uint32_t* __restrict__ row_ptr, uint32_t n_docs,
                                                          int4* __restrict__ msgs) {
    const uint32_t d = blockIdx.x;
    if (d >= n_docs) return;
    const int lane = lane_id();
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    int cnt = 0;
    for (uint32_t base = r0; base < r1; base += 64) {
        const int n = (int)min(64u, r1 - base);
        int cl = 0, rf = 0;
        if (lane < n) {
            cl = ops[base + lane].client;
            rf = ops[base + lane].ref_seq;
        }
        int mine = 0;
        for (int j = 0; j < n; j++) {
            const int c = __builtin_amdgcn_readlane(cl, j) & (MT_MAX_CLIENTS - 1);
            if (lane == c) cnt++;
            const int v = __builtin_amdgcn_readlane(cnt, c);
            if (lane == j) mine = v;
        }
        if (lane < n) msgs[base + lane] = make_int4(mine, rf, (cl & 0xFFFF) | (MT_RAW_OP << 16), (int)(base + lane + 1));
    }
}

// a new document's raw stream: n_join joins, then the op messages (refSeq + n_join)
__global__ __launch_bounds__(64) void raw_stream_kernel(const mt_op_rec* __restrict__ ops,
                                                        const uint32_t* __restrict__ row_ptr, uint32_t n_docs,
                                                        uint32_t n_join, int4* __restrict__ msgs,
                                                        uint32_t* __restrict__ msg_row) {
    const uint32_t d = blockIdx.x;
    if (d >= n_docs) return;
    const int lane = lane_id();
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    const uint32_t m0 = r0 + d * n_join;
    if (lane == 0) {
        msg_row[d] = m0;
        if (d + 1 == n_docs) msg_row[n_docs] = r1 + n_docs * n_join;
    }
    for (uint32_t j = (uint32_t)lane; j < n_join; j += 64)
        msgs[m0 + j] = make_int4(-1, -1, (int)((j + 1) & 0xFFFF) | (MT_RAW_JOIN << 16), 0);
    int cnt = 0;
    for (uint32_t base = r0; base < r1; base += 64) {
        const int n = (int)min(64u, r1 - base);
        int cl = 0, rf = 0;
        if (lane < n) {
            cl = ops[base + lane].client;
            rf = ops[base + lane].ref_seq;
        }
        int mine = 0;
        for (int j = 0; j < n; j++) {
            const int c = __builtin_amdgcn_readlane(cl, j) & (MT_MAX_CLIENTS - 1);
            if (lane == c) cnt++;
            const int v = __builtin_amdgcn_readlane(cnt, c);
            if (lane == j) mine = v;
        }
        if (lane < n)
            msgs[m0 + n_join + (base - r0) + lane] =
                make_int4(mine, rf + (int)n_join, (cl & 0xFFFF) | (MT_RAW_OP << 16), (int)(base + lane + 1));
    }
}

}  // namespace mtd

struct mt_deli {
    int32_t device = 0;
    uint32_t max_docs = 0;
    hipStream_t stream = nullptr;
    mtd::DeliState g{};
    hipEvent_t e0 = nullptr, e1 = nullptr;
};
// rows of the big pool (documents past client 63 at once): one per 16 documents, at least 64
static uint32_t deli_big_rows(uint32_t max_docs) { return std::max<uint32_t>(64u, max_docs / 16u); }

#define DL_HIP(x)                                                                                            \
    do {                                                                                                     \
        hipError_t e_ = (x);                                                                                 \
        if (e_ != hipSuccess) {                                                                              \
            fprintf(stderr, "libmtgpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return MT_ERR_HIP;                                                                               \
        }                                                                                                    \
    } while (0)

namespace {
// the constructor's msn (lambda.ts:166-167): min refSeq over the checkpoint's clients, or seq
template <class CK>
int32_t ckpt_msn(const CK& ck) {
    constexpr int NC = sizeof(ck.clients) / sizeof(ck.clients[0]);
    int32_t m = INT_MAX;
    for (int c = 0; c < NC; c++)
        if (ck.clients[c].joined) m = std::min(m, ck.clients[c].ref_seq);
    return m == INT_MAX ? ck.seq : m;
}
uint8_t client_flags(const mt_deli_client& c) {
    return (uint8_t)((c.joined ? mtd::CL_JOINED : 0) | (c.nack ? mtd::CL_NACK : 0));
}
// the rows of the big pool held by documents [doc0, doc0 + n) go back to its free list (their
// documents are about to be restored); the stream is idle
mt_status release_rows(mt_deli* dl, uint32_t doc0, uint32_t n) {
    std::vector<uint32_t> big(n);
    DL_HIP(hipMemcpy(big.data(), dl->g.big + doc0, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint32_t> rows;
    for (uint32_t r : big)
        if (r != mtd::kNoRow) rows.push_back(r);
    if (rows.empty()) return MT_OK;
    int32_t nfree = 0;
    DL_HIP(hipMemcpy(&nfree, dl->g.ctl + 2, sizeof nfree, hipMemcpyDeviceToHost));
    nfree = std::max(nfree, 0);  // (pops past empty left it below zero)
    if ((uint64_t)nfree + rows.size() > dl->g.big_cap) return MT_ERR_STATE;  // (a row freed twice)
    DL_HIP(hipMemcpy(dl->g.free_rows + nfree, rows.data(), rows.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    nfree += (int32_t)rows.size();
    DL_HIP(hipMemcpy(dl->g.ctl + 2, &nfree, sizeof nfree, hipMemcpyHostToDevice));
    return MT_OK;
}
// the common form over every document, then the wide form over the documents it queued (past client
// 63: promoted now or earlier), on one stream
mt_status launch_forms(mt_deli* dl, hipStream_t st, const mt_raw_msg* d_msgs, const uint32_t* d_row, uint32_t n_docs,
                       mt_ticket* d_out, mt_op_rec* d_ops, uint64_t n_ops) {
    DL_HIP(hipMemsetAsync(dl->g.ctl + 1, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(mtd::deli_kernel, dim3((n_docs + 7) / 8), dim3(64), 0, st, dl->g,
                       reinterpret_cast<const int4*>(d_msgs), d_row, n_docs, reinterpret_cast<int4*>(d_out), d_ops,
                       n_ops);
    DL_HIP(hipGetLastError());
    hipLaunchKernelGGL(mtd::deli_wide_kernel, dim3(std::min<uint32_t>(1024u, n_docs)), dim3(64), 0, st, dl->g,
                       reinterpret_cast<const int4*>(d_msgs), d_row, reinterpret_cast<int4*>(d_out), d_ops, n_ops);
    DL_HIP(hipGetLastError());
    return MT_OK;
}
mt_status launch_ticket(mt_deli* dl, const mt_raw_msg* d_msgs, const uint32_t* d_row, uint32_t n_docs,
                        mt_ticket* d_out, mt_op_rec* d_ops, uint64_t n_ops) {
    DL_HIP(hipEventRecord(dl->e0, dl->stream));
    const mt_status st = launch_forms(dl, dl->stream, d_msgs, d_row, n_docs, d_out, d_ops, n_ops);
    if (st) return st;
    DL_HIP(hipEventRecord(dl->e1, dl->stream));
    return MT_OK;
}
}  // namespace

extern "C" {

mt_status mt_deli_create(int32_t device, uint32_t max_docs, mt_deli** out) {
    if (!out || max_docs == 0) return MT_ERR_ARG;
    DL_HIP(hipSetDevice(device));
    auto* dl = new mt_deli();
    dl->device = device;
    dl->max_docs = max_docs;
    const size_t nc = (size_t)max_docs * MT_MAX_CLIENTS;
    dl->g.big_cap = deli_big_rows(max_docs);
    const size_t nb = (size_t)dl->g.big_cap * MT_DELI_MAX_CLIENTS;
    bool ok = hipStreamCreateWithFlags(&dl->stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreate(&dl->e0) == hipSuccess && hipEventCreate(&dl->e1) == hipSuccess &&
              hipMalloc(&dl->g.sc, max_docs * sizeof(int4)) == hipSuccess &&
              hipMalloc(&dl->g.err_at, max_docs * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.csn, nc * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.ref, nc * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.fl, nc) == hipSuccess &&
              hipMalloc(&dl->g.big, max_docs * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&dl->g.resume, max_docs * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.queue, max_docs * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&dl->g.ctl, 4 * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&dl->g.bcsn, nb * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.bref, nb * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.bfl, nb) == hipSuccess &&
              hipMalloc(&dl->g.free_rows, dl->g.big_cap * sizeof(uint32_t)) == hipSuccess &&
              hipMemset(dl->g.big, 0xFF, max_docs * sizeof(uint32_t)) == hipSuccess &&
              hipMemset(dl->g.ctl, 0, 4 * sizeof(uint32_t)) == hipSuccess;
    if (!ok) {
        mt_deli_destroy(dl);
        return MT_ERR_NOMEM;
    }
    mt_status st = mt_deli_restore(dl, 0, max_docs, nullptr);
    if (st != MT_OK) {
        mt_deli_destroy(dl);
        return st;
    }
    *out = dl;
    return MT_OK;
}

mt_status mt_deli_destroy(mt_deli* dl) {
    if (!dl) return MT_ERR_ARG;
    hipSetDevice(dl->device);
    if (dl->stream) hipStreamSynchronize(dl->stream);
    for (void* p : {(void*)dl->g.sc, (void*)dl->g.err_at, (void*)dl->g.csn, (void*)dl->g.ref, (void*)dl->g.fl,
                    (void*)dl->g.big, (void*)dl->g.resume, (void*)dl->g.queue, (void*)dl->g.ctl, (void*)dl->g.bcsn,
                    (void*)dl->g.bref, (void*)dl->g.bfl, (void*)dl->g.free_rows})
        if (p) hipFree(p);
    if (dl->e0) hipEventDestroy(dl->e0);
    if (dl->e1) hipEventDestroy(dl->e1);
    if (dl->stream) hipStreamDestroy(dl->stream);
    delete dl;
    return MT_OK;
}

mt_status mt_deli_restore(mt_deli* dl, uint32_t doc0, uint32_t n, const mt_deli_checkpoint* ckpts) {
    if (!dl || doc0 > dl->max_docs || n > dl->max_docs - doc0) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    DL_HIP(hipStreamSynchronize(dl->stream));
    if (const mt_status rs = release_rows(dl, doc0, n)) return rs;
    std::vector<int4> sc(n);
    std::vector<int32_t> err_at(n, -1), csn((size_t)n * MT_MAX_CLIENTS, 0), ref((size_t)n * MT_MAX_CLIENTS, 0);
    std::vector<uint8_t> fl((size_t)n * MT_MAX_CLIENTS, 0);
    for (uint32_t i = 0; i < n; i++) {
        if (!ckpts) {
            sc[i] = make_int4(0, 0, 0, 0);  // a new document: sequenceNumber 0, no clients
            continue;
        }
        const mt_deli_checkpoint& ck = ckpts[i];
        sc[i] = make_int4(ck.seq, ckpt_msn(ck), ck.last_sent_msn, 0);
        for (int c = 0; c < MT_MAX_CLIENTS; c++) {
            const size_t k = (size_t)i * MT_MAX_CLIENTS + c;
            csn[k] = ck.clients[c].csn;
            ref[k] = ck.clients[c].ref_seq;
            fl[k] = client_flags(ck.clients[c]);
        }
    }
    const size_t c0 = (size_t)doc0 * MT_MAX_CLIENTS, nc = (size_t)n * MT_MAX_CLIENTS;
    DL_HIP(hipMemcpyAsync(dl->g.sc + doc0, sc.data(), n * sizeof(int4), hipMemcpyHostToDevice, dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.err_at + doc0, err_at.data(), n * sizeof(int32_t), hipMemcpyHostToDevice,
                          dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.csn + c0, csn.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.ref + c0, ref.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.fl + c0, fl.data(), nc, hipMemcpyHostToDevice, dl->stream));
    // (a restored document is back in the common form; the row it held is on the free list now)
    DL_HIP(hipMemsetAsync(dl->g.big + doc0, 0xFF, n * sizeof(uint32_t), dl->stream));
    DL_HIP(hipStreamSynchronize(dl->stream));
    return MT_OK;
}

mt_status mt_deli_restore_all(mt_deli* dl, uint32_t n_docs, const mt_deli_checkpoint* ckpt) {
    if (!dl || !ckpt || n_docs > dl->max_docs) return MT_ERR_ARG;
    if (n_docs == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    mt_deli_checkpoint ck = *ckpt;
    ck.msn = ckpt_msn(ck);
    const uint32_t threads = n_docs * MT_MAX_CLIENTS;
    hipLaunchKernelGGL(mtd::restore_all_kernel, dim3((threads + 255) / 256), dim3(256), 0, dl->stream, dl->g, n_docs,
                       ck);
    DL_HIP(hipGetLastError());
    DL_HIP(hipStreamSynchronize(dl->stream));
    return MT_OK;
}

mt_status mt_deli_ticket(mt_deli* dl, const mt_raw_msg* msgs, uint64_t n_msgs, const uint32_t* doc_row_ptr,
                         uint32_t n_docs, mt_ticket* out) {
    if (!dl || !doc_row_ptr || n_docs > dl->max_docs || (n_msgs && (!msgs || !out))) return MT_ERR_ARG;
    if (doc_row_ptr[0] != 0 || doc_row_ptr[n_docs] != n_msgs || n_msgs > 0xFFFFFFFFull) return MT_ERR_ARG;
    for (uint32_t d = 0; d < n_docs; d++)
        if (doc_row_ptr[d] > doc_row_ptr[d + 1]) return MT_ERR_ARG;
    if (n_docs == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    mt_raw_msg* d_msgs = nullptr;
    mt_ticket* d_out = nullptr;
    uint32_t* d_row = nullptr;
    mt_status st = MT_OK;
    if (hipMalloc(&d_msgs, std::max<uint64_t>(1, n_msgs) * sizeof(mt_raw_msg)) != hipSuccess ||
        hipMalloc(&d_out, std::max<uint64_t>(1, n_msgs) * sizeof(mt_ticket)) != hipSuccess ||
        hipMalloc(&d_row, (n_docs + 1) * sizeof(uint32_t)) != hipSuccess) {
        st = MT_ERR_NOMEM;
    }
    if (st == MT_OK &&
        (hipMemcpyAsync(d_msgs, msgs, n_msgs * sizeof(mt_raw_msg), hipMemcpyHostToDevice, dl->stream) != hipSuccess ||
         hipMemcpyAsync(d_row, doc_row_ptr, (n_docs + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, dl->stream) !=
             hipSuccess))
        st = MT_ERR_HIP;
    if (st == MT_OK) st = launch_ticket(dl, d_msgs, d_row, n_docs, d_out, nullptr, 0);
    if (st == MT_OK &&
        (hipMemcpyAsync(out, d_out, n_msgs * sizeof(mt_ticket), hipMemcpyDeviceToHost, dl->stream) != hipSuccess ||
         hipStreamSynchronize(dl->stream) != hipSuccess))
        st = MT_ERR_HIP;
    hipStreamSynchronize(dl->stream);
    hipFree(d_msgs);
    hipFree(d_out);
    hipFree(d_row);
    return st;
}

mt_status mt_deli_ticket_device(mt_deli* dl, const mt_raw_msg* d_msgs, const uint32_t* d_row_ptr, uint32_t n_docs,
                                mt_ticket* d_out, mt_op_rec* d_ops, uint64_t n_ops) {
    if (!dl || !d_msgs || !d_row_ptr || !d_out || n_docs > dl->max_docs) return MT_ERR_ARG;
    if (n_docs == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    return launch_ticket(dl, d_msgs, d_row_ptr, n_docs, d_out, d_ops, n_ops);
}

// (internal, mt_engine.cpp's mt_submit_ticks_deli) the ticket kernel on the apply engine's stream,
// for the documents [0, n_docs) of a deli on `device`
mt_status mt_deli_ticket_on_stream(mt_deli* dl, int32_t device, hipStream_t st, const mt_raw_msg* d_msgs,
                                   const uint32_t* d_row_ptr, uint32_t n_docs, mt_ticket* d_out, mt_op_rec* d_ops,
                                   uint64_t n_ops) {
    if (!dl || dl->device != device || n_docs > dl->max_docs) return MT_ERR_ARG;
    if (n_docs == 0) return MT_OK;
    return launch_forms(dl, st, d_msgs, d_row_ptr, n_docs, d_out, d_ops, n_ops);
}

mt_status mt_deli_raw_from_ops(mt_deli* dl, const mt_op_rec* d_ops, const uint32_t* d_row_ptr, uint32_t n_docs,
                               mt_raw_msg* d_msgs) {
    if (!dl || !d_ops || !d_row_ptr || !d_msgs) return MT_ERR_ARG;
    if (n_docs == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    hipLaunchKernelGGL(mtd::raw_from_ops_kernel, dim3(n_docs), dim3(64), 0, dl->stream, d_ops, d_row_ptr, n_docs,
                       reinterpret_cast<int4*>(d_msgs));
    DL_HIP(hipGetLastError());
    return MT_OK;
}

mt_status mt_deli_raw_stream(mt_deli* dl, const mt_op_rec* d_ops, const uint32_t* d_row_ptr, uint32_t n_docs,
                             uint32_t n_join, mt_raw_msg* d_msgs, uint32_t* d_msg_row_ptr) {
    if (!dl || !d_ops || !d_row_ptr || !d_msgs || !d_msg_row_ptr || n_join >= MT_MAX_CLIENTS) return MT_ERR_ARG;
    if (n_docs == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    hipLaunchKernelGGL(mtd::raw_stream_kernel, dim3(n_docs), dim3(64), 0, dl->stream, d_ops, d_row_ptr, n_docs, n_join,
                       reinterpret_cast<int4*>(d_msgs), d_msg_row_ptr);
    DL_HIP(hipGetLastError());
    return MT_OK;
}

mt_status mt_deli_sync(mt_deli* dl) {
    if (!dl) return MT_ERR_ARG;
    DL_HIP(hipSetDevice(dl->device));
    DL_HIP(hipStreamSynchronize(dl->stream));
    return MT_OK;
}

mt_status mt_deli_last_ms(mt_deli* dl, float* kernel_ms) {
    if (!dl || !kernel_ms) return MT_ERR_ARG;
    DL_HIP(hipSetDevice(dl->device));
    DL_HIP(hipEventSynchronize(dl->e1));
    DL_HIP(hipEventElapsedTime(kernel_ms, dl->e0, dl->e1));
    return MT_OK;
}

}  // extern "C"

// clients [c0, c0 + n) of a document, from its row of the big pool once promoted
static mt_status read_clients(mt_deli* dl, uint32_t doc, uint32_t c0, uint32_t n, mt_deli_client* out) {
    uint32_t row = mtd::kNoRow;
    DL_HIP(hipStreamSynchronize(dl->stream));
    DL_HIP(hipMemcpy(&row, dl->g.big + doc, sizeof row, hipMemcpyDeviceToHost));
    std::vector<int32_t> csn(n, 0), ref(n, 0);
    std::vector<uint8_t> fl(n, 0);
    const bool big = row != mtd::kNoRow;
    const uint32_t m = big ? n : (c0 < MT_MAX_CLIENTS ? std::min(n, MT_MAX_CLIENTS - c0) : 0u);
    const size_t o = big ? (size_t)row * MT_DELI_MAX_CLIENTS + c0 : (size_t)doc * MT_MAX_CLIENTS + c0;
    if (m) {
        DL_HIP(hipMemcpy(csn.data(), (big ? dl->g.bcsn : dl->g.csn) + o, m * sizeof(int32_t), hipMemcpyDeviceToHost));
        DL_HIP(hipMemcpy(ref.data(), (big ? dl->g.bref : dl->g.ref) + o, m * sizeof(int32_t), hipMemcpyDeviceToHost));
        DL_HIP(hipMemcpy(fl.data(), (big ? dl->g.bfl : dl->g.fl) + o, m, hipMemcpyDeviceToHost));
    }
    for (uint32_t i = 0; i < n; i++) {
        const bool joined = (fl[i] & mtd::CL_JOINED) != 0;
        out[i] = mt_deli_client{};
        out[i].joined = joined;
        out[i].nack = (fl[i] & mtd::CL_NACK) != 0;
        out[i].csn = joined ? csn[i] : 0;
        out[i].ref_seq = joined ? ref[i] : 0;
    }
    return MT_OK;
}

template <class CK>
static mt_status get_checkpoint(mt_deli* dl, uint32_t doc, CK* out) {
    constexpr uint32_t NC = sizeof(out->clients) / sizeof(out->clients[0]);
    if (!dl || !out || doc >= dl->max_docs) return MT_ERR_ARG;
    DL_HIP(hipSetDevice(dl->device));
    int4 sc;
    uint32_t row = mtd::kNoRow;
    DL_HIP(hipStreamSynchronize(dl->stream));
    DL_HIP(hipMemcpy(&sc, dl->g.sc + doc, sizeof sc, hipMemcpyDeviceToHost));
    DL_HIP(hipMemcpy(&row, dl->g.big + doc, sizeof row, hipMemcpyDeviceToHost));
    // a promoted document whose clients past 63 hold state does not fit the narrow checkpoint: refuse
    // rather than drop them (a restore from it would lose them and derive another msn)
    if (NC <= MT_MAX_CLIENTS && row != mtd::kNoRow) {
        std::vector<uint8_t> fl(MT_DELI_MAX_CLIENTS - MT_MAX_CLIENTS);
        DL_HIP(hipMemcpy(fl.data(), dl->g.bfl + (size_t)row * MT_DELI_MAX_CLIENTS + MT_MAX_CLIENTS, fl.size(),
                         hipMemcpyDeviceToHost));
        for (uint8_t f : fl)
            if (f) return MT_ERR_WIDE;
    }
    memset(out, 0, sizeof *out);
    out->seq = sc.x;
    out->msn = sc.y;
    out->last_sent_msn = sc.z;
    out->err = sc.w;
    return read_clients(dl, doc, 0, NC, out->clients);
}

extern "C" {

mt_status mt_deli_get_checkpoint(mt_deli* dl, uint32_t doc, mt_deli_checkpoint* out) {
    return get_checkpoint(dl, doc, out);
}

mt_status mt_deli_get_checkpoint_wide(mt_deli* dl, uint32_t doc, mt_deli_checkpoint_wide* out) {
    return get_checkpoint(dl, doc, out);
}

mt_status mt_deli_restore_wide(mt_deli* dl, uint32_t doc0, uint32_t n, const mt_deli_checkpoint_wide* ckpts) {
    if (!dl || !ckpts || doc0 > dl->max_docs || n > dl->max_docs - doc0) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    DL_HIP(hipStreamSynchronize(dl->stream));
    // the documents needing a row (a client >= 64 joined or nacked), and whether the pool holds them
    // once the rows of [doc0, doc0 + n) are back on the free list
    std::vector<uint32_t> wide;
    for (uint32_t i = 0; i < n; i++)
        for (int c = MT_MAX_CLIENTS; c < MT_DELI_MAX_CLIENTS; c++)
            if (ckpts[i].clients[c].joined || ckpts[i].clients[c].nack) {
                wide.push_back(i);
                break;
            }
    std::vector<uint32_t> held(n);
    DL_HIP(hipMemcpy(held.data(), dl->g.big + doc0, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    uint32_t ctl[3] = {0, 0, 0};
    DL_HIP(hipMemcpy(ctl, dl->g.ctl, sizeof ctl, hipMemcpyDeviceToHost));
    const uint32_t fresh = std::min(ctl[0], dl->g.big_cap);
    const uint32_t nfree = (uint32_t)std::max((int32_t)ctl[2], 0);
    const uint32_t freed = (uint32_t)std::count_if(held.begin(), held.end(), [](uint32_t r) { return r != mtd::kNoRow; });
    if (wide.size() > (size_t)(dl->g.big_cap - fresh) + nfree + freed) return MT_ERR_NOMEM;
    // the narrow part (clients 0..63, scalars) through mt_deli_restore, which also frees the rows
    std::vector<mt_deli_checkpoint> narrow(n);
    for (uint32_t i = 0; i < n; i++) {
        mt_deli_checkpoint& k = narrow[i];
        k.seq = ckpts[i].seq;
        k.msn = 0;
        k.last_sent_msn = ckpts[i].last_sent_msn;
        k.err = 0;
        memcpy(k.clients, ckpts[i].clients, sizeof k.clients);
    }
    if (const mt_status st = mt_deli_restore(dl, doc0, n, narrow.data())) return st;
    if (wide.empty()) return MT_OK;
    // rows for the wide documents: free list first (mt_deli_restore just pushed), then fresh ones
    DL_HIP(hipMemcpy(ctl, dl->g.ctl, sizeof ctl, hipMemcpyDeviceToHost));
    int32_t top = std::max((int32_t)ctl[2], 0);
    uint32_t next = std::min(ctl[0], dl->g.big_cap);
    std::vector<uint32_t> stack((size_t)top);
    if (top) DL_HIP(hipMemcpy(stack.data(), dl->g.free_rows, top * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<int32_t> csn(MT_DELI_MAX_CLIENTS), ref(MT_DELI_MAX_CLIENTS);
    std::vector<uint8_t> fl(MT_DELI_MAX_CLIENTS);
    for (uint32_t i : wide) {
        const uint32_t row = top > 0 ? stack[--top] : next++;  // (capacity checked above)
        const mt_deli_checkpoint_wide& ck = ckpts[i];
        for (int c = 0; c < MT_DELI_MAX_CLIENTS; c++) {
            csn[c] = ck.clients[c].csn;
            ref[c] = ck.clients[c].ref_seq;
            fl[c] = client_flags(ck.clients[c]);
        }
        const size_t o = (size_t)row * MT_DELI_MAX_CLIENTS;
        DL_HIP(hipMemcpy(dl->g.bcsn + o, csn.data(), MT_DELI_MAX_CLIENTS * sizeof(int32_t), hipMemcpyHostToDevice));
        DL_HIP(hipMemcpy(dl->g.bref + o, ref.data(), MT_DELI_MAX_CLIENTS * sizeof(int32_t), hipMemcpyHostToDevice));
        DL_HIP(hipMemcpy(dl->g.bfl + o, fl.data(), MT_DELI_MAX_CLIENTS, hipMemcpyHostToDevice));
        DL_HIP(hipMemcpy(dl->g.big + doc0 + i, &row, sizeof row, hipMemcpyHostToDevice));
        // the constructor's msn over every client (lambda.ts:166-167)
        const int4 sc = make_int4(ck.seq, ckpt_msn(ck), ck.last_sent_msn, 0);
        DL_HIP(hipMemcpy(dl->g.sc + doc0 + i, &sc, sizeof sc, hipMemcpyHostToDevice));
    }
    ctl[0] = std::max(ctl[0], next);
    ctl[2] = (uint32_t)top;
    DL_HIP(hipMemcpy(dl->g.ctl, ctl, sizeof ctl, hipMemcpyHostToDevice));  // ([1] is per call: rewritten as read)
    return MT_OK;
}

mt_status mt_deli_get_clients(mt_deli* dl, uint32_t doc, uint32_t first, uint32_t n, mt_deli_client* out) {
    if (!dl || (n && !out) || doc >= dl->max_docs || first > MT_DELI_MAX_CLIENTS || n > MT_DELI_MAX_CLIENTS - first)
        return MT_ERR_ARG;
    DL_HIP(hipSetDevice(dl->device));
    return read_clients(dl, doc, first, n, out);
}

mt_status mt_deli_doc_error(mt_deli* dl, uint32_t doc, int32_t* err, int32_t* index) {
    if (!dl || !err || !index || doc >= dl->max_docs) return MT_ERR_ARG;
    DL_HIP(hipSetDevice(dl->device));
    int4 sc;
    DL_HIP(hipStreamSynchronize(dl->stream));
    DL_HIP(hipMemcpy(&sc, dl->g.sc + doc, sizeof sc, hipMemcpyDeviceToHost));
    DL_HIP(hipMemcpy(index, dl->g.err_at + doc, sizeof(int32_t), hipMemcpyDeviceToHost));
    *err = sc.w;
    return MT_OK;
}

}  // extern "C"
