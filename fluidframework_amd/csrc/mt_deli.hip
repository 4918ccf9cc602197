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

// A pool of client rows for documents past a form's client range: tier 0 (the big pool) holds
// MT_DELI_BIG_CLIENTS clients per row, tier 1 (the huge pool) MT_DELI_MAX_CLIENTS
struct Pool {
    uint32_t* row;        // per document: its row of this pool, or kNoRow
    int32_t* csn;         // [row][clients]
    int32_t* ref;
    uint8_t* fl;
    uint32_t* free_rows;  // [cap]: rows given back by restored documents, a stack of ctl[tier][2]
    uint32_t cap;         // rows
    uint32_t* queue;      // [max_docs]: the documents queued for this tier's form in this call
    int32_t* resume;      // per queued document: its first message this form tickets
};
// per-document state in HBM (structure of arrays; the narrow client arrays are [doc * 64 + client]);
// a document that ever sees a client id >= 64 is promoted, for good, to a row of the big pool and
// ticketed by the wide form (one document per wave, 512 clients); past client 511, to a row of the
// huge pool and the huge form (4096 clients)
struct DeliState {
    int4* sc;         // {sequenceNumber, minimumSequenceNumber, lastSentMSN, err}
    int32_t* err_at;  // message index (inside the document's stream) of the sticky error
    int32_t* csn;
    int32_t* ref;
    uint8_t* fl;      // CL_JOINED | CL_NACK
    Pool pool[2];
    // per tier t, ctl[4t + 0]: rows handed out fresh (a count that may pass cap: the attempts),
    // [4t + 1]: documents queued for the tier's form in this call, [4t + 2]: rows on the free list
    // (as int: a pop that finds it empty adds its 1 back, so it is never negative between kernels)
    uint32_t* ctl;
};
constexpr uint32_t kNoRow = 0xFFFFFFFFu;
constexpr int kTierClients[3] = {MT_MAX_CLIENTS, MT_DELI_BIG_CLIENTS, MT_DELI_MAX_CLIENTS};

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
// slot k of a lane's P client slots (k differs between groups: a select chain, not an index)
template <class V, int P>
MT_DEV int pick(const V& a, int k) {
    int r = a[0];
#pragma unroll
    for (int i = 1; i < P; i++) r = k == i ? a[i] : r;
    return r;
}

// One document per group of G lanes, lane q of the group owning the document's clients
// Pq..Pq+P-1 (csn, refSeq in VGPRs; joined / nacked as 2-bit fields, 16 per VGPR): G = 8, P = 8,
// eight documents per wave, 64 clients each (the common form); G = 64, P = 8, one document per
// wave with 512 (the wide form, for documents past client 63); G = 64, P = 64, 4096 (the huge form,
// past client 511).  Every branch of ticket() is evaluated as per-lane selects, so the CU's four
// SIMDs do the work in parallel (a wave-per-document form runs the decision tree on the CU's single
// scalar unit).  A client lookup is one ds_bpermute from its owner lane; the heap minimum is P local
// mins and a group reduction.  Messages are staged through LDS G per document at a time (one
// coalesced 16-byte load per lane, prefetched a chunk ahead); tickets go back the same way.
// Messages [m0, len) of the document's stream are ticketed; a form with a next tier (NEXT >= 0)
// stops a document at its first message from a client past the form's range and queues it for the
// next tier's form (`stop`), which promotes it and tickets the rest.
template <int G, int P, int NEXT>
MT_DEV void deli_group(DeliState& g, const int4* __restrict__ msgs, uint32_t d, bool live, uint32_t r0, int len,
                       int m0, int32_t* ccsn_p, int32_t* cref_p, uint8_t* cfl_p, int4* __restrict__ out,
                       mt_op_rec* __restrict__ ops, uint64_t n_ops, int4 (&stage)[64]) {
    constexpr int NC = G * P;        // clients this form holds
    constexpr int FW = (P + 15) / 16;  // flag words per lane
    typedef int32_t VP __attribute__((ext_vector_type(P)));
    typedef uint32_t VF __attribute__((ext_vector_type(FW == 1 ? 2 : FW)));  // (one-element vectors: 2)
    const int lane = lane_id();
    const int li = lane & (G - 1), gbase = lane & ~(G - 1);
    int4 s0 = make_int4(0, 0, 0, 0);
    int err_at = -1;
    VP csn = 0, ref = 0;
    VF fl = 0;
    if (live) {
        s0 = g.sc[d];
        err_at = g.err_at[d];
#pragma unroll
        for (int q = 0; q < P / 4; q++) {
            const int4 c = reinterpret_cast<const int4*>(ccsn_p)[q], f = reinterpret_cast<const int4*>(cref_p)[q];
            csn[4 * q] = c.x, csn[4 * q + 1] = c.y, csn[4 * q + 2] = c.z, csn[4 * q + 3] = c.w;
            ref[4 * q] = f.x, ref[4 * q + 1] = f.y, ref[4 * q + 2] = f.z, ref[4 * q + 3] = f.w;
        }
#pragma unroll
        for (int q = 0; q < P / 8; q++) {
            const uint2 fb = reinterpret_cast<const uint2*>(cfl_p)[q];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int s = 8 * q + i;
                fl[s / 16] |= (((i < 4 ? fb.x >> (8 * i) : fb.y >> (8 * (i - 4)))) & 3u) << (2 * (s % 16));
            }
        }
    }
    auto flag = [&](int s) -> uint32_t {  // (s: a compile-time slot)
        return (fl[s / 16] >> (2 * (s % 16))) & 3u;
    };
    int seq = s0.x, msn = s0.y, last = s0.z, err = s0.w;
    int stop = -1;  // (NEXT >= 0) the message from a client past this form this document stops at
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
            if (NEXT >= 0 && live && jb + jj < len && !err && stop < 0 && c >= NC && c < MT_DELI_MAX_CLIENTS &&
                kind <= MT_RAW_CONTROL)
                stop = jb + jj;  // (group-uniform: every lane of the group reads the same message)
            const bool act = live && jb + jj < len && stop < 0;
            const bool bad = c >= NC || kind > MT_RAW_CONTROL;
            const int cq = c & (P - 1), owner = gbase + ((c / P) & (G - 1));
            // client c's record, from its owner lane
            const int ccsn = __builtin_amdgcn_ds_bpermute(owner << 2, pick<VP, P>(csn, cq));
            const uint32_t fw = FW == 1 ? fl[0] : (uint32_t)pick<VF, FW>(fl, cq / 16);
            const int cfl = __builtin_amdgcn_ds_bpermute(owner << 2, (int)((fw >> (2 * (cq % 16))) & 3u));
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
                for (int i = 0; i < P; i++) {
                    csn[i] = (ups && cq == i) ? ucsn : csn[i];
                    ref[i] = (ups && cq == i) ? uref : ref[i];
                }
                const uint32_t ufl = ups ? (uint32_t)(CL_JOINED | (nackr ? CL_NACK : 0)) : 0u;
                const uint32_t sh = 2 * (cq % 16);
#pragma unroll
                for (int w = 0; w < FW; w++)
                    fl[w] = w == cq / 16 ? ((fl[w] & ~(3u << sh)) | (ufl << sh)) : fl[w];
            }
            const int s2 = s1 + ((leave_ok || join_new) ? 1 : 0);  // join / leave rev (:437-442)
            // getMinimumSequenceNumber (:446-455)
            int mv = INT_MAX;
#pragma unroll
            for (int i = 0; i < P; i++) mv = min(mv, (flag(i) & 1u) ? ref[i] : INT_MAX);
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
        if (NEXT >= 0 && stop >= 0) {  // the rest of the stream goes to the next tier's form
            const uint32_t q = atomicAdd(&g.ctl[4 * NEXT + 1], 1u);
            g.pool[NEXT].queue[q] = d;
            g.pool[NEXT].resume[d] = stop;
        }
    }
#pragma unroll
    for (int q = 0; q < P / 4; q++) {
        reinterpret_cast<int4*>(ccsn_p)[q] = make_int4(csn[4 * q], csn[4 * q + 1], csn[4 * q + 2], csn[4 * q + 3]);
        reinterpret_cast<int4*>(cref_p)[q] = make_int4(ref[4 * q], ref[4 * q + 1], ref[4 * q + 2], ref[4 * q + 3]);
    }
#pragma unroll
    for (int q = 0; q < P / 8; q++) {
        uint2 fb = make_uint2(0u, 0u);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t v = flag(8 * q + i);
            if (i < 4) fb.x |= v << (8 * i);
            else fb.y |= v << (8 * (i - 4));
        }
        reinterpret_cast<uint2*>(cfl_p)[q] = fb;
    }
}

// eight documents per wave (the common form); a document already promoted is queued whole for the
// form of its tier
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
        const int tier = g.pool[1].row[d] != kNoRow ? 1 : (g.pool[0].row[d] != kNoRow ? 0 : -1);
        if (tier >= 0) {  // promoted earlier: its tier's form tickets it
            if (len > 0 && li == 0) {
                const uint32_t q = atomicAdd(&g.ctl[4 * tier + 1], 1u);
                g.pool[tier].queue[q] = d;
                g.pool[tier].resume[d] = 0;
            }
            live = false;
        }
    }
    if (wave_ballot(live && len > 0) == 0) return;
    const size_t cb = (size_t)(live ? d : 0) * MT_MAX_CLIENTS + (size_t)li * 8;
    deli_group<8, 8, 0>(g, msgs, d, live, r0, len, 0, g.csn + cb, g.ref + cb, g.fl + cb, out, ops, n_ops, stage);
}

// the forms of the pools, one document per wave (persistent over the tier's queue): TIER 0 the wide
// form (512 clients, P = 8), TIER 1 the huge form (4096, P = 64).  A document's first visit promotes it
// -- a row of the tier's pool (its free list first, else a fresh one), the clients of its previous
// form copied in (the narrow arrays, or for the huge form the big row when it has one)
template <int TIER>
__global__ __launch_bounds__(64) void deli_pool_kernel(DeliState g, const int4* __restrict__ msgs,
                                                       const uint32_t* __restrict__ row_ptr, int4* __restrict__ out,
                                                       mt_op_rec* __restrict__ ops, uint64_t n_ops) {
    constexpr int NCL = kTierClients[TIER + 1];  // clients per row
    constexpr int P = NCL / 64;
    __shared__ int4 stage[64];
    const int lane = lane_id();
    Pool& pl = g.pool[TIER];
    const uint32_t nq = g.ctl[4 * TIER + 1];
    for (uint32_t i = blockIdx.x; i < nq; i += gridDim.x) {
        const uint32_t d = pl.queue[i];
        const uint32_t r0 = row_ptr[d];
        const int len = (int)(row_ptr[d + 1] - r0);
        const int m0 = pl.resume[d];
        uint32_t row = pl.row[d];
        if (row == kNoRow) {
            uint32_t r = 0;
            if (lane == 0) {
                const int fr = atomicSub(reinterpret_cast<int*>(&g.ctl[4 * TIER + 2]), 1);
                if (fr > 0) {
                    r = pl.free_rows[fr - 1];
                } else {
                    atomicAdd(reinterpret_cast<int*>(&g.ctl[4 * TIER + 2]), 1);  // (empty: the pop gives its 1 back)
                    r = atomicAdd(&g.ctl[4 * TIER], 1u);
                }
            }
            r = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);
            if (r >= pl.cap) {  // no row left: the document halts at the message that needed one
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
            // the previous form's clients
            const uint32_t prow = TIER == 1 ? g.pool[0].row[d] : kNoRow;
            const int npc = prow != kNoRow ? MT_DELI_BIG_CLIENTS : MT_MAX_CLIENTS;
            const int32_t* scsn = prow != kNoRow ? g.pool[0].csn + (size_t)prow * MT_DELI_BIG_CLIENTS : g.csn + (size_t)d * MT_MAX_CLIENTS;
            const int32_t* sref = prow != kNoRow ? g.pool[0].ref + (size_t)prow * MT_DELI_BIG_CLIENTS : g.ref + (size_t)d * MT_MAX_CLIENTS;
            const uint8_t* sfl = prow != kNoRow ? g.pool[0].fl + (size_t)prow * MT_DELI_BIG_CLIENTS : g.fl + (size_t)d * MT_MAX_CLIENTS;
            const size_t dst = (size_t)row * NCL;
            for (int c = lane; c < NCL; c += 64) {
                const bool in = c < npc;
                pl.csn[dst + c] = in ? scsn[c] : 0;
                pl.ref[dst + c] = in ? sref[c] : 0;
                pl.fl[dst + c] = in ? sfl[c] : (uint8_t)0;
            }
            __threadfence_block();
            if (lane == 0) pl.row[d] = row;
        }
        const size_t cb = (size_t)row * NCL + (size_t)lane * P;
        deli_group<64, P, TIER == 0 ? 1 : -1>(g, msgs, d, true, r0, len, m0, pl.csn + cb, pl.ref + cb, pl.fl + cb,
                                              out, ops, n_ops, stage);
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
        g.pool[0].row[d] = kNoRow;  // (every document restored: the pools start over)
        g.pool[1].row[d] = kNoRow;
        if (d == 0) {
            g.ctl[0] = g.ctl[2] = 0u;
            g.ctl[4] = g.ctl[6] = 0u;
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
// rows of the pools (documents past client 63 / 511 at once): the big pool one per 16 documents, at
// least 64; the huge pool one per 256, at least 8 (a row of it is 4096 clients, 36 KiB)
static uint32_t deli_pool_rows(int tier, uint32_t max_docs) {
    return tier == 0 ? std::max<uint32_t>(64u, max_docs / 16u) : std::max<uint32_t>(8u, max_docs / 256u);
}
static constexpr uint32_t kPoolClients[2] = {MT_DELI_BIG_CLIENTS, MT_DELI_MAX_CLIENTS};

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
// the rows of both pools held by documents [doc0, doc0 + n) go back to their free lists (their
// documents are about to be restored); the stream is idle
mt_status release_rows(mt_deli* dl, uint32_t doc0, uint32_t n) {
    for (int t = 0; t < 2; t++) {
        const mtd::Pool& pl = dl->g.pool[t];
        std::vector<uint32_t> held(n);
        DL_HIP(hipMemcpy(held.data(), pl.row + doc0, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
        std::vector<uint32_t> rows;
        for (uint32_t r : held)
            if (r != mtd::kNoRow) rows.push_back(r);
        if (rows.empty()) continue;
        int32_t nfree = 0;
        DL_HIP(hipMemcpy(&nfree, dl->g.ctl + 4 * t + 2, sizeof nfree, hipMemcpyDeviceToHost));
        nfree = std::max(nfree, 0);
        if ((uint64_t)nfree + rows.size() > pl.cap) return MT_ERR_STATE;  // (a row freed twice)
        DL_HIP(hipMemcpy(pl.free_rows + nfree, rows.data(), rows.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        nfree += (int32_t)rows.size();
        DL_HIP(hipMemcpy(dl->g.ctl + 4 * t + 2, &nfree, sizeof nfree, hipMemcpyHostToDevice));
        DL_HIP(hipMemset(pl.row + doc0, 0xFF, n * sizeof(uint32_t)));
    }
    return MT_OK;
}
// the common form over every document, then the wide form over the documents it queued (past client
// 63: promoted now or earlier), then the huge form over those the wide form queued (past client 511),
// on one stream
mt_status launch_forms(mt_deli* dl, hipStream_t st, const mt_raw_msg* d_msgs, const uint32_t* d_row, uint32_t n_docs,
                       mt_ticket* d_out, mt_op_rec* d_ops, uint64_t n_ops) {
    DL_HIP(hipMemsetAsync(dl->g.ctl + 1, 0, sizeof(uint32_t), st));
    DL_HIP(hipMemsetAsync(dl->g.ctl + 5, 0, sizeof(uint32_t), st));
    hipLaunchKernelGGL(mtd::deli_kernel, dim3((n_docs + 7) / 8), dim3(64), 0, st, dl->g,
                       reinterpret_cast<const int4*>(d_msgs), d_row, n_docs, reinterpret_cast<int4*>(d_out), d_ops,
                       n_ops);
    DL_HIP(hipGetLastError());
    hipLaunchKernelGGL(mtd::deli_pool_kernel<0>, dim3(std::min<uint32_t>(1024u, n_docs)), dim3(64), 0, st, dl->g,
                       reinterpret_cast<const int4*>(d_msgs), d_row, reinterpret_cast<int4*>(d_out), d_ops, n_ops);
    DL_HIP(hipGetLastError());
    hipLaunchKernelGGL(mtd::deli_pool_kernel<1>, dim3(std::min<uint32_t>(256u, n_docs)), dim3(64), 0, st, dl->g,
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
    bool ok = hipStreamCreateWithFlags(&dl->stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreate(&dl->e0) == hipSuccess && hipEventCreate(&dl->e1) == hipSuccess &&
              hipMalloc(&dl->g.sc, max_docs * sizeof(int4)) == hipSuccess &&
              hipMalloc(&dl->g.err_at, max_docs * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.csn, nc * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.ref, nc * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&dl->g.fl, nc) == hipSuccess &&
              hipMalloc(&dl->g.ctl, 8 * sizeof(uint32_t)) == hipSuccess &&
              hipMemset(dl->g.ctl, 0, 8 * sizeof(uint32_t)) == hipSuccess;
    for (int t = 0; t < 2 && ok; t++) {
        mtd::Pool& pl = dl->g.pool[t];
        pl.cap = deli_pool_rows(t, max_docs);
        const size_t nb = (size_t)pl.cap * kPoolClients[t];
        ok = hipMalloc(&pl.row, max_docs * sizeof(uint32_t)) == hipSuccess &&
             hipMalloc(&pl.resume, max_docs * sizeof(int32_t)) == hipSuccess &&
             hipMalloc(&pl.queue, max_docs * sizeof(uint32_t)) == hipSuccess &&
             hipMalloc(&pl.csn, nb * sizeof(int32_t)) == hipSuccess &&
             hipMalloc(&pl.ref, nb * sizeof(int32_t)) == hipSuccess && hipMalloc(&pl.fl, nb) == hipSuccess &&
             hipMalloc(&pl.free_rows, pl.cap * sizeof(uint32_t)) == hipSuccess &&
             hipMemset(pl.row, 0xFF, max_docs * sizeof(uint32_t)) == hipSuccess;
    }
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
                    (void*)dl->g.ctl})
        if (p) hipFree(p);
    for (const mtd::Pool& pl : dl->g.pool)
        for (void* p : {(void*)pl.row, (void*)pl.resume, (void*)pl.queue, (void*)pl.csn, (void*)pl.ref, (void*)pl.fl,
                        (void*)pl.free_rows})
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
    // (a restored document is back in the common form; the rows it held are on the free lists now)
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

// the form holding a document's clients: its row of the huge pool (tier 1), else of the big pool
// (tier 0), else the narrow arrays (tier -1, row kNoRow)
static mt_status doc_tier(mt_deli* dl, uint32_t doc, int* tier, uint32_t* row) {
    uint32_t r[2];
    for (int t = 0; t < 2; t++) DL_HIP(hipMemcpy(&r[t], dl->g.pool[t].row + doc, sizeof r[t], hipMemcpyDeviceToHost));
    *tier = r[1] != mtd::kNoRow ? 1 : (r[0] != mtd::kNoRow ? 0 : -1);
    *row = *tier >= 0 ? r[*tier] : mtd::kNoRow;
    return MT_OK;
}
// clients [c0, c0 + n) of a document, from the form holding them
static mt_status read_clients(mt_deli* dl, uint32_t doc, uint32_t c0, uint32_t n, mt_deli_client* out) {
    int tier = -1;
    uint32_t row = mtd::kNoRow;
    DL_HIP(hipStreamSynchronize(dl->stream));
    if (const mt_status st = doc_tier(dl, doc, &tier, &row)) return st;
    std::vector<int32_t> csn(n, 0), ref(n, 0);
    std::vector<uint8_t> fl(n, 0);
    const uint32_t held = tier >= 0 ? kPoolClients[tier] : MT_MAX_CLIENTS;
    const uint32_t m = c0 < held ? std::min(n, held - c0) : 0u;
    const size_t o = tier >= 0 ? (size_t)row * held + c0 : (size_t)doc * MT_MAX_CLIENTS + c0;
    const int32_t* scsn = tier >= 0 ? dl->g.pool[tier].csn : dl->g.csn;
    const int32_t* sref = tier >= 0 ? dl->g.pool[tier].ref : dl->g.ref;
    const uint8_t* sfl = tier >= 0 ? dl->g.pool[tier].fl : dl->g.fl;
    if (m) {
        DL_HIP(hipMemcpy(csn.data(), scsn + o, m * sizeof(int32_t), hipMemcpyDeviceToHost));
        DL_HIP(hipMemcpy(ref.data(), sref + o, m * sizeof(int32_t), hipMemcpyDeviceToHost));
        DL_HIP(hipMemcpy(fl.data(), sfl + o, m, hipMemcpyDeviceToHost));
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
    int tier = -1;
    uint32_t row = mtd::kNoRow;
    DL_HIP(hipStreamSynchronize(dl->stream));
    DL_HIP(hipMemcpy(&sc, dl->g.sc + doc, sizeof sc, hipMemcpyDeviceToHost));
    if (const mt_status st = doc_tier(dl, doc, &tier, &row)) return st;
    // a promoted document whose clients past the checkpoint's range hold state does not fit it:
    // refuse rather than drop them (a restore from it would lose them and derive another msn)
    if (tier >= 0 && NC < kPoolClients[tier]) {
        std::vector<uint8_t> fl(kPoolClients[tier] - NC);
        DL_HIP(hipMemcpy(fl.data(), dl->g.pool[tier].fl + (size_t)row * kPoolClients[tier] + NC, fl.size(),
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
    // each document's tier: the form holding its highest client with state (joined or nacked)
    std::vector<int> tier(n, -1);
    uint32_t need[2] = {0, 0};
    for (uint32_t i = 0; i < n; i++) {
        int top = -1;
        for (int c = MT_DELI_MAX_CLIENTS - 1; c >= MT_MAX_CLIENTS && top < 0; c--)
            if (ckpts[i].clients[c].joined || ckpts[i].clients[c].nack) top = c;
        tier[i] = top < 0 ? -1 : (top < MT_DELI_BIG_CLIENTS ? 0 : 1);
        if (tier[i] >= 0) need[tier[i]]++;
    }
    // whether the pools hold them once the rows of [doc0, doc0 + n) are back on the free lists
    uint32_t ctl[8];
    DL_HIP(hipMemcpy(ctl, dl->g.ctl, sizeof ctl, hipMemcpyDeviceToHost));
    for (int t = 0; t < 2; t++) {
        std::vector<uint32_t> held(n);
        DL_HIP(hipMemcpy(held.data(), dl->g.pool[t].row + doc0, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
        const uint32_t freed = (uint32_t)std::count_if(held.begin(), held.end(), [](uint32_t r) { return r != mtd::kNoRow; });
        const uint32_t fresh = std::min(ctl[4 * t], dl->g.pool[t].cap);
        const uint32_t nfree = (uint32_t)std::max((int32_t)ctl[4 * t + 2], 0);
        if (need[t] > (size_t)(dl->g.pool[t].cap - fresh) + nfree + freed) return MT_ERR_NOMEM;
    }
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
    if (need[0] + need[1] == 0) return MT_OK;
    // rows for the promoted documents: each tier's free list first (mt_deli_restore just pushed), then fresh
    DL_HIP(hipMemcpy(ctl, dl->g.ctl, sizeof ctl, hipMemcpyDeviceToHost));
    for (int t = 0; t < 2; t++) {
        mtd::Pool& pl = dl->g.pool[t];
        const uint32_t NCL = kPoolClients[t];
        int32_t top = std::max((int32_t)ctl[4 * t + 2], 0);
        uint32_t next = std::min(ctl[4 * t], pl.cap);
        std::vector<uint32_t> stack((size_t)top);
        if (top) DL_HIP(hipMemcpy(stack.data(), pl.free_rows, top * sizeof(uint32_t), hipMemcpyDeviceToHost));
        std::vector<int32_t> csn(NCL), ref(NCL);
        std::vector<uint8_t> fl(NCL);
        for (uint32_t i = 0; i < n; i++) {
            if (tier[i] != t) continue;
            const uint32_t row = top > 0 ? stack[--top] : next++;  // (capacity checked above)
            const mt_deli_checkpoint_wide& ck = ckpts[i];
            for (uint32_t c = 0; c < NCL; c++) {
                csn[c] = ck.clients[c].csn;
                ref[c] = ck.clients[c].ref_seq;
                fl[c] = client_flags(ck.clients[c]);
            }
            const size_t o = (size_t)row * NCL;
            DL_HIP(hipMemcpy(pl.csn + o, csn.data(), NCL * sizeof(int32_t), hipMemcpyHostToDevice));
            DL_HIP(hipMemcpy(pl.ref + o, ref.data(), NCL * sizeof(int32_t), hipMemcpyHostToDevice));
            DL_HIP(hipMemcpy(pl.fl + o, fl.data(), NCL, hipMemcpyHostToDevice));
            DL_HIP(hipMemcpy(pl.row + doc0 + i, &row, sizeof row, hipMemcpyHostToDevice));
            // the constructor's msn over every client (lambda.ts:166-167)
            const int4 sc = make_int4(ck.seq, ckpt_msn(ck), ck.last_sent_msn, 0);
            DL_HIP(hipMemcpy(dl->g.sc + doc0 + i, &sc, sizeof sc, hipMemcpyHostToDevice));
        }
        ctl[4 * t] = std::max(ctl[4 * t], next);
        ctl[4 * t + 2] = (uint32_t)top;
    }
    DL_HIP(hipMemcpy(dl->g.ctl, ctl, sizeof ctl, hipMemcpyHostToDevice));  // ([1] / [5] are per call)
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
