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
// Device mapping: one wave64 per document, lane c owns client c's record (clientSequenceNumber,
// referenceSequenceNumber, joined / nacked) in VGPRs, so the heap becomes a wave-wide min (six
// DPP steps, no data-dependent memory traffic) and a client lookup is one v_readlane.  The
// document's scalars (sequenceNumber, msn, lastSentMSN) live in SGPRs; the per-message decision
// tree is wave-uniform scalar code.  Messages are read 64 at a time with one coalesced 16-byte
// load per lane, and tickets are written back the same way.  HBM traffic is the algorithmic
// minimum: 16 B in + 16 B out per message, plus 9 B per client slot in and out per document.
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

// per-document state in HBM (structure of arrays; client arrays are [doc * 64 + client])
struct DeliState {
    int4* sc;         // {sequenceNumber, minimumSequenceNumber, lastSentMSN, err}
    int32_t* err_at;  // message index (inside the document's stream) of the sticky error
    int32_t* csn;
    int32_t* ref;
    uint8_t* fl;      // CL_JOINED | CL_NACK
};

// wave-wide minimum: row_shr 1/2/4/8 leave each 16-lane row's minimum in its lane 15,
// row_bcast:15 / row_bcast:31 carry it across rows, lane 63 ends with the wave's minimum
MT_DEV int wave_min_dpp(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x111, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x112, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x114, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x118, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x142, 0xa, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}

// One wave per document: ticket every raw message of the document in order.
__global__ __launch_bounds__(64) void deli_kernel(DeliState g, const int4* __restrict__ msgs,
                                                  const uint32_t* __restrict__ row_ptr, uint32_t n_docs,
                                                  int4* __restrict__ out, mt_op_rec* __restrict__ ops) {
    const uint32_t d = blockIdx.x;
    if (d >= n_docs) return;
    const int lane = lane_id();
    const uint32_t r0 = row_ptr[d], r1 = row_ptr[d + 1];
    if (r0 >= r1) return;
    const int4 s0 = g.sc[d];
    int seq = s0.x, msn = s0.y, last = s0.z, err = s0.w;
    int err_at = g.err_at[d];
    const size_t cb = (size_t)d * MT_MAX_CLIENTS + lane;
    int csn = g.csn[cb], ref = g.ref[cb], fl = g.fl[cb];

    int4 m = make_int4(0, 0, 0, 0);
    if (r0 + lane < r1) m = msgs[r0 + lane];
    for (uint32_t base = r0; base < r1; base += 64) {
        const int n = (int)min(64u, r1 - base);
        const int4 cur = m;
        // the next 64 messages are in flight while these are ticketed
        if (base + 64 + lane < r1) m = msgs[base + 64 + lane];
        int4 t = make_int4(0, 0, 0, 0);
        for (int j = 0; j < n; j++) {
            const int mc = __builtin_amdgcn_readlane(cur.x, j);
            const int mr = __builtin_amdgcn_readlane(cur.y, j);
            const int w = __builtin_amdgcn_readlane(cur.z, j);
            const int c = w & 0xFFFF, kind = (w >> 16) & 0xFF;
            int ts = seq, tr = mr, st = MT_TK_SENT;
            if (err) {
                st = MT_TK_HALTED;
            } else if (c >= MT_MAX_CLIENTS || kind > MT_RAW_CONTROL) {
                err = c >= MT_MAX_CLIENTS ? MT_DELI_ERR_CLIENT : MT_DELI_ERR_KIND;
                err_at = (int)(base + j - r0);
                st = MT_TK_HALTED;
            } else {
                const int cfl = __builtin_amdgcn_readlane(fl, c);
                const int ccsn = __builtin_amdgcn_readlane(csn, c);
                const bool joined = (cfl & CL_JOINED) != 0;
                int upd = 0, ucsn = 0, uref = 0, unack = 0;  // upd: 1 upsert, 2 remove
                if (kind <= MT_RAW_NOOP_DATA) {  // a client message (message.clientId set)
                    if (joined && mc > ccsn + 1) {
                        st = MT_TK_NACK_GAP;           // checkOrder Gap (:613-620, 269-275)
                    } else if (joined && mc < ccsn + 1) {
                        st = MT_TK_DROPPED;            // checkOrder Duplicate (:621-625, 267-268)
                    } else if (!joined || (cfl & CL_NACK)) {
                        st = MT_TK_NACK_CLIENT;        // (:308-316)
                    } else if (mr != -1 && mr < msn) {  // (:317-335): the client stays nacked
                        st = MT_TK_NACK_REFSEQ;
                        upd = 1, ucsn = mc, uref = msn, unack = CL_NACK;
                    } else {
                        if (kind == MT_RAW_OP) {       // client no-ops do not rev (:414-425)
                            ts = ++seq;
                            if (mr == -1) tr = ts;
                        }
                        if (tr < msn) {                // assert(refSeq >= msn) (:426-428) throws
                            err = MT_DELI_ERR_ASSERT;
                            err_at = (int)(base + j - r0);
                            st = MT_TK_HALTED;
                        } else {
                            upd = 1, ucsn = mc, uref = tr;  // upsertClient (:430-435)
                        }
                    }
                } else if (kind == MT_RAW_LEAVE) {     // removeClient (:281-285)
                    if (!joined) st = MT_TK_DROPPED;
                    else upd = 2, ts = ++seq;
                } else if (kind == MT_RAW_JOIN) {      // upsertClient(c, 0, msn) (:286-299)
                    upd = 1, ucsn = 0, uref = msn;
                    if (joined) st = MT_TK_DROPPED;    // the state is reset all the same
                    else ts = ++seq;
                }
                if (upd && lane == c) {
                    if (upd == 2) {
                        fl = 0;
                    } else {
                        csn = ucsn;
                        ref = uref;
                        fl = CL_JOINED | unack;
                    }
                }
                if (st == MT_TK_SENT) {
                    // getMinimumSequenceNumber over the tracked clients (:446-455)
                    const int mn = wave_min_dpp((fl & CL_JOINED) ? ref : INT_MAX);
                    const bool none = mn == INT_MAX;
                    msn = none ? ts : mn;
                    if (kind == MT_RAW_NOOP) {                 // contents null: Later (:463-465)
                        st = MT_TK_LATER;
                    } else if (kind == MT_RAW_NOOP_DATA) {     // (:466-471)
                        if (msn <= last) st = MT_TK_LATER;
                        else ts = ++seq;
                    } else if (kind == MT_RAW_SERVER_NOOP) {   // (:473-479)
                        if (msn <= last) st = MT_TK_NEVER;
                        else ts = ++seq;
                    } else if (kind == MT_RAW_NOCLIENT) {      // (:481-489)
                        if (none) {
                            ts = ++seq;
                            tr = ts;
                            msn = ts;
                        } else {
                            st = MT_TK_NEVER;
                        }
                    } else if (kind == MT_RAW_CONTROL) {       // (:490-517)
                        st = MT_TK_NEVER;
                    }
                    if (st == MT_TK_SENT) last = msn;          // handler (:217-218)
                } else if (st >= MT_TK_NACK_GAP && st <= MT_TK_NACK_REFSEQ) {
                    ts = msn;                                  // createNackMessage (:683-712)
                    last = msn;
                }
            }
            if (lane == j) t = make_int4(ts, msn, tr, st);
        }
        if (lane < n) {
            out[base + lane] = t;
            if (ops) {
                mt_op_rec* o = ops + base + lane;
                o->seq = t.w == MT_TK_SENT ? t.x : -1;
                o->msn = t.y;
                o->ref_seq = t.z;
            }
        }
    }
    if (lane == 0) {
        g.sc[d] = make_int4(seq, msn, last, err);
        g.err_at[d] = err_at;
    }
    g.csn[cb] = csn;
    g.ref[cb] = ref;
    g.fl[cb] = (uint8_t)fl;
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
        if (lane < n) msgs[base + lane] = make_int4(mine, rf, (cl & 0xFFFF) | (MT_RAW_OP << 16), 0);
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
int32_t ckpt_msn(const mt_deli_checkpoint& ck) {
    int32_t m = INT_MAX;
    for (int c = 0; c < MT_MAX_CLIENTS; c++)
        if (ck.clients[c].joined) m = std::min(m, ck.clients[c].ref_seq);
    return m == INT_MAX ? ck.seq : m;
}
mt_status launch_ticket(mt_deli* dl, const mt_raw_msg* d_msgs, const uint32_t* d_row, uint32_t n_docs,
                        mt_ticket* d_out, mt_op_rec* d_ops) {
    DL_HIP(hipEventRecord(dl->e0, dl->stream));
    hipLaunchKernelGGL(mtd::deli_kernel, dim3(n_docs), dim3(64), 0, dl->stream, dl->g,
                       reinterpret_cast<const int4*>(d_msgs), d_row, n_docs, reinterpret_cast<int4*>(d_out), d_ops);
    DL_HIP(hipGetLastError());
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
              hipMalloc(&dl->g.fl, nc) == hipSuccess;
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
    hipFree(dl->g.sc);
    hipFree(dl->g.err_at);
    hipFree(dl->g.csn);
    hipFree(dl->g.ref);
    hipFree(dl->g.fl);
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
            fl[k] = (uint8_t)((ck.clients[c].joined ? mtd::CL_JOINED : 0) | (ck.clients[c].nack ? mtd::CL_NACK : 0));
        }
    }
    const size_t c0 = (size_t)doc0 * MT_MAX_CLIENTS, nc = (size_t)n * MT_MAX_CLIENTS;
    DL_HIP(hipMemcpyAsync(dl->g.sc + doc0, sc.data(), n * sizeof(int4), hipMemcpyHostToDevice, dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.err_at + doc0, err_at.data(), n * sizeof(int32_t), hipMemcpyHostToDevice,
                          dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.csn + c0, csn.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.ref + c0, ref.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, dl->stream));
    DL_HIP(hipMemcpyAsync(dl->g.fl + c0, fl.data(), nc, hipMemcpyHostToDevice, dl->stream));
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
    if (st == MT_OK) st = launch_ticket(dl, d_msgs, d_row, n_docs, d_out, nullptr);
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
                                mt_ticket* d_out, mt_op_rec* d_ops) {
    if (!dl || !d_msgs || !d_row_ptr || !d_out || n_docs > dl->max_docs) return MT_ERR_ARG;
    if (n_docs == 0) return MT_OK;
    DL_HIP(hipSetDevice(dl->device));
    return launch_ticket(dl, d_msgs, d_row_ptr, n_docs, d_out, d_ops);
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

mt_status mt_deli_get_checkpoint(mt_deli* dl, uint32_t doc, mt_deli_checkpoint* out) {
    if (!dl || !out || doc >= dl->max_docs) return MT_ERR_ARG;
    DL_HIP(hipSetDevice(dl->device));
    int4 sc;
    int32_t csn[MT_MAX_CLIENTS], ref[MT_MAX_CLIENTS];
    uint8_t fl[MT_MAX_CLIENTS];
    const size_t c0 = (size_t)doc * MT_MAX_CLIENTS;
    DL_HIP(hipStreamSynchronize(dl->stream));
    DL_HIP(hipMemcpy(&sc, dl->g.sc + doc, sizeof sc, hipMemcpyDeviceToHost));
    DL_HIP(hipMemcpy(csn, dl->g.csn + c0, sizeof csn, hipMemcpyDeviceToHost));
    DL_HIP(hipMemcpy(ref, dl->g.ref + c0, sizeof ref, hipMemcpyDeviceToHost));
    DL_HIP(hipMemcpy(fl, dl->g.fl + c0, sizeof fl, hipMemcpyDeviceToHost));
    memset(out, 0, sizeof *out);
    out->seq = sc.x;
    out->msn = sc.y;
    out->last_sent_msn = sc.z;
    out->err = sc.w;
    for (int c = 0; c < MT_MAX_CLIENTS; c++) {
        const bool joined = (fl[c] & mtd::CL_JOINED) != 0;
        out->clients[c].joined = joined;
        out->clients[c].nack = (fl[c] & mtd::CL_NACK) != 0;
        out->clients[c].csn = joined ? csn[c] : 0;
        out->clients[c].ref_seq = joined ? ref[c] : 0;
    }
    return MT_OK;
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
