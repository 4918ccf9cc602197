// mt_comm.cpp -- the multi-GPU side of libmtgpu.so: document routing and the one collective.
//
// The reference partitions its ordering service by document: Kafka messages are keyed by
// documentId (server/routerlicious/packages/services/src/kafkaNodeProducer.ts:131, keyed
// partitioner :156) and the per-document lambdas are routed on the same key
// (server/routerlicious/packages/lambdas-driver/src/document-router/documentLambda.ts:52-58).
// Here a document lives on GPU splitmix64(docId) mod n_gpus; its deli state, op log and merge
// tree never leave that GPU, so the apply loop has no collective at all.  The one exchange is at
// the end: every rank's per-document checksums are gathered to rank 0 over RCCL (xGMI), straight
// from HBM (ncclGather), plus the scalar all-reduce / barrier a benchmark needs for its clock.
// One process per GPU; ranks rendezvous through an ncclUniqueId the host hands around.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "../../include/mtgpu.h"
#include "mt_synth.h"

static_assert(MT_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "mt_comm id size");

struct mt_comm {
    int32_t device = 0, rank = 0, n_ranks = 1;
    ncclComm_t nc = nullptr;
    hipStream_t stream = nullptr;
    double* d_scalar = nullptr;
};

#define CM_HIP(x)                                                                                            \
    do {                                                                                                     \
        hipError_t e_ = (x);                                                                                 \
        if (e_ != hipSuccess) {                                                                              \
            fprintf(stderr, "libmtgpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return MT_ERR_HIP;                                                                               \
        }                                                                                                    \
    } while (0)
#define CM_NCCL(x)                                                                                           \
    do {                                                                                                     \
        ncclResult_t r_ = (x);                                                                               \
        if (r_ != ncclSuccess) {                                                                             \
            fprintf(stderr, "libmtgpu: %s failed: %s (%s:%d)\n", #x, ncclGetErrorString(r_), __FILE__,         \
                    __LINE__);                                                                               \
            return MT_ERR_COMM;                                                                              \
        }                                                                                                    \
    } while (0)

extern "C" {

uint32_t mt_route_doc(uint64_t doc_id, uint32_t n_shards) {
    return n_shards ? (uint32_t)(mt_mix64(doc_id) % n_shards) : 0u;
}

mt_status mt_route_docs(const uint64_t* doc_ids, uint64_t n, uint32_t n_shards, uint32_t* shard_out) {
    if ((n && (!doc_ids || !shard_out)) || n_shards == 0) return MT_ERR_ARG;
    for (uint64_t i = 0; i < n; i++) shard_out[i] = mt_route_doc(doc_ids[i], n_shards);
    return MT_OK;
}

mt_status mt_comm_unique_id(uint8_t* id) {
    if (!id) return MT_ERR_ARG;
    ncclUniqueId u;
    CM_NCCL(ncclGetUniqueId(&u));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return MT_OK;
}

mt_status mt_comm_create(int32_t device, int32_t rank, int32_t n_ranks, const uint8_t* id, mt_comm** out) {
    if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) return MT_ERR_ARG;
    CM_HIP(hipSetDevice(device));
    auto* c = new mt_comm();
    c->device = device;
    c->rank = rank;
    c->n_ranks = n_ranks;
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_scalar, sizeof(double)) != hipSuccess) {
        mt_comm_destroy(c);
        return MT_ERR_HIP;
    }
    const ncclResult_t r = ncclCommInitRank(&c->nc, n_ranks, u, rank);
    if (r != ncclSuccess) {
        fprintf(stderr, "libmtgpu: ncclCommInitRank failed: %s\n", ncclGetErrorString(r));
        c->nc = nullptr;
        mt_comm_destroy(c);
        return MT_ERR_COMM;
    }
    *out = c;
    return MT_OK;
}

mt_status mt_comm_destroy(mt_comm* c) {
    if (!c) return MT_ERR_ARG;
    hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->nc) ncclCommDestroy(c->nc);
    if (c->d_scalar) (void)hipFree(c->d_scalar);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return MT_OK;
}

mt_status mt_comm_allreduce_max_f64(mt_comm* c, double* v) {
    if (!c || !v) return MT_ERR_ARG;
    CM_HIP(hipSetDevice(c->device));
    CM_HIP(hipMemcpyAsync(c->d_scalar, v, sizeof(double), hipMemcpyHostToDevice, c->stream));
    CM_NCCL(ncclAllReduce(c->d_scalar, c->d_scalar, 1, ncclFloat64, ncclMax, c->nc, c->stream));
    CM_HIP(hipMemcpyAsync(v, c->d_scalar, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    CM_HIP(hipStreamSynchronize(c->stream));
    return MT_OK;
}

mt_status mt_comm_barrier(mt_comm* c) {
    if (!c) return MT_ERR_ARG;
    double z = 0.0;
    mt_status st = mt_comm_allreduce_max_f64(c, &z);
    if (st) return st;
    CM_HIP(hipDeviceSynchronize());
    return MT_OK;
}

// Every rank enters the gather: a rank whose own part fails after the argument checks (engine
// query, more documents than the agreed bound, the checksum kernel) takes part with a poisoned row
// (count = ~0), which rank 0 reports as MT_ERR_COMM -- so no peer is left blocked in ncclGather.
// Only a rank that cannot take part at all (no device, no memory for its row) aborts the
// communicator; that is best effort: RCCL gives intra-node peers no failure detection, so an
// in-flight collective on another rank may still wait.
static mt_status comm_abort(mt_comm* c, mt_status st) {
    fprintf(stderr, "libmtgpu: rank %d cannot join the checksum gather: aborting the communicator\n", c->rank);
    if (c->nc) (void)ncclCommAbort(c->nc);
    c->nc = nullptr;
    return st;
}

mt_status mt_comm_gather_checksums(mt_comm* c, mt_engine* eng, uint32_t max_docs_per_rank, uint64_t* out,
                                   uint32_t* counts) {
    if (!c || !eng || !c->nc) return MT_ERR_ARG;
    if (c->rank == 0 && (!out || !counts)) return MT_ERR_ARG;
    mt_status fail = MT_OK;  // this rank's own failure: its row goes out poisoned
    uint32_t n_docs = 0;
    if (mt_engine_info(eng, &n_docs, nullptr) != MT_OK) {
        fail = MT_ERR_ARG;
        n_docs = 0;
    } else if (n_docs > max_docs_per_rank) {  // (the bound must be agreed; a rank past it still joins)
        fprintf(stderr, "libmtgpu: rank %d holds %u documents, past the gather's bound %u\n", c->rank, n_docs,
                max_docs_per_rank);
        fail = MT_ERR_ARG;
        n_docs = 0;
    }
    if (hipSetDevice(c->device) != hipSuccess) return comm_abort(c, MT_ERR_HIP);
    // [0] = this rank's document count, [1 .. max] = its checksums (zero padded): one gather
    const size_t row = (size_t)max_docs_per_rank + 1;
    uint64_t *d_send = nullptr, *d_recv = nullptr;
    if (hipMalloc(&d_send, row * sizeof(uint64_t)) != hipSuccess) return comm_abort(c, MT_ERR_NOMEM);
    if (c->rank == 0 && hipMalloc(&d_recv, row * c->n_ranks * sizeof(uint64_t)) != hipSuccess) {
        (void)hipFree(d_send);
        return comm_abort(c, MT_ERR_NOMEM);
    }
    uint64_t cnt = n_docs;
    bool ok = hipMemsetAsync(d_send, 0, row * sizeof(uint64_t), c->stream) == hipSuccess &&
              hipStreamSynchronize(c->stream) == hipSuccess;
    if (ok && n_docs) ok = mt_checksums_device(eng, d_send + 1, n_docs) == MT_OK;
    if (!ok && !fail) fail = MT_ERR_HIP;
    const bool local_ok = !fail;
    if (!local_ok) cnt = ~0ull;  // poisoned row: this rank's checksums are not valid
    ok = hipMemcpyAsync(d_send, &cnt, sizeof cnt, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
         hipStreamSynchronize(c->stream) == hipSuccess;
    if (!ok) {
        (void)hipFree(d_send);
        if (d_recv) (void)hipFree(d_recv);
        return comm_abort(c, MT_ERR_HIP);
    }
    const ncclResult_t r = ncclGather(d_send, d_recv, row, ncclUint64, 0, c->nc, c->stream);
    ok = r == ncclSuccess && hipStreamSynchronize(c->stream) == hipSuccess;
    bool poisoned = false;
    if (ok && c->rank == 0) {
        uint64_t* h = new uint64_t[row * c->n_ranks];
        ok = hipMemcpy(h, d_recv, row * c->n_ranks * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess;
        for (int q = 0; ok && q < c->n_ranks; q++) {
            poisoned = poisoned || h[(size_t)q * row] > max_docs_per_rank;
            counts[q] = poisoned ? 0u : (uint32_t)h[(size_t)q * row];
            memcpy(out + (size_t)q * max_docs_per_rank, h + (size_t)q * row + 1, max_docs_per_rank * sizeof(uint64_t));
        }
        delete[] h;
    }
    (void)hipFree(d_send);
    if (d_recv) (void)hipFree(d_recv);
    if (r != ncclSuccess) {
        fprintf(stderr, "libmtgpu: ncclGather failed: %s\n", ncclGetErrorString(r));
        return MT_ERR_COMM;
    }
    if (!local_ok) return fail;
    if (poisoned) {
        fprintf(stderr, "libmtgpu: a rank's checksums failed: the gather is incomplete\n");
        return MT_ERR_COMM;
    }
    return ok ? MT_OK : MT_ERR_HIP;
}

}  // extern "C"
