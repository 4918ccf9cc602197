"""Document sharding across GPUs (one process per GPU) and the end-of-run checksum gather.

Documents are independent (one Client / DeliLambda per document).  The reference partitions
its ordering service by documentId: Kafka messages are keyed by it
(server/routerlicious/packages/services/src/kafkaNodeProducer.ts:131, keyed partitioner :156)
and the per-document lambdas are routed on it (lambdas-driver/src/document-router/
documentLambda.ts:52-58).  Here document `docId` lives on rank splitmix64(docId) mod n_ranks
(`route`, the same function as libmtgpu's mt_route_doc), so the apply loop has no collective.
The one exchange is the final gather of per-document checksums to rank 0, XOR-folded into a node
digest:

* `RcclComm`  -- libmtgpu's mt_comm_* over RCCL (xGMI), straight from HBM; ranks on distinct
                 GPUs (the bench on a node).  Bootstrap: rank 0's ncclUniqueId handed to the other
                 ranks through a rendezvous file (`FileRendezvous`; all ranks of a job run on one
                 node), so no process loads another runtime for a side channel.
* `GlooComm`  -- torch.distributed over gloo on host memory (CPU tests; ranks sharing one GPU,
                 which RCCL does not allow).
"""
import ctypes
import os
import tempfile
import time

import numpy as np

_M64 = (1 << 64) - 1


def splitmix64(x):
    """mt_mix64 (fluidframework_amd/csrc/mt_synth.h) on a numpy uint64 array."""
    z = np.asarray(x, dtype=np.uint64).copy()
    with np.errstate(over='ignore'):
        z += np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def route(doc_ids, n_ranks):
    """Rank owning each document: splitmix64(docId) mod n_ranks (= mt_route_docs)."""
    return (splitmix64(doc_ids) % np.uint64(n_ranks)).astype(np.uint32)


def shard_ids(rank, n_ranks, n_total):
    """Global ids (ascending) of the documents of [0, n_total) that live on `rank`."""
    ids = np.arange(n_total, dtype=np.uint64)
    return ids[route(ids, n_ranks) == rank].astype(np.uint32)


def digest(checksums):
    cs = np.ascontiguousarray(checksums, dtype=np.uint64)
    return int(np.bitwise_xor.reduce(cs.view(np.int64))) & _M64 if len(cs) else 0


def assemble(parts, ids_per_rank):
    """Rank-ordered checksum lists -> checksums in global document order."""
    n = sum(len(i) for i in ids_per_rank)
    out = np.zeros(n, dtype=np.uint64)
    for cs, ids in zip(parts, ids_per_rank):
        out[np.asarray(ids, dtype=np.int64)] = cs
    return out


class LocalComm:
    """World size 1: nothing to exchange."""
    rank, world = 0, 1

    def barrier(self):
        pass

    def max(self, x):
        return x

    def gather_checksums(self, cs_or_engine, max_docs=None):
        cs = cs_or_engine.checksums() if hasattr(cs_or_engine, 'checksums') else cs_or_engine
        return [np.ascontiguousarray(cs, dtype=np.uint64)]

    def close(self):
        pass


class GlooComm:
    """torch.distributed (gloo, host tensors) -- the CPU tests' and shared-GPU ranks' path."""

    def __init__(self, dist):
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def barrier(self):
        self.dist.barrier()

    def max(self, x):
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_checksums(self, cs_or_engine, max_docs):
        """Rank 0: list of every rank's checksums (rank order); others: None."""
        import torch
        cs = cs_or_engine.checksums() if hasattr(cs_or_engine, 'checksums') else cs_or_engine
        cs = np.ascontiguousarray(cs, dtype=np.uint64)
        row = np.zeros(max_docs + 1, dtype=np.int64)
        row[0] = len(cs)
        row[1:1 + len(cs)] = cs.view(np.int64)
        t = torch.from_numpy(row)
        got = [torch.empty_like(t) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(t, got, dst=0)
        if self.rank != 0:
            return None
        return [g.numpy()[1:1 + int(g[0])].view(np.uint64).copy() for g in got]

    def close(self):
        pass


class FileRendezvous:
    """Hands rank 0's bytes to the other ranks of a single-node job through a file under /tmp,
    keyed by the job's MASTER_ADDR/PORT and launcher (torchrun's agent or bench.py's spawner)."""

    def __init__(self, key=None, timeout=300.0):
        if key is None:
            key = '_'.join([os.environ.get('MASTER_ADDR', '127.0.0.1'), os.environ.get('MASTER_PORT', '0'),
                            os.environ.get('MTGPU_RUN_ID') or os.environ.get('TORCHELASTIC_RUN_ID', 'none'),
                            str(os.getppid())])
        self.path = os.path.join(tempfile.gettempdir(), f'mtgpu_rdv_{key.replace("/", "_")}')
        self.timeout = timeout

    def publish(self, data: bytes):
        tmp = self.path + f'.{os.getpid()}.tmp'
        with open(tmp, 'wb') as f:
            f.write(data)
        os.replace(tmp, self.path)

    def fetch(self, nbytes):
        t0 = time.time()
        while True:
            try:
                with open(self.path, 'rb') as f:
                    data = f.read()
                if len(data) == nbytes:
                    return data
            except FileNotFoundError:
                pass
            if time.time() - t0 > self.timeout:
                raise TimeoutError(f'rendezvous {self.path}: no id from rank 0 after {self.timeout} s')
            time.sleep(0.05)

    def cleanup(self):
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass


class RcclComm:
    """libmtgpu's RCCL communicator (mt_comm_*): one rank per GPU of one node."""

    def __init__(self, rank, world, device, rendezvous=None):
        from .engine import _check, lib
        self._check = _check
        L = self.L = lib()
        vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32
        L.mt_comm_unique_id.argtypes = [ctypes.c_char_p]
        L.mt_comm_create.argtypes = [i32, i32, i32, ctypes.c_char_p, ctypes.POINTER(vp)]
        L.mt_comm_destroy.argtypes = [vp]
        L.mt_comm_gather_checksums.argtypes = [vp, vp, u32, vp, vp]
        L.mt_comm_allreduce_max_f64.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.mt_comm_barrier.argtypes = [vp]
        for f in ('mt_comm_unique_id', 'mt_comm_create', 'mt_comm_destroy', 'mt_comm_gather_checksums',
                  'mt_comm_allreduce_max_f64', 'mt_comm_barrier'):
            getattr(L, f).restype = ctypes.c_int
        self.rank, self.world = rank, world
        self.rdv = rendezvous or FileRendezvous()
        idb = ctypes.create_string_buffer(128)
        if rank == 0:
            _check(L.mt_comm_unique_id(idb), 'mt_comm_unique_id')
            self.rdv.publish(idb.raw)
        else:
            idb = ctypes.create_string_buffer(self.rdv.fetch(128), 128)
        self.h = ctypes.c_void_p()
        _check(L.mt_comm_create(device, rank, world, idb, ctypes.byref(self.h)), 'mt_comm_create')
        if rank == 0:
            self.rdv.cleanup()

    def barrier(self):
        self._check(self.L.mt_comm_barrier(self.h), 'mt_comm_barrier')

    def max(self, x):
        v = ctypes.c_double(x)
        self._check(self.L.mt_comm_allreduce_max_f64(self.h, ctypes.byref(v)), 'mt_comm_allreduce_max_f64')
        return v.value

    def gather_checksums(self, engine, max_docs):
        """ncclGather of every rank's per-document checksums (computed in HBM) to rank 0."""
        from .engine import _ptr
        out = np.zeros(self.world * max_docs if self.rank == 0 else 1, dtype=np.uint64)
        counts = np.zeros(self.world, dtype=np.uint32)
        self._check(self.L.mt_comm_gather_checksums(self.h, engine.h, max_docs, _ptr(out), _ptr(counts)),
                    'mt_comm_gather_checksums')
        if self.rank != 0:
            return None
        return [out[r * max_docs:r * max_docs + int(counts[r])].copy() for r in range(self.world)]

    def close(self):
        if getattr(self, 'h', None):
            self.L.mt_comm_destroy(self.h)
            self.h = None
