"""Document sharding across ranks (one process per GPU) and the end-of-run checksum gather.

Documents are independent (one Client / DeliLambda per document; reference analogue: Kafka keyed
by documentId, server/routerlicious/packages/kafka-orderer/src/kafkaNodeProducer.ts:131,156), so
each rank owns a contiguous block of global document ids and runs the apply with no collective.
The only collective is the final gather of per-document checksums to rank 0 (RCCL on the GPU
box, gloo in the CPU tests), XOR-folded into a node-level digest."""
import numpy as np


def doc_id_base(rank, docs_per_rank):
    """Global id of a rank's document 0 (weak scaling: every rank its own docs_per_rank docs)."""
    return rank * docs_per_rank


def digest(checksums):
    cs = np.ascontiguousarray(checksums, dtype=np.uint64)
    return int(np.bitwise_xor.reduce(cs.view(np.int64))) & 0xFFFFFFFFFFFFFFFF if len(cs) else 0


def gather_checksums(checksums, dist=None, device='cpu'):
    """Rank 0 gets every rank's per-document checksums (rank order = global doc order) and the
    node digest; other ranks get (None, None).  Without a process group: the local values."""
    cs = np.ascontiguousarray(checksums, dtype=np.uint64)
    if dist is None:
        return cs, digest(cs)
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    t = torch.from_numpy(cs.view(np.int64).copy()).to(device)
    gathered = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gathered, dst=0)
    if rank != 0:
        return None, None
    allcs = torch.cat(gathered).cpu().numpy().view(np.uint64)
    return allcs, digest(allcs)


def max_over_ranks(seconds, dist=None, device='cpu'):
    """The job's time: the slowest rank's."""
    if dist is None:
        return seconds
    import torch
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
