"""The multi-GPU path on the CPU and, with -m gpu, on the GPU box.

Documents are hash-routed to ranks (splitmix64(docId) mod n_ranks: fluidframework_amd/shard.py
`route` == libmtgpu `mt_route_docs`, the reference's documentId-keyed partitioning,
kafkaNodeProducer.ts:131,156); every rank replays only its documents; the per-document checksums
are gathered to rank 0 and assembled in global document order; the clock is the max over ranks.
CPU: world size 2 over gloo, each rank replaying its shard on the CPU oracle.  GPU box: bench.py
itself with --gpus 2 (its own rank spawner) -- two processes driving libmtgpu on device 0 with
the gloo exchange (RCCL refuses two ranks on one GPU) -- against the single-process run."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

CFG = dict(n_clients=8, ops_per_doc=96, max_lag=8, n_keys=2, n_values=4, p_insert=0.5, p_remove=0.3,
           p_insert_props=0.2)
N_TOTAL = 48


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from fluidframework_amd import shard
    from fluidframework_amd.oplog import OpBatch
    from oracle import oracle
    comm = shard.GlooComm(dist)
    ids = shard.shard_ids(rank, world, N_TOTAL)
    whole = oracle.generate(N_TOTAL, d0=0, threads=1, seed=5, **CFG)
    mine = whole.select(ids)
    o = oracle.Oracle(len(ids)).apply(mine)
    max_docs = int(comm.max(float(len(ids))))
    parts = comm.gather_checksums(o.checksums(), max_docs)
    t = comm.max(float(rank + 1))
    if rank == 0:
        allcs = shard.assemble(parts, [shard.shard_ids(r, world, N_TOTAL) for r in range(world)])
        np.save(out_path, np.concatenate([allcs.view(np.int64),
                                          np.array([shard.digest(allcs), int(t), len(parts[0]), len(parts[1])],
                                                   dtype=np.uint64).view(np.int64)]))
    comm.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_routing_and_gather(tmp_path, oracle_lib):
    import torch.multiprocessing as mp
    from fluidframework_amd.shard import digest, route
    world = 2
    out = str(tmp_path / 'rank0.npy')
    mp.spawn(_rank_main, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    allcs, (dg, t, n0, n1) = got[:-4].view(np.uint64), got[-4:].view(np.uint64).tolist()
    whole = oracle_lib.generate(N_TOTAL, d0=0, threads=2, seed=5, **CFG)
    want = oracle_lib.Oracle(N_TOTAL).apply(whole).checksums()
    assert np.array_equal(allcs, want)          # assembled in global document order
    assert dg == digest(want)
    assert t == world                           # the slowest rank's clock
    counts = np.bincount(route(np.arange(N_TOTAL), world), minlength=world)
    assert (n0, n1) == tuple(counts) and n0 and n1   # hash routing, both ranks hold documents


def test_route_matches_library():
    """shard.route (numpy) == mt_route_docs (libmtgpu host code; no GPU needed) and is balanced."""
    from fluidframework_amd.engine import _ptr, lib
    from fluidframework_amd.shard import route
    L = lib()
    L.mt_route_docs.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
    L.mt_route_docs.restype = ctypes.c_int
    L.mt_route_doc.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
    L.mt_route_doc.restype = ctypes.c_uint32
    ids = np.concatenate([np.arange(100_000, dtype=np.uint64),
                          np.array([2**63, 2**64 - 1, 123456789012345], dtype=np.uint64)])
    for n in (1, 2, 4, 8):
        out = np.zeros(len(ids), dtype=np.uint32)
        assert L.mt_route_docs(_ptr(ids), len(ids), n, _ptr(out)) == 0
        assert np.array_equal(out, route(ids, n))
        assert L.mt_route_doc(2**64 - 1, n) == route(np.array([2**64 - 1], np.uint64), n)[0]
        c = np.bincount(out[:100_000], minlength=n)
        assert c.max() - c.min() <= 8 * np.sqrt(100_000 / n)   # binomial spread, ~4 sigma each side


def test_file_rendezvous(tmp_path):
    from fluidframework_amd.shard import FileRendezvous
    a = FileRendezvous(key=f'test_{os.getpid()}', timeout=2)
    b = FileRendezvous(key=f'test_{os.getpid()}', timeout=2)
    a.publish(b'x' * 128)
    assert b.fetch(128) == b'x' * 128
    a.cleanup()
    with pytest.raises(TimeoutError):
        FileRendezvous(key=f'absent_{os.getpid()}', timeout=0.2).fetch(128)


def _bench(*args, timeout=600):
    out = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--no-cpu-baseline', '--steps', '1',
                          '--warmup', '1', '--docs', '600', '--ops', '160'] + list(args),
                         capture_output=True, text=True, timeout=timeout, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.strip().split('\n') if x.startswith('{')]
    assert len(lines) == 1, out.stdout
    return lines[0]


@pytest.mark.gpu
@pytest.mark.parametrize('config', ['C3', 'C4', 'C5'])
def test_bench_two_ranks_match_one(config, oracle_lib):
    """bench.py --gpus 2 (spawned ranks, hash-routed shards, gather) == bench.py on one GPU over
    the same 1,200-document universe, and == the oracle's digest of that universe (C3, C4: the
    config quoted at 1/2/4 GPUs)."""
    from fluidframework_amd import shard
    from fluidframework_amd.oplog import CONFIGS
    two = _bench('--config', config, '--gpus', '2', '--comm', 'gloo', '--devices', '0,0')
    one = _bench('--config', config, '--docs', '1200')
    assert two['n_gpus'] == 2 and one['n_gpus'] == 1
    assert two['config']['docs_total'] == one['config']['docs_total'] == 1200
    assert two['checksum_digest'] == one['checksum_digest']
    assert two['doc_errors_sampled'] == 0
    if config in ('C3', 'C4'):
        cfg = dict(CONFIGS[config])
        cfg.pop('n_docs')
        cfg['ops_per_doc'] = 160
        whole = oracle_lib.generate(1200, d0=0, seed=20261015, **cfg)
        want = oracle_lib.Oracle(1200).apply(whole, threads=8).checksums()
        assert one['checksum_digest'] == '%016x' % shard.digest(want)
