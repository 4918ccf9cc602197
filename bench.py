#!/usr/bin/env python3
"""Headline benchmark: sequenced merge-tree ops applied/sec on MI355X (BASELINE.json metric).

Workload (N=1): BASELINE.json config "100K docs x 32 clients with annotate property merges and
markRangeRemoved overlap, 1 MI355X" (C3 in SURVEY.md): 100,000 documents per GPU, 32 remote
clients, 1024 sequenced ops per document (45 % insert, 30 % remove -- half of them aimed to
overlap a concurrent remove -- 25 % annotate over 8 keys x 16 values, 5 % nulls, 2 % rewrite),
refSeq lag U[0, 32].  Synthetic, observer-driven, generated ON THE DEVICE into HBM before the
timed region (mt_synth.h; the same stream as the oracle's host generator, byte for byte).

A step = one full replay of every document's op log from empty documents, applied as launches of
`--ops-per-launch` (b = 32) ops per document (the serving tick of SURVEY.md §8d); the reset of
the documents (a one-kernel init) is inside the timed region.  Multi-GPU (torchrun): documents
are sharded across ranks (weak scaling, each rank its own 100K documents, global doc id = rank *
docs + i); no collective in the apply loop; RCCL gathers the per-document checksums at the end.

Prints ONE JSON line (rank 0).  `roofline` prices the apply kernels against HBM with the
algorithmic bytes they must move per launch (DESIGN.md "Roofline accounting"); `cpu_baseline`
replays a bounded sample of the same logs on the CPU oracle (oracle/mtcpu.cpp, a port of the
reference's observer path) on this host's cores, and the GPU's checksums for that sample are
checked against it (`parity`).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = 'sequenced merge-tree ops applied/sec (node) at 100K docs; % HBM roofline'
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# HBM bytes per launch from the rocprofv3 PMC passes (tools/rocprof_r01.sh -> tools/pmc_traffic.py)
PMC_TRAFFIC = os.path.join(HERE, 'profiles', 'r01_pmc_traffic.json')  # C3; other configs: _<config>.json


def pmc_path(config):
    return PMC_TRAFFIC if config == 'C3' else PMC_TRAFFIC.replace('.json', f'_{config}.json')


CONFIG_NAMES = {'C2': 'BASELINE.json configs[1]', 'C3': 'BASELINE.json configs[2]', 'C4': 'BASELINE.json configs[3]',
                'C5': 'BASELINE.json configs[4], per-GPU share of 1M docs'}


def pmc_traffic(kernel, config):
    """Measured HBM bytes per launch of `kernel` (2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected),
    from the committed PMC summary of the same bench command and config; None if not profiled."""
    try:
        with open(pmc_path(config)) as f:
            k = json.load(f)['kernels'].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    return int(k['hbm_bytes_per_launch']) if k else None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=3)
    p.add_argument('--warmup', type=int, default=1)
    p.add_argument('--config', default='C3')
    p.add_argument('--docs', type=int, default=0, help='documents per GPU (default: the config)')
    p.add_argument('--ops', type=int, default=0, help='ops per document (default: the config)')
    p.add_argument('--ops-per-launch', type=int, default=32)
    p.add_argument('--cpu-seconds', type=float, default=12.0, help='budget of the cpu_baseline sample')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--seed', type=int, default=20261015)
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    import torch
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import CONFIGS, DELI_CONFIGS
    from fluidframework_amd.shard import doc_id_base, gather_checksums, max_over_ranks

    cfg = dict(CONFIGS[args.config])
    n_docs = args.docs or cfg.pop('n_docs')
    cfg.pop('n_docs', None)
    if args.ops:
        cfg['ops_per_doc'] = args.ops
    ops_per_doc = cfg['ops_per_doc']

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    eng = MergeEngine(n_docs, device=local_rank, ops_per_launch=args.ops_per_launch)
    t0 = time.time()
    dev = eng.synthesize(doc_id_base=doc_id_base(rank, n_docs), seed=args.seed, **cfg)
    gen_s = time.time() - t0
    gen_cs = eng.checksums()
    n_ops = dev.n_ops

    deli = None
    if args.config in DELI_CONFIGS:
        # C5: the op records' seq / msn are re-derived by deli from the raw client messages inside
        # every step (deli_kernel stamps them into the staged records; the apply then reads them)
        from fluidframework_amd.deli import RAW_DTYPE, TICKET_DTYPE, DeliSequencer, batch_device_ptrs
        from fluidframework_amd.hipmem import DeviceBuffer
        d_ops, _, d_row = batch_device_ptrs(dev)
        deli = DeliSequencer(n_docs, device=local_rank)
        d_msgs = DeviceBuffer(n_ops * RAW_DTYPE.itemsize)
        d_tick = DeviceBuffer(n_ops * TICKET_DTYPE.itemsize)
        joined = {c: (0, 0, False) for c in range(1, cfg['n_clients'] + 1)}
        deli.raw_from_ops(d_ops, d_row, n_docs, d_msgs.ptr)
        deli.sync()
    deli_ms = 0.0

    def step():
        nonlocal deli_ms
        if deli is not None:
            deli.restore_all(seq=0, clients=joined)
            deli.ticket_device(d_msgs.ptr, d_row, n_docs, d_tick.ptr, d_ops)
            deli.sync()
            deli_ms += deli.last_ms()
        eng.reset()
        eng.apply_staged(dev)

    for _ in range(args.warmup):
        step()
    deli_ms = 0.0

    kern_ms = 0.0
    wall_ms = 0.0
    launches = 0
    alg_bytes = 0
    cls = {}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        k, w, nl, nb = eng.last_stats()
        kern_ms += k
        wall_ms += w
        launches += nl
        alg_bytes += nb
        for cap, ms, n, b in eng.last_class_stats():
            a = cls.setdefault(cap, [0.0, 0, 0])
            a[0] += ms
            a[1] += n
            a[2] += b
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, device='cuda')

    # the dominant kernel's roofline: one more (untimed) step with the classes serialized, so each
    # class kernel has the GPU to itself and its launch duration is its own (in the timed steps the
    # classes of a tick overlap on separate streams, which stretches every launch)
    rcls = cls
    if os.environ.get('MTGPU_SERIAL') != '1':
        eng.set_concurrent_classes(False)
        step()
        eng.set_concurrent_classes(True)
        rcls = {}
        for cap, ms, n, b in eng.last_class_stats():
            rcls[cap] = [ms, n, b]

    cs = eng.checksums()
    errs = sum(1 for d in range(0, n_docs, max(1, n_docs // 64)) if eng.error(d)[0])
    assert np.array_equal(cs, gen_cs), 'replay does not reproduce the generation state'
    if deli is not None:
        t = d_tick.download(TICKET_DTYPE)
        assert np.all(t['status'] == 1), 'deli nacked or dropped a message of the synthetic stream'

    # final per-document checksum gather to rank 0 over RCCL (the only collective)
    _, digest = gather_checksums(cs, dist, device='cuda')

    total_ops = n_ops * world * args.steps
    value = total_ops / elapsed
    # the dominant kernel = the capacity class with the most device time (one kernel symbol)
    dom = max(rcls, key=lambda c: rcls[c][0])
    d_ms, d_n, d_b = rcls[dom]
    avg_launch_ms = d_ms / max(1, d_n)
    bytes_per_launch = d_b / max(1, d_n)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if d_n else 0.0
    all_achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms else 0.0

    cpu = None
    parity = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(eng, dev, cs, n_docs, args.cpu_seconds)

    if rank == 0:
        line = {
            'metric': METRIC,
            'value': round(value, 1),
            'unit': 'ops/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(elapsed / args.steps * 1e3, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'int32',
            'data': 'synthetic (device-generated observer-driven op logs, mt_synth.h)',
            'config': {
                'workload': f'{args.config}: {n_docs} docs/GPU x {cfg["n_clients"]} clients x {ops_per_doc} '
                            f'sequenced ops/doc ({CONFIG_NAMES.get(args.config, args.config)}), '
                            + ('deli seq/msn ticketing + ' if deli is not None else '')
                            + 'full merge-tree apply incl. zamboni',
                'docs_per_gpu': n_docs, 'ops_per_doc': ops_per_doc, 'ops_per_launch': args.ops_per_launch,
                'ops_per_step': n_ops * world, 'parallelism': f'doc-sharded x{world} (no collective in apply)',
            },
            'roofline': {
                'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': pmc_traffic(eng.class_kernel(dom), args.config),
                'traffic_source': os.path.relpath(pmc_path(args.config), HERE) + ' (bytes per launch)',
                'kernel': eng.class_kernel(dom), 'launches': d_n,
                'measured_in': 'an extra untimed step with the capacity classes serialized'
                               if rcls is not cls else 'the timed steps (classes serialized)',
                'avg_launch_ms': round(avg_launch_ms, 4), 'alg_bytes_per_launch': int(bytes_per_launch),
                'all_apply_kernels': {'launches': launches, 'kernel_ms': round(kern_ms, 2),
                                      'achieved_GBps': round(all_achieved, 1),
                                      'apply_wall_ms': round(wall_ms, 2),
                                      'achieved_GBps_wall': round(alg_bytes / (wall_ms * 1e-3) / 1e9, 1) if wall_ms else None,
                                      'classes_concurrent': os.environ.get('MTGPU_SERIAL') != '1',
                                      'kernel_share_of_step': round(kern_ms / (elapsed * 1e3), 3)},
            },
            'deli': None if deli is None else {
                'kernel_ms_per_step': round(deli_ms / args.steps, 3),
                'tickets_per_s_kernel': round(n_ops / (deli_ms / args.steps * 1e-3), 1) if deli_ms else None,
                'share_of_step': round(deli_ms / (elapsed * 1e3), 4)},
            'cpu_baseline': cpu,
            'parity': parity,
            'doc_errors_sampled': errs,
            'checksum_digest': '%016x' % digest,
            'gen_seconds': round(gen_s, 2),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(eng, dev, gpu_cs, n_docs, budget_s):
    """Replay a bounded sample of the same op logs on the CPU oracle (port of the reference's
    observer path) with this host's cores; check the GPU checksums of the sample."""
    from oracle import oracle
    oracle.build()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count()
    threads = max(1, min(16, cores))
    chunk = 1024
    done_docs, ops, secs, mism = 0, 0, 0.0, 0
    d0 = 0
    while d0 < n_docs and secs < budget_s:
        d1 = min(n_docs, d0 + chunk)
        hb = dev.to_host(d0, d1)
        o = oracle.Oracle(d1 - d0)
        t = time.perf_counter()
        o.apply(hb, threads=threads)
        secs += time.perf_counter() - t
        mism += int(np.count_nonzero(o.checksums() != gpu_cs[d0:d1]))
        done_docs += d1 - d0
        ops += hb.n_ops
        d0 = d1
    cpu = {'value': round(ops / secs, 1), 'unit': 'ops/s', 'cores': threads, 'kind': 'port',
           'sample': f'docs [0, {done_docs}) of the same device-generated logs ({ops} ops, {secs:.1f} s), '
                     f'oracle/mtcpu.cpp observer replay, {threads} threads'}
    parity = {'docs_checked': done_docs, 'mismatches': mism, 'against': 'oracle/mtcpu.cpp'}
    return cpu, parity


if __name__ == '__main__':
    main()
