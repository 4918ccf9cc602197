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
the documents (a one-kernel init) is inside the timed region.  `--config C5`: each document's raw
client stream -- the ClientJoin of its 8 clients, then its op messages -- is ticketed by the deli
kernel (seq / msn assigned and stamped into the op records) inside every step, then applied.

Multi-GPU (`--gpus N`, or launched by torchrun): one process per GPU; this script spawns the N
ranks itself when started without WORLD_SIZE.  Documents are hash-routed (splitmix64(docId) mod
N, the reference's documentId-keyed partitioning) from a universe of N x docs-per-GPU documents:
weak scaling.  No collective in the apply loop; RCCL (libmtgpu mt_comm, over xGMI) gathers the
per-document checksums to rank 0 at the end and provides the barrier and max-over-ranks clock.
No process imports torch: libmtgpu's HIP runtime is the only one.

Prints ONE JSON line (rank 0).  `roofline` prices the dominant apply kernel against HBM with the
algorithmic bytes it must move per launch (DESIGN.md "Roofline accounting"); `cpu_baseline`
replays a bounded sample of the same logs on the CPU oracle (oracle/mtcpu.cpp, a port of the
reference's observer path) with every host core, and the GPU's checksums for that sample are
checked against it (`parity`).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time
import uuid

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = 'sequenced merge-tree ops applied/sec (node) at 100K docs; % HBM roofline'
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# HBM bytes per launch from the rocprofv3 PMC passes (tools/rocprof.sh -> tools/pmc_traffic.py)
PROFILES = os.path.join(HERE, 'profiles')
PMC_ROUND = 'r06'
SQ_ROUND = 'r06'   # profiles/<round>_sq_counters_C3_pass{1,2}.txt (tools/sq_pass.sh): the issue roofline
# instruction issue peaks (MI355X_MICROARCH.md "Wave scheduling"): 256 CUs x 4 SIMDs, a wave64 VALU
# instruction every 2 cycles per SIMD at 2.4 GHz; one scalar (SALU) instruction per CU per cycle
VALU_PEAK = 1024 * 2.4e9 / 2
SALU_PEAK = 256 * 2.4e9
CAL_ROUND = 'r04'  # profiles/<round>_js_calibration_<config>.json: r of the JS baseline (oracle/tsref/calibrate.py)

CONFIG_NAMES = {'C2': 'BASELINE.json configs[1]', 'C3': 'BASELINE.json configs[2]', 'C4': 'BASELINE.json configs[3]',
                'C5': 'BASELINE.json configs[4], per-GPU share of 1M docs',
                'C3W': 'BASELINE.json configs[2] with 48 clients'}


def pmc_path(config):
    return os.path.join(PROFILES, f'{PMC_ROUND}_pmc_traffic_{config}.json')


def pmc_traffic(kernel, config):
    """Measured HBM bytes per launch of `kernel` (2 x FETCH_SIZE + WRITE_SIZE, gfx950-corrected),
    from the committed PMC summary of the same bench command and config; None if not profiled."""
    try:
        with open(pmc_path(config)) as f:
            ks = json.load(f)['kernels']
    except (OSError, ValueError, KeyError):
        return None
    k = ks.get(kernel)
    if k is None and kernel.endswith('>'):
        # the engine names a kernel without its defaulted template arguments; the trace spells them
        # out ("mt::apply_kernel_g<1024, true>" -> "mt::apply_kernel_g<1024, true, false, 1>")
        hit = [v for n, v in ks.items() if n.startswith(kernel[:-1] + ', ')]
        k = hit[0] if len(hit) == 1 else None
    return int(k['hbm_bytes_per_launch']) if k else None


def mangled_stem(kernel):
    """'mtr::reg_apply_kernel<9>' -> '3mtr16reg_apply_kernelILi9E' (the Itanium-mangled prefix rocprof prints)."""
    ns, _, rest = kernel.partition('::')
    name, _, targ = rest.partition('<')
    k = targ.split(',')[0].strip(' >')
    return f'{len(ns)}{ns}{len(name)}{name}ILi{k}E'


def sq_counters(kernel, config='C3'):
    """Per-dispatch SQ counters of `kernel` from the committed SQ passes (both files merged), or None."""
    stem, got = mangled_stem(kernel), {}
    for pss in (1, 2):
        path = os.path.join(PROFILES, f'{SQ_ROUND}_sq_counters_{config}_pass{pss}.txt')
        try:
            lines = open(path).read().split('\n')
        except OSError:
            return None
        cur = None
        for ln in lines:
            if ln and not ln.startswith(' '):
                cur = ln.split(',')[0]
            elif cur and stem in cur and 'per dispatch' in ln:
                f = ln.split()
                got[f[0]] = float(f[-1])
    return got or None


def issue_roofline(kernel, ops_per_launch, avg_launch_ms, config='C3'):
    """The dominant kernel against the instruction-issue peaks: VALU / SALU / LDS instructions per op
    from the committed SQ passes of the same kernel (per dispatch / (waves x ops per wave), each wave
    applying ops_per_launch ops), times its ops/s in this run (ops per launch / the live launch time)."""
    c = sq_counters(kernel, config)
    if not c or not c.get('SQ_WAVES') or not avg_launch_ms:
        return None
    ops = c['SQ_WAVES'] * ops_per_launch
    valu, salu = c.get('SQ_INSTS_VALU', 0) / ops, c.get('SQ_INSTS_SALU', 0) / ops
    ops_s = ops / (avg_launch_ms * 1e-3)
    return {'bound': 'issue', 'valu_per_op': round(valu, 1), 'salu_per_op': round(salu, 1),
            'lds_per_op': round(c.get('SQ_INSTS_LDS', 0) / ops, 1),
            'valu_frac': round(valu * ops_s / VALU_PEAK, 4), 'salu_frac': round(salu * ops_s / SALU_PEAK, 4),
            'wait_frac': round(c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES'], 4)
            if c.get('SQ_WAIT_ANY') and c.get('SQ_WAVE_CYCLES') else None,
            'peaks': {'valu_instr_per_s': VALU_PEAK, 'salu_instr_per_s': SALU_PEAK},
            'source': f'profiles/{SQ_ROUND}_sq_counters_{config}_pass{{1,2}}.txt (per dispatch / SQ_WAVES x '
                      f'{ops_per_launch} ops); ops/s = ops per launch / avg_launch_ms of this run'}


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
    p.add_argument('--comm', choices=['auto', 'rccl', 'gloo'], default='auto',
                   help='rank exchange: RCCL over xGMI (default for N > 1; "rccl" also at N = 1, a one-rank '
                        'communicator), or gloo (ranks sharing one GPU, tests)')
    p.add_argument('--devices', default='', help='device of each local rank, e.g. "0,0" (default: rank i -> GPU i)')
    p.add_argument('--hbm-only', action='store_true',
                   help='tooling (A/Bs, profiles): skip the host-fed steps; value is then the HBM-resident figure')
    p.add_argument('--no-tickets', action='store_true', help='C5: the host-fed steps do not copy the tickets back')
    p.add_argument('--first-tick', type=int, default=0,
                   help='a ramp of short first ticks in the host-fed feed (mt_log_to_ticks_ramp: tick t holds '
                        'min(b, N << t) ops per document; 0: none -- the ramp measured slower on C3 and C5, '
                        'profiles/r06_ab/ab9_*)')
    p.add_argument('--no-slow-paths', action='store_true',
                   help='skip the N=1 side lines for the paths off the narrow register engine (C3 with delta '
                        'events recorded, C3 with 48 clients, the editing-client farm at 100K documents)')
    return p.parse_args()


def free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn(n):
    """--gpus N without a launcher: start N rank processes (this script), one per GPU, before
    anything here touches a GPU; exit with the first failing rank's status."""
    env = dict(os.environ, WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(free_port()),
               MTGPU_RUN_ID=uuid.uuid4().hex)
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e))
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c), 0)


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn(args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    devices = [int(x) for x in args.devices.split(',')] if args.devices else None
    device = devices[local_rank] if devices else local_rank

    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.hipmem import device_synchronize
    from fluidframework_amd.oplog import CONFIGS, DELI_CONFIGS
    from fluidframework_amd import shard
    from fluidframework_amd.ticks import TickLog

    if world == 1 and args.comm != 'rccl':
        comm = shard.LocalComm()
    elif args.comm == 'gloo':
        import torch.distributed as tdist
        tdist.init_process_group('gloo', rank=rank, world_size=world)
        comm = shard.GlooComm(tdist)
    else:
        comm = shard.RcclComm(rank, world, device)

    cfg = dict(CONFIGS[args.config])
    docs_per_gpu = args.docs or cfg.pop('n_docs')
    cfg.pop('n_docs', None)
    if args.ops:
        cfg['ops_per_doc'] = args.ops
    ops_per_doc = cfg['ops_per_doc']
    n_total = docs_per_gpu * world
    # this rank's documents: global ids routed here (world 1: all of them, in order)
    ids = shard.shard_ids(rank, world, n_total) if world > 1 else np.arange(n_total, dtype=np.uint32)
    n_docs = len(ids)
    max_docs = int(comm.max(float(n_docs)))

    def barrier():
        device_synchronize()
        comm.barrier()

    eng = MergeEngine(n_docs, device=device, ops_per_launch=args.ops_per_launch)
    t0 = time.time()
    dev = eng.synthesize(doc_ids=ids if world > 1 else None, seed=args.seed, **cfg)
    gen_s = time.time() - t0
    gen_cs = eng.checksums()
    n_ops = dev.n_ops

    deli = None
    if args.config in DELI_CONFIGS:
        # C5: every document starts new at the deli (no clients); its raw stream = the ClientJoin
        # of its n_clients clients + its op messages (refSeq past the joins).  Inside every step
        # deli tickets the whole stream and stamps seq / msn / refSeq into the staged op records,
        # which the apply then reads: the joins revs the sequence numbers (lambda.ts:286-299).
        from fluidframework_amd.deli import RAW_DTYPE, TICKET_DTYPE, DeliSequencer, batch_device_ptrs
        from fluidframework_amd.hipmem import DeviceBuffer
        n_join = cfg['n_clients']
        d_ops, _, d_row = batch_device_ptrs(dev)
        deli = DeliSequencer(n_docs, device=device)
        n_msgs = n_ops + n_docs * n_join
        d_msgs = DeviceBuffer(n_msgs * RAW_DTYPE.itemsize)
        d_mrow = DeviceBuffer((n_docs + 1) * 4)
        d_tick = DeviceBuffer(n_msgs * TICKET_DTYPE.itemsize)
        deli.raw_stream(d_ops, d_row, n_docs, n_join, d_msgs.ptr, d_mrow.ptr)
        deli.sync()
    deli_ms = 0.0

    # SURVEY.md §8(d) times the apply "from the first H2D of the op batch": the job's op log (and for
    # C5 its raw client messages) starts in page-locked host memory, laid out tick-major -- the next
    # b ops of every document per tick, what a serving node receives -- and mt_submit_ticks copies
    # tick k + 1 on a copy stream while tick k applies.  Laying the log out is log generation (not
    # timed); the upload, deli and the apply are.
    # (--first-tick: a ramp of short first ticks, so the apply starts after a short copy)
    first_tick = max(1, min(args.first_tick, args.ops_per_launch)) if args.first_tick > 0 else None
    t0 = time.time()
    host = dev.to_host() if not args.hbm_only else None
    if args.hbm_only:
        log = None
    elif deli is None:
        log = TickLog.from_batch(host, args.ops_per_launch, first=first_tick)
    else:
        log = TickLog.from_batch(host, args.ops_per_launch, first=first_tick, msgs=d_msgs.download(RAW_DTYPE, n_msgs),
                                 msg_row_ptr=d_mrow.download(np.uint32, n_docs + 1), tickets=not args.no_tickets)
    del host
    layout_s = time.time() - t0

    def step():
        eng.reset()
        if deli is not None:
            deli.restore_all(seq=0, clients={})   # new documents (lambda.ts:124-167)
        eng.apply_ticks(log, deli=deli)

    def step_hbm():
        # the same job with its op log already resident in HBM (generated there): reset + apply
        nonlocal deli_ms
        if deli is not None:
            deli.restore_all(seq=0, clients={})
            deli.ticket_device(d_msgs.ptr, d_mrow.ptr, n_docs, d_tick.ptr, d_ops, n_ops)
            deli.sync()
            deli_ms += deli.last_ms()
        eng.reset()
        eng.apply_staged(dev)

    def timed(fn):
        kern_ms = wall_ms = 0.0
        launches = alg_bytes = 0
        cls = {}
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
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
        return comm.max(time.perf_counter() - t0), kern_ms, wall_ms, launches, alg_bytes, cls

    main_step = step_hbm if args.hbm_only else step
    for _ in range(args.warmup):
        main_step()
    ref_cs = eng.checksums() if deli is not None and args.warmup else None
    deli_ms = 0.0
    elapsed, kern_ms, wall_ms, launches, alg_bytes, cls = timed(main_step)
    cs_fed = eng.checksums()
    tk_ok = bool(np.all(log.tickets['status'] == 1)) if log is not None and log.tickets is not None else None

    # the HBM-resident figure (side field): the same steps with the log generated in HBM
    if args.hbm_only:
        elapsed_hbm = elapsed
    else:
        step_hbm()
        deli_ms = 0.0
        elapsed_hbm = timed(step_hbm)[0]

    # the dominant kernel's roofline: one more (untimed) step with the classes serialized, so each
    # class kernel has the GPU to itself and its launch duration is its own (in the timed steps the
    # classes of a tick overlap on separate streams, which stretches every launch)
    rcls = cls
    if os.environ.get('MTGPU_SERIAL') != '1':
        eng.set_concurrent_classes(False)
        step_hbm()
        eng.set_concurrent_classes(True)
        rcls = {cap: [ms, n, b] for cap, ms, n, b in eng.last_class_stats()}

    cs = eng.checksums()
    errs = sum(1 for d in range(0, n_docs, max(1, n_docs // 64)) if eng.error(d)[0])
    # SURVEY.md §8(d)'s b = infinity figure (the minimal traffic of the job): every op record and its
    # payload read once, each document's state read once (empty after the reset: its 80-byte scalar
    # header) and written once (35 B per final segment + the header)
    if log is not None:
        pay_b = float(log.tick_payload[-1])
    else:  # the mean payload per op from the first 512 documents' logs
        samp = dev.to_host(0, min(n_docs, 512))
        pay_b = float(samp.ops['payload_len'].astype(np.float64).sum()) * n_ops / max(1, samp.n_ops)
        del samp
    ops_b = n_ops * 32 + pay_b
    min_bytes = ops_b + 35.0 * float(eng.seg_counts().astype(np.float64).sum()) + 2 * 80.0 * n_docs
    assert np.array_equal(cs_fed, cs), 'the host-fed tick steps differ from the HBM-resident replay'
    if deli is None:
        assert np.array_equal(cs, gen_cs), 'replay does not reproduce the generation state'
    else:
        if ref_cs is not None:
            assert np.array_equal(cs, ref_cs), 'deli + apply is not deterministic across steps'
        t = d_tick.download(TICKET_DTYPE)
        assert np.all(t['status'] == 1), 'deli nacked or dropped a message of the synthetic stream'
        assert tk_ok is not False, 'a ticket of the host-fed steps is not SENT'
    upload = None if log is None else {
              'bytes_per_step': log.upload_bytes(), 'ticks': log.n_ticks, 'first_tick_ops_per_doc': first_tick or args.ops_per_launch,
              'layout_s': round(layout_s, 2),
              'note': 'page-locked host memory, tick-major (mt_log_to_ticks), payload compacted per tick; '
                      'copied on a copy stream into a ring of 3 device slots while the previous tick applies'
                      + ('; tickets copied back per tick' if deli is not None and not args.no_tickets else '')}
    if log is not None:
        log.free()

    # final per-document checksum gather to rank 0 (RCCL ncclGather from HBM; the only collective)
    parts = comm.gather_checksums(eng, max_docs)
    digest = None
    if rank == 0:
        all_ids = [shard.shard_ids(r, world, n_total) for r in range(world)] if world > 1 else [ids]
        allcs = shard.assemble(parts, all_ids)
        digest = shard.digest(allcs)

    total_ops = n_total * ops_per_doc * args.steps
    value = total_ops / elapsed
    dom = max(rcls, key=lambda c: rcls[c][0])  # the capacity class with the most device time
    d_ms, d_n, d_b = rcls[dom]
    avg_launch_ms = d_ms / max(1, d_n)
    bytes_per_launch = d_b / max(1, d_n)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if d_n else 0.0
    all_achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms else 0.0

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(dev, cs, n_docs, args.cpu_seconds, args.config)

    kname_of = {c: eng.class_kernel(c) for c in rcls}
    slow = None
    if world == 1 and args.config == 'C3' and not args.no_slow_paths and not args.docs and not args.ops:
        # the main engine's HBM goes back before the side lines allocate theirs
        kname_main = eng.class_kernel(max(rcls, key=lambda c: rcls[c][0]))
        dev.free()
        eng.close()
        slow = slow_paths(device, docs_per_gpu, args.seed)

    if rank == 0:
        kname = kname_main if slow is not None else eng.class_kernel(dom)
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
            'data': 'synthetic (device-generated observer-driven op logs, mt_synth.h), ' + (
                'HBM-resident (--hbm-only tooling run)' if args.hbm_only else
                'fed from page-locked host memory tick by tick inside the timed region (SURVEY.md 8(d): from the '
                'first H2D)'),
            'config': {
                'workload': f'{args.config}: {docs_per_gpu} docs/GPU x {cfg["n_clients"]} clients x {ops_per_doc} '
                            f'sequenced ops/doc ({CONFIG_NAMES.get(args.config, args.config)}), '
                            + ('deli seq/msn ticketing of the raw streams (joins + ops) + ' if deli is not None else '')
                            + 'full merge-tree apply incl. zamboni',
                'docs_total': n_total, 'docs_per_gpu': docs_per_gpu, 'docs_rank0': n_docs,
                'ops_per_doc': ops_per_doc, 'ops_per_launch': args.ops_per_launch,
                'ops_per_step': n_total * ops_per_doc,
                'parallelism': f'hash-routed docs x{world} (splitmix64(docId) mod {world}; no collective in apply)',
                'comm': type(comm).__name__,
            },
            'roofline': {
                'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': pmc_traffic(kname, args.config),
                'traffic_source': os.path.relpath(pmc_path(args.config), HERE) + ' (bytes per launch)',
                'kernel': kname, 'launches': d_n,
                'measured_in': 'an extra untimed step with the capacity classes serialized'
                               if rcls is not cls else 'the timed steps (classes serialized)',
                'avg_launch_ms': round(avg_launch_ms, 4), 'alg_bytes_per_launch': int(bytes_per_launch),
                'class_ms_serialized': {class_label(c): round(v[0], 2) for c, v in sorted(rcls.items()) if v[1]},
                'classes': class_table(rcls, args.config, kname_of),
                'issue': issue_roofline(kname, args.ops_per_launch, avg_launch_ms, args.config),
                'b_infinity': {'bytes_per_step_rank0': int(min_bytes),
                               'frac': round(min_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 5),
                               'note': 'SURVEY.md 8(d): state read + written once per step, every op once; '
                                       'the step time of the timed steps'},
                'all_apply_kernels': {'launches': launches, 'kernel_ms': round(kern_ms, 2),
                                      'achieved_GBps': round(all_achieved, 1),
                                      'apply_wall_ms': round(wall_ms, 2),
                                      'achieved_GBps_wall': round(alg_bytes / (wall_ms * 1e-3) / 1e9, 1) if wall_ms else None,
                                      'classes_concurrent': os.environ.get('MTGPU_SERIAL') != '1',
                                      'kernel_share_of_step': round(kern_ms / (elapsed * 1e3), 3)},
            },
            'deli': None if deli is None else {
                'messages_per_step': n_msgs, 'joins_per_doc': n_join,
                'kernel_ms_per_step': round(deli_ms / args.steps, 3),
                'tickets_per_s_kernel': round(n_msgs / (deli_ms / args.steps * 1e-3), 1) if deli_ms else None,
                'share_of_step': round(deli_ms / (elapsed_hbm * 1e3), 4),
                'note': 'kernel time from the HBM-resident steps (in the host-fed steps deli runs per tick on the '
                        'engine stream)'},
            'value_hbm_resident': {'value': round(total_ops / elapsed_hbm, 1), 'unit': 'ops/s',
                                   'ms_per_step': round(elapsed_hbm / args.steps * 1e3, 3),
                                   'note': 'the same steps with the op log already resident in HBM (generated '
                                           'there): reset + apply' + (' (+ deli ticketing)' if deli is not None else '')},
            'upload': upload,
            'slow_paths': slow,
            'cpu_baseline': cpu,
            'parity': parity,
            'doc_errors_sampled': errs,
            'checksum_digest': '%016x' % digest,
            'gen_seconds': round(gen_s, 2),
        }
        print(json.dumps(line), flush=True)
    comm.close()


MT_CLASS_EDITING = 0x40000000  # include/mtgpu.h: the editing documents' bucket in the class stats
MT_CLASS_LDS = 0x20000000      # the LDS engine inside a register class (declared label keys)
MT_CLASS_C64 = 0x10000000      # the register engine's C64 form (client ids 33..63)
MT_CLASS_WIDE = 0x04000000     # the wide form (u16 ids, UTF-16, keys 8..15)
MT_CLASS_GROUPS = 0x08000000   # with MT_CLASS_EDITING: the form for more than 64 pending edits


def class_label(cap):
    if cap & MT_CLASS_EDITING:
        if cap & MT_CLASS_GROUPS:
            return f'editing_groups{cap & ~(MT_CLASS_EDITING | MT_CLASS_GROUPS)}'
        return f'editing{cap & ~MT_CLASS_EDITING}'
    if cap & MT_CLASS_LDS:
        return f'lds{cap & ~MT_CLASS_LDS}'
    if cap & MT_CLASS_C64:
        return f'c64_{cap & ~MT_CLASS_C64}'
    if cap & MT_CLASS_WIDE:
        return f'wide{cap & ~MT_CLASS_WIDE}'
    return str(cap)


def class_table(rcls, config, kname_of):
    """Per capacity class of the serialized step: its kernel, device time, launches, algorithmic bytes
    per launch and -- from the committed PMC passes of the same config -- the HBM bytes it actually
    moved per launch and their ratio (every class's traffic ratio visible)."""
    out = {}
    tot = sum(v[0] for v in rcls.values()) or 1.0
    for c, (ms, n, b) in sorted(rcls.items()):
        if not n:
            continue
        k = kname_of[c]
        alg = b / n
        pmc = pmc_traffic(k, config)
        out[class_label(c)] = {'kernel': k, 'ms': round(ms, 2), 'share': round(ms / tot, 3), 'launches': n,
                               'avg_launch_ms': round(ms / n, 4), 'alg_bytes_per_launch': int(alg),
                               'pmc_bytes_per_launch': pmc,
                               'pmc_over_alg': round(pmc / alg, 2) if pmc and alg else None}
    return out


def roofline_of(eng, rcls):
    """The dominant kernel of one serialized step: its average launch time and algorithmic bytes
    per launch against the HBM peak (the main line's accounting)."""
    dom = max(rcls, key=lambda c: rcls[c][0])
    ms, n, b = rcls[dom]
    avg = ms / max(1, n)
    per = b / max(1, n)
    ach = per / (avg * 1e-3) / 1e9 if n and avg else 0.0
    return {'bound': 'hbm', 'achieved': round(ach, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(ach / HBM_PEAK_GBS, 4), 'traffic': pmc_traffic(eng.class_kernel(dom), 'C3'),
            'traffic_source': os.path.relpath(pmc_path('C3'), HERE) + ' (the PMC passes of the full C3 bench, side lines '
                              'included; bytes per launch)', 'kernel': eng.class_kernel(dom), 'launches': n,
            'avg_launch_ms': round(avg, 4), 'alg_bytes_per_launch': int(per),
            'class_ms_serialized': {class_label(c): round(v[0], 2) for c, v in sorted(rcls.items()) if v[1]}}


def timed_side_step(eng, dbatch, warmup=1, after=None):
    """Warm-up, one timed replay (reset + apply of the HBM-resident batch), then one serialized
    replay for the dominant kernel's roofline; `after(timed)` runs after every replay (the events
    line drains there, timing the drain of the timed replay).  Returns (seconds, roofline, the
    timed replay's after() result)."""
    from fluidframework_amd.hipmem import device_synchronize
    for _ in range(warmup):
        eng.reset()
        eng.apply_staged(dbatch)
        if after:
            after(False)
    device_synchronize()
    t0 = time.perf_counter()
    eng.reset()
    eng.apply_staged(dbatch)
    device_synchronize()
    el = time.perf_counter() - t0
    res = after(True) if after else None
    eng.set_concurrent_classes(False)
    eng.reset()
    eng.apply_staged(dbatch)
    eng.set_concurrent_classes(True)
    rcls = {cap: [ms, n, b] for cap, ms, n, b in eng.last_class_stats()}
    if after:
        after(False)
    return el, roofline_of(eng, rcls), res


def widen_payloads(batch):
    """Every record of `batch` in the wide form (include/mtgpu.h MT_OP_WIDE): its text as UTF-16 code
    units -- "a" as U+4E2D, so the documents hold non-Latin-1 text -- and (key u8, value u16) pairs."""
    from fluidframework_amd.oplog import OpBatch
    ops, pay = batch.ops.copy(), batch.payload
    npairs = (((ops['flags'].astype(np.int64) >> 3) & 0xF) | np.where(ops['type'] & 0x40, 16, 0) |
              np.where(ops['type'] & 0x20, 32, 0))
    tl = ops['payload_len'].astype(np.int64) - 2 * npairs
    new_len = 2 * tl + 3 * npairs
    new_off = np.concatenate([[0], np.cumsum(new_len)[:-1]]).astype(np.int64)
    out = np.zeros(int(new_len.sum()), dtype=np.uint8)
    src_off = ops['payload_off'].astype(np.int64)

    def ranks(counts):  # 0..c-1 for every op, concatenated
        return np.arange(int(counts.sum())) - np.repeat(np.cumsum(counts) - counts, counts)
    k = ranks(tl)
    b = pay[np.repeat(src_off, tl) + k]
    d = np.repeat(new_off, tl) + 2 * k
    cjk = b == ord('a')
    out[d] = np.where(cjk, 0x2D, b)
    out[d + 1] = np.where(cjk, 0x4E, 0)
    q = ranks(npairs)
    s0 = np.repeat(src_off + tl, npairs) + 2 * q
    d0 = np.repeat(new_off + 2 * tl, npairs) + 3 * q
    out[d0] = pay[s0]
    out[d0 + 1] = pay[s0 + 1]
    ops['type'] = ops['type'] | 0x80
    ops['payload_off'] = new_off.astype(np.uint32)
    ops['payload_len'] = new_len.astype(np.uint32)
    return OpBatch(ops, out, batch.row_ptr)


def slow_paths(device, n_docs, seed):
    """N = 1 side lines for the paths off the register engine's narrow form: C3 with
    the delta callbacks recorded (any SharedString with a sequenceDelta listener: the register
    engine's event-recording kernels, reg_apply_kernel_ev), C3
    with 48 clients (overlap sets past 32 bits: the register engine's C64 form), and the
    editing-client farm (local edits + remote ops + acks: the LDS engine's editing form) tiled over
    100K documents.  Each is a full replay of HBM-resident logs, checked against the generation
    state or the oracle."""
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import CONFIGS, OpBatch
    out = {}
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    ops = n_docs * cfg['ops_per_doc']

    # C3 with delta events: every callback recorded on the device; the drain (one CSR gather + D2H
    # of every record) is timed on its own
    eng = MergeEngine(n_docs, device=device, ops_per_launch=32)
    eng.enable_events(per_doc=8192)  # a C3 document fires <= ~6.5 K callbacks per replay
    dev = eng.synthesize(seed=seed, **cfg)
    gen_cs = eng.checksums()
    eng.drain_event_rows()

    def drain(timed):
        t0 = time.perf_counter()
        rows, rp = eng.drain_event_rows()
        return (time.perf_counter() - t0, int(rp[-1])) if timed else None
    el, rf, (drain_s, n_ev) = timed_side_step(eng, dev, after=drain)
    ok = bool(np.array_equal(eng.checksums(), gen_cs))
    errs = sum(1 for d in range(0, n_docs, max(1, n_docs // 256)) if eng.error(d)[0])
    out['C3_events'] = {'workload': f'C3 ({n_docs} docs x 32 clients x 1024 ops) with every delta callback recorded '
                                    '(mt_events_enable; register engine, reg_apply_kernel_ev)',
                        'value': round(ops / el, 1), 'unit': 'ops/s', 'ms_per_step': round(el * 1e3, 2),
                        'events_per_step': n_ev, 'drain_s': round(drain_s, 3),
                        'note': 'the drain (CSR gather of every callback record + D2H) follows the timed replay',
                        'roofline': rf, 'parity': {'replay_equals_generation': ok, 'doc_errors_sampled': errs}}
    dev.free()
    eng.close()

    # C3 with 48 clients: client ids past 32 (the register engine's overlap set) -> its C64 form
    cfg48 = dict(CONFIGS['C3W'])
    cfg48.pop('n_docs')
    eng = MergeEngine(n_docs, device=device, ops_per_launch=32)
    dev = eng.synthesize(seed=seed, **cfg48)
    gen_cs = eng.checksums()
    el, rf, _ = timed_side_step(eng, dev)
    cs = eng.checksums()
    par = {'replay_equals_generation': bool(np.array_equal(cs, gen_cs))}
    try:
        from oracle import oracle
        k = 256
        o = oracle.Oracle(k).apply(dev.to_host(0, k), threads=int(os.environ.get('OMP_NUM_THREADS') or 8))
        par.update(docs_checked=k, mismatches=int(np.count_nonzero(o.checksums() != cs[:k])), against='oracle/mtcpu.cpp')
    except Exception as ex:  # the checker is optional on a box without a compiler
        par['oracle'] = f'unavailable: {ex}'
    out['C3_48_clients'] = {'workload': f'C3 with 48 clients ({n_docs} docs x 1024 ops; the register engine\'s C64 '
                                        'form: 64-bit overlap sets)',
                            'value': round(ops / el, 1), 'unit': 'ops/s', 'ms_per_step': round(el * 1e3, 2),
                            'roofline': rf, 'parity': par}
    dev.free()
    eng.close()

    # C3 with client ids past 255: the wide form (u16 short ids, UTF-16 arena, structure in an HBM
    # workspace; include/mtgpu.h "limits").  The device generator keeps ids below 64, so the C3 logs
    # of n_docs / 5 documents are generated, copied out, every client id shifted by 300 and staged
    # again: the same edits by clients 301..332
    n_w = max(1, n_docs // 5)
    eng = MergeEngine(n_w, device=device, ops_per_launch=32)
    dev = eng.synthesize(seed=seed, **cfg)
    host = dev.to_host(0, n_w)
    dev.free()
    eng.close()
    host.ops['client'] = np.where(host.ops['client'] > 0, host.ops['client'] + 300, 0).astype(host.ops['client'].dtype)
    host = widen_payloads(host)
    eng = MergeEngine(n_w, device=device, ops_per_launch=32)
    dev = eng.stage(host)
    el, rf, _ = timed_side_step(eng, dev)
    cs = eng.checksums()
    par = {'doc_errors_sampled': sum(1 for d in range(0, n_w, max(1, n_w // 256)) if eng.error(d)[0])}
    try:
        from oracle import oracle
        k = 256
        sub = dev.to_host(0, k)
        o = oracle.Oracle(k).apply(sub, threads=int(os.environ.get('OMP_NUM_THREADS') or 8))
        par.update(docs_checked=k, mismatches=int(np.count_nonzero(o.checksums() != cs[:k])), against='oracle/mtcpu.cpp')
    except Exception as ex:
        par['oracle'] = f'unavailable: {ex}'
    wops = n_w * cfg['ops_per_doc']
    out['C3_wide_ids'] = {'workload': f'C3 with client ids 301..332 and UTF-16 text ({n_w} docs x 1024 ops, every '
                                      'record wide, "a" as U+4E2D; the wide form: u16 short ids, UTF-16 arena, '
                                      'HBM workspace)',
                          'value': round(wops / el, 1), 'unit': 'ops/s', 'ms_per_step': round(el * 1e3, 2),
                          'roofline': rf, 'parity': par}
    dev.free()
    eng.close()
    del host

    # the editing-client farm (tests/golden/local_big: reference clients' logs as one of them sees
    # them) tiled over n_docs documents
    src = OpBatch.load(os.path.join(HERE, 'tests', 'golden', 'local_big.mtlog'))
    lens = np.diff(src.row_ptr.astype(np.int64))
    pick = np.arange(n_docs) % src.n_docs
    starts = src.row_ptr[:-1].astype(np.int64)[pick]
    rp = np.concatenate([[0], np.cumsum(lens[pick])]).astype(np.int64)
    idx = np.repeat(starts - rp[:-1], lens[pick]) + np.arange(rp[-1])
    batch = OpBatch(src.ops[idx], src.payload, rp.astype(np.uint32))
    n_rec = int(rp[-1])
    eng = MergeEngine(n_docs, device=device, ops_per_launch=32)
    dev = eng.stage(batch)
    del batch, idx
    el, rf, _ = timed_side_step(eng, dev)
    cs = eng.checksums()
    par = {}
    try:
        from oracle import oracle
        o = oracle.Oracle(src.n_docs).apply(src, threads=int(os.environ.get('OMP_NUM_THREADS') or 8))
        par = {'docs_checked': n_docs, 'mismatches': int(np.count_nonzero(o.checksums()[pick] != cs)),
               'against': 'oracle/mtcpu.cpp on the source logs'}
    except Exception as ex:
        par['oracle'] = f'unavailable: {ex}'
    errs = sum(1 for d in range(0, n_docs, max(1, n_docs // 256)) if eng.error(d)[0])
    par['doc_errors_sampled'] = errs
    out['editing_farm'] = {'workload': f'tests/golden/local_big (reference editing-client farm logs: local edits, '
                                       f'remote ops, acks) tiled over {n_docs} docs ({n_rec} records)',
                           'value': round(n_rec / el, 1), 'unit': 'records/s', 'ms_per_step': round(el * 1e3, 2),
                           'roofline': rf, 'parity': par}
    dev.free()
    eng.close()
    return out


def cpu_baseline(dev, gpu_cs, n_docs, budget_s, config='C3'):
    """Replay a bounded sample of the same op logs on the CPU oracle (port of the reference's
    observer path) with all of this host's cores; check the GPU checksums of the sample."""
    from oracle import oracle
    oracle.build()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count()
    # one thread per core of this host's share: the GPU box hands a 1-GPU job 16 cores and says so
    # in OMP_NUM_THREADS (its affinity mask still shows the whole machine)
    threads = max(1, int(os.environ.get('OMP_NUM_THREADS') or cores))
    chunk = max(1024, 8 * threads)
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
    cpp = {'value': round(ops / secs, 1), 'unit': 'ops/s', 'cores': threads, 'kind': 'port',
           'sample': f'docs [0, {done_docs}) of the same device-generated logs ({ops} ops, {secs:.1f} s), '
                     f'oracle/mtcpu.cpp observer replay (C++), {threads} threads (one per core of the host share)'}
    parity = {'docs_checked': done_docs, 'mismatches': mism, 'against': 'oracle/mtcpu.cpp'}
    js = js_baseline(dev, n_docs, threads, config)
    if js is None:
        return cpp, parity
    js['cpp_port'] = cpp
    return js, parity


def js_baseline(dev, n_docs, threads, config='C3', docs=1536):
    """The reference's own form of the baseline (BASELINE.json north_star: the TypeScript merge-tree
    with one worker_thread per host core): js/observerReplay.js, a JavaScript restatement of the
    observer path, over a sample of the same logs, scaled by r = reference / restatement measured
    in the build container on identical logs (oracle/tsref/calibrate.py)."""
    import shutil
    import subprocess
    import tempfile
    node = shutil.which('node')
    if not node:
        return None
    d1 = min(n_docs, docs)
    path = os.path.join(tempfile.gettempdir(), f'mtgpu_js_sample_{os.getpid()}.mtlog')
    dev.to_host(0, d1).save(path)
    try:
        out = subprocess.run([node, os.path.join(HERE, 'js', 'observerReplay.js'), 'bench', path, str(threads)],
                             capture_output=True, text=True, timeout=300)
        res = json.loads(out.stdout.strip().split('\n')[-1])
    except (subprocess.SubprocessError, ValueError, IndexError):
        return None
    finally:
        os.unlink(path)
    cal, cal_src = {}, None
    for name in (f'{CAL_ROUND}_js_calibration_{config}.json', f'r03_js_calibration_{config}.json',
                 'r02_js_calibration.json'):
        try:
            with open(os.path.join(PROFILES, name)) as f:
                c = json.load(f)
        except (OSError, ValueError):
            continue
        if c.get('config') == config:
            cal, cal_src = c, name
            break
    v = res['ops_per_sec']
    line = {'value': round(v, 1), 'unit': 'ops/s', 'cores': threads, 'kind': 'port',
            'sample': f'docs [0, {d1}) of the same device-generated logs ({res["ops"]} ops), js/observerReplay.js '
                      f'(JavaScript restatement of the observer Client path, node {os.popen(node + " --version").read().strip()}), '
                      f'{threads} worker_threads, apply-only time ({res["apply_seconds"]:.1f} s, slowest worker)'}
    if cal.get('r'):
        line['reference_estimate'] = round(v * cal['r'], 1)
        line['calibration'] = {'r': round(cal['r'], 4), 'reference_ops_per_sec': round(cal['reference_ops_per_sec'], 1),
                               'restatement_ops_per_sec': round(cal['restatement_ops_per_sec'], 1),
                               'threads': cal['threads'], 'config': cal['config'], 'docs': cal['docs'],
                               'source': f'profiles/{cal_src} (the transpiled reference '
                                         'vs this restatement, build container, identical logs)'}
    return line


if __name__ == '__main__':
    main()
