"""libmtgpu's RCCL surface (fluidframework_amd/csrc/mt_comm.cpp) on the box's one GPU: a one-rank
communicator runs every mt_comm_* call -- ncclGetUniqueId, ncclCommInitRank, the all-reduce behind
the max-over-ranks clock and the barrier, and the ncclGather of per-document checksums from HBM --
except the cross-GPU transfer itself.  The driver's 8-GPU
scaling run covers the transfer."""
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_one_rank_rccl_gathers_the_engine_checksums():
    from fluidframework_amd import shard
    from fluidframework_amd.engine import MergeEngine
    from fluidframework_amd.oplog import CONFIGS
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 128
    n = 1000
    eng = MergeEngine(n, ops_per_launch=32)
    dev = eng.synthesize(seed=5, **cfg)
    eng.reset()
    eng.apply_staged(dev)
    want = eng.checksums()
    comm = shard.RcclComm(0, 1, 0, rendezvous=shard.FileRendezvous(key='test_' + uuid.uuid4().hex))
    try:
        assert comm.max(3.25) == 3.25
        comm.barrier()
        parts = comm.gather_checksums(eng, n + 24)   # padded rows, as a rank with fewer documents sends
        assert len(parts) == 1 and parts[0].dtype == np.uint64
        assert np.array_equal(parts[0], want)
        assert shard.digest(shard.assemble(parts, [np.arange(n)])) == shard.digest(want)
    finally:
        comm.close()


def test_bench_with_a_one_rank_rccl_communicator():
    """bench.py --comm rccl at world size 1: the headline script's RCCL path end to end."""
    env = dict(os.environ, MTGPU_RUN_ID=uuid.uuid4().hex)
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--comm', 'rccl', '--docs', '2048',
                          '--ops', '128', '--steps', '1', '--warmup', '0', '--no-cpu-baseline'],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().split('\n')[-1])
    assert line['config']['comm'] == 'RcclComm' and line['n_gpus'] == 1 and line['value'] > 0


def test_rank_past_the_gather_bound_still_joins_and_reports():
    """A rank holding more documents than the agreed bound sends a poisoned row instead of skipping
    the collective (a skipped ncclGather leaves the peers blocked): the call returns the
    rank's error, and the communicator stays usable for the next gather."""
    from fluidframework_amd import shard
    from fluidframework_amd.engine import MergeEngine, MtError
    from fluidframework_amd.oplog import CONFIGS
    cfg = dict(CONFIGS['C3'])
    cfg.pop('n_docs')
    cfg['ops_per_doc'] = 64
    n = 256
    eng = MergeEngine(n, ops_per_launch=32)
    dev = eng.synthesize(seed=9, **cfg)
    eng.reset()
    eng.apply_staged(dev)
    comm = shard.RcclComm(0, 1, 0, rendezvous=shard.FileRendezvous(key='test_' + uuid.uuid4().hex))
    try:
        with pytest.raises(MtError):
            comm.gather_checksums(eng, n - 1)
        parts = comm.gather_checksums(eng, n)
        assert np.array_equal(parts[0], eng.checksums())
    finally:
        comm.close()
