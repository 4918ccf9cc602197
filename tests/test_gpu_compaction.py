"""Text-arena compaction inside the register engine (mt_apply_reg.hip compact_text): documents whose
inserts and zamboni appends write more text than a tight arena half holds, so the arena is compacted
many times inside a replay (by segment id, from the per-id lengths in LDS), while deferred
ENDS_WITH_NEWLINE flags of split segments (F_NLQ) are resolved from the text at scour and store.
Bit-exact against the CPU oracle (state and checksum)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# heavy churn with 32 clients: ~12.6 K characters inserted per document against ~2-3 K linked at
# the end; an 8 KiB arena half overflows (and compacts) in every document
CHURN = dict(n_clients=32, ops_per_doc=2560, max_lag=8, n_keys=8, n_values=16, p_insert=0.5, p_remove=0.48,
             p_overlap=0.5, p_insert_props=0.1)


def _linked_text(o, d):
    return sum(len(s[0]) if isinstance(s[0], str) else 1 for s in o.state(d)['segs'])


def test_register_engine_compacts_tight_arenas(oracle_lib):
    from fluidframework_amd.engine import MergeEngine
    n = 128
    batch = oracle_lib.generate(n, seed=77, **CHURN)
    o = oracle_lib.Oracle(n).apply(batch, threads=8)
    cap = 8192
    linked = [_linked_text(o, d) for d in range(n)]
    assert max(linked) < cap // 2, max(linked)
    ins = np.array([int(batch.ops['payload_len'][batch.row_ptr[d]:batch.row_ptr[d + 1]][
        batch.ops['type'][batch.row_ptr[d]:batch.row_ptr[d + 1]] == 0].sum()) for d in range(n)])
    assert int((ins > cap).sum()) > n // 2, 'the workload must overflow most arenas'
    eng = MergeEngine(n, text_capacity=cap, ops_per_launch=32)
    assert eng.class_kernel(512).startswith('mtr::reg_apply_kernel')
    eng.apply(batch)
    got, want = eng.checksums(), o.checksums()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (bad[:8], [eng.error(int(d)) for d in bad[:4]])
    for d in range(0, n, 9):
        assert eng.error(d) == (0, 0), eng.error(d)
        assert eng.state(d) == o.state(d), d
        assert eng.text(d) == o.text(d), d
