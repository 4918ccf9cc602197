"""Deli ticketing on the CPU: the oracle (oracle/deli.py, a restatement of
DeliLambda.ticket) against the known answers of the reference's own deli tests
(server/routerlicious/packages/lambdas/src/test/deli/lambda.spec.ts:101-248), and the
invariants the ordering service guarantees on random streams."""
import numpy as np
import pytest

from deli_streams import FIELDS, SPEC, oracle_tickets, random_streams
from oracle import deli as od


@pytest.mark.parametrize('name,stream,checks', SPEC, ids=[s[0] for s in SPEC])
def test_oracle_matches_lambda_spec(name, stream, checks):
    t, _ = oracle_tickets([stream])
    for i, field, want in checks:
        assert t[i, FIELDS[field]] == want, (name, i, field, t[i].tolist())


def test_spec_last_sent_message_is_the_asserted_one():
    """The spec reads testKafka.getLastMessage(): the last ticket that was sent (or nacked) is
    the one whose msn it asserts -- no later message of the scenario is sent."""
    sent = {od.SENT, od.NACK_GAP, od.NACK_CLIENT, od.NACK_REFSEQ}
    for name, stream, checks in SPEC:
        t, _ = oracle_tickets([stream])
        last_checked = max(i for i, f, _ in checks)
        later = [i for i in range(last_checked + 1, len(stream)) if t[i, 3] in sent]
        if name != 'idle_clients':   # its trailing asserts are commented out in the spec (:190)
            assert not later, (name, later)


def test_random_stream_invariants():
    """Sequenced messages: seq strictly +1 per sent message, msn monotone, refSeq >= msn
    (deltaManager.ts:1305, lambda.ts:426-428); every branch of ticket() is taken."""
    from deli_streams import to_batch
    streams = random_streams(64, 400, seed=7)
    t, docs = oracle_tickets(streams)
    msgs, row_ptr = to_batch(streams)
    seen = set()
    for d in range(len(streams)):
        rows = t[row_ptr[d]:row_ptr[d + 1]]
        kinds = msgs['kind'][row_ptr[d]:row_ptr[d + 1]]
        seen.update(rows[:, 3].tolist())
        sent = rows[rows[:, 3] == od.SENT]
        if len(sent):
            assert np.all(np.diff(sent[:, 0]) == 1)       # no sequence number is skipped
            assert np.all(np.diff(sent[:, 1]) >= 0)       # msn never goes back
            assert sent[-1, 0] == docs[d].seq
        ops = rows[(rows[:, 3] == od.SENT) & (kinds == od.OP)]
        assert np.all(ops[:, 2] >= ops[:, 1]) and np.all(ops[:, 2] <= ops[:, 0])
    assert {od.DROPPED, od.SENT, od.LATER, od.NEVER, od.NACK_GAP, od.NACK_CLIENT, od.NACK_REFSEQ} <= seen


def test_checkpoint_restore_equals_continuing():
    """new DeliLambda(lastCheckpoint) (lambda.ts:112-171) continues exactly where the
    checkpointed lambda stopped (lastSentMSN restarts at 0 in the reference; carried here)."""
    streams = random_streams(16, 300, seed=11)
    for s in streams:
        h = len(s) // 2
        whole = od.DeliDoc()
        a = [whole.ticket(*m) for m in s]
        first = od.DeliDoc()
        for m in s[:h]:
            first.ticket(*m)
        ck = first.checkpoint()
        if ck['err']:
            continue
        resumed = od.DeliDoc(seq=ck['seq'], clients=ck['clients'], last_sent_msn=ck['last_sent_msn'])
        assert resumed.msn == first.msn
        b = [resumed.ticket(*m) for m in s[h:]]
        assert a[h:] == b


def test_errors_are_sticky():
    d = od.DeliDoc()
    assert d.ticket(od.JOIN, 3, -1, -1)[3] == od.SENT
    assert d.ticket(od.NOOP, 3, 1, -1)[3] == od.HALTED          # assert(ref >= msn) throws
    assert (d.err, d.err_at) == (od.ERR_ASSERT, 1)
    assert d.ticket(od.OP, 3, 1, 0)[3] == od.HALTED
    e = od.DeliDoc()
    assert e.ticket(od.OP, od.MAX_CLIENTS + 6, 1, 0)[3] == od.HALTED and e.err == od.ERR_CLIENT
