"""Raw-message streams for the deli tests: the known-answer scenarios of the reference's
lambda.spec.ts, and seeded random streams that reach every branch of DeliLambda.ticket
(joins / re-joins, leaves of absent clients, csn gaps and duplicates, refSeq below the msn,
REST ops with refSeq -1, client and server no-ops, NoClient, Control, client ids past the
device limit, the refSeq >= msn assert)."""
import random

import numpy as np

from fluidframework_amd.deli import RAW_DTYPE
from oracle import deli as od

A, B, C = 0, 1, 2   # "quiet-rat", "test2", "test3" of lambda.spec.ts

# (name, [(kind, client, csn, ref)], checks) -- checks: list of (message index, field, value) on
# the ticket of that message, restating each spec's asserts.  MessageFactory numbers a client's
# ops 1, 2, ... (messageFactory.ts:78-88); joins / leaves carry csn = ref = -1 (:95-131).
SPEC = [
    # "Should nack a client that has not sent a join" (lambda.spec.ts:102-108)
    ('nack_without_join', [(od.OP, A, 1, 10)], [(0, 'status', od.NACK_CLIENT)]),
    # "Should nack a client that sends a message under the min sequence number" (:110-115, forceNack :57-69)
    ('nack_below_msn', [(od.JOIN, A, -1, -1), (od.OP, A, 1, 10), (od.JOIN, B, -1, -1), (od.OP, B, 1, 5)],
     [(3, 'status', od.NACK_REFSEQ)]),
    # "Should nack all future messages from a nacked client" (:117-128)
    ('nack_after_nack', [(od.JOIN, A, -1, -1), (od.OP, A, 1, 10), (od.JOIN, B, -1, -1), (od.OP, B, 1, 5),
                         (od.OP, B, 2, 15)],
     [(3, 'status', od.NACK_REFSEQ), (4, 'status', od.NACK_CLIENT)]),
    # "Should be able to ticket an incoming message" (:130-147): 2 sent, the op gets seq 2
    ('ticket_message', [(od.JOIN, A, -1, -1), (od.OP, A, 1, 0)],
     [(0, 'status', od.SENT), (1, 'status', od.SENT), (1, 'seq', 2)]),
    # "Should ticket new clients connecting above msn" (:149-167): msn 20, then 22
    ('join_above_msn', [(od.JOIN, A, -1, -1), (od.OP, A, 1, 10), (od.OP, A, 2, 20), (od.JOIN, B, -1, -1),
                        (od.OP, B, 1, 25), (od.OP, A, 3, 22)],
     [(2, 'msn', 20), (5, 'msn', 22)]),
    # "Should timeout idle clients" (:169-191): msn 10 after the first four messages
    ('idle_clients', [(od.JOIN, A, -1, -1), (od.OP, A, 1, 10), (od.JOIN, B, -1, -1), (od.OP, B, 1, 20),
                      (od.OP, B, 2, 20), (od.OP, B, 3, 20)],
     [(3, 'msn', 10)]),
    # "Should remove clients after a disconnect" (:193-247): msn 0, 1, 4, 7, 7
    ('disconnect', [(od.JOIN, A, -1, -1), (od.JOIN, B, -1, -1), (od.OP, A, 1, 1), (od.OP, B, 1, 2),
                    (od.LEAVE, A, -1, -1), (od.OP, B, 2, 4), (od.LEAVE, B, -1, -1), (od.JOIN, C, -1, -1),
                    (od.OP, C, 1, 7)],
     [(0, 'msn', 0), (3, 'msn', 1), (5, 'msn', 4), (6, 'msn', 7), (8, 'msn', 7)]),
]
FIELDS = {'seq': 0, 'msn': 1, 'ref_seq': 2, 'status': 3}


def to_batch(streams):
    """[[(kind, client, csn, ref)]] per document -> (RAW_DTYPE array, row_ptr)."""
    rows = [m for s in streams for m in s]
    msgs = np.zeros(len(rows), dtype=RAW_DTYPE)
    if rows:
        arr = np.array(rows, dtype=np.int64)
        msgs['kind'], msgs['client'], msgs['csn'], msgs['ref_seq'] = arr[:, 0], arr[:, 1], arr[:, 2], arr[:, 3]
    row_ptr = np.zeros(len(streams) + 1, dtype=np.uint32)
    row_ptr[1:] = np.cumsum([len(s) for s in streams])
    return msgs, row_ptr


def random_stream(rng, n_msgs, n_clients=12, p_assert=0.0, wide=False):
    """One document's raw messages, chosen against a shadow DeliDoc so that most ops are
    in order and in the window (the interesting branches are taken at controlled rates)."""
    shadow = od.DeliDoc()
    out = []
    pool = list(range(min(n_clients, od.MAX_CLIENTS)))
    for _ in range(n_msgs):
        r = rng.random()
        if wide and rng.random() < 0.01:
            m = (od.OP, od.MAX_CLIENTS + rng.randrange(8), 1, shadow.seq)
        elif r < 0.08:
            m = (od.JOIN, rng.choice(pool), -1, -1)
        elif r < 0.12:
            m = (od.LEAVE, rng.choice(pool), -1, -1)
        elif r < 0.86:
            joined = list(shadow.clients)
            c = rng.choice(joined) if joined and rng.random() < 0.93 else rng.choice(pool)
            cl = shadow.clients.get(c)
            exp = (cl.csn + 1) if cl else 1
            q = rng.random()
            csn = exp if q < 0.9 else (exp + rng.randrange(1, 3) if q < 0.95 else max(0, exp - rng.randrange(1, 3)))
            q = rng.random()
            lo = shadow.msn
            if q < 0.8:
                ref = rng.randint(min(lo, shadow.seq), shadow.seq)
                if cl:
                    ref = max(ref, min(cl.ref, shadow.seq))
            elif q < 0.87 and lo > 0:
                ref = rng.randrange(0, lo)
            elif q < 0.95:
                ref = -1
            else:
                ref = shadow.seq
            q = rng.random()
            if q < 0.8:
                kind = od.OP
            elif q < 0.9:
                kind = od.NOOP_DATA
            else:
                kind = od.NOOP
            if kind != od.OP and ref == -1 and rng.random() >= p_assert:
                ref = shadow.seq     # a no-op with refSeq -1 trips the lambda's assert
            m = (kind, c, csn, ref)
        elif r < 0.94:
            m = (od.SERVER_NOOP, 0, -1, -1)
        elif r < 0.97:
            m = (od.NOCLIENT, 0, -1, -1)
        else:
            m = (od.CONTROL, 0, -1, -1)
        shadow.ticket(*m)
        out.append(m)
    return out


def random_streams(n_docs, n_msgs, seed=1, **kw):
    rng = random.Random(seed)
    return [random_stream(rng, rng.randint(0, n_msgs), **kw) for _ in range(n_docs)]


def oracle_tickets(streams, checkpoints=None):
    """Expected tickets (n, 4) [seq, msn, ref, status] and final DeliDoc per document."""
    docs = [od.DeliDoc(**(checkpoints[i] if checkpoints else {})) for i in range(len(streams))]
    msgs, row_ptr = to_batch(streams)
    return od.ticket_batch(msgs, row_ptr, docs)
