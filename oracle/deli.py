"""CPU restatement of the deli sequencer -- TEST INFRASTRUCTURE ONLY.

Imported by tests/ (and nothing on the product path) as the checker of the GPU deli kernel
(fluidframework_amd/csrc/mt_deli.hip).  Follows, statement by statement:

  DeliLambda.ticket            server/routerlicious/packages/lambdas/src/deli/lambda.ts:255-544
  DeliLambda.checkOrder        lambda.ts:590-626
  DeliLambda.handler           lambda.ts:173-246 (only the lastSentMSN bookkeeping, :192-219)
  DeliLambda.createNackMessage lambda.ts:683-712 (a nack carries the current msn, :698,706)
  DeliLambda.revSequenceNumber lambda.ts:769-771
  ClientSequenceNumberManager  deli/clientSeqManager.ts:70-143
  Heap                         common/lib/common-utils/src/heap.ts:50-169

The Heap in ClientSequenceNumberManager is a correct binary min-heap on referenceSequenceNumber
(add/update/remove restore the heap invariant, heap.ts:88-123), so `getMinimumSequenceNumber`
(clientSeqManager.ts:136-143) is the plain minimum over tracked clients; it is restated as min().

Pinned by the known-answer tests of lambda.spec.ts (tests/test_deli.py restates each one with
its line numbers).  Messages are tuples (kind, client, csn, ref) with the kinds of
include/mtgpu.h (mt_raw_kind); tickets are (seq, msn, ref, status) with mt_ticket_status.
"""

# mt_raw_kind
OP, NOOP, NOOP_DATA, JOIN, LEAVE, SERVER_NOOP, NOCLIENT, CONTROL = range(8)
# mt_ticket_status
DROPPED, SENT, LATER, NEVER, NACK_GAP, NACK_CLIENT, NACK_REFSEQ, HALTED = range(8)
# mt_deli_err
ERR_CLIENT, ERR_KIND, ERR_ASSERT = 1, 2, 3
MAX_CLIENTS = 4096  # include/mtgpu.h MT_DELI_MAX_CLIENTS (the engine's limit; the lambda has none)


class Client:
    """IClientSequenceNumber (server-services-core) -- the fields ticket() reads."""
    __slots__ = ('csn', 'ref', 'nack')

    def __init__(self, csn, ref, nack=False):
        self.csn, self.ref, self.nack = csn, ref, nack


class DeliDoc:
    """One document's DeliLambda, constructed from a checkpoint (lambda.ts:112-171)."""

    def __init__(self, seq=0, clients=None, last_sent_msn=0):
        self.clients = {}                       # clientNodeMap (clientSeqManager.ts:23)
        for c, (csn, ref, nack) in (clients or {}).items():
            self.clients[c] = Client(csn, ref, nack)    # upsertClient per checkpoint client (:125-136)
        self.seq = seq                          # this.sequenceNumber = lastCheckpoint.sequenceNumber (:162)
        m = self._min_ref()
        self.msn = self.seq if m == -1 else m   # (:166-167)
        self.last_sent = last_sent_msn          # lastSentMSN = 0 (:103)
        self.err = 0
        self.err_at = -1
        self.n = 0                              # messages seen (for err_at)

    # ClientSequenceNumberManager ------------------------------------------------------------
    def _upsert(self, c, csn, ref, nack=False):
        """upsertClient (clientSeqManager.ts:70-97): add if new, then update every field."""
        new = c not in self.clients
        if new:
            self.clients[c] = Client(csn, ref, nack)
        cl = self.clients[c]                    # updateClient (:102-115)
        cl.ref, cl.csn, cl.nack = ref, csn, nack
        return new

    def _min_ref(self):
        """getMinimumSequenceNumber (clientSeqManager.ts:136-143): heap peek, or -1 if empty."""
        return min((cl.ref for cl in self.clients.values()), default=-1)

    # DeliLambda ------------------------------------------------------------------------------
    def _rev(self):
        self.seq += 1                           # revSequenceNumber (:769-771)
        return self.seq

    def ticket(self, kind, c, csn, ref):
        """ticket() + the handler's lastSentMSN update; returns (seq, msn, ref, status)."""
        idx = self.n
        self.n += 1
        if self.err:
            return (self.seq, self.msn, ref, HALTED)
        if c >= MAX_CLIENTS or kind > CONTROL:
            self.err, self.err_at = (ERR_CLIENT if c >= MAX_CLIENTS else ERR_KIND), idx
            return (self.seq, self.msn, ref, HALTED)
        client_msg = kind in (OP, NOOP, NOOP_DATA)     # message.clientId is set

        # checkOrder (:590-626): only client messages of a tracked client are checked
        if client_msg and c in self.clients:
            expected = self.clients[c].csn + 1
            if csn > expected:                  # Gap -> nack (:269-275)
                return self._nack(ref, NACK_GAP)
            if csn < expected:                  # Duplicate -> dropped (:267-268)
                return (self.seq, self.msn, ref, DROPPED)

        if not client_msg:
            if kind == LEAVE:                   # (:281-285)
                if c not in self.clients:
                    return (self.seq, self.msn, ref, DROPPED)
                del self.clients[c]             # removeClient (clientSeqManager.ts:121-131)
            elif kind == JOIN:                  # (:286-299): upsert at the current msn
                if not self._upsert(c, 0, self.msn):
                    return (self.seq, self.msn, ref, DROPPED)
        else:
            cl = self.clients.get(c)            # (:308-316)
            if cl is None or cl.nack:
                return self._nack(ref, NACK_CLIENT)
            if ref != -1 and ref < self.msn:    # (:317-335)
                self._upsert(c, csn, self.msn, True)
                return self._nack(ref, NACK_REFSEQ)

        seq = self.seq                          # (:352)
        if client_msg:
            if kind != NOOP and kind != NOOP_DATA:   # don't rev for client no-ops (:415-425)
                seq = self._rev()
                if ref == -1:
                    ref = seq
            if not ref >= self.msn:             # assert (:426-428) throws inside the lambda
                self.err, self.err_at = ERR_ASSERT, idx
                return (seq, self.msn, ref, HALTED)
            self._upsert(c, csn, ref)           # (:430-435)
        elif kind not in (SERVER_NOOP, NOCLIENT, CONTROL):
            seq = self._rev()                   # join / leave rev (:437-442)

        m = self._min_ref()                     # (:446-455)
        no_active = m == -1
        self.msn = seq if no_active else m

        send = SENT
        if kind in (NOOP, NOOP_DATA):           # client no-ops (:461-472)
            if kind == NOOP:                    # contents === null
                send = LATER
            elif self.msn <= self.last_sent:
                send = LATER
            else:
                seq = self._rev()
        elif kind == SERVER_NOOP:               # (:473-479)
            if self.msn <= self.last_sent:
                send = NEVER
            else:
                seq = self._rev()
        elif kind == NOCLIENT:                  # (:481-489)
            if no_active:
                seq = self._rev()
                ref = seq
                self.msn = seq
            else:
                send = NEVER
        elif kind == CONTROL:                   # (:490-517)
            send = NEVER
        if send == SENT:                        # handler: lastSentMSN = msn of what is sent (:217-218)
            self.last_sent = self.msn
        return (seq, self.msn, ref, send)

    def _nack(self, ref, status):
        """createNackMessage (:683-712): carries the current msn; the handler records it as the
        last sent msn (:192-219, a nacked ticket skips the send-type checks)."""
        self.last_sent = self.msn
        return (self.msn, self.msn, ref, status)

    def checkpoint(self):
        return {'seq': self.seq, 'msn': self.msn, 'last_sent_msn': self.last_sent, 'err': self.err,
                'clients': {c: (cl.csn, cl.ref, cl.nack) for c, cl in self.clients.items()}}


def ticket_batch(msgs, row_ptr, docs=None):
    """Ticket a CSR batch (numpy structured array of RAW_DTYPE + row pointers); returns the
    tickets as an (n, 4) int array [seq, msn, ref, status] and the DeliDoc objects."""
    import numpy as np
    n_docs = len(row_ptr) - 1
    docs = docs if docs is not None else [DeliDoc() for _ in range(n_docs)]
    out = np.zeros((len(msgs), 4), dtype=np.int64)
    kind, client, csn, ref = (msgs['kind'].tolist(), msgs['client'].tolist(), msgs['csn'].tolist(),
                              msgs['ref_seq'].tolist())
    for d in range(n_docs):
        doc = docs[d]
        for i in range(int(row_ptr[d]), int(row_ptr[d + 1])):
            out[i] = doc.ticket(kind[i], client[i], csn[i], ref[i])
    return out, docs
