"""Python host binding of the deli sequencer in libmtgpu.so (include/mtgpu.h, "deli" section).

`DeliSequencer` is the batched drop-in for the ordering service's per-document `DeliLambda`
(server/routerlicious/packages/lambdas/src/deli/lambda.ts:87-171): one object holds the
sequencing state of many documents on one MI355X, and `ticket(msgs, row_ptr)` runs
`DeliLambda.ticket` (:255-544) over every raw message of every document.  Client ids are
per-document short ids (< 64) interned by the caller.  No CPU fallback: the HIP library is
required (engine.lib() raises when it is missing).
"""
import ctypes

import numpy as np

from .engine import MtError, _check, _ptr, lib

# mt_raw_kind
OP, NOOP, NOOP_DATA, JOIN, LEAVE, SERVER_NOOP, NOCLIENT, CONTROL = range(8)
# mt_ticket_status
DROPPED, SENT, LATER, NEVER, NACK_GAP, NACK_CLIENT, NACK_REFSEQ, HALTED = range(8)
STATUS_NAMES = ['dropped', 'sent', 'later', 'never', 'nack-gap', 'nack-client', 'nack-refseq', 'halted']
DELI_ERRORS = {0: None, 1: 'client id out of range', 2: 'unknown message kind',
               3: 'assert(referenceSequenceNumber >= minimumSequenceNumber) (lambda.ts:426-428)',
               4: 'capacity: no big-pool row left for a document past client 63'}
ERR_CAPACITY = 4  # mt_deli_err MT_DELI_ERR_CAPACITY
MAX_CLIENTS = 4096  # include/mtgpu.h MT_DELI_MAX_CLIENTS (up to 63: eight documents per wave; to 511 the wide
# form; then the huge form)
CKPT_CLIENTS = 64  # mt_deli_checkpoint's client slots

RAW_DTYPE = np.dtype([('csn', '<i4'), ('ref_seq', '<i4'), ('client', '<u2'), ('kind', 'u1'), ('pad', 'u1'),
                      ('op_index', '<u4')])  # 1 + linked op record (fused hand-off), 0 = none
TICKET_DTYPE = np.dtype([('seq', '<i4'), ('msn', '<i4'), ('ref_seq', '<i4'), ('status', 'u1'), ('pad', 'u1', (3,))])
assert RAW_DTYPE.itemsize == 16 and TICKET_DTYPE.itemsize == 16


class _Client(ctypes.Structure):
    _fields_ = [('csn', ctypes.c_int32), ('ref_seq', ctypes.c_int32), ('joined', ctypes.c_uint8),
                ('nack', ctypes.c_uint8), ('pad', ctypes.c_uint8 * 2)]


class _Checkpoint(ctypes.Structure):
    _fields_ = [('seq', ctypes.c_int32), ('msn', ctypes.c_int32), ('last_sent_msn', ctypes.c_int32),
                ('err', ctypes.c_int32), ('clients', _Client * CKPT_CLIENTS)]


class _CheckpointWide(ctypes.Structure):  # mt_deli_checkpoint_wide: every client slot
    _fields_ = [('seq', ctypes.c_int32), ('msn', ctypes.c_int32), ('last_sent_msn', ctypes.c_int32),
                ('err', ctypes.c_int32), ('clients', _Client * MAX_CLIENTS)]


_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
        L.mt_deli_create.argtypes = [i32, u32, ctypes.POINTER(vp)]
        L.mt_deli_destroy.argtypes = [vp]
        L.mt_deli_restore.argtypes = [vp, u32, u32, vp]
        L.mt_deli_restore_all.argtypes = [vp, u32, vp]
        L.mt_deli_ticket.argtypes = [vp, vp, u64, vp, u32, vp]
        L.mt_deli_ticket_device.argtypes = [vp, vp, vp, u32, vp, vp, u64]
        L.mt_deli_raw_from_ops.argtypes = [vp, vp, vp, u32, vp]
        L.mt_deli_raw_stream.argtypes = [vp, vp, vp, u32, u32, vp, vp]
        L.mt_deli_sync.argtypes = [vp]
        L.mt_deli_last_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
        L.mt_deli_get_checkpoint.argtypes = [vp, u32, vp]
        L.mt_deli_get_checkpoint_wide.argtypes = [vp, u32, vp]
        L.mt_deli_restore_wide.argtypes = [vp, u32, u32, vp]
        L.mt_deli_get_clients.argtypes = [vp, u32, u32, u32, vp]
        L.mt_deli_doc_error.argtypes = [vp, u32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.mt_batch_device_ptrs.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp)]
        for name in ('mt_deli_create', 'mt_deli_destroy', 'mt_deli_restore', 'mt_deli_restore_all', 'mt_deli_ticket',
                     'mt_deli_ticket_device', 'mt_deli_raw_from_ops', 'mt_deli_raw_stream', 'mt_deli_sync', 'mt_deli_last_ms',
                     'mt_deli_get_checkpoint', 'mt_deli_get_clients', 'mt_deli_doc_error', 'mt_batch_device_ptrs',
                     'mt_deli_get_checkpoint_wide', 'mt_deli_restore_wide'):
            getattr(L, name).restype = ctypes.c_int
        _bound = True
    return L


def make_checkpoint(seq=0, clients=None, last_sent_msn=0, wide=False):
    """IDeliState -> mt_deli_checkpoint (wide: mt_deli_checkpoint_wide, client ids up to MAX_CLIENTS - 1).
    clients: {short id: (csn, ref_seq, nack)}."""
    ck = _CheckpointWide() if wide else _Checkpoint()
    ck.seq, ck.last_sent_msn = seq, last_sent_msn
    for c, (csn, ref, nack) in (clients or {}).items():
        if not 0 <= c < (MAX_CLIENTS if wide else CKPT_CLIENTS):
            raise MtError(f'client id {c} out of range of a checkpoint')
        ck.clients[c].csn, ck.clients[c].ref_seq = csn, ref
        ck.clients[c].joined, ck.clients[c].nack = 1, int(bool(nack))
    return ck


class DeliSequencer:
    """Sequencing state of `n_docs` documents (new documents: sequenceNumber 0, no clients)."""

    def __init__(self, n_docs, device=0):
        self.h = ctypes.c_void_p()
        _check(_lib().mt_deli_create(device, n_docs, ctypes.byref(self.h)), 'mt_deli_create')
        self.n_docs = n_docs

    def close(self):
        if getattr(self, 'h', None):
            _lib().mt_deli_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def restore(self, checkpoints, doc0=0):
        """new DeliLambda(..., lastCheckpoint) for documents doc0.. (lambda.ts:112-171);
        checkpoints: list of dicts {seq, clients: {id: (csn, ref, nack)}, last_sent_msn}.  A checkpoint
        with a client id >= 64 goes through the wide form (mt_deli_restore_wide: a big-pool row)."""
        cks = [{k: v for k, v in ck.items() if k in ('seq', 'clients', 'last_sent_msn')} for ck in checkpoints]
        if any(c >= CKPT_CLIENTS for ck in cks for c in (ck.get('clients') or {})):
            arr = (_CheckpointWide * len(cks))(*[make_checkpoint(wide=True, **ck) for ck in cks])
            _check(_lib().mt_deli_restore_wide(self.h, doc0, len(cks), ctypes.cast(arr, ctypes.c_void_p)),
                   'mt_deli_restore_wide')
            return
        arr = (_Checkpoint * len(cks))(*[make_checkpoint(**ck) for ck in cks])
        _check(_lib().mt_deli_restore(self.h, doc0, len(cks), ctypes.cast(arr, ctypes.c_void_p)),
               'mt_deli_restore')

    def restore_all(self, n_docs=None, **checkpoint):
        ck = make_checkpoint(**checkpoint)
        _check(_lib().mt_deli_restore_all(self.h, self.n_docs if n_docs is None else n_docs, ctypes.byref(ck)),
               'mt_deli_restore_all')

    def ticket(self, msgs, row_ptr):
        """DeliLambda.ticket over a CSR batch of raw messages (RAW_DTYPE rows grouped by
        document); returns one TICKET_DTYPE row per message."""
        msgs = np.ascontiguousarray(msgs, dtype=RAW_DTYPE)
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint32)
        out = np.zeros(len(msgs), dtype=TICKET_DTYPE)
        _check(_lib().mt_deli_ticket(self.h, _ptr(msgs), len(msgs), _ptr(row_ptr), len(row_ptr) - 1, _ptr(out)),
               'mt_deli_ticket')
        return out

    def ticket_device(self, d_msgs, d_row_ptr, n_docs, d_out, d_ops=None, n_ops=0):
        """Asynchronous ticketing of device-resident buffers (raw device pointers as ints); with
        d_ops, messages whose op_index = k + 1 stamp op record k (k < n_ops)."""
        _check(_lib().mt_deli_ticket_device(self.h, d_msgs, d_row_ptr, n_docs, d_out, d_ops, n_ops),
               'mt_deli_ticket_device')

    def raw_from_ops(self, d_ops, d_row_ptr, n_docs, d_msgs):
        _check(_lib().mt_deli_raw_from_ops(self.h, d_ops, d_row_ptr, n_docs, d_msgs), 'mt_deli_raw_from_ops')

    def raw_stream(self, d_ops, d_row_ptr, n_docs, n_join, d_msgs, d_msg_row_ptr):
        """C5's raw streams: n_join joins then the log's op messages, per document (mtgpu.h)."""
        _check(_lib().mt_deli_raw_stream(self.h, d_ops, d_row_ptr, n_docs, n_join, d_msgs, d_msg_row_ptr),
               'mt_deli_raw_stream')

    def sync(self):
        _check(_lib().mt_deli_sync(self.h), 'mt_deli_sync')

    def last_ms(self):
        ms = ctypes.c_float()
        _check(_lib().mt_deli_last_ms(self.h, ctypes.byref(ms)), 'mt_deli_last_ms')
        return ms.value

    def checkpoint(self, doc):
        """generateDeliCheckpoint (lambda.ts:754-764), device-representable part: every joined client
        (ids up to MAX_CLIENTS - 1, mt_deli_get_clients)."""
        ck = _CheckpointWide()
        _check(_lib().mt_deli_get_checkpoint_wide(self.h, doc, ctypes.byref(ck)), 'mt_deli_get_checkpoint_wide')
        cl = ck.clients
        return {'seq': ck.seq, 'msn': ck.msn, 'last_sent_msn': ck.last_sent_msn, 'err': ck.err,
                'clients': {c: (cl[c].csn, cl[c].ref_seq, bool(cl[c].nack)) for c in range(MAX_CLIENTS) if cl[c].joined}}

    def checkpoint_narrow(self, doc):
        """mt_deli_get_checkpoint: the 64-client form; raises (MT_ERR_WIDE) for a document past client 63."""
        ck = _Checkpoint()
        _check(_lib().mt_deli_get_checkpoint(self.h, doc, ctypes.byref(ck)), 'mt_deli_get_checkpoint')
        return {'seq': ck.seq, 'msn': ck.msn, 'last_sent_msn': ck.last_sent_msn, 'err': ck.err,
                'clients': {c: (ck.clients[c].csn, ck.clients[c].ref_seq, bool(ck.clients[c].nack))
                            for c in range(CKPT_CLIENTS) if ck.clients[c].joined}}

    def error(self, doc):
        err, idx = ctypes.c_int32(), ctypes.c_int32()
        _check(_lib().mt_deli_doc_error(self.h, doc, ctypes.byref(err), ctypes.byref(idx)), 'mt_deli_doc_error')
        return err.value, idx.value


def batch_device_ptrs(dbatch):
    """(ops, payload, row_ptr) device pointers of a DeviceBatch (to chain deli -> apply)."""
    o, p, r = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    _check(_lib().mt_batch_device_ptrs(dbatch.h, ctypes.byref(o), ctypes.byref(p), ctypes.byref(r)),
           'mt_batch_device_ptrs')
    return o.value, p.value, r.value
