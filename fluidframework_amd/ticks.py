"""Tick-major op feeds (include/mtgpu.h "tick-major feed"): the next ops of every document, tick
after tick, applied from page-locked host memory with the upload overlapped (mt_submit_ticks).

A serving loop behind SharedSegmentSequence.processMergeTreeMsg
(packages/dds/sequence/src/sequence.ts:593-633) sees each document's sequenced ops one message at a
time; a node serving many documents receives, per tick, the next ops of all of them.  `TickLog`
holds such a feed: either built tick by tick by the caller, or laid out from a document-major
`OpBatch` (mt_log_to_ticks, host cores, no device work).  `MergeEngine.apply_ticks` applies it:
tick k + 1 is copied into a ring of device slots while tick k applies, so every launch still holds
every document (SURVEY.md §8(d) times the apply from the first H2D)."""
import ctypes

import numpy as np

from .engine import _check, _ptr, lib
from .hipmem import PinnedArray
from .oplog import OP_DTYPE, OpBatch


class Tick(ctypes.Structure):
    """mt_tick"""
    _fields_ = [('ops', ctypes.c_void_p), ('n_ops', ctypes.c_uint64), ('payload', ctypes.c_void_p),
                ('payload_bytes', ctypes.c_uint64), ('doc_row_ptr', ctypes.c_void_p), ('msgs', ctypes.c_void_p),
                ('n_msgs', ctypes.c_uint64), ('msg_row_ptr', ctypes.c_void_p), ('tickets', ctypes.c_void_p)]


class _Layout(ctypes.Structure):
    """mt_tick_layout"""
    _fields_ = [('n_ticks', ctypes.c_uint32), ('pad', ctypes.c_uint32), ('payload_bytes', ctypes.c_uint64),
                ('ops', ctypes.c_void_p), ('payload', ctypes.c_void_p), ('row_ptrs', ctypes.c_void_p),
                ('tick_ops', ctypes.c_void_p), ('tick_payload', ctypes.c_void_p), ('msgs', ctypes.c_void_p),
                ('msg_row_ptrs', ctypes.c_void_p), ('tick_msgs', ctypes.c_void_p)]


_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.mt_submit_ticks.argtypes = [vp, vp, u32]
        L.mt_submit_ticks_deli.argtypes = [vp, vp, vp, u32]
        L.mt_log_to_ticks.argtypes = [vp, u64, vp, u64, vp, u32, u32, vp, u64, vp, ctypes.POINTER(_Layout)]
        L.mt_log_to_ticks_ramp.argtypes = [vp, u64, vp, u64, vp, u32, u32, u32, vp, u64, vp, ctypes.POINTER(_Layout)]
        for name in ('mt_submit_ticks', 'mt_submit_ticks_deli', 'mt_log_to_ticks', 'mt_log_to_ticks_ramp'):
            getattr(L, name).restype = ctypes.c_int
        _bound = True
    return L


class TickLog:
    """A tick-major feed of `n_docs` documents in host memory (page-locked by default).

    `TickLog.from_batch(batch, per)` lays a document-major OpBatch out tick-major: tick t holds
    records [t*per, (t+1)*per) of every document, payload compacted per tick (`first`: a ramp, tick t
    holds min(per, first << t) records -- mt_log_to_ticks_ramp, short first ticks for the copies the
    apply waits for at the start).  With `msgs` /
    `msg_row_ptr` (deli RAW_DTYPE rows in the mt_deli_raw_stream layout, op_index = 1 + the record's
    index in the batch) each tick also carries its raw messages for mt_submit_ticks_deli;
    `tickets=True` gives every tick a host buffer its tickets come back to (`tickets_of(t)`)."""

    def __init__(self, n_docs, n_ops, payload_bytes, n_ticks, n_msgs=0, pinned=True, tickets=False):
        def arr(count, dtype):
            if pinned:
                p = PinnedArray(count, dtype)
                self._pins.append(p)
                return p.a
            return np.zeros(count, dtype=dtype)
        self._pins = []
        self.n_docs, self.n_ticks = n_docs, n_ticks
        self.ops = arr(n_ops, OP_DTYPE)
        self.payload = arr(max(1, payload_bytes), np.uint8)
        self.row_ptrs = arr(n_ticks * (n_docs + 1), np.uint32)
        self.tick_ops = np.zeros(n_ticks + 1, dtype=np.uint64)
        self.tick_payload = np.zeros(n_ticks + 1, dtype=np.uint64)
        self.n_msgs = n_msgs
        if n_msgs:
            from .deli import RAW_DTYPE, TICKET_DTYPE
            self.msgs = arr(n_msgs, RAW_DTYPE)
            self.msg_row_ptrs = arr(n_ticks * (n_docs + 1), np.uint32)
            self.tick_msgs = np.zeros(n_ticks + 1, dtype=np.uint64)
            self.tickets = arr(n_msgs, TICKET_DTYPE) if tickets else None
        else:
            self.msgs = self.msg_row_ptrs = self.tick_msgs = self.tickets = None
        self._ticks = None

    @classmethod
    def from_batch(cls, batch: OpBatch, per, msgs=None, msg_row_ptr=None, pinned=True, tickets=False, first=None):
        L = _lib()
        lay = _Layout()
        n_msgs = 0 if msgs is None else len(msgs)
        mp = None if msgs is None else _ptr(np.ascontiguousarray(msgs))
        mr = None if msgs is None else _ptr(np.ascontiguousarray(msg_row_ptr, dtype=np.uint32))
        args = (_ptr(batch.ops), batch.n_ops, _ptr(batch.payload), len(batch.payload), _ptr(batch.row_ptr),
                batch.n_docs, per, per if first is None else first, mp, n_msgs, mr)
        _check(L.mt_log_to_ticks_ramp(*args, ctypes.byref(lay)), 'mt_log_to_ticks_ramp')
        self = cls(batch.n_docs, batch.n_ops, lay.payload_bytes, lay.n_ticks, n_msgs, pinned, tickets)
        lay.ops, lay.payload, lay.row_ptrs = self.ops.ctypes.data, self.payload.ctypes.data, self.row_ptrs.ctypes.data
        lay.tick_ops, lay.tick_payload = self.tick_ops.ctypes.data, self.tick_payload.ctypes.data
        if n_msgs:
            lay.msgs, lay.msg_row_ptrs = self.msgs.ctypes.data, self.msg_row_ptrs.ctypes.data
            lay.tick_msgs = self.tick_msgs.ctypes.data
        _check(L.mt_log_to_ticks_ramp(*args, ctypes.byref(lay)), 'mt_log_to_ticks_ramp')
        return self

    def ticks(self):
        """The mt_tick array (pointers into this log's arrays)."""
        if self._ticks is None:
            D = self.n_docs
            arr = (Tick * self.n_ticks)()
            rec = OP_DTYPE.itemsize
            for t in range(self.n_ticks):
                o0, o1 = int(self.tick_ops[t]), int(self.tick_ops[t + 1])
                p0, p1 = int(self.tick_payload[t]), int(self.tick_payload[t + 1])
                x = arr[t]
                x.ops, x.n_ops = self.ops.ctypes.data + o0 * rec, o1 - o0
                x.payload, x.payload_bytes = self.payload.ctypes.data + p0, p1 - p0
                x.doc_row_ptr = self.row_ptrs.ctypes.data + t * (D + 1) * 4
                if self.n_msgs:
                    m0, m1 = int(self.tick_msgs[t]), int(self.tick_msgs[t + 1])
                    x.msgs, x.n_msgs = self.msgs.ctypes.data + m0 * 16, m1 - m0
                    x.msg_row_ptr = self.msg_row_ptrs.ctypes.data + t * (D + 1) * 4
                    if self.tickets is not None:
                        x.tickets = self.tickets.ctypes.data + m0 * 16
            self._ticks = arr
        return self._ticks

    def tick_batch(self, t):
        """Tick t as an OpBatch (a view; payload offsets relative to the tick)."""
        o0, o1 = int(self.tick_ops[t]), int(self.tick_ops[t + 1])
        p0, p1 = int(self.tick_payload[t]), int(self.tick_payload[t + 1])
        rp = self.row_ptrs[t * (self.n_docs + 1):(t + 1) * (self.n_docs + 1)]
        return OpBatch(self.ops[o0:o1], self.payload[p0:max(p1, p0 + 1)], rp)

    def upload_bytes(self):
        """Bytes a full submit moves host -> device (records, payload, row pointers, messages)."""
        n = self.ops.nbytes + int(self.tick_payload[-1]) + self.n_ticks * (self.n_docs + 1) * 4
        if self.n_msgs:
            n += self.msgs.nbytes + self.n_ticks * (self.n_docs + 1) * 4
        return n

    def free(self):
        self._ticks = None
        self.ops = self.payload = self.row_ptrs = self.msgs = self.msg_row_ptrs = self.tickets = None
        for p in self._pins:
            p.free()
        self._pins = []


def submit_ticks(engine, log: TickLog, deli=None):
    """mt_submit_ticks (or, with a DeliSequencer, mt_submit_ticks_deli) over every tick of `log`."""
    t = log.ticks()
    if deli is None:
        _check(_lib().mt_submit_ticks(engine.h, ctypes.cast(t, ctypes.c_void_p), log.n_ticks), 'mt_submit_ticks')
    else:
        _check(_lib().mt_submit_ticks_deli(engine.h, deli.h, ctypes.cast(t, ctypes.c_void_p), log.n_ticks),
               'mt_submit_ticks_deli')
    return engine
