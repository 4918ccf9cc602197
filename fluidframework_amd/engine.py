"""Python host binding of libmtgpu.so (ctypes over the C-ABI in include/mtgpu.h).

`MergeEngine` owns many independent documents on one MI355X; `apply(batch)` is the batched
drop-in for calling `Client.applyMsg` (client.ts:797-819) on every op of every document.
The HIP library is required: there is no CPU fallback, and a missing/unbuilt library raises.
"""
import ctypes
import json
import os

import numpy as np

from .oplog import OP_DTYPE, OpBatch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('MTGPU_LIB') or os.path.join(HERE, 'libmtgpu.so')

MT_ERRORS = {0: 'ok', 1: 'bad argument', 2: 'HIP error', 3: 'out of device memory', 4: 'bad state',
             5: 'document error', 6: 'RCCL error', 7: 'document past the form of the call (wide)'}
DOC_ERRORS = {0: None,
              1: "Incoming remote op sequence# <= local collabWindow's currentSequence#",
              2: "Incoming remote op minSequence# < local collabWindow's minSequence#",
              3: 'MergeTree insert failed',
              4: 'device capacity exceeded',
              5: 'text arena exhausted',
              6: 'client id / property key / value id out of range',
              7: 'malformed op record',
              8: 'delta-event buffer full'}


# mt_tile_query / mt_tile_result (include/mtgpu.h "findTile")
TILE_QUERY_DTYPE = np.dtype([('doc', '<u4'), ('pos', '<i4'), ('key', 'u1'), ('preceding', 'u1'), ('pad0', 'u1'),
                             ('pad1', 'u1'), ('vmask', '<u4', (8,)), ('pad2', '<u4')])
TILE_RESULT_DTYPE = np.dtype([('pos', '<i4'), ('ordinal', '<i4')])
# mt_pos_query / mt_pos_result (include/mtgpu.h): getContainingSegment / getPosition queries
POS_QUERY_DTYPE = np.dtype([('doc', '<u4'), ('pos', '<i4'), ('ref_seq', '<i4'), ('client', '<u2'), ('kind', '<u2')])
POS_RESULT_DTYPE = np.dtype([('ordinal', '<i4'), ('offset', '<i4'), ('position', '<i4'), ('length', '<u4')])
POS_CONTAINING, POS_OF_ORDINAL, POS_LOCAL = 0, 1, -2**31
assert POS_QUERY_DTYPE.itemsize == 16 and POS_RESULT_DTYPE.itemsize == 16
assert TILE_QUERY_DTYPE.itemsize == 48
# mt_stack_item (include/mtgpu.h "range stacks")
STACK_ITEM_DTYPE = np.dtype([('pos', '<i4'), ('ordinal', '<i4'), ('ref_type', '<u4')])


class MtError(RuntimeError):
    pass


class _Cfg(ctypes.Structure):
    _fields_ = [('device', ctypes.c_int32), ('max_docs', ctypes.c_uint32), ('seg_capacity', ctypes.c_uint32),
                ('text_capacity', ctypes.c_uint32), ('heap_capacity', ctypes.c_uint32),
                ('ops_per_launch', ctypes.c_uint32)]


_lib = None


def lib():
    """Load libmtgpu.so (built in-tree by fluidframework_amd/build.py); raise if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MtError(f'{LIB_PATH} is missing: build it with `python fluidframework_amd/build.py` '
                          '(there is no CPU fallback)')
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
        L.mt_engine_create.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(vp)]
        L.mt_engine_destroy.argtypes = [vp]
        L.mt_docs_init.argtypes = [vp, u32]
        L.mt_batch_upload.argtypes = [vp, vp, u64, vp, u64, vp, ctypes.POINTER(vp)]
        L.mt_batch_apply.argtypes = [vp, vp]
        L.mt_batch_free.argtypes = [vp, vp]
        L.mt_submit.argtypes = [vp, vp, u64, vp, u64, vp]
        L.mt_sync.argtypes = [vp]
        L.mt_get_length.argtypes = [vp, u32, ctypes.POINTER(u32)]
        L.mt_get_text.argtypes = [vp, u32, ctypes.c_char_p, u64, ctypes.POINTER(u64)]
        L.mt_get_state.argtypes = [vp, u32, ctypes.c_char_p, u64, ctypes.POINTER(u64)]
        L.mt_checksums.argtypes = [vp, vp, u32]
        L.mt_doc_error.argtypes = [vp, u32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.mt_last_apply_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                          ctypes.POINTER(u32), ctypes.POINTER(u64)]
        L.mt_seg_counts.argtypes = [vp, vp, u32]
        L.mt_set_concurrent_classes.argtypes = [vp, i32]
        L.mt_last_apply_class_stats.argtypes = [vp, u32, ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_float),
                                                ctypes.POINTER(u32), ctypes.POINTER(u64)]
        L.mt_synth_generate.argtypes = [vp, vp, u32, u32, ctypes.POINTER(vp)]
        for name, at in (('mt_synth_generate_ids', [vp, vp, vp, u32, ctypes.POINTER(vp)]),
                         ('mt_engine_info', [vp, ctypes.POINTER(u32), ctypes.POINTER(u32)]),
                         ('mt_checksums_device', [vp, vp, u32])):
            if hasattr(L, name):  # (an older build loaded for an A/B lacks them)
                getattr(L, name).argtypes = at
                getattr(L, name).restype = ctypes.c_int
        L.mt_batch_copy_docs.argtypes = [vp, vp, u32, u32, vp, ctypes.POINTER(u64), vp, ctypes.POINTER(u64), vp]
        L.mt_batch_info.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u32)]
        L.mt_class_kernel_name.argtypes = [vp, u32, ctypes.c_char_p, u64]
        L.mt_get_snapshot.argtypes = [vp, u32, u32, ctypes.POINTER(ctypes.c_char_p), u32, ctypes.c_char_p, u64,
                                      ctypes.POINTER(u64)]
        L.mt_snapshot_extract.argtypes = [vp, u32, u32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(u64)]
        L.mt_get_snapshots.argtypes = [vp, u32, u32, u32, ctypes.POINTER(ctypes.c_char_p), u32, ctypes.c_char_p, u64,
                                       vp]
        L.mt_find_tiles.argtypes = [vp, vp, u32, vp]
        for name in ('mt_resolve_positions', 'mt_resolve_positions_device'):  # (absent from older A/B builds)
            if hasattr(L, name):
                getattr(L, name).argtypes = [vp, vp, u32, vp]
                getattr(L, name).restype = ctypes.c_int
        L.mt_range_stacks.argtypes = [vp, vp, u32, u32, vp, vp]
        L.mt_regen_drain.argtypes = [vp, u32, vp, u32, vp, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.mt_events_enable.argtypes = [vp, u32]
        L.mt_events_drain.argtypes = [vp, vp, u64, vp, ctypes.POINTER(u64)]
        L.mt_set_label_keys.argtypes = [vp, u32, i32, i32]
        L.mt_version.restype = ctypes.c_char_p
        for name in ('mt_engine_create', 'mt_engine_destroy', 'mt_docs_init', 'mt_batch_upload', 'mt_batch_apply',
                     'mt_batch_free', 'mt_submit', 'mt_sync', 'mt_get_length', 'mt_get_text', 'mt_get_state',
                     'mt_checksums', 'mt_doc_error', 'mt_last_apply_stats', 'mt_seg_counts', 'mt_synth_generate',
                     'mt_batch_copy_docs', 'mt_batch_info', 'mt_last_apply_class_stats', 'mt_class_kernel_name',
                     'mt_get_snapshot', 'mt_get_snapshots', 'mt_snapshot_extract', 'mt_find_tiles', 'mt_range_stacks', 'mt_regen_drain', 'mt_set_concurrent_classes',

                     'mt_events_enable', 'mt_events_drain', 'mt_set_label_keys'):
            getattr(L, name).restype = ctypes.c_int
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        raise MtError(f'{what}: {MT_ERRORS.get(rc, rc)}')


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class DeviceBatch:
    """An op batch resident in HBM: staged from the host (mt_batch_upload) or synthesised on the
    device (mt_synth_generate).  Apply it with MergeEngine.apply_staged."""

    def __init__(self, engine, batch=None, handle=None):
        self.engine = engine
        if handle is not None:
            self.h = handle
        else:
            self.h = ctypes.c_void_p()
            _check(lib().mt_batch_upload(engine.h, _ptr(batch.ops), batch.n_ops, _ptr(batch.payload),
                                         len(batch.payload), _ptr(batch.row_ptr), ctypes.byref(self.h)),
                   'mt_batch_upload')
        n_ops, nbytes, mx = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
        _check(lib().mt_batch_info(self.h, ctypes.byref(n_ops), ctypes.byref(nbytes), ctypes.byref(mx)),
               'mt_batch_info')
        self.n_ops, self.payload_region, self.max_ops_per_doc = n_ops.value, nbytes.value, mx.value

    def to_host(self, d0=0, d1=None):
        """Documents [d0, d1) as a host OpBatch (payload offsets rebased)."""
        d1 = self.engine.n_docs if d1 is None else d1
        n_ops, nbytes = ctypes.c_uint64(), ctypes.c_uint64()
        L = lib()
        _check(L.mt_batch_copy_docs(self.engine.h, self.h, d0, d1, None, ctypes.byref(n_ops), None,
                                    ctypes.byref(nbytes), None), 'mt_batch_copy_docs')
        from .oplog import OP_DTYPE
        ops = np.zeros(n_ops.value, dtype=OP_DTYPE)
        payload = np.zeros(nbytes.value, dtype=np.uint8)
        row_ptr = np.zeros(d1 - d0 + 1, dtype=np.uint32)
        _check(L.mt_batch_copy_docs(self.engine.h, self.h, d0, d1, _ptr(ops), ctypes.byref(n_ops), _ptr(payload),
                                    ctypes.byref(nbytes), _ptr(row_ptr)), 'mt_batch_copy_docs')
        return OpBatch(ops, payload, row_ptr)

    def free(self):
        if self.h:
            lib().mt_batch_free(self.engine.h, self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class MergeEngine:
    def __init__(self, n_docs, device=0, seg_capacity=2048, text_capacity=64 * 1024, heap_capacity=0,
                 ops_per_launch=0):
        cfg = _Cfg(device, n_docs, seg_capacity, text_capacity, heap_capacity, ops_per_launch)
        self.h = ctypes.c_void_p()
        _check(lib().mt_engine_create(ctypes.byref(cfg), ctypes.byref(self.h)), 'mt_engine_create')
        self.n_docs = n_docs
        _check(lib().mt_docs_init(self.h, n_docs), 'mt_docs_init')

    def close(self):
        if getattr(self, 'h', None):
            lib().mt_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- apply --------------------------------------------------------------------------
    def apply(self, batch: OpBatch):
        """Synchronous drop-in for applyMsg over every op of the batch."""
        assert batch.n_docs == self.n_docs, 'a batch covers every document of the engine'
        _check(lib().mt_submit(self.h, _ptr(batch.ops), batch.n_ops, _ptr(batch.payload), len(batch.payload),
                               _ptr(batch.row_ptr)), 'mt_submit')
        return self

    def apply_ticks(self, log, deli=None):
        """A tick-major feed (ticks.TickLog) from host memory with the upload overlapped
        (mt_submit_ticks; with a DeliSequencer, each tick's raw messages are ticketed first:
        mt_submit_ticks_deli).  The same states as apply() of each tick in order."""
        from .ticks import submit_ticks
        return submit_ticks(self, log, deli)

    def stage(self, batch: OpBatch):
        assert batch.n_docs == self.n_docs
        return DeviceBatch(self, batch)

    def synthesize(self, payload_per_doc=32 * 1024, doc_id_base=0, doc_ids=None, **cfg):
        """Generate a synthetic op log for every document ON THE DEVICE (mt_synth.h model; the
        documents end in the post-generation state -- call reset() before replaying it).  The
        RNG stream of engine document i is global document doc_ids[i] (a hash-routed shard), or
        doc_id_base + i."""
        from .oplog import synth_cfg_array
        raw = ctypes.create_string_buffer(synth_cfg_array(**cfg))
        h = ctypes.c_void_p()
        if doc_ids is not None:
            ids = np.ascontiguousarray(doc_ids, dtype=np.uint32)
            assert len(ids) == self.n_docs
            _check(lib().mt_synth_generate_ids(self.h, raw, _ptr(ids), payload_per_doc, ctypes.byref(h)),
                   'mt_synth_generate_ids')
        else:
            _check(lib().mt_synth_generate(self.h, raw, doc_id_base, payload_per_doc, ctypes.byref(h)),
                   'mt_synth_generate')
        return DeviceBatch(self, handle=h)

    def reset(self):
        """All documents back to empty (mt_docs_init)."""
        _check(lib().mt_docs_init(self.h, self.n_docs), 'mt_docs_init')

    def apply_staged(self, dbatch: DeviceBatch):
        _check(lib().mt_batch_apply(self.h, dbatch.h), 'mt_batch_apply')
        return self

    def last_stats(self):
        """(kernel_ms, wall_ms, launches, alg_bytes) of the last apply (see mtgpu.h)."""
        ms, wall, launches, nbytes = ctypes.c_float(), ctypes.c_float(), ctypes.c_uint32(), ctypes.c_uint64()
        _check(lib().mt_last_apply_stats(self.h, ctypes.byref(ms), ctypes.byref(wall), ctypes.byref(launches),
                                         ctypes.byref(nbytes)), 'mt_last_apply_stats')
        return ms.value, wall.value, launches.value, nbytes.value

    def set_concurrent_classes(self, on):
        """Capacity classes of a tick on concurrent streams (True, default) or serialized (False)."""
        _check(lib().mt_set_concurrent_classes(self.h, 1 if on else 0), 'mt_set_concurrent_classes')

    def last_class_stats(self):
        """[(capacity, kernel_ms, launches, alg_bytes)] per capacity class of the last apply (then the
        editing bucket, MT_CLASS_EDITING | 1024, and the LDS engine inside each register class,
        MT_CLASS_LDS | capacity: include/mtgpu.h)."""
        out = []
        for c in range(256):  # classes 0.. until the library reports MT_ERR_ARG
            cap, ms, n, nb = ctypes.c_uint32(), ctypes.c_float(), ctypes.c_uint32(), ctypes.c_uint64()
            if lib().mt_last_apply_class_stats(self.h, c, ctypes.byref(cap), ctypes.byref(ms), ctypes.byref(n),
                                               ctypes.byref(nb)) != 0:
                break
            out.append((cap.value, ms.value, n.value, nb.value))
        return out

    def class_kernel(self, capacity):
        """Kernel symbol (as rocprof names it) that applies documents of a capacity class."""
        buf = ctypes.create_string_buffer(128)
        _check(lib().mt_class_kernel_name(self.h, capacity, buf, 128), 'mt_class_kernel_name')
        return buf.value.decode()

    # -- findTile (include/mtgpu.h) --------------------------------------------------------
    def set_label_keys(self, tile_key, range_key, doc=None):
        """Declare the key ids of "referenceTileLabels" / "referenceRangeLabels" (-1: unused) for one
        document or all (mt_set_label_keys): its findTile / getStackContext then follow the reference's
        block caches after label annotates."""
        _check(lib().mt_set_label_keys(self.h, 0xFFFFFFFF if doc is None else doc, tile_key, range_key),
               'mt_set_label_keys')

    def find_tiles(self, queries):
        """Client.findTile for a batch of TILE_QUERY_DTYPE rows: TILE_RESULT_DTYPE rows (pos -1: none)."""
        q = np.ascontiguousarray(queries, dtype=TILE_QUERY_DTYPE)
        out = np.zeros(len(q), dtype=TILE_RESULT_DTYPE)
        _check(lib().mt_find_tiles(self.h, _ptr(q), len(q), _ptr(out)), 'mt_find_tiles')
        return out

    def resolve_positions(self, queries):
        """MergeTree.getContainingSegment / getPosition for a batch of POS_QUERY_DTYPE rows
        (mt_resolve_positions): POS_RESULT_DTYPE rows (ordinal -1: none)."""
        q = np.ascontiguousarray(queries, dtype=POS_QUERY_DTYPE)
        out = np.zeros(len(q), dtype=POS_RESULT_DTYPE)
        _check(lib().mt_resolve_positions(self.h, _ptr(q), len(q), _ptr(out)), 'mt_resolve_positions')
        return out

    def resolve_positions_device(self, d_queries, n, d_out):
        """mt_resolve_positions_device: device-resident POS_QUERY_DTYPE rows -> POS_RESULT_DTYPE rows
        (device pointers as ints; asynchronous on the engine's stream, complete after sync())."""
        _check(lib().mt_resolve_positions_device(self.h, d_queries, n, d_out), 'mt_resolve_positions_device')
        _check(lib().mt_sync(self.h), 'mt_sync')

    def regen_drain(self, doc):
        """The ops the document regenerated at its MT_SEQ_REGEN records (Client.regeneratePendingOp)
        since the last drain: [[record index, [[type, pos1, pos2, text | None, props | None,
        flags], ...]], ...] (flags: 128 marker, 1 rewrite; props keyed by key id as strings)."""
        n, pn = ctypes.c_uint32(0), ctypes.c_uint32(0)
        _check(lib().mt_regen_drain(self.h, doc, None, 0, None, 0, ctypes.byref(n), ctypes.byref(pn)), 'mt_regen_drain')
        recs = np.zeros(n.value, dtype=OP_DTYPE)
        pay = np.zeros(max(1, pn.value), dtype=np.uint8)
        _check(lib().mt_regen_drain(self.h, doc, _ptr(recs), n.value, _ptr(pay), pn.value, ctypes.byref(n),
                                    ctypes.byref(pn)), 'mt_regen_drain')
        out = []
        for r in recs:
            t = int(r['type'])
            if t == 3:  # header: the resetting record's index
                out.append([int(r['seq']), []])
                continue
            fl = int(r['flags'])
            npairs = (fl >> 3) & 15
            off, ln = int(r['payload_off']), int(r['payload_len'])
            body = bytes(pay[off:off + ln])
            pairs = body[ln - 2 * npairs:]
            if t == 0:
                props = {str(pairs[2 * q]): int(pairs[2 * q + 1]) for q in range(npairs)} if fl & 2 else None
                out[-1][1].append([0, int(r['pos1']), 0, body[:ln - 2 * npairs].decode('latin-1'), props, fl & 128])
            elif t == 1:
                out[-1][1].append([1, int(r['pos1']), int(r['pos2']), None, None, 0])
            else:
                props = {str(pairs[2 * q]): (int(pairs[2 * q + 1]) or None) for q in range(npairs)}
                out[-1][1].append([2, int(r['pos1']), int(r['pos2']), None, props, fl & 1])
        return out

    def range_stacks(self, queries, cap=64):
        """Client.getStackContext for a batch of TILE_QUERY_DTYPE rows (key: the range-labels key id,
        vmask: the label's value ids; preceding ignored): one list of STACK_ITEM_DTYPE rows per
        query, bottom to top.  A stack deeper than `cap` is asked again with room for it."""
        q = np.ascontiguousarray(queries, dtype=TILE_QUERY_DTYPE)
        items = np.zeros((len(q), cap), dtype=STACK_ITEM_DTYPE)
        depth = np.zeros(len(q), dtype=np.uint32)
        _check(lib().mt_range_stacks(self.h, _ptr(q), len(q), cap, _ptr(items), _ptr(depth)), 'mt_range_stacks')
        depth &= 0x7FFFFFFF  # MT_STACK_DEPTH
        if len(q) and int(depth.max()) > cap:
            return self.range_stacks(q, int(depth.max()))
        return [items[i, :int(depth[i])] for i in range(len(q))]

    # -- delta / maintenance events (mergeTreeDeltaCallback.ts; include/mtgpu.h) --------------
    def enable_events(self, per_doc=4096):
        """Record the callbacks of every later apply, `per_doc` records per document between drains
        (0 stops recording).  Recording runs every document on the LDS engine."""
        _check(lib().mt_events_enable(self.h, per_doc), 'mt_events_enable')
        return self

    def drain_event_rows(self):
        """(rows, row_ptr): every document's mt_event records since the last drain (then cleared)."""
        from .events import EVENT_DTYPE
        row_ptr = np.zeros(self.n_docs + 1, dtype=np.uint32)
        total = ctypes.c_uint64()
        _check(lib().mt_events_drain(self.h, None, 0, _ptr(row_ptr), ctypes.byref(total)), 'mt_events_drain')
        rows = np.zeros(max(1, total.value), dtype=EVENT_DTYPE)
        _check(lib().mt_events_drain(self.h, _ptr(rows), total.value, _ptr(row_ptr), ctypes.byref(total)),
               'mt_events_drain')
        return rows[:total.value], row_ptr

    def drain_events(self):
        """Per document, its callbacks since the last drain in canonical form (events.callbacks)."""
        from .events import callbacks
        rows, rp = self.drain_event_rows()
        return [callbacks(rows[rp[d]:rp[d + 1]]) for d in range(self.n_docs)]

    # -- readout -------------------------------------------------------------------------
    def checksums(self):
        out = np.zeros(self.n_docs, dtype=np.uint64)
        _check(lib().mt_checksums(self.h, _ptr(out), self.n_docs), 'mt_checksums')
        return out

    def seg_counts(self):
        out = np.zeros(self.n_docs, dtype=np.uint32)
        _check(lib().mt_seg_counts(self.h, _ptr(out), self.n_docs), 'mt_seg_counts')
        return out

    def error(self, doc):
        code, seq = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().mt_doc_error(self.h, doc, ctypes.byref(code), ctypes.byref(seq)), 'mt_doc_error')
        return code.value, seq.value

    def _raw(self, fn, doc):
        n = ctypes.c_uint64()
        _check(fn(self.h, doc, None, 0, ctypes.byref(n)), fn.__name__)
        buf = ctypes.create_string_buffer(n.value + 1)
        _check(fn(self.h, doc, buf, n.value + 1, ctypes.byref(n)), fn.__name__)
        return buf.raw[:n.value]

    def _string(self, fn, doc):
        return self._raw(fn, doc).decode('latin-1')

    def state(self, doc):
        return json.loads(self._string(lib().mt_get_state, doc))

    def snapshot(self, doc, chunk_size=0, client_names=None):
        """SnapshotV1 extractSync + emit of one document (snapshotV1.ts:85-247): the emitted
        tree's blobs as {path: parsed JSON}.  client_names[short id] -> long client id."""
        names = None
        n = 0
        if client_names is not None:
            n = len(client_names)
            names = (ctypes.c_char_p * n)(*[x.encode() for x in client_names])
        L = lib()
        ln = ctypes.c_uint64()
        _check(L.mt_get_snapshot(self.h, doc, chunk_size, names, n, None, 0, ctypes.byref(ln)), 'mt_get_snapshot')
        buf = ctypes.create_string_buffer(ln.value + 1)
        _check(L.mt_get_snapshot(self.h, doc, chunk_size, names, n, buf, ln.value + 1, ctypes.byref(ln)),
               'mt_get_snapshot')
        return json.loads(buf.raw[:ln.value].decode('latin-1'))

    def snapshots_raw(self, d0=0, n=None, chunk_size=0, client_names=None):
        """mt_get_snapshots: (bytes, offsets) of documents [d0, d0+n), their JSON written on all host cores."""
        n = self.n_docs - d0 if n is None else n
        names, nn = None, 0
        if client_names is not None:
            nn = len(client_names)
            names = (ctypes.c_char_p * nn)(*[x.encode() for x in client_names])
        off = np.zeros(n + 1, dtype=np.uint64)
        L = lib()
        _check(L.mt_get_snapshots(self.h, d0, n, chunk_size, names, nn, None, 0, _ptr(off)), 'mt_get_snapshots')
        buf = ctypes.create_string_buffer(max(1, int(off[-1])))
        _check(L.mt_get_snapshots(self.h, d0, n, chunk_size, names, nn, buf, int(off[-1]), _ptr(off)),
               'mt_get_snapshots')
        return buf.raw[:int(off[-1])], off

    def snapshots(self, d0=0, n=None, chunk_size=0, client_names=None):
        """SnapshotV1 extractSync + emit of documents [d0, d0+n) in one batched call: a list of
        {path: parsed JSON} (the same as snapshot() per document)."""
        raw, off = self.snapshots_raw(d0, n, chunk_size, client_names)
        return [json.loads(raw[int(off[i]):int(off[i + 1])].decode('latin-1')) for i in range(len(off) - 1)]

    def snapshot_extract(self, d0=0, n=None):
        """Device extraction for documents [d0, d0+n): (kernel_ms, segment specs)."""
        n = self.n_docs - d0 if n is None else n
        ms, cnt = ctypes.c_float(), ctypes.c_uint64()
        _check(lib().mt_snapshot_extract(self.h, d0, n, ctypes.byref(ms), ctypes.byref(cnt)), 'mt_snapshot_extract')
        return ms.value, cnt.value

    def text(self, doc):
        """MergeTreeTextHelper.getText: the UTF-16 code units as a str (surrogate halves kept)."""
        return self._raw(lib().mt_get_text, doc).decode('utf-16-le', 'surrogatepass')

    def length(self, doc):
        n = ctypes.c_uint32()
        _check(lib().mt_get_length(self.h, doc, ctypes.byref(n)), 'mt_get_length')
        return n.value
