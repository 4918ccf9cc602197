"""Sequenced op-log batches: the binary CSR format behind mt_op_rec (include/mtgpu.h).

A batch is (ops, payload, row_ptr): `ops` is a numpy structured array of 32-byte records grouped
by document and seq-ascending inside a document; `row_ptr[d]:row_ptr[d+1]` are document d's ops;
`payload` holds insert text and property pairs.  The MTLOG file container is used for golden
fixtures and cached workloads.
"""
import struct

import numpy as np

OP_DTYPE = np.dtype([
    ('seq', '<i4'), ('ref_seq', '<i4'), ('msn', '<i4'), ('client', '<u2'), ('type', 'u1'),
    ('flags', 'u1'), ('pos1', '<i4'), ('pos2', '<i4'), ('payload_off', '<u4'), ('payload_len', '<u4'),
])
assert OP_DTYPE.itemsize == 32

INSERT, REMOVE, ANNOTATE, NOOP = 0, 1, 2, 3
F_REWRITE, F_PROPS, F_GROUP_MORE = 1, 2, 4
F_MARKER = 128          # insert of a Marker: the one text byte is its ReferenceType (ops.ts:6-16)
NPAIRS_SHIFT = 3        # bits 3..6: property pairs in the payload, mod 16
OP_NP16 = 0x40          # type bit 6 (MT_OP_NP16): pair count bit 4 (16 pairs: wide records only)
OP_NP32 = 0x20          # type bit 5 (MT_OP_NP32): pair count bit 5 (wide records only)
REF_TILE, REF_NEST_BEGIN, REF_NEST_END = 1, 2, 4


OP_WIDE = 0x80          # type bit 7 (MT_OP_WIDE): UTF-16 text, 3-byte pairs (key u8, value u16 LE)


def npairs(flags, typ=0):
    """Property pairs of a record (MT_OP_NPAIRS): flags bits 3..6, plus 16 if type bit 6 is set and
    32 if type bit 5 is."""
    return ((int(flags) >> NPAIRS_SHIFT) & 15) | (16 if int(typ) & OP_NP16 else 0) | (32 if int(typ) & OP_NP32 else 0)


def pack_npairs(n, wide):
    """(flags bits, type bits) that carry n property pairs; a narrow record holds at most 8 keys and a
    wide one 32 (include/mtgpu.h MT_OP_NP16 / MT_OP_NP32): anything else is rejected, never wrapped."""
    if n < 0 or n > (32 if wide else 8):
        raise ValueError('a record carries at most %d property pairs, not %d' % (32 if wide else 8, n))
    return (n & 15) << NPAIRS_SHIFT, (OP_NP16 if n & 16 else 0) | (OP_NP32 if n & 32 else 0)


def encode_text(text, force_wide=False):
    """(bytes, wide) of a str as the engine carries text: one Latin-1 byte per UTF-16 code unit when
    every unit fits, else the UTF-16 code units little endian (lone surrogates kept)."""
    if not force_wide:
        try:
            return text.encode('latin-1'), False
        except UnicodeEncodeError:
            pass
    return text.encode('utf-16-le', 'surrogatepass'), True


def decode_text(b, wide):
    return b.decode('utf-16-le', 'surrogatepass') if wide else b.decode('latin-1')

MAGIC = b'MTLOG001'


class OpBatch:
    __slots__ = ('ops', 'payload', 'row_ptr')

    def __init__(self, ops, payload, row_ptr):
        self.ops = np.ascontiguousarray(ops, dtype=OP_DTYPE)
        self.payload = np.ascontiguousarray(payload, dtype=np.uint8)
        self.row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint32)

    @property
    def n_docs(self):
        return len(self.row_ptr) - 1

    @property
    def n_ops(self):
        return len(self.ops)

    def doc_slice(self, d0, d1):
        """Documents [d0, d1) as a self-contained batch (payload offsets rebased)."""
        a, b = int(self.row_ptr[d0]), int(self.row_ptr[d1])
        ops = self.ops[a:b].copy()
        if len(ops):
            lo = int(ops['payload_off'].min())
            hi = int((ops['payload_off'].astype(np.int64) + ops['payload_len']).max())
        else:
            lo = hi = 0
        ops['payload_off'] -= lo
        return OpBatch(ops, self.payload[lo:hi].copy(), self.row_ptr[d0:d1 + 1] - a)

    def select(self, docs):
        """The given documents (in the given order) as a self-contained batch."""
        parts = [self.doc_slice(int(d), int(d) + 1) for d in docs]
        return OpBatch.concat(parts)

    @staticmethod
    def concat(parts):
        """Documents of several batches, in order, as one batch."""
        ops, pays, rows, off, nops = [], [], [np.zeros(1, np.uint32)], 0, 0
        for b in parts:
            o = b.ops.copy()
            o['payload_off'] += off
            ops.append(o)
            pays.append(b.payload)
            rows.append(b.row_ptr[1:].astype(np.int64) + nops)
            off += len(b.payload)
            nops += b.n_ops
        return OpBatch(np.concatenate(ops) if ops else np.zeros(0, OP_DTYPE),
                       np.concatenate(pays) if pays else np.zeros(0, np.uint8),
                       np.concatenate(rows).astype(np.uint32))

    def save(self, path):
        with open(path, 'wb') as f:
            f.write(MAGIC)
            f.write(struct.pack('<IIQQ', self.n_docs, 0, self.n_ops, len(self.payload)))
            f.write(self.row_ptr.tobytes())
            f.write(self.ops.tobytes())
            f.write(self.payload.tobytes())

    @staticmethod
    def load(path):
        with open(path, 'rb') as f:
            if f.read(8) != MAGIC:
                raise ValueError(f'{path}: not an MTLOG file')
            n_docs, _, n_ops, nbytes = struct.unpack('<IIQQ', f.read(24))
            row_ptr = np.frombuffer(f.read(4 * (n_docs + 1)), dtype=np.uint32)
            ops = np.frombuffer(f.read(32 * n_ops), dtype=OP_DTYPE)
            payload = np.frombuffer(f.read(nbytes), dtype=np.uint8)
        return OpBatch(ops, payload, row_ptr)

    def split_ops(self, b):
        """Split into consecutive launches of at most `b` ops per document (the serving tick
        model of DESIGN.md); returns a list of OpBatch sharing the payload buffer."""
        counts = np.diff(self.row_ptr.astype(np.int64))
        n_ticks = int((counts.max() + b - 1) // b) if len(counts) and counts.max() > 0 else 0
        out = []
        for t in range(n_ticks):
            lo = np.minimum(self.row_ptr[:-1].astype(np.int64) + t * b, self.row_ptr[1:])
            hi = np.minimum(lo + b, self.row_ptr[1:])
            n = hi - lo
            rp = np.zeros(self.n_docs + 1, dtype=np.uint32)
            rp[1:] = np.cumsum(n)
            idx = np.concatenate([np.arange(a, c) for a, c in zip(lo, hi)]) if n.sum() else np.zeros(0, np.int64)
            out.append(OpBatch(self.ops[idx], self.payload, rp))
        return out


def synth_cfg_array(seed=1, n_clients=8, ops_per_doc=1024, max_lag=8, stall_ops=0, n_keys=0, n_values=16,
                    p_insert=0.6, p_remove=0.4, p_overlap=0.0, p_null=0.05, p_rewrite=0.0, p_insert_props=0.0,
                    p_marker=0.0):
    """mt_synth_cfg (fluidframework_amd/csrc/mt_synth.h) as raw little-endian bytes."""
    def fx(p):
        return min(int(round(p * 4294967296.0)), 0xFFFFFFFF)
    return struct.pack('<14I', seed, n_clients, ops_per_doc, max_lag, stall_ops, n_keys, n_values,
                       fx(p_insert), fx(p_remove), fx(p_overlap), fx(p_null), fx(p_rewrite), fx(p_insert_props),
                       fx(p_marker))


# The BASELINE.json configurations, as synthetic-workload parameters.
CONFIGS = {
    'C1': dict(n_docs=1, n_clients=8, ops_per_doc=2048, max_lag=16, p_insert=0.6, p_remove=0.4),
    'C2': dict(n_docs=10_000, n_clients=8, ops_per_doc=1024, max_lag=8, p_insert=0.6, p_remove=0.4),
    'C3': dict(n_docs=100_000, n_clients=32, ops_per_doc=1024, max_lag=32, n_keys=8, n_values=16,
               p_insert=0.45, p_remove=0.30, p_overlap=0.5, p_null=0.05, p_rewrite=0.02, p_insert_props=0.1),
    'C4': dict(n_docs=100_000, n_clients=8, ops_per_doc=1024, max_lag=256, stall_ops=200,
               p_insert=0.6, p_remove=0.4),
    # C3 with 48 clients: overlap sets past 32 bits (side line of bench.py)
    'C3W': dict(n_docs=100_000, n_clients=48, ops_per_doc=1024, max_lag=32, n_keys=8, n_values=16,
                p_insert=0.45, p_remove=0.30, p_overlap=0.5, p_null=0.05, p_rewrite=0.02, p_insert_props=0.1),
    # 1M documents over the 8 GPUs of a node (n_docs is per GPU): raw client messages go through
    # the deli kernel (seq / msn assigned and stamped into the op records), then the apply.  The
    # 8 clients' joins are the deli checkpoint the documents start from (joined at seq 0).
    'C5': dict(n_docs=125_000, n_clients=8, ops_per_doc=256, max_lag=8, p_insert=0.6, p_remove=0.4),
}
# configurations whose step runs deli before the apply
DELI_CONFIGS = ('C5',)
