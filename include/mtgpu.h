/*
 * mtgpu.h -- C-ABI of the MI355X batched merge-tree engine (libmtgpu.so).
 *
 * Drop-in boundary for the reference's op-apply surface:
 *   Client.applyMsg(msg: ISequencedDocumentMessage)       packages/dds/merge-tree/src/client.ts:797-819
 *   new Client(...) + startOrUpdateCollaboration(longId)  client.ts:74-83, 1051-1071
 *   Client.getLength()                                    client.ts:1049
 *   TestClient.getText() / MergeTreeTextHelper.getText    src/test/testClient.ts:102-104, textSegment.ts:154-172
 * One engine owns many independent documents (one reference `Client` observer per document);
 * a batch of sequenced ops from many documents is applied in one submit.  The host shim
 * (js/batchClient.js over the N-API addon, or fluidframework_amd/client.py over ctypes) turns
 * ISequencedDocumentMessage JSON into mt_op_rec rows: long client ids are interned per document
 * in first-appearance order with the observer as short id 0 (client.ts:636-660, 1057-1062);
 * property keys/values are interned per document (properties.ts; ids are opaque, equality only).
 *
 * Plain pointers and sizes only; no torch or HIP types.  All functions return mt_status.
 */
#ifndef MTGPU_H
#define MTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- op record: one merge-tree delta op of one sequenced message (32 bytes) -------------- */
enum mt_op_type {
    MT_OP_INSERT = 0,   /* ops.ts:29-34 MergeTreeDeltaType.INSERT   (client.ts:393-441)      */
    MT_OP_REMOVE = 1,   /* MergeTreeDeltaType.REMOVE                (client.ts:320-351)      */
    MT_OP_ANNOTATE = 2, /* MergeTreeDeltaType.ANNOTATE              (client.ts:358-386)      */
    MT_OP_NOOP = 3,     /* non-op message: only updateSeqNumbers(msn, seq) (client.ts:818)  */
    MT_OP_LOAD = 4      /* snapshot body segment: MergeTree.insertSegments(pos1, [seg], ref_seq,
                           client, seq) as SnapshotLoader.loadBody appends it (snapshotLoader.ts:
                           192-224) -- no collab-window asserts, no updateSeqNumbers.  The segment
                           may arrive removed: pos2 = its removedSeq (-1: not removed) and the
                           high byte of `client` the low byte of its removedClient; `msn` holds the
                           high bytes of both short ids (client's in bits 0..7, removedClient's in
                           8..15: 0 below 256).  See mt_docs_load. */
};
enum mt_op_flags {
    MT_F_REWRITE = 1u << 0,    /* annotate with combiningOp {name:"rewrite"} (properties.ts:118-124) */
    MT_F_PROPS = 1u << 1,      /* insert spec carries a props object (TextSegment.make, textSegment.ts:24-30) */
    MT_F_GROUP_MORE = 1u << 2, /* GROUP member: next record is the next member of the same message
                                  (client.ts:782-790); the window update waits for the last member */
    MT_F_MARKER = 1u << 7      /* insert of a Marker (mergeTree.ts:630-798, IJSONMarkerSegment): the
                                  payload's text part is one byte, its ReferenceType (ops.ts:6-16;
                                  Simple/Tile/NestBegin/NestEnd/RangeBegin/RangeEnd/Slide/Stay); the
                                  segment has length 1 and never appends (Marker.canAppend) */
};
#define MT_F_NPAIRS_SHIFT 3    /* bits 3..6: number of (key,value) property pairs in the payload, mod 16 */
/* A wide record may carry up to 32 pairs (one per wide key, MT_MAX_KEYS_WIDE): the count's bit 4 is
 * type bit 6 (MT_OP_NP16) and its bit 5 type bit 5 (MT_OP_NP32), set only on wide records.
 * MT_OP_NPAIRS takes the record. */
#define MT_OP_NP16 0x40u
#define MT_OP_NP32 0x20u
#define MT_OP_NPAIRS(o) ((((o).flags >> MT_F_NPAIRS_SHIFT) & 0xF) | (((o).type & MT_OP_NP16) ? 16 : 0) | \
                         (((o).type & MT_OP_NP32) ? 32 : 0))
/* an MT_OP_LOAD record's segment client and removedClient (short ids; see MT_OP_LOAD) */
#define MT_LOAD_CLIENT(o) (((uint32_t)(o).client & 0xFFu) | (((uint32_t)(o).msn & 0xFFu) << 8))
#define MT_LOAD_RCLIENT(o) (((uint32_t)(o).client >> 8) | ((((uint32_t)(o).msn >> 8) & 0xFFu) << 8))
/* Wide payload (type bit 7): the op's text is UTF-16 code units (2 bytes each, little endian:
 * cachedLength = text.length, textSegment.ts:45 -- any string, surrogate halves included) and each
 * property pair is 3 bytes (key u8 < MT_MAX_KEYS_WIDE, value id u16 LE).  The host sets it on every
 * op whose text, keys or value ids do not fit the narrow form ([Latin-1 bytes][key u8 < 8, value u8]).
 * A document that receives a wide op, or a client id >= MT_MAX_CLIENTS, becomes a WIDE document for
 * good (see "limits" below); narrow-form ops apply to wide documents unchanged. */
#define MT_OP_WIDE 0x80u
#define MT_OP_TYPE(o) ((o).type & 0x1Fu)
#define MT_OP_PAIR_BYTES(o) (((o).type & MT_OP_WIDE) ? 3u : 2u)
#define MT_OP_PAIRS_LEN(o) (MT_OP_PAIR_BYTES(o) * MT_OP_NPAIRS(o))
/* a remove or annotate record carries no text: its payload is exactly its pairs (else MT_DERR_BAD_OP) */
#define MT_OP_NO_TEXT_OK(o) ((MT_OP_TYPE(o) != MT_OP_REMOVE && MT_OP_TYPE(o) != MT_OP_ANNOTATE) || \
                             (o).payload_len == MT_OP_PAIRS_LEN(o))
/* An insert whose segment spec is the empty string is dropped by Client.applyInsertOp before it
 * touches the tree (`if (op.seg)`, client.ts:403-407: no boundary split, no completeAndLogOp
 * asserts, no callback); only updateSeqNumbers runs.  Such a record (text insert, no props, no
 * text bytes) is applied exactly as an MT_OP_NOOP.  An empty text WITH a props object is a real
 * insert: the boundary split happens and blockInsert skips the zero-length segment. */
#define MT_OP_IS_EMPTY_INSERT(o)                                                      \
    (MT_OP_TYPE(o) == MT_OP_INSERT && !((o).flags & (MT_F_PROPS | MT_F_MARKER)) &&    \
     (o).payload_len <= MT_OP_PAIRS_LEN(o))
#define MT_OP_IS_NOOP(o) (MT_OP_TYPE(o) == MT_OP_NOOP || MT_OP_IS_EMPTY_INSERT(o))
/* An editing client.  A record with seq = MT_SEQ_LOCAL is a local edit of the
 * document's editing client (insertSegmentLocal / removeRangeLocal / annotateRangeLocal,
 * client.ts:163-214): INSERT / REMOVE / ANNOTATE at positions of its local view, applied at once
 * with refSeq = its currentSeq (ref_seq and msn are ignored), no window asserts, no seq update.
 * The first such record names the document's editing client (its `client`); from then on that
 * client's sequenced records are its acks (client.ts:804-806 -> ackPendingSegment,
 * mergeTree.ts:1893-1920): each settles the oldest pending edit and then updates the window.
 * Remote ops see the pending segments as the reference does (nodeLength, breakTie,
 * blockInsert's continuePredicate, pending property keys).  Such a document runs on the LDS
 * engine's editing form (in LDS up to MT_LOC_CAP = 1024 segments, then with its structure in an HBM
 * workspace at 2048 / 4096 / 8192; past 64 pending edits at once the workspace form with 256
 * pending-edit slots, for good; at most 8192 segments and 512 pending edits; beyond:
 * MT_DERR_CAPACITY); its delta events include the local edits' callbacks (seq -1). */
#define MT_SEQ_LOCAL (-1)
/* Reconnect (Client.regeneratePendingOp, client.ts:708-766, 855-893): a record with seq =
 * MT_SEQ_REGEN from the editing client holds the pending op to regenerate (the oldest one): its
 * segments, in document order, each at its findReconnectionPostition as of the edit's localSeq,
 * become new ops (a removal only while the segment is still locally removed), each with a new
 * pending group at the queue's tail.  The new ops are read with mt_regen_drain. */
#define MT_SEQ_REGEN (-2)
/* An op record whose message deli did not send (nacked, dropped, deferred or never sent; the fused
 * hand-off of mt_deli_ticket_device stamps it).  Any seq below MT_SEQ_REGEN is such a record: it is
 * never a local edit, and the apply engine halts the document on it with MT_DERR_SEQ_ORDER
 * ("Incoming remote op sequence# <= local collabWindow's currentSequence#", client.ts:461-462). */
#define MT_SEQ_NACK (-3)

typedef struct mt_op_rec {
    int32_t seq;          /* sequenceNumber                     (protocol.ts:132-172)           */
    int32_t ref_seq;      /* referenceSequenceNumber                                            */
    int32_t msn;          /* minimumSequenceNumber                                              */
    uint16_t client;      /* per-document short client id (observer = 0, never in ops)          */
    uint8_t type;         /* mt_op_type                                                         */
    uint8_t flags;        /* mt_op_flags | npairs << MT_F_NPAIRS_SHIFT                          */
    int32_t pos1;         /* insert position / range start                                      */
    int32_t pos2;         /* range end (remove, annotate)                                       */
    uint32_t payload_off; /* byte offset into the batch payload                                 */
    uint32_t payload_len; /* text bytes + 2*npairs: [text][key u8, value u8]*; value 0 = null
                             (MT_OP_WIDE: 2 * text units + 3 * npairs)                            */
} mt_op_rec;

/* NonCollabClient (constants.ts:15): the client of a segment loaded from a snapshot below the
 * MSN (snapshotLoader.ts:107-114); canonical state and checksum report it as -2 */
#define MT_CLIENT_NONCOLLAB 0xFE

/* ---- limits of the device representation (checked; violations become per-doc errors) ------
 * A NARROW document (every document starts narrow) holds short client ids < 64 (overlap sets as a
 * u64 bitmask), keys < 8 with u8 value ids and one byte per text code unit (Latin-1): the register
 * engine's and the LDS engine's fast forms.  A WIDE document (promoted for good by its first wide
 * op, client id >= 64 or wide snapshot segment) holds client ids < 65535 (u16; 254 = 0xFE is
 * NonCollabClient, so a host interning more than 253 clients skips it), keys < 32 with u16 value
 * ids, UTF-16 text (2 bytes per code unit in the same arena: half the units), and overlap sets of
 * the ids < 64 plus up to MT_OVX_IDS ids >= 64 per segment.  Wide
 * documents run on the LDS engine's wide form (its structure in an HBM workspace); their extra
 * per-segment state (122 B) is allocated by the engine on first need.  Value ids are opaque
 * (equality only) and may be interned per key. */
#define MT_MAX_CLIENTS 64      /* narrow: short client ids 0..63 (overlap set is a u64 bitmask)  */
#define MT_MAX_KEYS 8          /* narrow: property keys per document (u8 value id per key)      */
#define MT_MAX_VALUES 255      /* narrow: property value ids 1..255 (0 = absent/null)           */
#define MT_MAX_CLIENTS_WIDE 65535 /* wide: short client ids 1..65534, except 254 (NonCollabClient) */
#define MT_MAX_KEYS_WIDE 32    /* wide: property keys 0..31                                      */
#define MT_MAX_VALUES_WIDE 65535 /* wide: property value ids 1..65535 per key                    */
#define MT_OVX_IDS 32          /* wide: overlapping removers with ids >= 64 per segment          */
#define MT_MAX_TEXTCAP (64u << 20) /* text arena bytes per document half (mt_cfg.text_capacity)       */

typedef enum mt_status {
    MT_OK = 0,
    MT_ERR_ARG = 1,
    MT_ERR_HIP = 2,
    MT_ERR_NOMEM = 3,
    MT_ERR_STATE = 4,
    MT_ERR_DOC = 5,         /* at least one document has a sticky error (see mt_doc_error) */
    MT_ERR_COMM = 6,        /* an RCCL call failed (mt_comm_*) */
    MT_ERR_WIDE = 7         /* the call's form cannot express the document (a deli checkpoint of a
                               document past client 63: mt_deli_get_checkpoint_wide) */
} mt_status;

/* per-document sticky error codes (mirror the reference's assert/throw sites) */
enum mt_doc_err {
    MT_DERR_NONE = 0,
    MT_DERR_SEQ_ORDER = 1,      /* "Incoming remote op sequence# <= local collabWindow's currentSequence#" client.ts:461-462 */
    MT_DERR_MSN_ORDER = 2,      /* "Incoming remote op minSequence# < local collabWindow's minSequence#"  client.ts:463-464 */
    MT_DERR_INSERT_FAILED = 3,  /* "MergeTree insert failed" mergeTree.ts:2210-2216                      */
    MT_DERR_CAPACITY = 4,       /* segment/block/heap capacity of the device representation exceeded    */
    MT_DERR_TEXT_ARENA = 5,     /* per-document text arena exhausted                                    */
    MT_DERR_LIMITS = 6,         /* client id / property key / value id outside MT_MAX_* */
    MT_DERR_BAD_OP = 7,         /* malformed record (type, payload bounds, negative positions) */
    MT_DERR_EVENTS = 8          /* delta-event buffer of the document full (mt_events_enable): the
                                   document halts rather than drop callbacks                   */
};

typedef struct mt_cfg {
    int32_t device;             /* HIP device ordinal                                             */
    uint32_t max_docs;          /* documents this engine can hold                                 */
    uint32_t seg_capacity;      /* max linked segments per document (device slot pool)            */
    uint32_t text_capacity;     /* text arena bytes per document                                  */
    uint32_t heap_capacity;     /* zamboni LRU heap entries per document                          */
    uint32_t ops_per_launch;    /* b: ops per document per kernel launch (0 = whole batch)        */
} mt_cfg;

typedef struct mt_engine mt_engine;
typedef struct mt_batch mt_batch;

/* seg_capacity: 0 = 2048; 2048 ... 65472 (else MT_ERR_ARG) -- the capacity classes go up to the
 * engine's seg_capacity (2048 / 4096 / 8192 / 16384 / 32768 / 65472 above the register classes:
 * 64 K - 64, as slot indices are u16) and every document's slot rows hold the largest one.
 * text_capacity: 0 = 64 KiB; at most MT_MAX_TEXTCAP (MT_ERR_ARG above).  Each document has two
 * halves of this size (compaction copies the live text into the other half); a zamboni append
 * copies its run to the top of the arena, so documents whose live text approaches the capacity
 * stop with MT_DERR_TEXT_ARENA -- size it at a few times the largest expected document. */
mt_status mt_engine_create(const mt_cfg* cfg, mt_engine** out);
mt_status mt_engine_destroy(mt_engine* eng);
/* documents started by the last mt_docs_init, and the engine's max_docs (either may be NULL) */
mt_status mt_engine_info(const mt_engine* eng, uint32_t* n_docs, uint32_t* max_docs);

/* Start `n_docs` empty documents: Client + startOrUpdateCollaboration(observer, 0, 0)
 * (client.ts:1051-1071, mergeTree.ts:1254-1271). */
mt_status mt_docs_init(mt_engine* eng, uint32_t n_docs);

/* ---- snapshot load ---------------------------------------------------
 * One segment of a snapshot's header chunk (IJSONSegmentWithMergeInfo, snapshotChunks.ts:60-66,
 * after SnapshotLoader.specToSegment, snapshotLoader.ts:85-117): 96 bytes. */
typedef struct mt_load_seg {  /* 96 bytes */
    int32_t seq;          /* spec.seq, or UniversalSequenceNumber (0) without merge info            */
    int32_t rseq;         /* spec.removedSeq; -1 = not removed                                      */
    uint8_t client;       /* short id of spec.client, or MT_CLIENT_NONCOLLAB                        */
    uint8_t rclient;      /* short id of spec.removedClient (when removed)                          */
    uint8_t flags;        /* MT_SF_PDEF (2) when the spec carries props, MT_SF_MARKER (16) for a
                             Marker spec (text_len 1: its ReferenceType byte), MT_LSF_U16 (64):
                             the text is UTF-16 code units (2 bytes each, LE)  (mt_state.h)        */
    uint8_t pad;
    uint32_t text_off;    /* the segment's text: byte offset in the batch's text bytes              */
    uint32_t text_len;    /* code units (= bytes without MT_LSF_U16)                                */
    uint8_t client_hi;    /* high bytes of the short ids (a wide document's ids >= 256)             */
    uint8_t rclient_hi;
    uint16_t pad2;
    uint16_t props[MT_MAX_KEYS_WIDE]; /* value id per key (0 = absent)                               */
    uint64_t pad3;
} mt_load_seg;
#define MT_LSF_U16 64u

/* SnapshotLoader.loadHeader for documents doc_ids[0..n): MergeTree.reloadFromSegments (mergeTree.ts:
 * 1195-1251: the leaves in blocks of MaxNodesInBlock - 1 = 7, levels built bottom-up until one
 * block is left) then startOrUpdateCollaboration(id, min_seq[i], cur_seq[i]) (snapshotLoader.ts:
 * 138-154, client.ts:1051-1071; an empty LRU heap, every block's needsScour undefined).  Document
 * i's segments are segs[seg_row_ptr[i] .. seg_row_ptr[i+1]) in order; texts are byte ranges of
 * `text` (Latin-1, one byte per UTF-16 unit, or UTF-16 LE with MT_LSF_U16).  A document with any
 * segment beyond the narrow limits (UTF-16 text, key >= 8, value id >= 256, client id >= 64) loads
 * as a wide document.  Built on the device, one wave per document.
 * The body chunks (and catch-up ops) follow through mt_submit as MT_OP_LOAD records (and normal
 * ops).  A document over the engine's capacities gets MT_DERR_CAPACITY / MT_DERR_TEXT_ARENA. */
mt_status mt_docs_load(mt_engine* eng, uint32_t n, const uint32_t* doc_ids, const uint32_t* seg_row_ptr,
                       const mt_load_seg* segs, const uint8_t* text, uint64_t text_bytes, const int32_t* min_seq,
                       const int32_t* cur_seq);

/* Host -> device staging of a CSR op batch.  Ops are grouped by document (doc_row_ptr has
 * n_docs+1 entries) and seq-ascending within a document.  Buffers are caller-owned and copied
 * before return. */
mt_status mt_batch_upload(mt_engine* eng, const mt_op_rec* ops, uint64_t n_ops,
                          const uint8_t* payload, uint64_t payload_bytes,
                          const uint32_t* doc_row_ptr, mt_batch** out);
/* Apply a staged batch (asynchronous on the engine's stream; = applyMsg for every op). */
mt_status mt_batch_apply(mt_engine* eng, const mt_batch* batch);
mt_status mt_batch_free(mt_engine* eng, mt_batch* batch);
/* upload + apply + free (the synchronous drop-in for a loop of applyMsg calls) */
mt_status mt_submit(mt_engine* eng, const mt_op_rec* ops, uint64_t n_ops,
                    const uint8_t* payload, uint64_t payload_bytes, const uint32_t* doc_row_ptr);
/* (mt_submit with the upload overlapped: mt_submit_ticks, "tick-major feed" below) */
mt_status mt_sync(mt_engine* eng);

/* Readout (synchronises).  Text = MergeTreeTextHelper.getText for the observer, as UTF-16 code
 * units (2 bytes each, little endian; *len in bytes) -- the JS string, surrogate halves included. */
mt_status mt_get_length(mt_engine* eng, uint32_t doc, uint32_t* len);
mt_status mt_get_text(mt_engine* eng, uint32_t doc, char* buf, uint64_t cap, uint64_t* len);
/* Canonical state (JSON, see DESIGN.md "Canonical state"): L1 text, L2 linked leaves,
 * L3 block shape, currentSeq/minSeq.  ASCII JSON: non-ASCII code units as \uXXXX (here and in the
 * snapshot blobs: the same JSON values the reference's JSON.stringify writes). */
mt_status mt_get_state(mt_engine* eng, uint32_t doc, char* buf, uint64_t cap, uint64_t* len);
/* Per-document 64-bit checksum of the canonical state (DESIGN.md "Checksum"). */
mt_status mt_checksums(mt_engine* eng, uint64_t* out, uint32_t n_docs);
/* The same into device memory (HBM, n_docs u64), complete on return. */
mt_status mt_checksums_device(mt_engine* eng, uint64_t* d_out, uint32_t n_docs);
mt_status mt_doc_error(mt_engine* eng, uint32_t doc, int32_t* code, int32_t* seq);

/* Measurement hooks for bench.py, for the last mt_batch_apply: kernel_ms = sum of the apply
 * kernels' durations (HIP events bracketing each launch on the engine stream), wall_ms = first
 * to last event (incl. binning and the per-tick host sync), launches = apply kernels issued,
 * alg_bytes = algorithmic bytes they move (DESIGN.md "Roofline accounting"). */
mt_status mt_last_apply_stats(mt_engine* eng, float* kernel_ms, float* wall_ms, uint32_t* launches,
                              uint64_t* alg_bytes);
/* Capacity classes of one tick run concurrently on their own streams (on = 1, the default; the
 * environment variable MTGPU_SERIAL=1 starts an engine with 0) or one after another on the
 * engine stream (on = 0: each class kernel has the GPU to itself, for per-kernel rooflines). */
mt_status mt_set_concurrent_classes(mt_engine* eng, int on);
/* The same, per capacity class (cls = 0, 1, ... for 128, 192, 256 ... 1024 segments in steps of 64,
 * then 2048 / 4096 / 8192 / 16384 / 32768 / 65472, then one entry for the editing documents' bucket, whose capacity
 * reads MT_CLASS_EDITING | MT_LOC_CAP, then one per register class for the documents the LDS engine
 * runs at that capacity (declared label keys), reading MT_CLASS_LDS | capacity, then one per register
 * class for the documents with client ids above 32 (the register engine's 64-bit overlap form),
 * reading MT_CLASS_C64 | capacity, then the editing form's other sizes, MT_CLASS_EDITING | 256 / 512
 * (LDS) and | 2048 / 4096 (HBM workspace), then MT_CLASS_EDITING | MT_CLASS_GROUPS | 1024 / 4096 (the
 * HBM-workspace form with 512 pending-edit slots), then the wide form per class from the 256 class on
 * (staged in LDS up to 512 segments, in an HBM workspace above), MT_CLASS_WIDE | capacity; MT_ERR_ARG
 * past the last): each class is one kernel instantiation (see
 * mt_class_kernel_name). */
#define MT_CLASS_EDITING 0x40000000u
#define MT_CLASS_GROUPS 0x08000000u  /* with MT_CLASS_EDITING: the form for more than 64 pending edits */
#define MT_CLASS_LDS 0x20000000u
#define MT_CLASS_C64 0x10000000u
#define MT_CLASS_WIDE 0x04000000u  /* the wide form (include/mtgpu.h "limits") */
mt_status mt_last_apply_class_stats(mt_engine* eng, uint32_t cls, uint32_t* capacity, float* kernel_ms,
                                    uint32_t* launches, uint64_t* alg_bytes);
/* Kernel symbol (as a rocprof trace names it) that applies documents of capacity class
 * `capacity` on this engine: the register engine for <= 1024 segments, else the LDS engine; with
 * MT_CLASS_C64 the register engine's 64-bit overlap form, MT_CLASS_LDS / MT_CLASS_EDITING the LDS
 * engine at that capacity / its editing form. */
mt_status mt_class_kernel_name(mt_engine* eng, uint32_t capacity, char* buf, uint64_t cap);
/* Snapshot of one document: what `new SnapshotV1(mergeTree).extractSync()`
 * + `emit()` write (packages/dds/merge-tree/src/snapshotV1.ts:85-247) -- the segments below the
 * MSN coalesced (canAppend + matchProperties), the others with their merge info -- as one JSON
 * object {"header": chunk, "body_0": chunk, ...} of the emitted tree's blobs.  The extraction
 * decisions run on the device (mt_service.hip); the JSON is written on the host.  chunk_size =
 * mergeTreeSnapshotChunkSize (0: 10000).  client_names[short id] = long client id (NULL or a
 * short table: the short id in decimal).  Props are written as {"k<key id>": value id} (ids as
 * interned by the host; JSON key order is key-id order, the reference's is insertion order). */
mt_status mt_get_snapshot(mt_engine* eng, uint32_t doc, uint32_t chunk_size, const char* const* client_names,
                          uint32_t n_names, char* buf, uint64_t cap, uint64_t* len);
/* The same for documents [d0, d0+n) at once (a summary of many documents): one extraction launch,
 * one copy per state array, the JSON written on all host cores.  Document d0+i's object is
 * buf[offsets[i] .. offsets[i+1]) (offsets: n+1 entries, no separators, no NUL).  Call once with
 * buf = NULL for the sizes (the result is kept), then with a buffer of offsets[n] bytes. */
mt_status mt_get_snapshots(mt_engine* eng, uint32_t d0, uint32_t n, uint32_t chunk_size, const char* const* client_names,
                           uint32_t n_names, char* buf, uint64_t cap, uint64_t* offsets);
/* Run the device extraction for documents [d0, d0+n) (all docs of a summary in one launch);
 * reports the kernel time and the number of segment specs produced (bench tooling). */
mt_status mt_snapshot_extract(mt_engine* eng, uint32_t d0, uint32_t n, float* kernel_ms, uint64_t* n_specs);
/* Segment count of every document (after sync). */
mt_status mt_seg_counts(mt_engine* eng, uint32_t* out, uint32_t n_docs);

/* ---- findTile (tiles) ------------------------------------------------
 * Client.findTile(startPos, tileLabel, preceding) (client.ts:1073-1076 -> MergeTree.findTile,
 * mergeTree.ts:1763-1789) for a batch of queries, in the document's local view: preceding = 1
 * (search, :1793-1829): the last live tile at a position <= pos; preceding = 0 (backwardSearch,
 * :1831-1870): none past the length; else the leaf the search stops on (the last segment starting
 * at or before pos -- removed or not -- unless a trailing empty leaf block comes after it) if that
 * is a tile, otherwise the first live tile after it.  A tile is a Marker whose refType has Tile
 * (ops.ts:8) and whose "referenceTileLabels" property (key id `key` of the document) holds the
 * label; the host passes the label as the set of value ids whose label arrays contain it.
 * The reference answers through HierMergeBlock caches (rightmostTiles / leftmostTiles,
 * mergeTree.ts:263-318) that blockUpdate rebuilds whenever a block's children change -- inserts,
 * boundary splits, removes (every block the removal's mapRange enters), zamboni scours that unlink
 * or append, packs, acks -- but annotateRange does not (mergeTree.ts:2565-2605): a tile found by
 * shifting over a block answers with the labels its markers had at that block's last rebuild, a tile
 * in the leaf block of the search path with its current labels.  The engine reproduces this for the
 * documents whose label keys the host declared (mt_set_label_keys): a marker annotated since its leaf
 * block's last rebuild keeps the tile / range label value ids it had then (a "stale" marker), and the
 * queries read those outside the search path's leaf block.  Without declared keys the engine
 * answers from the current labels. */
typedef struct mt_tile_query {  /* 48 bytes */
    uint32_t doc;
    int32_t pos;                /* startPos */
    uint8_t key;                /* key id of "referenceTileLabels" in this document (>= 16: no tiles) */
    uint8_t preceding;
    uint8_t pad[2];
    uint32_t vmask[8];          /* bit v: value id v's label array holds the label */
    uint32_t pad2;
} mt_tile_query;
typedef struct mt_tile_result {
    int32_t pos;                /* the tile's local position (getPosition), -1: none */
    int32_t ordinal;            /* its index among the document's segments, -1: none */
} mt_tile_result;
/* (vmask covers value ids 0..255 of the label key: a host interning that key's values past 255
 * refuses the query, so a label never goes unmatched silently) */
mt_status mt_find_tiles(mt_engine* eng, const mt_tile_query* q, uint32_t n, mt_tile_result* out);

/* ---- position queries (SURVEY.md §8(b) read surface) -------------------------------------------
 * MergeTree.getContainingSegment(pos, refSeq, clientId) (mergeTree.ts:1623-1634 through searchBlock,
 * :1797-1829; Client.getContainingSegment client.ts:1004-1007 uses the local view) and
 * MergeTree.getPosition(segment, currentSeq, own client) (mergeTree.ts:1585-1602; Client.getPosition
 * client.ts:290-292) for a batch of queries, one wave per query over the document's state in HBM:
 *   MT_POS_CONTAINING: the first segment whose view length exceeds what is left of pos (pos minus the
 *     view lengths of the segments before it) -- for pos < 0 the first segment, for pos past the
 *     view's length none (ordinal -1); offset = pos minus the view length before it;
 *   MT_POS_OF_ORDINAL: the segment of ordinal `pos` (its index among the linked segments).
 * With no such segment: ordinal -1, offset = pos minus the view's whole length, position = the
 * local view's whole length (resolveRemoteClientPosition's end-of-view case, mergeTree.ts:2105-2127). 
 * The view is (ref_seq, client) -- nodeLength's leaf branch, mergeTree.ts:1659-1697 -- or, with
 * ref_seq = MT_POS_LOCAL, the local view (a removed segment has length 0; an editing client's
 * pending inserts count): Client's own reads.  position is always the local view's (getPosition). */
#define MT_POS_CONTAINING 0u
#define MT_POS_OF_ORDINAL 1u
#define MT_POS_LOCAL INT32_MIN
typedef struct mt_pos_query {   /* 16 bytes */
    uint32_t doc;
    int32_t pos;                /* a position in the view, or an ordinal (MT_POS_OF_ORDINAL) */
    int32_t ref_seq;            /* the view's refSeq, or MT_POS_LOCAL */
    uint16_t client;            /* the view's short client id (ignored for MT_POS_LOCAL) */
    uint16_t kind;              /* MT_POS_CONTAINING / MT_POS_OF_ORDINAL */
} mt_pos_query;
typedef struct mt_pos_result {  /* 16 bytes */
    int32_t ordinal;            /* the segment's index among the linked segments, -1: none */
    int32_t offset;             /* MT_POS_CONTAINING: pos relative to the segment's start in the view */
    int32_t position;           /* the segment's local-view position (getPosition) */
    uint32_t length;            /* its cachedLength */
} mt_pos_result;
mt_status mt_resolve_positions(mt_engine* eng, const mt_pos_query* q, uint32_t n, mt_pos_result* out);
/* the same with device-resident queries and results (no copies, no synchronisation beyond the stream);
 * a query the host could not check -- doc >= n_docs or an unknown kind -- gets ordinal
 * MT_POS_BAD_QUERY instead of an answer */
#define MT_POS_BAD_QUERY (-2)
mt_status mt_resolve_positions_device(mt_engine* eng, const mt_pos_query* d_q, uint32_t n, mt_pos_result* d_out);

/* One segment's fields, by ordinal, for a batch of (document, ordinal) pairs (a reader that holds a
 * segment found by mt_resolve_positions, e.g. Client.getPropertiesAtPosition client.ts:1009-1023):
 * one small gather kernel and one copy, not a whole-document read.  ordinal past the document's
 * segments: seq = INT32_MIN.  Text: mt_segment_text. */
typedef struct mt_seg_info {    /* 168 bytes */
    int32_t seq;                /* INT32_MIN: no such segment */
    int32_t rseq;               /* removedSeq, -1: not removed */
    int32_t client;             /* short client id; -2 = NonCollabClient (constants.ts:15) */
    int32_t rclient;            /* removedClientId, -1: not removed */
    uint32_t len;               /* cachedLength (UTF-16 code units) */
    uint32_t flags;             /* MT_SF_* of mt_state.h: 1 removed, 2 properties defined, 16 marker */
    uint32_t toff;              /* its text in the document's arena (code units) */
    uint32_t wide;              /* 1: a wide document (UTF-16 arena) */
    uint64_t overlap;           /* removedClientOverlap: bit c for ids c < 64 */
    uint16_t props[MT_MAX_KEYS_WIDE]; /* value id per key (0: absent) */
    uint16_t overlap_hi[MT_OVX_IDS]; /* a wide document's overlapping removers >= 64, ascending (0: none) */
} mt_seg_info;
mt_status mt_segment_infos(mt_engine* eng, const uint32_t* docs, const int32_t* ordinals, uint32_t n, mt_seg_info* out);
/* a segment's text: `len` code units of document doc's arena at `toff` (from mt_seg_info) */
mt_status mt_segment_text(mt_engine* eng, uint32_t doc, uint32_t toff, uint32_t len, uint16_t* out);

/* The ops document `doc` regenerated at its MT_SEQ_REGEN records since the last drain (at most 256
 * records / 4 KiB of payload between drains, else MT_DERR_CAPACITY): per regenerated op one
 * MT_OP_NOOP header record whose seq is the index of the resetting record within the document's
 * records, then the new ops (mt_op_rec, payload offsets into `payload`: an insert carries its text
 * or refType byte and its props, F_PROPS when its properties are defined; an annotate the reset
 * op's props).  *n / *pn: records / payload bytes available; with recs != NULL the buffer is
 * drained -- all of it: with cap < *n or pcap < *pn nothing is copied or cleared (MT_ERR_ARG). */
mt_status mt_regen_drain(mt_engine* eng, uint32_t doc, mt_op_rec* recs, uint32_t cap, uint8_t* payload, uint32_t pcap,
                         uint32_t* n, uint32_t* pn);

/* ---- range stacks -----------------------------------------------------
 * Client.getStackContext(startPos, [rangeLabel]) (client.ts:946-948 -> MergeTree.getStackContext,
 * mergeTree.ts:1750-1760) for a batch of (document, position, label) queries in the local view: the
 * live range markers (refType NestBegin | NestEnd, ops.ts:8) whose "referenceRangeLabels" property
 * (key id `q.key`) holds the label, at positions <= pos (the shifted ones and the leaf holding pos),
 * folded in document order by applyRangeReference (mergeTree.ts:246-261: NestBegin pushes; an end
 * pops a NestBegin top and is pushed otherwise).  The stack is therefore its unmatched ends followed
 * by its unmatched begins.  Query i's stack, bottom to top, goes to items[i*cap ...] (at most cap
 * entries) and its full depth to depth[i] & MT_STACK_DEPTH; MT_STACK_TOUCHED is set when any such
 * marker was folded (the reference's RangeStackMap then holds the label, possibly with an empty
 * stack; otherwise the label is absent).  q.preceding is ignored.  Like findTile, the reference
 * folds HierMergeBlock rangeStacks caches that annotateRange does not refresh; with declared label
 * keys the engine folds the markers of other leaf blocks with their labels as of their block's last
 * rebuild, as findTile does. */
#define MT_STACK_DEPTH 0x7FFFFFFFu
#define MT_STACK_TOUCHED 0x80000000u
typedef struct mt_stack_item {  /* 12 bytes */
    int32_t pos;                /* the marker's local position (getPosition) */
    int32_t ordinal;            /* its index among the document's segments */
    uint32_t ref_type;          /* its refType */
} mt_stack_item;
mt_status mt_range_stacks(mt_engine* eng, const mt_tile_query* q, uint32_t n, uint32_t cap, mt_stack_item* items,
                          uint32_t* depth);

/* Declare the key ids of "referenceTileLabels" (tile_key) and "referenceRangeLabels" (range_key) in
 * document `doc` (MT_ALL_DOCS: every document), -1 for a key the document does not use.  From then on
 * the engine tracks the reference's block caches for those labels (see findTile above); the host calls
 * it when it interns either key for a document, before submitting the op that first carries it (-1
 * leaves a key as it is, so the two may be declared by separate calls).  A document with declared keys
 * runs on the LDS engine (at its capacity class's size).  A key is declared once per document: declaring it again as a different id
 * returns MT_ERR_ARG. */
#define MT_ALL_DOCS 0xFFFFFFFFu
mt_status mt_set_label_keys(mt_engine* eng, uint32_t doc, int tile_key, int range_key);

/* ---- delta / maintenance events -------------------------------------
 * What Client.mergeTreeDeltaCallback and mergeTreeMaintenanceCallback receive
 * (mergeTreeDeltaCallback.ts:15-73), fired synchronously inside applyMsg at mergeTree.ts:1981-1988
 * (INSERT), 2705-2712 (REMOVE: the segments this op removed, not the overlapping ones),
 * 2592-2600 (ANNOTATE, with propertyDeltas), 2231-2236 (SPLIT), 1335-1340 (APPEND), 1310-1315
 * (UNLINK).  The engine records them per document, in firing order, one mt_event per delta
 * segment (a callback with no delta segments -- a remove that only overlapped -- is one record
 * flagged MT_EVF_EMPTY).  Segments are identified by position, not object identity:
 *   leaf = ordinal of the segment among the leaves still linked at callback time (document order;
 *          for SPLIT the second segment is not linked yet: leaf of the first + 1; -1 = not linked,
 *          the zero-length insert of an empty text with props),
 *   pos  = op callbacks: local-view position (characters of unremoved linked leaves before it);
 *          maintenance callbacks: -1,
 *   len  = segment.cachedLength at callback time (APPEND: the first segment's grown length).
 * ANNOTATE records carry propertyDeltas as a key mask + the previous value id per key (0 =
 * null: the key was absent).  Recording routes every document to the LDS engine (wide documents:
 * its wide form). */
enum mt_event_op {
    MT_EV_INSERT = 0, MT_EV_REMOVE = 1, MT_EV_ANNOTATE = 2,   /* MergeTreeDeltaType (ops.ts:17-24)   */
    MT_EV_APPEND = -1, MT_EV_SPLIT = -2, MT_EV_UNLINK = -3    /* MergeTreeMaintenanceType            */
};
#define MT_EVF_FIRST 1u   /* first record of a callback */
#define MT_EVF_NOPD 4u  /* ANNOTATE delta segment whose propertyDeltas is undefined (a remote annotate
                         dropped while the editing client's rewrite is pending) */
#define MT_EVF_EMPTY 2u   /* the callback's deltaSegments is empty (no segment in this record) */
typedef struct mt_event {   /* 96 bytes */
    int32_t seq;            /* sequenceNumber of the message being applied                        */
    int8_t op;              /* mt_event_op                                                        */
    uint8_t flags;          /* MT_EVF_*                                                           */
    uint16_t pad;
    int32_t leaf;
    int32_t pos;
    uint32_t len;
    uint32_t pmask;         /* ANNOTATE: keys present in propertyDeltas (bit k = key id k)        */
    uint16_t pvals[MT_MAX_KEYS_WIDE]; /* ANNOTATE: previous value id of key k (0 = null)          */
    uint64_t pad2;
} mt_event;
/* Start recording: `per_doc` records per document between drains (0 stops recording).  A
 * document that would exceed it halts with MT_DERR_EVENTS. */
mt_status mt_events_enable(mt_engine* eng, uint32_t per_doc);
/* Move every document's recorded events to the host (synchronises) and clear them: document d's
 * records are out[row_ptr[d] .. row_ptr[d+1]) (row_ptr: n_docs + 1 entries).  With out == NULL
 * (or cap too small: MT_ERR_ARG) only row_ptr / *total are filled and nothing is cleared. */
mt_status mt_events_drain(mt_engine* eng, mt_event* out, uint64_t cap, uint32_t* row_ptr, uint64_t* total);

/* ---- bench tooling (not part of the applyMsg boundary) -------------------------------------
 * Synthetic multi-client op streams (DESIGN.md "Synthetic workloads", after SURVEY.md §8d),
 * generated ON THE DEVICE straight into HBM: every document's observer state drives the
 * positions of its next op, so each op is valid for what its client had seen.  The engine's
 * documents are left in the post-generation state (call mt_docs_init to replay from empty). */
typedef struct mt_synth_cfg {
    uint32_t seed;
    uint32_t n_clients;      /* remote clients 1..n_clients (< MT_MAX_CLIENTS)              */
    uint32_t ops_per_doc;
    uint32_t max_lag;        /* refSeq lag U[0, max_lag] behind the latest seq               */
    uint32_t stall_ops;      /* >0: client 1 holds its refSeq for stretches of this many ops */
    uint32_t n_keys;         /* property keys used by annotate / insert props (<= 8)         */
    uint32_t n_values;       /* property value ids 1..n_values (<= 255)                      */
    uint32_t p_insert, p_remove;  /* probabilities as fixed point p * 2^32; rest = annotate   */
    uint32_t p_overlap;      /* a remove aims at a segment removed concurrently, still visible */
    uint32_t p_null;         /* annotate value null = delete the key                         */
    uint32_t p_rewrite;      /* annotate with combiningOp "rewrite"                          */
    uint32_t p_insert_props; /* insert carries a props object                                */
    uint32_t p_marker;       /* an insert is a Marker (refType Tile, NestBegin or NestEnd)    */
} mt_synth_cfg;

/* doc_id_base: global id of the engine's document 0 (a rank's shard of a multi-GPU job) */
mt_status mt_synth_generate(mt_engine* eng, const mt_synth_cfg* cfg, uint32_t doc_id_base, uint32_t payload_per_doc,
                            mt_batch** out);
/* The same with an explicit global id per engine document (host array of n_docs ids): a rank's
 * hash-routed shard of a multi-GPU job (mt_route_docs). */
mt_status mt_synth_generate_ids(mt_engine* eng, const mt_synth_cfg* cfg, const uint32_t* doc_ids,
                                uint32_t payload_per_doc, mt_batch** out);
/* Copy documents [d0, d1) of a staged batch to the host: ops (payload_off rebased so the
 * first copied document's payload region starts at 0), payload and row_ptr (d1-d0+1 entries).
 * Sizes for a dry run: pass NULL buffers. */
mt_status mt_batch_copy_docs(mt_engine* eng, const mt_batch* batch, uint32_t d0, uint32_t d1, mt_op_rec* ops,
                             uint64_t* n_ops, uint8_t* payload, uint64_t* payload_bytes, uint32_t* row_ptr);
/* algorithmic bytes of a batch's ops + payload (for the roofline accounting in bench.py) */
mt_status mt_batch_info(const mt_batch* batch, uint64_t* n_ops, uint64_t* payload_bytes, uint32_t* max_ops_per_doc);
/* device pointers of a staged batch (to chain device-side stages, e.g. deli -> apply) */
mt_status mt_batch_device_ptrs(const mt_batch* batch, mt_op_rec** ops, uint8_t** payload, uint32_t** row_ptr);

const char* mt_version(void);

/* ---- multi-GPU: document routing and the end-of-run gather -----------------
 * Documents are independent; the reference partitions by documentId (Kafka key,
 * server/routerlicious/packages/services/src/kafkaNodeProducer.ts:131,156; lambda routing
 * lambdas-driver/src/document-router/documentLambda.ts:52-58).  Here document docId lives on GPU
 * splitmix64(docId) mod n_gpus (mt_route_doc), with no collective in the apply loop; one process
 * per GPU.  RCCL (over xGMI) is used only for the final per-document checksum gather. */
uint32_t mt_route_doc(uint64_t doc_id, uint32_t n_shards);
mt_status mt_route_docs(const uint64_t* doc_ids, uint64_t n, uint32_t n_shards, uint32_t* shard_out);

#define MT_COMM_ID_BYTES 128
typedef struct mt_comm mt_comm;
/* rank 0 makes the id, every rank passes the same bytes to mt_comm_create (ncclUniqueId) */
mt_status mt_comm_unique_id(uint8_t* id /* [MT_COMM_ID_BYTES] */);
mt_status mt_comm_create(int32_t device, int32_t rank, int32_t n_ranks, const uint8_t* id, mt_comm** out);
mt_status mt_comm_destroy(mt_comm* comm);
/* Gather every rank's per-document checksums (mt_checksums of `eng`) to rank 0: ncclGather from
 * HBM.  Rank 0: out[r * max_docs_per_rank + i] = rank r's document i, counts[r] = rank r's
 * n_docs (other ranks may pass NULL).  Every rank that passes the argument checks enters the
 * gather: one whose own part fails (more documents than max_docs_per_rank, the checksum kernel)
 * sends a poisoned row and returns its error, and rank 0 returns MT_ERR_COMM; a rank that cannot
 * allocate its row aborts the communicator (best effort). */
mt_status mt_comm_gather_checksums(mt_comm* comm, mt_engine* eng, uint32_t max_docs_per_rank, uint64_t* out,
                                   uint32_t* counts);
/* max over ranks (the job's clock), and a barrier (all-reduce + device synchronize) */
mt_status mt_comm_allreduce_max_f64(mt_comm* comm, double* v);
mt_status mt_comm_barrier(mt_comm* comm);

/* ---- deli: per-document sequence-number / MSN ticketing ----------------
 * Replaces, for many documents at once, the ordering service's per-document sequencer:
 *   DeliLambda.ticket(rawMessage)        server/routerlicious/packages/lambdas/src/deli/lambda.ts:255-544
 *   DeliLambda.handler's lastSentMSN     lambda.ts:173-246 (lastSentMSN = msn of every sent or nacked ticket)
 *   ClientSequenceNumberManager          deli/clientSeqManager.ts:70-143 (upsert/remove/min refSeq)
 *   new DeliLambda(.., lastCheckpoint)   lambda.ts:112-171 (clients + sequenceNumber from IDeliState)
 * Raw messages arrive grouped by document (CSR row_ptr, each document's messages in log order);
 * client ids are per-document short ids 0..511 interned by the host (the reference keys clients by
 * their long id string).  One output ticket per raw message.  Out of scope: branch Integrate
 * messages, idle-client eviction and NoClient/idle timers (they only enqueue new raw messages back
 * to the ordering service, which a host feeds in as MT_RAW_LEAVE / MT_RAW_SERVER_NOOP), summarize
 * scopes (every client may summarize), traces, DSN bookkeeping of Control messages. */
typedef enum mt_raw_kind {
    MT_RAW_OP = 0,          /* client op (Operation, Summarize, ...): revs seq        lambda.ts:414-435 */
    MT_RAW_NOOP = 1,        /* client NoOp, contents null: consolidated later       lambda.ts:463-465 */
    MT_RAW_NOOP_DATA = 2,   /* client NoOp with contents: revs only if the msn moved lambda.ts:466-471 */
    MT_RAW_JOIN = 3,        /* ClientJoin of `client` (system message)              lambda.ts:286-299 */
    MT_RAW_LEAVE = 4,       /* ClientLeave of `client`                              lambda.ts:281-285 */
    MT_RAW_SERVER_NOOP = 5, /* server NoOp: revs if the msn moved, else never sent  lambda.ts:473-479 */
    MT_RAW_NOCLIENT = 6,    /* NoClient: revs (ref = msn = seq) when nobody joined  lambda.ts:481-489 */
    MT_RAW_CONTROL = 7      /* Control: never sent, never revs                      lambda.ts:490-517 */
} mt_raw_kind;

typedef struct mt_raw_msg {  /* 16 bytes */
    int32_t csn;             /* operation.clientSequenceNumber                                     */
    int32_t ref_seq;         /* operation.referenceSequenceNumber; -1 = REST op (revved to its seq) */
    uint16_t client;         /* short id of the sending client, or of the joiner / leaver
                                (< MT_DELI_MAX_CLIENTS)                                              */
    uint8_t kind;            /* mt_raw_kind                                                        */
    uint8_t pad;
    uint32_t op_index;       /* fused hand-off (mt_deli_ticket_device with d_ops): 1 + index of the op
                                record this message carries, 0 = none (joins, leaves, no-ops)     */
} mt_raw_msg;

typedef enum mt_ticket_status {
    MT_TK_DROPPED = 0,      /* ticket() returns nothing: duplicate csn (lambda.ts:267-268), join of a
                               joined client (:295-298), leave of an absent one (:283-285)          */
    MT_TK_SENT = 1,         /* sequenced and sent (SendType.Immediate)                              */
    MT_TK_LATER = 2,        /* SendType.Later: a consolidated client no-op                          */
    MT_TK_NEVER = 3,        /* SendType.Never                                                       */
    MT_TK_NACK_GAP = 4,     /* "Gap detected in incoming op"              lambda.ts:269-275, 613-620 */
    MT_TK_NACK_CLIENT = 5,  /* "Nonexistent client" (never joined, left, or nacked) lambda.ts:309-316 */
    MT_TK_NACK_REFSEQ = 6,  /* "Refseq r < msn"; the client stays nacked          lambda.ts:319-335 */
    MT_TK_HALTED = 7        /* the document stopped at an earlier error (mt_deli_doc_error)         */
} mt_ticket_status;

typedef struct mt_ticket {  /* 16 bytes */
    int32_t seq;            /* sequenceNumber of the output message (a nack: the msn it carries)   */
    int32_t msn;            /* minimumSequenceNumber of the output message                         */
    int32_t ref_seq;        /* referenceSequenceNumber as sequenced (REST -1 and NoClient: = seq)  */
    uint8_t status;         /* mt_ticket_status                                                    */
    uint8_t pad[3];
} mt_ticket;

/* Client ids: a document holds short ids 0..MT_DELI_MAX_CLIENTS-1.  Up to id 63 it is ticketed eight
 * documents per wave; its first message from a client >= 64 promotes it, for good, to the wide form
 * (one document per wave, its clients in a row of the deli's big pool, MT_DELI_BIG_CLIENTS per row:
 * one row per 16 documents of max_docs, at least 64), and its first from a client >= 512 to the huge
 * form (a row of MT_DELI_MAX_CLIENTS clients in the huge pool: one row per 256 documents, at least 8).
 * mt_deli_restore / mt_deli_restore_wide give a restored document's rows back to the pools (free lists
 * the next promotion takes first), mt_deli_restore_all empties them.  The reference keeps a Map and a
 * heap (clientSeqManager.ts:70-143, joins at lambda.ts:280-306): no limit. */
#define MT_DELI_BIG_CLIENTS 512
#define MT_DELI_MAX_CLIENTS 4096

/* per-document sticky deli errors (the reference lambda throws / has no representation) */
typedef enum mt_deli_err {
    MT_DELI_OK = 0,
    MT_DELI_ERR_CLIENT = 1, /* short client id >= MT_DELI_MAX_CLIENTS                               */
    MT_DELI_ERR_KIND = 2,   /* unknown mt_raw_kind                                                  */
    MT_DELI_ERR_ASSERT = 3, /* assert(refSeq >= msn) lambda.ts:426-428 (a client no-op with ref -1) */
    MT_DELI_ERR_CAPACITY = 4 /* a client >= 64 needed a big-pool row and none was left (a capacity
                               limit of this engine, not an error of the stream)                    */
} mt_deli_err;

typedef struct mt_deli_client {
    int32_t csn;            /* clientSequenceNumber (IClientSequenceNumber)                         */
    int32_t ref_seq;        /* referenceSequenceNumber                                              */
    uint8_t joined;         /* tracked by the ClientSequenceNumberManager                           */
    uint8_t nack;           /* nacked: every later message of this client is nacked                 */
    uint8_t pad[2];
} mt_deli_client;

typedef struct mt_deli_checkpoint {  /* IDeliState (lambda.ts:754-764), device-representable part */
    int32_t seq;            /* sequenceNumber                                                       */
    int32_t msn;            /* minimumSequenceNumber (read back; derived on restore, lambda.ts:166-167) */
    int32_t last_sent_msn;  /* lastSentMSN (0 for a freshly constructed lambda, lambda.ts:103)      */
    int32_t err;            /* mt_deli_err (read back; ignored on restore)                          */
    mt_deli_client clients[MT_MAX_CLIENTS];
} mt_deli_checkpoint;

typedef struct mt_deli_checkpoint_wide {  /* the same with every client slot (documents past client 63) */
    int32_t seq;
    int32_t msn;
    int32_t last_sent_msn;
    int32_t err;
    mt_deli_client clients[MT_DELI_MAX_CLIENTS];
} mt_deli_checkpoint_wide;

typedef struct mt_deli mt_deli;
mt_status mt_deli_create(int32_t device, uint32_t max_docs, mt_deli** out);
mt_status mt_deli_destroy(mt_deli* dl);
/* Construct documents [doc0, doc0+n) from checkpoints (NULL: new documents, sequenceNumber 0, no
 * clients; lambda.ts:124-167).  The msn is derived from the clients as the constructor does. */
mt_status mt_deli_restore(mt_deli* dl, uint32_t doc0, uint32_t n, const mt_deli_checkpoint* ckpts);
/* Ticket a CSR batch of raw messages (host buffers, synchronous): n_docs+1 row pointers, document
 * d's messages are msgs[row_ptr[d] .. row_ptr[d+1]).  out: one ticket per message. */
mt_status mt_deli_ticket(mt_deli* dl, const mt_raw_msg* msgs, uint64_t n_msgs, const uint32_t* doc_row_ptr,
                         uint32_t n_docs, mt_ticket* out);
/* The same on device-resident buffers (HBM), asynchronous on the deli's stream.  d_ops (optional)
 * fuses the hand-off to the apply engine: a message with op_index = k + 1 carries op record k, and
 * that record gets the seq / msn / ref_seq of its ticket (seq = MT_SEQ_NACK when the message was not
 * sent, which the apply engine rejects as MT_DERR_SEQ_ORDER); op_index past n_ops links nothing. */
mt_status mt_deli_ticket_device(mt_deli* dl, const mt_raw_msg* d_msgs, const uint32_t* d_row_ptr, uint32_t n_docs,
                                mt_ticket* d_out, mt_op_rec* d_ops, uint64_t n_ops);
/* Bench tooling: construct documents [0, n_docs) all from the same checkpoint (device fill). */
mt_status mt_deli_restore_all(mt_deli* dl, uint32_t n_docs, const mt_deli_checkpoint* ckpt);
/* Bench tooling: the raw op messages behind a device op log (one MT_RAW_OP per record, client
 * sequence numbers counted per client, ref_seq copied, op_index = record + 1).  With every client
 * joined at seq 0 (mt_deli_restore_all), deli re-derives exactly the seq / msn the log carries. */
mt_status mt_deli_raw_from_ops(mt_deli* dl, const mt_op_rec* d_ops, const uint32_t* d_row_ptr, uint32_t n_docs,
                               mt_raw_msg* d_msgs);
/* Bench tooling: a new document's whole raw stream (BASELINE config C5): the ClientJoin of clients
 * 1..n_join (lambda.ts:286-299, each revs the sequence number) followed by the op messages of
 * the log, their refSeq moved past the joins (+ n_join, so each op still references what its
 * client had seen).  Document d's messages are d_msgs[msg_row_ptr[d] .. msg_row_ptr[d+1]) with
 * msg_row_ptr[d] = d_row_ptr[d] + d * n_join (device arrays; msg_row_ptr has n_docs + 1
 * entries).  Ticketed from new documents (mt_deli_restore with NULL) with fused stamping, the
 * op records get seq = log seq + n_join and deli's msn. */
mt_status mt_deli_raw_stream(mt_deli* dl, const mt_op_rec* d_ops, const uint32_t* d_row_ptr, uint32_t n_docs,
                             uint32_t n_join, mt_raw_msg* d_msgs, uint32_t* d_msg_row_ptr);
mt_status mt_deli_sync(mt_deli* dl);
/* Kernel time of the last mt_deli_ticket / mt_deli_ticket_device (HIP events around the launch). */
mt_status mt_deli_last_ms(mt_deli* dl, float* kernel_ms);
/* generateDeliCheckpoint (lambda.ts:754-764).  A document holding a client >= 64 (joined or nacked)
 * does not fit mt_deli_checkpoint: the call returns MT_ERR_WIDE and writes nothing -- read it
 * with mt_deli_get_checkpoint_wide, which serves every document (clients past 63 zero when unpromoted). */
mt_status mt_deli_get_checkpoint(mt_deli* dl, uint32_t doc, mt_deli_checkpoint* out);
mt_status mt_deli_get_checkpoint_wide(mt_deli* dl, uint32_t doc, mt_deli_checkpoint_wide* out);
/* mt_deli_restore from wide checkpoints: a document with any client >= 64 joined or nacked takes a row of
 * the big pool (its free list first); MT_ERR_NOMEM and nothing restored when the pool cannot hold them. */
mt_status mt_deli_restore_wide(mt_deli* dl, uint32_t doc0, uint32_t n, const mt_deli_checkpoint_wide* ckpts);
/* clients [first, first + n) of a document (any id < MT_DELI_MAX_CLIENTS; not joined: zeros) */
mt_status mt_deli_get_clients(mt_deli* dl, uint32_t doc, uint32_t first, uint32_t n, mt_deli_client* out);
/* err = mt_deli_err, index = position of the failing message inside the document's stream */
mt_status mt_deli_doc_error(mt_deli* dl, uint32_t doc, int32_t* err, int32_t* index);

/* ---- tick-major feed (timed from the first H2D of the op batch) -------------
 * A serving loop receives, per tick, the next sequenced ops of every document -- what
 * SharedSegmentSequence.processMergeTreeMsg sees one message at a time
 * (packages/dds/sequence/src/sequence.ts:593-633), for many documents at once.  mt_submit_ticks
 * applies a list of such ticks from host memory with the upload overlapped: tick k + 1 (and k + 2)
 * is copied into a ring of device slots on a copy stream while tick k applies, so every launch
 * still holds every document of the tick.  The same states as mt_submit of each tick in order.
 * Host buffers should be page-locked (hipHostMalloc; hipmem.PinnedArray) for the copies to be
 * asynchronous; they must stay valid until the call returns. */
typedef struct mt_tick {
    const mt_op_rec* ops;         /* the tick's records, grouped by document, seq-ascending within one */
    uint64_t n_ops;
    const uint8_t* payload;       /* the records' payload_off are offsets into this tick's payload     */
    uint64_t payload_bytes;
    const uint32_t* doc_row_ptr;  /* n_docs + 1 entries: [0] = 0, [n_docs] = n_ops, non-decreasing     */
    /* deli feed (mt_submit_ticks_deli; NULL / 0 otherwise): the tick's raw client messages grouped by
     * document (msg_row_ptr, n_docs + 1 entries), ticketed before the tick applies; a message with
     * op_index = k + 1 carries this tick's record k and stamps its seq / msn / ref_seq (fused hand-off,
     * mt_deli_ticket_device). */
    const mt_raw_msg* msgs;
    uint64_t n_msgs;
    const uint32_t* msg_row_ptr;
    mt_ticket* tickets;           /* optional: one ticket per message, copied back to the host         */
} mt_tick;
/* Apply ticks[0 .. n_ticks) in order.  Each tick is checked on the host while earlier ticks apply
 * (row pointers, payload bounds, as mt_batch_upload does) -- the first tick's records on the device
 * once they have landed, before anything of it runs; a malformed tick returns MT_ERR_ARG with the
 * ticks before it applied, as a loop of applyMsg stops at the message that throws.
 * mt_last_apply_stats / mt_last_apply_class_stats then cover the whole call. */
mt_status mt_submit_ticks(mt_engine* eng, const mt_tick* ticks, uint32_t n_ticks);
/* The same with each tick's raw messages ticketed by `dl` on the engine's stream first (deli -> apply
 * in one pipeline; the deli must be on the engine's device; its documents are the engine's).  A
 * document's mt_deli_doc_error index is then relative to the tick it failed in. */
mt_status mt_submit_ticks_deli(mt_engine* eng, mt_deli* dl, const mt_tick* ticks, uint32_t n_ticks);

/* Host tooling (no device work): lays a document-major CSR op log (and, optionally, its raw
 * messages in the mt_deli_raw_stream layout, op_index = 1 + the record's index in `ops`) out
 * tick-major for mt_submit_ticks: tick t holds the records [t * per, (t + 1) * per) of every
 * document, grouped by document, with the payload bytes of the tick compacted in record order
 * (payload_off rebased to the tick).  A message carrying a record goes to that record's tick (its
 * op_index rebased to the tick); a message carrying none to the tick of the document's previous
 * record (tick 0 before the first).  Call first with out->ops == NULL: n_ticks and payload_bytes are
 * filled in; then with every output array allocated. */
typedef struct mt_tick_layout {
    uint32_t n_ticks;          /* out: ceil(max ops per document / per), at least 1                    */
    uint32_t pad;
    uint64_t payload_bytes;    /* out: the compacted payload of all ticks                               */
    mt_op_rec* ops;            /* n_ops records                                                         */
    uint8_t* payload;          /* payload_bytes                                                         */
    uint32_t* row_ptrs;        /* n_ticks * (n_docs + 1): tick t's doc_row_ptr at t * (n_docs + 1)      */
    uint64_t* tick_ops;        /* n_ticks + 1: tick t's records are ops[tick_ops[t] .. tick_ops[t + 1]) */
    uint64_t* tick_payload;    /* n_ticks + 1: its payload bytes                                        */
    mt_raw_msg* msgs;          /* n_msgs (with msgs)                                                    */
    uint32_t* msg_row_ptrs;    /* n_ticks * (n_docs + 1) (with msgs)                                    */
    uint64_t* tick_msgs;       /* n_ticks + 1 (with msgs)                                               */
} mt_tick_layout;
mt_status mt_log_to_ticks(const mt_op_rec* ops, uint64_t n_ops, const uint8_t* payload, uint64_t payload_bytes,
                          const uint32_t* doc_row_ptr, uint32_t n_docs, uint32_t per, const mt_raw_msg* msgs,
                          uint64_t n_msgs, const uint32_t* msg_row_ptr, mt_tick_layout* out);
/* The same with a ramp of short first ticks: tick t holds min(per, first << t) records of each document
 * (first, 2 first, 4 first, ... then per; 1 <= first <= per).  A feed starts applying once its first
 * tick has landed and the copy runs ahead of the apply only once the ticks' apply outlasts their copy:
 * the ramp cuts the copies the apply waits for at the start. */
mt_status mt_log_to_ticks_ramp(const mt_op_rec* ops, uint64_t n_ops, const uint8_t* payload, uint64_t payload_bytes,
                               const uint32_t* doc_row_ptr, uint32_t n_docs, uint32_t per, uint32_t first,
                               const mt_raw_msg* msgs, uint64_t n_msgs, const uint32_t* msg_row_ptr,
                               mt_tick_layout* out);

#ifdef __cplusplus
}
#endif
#endif /* MTGPU_H */
