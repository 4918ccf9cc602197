// mt_state.h -- device-resident per-document merge-tree state (HBM layout) shared by the
// kernels and the host side of libmtgpu.so.  See DESIGN.md "Data layout in HBM".
//
// Between launches a document is stored COMPACT and IN DOCUMENT ORDER: entry i of every
// segment array is the i-th linked leaf (what walkAllSegments visits, mergeTree.ts:2969-2983).
// Arrays are structure-of-arrays with a fixed per-document stride so a wave loads/stores a
// document's first N entries with coalesced accesses.
#pragma once
#include <stdint.h>

#define MT_MAXLEV 7
// bytes of one segment's persistent state: seq, rseq, len, toff (4 each), overlap, props (8 each),
// client, rclient, flags (1 each)
#define MT_SEG_STATE_BYTES 35          // block levels incl. leaf blocks: 8^7 leaves
#define MT_DEAD_SLOT 0xFFFFu // heap entry whose segment was unlinked (segment.parent === undefined)

// segment flag bits
#define MT_SF_REMOVED 1u     // removedSeq !== undefined
#define MT_SF_PDEF 2u        // properties !== undefined (possibly empty)
#define MT_SF_NL 4u          // text ends with "\n" (TextSegment.canAppend, textSegment.ts:63-68)
#define MT_SF_HASNL 8u       // text contains a "\n" somewhere (a split of a segment without one needs no text read)
#define MT_SF_MARKER 16u     // a Marker (length 1; its one arena byte is its ReferenceType)
#define MT_SF_STALE 32u      // a marker annotated since its leaf block's last blockUpdate: the block caches
                             // (HierMergeBlock rightmostTiles / leftmostTiles / rangeStacks) still hold the
                             // label value ids in `slab` (documents with declared label keys only)
#define MT_SF_OVW 128u       // (within one op only) a pending local removal this remote removal took over

// needsScour tri-state (mergeTree.ts:63, 1279, 1438, 1445)
#define MT_SC_UNDEF 0
#define MT_SC_TRUE 1
#define MT_SC_FALSE 2

struct mt_doc_scalars {      // 84 bytes
    int32_t nseg;            // linked segments
    int32_t nlev;            // block levels (1 = the root is the only, leaf, block)
    int32_t nb[MT_MAXLEV];   // blocks per level (level 0 = leaf blocks)
    int32_t heap_n;          // zamboni LRU heap size (entries 1..heap_n)
    int32_t cur_seq, min_seq;// collabWindow.currentSeq / minSeq
    int32_t err, err_seq;    // sticky per-document error (mt_doc_err) and the seq that raised it
    uint32_t text_top;       // bytes used in the current half of the document's text arena
    uint32_t text_half;      // which half of the double-buffered arena is current (0/1)
    uint32_t n_empty;        // leaf blocks without children (the register engine pads one slot each)
    uint32_t wide;           // MT_WIDE_LDS: a client id above 32 was seen (the document stays on the LDS
                             // engine); MT_WIDE_DOC: the wide representation (include/mtgpu.h "limits")
    int32_t win_op;          // batch index of the first op failing a window assert (binning's
                             // replay of the window), -1 if none, -2 once mt_fixup_kernel
                             // (its reader) consumed it
    uint32_t label_keys;     // key ids of "referenceTileLabels" (bits 0-7) and "referenceRangeLabels"
                             // (bits 8-15), 0xFF: none; MT_NO_LABEL_KEYS: block caches not tracked
};
#define MT_NO_LABEL_KEYS 0xFFFFu

#define MT_WIDE_LDS 1u  // needs the LDS engine (declared label keys, the wide form)
#define MT_WIDE_DOC 2u  // the wide document form (include/mtgpu.h "limits")
#define MT_WIDE_C64 4u  // has seen a client id above 32: 64-bit overlap sets (register engine: its C64 form)
#define MT_WIDE_GROUPS 8u  // an editing document past 64 pending edits at once: the editing form with
                           // MT_LOC_GROUPS_WIDE group slots (its HBM-workspace form), for good
// The wide form's extension: property keys 16..31 (pxx) and overlapping removers >= 64 past the 16th
// per segment (ovx words 4..7).  It never takes LDS: a launch stages it in an HBM workspace region
// per document (the LDS-staged classes) or in the document's HBM workspace (the others), and only
// for the documents binning asks it for (mt_bin_kernel):
//   MT_WIDE_XK  keys >= 16 in use, for good (a key >= 16 in a launch's ops, or in a loaded snapshot);
//   MT_WIDE_XO  this launch may grow an overlap list past 16 ids: the longest list at the last store
//               (MT_WIDE_OVN) plus the launch's removes by ids >= 64 exceeds 16 (set or cleared per launch);
//   MT_WIDE_XKV / MT_WIDE_XOV  the at-rest pxx / ovx words 4..7 are valid (written by the last store):
//               what readers test (mt_checksum.h mt_form).
#define MT_WIDE_XK 16u
#define MT_WIDE_XKV 32u
#define MT_WIDE_XO 64u
#define MT_WIDE_XOV 128u
// bits 24..31: the longest overlap list of ids >= 64 of any segment at the document's last store
#define MT_WIDE_OVN_SHIFT 24
#define MT_WIDE_OVN(w) ((uint32_t)(w) >> MT_WIDE_OVN_SHIFT)

// An editing client's document (client.ts:163-214, 588-625): its local
// edits are pending until their acks.  Pending edit ordinals [glo, ghi) (at most 64 at once) index
// the per-segment group masks (bit = ordinal % 64); gt[] holds the creation stamp counter at each
// edit, so an ack can rebuild its group's list order.
struct mt_loc {
    int32_t own;             // the editing client's short id; -1: an observer
    uint32_t glo, ghi;
    uint32_t stamp;          // creation stamps handed out (segments created while editing)
    uint32_t gt[64];
    uint32_t lseq;           // collabWindow.localSeq (mergeTree.ts:831)
    uint32_t gls[64];        // each pending group's localSeq
    uint32_t rgn, rgpn;      // regenerated op records / payload bytes not drained yet
};
// An editing document past 64 pending edits (MT_WIDE_GROUPS) keeps up to MT_LOC_GROUPS_WIDE: its
// group masks take MT_LOC_GROUPS_WIDE / 64 words per segment (mt_gstate.gmx) and each group's
// creation stamp and localSeq live here (bit / index = ordinal % MT_LOC_GROUPS_WIDE)
#define MT_LOC_GROUPS_WIDE 512
#define MT_LOC_GW (MT_LOC_GROUPS_WIDE / 64)  // group-mask words per segment of such a document
struct mt_locx {
    uint32_t gt[MT_LOC_GROUPS_WIDE];
    uint32_t gls[MT_LOC_GROUPS_WIDE];
};
#define MT_RG_RECS 256       // regenerated op records per document between drains
#define MT_RG_BYTES 4096     // and their payload bytes
#define MT_LOC_CAP 1024      // the editing form's largest LDS capacity (above: its HBM-workspace form)
#define MT_LOC_BIGCAP 8192   // the editing form's largest class: the slots of a big-pool row
#define MT_NO_ROW 0xFFFFFFFFu
// pending property counts per segment (SegmentPropertiesManager, segmentPropertiesManager.ts:11-12):
// 7 bits per key id 0..7 at bit 7k, the pending rewrite count in bits 56..63
#define MT_PK_KEY(pk, k) ((uint32_t)((pk) >> (7 * (k))) & 0x7Fu)
#define MT_PK_RW(pk) ((uint32_t)((pk) >> 56))

// Device pointers + capacities (one allocation per array, [n_docs][capacity]).
struct mt_gstate {
    int32_t* seq;      // [doc][segcap]
    int32_t* rseq;
    uint32_t* len;
    uint32_t* toff;    // text view: arena offset
    uint64_t* ovl;     // removedClientOverlap as a bitmask over short client ids < 64
    uint64_t* props;   // 8 keys x u8 value id (a wide document: the low bytes of keys 0..7's u16 ids)
    // a wide document's extra state (MT_WIDE_DOC; [doc][segcap], allocated on first need, else null):
    // ovx = its overlapping removers >= 64 ([doc][segcap][MT_OVX_WORDS]: up to MT_OVX_IDS u16 ids
    // ascending from the low half-word of word 0, 0 = none); chi = the high bytes of its short client
    // ids (client's in bits 0..7, removedClient's in 8..15); ph = the high bytes of keys 0..7's value
    // ids; pxl / pxh = keys 8..15, low / high bytes; pxx = keys 16..31 ([doc][segcap][4]: keys 16..23
    // low, high bytes, keys 24..31 low, high bytes).
    // Its text arena holds UTF-16 code units (2 bytes each; toff / len / text_top in units).
    uint64_t* ovx;
    uint16_t* chi;
    uint64_t* ph;
    uint64_t* pxl;
    uint64_t* pxh;
    uint64_t* pxx;
    uint32_t* slab;    // [doc][segcap] a stale marker's cached label value ids: tile key (low 16 bits),
                       // range key (high 16) -- allocated on the first mt_set_label_keys, else null
    uint32_t* ctx;     // [doc][MT_LOC_CAP] the LDS-staged editing form's creation stamps and localSeq
    uint64_t* lsqx;    // pairs and pending property counts by slot during a launch (mt_apply.hip
    uint64_t* pkx;     // Lds::ct / lsq / pk / gm)
    uint64_t* gmxs;
    uint32_t* slabx;   // [doc][segcap] the editing form's slot-indexed slab during a launch (its LDS
                       // has no room for it: mt_apply.hip Lds<.., LOC>); allocated with slab
    uint8_t* client;
    uint8_t* rclient;
    uint8_t* flags;
    uint8_t* lbcnt;    // [doc][lbcap]       leaf-block child counts, in order
    uint8_t* lbscour;  // [doc][lbcap]       leaf-block needsScour
    uint8_t* ibcnt;    // [doc][MT_MAXLEV-1][ibcap] interior-level child counts
    int32_t* hseq;     // [doc][hcap]        heap maxSeq (1-based, entry 0 unused)
    uint16_t* hslot;   // [doc][hcap]        heap segment (position between launches)
    mt_doc_scalars* sc;// [doc]
    uint8_t* text;     // [doc][2][textcap]  text arena, double-buffered for in-kernel compaction
    struct mt_event* ev;  // [doc][evcap] delta / maintenance events (mt_events_enable), or null
    uint32_t* evn;     // [doc] events recorded since the last drain (may exceed evcap: halted)
    // editing documents, [doc][MT_LOC_CAP]: MT_LOC_CAP slots per document (mt_loc_row)
    uint64_t* gm;      // pending group mask per segment
    uint64_t* pk;      // pending property counts (MT_PK_*)
    uint32_t* ct;      // creation stamp
    uint64_t* lsq;     // localSeq (low 32 bits) / localRemovedSeq (high), 0: undefined
    mt_loc* loc;       // [doc]
    // an editing document whose form needs more than MT_LOC_CAP slots (its HBM-workspace form) gets a
    // row of MT_LOC_BIGCAP slots in the big pool ([row][MT_LOC_BIGCAP], grown by the engine as
    // documents need rows) and keeps its state there from then on: locbig[doc] = that row, or MT_NO_ROW
    uint64_t* gmb;
    uint64_t* pkb;
    uint32_t* ctb;
    uint64_t* lsqb;
    uint32_t* locbig;  // [doc]
    // MT_WIDE_GROUPS documents: a row of the group pool (locgx[doc], or MT_NO_ROW), the group masks,
    // MT_LOC_GW words per segment ([row][MT_LOC_BIGCAP][MT_LOC_GW]), and the groups' stamps / localSeqs ([row])
    uint64_t* gmx;
    mt_locx* locx;
    uint32_t* locgx;   // [doc]
    struct mt_op_rec* rg;  // [doc][MT_RG_RECS] regenerated ops (seq = the resetting record's index)
    uint8_t* rgp;      // [doc][MT_RG_BYTES] their payload
    uint32_t segcap, lbcap, ibcap, hcap, textcap, evcap;
};
