// mtcpu.cpp -- CPU restatement of the reference merge-tree observer apply path (THE ORACLE).
//
// TEST INFRASTRUCTURE ONLY.  This file is the checker the GPU engine is compared against and
// the `cpu_baseline` ("port") leg of bench.py; it is never linked into libmtgpu.so and the
// product path never calls it.  Only tests/, __graft_entry__.smoke() and bench.py load it.
//
// It restates, for one "observer" Client per document (client 0 of the farm,
// mergeTreeOperationRunner.ts:107-108; the "readonly" client of clientReplayTool.ts:194):
//   Client.applyMsg / applyRemoteOp / updateSeqNumbers   client.ts:768-828, 989-1002
//   MergeTree.insertSegments / blockInsert / insertingWalk / breakTie / split / updateRoot
//                                                        mergeTree.ts:1968-1998, 2141-2277, 2345-2489, 1876-1887
//   ensureIntervalBoundary / splitLeafSegment / BaseSegment.splitAt / TextSegment split
//                                                        mergeTree.ts:2225-2245, 524-568; textSegment.ts:103-111
//   markRangeRemoved / addOverlappingClient / mapRange / nodeMap
//                                                        mergeTree.ts:2607-2719, 2544-2552, 2797-2807, 2903-2965
//   annotateRange + SegmentPropertiesManager.addProperties + Properties.matchProperties
//                                                        mergeTree.ts:2565-2605; segmentPropertiesManager.ts:35-111;
//                                                        properties.ts:62-93
//   nodeLength (remote view) / localNetLength            mergeTree.ts:1659-1699, 1161-1172
//   zamboni: addToLRUSet / zamboniSegments / scourNode / pack / underflow / setMinSeq
//                                                        mergeTree.ts:1273-1478, 1718-1736
//   Heap (binary heap, 1-based, strict compare)          collections.ts:213-265
//   TextSegment.canAppend / append                        textSegment.ts:63-85
// Block lengths are computed by summing the leaves (the reference caches them in
// PartialSequenceLengths, partialLengths.ts; that cache is an optimisation whose answers must
// equal the leaf sums -- the differential fuzz in tests/ pins this against the transpiled
// reference itself).
//
// Parity pinning: golden fixtures in tests/golden/ were produced by the reference itself
// (type-stripped from /root/reference by oracle/tsref/, replayed by oracle/tsref/replay_ref.js).
//
// Also here: the synthetic op-log generator (observer-driven), canonical state
// serialisation and the 64-bit checksum, all behind a small C ABI (mto_*).

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <list>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../include/mtgpu.h"
#include "mtcpu.h"

namespace {

constexpr int kMaxNodes = 8;           // MaxNodesInBlock, mergeTree.ts:334
constexpr int kTextGranularity = 256;  // MergeTree.TextSegmentGranularity, mergeTree.ts:1059
constexpr int kZamboniMax = 2;         // zamboniSegmentsMaxCount, mergeTree.ts:1061
constexpr int kMaxKeys = MT_MAX_KEYS_WIDE;  // property keys 0..31 (u16 value ids)
constexpr int32_t kUnassigned = -1;    // UnassignedSequenceNumber, constants.ts

struct Block;
struct Seg;
// SegmentGroup (mergeTree.ts:195-202): the segments one local edit touched, acked together
struct Group {
    std::vector<Seg*> segs;
    int32_t localSeq = 0;
};

struct Node {
    bool leaf;
    Block* parent = nullptr;
    int index = 0;
    explicit Node(bool l) : leaf(l) {}
};

struct Seg : Node {
    std::u16string text;              // UTF-16 code units: cachedLength = text.length (textSegment.ts:45)
    int32_t seq = 0, client = 0;
    bool removed = false;
    int32_t rseq = 0, rclient = 0;
    uint64_t overlap = 0;             // removedClientOverlap: the client ids < 64 as a bitmask ...
    std::vector<uint16_t> ovx;        // ... and the ids >= 64, ascending
    bool props_defined = false;
    uint16_t props[kMaxKeys] = {0};   // value id per key (0 = absent)
    bool marker = false;              // a Marker (mergeTree.ts:630-798): text = its one refType byte
    // an editing client's pending state: segmentGroups (FIFO, mergeTree.ts:441) and the
    // SegmentPropertiesManager counts (segmentPropertiesManager.ts:11-12)
    std::vector<Group*> groups;
    uint8_t pend[kMaxKeys] = {0};
    int pendRewrite = 0;
    int32_t lseq = 0, lrseq = 0;      // localSeq / localRemovedSeq (0: undefined; mergeTree.ts:91-92)
    Seg() : Node(true) {}
    int len() const { return (int)text.size(); }
    bool ovHas(int32_t c) const {
        if (c < 0) return false;
        if (c < 64) return (overlap >> c) & 1;
        return std::binary_search(ovx.begin(), ovx.end(), (uint16_t)c);
    }
    // addOverlappingClient; false when the device's wide form could not hold it (more than
    // MT_OVX_IDS overlapping removers with ids >= 64: MT_DERR_LIMITS, as the engine reports)
    bool ovAdd(int32_t c) {
        if (c < 0 || c >= MT_MAX_CLIENTS_WIDE) return false;
        if (c < 64) {
            overlap |= 1ull << c;
            return true;
        }
        if (ovHas(c)) return true;
        if (ovx.size() >= MT_OVX_IDS) return false;
        ovx.insert(std::upper_bound(ovx.begin(), ovx.end(), (uint16_t)c), (uint16_t)c);
        return true;
    }
};

// An op record's payload (include/mtgpu.h): its text as UTF-16 code units and its property pairs,
// narrow ([Latin-1 bytes][key u8, value u8]*) or wide (MT_OP_WIDE: [u16 LE units][key u8, value u16 LE]*)
struct Pay {
    std::u16string text;
    int np = 0;
    uint8_t key[64] = {0};   // (MT_OP_NPAIRS: at most 63)
    uint16_t val[64] = {0};
    bool ok = false;
};
// property keys an op may carry: < 8 in the narrow form, < 32 in the wide one (include/mtgpu.h)
int keyLimit(const mt_op_rec& op) { return (op.type & MT_OP_WIDE) ? MT_MAX_KEYS_WIDE : MT_MAX_KEYS; }
Pay decodePay(const mt_op_rec& op, const uint8_t* payload) {
    Pay p;
    p.np = MT_OP_NPAIRS(op);
    const uint32_t pl = MT_OP_PAIRS_LEN(op);
    if (op.payload_len < pl || !MT_OP_NO_TEXT_OK(op)) return p;
    const uint8_t* b = payload + op.payload_off;
    const uint32_t tb = op.payload_len - pl;
    const bool wide = (op.type & MT_OP_WIDE) != 0;
    if (wide && (tb & 1u)) return p;
    if (wide)
        for (uint32_t i = 0; i < tb; i += 2) p.text.push_back((char16_t)(b[i] | (b[i + 1] << 8)));
    else
        for (uint32_t i = 0; i < tb; i++) p.text.push_back((char16_t)b[i]);
    const uint8_t* q = b + tb;
    for (int k = 0; k < p.np; k++) {
        p.key[k] = q[wide ? 3 * k : 2 * k];
        p.val[k] = wide ? (uint16_t)(q[3 * k + 1] | (q[3 * k + 2] << 8)) : q[2 * k + 1];
    }
    p.ok = true;
    return p;
}

enum Scour : int8_t { kUndef = 0, kTrue = 1, kFalse = 2 };

// One entry of a block's label caches: a live marker under the block and its properties when the
// caches were last rebuilt (HierMergeBlock rightmostTiles / leftmostTiles / rangeStacks,
// mergeTree.ts:263-318, hold the markers keyed by their labels at that time)
struct Snap {
    const Seg* seg;
    uint16_t props[kMaxKeys];
};

struct Block : Node {
    int childCount = 0;
    Node* children[kMaxNodes] = {nullptr};
    int8_t needsScour = kUndef;
    std::vector<Snap> snap;  // the block's label caches as of its last blockUpdate, in document order
    Block() : Node(false) {}
};

void json_escape(std::string& o, const std::u16string& s);

struct LRU {
    Seg* seg;
    int32_t maxSeq;
};

struct Doc {
    Block* root;
    int32_t currentSeq = 0, minSeq = 0;
    std::vector<LRU> heap{LRU{nullptr, -2}};  // L[0] = comparer min (mergeTree.ts:923-926)
    std::vector<std::unique_ptr<Node>> pool;
    int32_t err = 0, err_seq = 0;
    // delta / maintenance callbacks (mergeTreeDeltaCallback.ts:15-73) in the engine's mt_event
    // form (include/mtgpu.h), recorded when `rec` is set
    bool rec = false;
    int32_t evSeq = 0;
    std::vector<mt_event> events;
    // the editing client (collabWindow.clientId): the client of the document's first local edit
    // (a record with seq -1); its sequenced messages are acks.  -100: an observer
    int32_t own = -100;
    std::list<Group> pending;          // MergeTree.pendingSegments (mergeTree.ts:1093)
    int32_t localSeq = 0;              // collabWindow.localSeq (mergeTree.ts:831)
    uint32_t nrec = 0;                 // records of this document applied so far
    // the device holds this document in its wide form (include/mtgpu.h "limits"): it received a wide
    // op or a client id >= 64, or loaded such segments.  An editing client's document cannot be wide.
    bool wide = false;
    std::string regenJson;             // the ops regeneratePendingOp produced: [[record, [op, ...]], ...]

    Doc() { root = newBlock(); }

    // ordinal among the leaves still linked (parent set) and local-view position of `s`, walking
    // the blocks as they stand at callback time ({-1, -1} when `s` is not linked)
    std::pair<int, int> where(const Seg* s) const {
        int ord = 0, pos = 0;
        bool found = false;
        walkWhere(root, s, ord, pos, found);
        return found ? std::make_pair(ord, pos) : std::make_pair(-1, -1);
    }
    static void walkWhere(const Block* b, const Seg* s, int& ord, int& pos, bool& found) {
        for (int i = 0; i < b->childCount && !found; i++) {
            const Node* ch = b->children[i];
            if (!ch->leaf) {
                walkWhere(static_cast<const Block*>(ch), s, ord, pos, found);
                continue;
            }
            if (!ch->parent) continue;
            if (ch == s) {
                found = true;
                return;
            }
            ord++;
            pos += localLen(static_cast<const Seg*>(ch));
        }
    }
    // propertyDeltas of one delta segment: keys present (bit k) and the previous value id per key
    struct PDelta {
        uint32_t mask = 0;
        uint16_t vals[kMaxKeys] = {0};
    };
    void ev(int op, unsigned flags, int leaf, int pos, int len, const PDelta* pd = nullptr) {
        mt_event e{};
        e.seq = evSeq;
        e.op = (int8_t)op;
        e.flags = (uint8_t)flags;
        e.leaf = leaf;
        e.pos = pos;
        e.len = (uint32_t)len;
        if (pd) {
            e.pmask = pd->mask;
            for (int k = 0; k < kMaxKeys; k++) e.pvals[k] = pd->vals[k];
        }
        events.push_back(e);
    }

    Block* newBlock() {
        auto* b = new Block();
        pool.emplace_back(b);
        return b;
    }
    Seg* newSeg() {
        auto* s = new Seg();
        pool.emplace_back(s);
        return s;
    }

    // ---------------------------------------------------------------- visibility
    // nodeLength leaf branch for a remote client (mergeTree.ts:1667-1697)
    static int segLen(const Seg* s, int32_t R, int32_t C) {
        if (s->client == C || (s->seq != kUnassigned && s->seq <= R)) {
            if (s->removed) {
                if (s->rclient == C || s->ovHas(C) || (s->rseq != kUnassigned && s->rseq <= R))
                    return 0;
            }
            return s->len();
        }
        return 0;
    }
    static int localLen(const Seg* s) { return s->removed ? 0 : s->len(); }

    static int nodeLen(const Node* n, int32_t R, int32_t C) {
        if (n->leaf) return segLen(static_cast<const Seg*>(n), R, C);
        const Block* b = static_cast<const Block*>(n);
        int t = 0;
        for (int i = 0; i < b->childCount; i++) t += nodeLen(b->children[i], R, C);
        return t;
    }
    static int localNodeLen(const Node* n) {
        if (n->leaf) return localLen(static_cast<const Seg*>(n));
        const Block* b = static_cast<const Block*>(n);
        int t = 0;
        for (int i = 0; i < b->childCount; i++) t += localNodeLen(b->children[i]);
        return t;
    }
    // nodeLength (mergeTree.ts:1659-1699): the editing client's own view is the local one
    int viewLen(const Node* n, int32_t R, int32_t C) const { return C == own ? localNodeLen(n) : nodeLen(n, R, C); }

    // breakTie, mergeTree.ts:2248-2277
    bool breakTie(int pos, const Node* n, int32_t R, int32_t C) const {
        if (!n->leaf) return true;
        if (pos == 0) {
            const Seg* s = static_cast<const Seg*>(n);
            if (s->removed && s->rseq <= R && s->rseq != kUnassigned) return false;
            if (C == own) return true;             // a local change sees everything
            return s->seq != kUnassigned;          // newer segments come before older ones
        }
        return false;
    }
    // blockInsert's continuePredicate (mergeTree.ts:2143-2160): rightExcursion from block b
    // (:2313-2343) reaches the first leaf after it that the local view shows, and the insert
    // continues past b when that leaf is a pending local insert
    bool continueLocal(const Block* b) const {
        const Node* node = b;
        for (const Block* parent = b->parent; parent; node = parent, parent = parent->parent) {
            bool after = false;
            for (int i = 0; i < parent->childCount; i++) {
                const Node* ch = parent->children[i];
                if (!after) {
                    after = ch == node;
                    continue;
                }
                if (ch->leaf) return static_cast<const Seg*>(ch)->seq == kUnassigned;  // leafAction, any length
                if (const Seg* f = firstLocal(ch)) return f->seq == kUnassigned;      // nodeMap, local view
            }
        }
        return false;
    }
    static const Seg* firstLocal(const Node* n) {
        if (n->leaf) return localLen(static_cast<const Seg*>(n)) > 0 ? static_cast<const Seg*>(n) : nullptr;
        const Block* b = static_cast<const Block*>(n);
        for (int i = 0; i < b->childCount; i++)
            if (const Seg* f = firstLocal(b->children[i])) return f;
        return nullptr;
    }

    static void assign(Block* b, Node* child, int i) {
        child->parent = b;
        child->index = i;
        b->children[i] = child;
    }

    // blockUpdate's cache half (mergeTree.ts:2748-2768, addNodeReferences :263-318): a leaf child that
    // is a live marker (localNetLength > 0) enters with its properties now; a block child contributes
    // its own caches as they stand
    static void blockUpdate(Block* b) {
        b->snap.clear();
        for (int i = 0; i < b->childCount; i++) {
            const Node* ch = b->children[i];
            if (ch->leaf) {
                const Seg* x = static_cast<const Seg*>(ch);
                if (x->marker && localLen(x) > 0) {
                    Snap e{x, {0}};
                    if (x->props_defined) std::memcpy(e.props, x->props, sizeof(e.props));
                    b->snap.push_back(e);
                }
            } else {
                const Block* c = static_cast<const Block*>(ch);
                b->snap.insert(b->snap.end(), c->snap.begin(), c->snap.end());
            }
        }
    }
    // blockUpdatePathLengths (mergeTree.ts:2770-2779): the block and every ancestor
    static void pathUpdate(Block* b) {
        for (; b; b = b->parent) blockUpdate(b);
    }

    // split, mergeTree.ts:2476-2489
    Block* split(Block* node) {
        const int half = kMaxNodes / 2;
        Block* nb = newBlock();
        nb->childCount = half;
        node->childCount = half;
        for (int i = 0; i < half; i++) {
            assign(nb, node->children[half + i], i);
            node->children[half + i] = nullptr;
        }
        blockUpdate(node);  // nodeUpdateLengthNewStructure of both halves
        blockUpdate(nb);
        return nb;
    }

    // updateRoot, mergeTree.ts:1876-1887
    void updateRoot(Block* splitNode) {
        if (!splitNode) return;
        Block* nr = newBlock();
        nr->childCount = 2;
        assign(nr, root, 0);
        assign(nr, splitNode, 1);
        root = nr;
        blockUpdate(nr);
    }

    // BaseSegment.splitAt + TextSegment.createSplitSegmentAt (mergeTree.ts:524-568)
    Seg* splitAt(Seg* s, int pos) {
        Seg* r = newSeg();
        r->text = s->text.substr(pos);
        s->text.resize(pos);
        r->props_defined = s->props_defined;
        std::memcpy(r->props, s->props, sizeof(r->props));
        r->parent = s->parent;
        r->removed = s->removed;
        r->rseq = s->rseq;
        r->rclient = s->rclient;
        r->seq = s->seq;
        r->client = s->client;
        r->overlap = s->overlap;
        r->ovx = s->ovx;
        r->marker = s->marker;
        // segmentGroups.copyTo and the property manager's pending counts (mergeTree.ts:555-560,
        // segmentPropertiesManager.ts:113-127)
        r->groups = s->groups;
        for (Group* g : r->groups) g->segs.push_back(r);
        std::memcpy(r->pend, s->pend, sizeof(r->pend));
        r->pendRewrite = s->pendRewrite;
        r->lseq = s->lseq;
        r->lrseq = s->lrseq;
        return r;
    }

    // insertingWalk, mergeTree.ts:2345-2474.  insertMode=false: ensureIntervalBoundary walk.
    // Returns the block produced by a split (or nullptr).  `ok` is cleared if an insert fell through.
    // `sequenced`: the insert has a sequence number (the continuePredicate applies).  Returns the
    // unfinished node (unfinished()) when the walk should go on past b.
    static Block* unfinished() { return reinterpret_cast<Block*>(uintptr_t(1)); }
    Block* insertingWalk(Block* b, int pos, int32_t R, int32_t C, Seg* cand, bool sequenced = true) {
        int ci;
        Node* newNode = nullptr;
        for (ci = 0; ci < b->childCount; ci++) {
            Node* child = b->children[ci];
            int len = viewLen(child, R, C);
            if (pos < len || (pos == len && breakTie(pos, child, R, C))) {
                if (!child->leaf) {
                    Block* sp = insertingWalk(static_cast<Block*>(child), pos, R, C, cand, sequenced);
                    if (sp == unfinished()) {  // act as if the child were shifted
                        pos -= len;
                        continue;
                    }
                    if (!sp) {
                        blockUpdate(b);  // blockUpdateLength on the way back up
                        return nullptr;
                    }
                    newNode = sp;
                    ci++;
                } else {
                    Seg* seg = static_cast<Seg*>(child);
                    if (cand) {  // onLeaf: candidate replaces current, current re-inserted after
                        assign(b, cand, ci);
                        newNode = seg;
                        ci++;
                    } else {     // splitLeafSegment
                        if (!(pos > 0)) return nullptr;
                        newNode = splitAt(seg, pos);
                        if (rec) {  // MergeTreeMaintenanceType.SPLIT, mergeTree.ts:2231-2236
                            const int k = where(seg).first;
                            ev(MT_EV_SPLIT, MT_EVF_FIRST, k, -1, seg->len());
                            ev(MT_EV_SPLIT, 0, k + 1, -1, static_cast<Seg*>(newNode)->len());
                        }
                        ci++;
                    }
                }
                break;
            } else {
                pos -= len;
            }
        }
        if (!newNode && pos == 0 && cand) {
            if (sequenced && !pending.empty() && continueLocal(b)) return unfinished();
            newNode = cand;  // leaf(undefined): append to this block
        }
        if (!newNode) return nullptr;
        for (int i = b->childCount; i > ci; i--) {
            b->children[i] = b->children[i - 1];
            b->children[i]->index = i;
        }
        assign(b, newNode, ci);
        b->childCount++;
        if (b->childCount < kMaxNodes) {
            blockUpdate(b);
            return nullptr;
        }
        return split(b);
    }

    void ensureIntervalBoundary(int pos, int32_t R, int32_t C) {
        updateRoot(insertingWalk(root, pos, R, C, nullptr));
    }

    // ------------------------------------------------------------------- zamboni
    void heapAdd(LRU x) {
        heap.push_back(x);
        size_t k = heap.size() - 1;
        while (k > 1 && heap[k >> 1].maxSeq - heap[k].maxSeq > 0) {
            std::swap(heap[k >> 1], heap[k]);
            k >>= 1;
        }
    }
    LRU heapGet() {
        LRU x = heap[1];
        heap[1] = heap[heap.size() - 1];
        heap.pop_back();
        size_t count = heap.size() - 1, k = 1;
        while ((k << 1) <= count) {
            size_t j = k << 1;
            if (j < count && heap[j].maxSeq - heap[j + 1].maxSeq > 0) j++;
            if (heap[k].maxSeq - heap[j].maxSeq <= 0) break;
            std::swap(heap[k], heap[j]);
            k = j;
        }
        return x;
    }

    // addToLRUSet, mergeTree.ts:1273-1283
    void addToLRUSet(Seg* s, int32_t seq) {
        if (s->parent->needsScour != kTrue && seq > currentSeq) {
            s->parent->needsScour = kTrue;
            heapAdd(LRU{s, seq});
        }
    }

    static bool matchProps(const Seg* a, const Seg* b) {
        if (a->props_defined != b->props_defined) return false;
        return std::memcmp(a->props, b->props, sizeof(a->props)) == 0;
    }
    // TextSegment.canAppend (textSegment.ts:63-68): both text segments (Marker.canAppend is false,
    // and a marker is not TextSegment.is, mergeTree.ts:793)
    static bool canAppend(const Seg* prev, const Seg* s) {
        if (prev->marker || s->marker) return false;
        if (!prev->text.empty() && prev->text.back() == u'\n') return false;
        return prev->len() <= kTextGranularity || s->len() <= kTextGranularity;
    }

    // scourNode, mergeTree.ts:1289-1365
    void scourNode(Block* node, std::vector<Node*>& hold) {
        Seg* prev = nullptr;
        for (int k = 0; k < node->childCount; k++) {
            Node* child = node->children[k];
            if (!child->leaf) {
                hold.push_back(child);
                prev = nullptr;
                continue;
            }
            Seg* s = static_cast<Seg*>(child);
            if (!s->groups.empty()) {  // pending local edits: held (mergeTree.ts:1295, 1356-1358)
                hold.push_back(s);
                prev = nullptr;
            } else if (s->removed) {
                if (s->rseq > minSeq) {
                    hold.push_back(s);
                } else {
                    if (rec) ev(MT_EV_UNLINK, MT_EVF_FIRST, where(s).first, -1, s->len());  // mergeTree.ts:1310-1315
                    s->parent = nullptr;  // UNLINK
                }
                prev = nullptr;
            } else if (s->seq <= minSeq) {
                bool app = prev && canAppend(prev, s) && matchProps(prev, s) && localLen(s) > 0;
                if (app) {
                    prev->text += s->text;  // APPEND
                    if (rec) {  // mergeTree.ts:1335-1340
                        ev(MT_EV_APPEND, MT_EVF_FIRST, where(prev).first, -1, prev->len());
                        ev(MT_EV_APPEND, 0, where(s).first, -1, s->len());
                    }
                    s->parent = nullptr;
                } else {
                    hold.push_back(s);
                    prev = localLen(s) > 0 ? s : nullptr;
                }
            } else {
                hold.push_back(s);
                prev = nullptr;
            }
        }
    }

    static bool underflow(const Block* b) { return b->childCount < kMaxNodes / 2; }

    // pack, mergeTree.ts:1368-1420
    void pack(Block* block) {
        Block* parent = block->parent;
        std::vector<Node*> hold;
        for (int ci = 0; ci < parent->childCount; ci++) {
            Block* cb = static_cast<Block*>(parent->children[ci]);
            scourNode(cb, hold);
            cb->parent = nullptr;
        }
        int total = (int)hold.size();
        const int half = kMaxNodes / 2;
        int cc = std::min(kMaxNodes - 1, total / half);
        if (cc < 1) cc = 1;
        int base = total / cc, extra = total % cc, rd = 0;
        Block* packed[kMaxNodes] = {nullptr};
        for (int ni = 0; ni < cc; ni++) {
            int nc = base;
            if (extra > 0) {
                nc++;
                extra--;
            }
            Block* pb = newBlock();
            pb->childCount = nc;
            for (int q = 0; q < nc; q++) assign(pb, hold[rd++], q);
            pb->parent = parent;
            packed[ni] = pb;
            blockUpdate(pb);  // nodeUpdateLengthNewStructure(packedBlock)
        }
        for (int j = 0; j < kMaxNodes; j++) parent->children[j] = nullptr;
        for (int j = 0; j < cc; j++) assign(parent, packed[j], j);
        parent->childCount = cc;
        if (underflow(parent) && parent->parent) pack(parent);
        else pathUpdate(parent);
    }

    // zamboniSegments, mergeTree.ts:1422-1478
    void zamboni() {
        for (int i = 0; i < kZamboniMax; i++) {
            if (heap.size() <= 1 || heap[1].maxSeq > minSeq) break;
            LRU t = heapGet();
            Seg* s = t.seg;
            if (s->parent && s->parent->needsScour != kFalse) {
                Block* b = s->parent;
                std::vector<Node*> hold;
                scourNode(b, hold);
                b->needsScour = kFalse;
                if ((int)hold.size() < b->childCount) {
                    for (int j = 0; j < kMaxNodes; j++) b->children[j] = nullptr;
                    b->childCount = (int)hold.size();
                    for (int j = 0; j < b->childCount; j++) assign(b, hold[j], j);
                    if (underflow(b) && b->parent) pack(b);
                    else pathUpdate(b);
                }
            }
        }
    }

    // ------------------------------------------------------------------- mapRange
    // (post: markRangeRemoved's post action, a blockUpdate of every block entered, mergeTree.ts:2656-2663)
    template <class F>
    bool nodeMap(Block* node, int32_t R, int32_t C, int start, int end, F&& leaf, bool post = false) {
        for (int ci = 0; ci < node->childCount; ci++) {
            Node* child = node->children[ci];
            int len = viewLen(child, R, C);
            if (end > 0 && len > 0 && start < len) {
                if (!child->leaf) {
                    nodeMap(static_cast<Block*>(child), R, C, start, end, leaf, post);
                } else {
                    leaf(static_cast<Seg*>(child));
                }
            }
            start -= len;
            end -= len;
        }
        if (post) blockUpdate(node);
        return true;
    }

    // ------------------------------------------------------------------------ ops
    void fail(int code, int32_t seq) {
        if (!err) {
            err = code;
            err_seq = seq;
        }
    }

    // SnapshotLoader.loadHeader (snapshotLoader.ts:119-157): specToSegment for every spec, then
    // MergeTree.reloadFromSegments (mergeTree.ts:1195-1251: blocks of MaxNodesInBlock - 1 children,
    // built bottom-up until one block is left) and startOrUpdateCollaboration(minSeq, currentSeq)
    // (client.ts:1051-1071, mergeTree.ts:1254-1271: an empty LRU heap)
    void reload(const mt_load_seg* segs, uint32_t n, const uint8_t* text, int32_t min_seq, int32_t cur_seq) {
        std::vector<Node*> nodes;
        for (uint32_t i = 0; i < n; i++) {
            const mt_load_seg& sg = segs[i];
            Seg* sx = newSeg();
            const uint8_t* t = text + sg.text_off;
            for (uint32_t q = 0; q < sg.text_len; q++)
                sx->text.push_back((sg.flags & MT_LSF_U16) ? (char16_t)(t[2 * q] | (t[2 * q + 1] << 8)) : (char16_t)t[q]);
            sx->seq = sg.seq;
            const int c = sg.client | (sg.client_hi << 8), rc = sg.rclient | (sg.rclient_hi << 8);
            sx->client = c == MT_CLIENT_NONCOLLAB ? -2 : c;
            if (sg.rseq >= 0) {
                sx->removed = true;
                sx->rseq = sg.rseq;
                sx->rclient = rc;
            }
            sx->marker = (sg.flags & 16u) != 0;  // MT_SF_MARKER
            wide = wide || (sg.flags & MT_LSF_U16) || (c >= MT_MAX_CLIENTS && c != MT_CLIENT_NONCOLLAB) ||
                   (sg.rseq >= 0 && rc >= MT_MAX_CLIENTS);
            for (int k = 0; k < kMaxKeys; k++) wide = wide || ((sg.flags & 2u) && (k >= MT_MAX_KEYS ? sg.props[k] != 0 : sg.props[k] > 255));
            if (sg.flags & 2u) {  // MT_SF_PDEF
                sx->props_defined = true;
                for (int k = 0; k < kMaxKeys; k++) sx->props[k] = sg.props[k];
            }
            nodes.push_back(sx);
        }
        const int per = kMaxNodes - 1;
        if (nodes.empty()) {
            root = newBlock();
        } else {
            for (;;) {
                std::vector<Node*> blocks;
                for (size_t i = 0; i < nodes.size(); i += per) {
                    Block* b = newBlock();
                    for (size_t j = i; j < std::min(nodes.size(), i + per); j++) assign(b, nodes[j], b->childCount++);
                    blockUpdate(b);
                    blocks.push_back(b);
                }
                if (blocks.size() == 1) {
                    root = static_cast<Block*>(blocks[0]);
                    break;
                }
                nodes.swap(blocks);
            }
        }
        root->parent = nullptr;
        minSeq = min_seq;
        currentSeq = cur_seq;
    }

    // SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111), collaborating, no
    // combining op but "rewrite": a local change (seq -1) counts its keys pending; a remote one
    // leaves keys with pending local changes alone and is dropped whole while a local rewrite is
    // pending.  propertyDeltas in pd.  Returns false when dropped.
    static bool addProps(Seg* s, const Pay& p, bool rewrite, bool local, PDelta& pd) {
        if (!s->props_defined) {
            s->props_defined = true;
            std::memset(s->props, 0, sizeof(s->props));
            std::memset(s->pend, 0, sizeof(s->pend));
            s->pendRewrite = 0;
        }
        if (s->pendRewrite > 0 && !local) return false;
        auto modify = [&](int k) { return local || s->pend[k] == 0; };
        auto delta = [&](int k, uint16_t prev) {
            pd.mask |= 1u << k;
            pd.vals[k] = prev;
        };
        if (rewrite) {
            if (local) s->pendRewrite++;
            for (int k = 0; k < kMaxKeys; k++) {
                bool keep = false;  // newProps[key] truthy
                for (int q = 0; q < p.np; q++) keep = keep || (p.key[q] == k && p.val[q] != 0);
                if (s->props[k] && !keep && modify(k)) {
                    delta(k, s->props[k]);
                    s->props[k] = 0;
                }
            }
        }
        for (int q = 0; q < p.np; q++) {
            const int k = p.key[q];
            if (local) {
                s->pend[k]++;
            } else if (!modify(k)) {
                continue;
            }
            delta(k, s->props[k]);
            s->props[k] = p.val[q];
        }
        return true;
    }

    // the REMOVE / ANNOTATE callback (mergeTree.ts:2705-2712, 2592-2600): its delta segments in order
    void emitRange(int opk, const std::vector<Seg*>& delta, const std::vector<PDelta>& pdel,
                   const std::vector<bool>& nopd) {
        if (delta.empty()) ev(opk, MT_EVF_FIRST | MT_EVF_EMPTY, -1, -1, 0);
        for (size_t i = 0; i < delta.size(); i++) {
            const auto w = where(delta[i]);
            unsigned f = i == 0 ? MT_EVF_FIRST : 0;
            if (i < nopd.size() && nopd[i]) f |= MT_EVF_NOPD;
            ev(opk, f, w.first, w.second, delta[i]->len(), pdel.empty() ? nullptr : &pdel[i]);
        }
    }

    // addToPendingList (mergeTree.ts:1922-1929): one group per local edit
    void join(Group*& g, Seg* s) {
        if (!g) {
            pending.emplace_back();
            g = &pending.back();
        }
        g->segs.push_back(s);
        s->groups.push_back(g);
    }

    // A local edit of the editing client (client.ts:163-214 -> applyInsertOp / applyRemoveRangeOp /
    // applyAnnotateRangeOp with refSeq = currentSeq, seq = UnassignedSequenceNumber): insertSegments
    // / markRangeRemoved / annotateRange in the local view, the touched segments joining a new
    // pending group; no zamboni, no window asserts, no seq update (mergeTree.ts:1968-1998,
    // 2607-2719, 2565-2605)
    void applyLocal(const mt_op_rec& op, const uint8_t* payload) {
        if (own == -100) own = op.client;
        // (an editing client's document stays narrow: the device's editing form has no wide state)
        if (op.client != own || op.client >= MT_MAX_CLIENTS || (op.type & MT_OP_WIDE) || wide)
            return fail(MT_DERR_LIMITS, kUnassigned);
        if (op.type > MT_OP_ANNOTATE) return fail(MT_DERR_BAD_OP, kUnassigned);
        const int32_t R = currentSeq, C = own, S = kUnassigned;
        evSeq = S;
        const Pay p = decodePay(op, payload);
        if (!p.ok) return fail(MT_DERR_BAD_OP, S);
        for (int q = 0; q < p.np; q++)
            if (p.key[q] >= MT_MAX_KEYS) return fail(MT_DERR_LIMITS, S);
        Group* g = nullptr;
        if (op.type == MT_OP_INSERT && p.text.empty()) return;  // insertSegmentLocal: nothing for an empty segment
        const int32_t L = ++localSeq;
        if (op.type == MT_OP_INSERT) {
            ensureIntervalBoundary(op.pos1, R, C);
            Seg* x = newSeg();
            x->text = p.text;
            if (op.flags & MT_F_PROPS) {
                x->props_defined = true;
                for (int q = 0; q < p.np; q++) x->props[p.key[q]] = p.val[q];
            }
            x->seq = S;
            x->client = C;
            x->marker = (op.flags & MT_F_MARKER) != 0;
            x->lseq = L;
            Block* sp = insertingWalk(root, op.pos1, R, C, x, false);
            if (!x->parent) return fail(MT_DERR_INSERT_FAILED, S);
            updateRoot(sp);
            join(g, x);  // saveIfLocal
            g->localSeq = L;
            if (rec) {  // MergeTreeDeltaType.INSERT (mergeTree.ts:1981-1988)
                const auto w = where(x);
                ev(MT_EV_INSERT, MT_EVF_FIRST, w.first, w.second, x->len());
            }
            return;
        }
        ensureIntervalBoundary(op.pos1, R, C);
        ensureIntervalBoundary(op.pos2, R, C);
        std::vector<Seg*> delta;
        std::vector<PDelta> pdel;
        if (op.type == MT_OP_REMOVE) {
            nodeMap(root, R, C, op.pos1, op.pos2, [&](Seg* x) {
                if (!x->removed) delta.push_back(x);  // removedSegments
                if (x->removed) {
                    if (x->rseq == kUnassigned) {
                        x->rclient = C;
                        x->rseq = S;
                        x->lrseq = 0;
                    } else {
                        x->ovAdd(C);
                    }
                } else {
                    x->removed = true;
                    x->rseq = S;
                    x->rclient = C;
                    x->lrseq = L;
                }
                if (x->removed && x->rseq == kUnassigned) join(g, x);
            }, true);
        } else {
            const bool rewrite = op.flags & MT_F_REWRITE;
            nodeMap(root, R, C, op.pos1, op.pos2, [&](Seg* x) {
                PDelta pd;
                addProps(x, p, rewrite, true, pd);
                delta.push_back(x);
                pdel.push_back(pd);
                join(g, x);
            });
        }
        if (g) g->localSeq = L;
        if (rec) emitRange(op.type == MT_OP_REMOVE ? MT_EV_REMOVE : MT_EV_ANNOTATE, delta, pdel, {});
    }

    // Client.regeneratePendingOp -> resetPendingDeltaToOps (client.ts:708-766, 855-893) for the
    // oldest pending edit, whose op is `op`: its segments in document order, each at its
    // findReconnectionPostition (:674-706, the view as of the edit's localSeq), become one new op
    // each (a removal only while still locally removed), each with a new pending group of the same
    // localSeq at the queue's tail.  The new ops go to regenJson.
    void applyRegen(const mt_op_rec& op, const uint8_t* payload) {
        if (pending.empty()) return fail(MT_DERR_BAD_OP, -2);
        Group* g = &pending.front();
        std::vector<std::pair<int, Seg*>> mem;
        int ord = 0;
        walkSegs(root, [&](const Seg* s) {
            for (Seg* x : g->segs)
                if (x == s) mem.emplace_back(ord, x);
            ord++;
        });
        std::sort(mem.begin(), mem.end(), [](const std::pair<int, Seg*>& a, const std::pair<int, Seg*>& b) {
            return a.first < b.first;
        });
        const Pay pp = decodePay(op, payload);
        if (!pp.ok) return fail(MT_DERR_BAD_OP, -2);
        std::string ops;
        for (auto& m : mem) {
            Seg* x = m.second;
            if (x->groups.empty() || x->groups.front() != g) return fail(MT_DERR_BAD_OP, -2);
            x->groups.erase(x->groups.begin());
            const int32_t L = g->localSeq;
            int pos = 0;
            bool found = false;
            walkSegs(root, [&](const Seg* s) {
                if (s == x) found = true;
                if (found) return;
                if ((s->lseq == 0 || s->lseq <= L) && (!s->removed || (s->lrseq != 0 && s->lrseq > L))) pos += s->len();
            });
            std::string one;
            auto propsJson = [](const uint8_t* ks, const uint16_t* vs, int n, bool nulls) {
                std::string o = "{";
                for (int q = 0; q < n; q++) {
                    if (!nulls && vs[q] == 0) continue;
                    if (o.size() > 1) o += ',';
                    o += "\"" + std::to_string(ks[q]) + "\":" + (vs[q] ? std::to_string(vs[q]) : "null");
                }
                return o + "}";
            };
            if (op.type == MT_OP_ANNOTATE) {
                one = "[2," + std::to_string(pos) + "," + std::to_string(pos + x->len()) + ",null," +
                      propsJson(pp.key, pp.val, pp.np, true) + "," + ((op.flags & MT_F_REWRITE) ? "1" : "0") + "]";
            } else if (op.type == MT_OP_INSERT) {
                std::string t;
                json_escape(t, x->text);
                std::string p = "null";
                if (x->props_defined) {
                    std::vector<uint8_t> ks;
                    std::vector<uint16_t> vs;
                    for (int k = 0; k < kMaxKeys; k++)
                        if (x->props[k]) ks.push_back((uint8_t)k), vs.push_back(x->props[k]);
                    p = propsJson(ks.data(), vs.data(), (int)ks.size(), false);
                }
                one = "[0," + std::to_string(pos) + ",0," + t + "," + p + "," + (x->marker ? "128" : "0") + "]";
            } else if (op.type == MT_OP_REMOVE) {
                if (x->lrseq != 0) one = "[1," + std::to_string(pos) + "," + std::to_string(pos + x->len()) + ",null,null,0]";
            } else {
                return fail(MT_DERR_BAD_OP, -2);
            }
            if (one.empty()) continue;
            if (!ops.empty()) ops += ',';
            ops += one;
            pending.emplace_back();
            Group& ng = pending.back();
            ng.localSeq = g->localSeq;
            ng.segs.push_back(x);
            x->groups.push_back(&ng);
        }
        pending.pop_front();
        if (!regenJson.empty()) regenJson += ',';
        regenJson += "[" + std::to_string(nrec) + ",[" + ops + "]]";
    }

    // ackPendingSegment (client.ts:588-625 -> mergeTree.ts:1893-1920, BaseSegment.ack :487-522):
    // the editing client's own sequenced message settles its oldest pending group
    void applyAck(const mt_op_rec& op, const uint8_t* payload, bool last_member) {
        const int32_t S = op.seq;
        evSeq = S;
        if (!pending.empty()) {
            Group& g = pending.front();
            const Pay pp = decodePay(op, payload);
            if (!pp.ok) return fail(MT_DERR_BAD_OP, S);
            for (Seg* x : g.segs) {
                if (x->groups.empty() || x->groups.front() != &g) return fail(MT_DERR_BAD_OP, S);
                x->groups.erase(x->groups.begin());
                if (op.type == MT_OP_INSERT) {
                    x->seq = S;
                    x->lseq = 0;
                } else if (op.type == MT_OP_REMOVE) {
                    x->lrseq = 0;
                    if (x->rseq == kUnassigned) x->rseq = S;  // else a remote removal overwrote it
                } else {  // ackPendingProperties (segmentPropertiesManager.ts:15-28)
                    if (op.flags & MT_F_REWRITE) x->pendRewrite--;
                    for (int q = 0; q < pp.np; q++)
                        if (x->pend[pp.key[q]] > 0) x->pend[pp.key[q]]--;
                }
                addToLRUSet(x, S);
            }
            std::vector<Block*> nodes;  // blockUpdatePathLengths of each member's parent (mergeTree.ts:1908-1915)
            for (Seg* x : g.segs)
                if (x->parent && std::find(nodes.begin(), nodes.end(), x->parent) == nodes.end()) nodes.push_back(x->parent);
            for (Block* b : nodes) pathUpdate(b);
            pending.pop_front();
        }
        zamboni();
        if (last_member) updateSeqNumbers(op.msn, S);
    }

    void applyOp(const mt_op_rec& op, const uint8_t* payload, bool last_member) {
        if (err) return;
        struct Count {  // the document's record index, for regenJson
            uint32_t& n;
            ~Count() { n++; }
        } count{nrec};
        if (MT_OP_TYPE(op) == MT_OP_LOAD) return loadInsert(op, payload);
        const bool wop = (op.type & MT_OP_WIDE) || ((op.client >= MT_MAX_CLIENTS) && !MT_OP_IS_NOOP(op));
        if (op.seq == kUnassigned) return applyLocal(op, payload);
        if (op.seq == -2) return applyRegen(op, payload);
        if (own != -100 && wop) return fail(MT_DERR_LIMITS, op.seq);  // (the editing form is narrow)
        if ((int32_t)op.client == own && op.type <= MT_OP_ANNOTATE) return applyAck(op, payload, last_member);
        const int32_t S = op.seq, R = op.ref_seq, C = op.client;
        const int type = MT_OP_TYPE(op);
        // Every assert the reference raises for this message is checked BEFORE anything is
        // applied, in the reference's order: the document halts in the state of the messages
        // before it (the reference throws after the op's tree edits, leaving them half-done).
        if (type > MT_OP_NOOP) return fail(MT_DERR_BAD_OP, S);
        evSeq = S;
        const bool noop = MT_OP_IS_NOOP(op);  // incl. an empty-string insert (client.ts:403-407)
        const Pay p = decodePay(op, payload);
        if (!noop) {
            if (op.client >= MT_MAX_CLIENTS_WIDE || op.client == 0 || op.client == MT_CLIENT_NONCOLLAB)
                return fail(MT_DERR_LIMITS, S);
            if (!p.ok) return fail(MT_DERR_BAD_OP, S);
            int wc = 0;
            if (!(currentSeq < S)) wc = MT_DERR_SEQ_ORDER;              // completeAndLogOp, client.ts:461-462
            else if (!(minSeq <= op.msn)) wc = MT_DERR_MSN_ORDER;       // client.ts:463-464
            else if (!(op.msn <= S)) wc = MT_DERR_MSN_ORDER;            // updateSeqNumbers, client.ts:826
            if (wc) {
                // those asserts run after the op: a failing insert throws first (mergeTree.ts:2210)
                if (type == MT_OP_INSERT && !p.text.empty() && op.pos1 > viewLen(root, op.ref_seq, op.client))
                    wc = MT_DERR_INSERT_FAILED;
                return fail(wc, S);
            }
        } else {
            if (!(currentSeq <= S)) return fail(MT_DERR_SEQ_ORDER, S);  // updateSeqNumbers, client.ts:824
            if (!(op.msn <= S)) return fail(MT_DERR_MSN_ORDER, S);      // client.ts:826
            if (!(minSeq <= op.msn)) return fail(MT_DERR_MSN_ORDER, S); // setMinSeq, mergeTree.ts:1722
        }
        if (!noop) {
            for (int q = 0; q < p.np; q++)
                if (p.key[q] >= keyLimit(op)) return fail(MT_DERR_LIMITS, S);
            if (wop) wide = true;
        }
        switch (noop ? MT_OP_NOOP : type) {
            case MT_OP_INSERT: {
                if (op.pos1 < 0) return fail(MT_DERR_BAD_OP, S);
                ensureIntervalBoundary(op.pos1, R, C);
                if (!p.text.empty()) {  // blockInsert skips zero-length segments (mergeTree.ts:2196)
                    Seg* s = newSeg();
                    s->text = p.text;
                    if (op.flags & MT_F_PROPS) {  // TextSegment.make -> addProperties (no collab)
                        s->props_defined = true;
                        for (int q = 0; q < p.np; q++) s->props[p.key[q]] = p.val[q];
                    }
                    s->seq = S;
                    s->client = C;
                    s->marker = (op.flags & MT_F_MARKER) != 0;
                    Block* sp = insertingWalk(root, op.pos1, R, C, s);
                    if (!s->parent) return fail(MT_DERR_INSERT_FAILED, S);
                    updateRoot(sp);
                    if (S > minSeq) addToLRUSet(s, S);  // saveIfLocal, mergeTree.ts:2164-2179
                    if (rec) {  // MergeTreeDeltaType.INSERT, mergeTree.ts:1981-1988
                        const auto w = where(s);
                        ev(MT_EV_INSERT, MT_EVF_FIRST, w.first, w.second, s->len());
                    }
                } else if (rec) {
                    ev(MT_EV_INSERT, MT_EVF_FIRST, -1, -1, 0);  // the zero-length segment is never linked
                }
                zamboni();
                break;
            }
            case MT_OP_REMOVE:
            case MT_OP_ANNOTATE: {
                if (op.pos1 < 0 || op.pos2 < 0) return fail(MT_DERR_BAD_OP, S);
                ensureIntervalBoundary(op.pos1, R, C);
                ensureIntervalBoundary(op.pos2, R, C);
                std::vector<Seg*> delta;  // deltaSegments of the op's callback
                std::vector<PDelta> pdel;
                std::vector<bool> nopd;
                bool over = false;
                if (type == MT_OP_REMOVE) {
                    nodeMap(root, R, C, op.pos1, op.pos2, [&](Seg* s) {
                        if (s->removed) {
                            if (s->rseq == kUnassigned) {  // a pending local removal: the remote one replaces it
                                s->rclient = C;
                                s->rseq = S;
                                s->lrseq = 0;
                            } else {
                                over = over || !s->ovAdd(C);  // addOverlappingClient
                            }
                        } else {
                            s->removed = true;
                            s->rseq = S;
                            s->rclient = C;
                            delta.push_back(s);          // removedSegments (mergeTree.ts:2637)
                        }
                        addToLRUSet(s, S);
                    }, true);
                } else {
                    const bool rewrite = op.flags & MT_F_REWRITE;
                    nodeMap(root, R, C, op.pos1, op.pos2, [&](Seg* s) {
                        PDelta pd;
                        // (dropped while a local rewrite is pending: propertyDeltas undefined)
                        const bool kept = addProps(s, p, rewrite, false, pd);
                        delta.push_back(s);
                        pdel.push_back(kept ? pd : PDelta());
                        nopd.push_back(!kept);
                        addToLRUSet(s, S);
                    });
                }
                // (the device's wide form holds MT_OVX_IDS overlapping removers >= 64 per segment)
                if (over) return fail(MT_DERR_LIMITS, S);
                if (rec) emitRange(type == MT_OP_REMOVE ? MT_EV_REMOVE : MT_EV_ANNOTATE, delta, pdel, nopd);
                zamboni();
                break;
            }
            case MT_OP_NOOP:
                break;
            default:
                return fail(MT_DERR_BAD_OP, S);
        }
        if (last_member) updateSeqNumbers(op.msn, S);
    }

    // SnapshotLoader.loadBody's append (snapshotLoader.ts:192-224): MergeTree.insertSegments(pos,
    // [seg], refSeq, client, seq) (mergeTree.ts:1968-1998) outside any Client -- no window asserts,
    // no updateSeqNumbers; the segment may carry removedSeq / removedClient from its spec
    void loadInsert(const mt_op_rec& op, const uint8_t* payload) {
        const int32_t S = op.seq, R = op.ref_seq;
        evSeq = S;
        const int c = (int)MT_LOAD_CLIENT(op), rc = (int)MT_LOAD_RCLIENT(op);
        const int32_t C = c == MT_CLIENT_NONCOLLAB ? -2 : c;
        if (!(c == MT_CLIENT_NONCOLLAB || (c >= 1 && c < MT_MAX_CLIENTS_WIDE)) ||
            (op.pos2 >= 0 && !(rc >= 1 && rc < MT_MAX_CLIENTS_WIDE && rc != MT_CLIENT_NONCOLLAB)))
            return fail(MT_DERR_LIMITS, S);
        const Pay p = decodePay(op, payload);
        if (!p.ok || op.pos1 < 0) return fail(MT_DERR_BAD_OP, S);
        for (int q = 0; q < p.np; q++)
            if (p.key[q] >= keyLimit(op)) return fail(MT_DERR_LIMITS, S);
        if ((op.type & MT_OP_WIDE) || (c >= MT_MAX_CLIENTS && c != MT_CLIENT_NONCOLLAB) ||
            (op.pos2 >= 0 && rc >= MT_MAX_CLIENTS))
            wide = true;
        ensureIntervalBoundary(op.pos1, R, C);
        if (!p.text.empty()) {
            Seg* sx = newSeg();
            sx->text = p.text;
            if (op.flags & MT_F_PROPS) {
                sx->props_defined = true;
                for (int q = 0; q < p.np; q++) sx->props[p.key[q]] = p.val[q];
            }
            sx->seq = S;
            sx->client = C;
            sx->marker = (op.flags & MT_F_MARKER) != 0;
            if (op.pos2 >= 0) {
                sx->removed = true;
                sx->rseq = op.pos2;
                sx->rclient = rc;
            }
            Block* sp = insertingWalk(root, op.pos1, R, C, sx);
            if (!sx->parent) return fail(MT_DERR_INSERT_FAILED, S);
            updateRoot(sp);
            if (S > minSeq) addToLRUSet(sx, S);
        }
        zamboni();
    }

    // Client.updateSeqNumbers + MergeTree.setMinSeq (client.ts:821-828, mergeTree.ts:1718-1736)
    void updateSeqNumbers(int32_t msn, int32_t seq) {
        if (!(currentSeq <= seq)) return fail(MT_DERR_SEQ_ORDER, seq);
        currentSeq = seq;
        if (!(msn <= seq)) return fail(MT_DERR_MSN_ORDER, seq);
        if (!(minSeq <= msn)) return fail(MT_DERR_MSN_ORDER, seq);
        if (msn > minSeq) {
            minSeq = msn;
            zamboni();
        }
    }

    // ----------------------------------------------------------------- readout
    template <class F>
    static void walkSegs(const Node* n, F&& f) {
        if (n->leaf) {
            f(static_cast<const Seg*>(n));
            return;
        }
        const Block* b = static_cast<const Block*>(n);
        for (int i = 0; i < b->childCount; i++) walkSegs(b->children[i], f);
    }
    std::u16string text() const {
        std::u16string t;
        walkSegs(root, [&](const Seg* s) {
            if (!s->removed && !s->marker) t += s->text;  // gatherText: text segments only
        });
        return t;
    }
    int length(int32_t R, int32_t C) const { return nodeLen(root, R, C); }

    // ------------------------------------------------------------------- findTile
    // Client.findTile -> MergeTree.findTile (client.ts:1073-1076, mergeTree.ts:1763-1789) for the
    // own client: search / backwardSearch (:1797-1870) in the local view, leaf action
    // recordTileStart and shift action tileShift (:996-1035), whose block case reads the
    // HierMergeBlock's rightmostTiles / leftmostTiles (the right- / leftmost live tile of the
    // block, addNodeReferences :263-318).  A tile: a Marker whose refType has Tile (ops.ts:8) and
    // whose "referenceTileLabels" (property `key`) value id is in `vmask` (refHasTileLabel :588).
    // A shifted block answers from its caches (the labels its markers had at its last blockUpdate,
    // Block::snap); a leaf from its current properties.
    struct TileQ {
        int key;
        const uint8_t* vmask;  // 256 bits
        bool hasv(int v) const { return v != 0 && v < 256 && ((vmask[v >> 3] >> (v & 7)) & 1); }
        bool has(const Seg* s) const {
            if (!s->marker || !(s->text.size() && ((uint8_t)s->text[0] & 1u))) return false;
            return hasv(s->props[key]);
        }
        bool has(const Snap& e) const { return ((uint8_t)e.seg->text[0] & 1u) && hasv(e.props[key]); }
    };
    static const Seg* edgeTile(const Node* n, const TileQ& q, bool rightmost) {
        if (n->leaf) {
            const Seg* s = static_cast<const Seg*>(n);
            return localLen(s) > 0 && q.has(s) ? s : nullptr;
        }
        const std::vector<Snap>& sn = static_cast<const Block*>(n)->snap;  // rightmostTiles / leftmostTiles
        for (size_t i = 0; i < sn.size(); i++) {
            const Snap& e = sn[rightmost ? sn.size() - 1 - i : i];
            if (q.has(e)) return e.seg;
        }
        return nullptr;
    }
    void searchTile(const Block* b, int pos, const TileQ& q, const Seg*& tile) const {
        for (int i = 0; i < b->childCount; i++) {
            const Node* ch = b->children[i];
            const int len = localNodeLen(ch);
            if (pos < len) {
                if (!ch->leaf) return searchTile(static_cast<const Block*>(ch), pos, q, tile);
                if (q.has(static_cast<const Seg*>(ch))) tile = static_cast<const Seg*>(ch);  // recordTileStart
                return;
            }
            if (const Seg* t = edgeTile(ch, q, true)) tile = t;  // tileShift
            pos -= len;
        }
    }
    void backwardSearchTile(const Block* b, int pos, int segEnd, const TileQ& q, const Seg*& tile) const {
        for (int i = b->childCount - 1; i >= 0; i--) {
            const Node* ch = b->children[i];
            const int len = localNodeLen(ch);
            const int segpos = segEnd - len;
            if (pos >= segpos) {
                if (!ch->leaf) return backwardSearchTile(static_cast<const Block*>(ch), pos, segEnd, q, tile);
                if (q.has(static_cast<const Seg*>(ch))) tile = static_cast<const Seg*>(ch);  // (removed or not)
                return;
            }
            if (const Seg* t = edgeTile(ch, q, false)) tile = t;
            segEnd = segpos;
        }
    }
    // the tile's local position (getPosition), or -1 when there is none
    int findTile(int pos, int key, const uint8_t* vmask, bool preceding) const {
        const TileQ q{key, vmask};
        const Seg* tile = nullptr;
        if (preceding) {
            searchTile(root, pos, q, tile);
        } else {
            const int len = localNodeLen(root);
            if (pos > len) return -1;
            backwardSearchTile(root, pos, len, q, tile);
        }
        if (!tile) return -1;
        int at = 0;
        bool found = false;
        walkSegs(root, [&](const Seg* s) {
            if (s == tile) found = true;
            if (!found) at += localLen(s);
        });
        return at;
    }

    // ------------------------------------------------------------------- getStackContext
    // Client.getStackContext -> MergeTree.getStackContext (client.ts:946-948, mergeTree.ts:1750-1760)
    // for one range label: search (:1797-1829) with leaf action recordRangeLeaf and shift action
    // rangeShift (:965-994) -- a shifted leaf applies itself when live, a shifted block applies its
    // HierMergeBlock rangeStacks (addNodeReferences :263-318, built from its live markers) through
    // applyStackDelta; applyRangeReference (:246-261): NestBegin pushes, an end pops a NestBegin
    // top and is pushed otherwise.  A range marker: refType NestBegin | NestEnd (ops.ts:8) whose
    // "referenceRangeLabels" (property `key`) value id is in `vmask` (hasRangeLabel).
    static void applyRange(std::vector<const Seg*>& st, const Seg* m) {
        const uint8_t rt = (uint8_t)m->text[0];
        if (rt & 2u) st.push_back(m);
        else if (!st.empty() && ((uint8_t)st.back()->text[0] & 2u)) st.pop_back();
        else st.push_back(m);
    }
    static bool rangeMarker(const Seg* s, const TileQ& q) {
        if (!s->marker || !s->text.size() || !((uint8_t)s->text[0] & 6u)) return false;
        return q.hasv(s->props[q.key]);
    }
    // a shifted leaf's contribution, or a block's rangeStacks entry for the label: the fold of its
    // cached markers (Block::snap, with their labels at its last blockUpdate; folding the block's
    // reduced stack is folding its markers, applyStackDelta)
    static std::vector<const Seg*> blockStack(const Node* n, const TileQ& q) {
        std::vector<const Seg*> st;
        if (n->leaf) {
            const Seg* s = static_cast<const Seg*>(n);
            if (localLen(s) > 0 && rangeMarker(s, q)) applyRange(st, s);
            return st;
        }
        for (const Snap& e : static_cast<const Block*>(n)->snap)
            if (((uint8_t)e.seg->text[0] & 6u) && q.hasv(e.props[q.key])) applyRange(st, e.seg);
        return st;
    }
    void searchRange(const Block* b, int pos, const TileQ& q, std::vector<const Seg*>& st) const {
        for (int i = 0; i < b->childCount; i++) {
            const Node* ch = b->children[i];
            const int len = localNodeLen(ch);
            if (pos < len) {
                if (!ch->leaf) return searchRange(static_cast<const Block*>(ch), pos, q, st);
                if (rangeMarker(static_cast<const Seg*>(ch), q)) applyRange(st, static_cast<const Seg*>(ch));
                return;  // recordRangeLeaf
            }
            for (const Seg* m : blockStack(ch, q)) applyRange(st, m);  // rangeShift
            pos -= len;
        }
    }
    // the label's stack bottom to top as (local position, refType)
    std::vector<std::pair<int, int>> stackContext(int pos, int key, const uint8_t* vmask) const {
        const TileQ q{key, vmask};
        std::vector<const Seg*> st;
        searchRange(root, pos, q, st);
        std::vector<std::pair<int, int>> out;
        for (const Seg* m : st) {
            int at = 0;
            bool found = false;
            walkSegs(root, [&](const Seg* s) {
                if (s == m) found = true;
                if (!found) at += localLen(s);
            });
            out.emplace_back(at, (int)(uint8_t)m->text[0]);
        }
        return out;
    }
};

// ------------------------------------------------------------------ checksum
inline uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// fnv1a over UTF-16 code units (h ^= unit): for text up to U+00FF, the fnv1a of its Latin-1 bytes
inline uint64_t fnv1a(const std::u16string& t) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (char16_t u : t) {
        h ^= (uint16_t)u;
        h *= 0x100000001B3ull;
    }
    return h;
}

// the wide terms of the segment hash (restated from DESIGN.md "Checksum"; the device's statement is
// fluidframework_amd/csrc/mt_checksum.h)
inline uint64_t mt_ovl_term(uint64_t mask, uint64_t ovx) { return ovx ? mask ^ mix64(ovx ^ 0x4F56584944530000ull) : mask; }
inline uint64_t mt_props_term(const uint64_t* w) {  // w: the 8 words of keys 0..31 (lo, hi per 8 keys)
    uint64_t t = w[0];
    if (w[1] | w[2] | w[3])
        t ^= mix64(mix64(w[1] ^ 0x1111111111111111ull) ^ mix64(w[2] ^ 0x2222222222222222ull) ^
                   mix64(w[3] ^ 0x3333333333333333ull));
    if (w[4] | w[5] | w[6] | w[7])
        t ^= mix64(mix64(w[4] ^ 0x4444444444444444ull) ^ mix64(w[5] ^ 0x5555555555555555ull) ^
                   mix64(w[6] ^ 0x6666666666666666ull) ^ mix64(w[7] ^ 0x7777777777777777ull));
    return t;
}

}  // namespace

// Shared definition with the device code (fluidframework_amd/csrc/mt_checksum.h); DESIGN.md.
uint64_t mto_seg_hash(uint64_t idx, uint64_t text_hash, int32_t seq, int32_t client, int32_t rseq,
                      int32_t rclient, uint64_t overlap, uint64_t props_lo, uint32_t props_defined) {
    uint64_t b = (uint64_t)(uint32_t)seq | ((uint64_t)(uint32_t)client << 32);
    uint64_t c = (uint64_t)(uint32_t)rseq | ((uint64_t)(uint32_t)rclient << 32);
    uint64_t h = mix64(text_hash ^ (idx * 0xD6E8FEB86659FD93ull));
    h = mix64(h ^ b);
    h = mix64(h ^ c);
    h = mix64(h ^ overlap);
    h = mix64(h ^ props_lo ^ ((uint64_t)props_defined << 63));
    return h;
}

namespace {

struct DocChecksum {
    uint64_t seg_sum = 0, tree_sum = 0;
    uint32_t nsegs = 0;
};

uint64_t finish_checksum(const DocChecksum& d, int32_t currentSeq, int32_t minSeq) {
    uint64_t s = mix64(d.seg_sum) ^ mix64(d.tree_sum ^ 0x5851F42D4C957F2Dull);
    s ^= mix64((uint64_t)(uint32_t)currentSeq | ((uint64_t)(uint32_t)minSeq << 32));
    return mix64(s ^ d.nsegs);
}

uint64_t doc_checksum(const Doc& doc) {
    DocChecksum d;
    uint64_t idx = 0;
    Doc::walkSegs(doc.root, [&](const Seg* s) {
        // the wide terms (DESIGN.md "Checksum"): u16 value ids and keys 8..31 as the device's eight
        // u64 property words, overlap ids >= 64 as its ascending byte list
        uint64_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < kMaxKeys; k++) {
            w[(k >> 3) * 2] |= (uint64_t)(s->props[k] & 0xFF) << (8 * (k & 7));
            w[(k >> 3) * 2 + 1] |= (uint64_t)(s->props[k] >> 8) << (8 * (k & 7));
        }
        // (mt_ovx_hash: up to eight ids below 256 as their byte list, any other list folded)
        uint64_t ovx = 0, fold = 0x9E3779B97F4A7C15ull;
        bool small = true;
        for (size_t q = 0; q < s->ovx.size(); q++) {
            const uint32_t v = s->ovx[q];
            if (v > 255u || q >= 8) small = false;
            else ovx |= (uint64_t)v << (8 * q);
            fold = mix64(fold ^ v);
        }
        if (!small) ovx = fold ? fold : 1ull;
        const uint64_t th = fnv1a(s->text) ^ (s->marker ? 0x4D41524B45520000ull : 0ull);
        d.seg_sum += mto_seg_hash(idx++, th, s->seq, s->client,
                                  s->removed ? s->rseq : -1, s->removed ? s->rclient : -1,
                                  mt_ovl_term(s->overlap, ovx), mt_props_term(w),
                                  s->props_defined);
    });
    d.nsegs = (uint32_t)idx;
    // block shape, level order (root level first), DESIGN.md
    std::vector<const Block*> lvl{doc.root};
    uint64_t level = 0;
    while (!lvl.empty()) {
        std::vector<const Block*> nxt;
        for (size_t b = 0; b < lvl.size(); b++) {
            d.tree_sum += mix64((uint64_t)lvl[b]->childCount ^ ((uint64_t)b << 8) ^ (level << 56));
            for (int i = 0; i < lvl[b]->childCount; i++)
                if (!lvl[b]->children[i]->leaf) nxt.push_back(static_cast<const Block*>(lvl[b]->children[i]));
        }
        lvl.swap(nxt);
        level++;
    }
    return finish_checksum(d, doc.currentSeq, doc.minSeq);
}

// a JSON string of UTF-16 code units: ASCII as itself, every other unit (surrogate halves
// included) as \\uXXXX -- pure ASCII output, any JS string representable
void json_escape(std::string& o, const std::u16string& s) {
    o += '"';
    for (char16_t u : s) {
        const unsigned c = (uint16_t)u;
        if (c == '"' || c == '\\') {
            o += '\\';
            o += (char)c;
        } else if (c < 0x20 || c >= 0x7F) {
            char buf[8];
            snprintf(buf, sizeof buf, "\\u%04x", c);
            o += buf;
        } else {
            o += (char)c;
        }
    }
    o += '"';
}

std::string doc_state_json(const Doc& doc) {
    std::string o = "{\"seq\":" + std::to_string(doc.currentSeq) + ",\"msn\":" + std::to_string(doc.minSeq) +
                    ",\"segs\":[";
    bool first = true;
    Doc::walkSegs(doc.root, [&](const Seg* s) {
        if (!first) o += ',';
        first = false;
        o += '[';
        if (s->marker)  // {"marker": refType}
            o += "{\"marker\":" + std::to_string((unsigned char)s->text[0]) + "}";
        else
            json_escape(o, s->text);
        o += ',' + std::to_string(s->seq) + ',' + std::to_string(s->client) + ',';
        o += (s->removed ? std::to_string(s->rseq) : "-1") + ',';
        o += (s->removed ? std::to_string(s->rclient) : "-1") + ",[";
        bool f2 = true;
        auto put = [&](int c) {
            if (!f2) o += ',';
            f2 = false;
            o += std::to_string(c);
        };
        for (int c = 0; c < 64; c++)
            if ((s->overlap >> c) & 1) put(c);
        for (uint16_t c : s->ovx) put(c);
        o += "],";
        if (!s->props_defined) {
            o += "null";
        } else {
            o += '{';
            bool f3 = true;
            for (int k = 0; k < kMaxKeys; k++)
                if (s->props[k]) {
                    if (!f3) o += ',';
                    f3 = false;
                    o += "\"k" + std::to_string(k) + "\":" + std::to_string(s->props[k]);
                }
            o += '}';
        }
        o += ']';
    });
    o += "],\"tree\":[";
    std::vector<const Block*> lvl{doc.root};
    bool f4 = true;
    while (!lvl.empty()) {
        std::vector<const Block*> nxt;
        if (!f4) o += ',';
        f4 = false;
        o += '[';
        for (size_t b = 0; b < lvl.size(); b++) {
            if (b) o += ',';
            o += std::to_string(lvl[b]->childCount);
            for (int i = 0; i < lvl[b]->childCount; i++)
                if (!lvl[b]->children[i]->leaf) nxt.push_back(static_cast<const Block*>(lvl[b]->children[i]));
        }
        o += ']';
        lvl.swap(nxt);
    }
    o += "]}";
    return o;
}

// -------------------------------------------------------------------- generator
// Observer-driven synthetic op logs (spec in DESIGN.md "Synthetic workloads").
// Every random draw is a counter-based hash r(doc, op, slot) so the device generator
// (fluidframework_amd/csrc/mt_synth.h, used by bench.py) produces the identical stream.
struct Gen {
    uint64_t key;
    explicit Gen(uint32_t seed, uint32_t doc) { key = mto_rng_key(seed, doc); }
    uint64_t r(uint32_t op, uint32_t slot) const { return mto_rng(key, op, slot); }
    uint32_t u(uint32_t op, uint32_t slot, uint32_t lo, uint32_t hi) const {  // inclusive
        return lo + (uint32_t)(((r(op, slot) >> 32) * (uint64_t)(hi - lo + 1)) >> 32);
    }
    bool p(uint32_t op, uint32_t slot, double prob) const {
        return (double)(r(op, slot) >> 11) * (1.0 / 9007199254740992.0) < prob;
    }
};
}  // namespace

// ============================================================================ C ABI
struct mto_engine {
    std::vector<Doc> docs;
};

extern "C" {

mto_engine* mto_create(uint32_t n_docs) {
    auto* e = new mto_engine();
    e->docs.resize(n_docs);
    return e;
}
void mto_destroy(mto_engine* e) { delete e; }

static void apply_range(mto_engine* e, const mt_op_rec* ops, const uint8_t* payload, const uint32_t* row_ptr,
                        uint32_t d0, uint32_t d1) {
    for (uint32_t d = d0; d < d1; d++) {
        Doc& doc = e->docs[d];
        for (uint32_t i = row_ptr[d]; i < row_ptr[d + 1]; i++) {
            bool last = !(ops[i].flags & MT_F_GROUP_MORE);
            doc.applyOp(ops[i], payload, last);
        }
    }
}

int mto_apply(mto_engine* e, const mt_op_rec* ops, const uint8_t* payload, const uint32_t* row_ptr,
              uint32_t n_docs, int n_threads) {
    if (n_docs > e->docs.size()) return MT_ERR_ARG;
    if (n_threads <= 1) {
        apply_range(e, ops, payload, row_ptr, 0, n_docs);
        return MT_OK;
    }
    std::atomic<uint32_t> next{0};
    const uint32_t chunk = 64;
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; t++)
        th.emplace_back([&] {
            for (;;) {
                uint32_t d0 = next.fetch_add(chunk);
                if (d0 >= n_docs) break;
                apply_range(e, ops, payload, row_ptr, d0, std::min(n_docs, d0 + chunk));
            }
        });
    for (auto& x : th) x.join();
    return MT_OK;
}

void mto_checksums(mto_engine* e, uint64_t* out, uint32_t n_docs) {
    for (uint32_t d = 0; d < n_docs && d < e->docs.size(); d++) out[d] = doc_checksum(e->docs[d]);
}

int mto_load(mto_engine* e, uint32_t doc, const mt_load_seg* segs, uint32_t n_segs, const uint8_t* text,
             int32_t min_seq, int32_t cur_seq) {
    if (doc >= e->docs.size()) return -1;
    e->docs[doc] = Doc();
    e->docs[doc].reload(segs, n_segs, text, min_seq, cur_seq);
    return 0;
}

// Client.findTile of document `doc` (tile labels: property `key`, value ids in the 256-bit vmask)
int32_t mto_find_tile(mto_engine* e, uint32_t doc, int32_t pos, uint32_t key, const uint8_t* vmask, int preceding) {
    return e->docs[doc].findTile(pos, (int)key, vmask, preceding != 0);
}

// Client.getStackContext of document `doc` for one range label (property `key`, value ids in vmask):
// writes up to cap (position, refType) pairs bottom to top into out; returns the stack depth
uint32_t mto_stack_context(mto_engine* e, uint32_t doc, int32_t pos, uint32_t key, const uint8_t* vmask, int32_t* out,
                           uint32_t cap) {
    const auto st = e->docs[doc].stackContext(pos, (int)key, vmask);
    for (uint32_t i = 0; i < st.size() && i < cap; i++) {
        out[2 * i] = st[i].first;
        out[2 * i + 1] = st[i].second;
    }
    return (uint32_t)st.size();
}

// the ops regeneratePendingOp produced for document `doc` (records with seq -2) as JSON
// [[record index, [[type, pos1, pos2, text | null, props | null, flags], ...]], ...]
uint64_t mto_doc_regen_json(mto_engine* e, uint32_t doc, char* buf, uint64_t cap) {
    const std::string j = "[" + e->docs[doc].regenJson + "]";
    if (buf && cap) std::memcpy(buf, j.data(), std::min<uint64_t>(cap, j.size()));
    return j.size();
}

// delta / maintenance events (mt_event form) of every document from now on
void mto_record_events(mto_engine* e, int on) {
    for (auto& d : e->docs) d.rec = on != 0;
}
// copies up to cap of document `doc`'s recorded events; returns how many it has
uint64_t mto_events(mto_engine* e, uint32_t doc, mt_event* out, uint64_t cap) {
    const auto& v = e->docs[doc].events;
    if (out) std::memcpy(out, v.data(), sizeof(mt_event) * std::min<uint64_t>(cap, v.size()));
    return v.size();
}

int mto_doc_error(mto_engine* e, uint32_t doc, int32_t* seq) {
    *seq = e->docs[doc].err_seq;
    return e->docs[doc].err;
}

// Writes the canonical state JSON; returns required length (including NUL).
uint64_t mto_doc_state(mto_engine* e, uint32_t doc, char* buf, uint64_t cap) {
    std::string s = doc_state_json(e->docs[doc]);
    if (buf && cap) {
        uint64_t n = std::min<uint64_t>(cap - 1, s.size());
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return s.size() + 1;
}

// the text as a JSON string (ASCII; json_escape)
uint64_t mto_doc_text(mto_engine* e, uint32_t doc, char* buf, uint64_t cap) {
    std::string s;
    json_escape(s, e->docs[doc].text());
    if (buf && cap) {
        uint64_t n = std::min<uint64_t>(cap - 1, s.size());
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return s.size() + 1;
}

// entries of the document's zamboni LRU heap (diagnostics: tools/class_bind.py)
uint32_t mto_doc_heap(mto_engine* e, uint32_t doc) { return (uint32_t)(e->docs[doc].heap.size() - 1); }

uint32_t mto_doc_nsegs(mto_engine* e, uint32_t doc) {
    uint32_t n = 0;
    Doc::walkSegs(e->docs[doc].root, [&](const Seg*) { n++; });
    return n;
}

// --------------------------------------------------------------------------- generator
// Pass 1 (ops == nullptr): counts ops/payload per doc into n_ops[d], n_payload[d].
// Pass 2: writes records and payload at the given per-doc offsets (payload_off is global).
static void gen_doc(const mt_synth_cfg& cfg, uint32_t doc, mt_op_rec* ops, uint8_t* payload, uint64_t pay_base,
                    uint32_t* n_ops_out, uint64_t* n_pay_out) {
    Gen g(cfg.seed, doc);
    Doc st;  // the observer, driving positions
    const uint32_t C = cfg.n_clients;
    std::vector<int32_t> cref(C + 1, 0);  // latest refSeq per client (deli clientSeqManager)
    int32_t stall_until = 0;
    int32_t seq = 0;
    uint32_t nops = 0;
    uint64_t npay = 0;
    uint8_t buf[512];
    for (uint32_t i = 0; i < cfg.ops_per_doc; i++) {
        mt_op_rec rec{};
        uint32_t len = mto_gen_op(cfg, g.key, i, seq, cref.data(), &stall_until, rec, buf,
            [&](int32_t R, int32_t c) { return st.length(R, c); },
            [&](int32_t R, int32_t c, uint32_t pick, int32_t* pos, int32_t* plen) {
                // pick-th (0-based) segment visible to (R,c) that was removed concurrently (rseq > R);
                // returns the count when pick == UINT32_MAX
                int p0 = 0;
                uint32_t cnt = 0;
                Doc::walkSegs(st.root, [&](const Seg* s) {
                    int vl = Doc::segLen(s, R, c);
                    if (vl > 0 && s->removed && s->rseq > R) {
                        if (cnt == pick) {
                            *pos = p0;
                            *plen = vl;
                        }
                        cnt++;
                    }
                    p0 += vl;
                });
                return cnt;
            });
        seq = rec.seq;
        rec.payload_off = (uint32_t)(pay_base + npay);
        if (ops) {
            ops[nops] = rec;
            std::memcpy(payload + pay_base + npay, buf, len);
        }
        mt_op_rec local = rec;
        local.payload_off = 0;
        st.applyOp(local, buf, true);
        nops++;
        npay += len;
    }
    if (n_ops_out) *n_ops_out = nops;
    if (n_pay_out) *n_pay_out = npay;
}

int mto_generate(const mt_synth_cfg* cfg, uint32_t d0, uint32_t n_docs, mt_op_rec* ops, uint8_t* payload,
                 uint32_t* row_ptr, uint64_t* pay_ptr, int n_threads) {
    // pass 1 would duplicate the work; the generator is deterministic per doc, so sizes are
    // computed by a dry run in parallel, then the write pass runs with known offsets.
    std::vector<uint32_t> nops(n_docs);
    std::vector<uint64_t> npay(n_docs);
    auto run = [&](bool write) {
        std::atomic<uint32_t> next{0};
        std::vector<std::thread> th;
        int nt = std::max(1, n_threads);
        for (int t = 0; t < nt; t++)
            th.emplace_back([&] {
                for (;;) {
                    uint32_t i = next.fetch_add(16);
                    if (i >= n_docs) break;
                    for (uint32_t d = i; d < std::min(n_docs, i + 16); d++) {
                        if (write) gen_doc(*cfg, d0 + d, ops + row_ptr[d], payload, pay_ptr[d], nullptr, nullptr);
                        else gen_doc(*cfg, d0 + d, nullptr, nullptr, 0, &nops[d], &npay[d]);
                    }
                }
            });
        for (auto& x : th) x.join();
    };
    if (!ops) {
        run(false);
        row_ptr[0] = 0;
        pay_ptr[0] = 0;
        for (uint32_t d = 0; d < n_docs; d++) {
            row_ptr[d + 1] = row_ptr[d] + nops[d];
            pay_ptr[d + 1] = pay_ptr[d] + npay[d];
        }
        return MT_OK;
    }
    run(true);
    return MT_OK;
}

}  // extern "C"
