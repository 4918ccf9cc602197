// mt_engine.cpp -- host side of libmtgpu.so: the C-ABI declared in include/mtgpu.h.
//
// Owns the device-resident document states (mt_state.h), stages CSR op batches into HBM and
// drives the apply kernels on one HIP stream.  A batch is applied as a sequence of launches of
// at most `ops_per_launch` ops per document (the serving tick; 0 = the whole batch in one
// launch).  Before every launch the documents with work are binned by the LDS capacity class
// they need (mt_bin_kernel), so small documents run at high occupancy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtgpu.h"
#include "mt_checksum.h"
#include "mt_state.h"

extern "C" hipError_t mt_launch_apply(int cap_class, const mt_gstate* g, const mt_op_rec* ops, const uint8_t* payload,
                                      const uint32_t* row_ptr, const uint32_t* doc_ids, uint32_t n_docs,
                                      uint32_t op_lo, uint32_t op_cnt, hipStream_t stream);
extern "C" hipError_t mt_launch_apply_reg(int cap_class, int form, const mt_gstate* g, const mt_op_rec* ops,
                                          const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                          uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, hipStream_t stream);
extern "C" size_t mt_lds_bytes(int cap_class);
extern "C" hipError_t mt_launch_apply_loc(int cap_class, const mt_gstate* g, const mt_op_rec* ops, const uint8_t* payload,
                                          const uint32_t* row_ptr, const uint32_t* doc_ids, uint32_t n_docs,
                                          uint32_t op_lo, uint32_t op_cnt, hipStream_t stream);
extern "C" hipError_t mt_launch_apply_big(int cap_class, const mt_gstate* g, const mt_op_rec* ops,
                                          const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                          uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, uint8_t* ws,
                                          hipStream_t stream);
extern "C" hipError_t mt_launch_apply_wide(int cap_class, const mt_gstate* g, const mt_op_rec* ops,
                                           const uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                           uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, uint8_t* ws, int xl,
                                           hipStream_t stream);
extern "C" size_t mt_lds_bytes_wide(int cap_class);
extern "C" hipError_t mt_launch_apply_loc_big(int cap_class, int gw, const mt_gstate* g, const mt_op_rec* ops,
                                              const uint8_t* payload, const uint32_t* row_ptr,
                                              const uint32_t* doc_ids, uint32_t n_docs, uint32_t op_lo,
                                              uint32_t op_cnt, uint8_t* ws, hipStream_t stream);
extern "C" size_t mt_lds_bytes_loc(int cap_class, int gw);
extern "C" hipError_t mt_launch_init(const mt_gstate* g, uint32_t n_docs, hipStream_t st);
extern "C" hipError_t mt_launch_label_keys(const mt_gstate* g, uint32_t d0, uint32_t d1, uint32_t keys, hipStream_t st);
extern "C" hipError_t mt_launch_load(const mt_gstate* g, uint32_t n, const uint32_t* doc_ids, const uint32_t* row_ptr,
                                     const mt_load_seg* segs, const uint8_t* text, const int32_t* min_seq,
                                     const int32_t* cur_seq, hipStream_t st);
extern "C" hipError_t mt_launch_bin(const mt_gstate* g, const uint32_t* row_ptr, uint32_t n_docs, uint32_t op_lo,
                                    uint32_t op_cnt, const int32_t* classes, int n_classes, int first_lds,
                                    int first_wide, uint32_t* counts, uint32_t* ids, const mt_op_rec* ops,
                                    const uint8_t* payload, unsigned long long* acc, hipStream_t st);
extern "C" hipError_t mt_launch_checksum(const mt_gstate* g, uint32_t n_docs, uint64_t* out, hipStream_t st);
extern "C" hipError_t mt_launch_stacks(const mt_gstate* g, const mt_tile_query* q, uint32_t n, uint32_t cap,
                                       mt_stack_item* items, uint32_t* depth, hipStream_t st);
extern "C" hipError_t mt_launch_tiles(const mt_gstate* g, const mt_tile_query* q, uint32_t n, mt_tile_result* out,
                                      hipStream_t st);
extern "C" hipError_t mt_launch_resolve(const mt_gstate* g, const mt_pos_query* q, uint32_t n, uint32_t n_docs,
                                        mt_pos_result* out,
                                        hipStream_t st);
extern "C" hipError_t mt_launch_seginfo(const mt_gstate* g, const uint32_t* docs, const int32_t* ords, uint32_t n,
                                        mt_seg_info* out, hipStream_t st);
extern "C" hipError_t mt_launch_events_pack(const mt_gstate* g, uint32_t n_docs, const uint64_t* off, mt_event* out,
                                            hipStream_t st);
extern "C" hipError_t mt_launch_fixup(const mt_gstate* g, const mt_op_rec* ops, uint32_t n_docs, hipStream_t st);
extern "C" hipError_t mt_launch_scan_records(const mt_op_rec* ops, uint64_t n_ops, uint64_t payload_bytes,
                                             uint32_t* flags, hipStream_t st);
extern "C" hipError_t mt_launch_snapshot(const mt_gstate* g, uint32_t d0, uint32_t n_docs, uint32_t cap,
                                         uint32_t* specs, uint32_t* counts, hipStream_t st);
extern "C" hipError_t mt_launch_gen(int cap_class, const mt_gstate* g, const mt_synth_cfg* cfg, uint32_t doc_id_base,
                                    const uint32_t* gids, int32_t* cref,
                                    int32_t* stall, uint32_t* pay_used, uint32_t paycap, mt_op_rec* ops,
                                    uint8_t* payload, const uint32_t* row_ptr, const uint32_t* doc_ids,
                                    uint32_t n_docs, uint32_t op_lo, uint32_t op_cnt, hipStream_t stream);

namespace {
// register engine <= 1024, LDS engine 2048, the LDS engine's HBM-workspace form above (only the
// classes with CAP <= the engine's seg_capacity are used: mt_engine::n_classes)
// (the register classes step by 64 slots -- K = 2 ... 16 registers per field -- so a document pays
// for the slots it can reach in a launch, not for the next power of two)
// (the largest class is 64 K - 64 slots: the LDS engine's slot indices and the heap's positions
// between launches are u16, 0xFFFF being MT_DEAD_SLOT)
const int32_t kClasses[] = {128, 192, 256, 320, 384, 448, 512, 576, 640, 704, 768, 832, 896, 960, 1024,
                            2048, 4096, 8192, 16384, 32768, 65472};
constexpr int kNumClasses = 21;
constexpr int kLdsClasses = 16;  // classes an LDS-resident kernel serves (the generator's)
constexpr int kFirstLds = 15;    // index of the 2048 class: the first the register engine does not serve
constexpr int kMaxSegCap = 65472;  // (the LDS engine's slot indices are u16: Lds::order / hslot)
// bins of a tick (mt_bin_kernel): the classes, the editing documents, and the wide documents of the
// classes from 2048 up (the LDS engine's wide form, include/mtgpu.h "limits")
// the wide form serves the classes from 256 segments on: up to 512 staged in LDS, above in the HBM
// workspace (mt_launch_apply_wide)
constexpr int kFirstWide = 2;
constexpr int kWideClasses = kNumClasses - kFirstWide;
// ... and, after those, per register class: the documents that need the LDS engine there (declared
// label keys), run by the LDS engine at that class's capacity, then the documents with client ids
// above 32, run by the register engine's C64 form (mt_bin_kernel)
// (then the editing documents that fit 256 / 512 slots: the editing form at that size; then those
// above MT_LOC_CAP = 1024: its HBM-workspace form at 2048 / 4096; then those past 64 pending edits
// (MT_WIDE_GROUPS): the HBM-workspace form with 4 group-mask words per slot at 1024 / 4096; then
// both forms at 8192)
constexpr int kLocForms = 8;
const int32_t kLocCaps[kLocForms] = {256, 512, 2048, 4096, 1024, 4096, 8192, 8192};
const int32_t kLocGW[kLocForms] = {1, 1, 1, 1, MT_LOC_GW, MT_LOC_GW, 1, MT_LOC_GW};
constexpr int kBuckets = kNumClasses + 1 + kWideClasses + 2 * kFirstLds + kLocForms;
// binning's counters: one per bucket, then per wide bucket the documents that stage the wide form's
// extension (mt_state.h MT_WIDE_XK / MT_WIDE_XO) -- their launch takes an HBM region for it
constexpr int kCounts = kBuckets + kWideClasses;
// per-class statistics: the classes, the editing bucket, the LDS engine inside each register class,
// the register engine's C64 form per class, the other editing forms
constexpr int kStatClasses = kNumClasses + 1 + 2 * kFirstLds + kLocForms + kWideClasses;
constexpr int kStatWide = kNumClasses + 1 + 2 * kFirstLds + kLocForms;  // the wide form's entries
// {CAP, LB, IB, H} per class: at most mt::Lds<lds_cap(CAP)>'s and mtr::RLds<CAP/64>'s (the 128 and 192
// classes take the 256 class's block and heap limits, which both hold: with CAP / 2 blocks and
// CAP / 8 + 8 interior blocks no b = 32 launch fits them)
const int32_t kClassParams[kNumClasses * 4] = {
    128, 128, 40, 192, 192, 128, 40, 192, 256, 128, 40, 192, 320, 160, 48, 224,
    384, 192, 56, 256, 448, 224, 64, 288, 512, 256, 72, 320, 576, 288, 80, 352,
    640, 320, 88, 384, 704, 352, 96, 416, 768, 384, 104, 448, 832, 416, 112, 480,
    896, 448, 120, 512, 960, 480, 128, 544, 1024, 512, 136, 576, 2048, 1024, 264, 1088,
    4096, 2048, 520, 2112, 8192, 4096, 1032, 4160, 16384, 8192, 2056, 8256, 32768, 16384, 4104, 16448,
    65472, 32736, 8192, 32800};
// the LDS engine serves the classes at 256 / 384 / 512 / 640 / 768 / 896 / 1024 / 2048 slots: the
// next one up serves a class.  Its LDS (≈ 55 B per slot) sets the waves per CU: the steps between 512
// and 1024 keep documents of 520-900 slots at 3-4 waves per CU instead of the 1024 form's 2.
int lds_cap(int cap) {
    static const int caps[] = {256, 384, 512, 640, 768, 896, 1024};  // (128: the 256 class's limits)
    for (int c : caps)
        if (cap <= c) return c;
    return cap;
}
}  // namespace

struct mt_batch {
    mt_op_rec* ops = nullptr;
    uint8_t* payload = nullptr;
    uint32_t* row_ptr = nullptr;
    uint64_t n_ops = 0, payload_bytes = 0;
    uint32_t n_docs = 0;
    uint32_t max_ops_per_doc = 0;
    bool wide = false;  // some record needs the wide form (its documents' wide state is allocated first)
};

struct mt_engine {
    mt_cfg cfg{};
    hipStream_t stream = nullptr;
    mt_gstate g{};
    uint32_t n_docs = 0;
    std::vector<void*> allocs;
    int32_t* d_classes = nullptr;
    uint32_t* d_counts = nullptr;
    uint32_t* d_ids = nullptr;
    uint32_t* h_counts = nullptr;  // pinned
    unsigned long long* d_acc = nullptr;
    std::vector<hipEvent_t> kev;   // per apply launch: start/stop pairs
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f, last_wall_ms = 0.f;
    // per capacity class, plus one entry for the editing documents' bucket (index kNumClasses)
    float cls_ms[kStatClasses] = {0};
    uint32_t cls_launches[kStatClasses] = {0};
    uint64_t cls_bytes[kStatClasses] = {0};
    std::vector<int> kev_cls;
    uint32_t last_launches = 0;
    uint64_t last_bytes = 0;
    // register-resident engine (mt_apply_reg.hip) for classes up to kRegMaxCap segments; the
    // LDS engine (mt_apply.hip) above that, or everywhere with MTGPU_ENGINE=lds
    bool use_reg = true;
    bool reg_default = true;       // use_reg when not recording delta events (mt_events_enable)
    int n_classes = kLdsClasses;   // classes with CAP <= seg_capacity
    int first_lds = kFirstLds;     // first class not served by the register engine
    uint8_t* ws = nullptr;         // HBM workspace of the classes above 2048 segments
    size_t ws_bytes = 0;
    // the capacity classes of one tick touch disjoint documents: each runs on its own stream
    // (fork/join around the tick) so the small classes and every class's tail overlap;
    // MTGPU_SERIAL=1 keeps them on the engine stream, one after another
    bool concurrent = true;
    bool desc_order = true;  // class kernels launched largest capacity first (see apply_launches)
    hipStream_t side[kNumClasses] = {};
    hipEvent_t fork_ev = nullptr, join_ev[kNumClasses] = {};
    uint64_t gen = 0;  // bumped by every call that can change document state (snap_cache's key)
    std::vector<uint16_t> lkeys;  // per document: its declared label keys (mt_set_label_keys), host copy
    // the editing documents' pool rows (mt_state.h locbig / locgx): host copies, rows in use, rows held
    std::vector<uint32_t> h_locbig, h_locgx, h_bucket;
    uint32_t nbig = 0, bigcap = 0, ngx = 0, gxcap = 0;
    std::vector<uint32_t> free_big, free_gx;  // rows given back by reloaded documents, reused first
    // mt_submit_ticks: a ring of device slots; tick k is copied into slot k % kRing on the h2d
    // stream while the ticks before it apply, and the slot is reused once its tick has applied (and
    // its tickets have gone back on the d2h stream)
    struct TickSlot {
        mt_op_rec* ops = nullptr;
        uint8_t* pay = nullptr;
        uint32_t* rp = nullptr;
        mt_raw_msg* msgs = nullptr;
        uint32_t* mrp = nullptr;
        mt_ticket* tk = nullptr;
        uint64_t ops_cap = 0, pay_cap = 0, msg_cap = 0;
        hipEvent_t ready = nullptr, applied = nullptr, drained = nullptr, ticketed = nullptr;
    } ring[6];
    hipStream_t h2d = nullptr, d2h = nullptr;
    uint32_t* d_scan = nullptr;  // the first tick's record check on the device (mt_scan_records_kernel)
    struct {  // mt_get_snapshots: the JSON of the last sizing call
        bool valid = false;
        uint64_t gen = 0;
        uint32_t d0 = 0, n = 0, chunk = 0, n_names = 0;
        const char* const* names = nullptr;
        std::string json;
        std::vector<uint64_t> off;
    } snap_cache;
};
static constexpr int32_t kRegMaxCap = 1024;

#define HIP_OK(x)                                                                                            \
    do {                                                                                                     \
        hipError_t e_ = (x);                                                                                 \
        if (e_ != hipSuccess) {                                                                              \
            fprintf(stderr, "libmtgpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return MT_ERR_HIP;                                                                               \
        }                                                                                                    \
    } while (0)

template <class T>
static mt_status dalloc(mt_engine* e, T** p, size_t count) {
    void* q = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc(&q, count * sizeof(T)) != hipSuccess) return MT_ERR_NOMEM;
    e->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return MT_OK;
}

// The wide documents' extra per-segment state (mt_state.h), allocated for every document the first
// time an engine sees wide content (a wide record or snapshot segment)
static mt_status ensure_wide(mt_engine* e) {
    if (e->g.ovx) return MT_OK;
    const size_t S = (size_t)e->cfg.max_docs * e->g.segcap;
    mt_gstate& g = e->g;
    mt_status st = MT_OK;
    if ((st = dalloc(e, &g.ph, S)) || (st = dalloc(e, &g.pxl, S)) || (st = dalloc(e, &g.pxh, S)) ||
        (st = dalloc(e, &g.pxx, S * 4)) || (st = dalloc(e, &g.chi, S)) ||
        (st = dalloc(e, &g.ovx, S * MT_OVX_WORDS))) {
        g.ovx = nullptr;  // (the kernels test ovx; the others are freed with the engine)
        return st;
    }
    return MT_OK;
}
// The editing documents' pools (mt_state.h): a document whose editing form needs more than
// MT_LOC_CAP slots gets a big-pool row, one past 64 pending edits a group-pool row, when it first
// reaches such a form; the pools grow geometrically (a grow re-allocates and copies the rows in use;
// nothing runs on the engine's streams meanwhile).  Memory scales with the documents that reach
// those forms, not with max_docs.
static bool pool_alloc(void** out, size_t bytes) {
    *out = nullptr;
    return hipMalloc(out, bytes) == hipSuccess;
}
static bool grow_big(mt_engine* e, uint32_t rows) {
    mt_gstate& g = e->g;
    const size_t C = MT_LOC_BIGCAP, n = (size_t)rows * C, u = (size_t)e->nbig * C;
    void *gm = nullptr, *pk = nullptr, *ct = nullptr, *lsq = nullptr;
    if (!pool_alloc(&gm, n * 8) || !pool_alloc(&pk, n * 8) || !pool_alloc(&ct, n * 4) || !pool_alloc(&lsq, n * 8)) {
        for (void* q : {gm, pk, ct, lsq})
            if (q) (void)hipFree(q);
        return false;
    }
    if (u && (hipMemcpy(gm, g.gmb, u * 8, hipMemcpyDeviceToDevice) != hipSuccess ||
              hipMemcpy(pk, g.pkb, u * 8, hipMemcpyDeviceToDevice) != hipSuccess ||
              hipMemcpy(ct, g.ctb, u * 4, hipMemcpyDeviceToDevice) != hipSuccess ||
              hipMemcpy(lsq, g.lsqb, u * 8, hipMemcpyDeviceToDevice) != hipSuccess)) {
        for (void* q : {gm, pk, ct, lsq}) (void)hipFree(q);
        return false;
    }
    for (void* q : {(void*)g.gmb, (void*)g.pkb, (void*)g.ctb, (void*)g.lsqb})
        if (q) (void)hipFree(q);
    g.gmb = (uint64_t*)gm;
    g.pkb = (uint64_t*)pk;
    g.ctb = (uint32_t*)ct;
    g.lsqb = (uint64_t*)lsq;
    e->bigcap = rows;
    return true;
}
static bool grow_gx(mt_engine* e, uint32_t rows) {
    mt_gstate& g = e->g;
    const size_t n = (size_t)rows * MT_LOC_BIGCAP * MT_LOC_GW, u = (size_t)e->ngx * MT_LOC_BIGCAP * MT_LOC_GW;
    void *gm = nullptr, *lx = nullptr;
    if (!pool_alloc(&gm, n * 8) || !pool_alloc(&lx, (size_t)rows * sizeof(mt_locx))) {
        for (void* q : {gm, lx})
            if (q) (void)hipFree(q);
        return false;
    }
    if (u && (hipMemcpy(gm, g.gmx, u * 8, hipMemcpyDeviceToDevice) != hipSuccess ||
              hipMemcpy(lx, g.locx, (size_t)e->ngx * sizeof(mt_locx), hipMemcpyDeviceToDevice) != hipSuccess)) {
        (void)hipFree(gm);
        (void)hipFree(lx);
        return false;
    }
    if (g.gmx) (void)hipFree(g.gmx);
    if (g.locx) (void)hipFree(g.locx);
    g.gmx = (uint64_t*)gm;
    g.locx = (mt_locx*)lx;
    e->gxcap = rows;
    return true;
}
// rows for `want` more documents: double the pool (at least 16 rows), else exactly what is needed;
// returns how many of them got rows
template <class Grow>
static uint32_t pool_reserve(uint32_t used, uint32_t cap, uint32_t want, Grow grow) {
    if (used + want <= cap) return want;
    const uint32_t need = used + want;
    if (grow(std::max<uint32_t>({need, 2 * cap, 16u}))) return want;
    if (grow(need)) return want;
    return cap > used ? cap - used : 0;
}
// Assigns the rows of one tick's editing buckets (bk: the bucket's index in d_ids); the documents that
// get no row halt in the kernel with MT_DERR_CAPACITY (mt_apply.hip loc_admit)
static mt_status assign_loc_rows(mt_engine* e, const uint32_t* ids, uint32_t cnt, bool big, bool gx) {
    mt_gstate& g = e->g;
    e->h_bucket.resize(cnt);
    HIP_OK(hipMemcpy(e->h_bucket.data(), ids, cnt * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint32_t> nb, ng;
    for (uint32_t d : e->h_bucket) {
        if (big && e->h_locbig[d] == MT_NO_ROW) nb.push_back(d);
        if (gx && e->h_locgx[d] == MT_NO_ROW) ng.push_back(d);
    }
    if (nb.empty() && ng.empty()) return MT_OK;
    HIP_OK(hipDeviceSynchronize());
    const uint32_t rb = std::min<uint32_t>((uint32_t)nb.size(), (uint32_t)e->free_big.size());
    const uint32_t kb = rb + pool_reserve(e->nbig, e->bigcap, (uint32_t)nb.size() - rb,
                                          [&](uint32_t r) { return grow_big(e, r); });
    for (uint32_t i = 0; i < kb; i++) {
        uint32_t r;
        if (i < rb) {
            r = e->free_big.back();
            e->free_big.pop_back();
        } else {
            r = e->nbig++;
        }
        const uint32_t d = nb[i];
        const size_t o = (size_t)r * MT_LOC_BIGCAP, s = (size_t)d * MT_LOC_CAP;
        HIP_OK(hipMemcpy(g.gmb + o, g.gm + s, MT_LOC_CAP * 8, hipMemcpyDeviceToDevice));
        HIP_OK(hipMemcpy(g.pkb + o, g.pk + s, MT_LOC_CAP * 8, hipMemcpyDeviceToDevice));
        HIP_OK(hipMemcpy(g.ctb + o, g.ct + s, MT_LOC_CAP * 4, hipMemcpyDeviceToDevice));
        HIP_OK(hipMemcpy(g.lsqb + o, g.lsq + s, MT_LOC_CAP * 8, hipMemcpyDeviceToDevice));
        e->h_locbig[d] = r;
        HIP_OK(hipMemcpy(g.locbig + d, &r, 4, hipMemcpyHostToDevice));
    }
    const uint32_t rg = std::min<uint32_t>((uint32_t)ng.size(), (uint32_t)e->free_gx.size());
    const uint32_t kg = rg + pool_reserve(e->ngx, e->gxcap, (uint32_t)ng.size() - rg,
                                          [&](uint32_t r) { return grow_gx(e, r); });
    for (uint32_t i = 0; i < kg; i++) {
        uint32_t r;
        if (i < rg) {
            r = e->free_gx.back();
            e->free_gx.pop_back();
        } else {
            r = e->ngx++;
        }
        const uint32_t d = ng[i];
        e->h_locgx[d] = r;
        HIP_OK(hipMemcpy(g.locgx + d, &r, 4, hipMemcpyHostToDevice));
    }
    return MT_OK;
}

// Documents that start over (mt_docs_load) give their pool rows back: the next document that needs
// such a form reuses them before the pools grow (its 1024-slot row is copied in then, as for a new
// row).  The host mirrors are updated per document; the device tables get one copy of the changed
// span each and one synchronization (not two round trips per document).
static mt_status release_loc_rows(mt_engine* e, const uint32_t* docs, uint32_t n) {
    uint32_t lo[2] = {UINT32_MAX, UINT32_MAX}, hi[2] = {0, 0};
    std::vector<uint32_t>* mirror[2] = {&e->h_locbig, &e->h_locgx};
    std::vector<uint32_t>* freel[2] = {&e->free_big, &e->free_gx};
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t d = docs[i];
        for (int k = 0; k < 2; k++) {
            if (d >= mirror[k]->size() || (*mirror[k])[d] == MT_NO_ROW) continue;
            freel[k]->push_back((*mirror[k])[d]);
            (*mirror[k])[d] = MT_NO_ROW;
            lo[k] = std::min(lo[k], d);
            hi[k] = std::max(hi[k], d + 1);
        }
    }
    uint32_t* dev[2] = {e->g.locbig, e->g.locgx};
    bool any = false;
    for (int k = 0; k < 2; k++) {
        if (lo[k] >= hi[k]) continue;
        HIP_OK(hipMemcpyAsync(dev[k] + lo[k], mirror[k]->data() + lo[k], 4ull * (hi[k] - lo[k]), hipMemcpyHostToDevice,
                              e->stream));
        any = true;
    }
    if (any) HIP_OK(hipStreamSynchronize(e->stream));
    return MT_OK;
}

// a record beyond the narrow limits (include/mtgpu.h "limits")
static bool wide_rec(const mt_op_rec& o) {
    if (o.type & MT_OP_WIDE) return true;
    if (MT_OP_TYPE(o) == MT_OP_LOAD) {
        const uint32_t c0 = MT_LOAD_CLIENT(o), c1 = MT_LOAD_RCLIENT(o);
        return (c0 != MT_CLIENT_NONCOLLAB && c0 >= MT_MAX_CLIENTS) || (o.pos2 >= 0 && c1 >= MT_MAX_CLIENTS);
    }
    return !MT_OP_IS_NOOP(o) && o.client >= MT_MAX_CLIENTS;
}
// Payload bounds (the kernels trust these) and whether any record needs the wide document form, in
// one pass; a big batch is checked on all host cores.  Result bit 0: a payload out of bounds, bit 1:
// wide.
static int scan_records(const mt_op_rec* ops, uint64_t n_ops, uint64_t payload_bytes) {
    auto scan_range = [&](uint64_t lo, uint64_t hi) {
        bool bad = false, wide = false;
        for (uint64_t i = lo; i < hi; i++) {
            bad |= (uint64_t)ops[i].payload_off + ops[i].payload_len > payload_bytes;
            wide |= wide_rec(ops[i]);
        }
        return (bad ? 1 : 0) | (wide ? 2 : 0);
    };
    const unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16u);
    if (n_ops < (1u << 20) || nt == 1) return scan_range(0, n_ops);
    std::vector<std::thread> th;
    std::vector<int> res(nt, 0);
    for (unsigned t = 0; t < nt; t++) th.emplace_back([&, t] { res[t] = scan_range(n_ops * t / nt, n_ops * (t + 1) / nt); });
    for (auto& x : th) x.join();
    int flags = 0;
    for (int r : res) flags |= r;
    return flags;
}
static uint32_t seg_client(const mt_load_seg& sg) { return sg.client | ((uint32_t)sg.client_hi << 8); }
static uint32_t seg_rclient(const mt_load_seg& sg) { return sg.rclient | ((uint32_t)sg.rclient_hi << 8); }
static bool wide_load_seg(const mt_load_seg& sg) {
    if ((sg.flags & MT_LSF_U16) || (seg_client(sg) >= MT_MAX_CLIENTS && seg_client(sg) != MT_CLIENT_NONCOLLAB) ||
        (sg.rseq >= 0 && seg_rclient(sg) >= MT_MAX_CLIENTS))
        return true;
    for (int k = 0; k < MT_MAX_KEYS_WIDE; k++)
        if ((sg.flags & MT_SF_PDEF) && (k >= MT_MAX_KEYS ? sg.props[k] != 0 : sg.props[k] > 255)) return true;
    return false;
}

extern "C" {

const char* mt_version(void) { return "libmtgpu 0.2 (gfx950)"; }

mt_status mt_engine_create(const mt_cfg* cfg, mt_engine** out) {
    if (!cfg || !out || cfg->max_docs == 0) return MT_ERR_ARG;
    // the register / LDS classes reach 2048 slots and read whole rows of that size
    if (cfg->seg_capacity != 0 && (cfg->seg_capacity < 2048 || cfg->seg_capacity > (uint32_t)kMaxSegCap))
        return MT_ERR_ARG;
    if (cfg->text_capacity > MT_MAX_TEXTCAP) return MT_ERR_ARG;  // (above 64 KiB: the LDS engine everywhere)
    HIP_OK(hipSetDevice(cfg->device));
    auto* e = new mt_engine();
    e->cfg = *cfg;
    if (e->cfg.seg_capacity == 0) e->cfg.seg_capacity = 2048;
    if (e->cfg.text_capacity == 0) e->cfg.text_capacity = 64 * 1024;
    if (e->cfg.heap_capacity == 0) e->cfg.heap_capacity = std::max<uint32_t>(1088, e->cfg.seg_capacity / 2 + 64);
    e->n_classes = 0;
    while (e->n_classes < kNumClasses && kClasses[e->n_classes] <= (int32_t)e->cfg.seg_capacity) e->n_classes++;
    mt_gstate& g = e->g;
    const size_t D = cfg->max_docs;
    g.segcap = e->cfg.seg_capacity;
    g.lbcap = g.segcap / 2;
    g.ibcap = g.segcap / 8 + 8;
    g.hcap = e->cfg.heap_capacity;
    g.textcap = e->cfg.text_capacity;
    mt_status st = MT_OK;
    const size_t S = D * g.segcap;
    if ((st = dalloc(e, &g.seq, S)) || (st = dalloc(e, &g.rseq, S)) || (st = dalloc(e, &g.len, S)) ||
        (st = dalloc(e, &g.toff, S)) || (st = dalloc(e, &g.ovl, S)) || (st = dalloc(e, &g.props, S)) ||
        (st = dalloc(e, &g.client, S)) || (st = dalloc(e, &g.rclient, S)) || (st = dalloc(e, &g.flags, S)) ||
        (st = dalloc(e, &g.lbcnt, D * g.lbcap)) || (st = dalloc(e, &g.lbscour, D * g.lbcap)) ||
        (st = dalloc(e, &g.ibcnt, D * (MT_MAXLEV - 1) * g.ibcap)) || (st = dalloc(e, &g.hseq, D * g.hcap)) ||
        (st = dalloc(e, &g.hslot, D * g.hcap)) || (st = dalloc(e, &g.sc, D)) ||
        (st = dalloc(e, &g.text, D * 2 * g.textcap)) || (st = dalloc(e, &e->d_classes, kNumClasses * 4)) ||
        (st = dalloc(e, &g.gm, D * MT_LOC_CAP)) || (st = dalloc(e, &g.pk, D * MT_LOC_CAP)) ||
        (st = dalloc(e, &g.ct, D * MT_LOC_CAP)) || (st = dalloc(e, &g.ctx, D * MT_LOC_CAP)) ||
        (st = dalloc(e, &g.lsqx, D * MT_LOC_CAP)) || (st = dalloc(e, &g.pkx, D * MT_LOC_CAP)) ||
        (st = dalloc(e, &g.gmxs, D * MT_LOC_CAP)) || (st = dalloc(e, &g.loc, D)) ||
        (st = dalloc(e, &g.lsq, D * MT_LOC_CAP)) || (st = dalloc(e, &g.rg, D * MT_RG_RECS)) ||
        (st = dalloc(e, &g.rgp, D * MT_RG_BYTES)) || (st = dalloc(e, &g.locbig, D)) ||
        (st = dalloc(e, &g.locgx, D)) ||
        // (the editing documents' and the wide documents' buckets after the capacity classes)
        (st = dalloc(e, &e->d_counts, kCounts)) || (st = dalloc(e, &e->d_acc, kBuckets)) ||
        (st = dalloc(e, &e->d_ids, D * kBuckets))) {
        mt_engine_destroy(e);
        return st;
    }
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&e->h_counts, kCounts * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess) {
        mt_engine_destroy(e);
        return MT_ERR_HIP;
    }
    HIP_OK(hipMemcpy(e->d_classes, kClassParams, sizeof(kClassParams), hipMemcpyHostToDevice));
    HIP_OK(hipMemset(g.locbig, 0xFF, D * sizeof(uint32_t)));  // MT_NO_ROW
    HIP_OK(hipMemset(g.locgx, 0xFF, D * sizeof(uint32_t)));
    e->h_locbig.assign(D, MT_NO_ROW);
    e->h_locgx.assign(D, MT_NO_ROW);
    {
        const char* v = getenv("MTGPU_ENGINE");
        // the register engine keeps text offsets in 16 bits (textcap <= 64 KiB)
        e->use_reg = !(v && strcmp(v, "lds") == 0) && e->cfg.text_capacity <= 65536;
        e->first_lds = e->use_reg ? kFirstLds : 0;
        e->reg_default = e->use_reg;
        const char* sv = getenv("MTGPU_SERIAL");
        e->concurrent = !(sv && strcmp(sv, "1") == 0);
        const char* ov = getenv("MTGPU_CLASS_ORDER");  // (A/B: "asc" launches the classes smallest first)
        e->desc_order = !(ov && strcmp(ov, "asc") == 0);
    }
    if (hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming) != hipSuccess) {
        mt_engine_destroy(e);
        return MT_ERR_HIP;
    }
    for (int c = 0; c < kNumClasses; c++) {
        if (hipStreamCreateWithFlags(&e->side[c], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e->join_ev[c], hipEventDisableTiming) != hipSuccess) {
            mt_engine_destroy(e);
            return MT_ERR_HIP;
        }
    }
    *out = e;
    return MT_OK;
}

mt_status mt_engine_destroy(mt_engine* e) {
    if (!e) return MT_ERR_ARG;
    hipSetDevice(e->cfg.device);
    if (e->stream) hipStreamSynchronize(e->stream);
    for (void* p : e->allocs) hipFree(p);
    if (e->g.ev) (void)hipFree(e->g.ev);
    if (e->g.evn) (void)hipFree(e->g.evn);
    if (e->ws) (void)hipFree(e->ws);
    for (void* p : {(void*)e->g.gmb, (void*)e->g.pkb, (void*)e->g.ctb, (void*)e->g.lsqb, (void*)e->g.gmx,
                    (void*)e->g.locx})
        if (p) (void)hipFree(p);
    if (e->h_counts) hipHostFree(e->h_counts);
    for (auto ev : e->kev) (void)hipEventDestroy(ev);
    if (e->ev0) hipEventDestroy(e->ev0);
    if (e->ev1) hipEventDestroy(e->ev1);
    if (e->stream) hipStreamDestroy(e->stream);
    for (int c = 0; c < kNumClasses; c++) {
        if (e->side[c]) {
            (void)hipStreamSynchronize(e->side[c]);
            (void)hipStreamDestroy(e->side[c]);
        }
        if (e->join_ev[c]) (void)hipEventDestroy(e->join_ev[c]);
    }
    if (e->fork_ev) (void)hipEventDestroy(e->fork_ev);
    for (hipStream_t s : {e->h2d, e->d2h})
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    if (e->d_scan) (void)hipFree(e->d_scan);
    for (auto& s : e->ring) {
        for (void* p : {(void*)s.ops, (void*)s.pay, (void*)s.rp, (void*)s.msgs, (void*)s.mrp, (void*)s.tk})
            if (p) (void)hipFree(p);
        for (hipEvent_t ev : {s.ready, s.applied, s.drained, s.ticketed})
            if (ev) (void)hipEventDestroy(ev);
    }
    delete e;
    return MT_OK;
}

mt_status mt_engine_info(const mt_engine* e, uint32_t* n_docs, uint32_t* max_docs) {
    if (!e) return MT_ERR_ARG;
    if (n_docs) *n_docs = e->n_docs;
    if (max_docs) *max_docs = e->cfg.max_docs;
    return MT_OK;
}

mt_status mt_docs_init(mt_engine* e, uint32_t n_docs) {
    if (!e || n_docs > e->cfg.max_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    e->n_docs = n_docs;
    e->gen++;
    e->lkeys.assign(e->cfg.max_docs, (uint16_t)MT_NO_LABEL_KEYS);
    // every document starts over: the editing pools' rows are all free again
    if (e->nbig || e->ngx) {
        HIP_OK(hipStreamSynchronize(e->stream));
        HIP_OK(hipMemset(e->g.locbig, 0xFF, e->cfg.max_docs * sizeof(uint32_t)));  // MT_NO_ROW
        HIP_OK(hipMemset(e->g.locgx, 0xFF, e->cfg.max_docs * sizeof(uint32_t)));
        e->h_locbig.assign(e->cfg.max_docs, MT_NO_ROW);
        e->h_locgx.assign(e->cfg.max_docs, MT_NO_ROW);
        e->nbig = e->ngx = 0;
        e->free_big.clear();
        e->free_gx.clear();
    }
    HIP_OK(mt_launch_init(&e->g, n_docs, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    return MT_OK;
}

mt_status mt_set_label_keys(mt_engine* e, uint32_t doc, int tile_key, int range_key) {
    if (!e || tile_key < -1 || tile_key >= MT_MAX_KEYS_WIDE || range_key < -1 || range_key >= MT_MAX_KEYS_WIDE)
        return MT_ERR_ARG;
    const uint32_t keys = (tile_key < 0 ? 0xFFu : (uint32_t)tile_key) | ((range_key < 0 ? 0xFFu : (uint32_t)range_key) << 8);
    const uint32_t d0 = doc == MT_ALL_DOCS ? 0 : doc, d1 = doc == MT_ALL_DOCS ? e->n_docs : doc + 1;
    if (d0 >= e->n_docs && doc != MT_ALL_DOCS) return MT_ERR_ARG;
    if (keys == MT_NO_LABEL_KEYS) return MT_OK;
    if (e->lkeys.size() < e->cfg.max_docs) e->lkeys.resize(e->cfg.max_docs, (uint16_t)MT_NO_LABEL_KEYS);
    auto merge = [](uint32_t old, uint32_t req) {  // each key: declared once, or left as it is (0xFF)
        uint32_t out = 0;
        for (int h = 0; h < 16; h += 8) {
            const uint32_t o = (old >> h) & 0xFFu, r = (req >> h) & 0xFFu;
            if (r != 0xFFu && o != 0xFFu && o != r) return 0xFFFFFFFFu;
            out |= (r != 0xFFu ? r : o) << h;
        }
        return out;
    };
    for (uint32_t d = d0; d < d1; d++)
        if (merge(e->lkeys[d], keys) == 0xFFFFFFFFu) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    if (!e->g.slab) {
        uint32_t *p = nullptr, *px = nullptr;
        if (dalloc(e, &p, (size_t)e->cfg.max_docs * e->g.segcap) ||
            dalloc(e, &px, (size_t)e->cfg.max_docs * e->g.segcap))
            return MT_ERR_NOMEM;
        e->g.slab = p;
        e->g.slabx = px;
    }
    for (uint32_t d = d0; d < d1; d++) e->lkeys[d] = (uint16_t)merge(e->lkeys[d], keys);
    e->gen++;
    HIP_OK(mt_launch_label_keys(&e->g, d0, d1, keys, e->stream));
    return MT_OK;
}

mt_status mt_docs_load(mt_engine* e, uint32_t n, const uint32_t* doc_ids, const uint32_t* seg_row_ptr,
                       const mt_load_seg* segs, const uint8_t* text, uint64_t text_bytes, const int32_t* min_seq,
                       const int32_t* cur_seq) {
    static_assert(sizeof(mt_load_seg) == 96, "mt_load_seg is 96 bytes");
    if (!e || (n && (!doc_ids || !seg_row_ptr || !min_seq || !cur_seq))) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    const uint64_t n_segs = seg_row_ptr[n] - seg_row_ptr[0];
    if (n_segs && !segs) return MT_ERR_ARG;
    for (uint32_t i = 0; i < n; i++) {
        if (doc_ids[i] >= e->n_docs || seg_row_ptr[i + 1] < seg_row_ptr[i]) return MT_ERR_ARG;
        if (!(min_seq[i] <= cur_seq[i])) return MT_ERR_ARG;
    }
    bool wide = false;
    for (uint64_t k = 0; k < n_segs; k++) {  // every text range inside `text`, ids in range
        const mt_load_seg& sg = segs[seg_row_ptr[0] + k];
        const uint64_t tb = (uint64_t)sg.text_len * ((sg.flags & MT_LSF_U16) ? 2u : 1u);
        if ((uint64_t)sg.text_off + tb > text_bytes) return MT_ERR_ARG;
        if (seg_client(sg) >= MT_MAX_CLIENTS_WIDE) return MT_ERR_ARG;
        if (sg.rseq >= 0 && (seg_rclient(sg) >= MT_MAX_CLIENTS_WIDE || seg_rclient(sg) == MT_CLIENT_NONCOLLAB))
            return MT_ERR_ARG;
        wide = wide || wide_load_seg(sg);
    }
    HIP_OK(hipSetDevice(e->cfg.device));
    if (const mt_status rs = release_loc_rows(e, doc_ids, n)) return rs;
    HIP_OK(hipSetDevice(e->cfg.device));
    if (wide) {
        const mt_status ws = ensure_wide(e);
        if (ws) return ws;
    }
    e->gen++;
    // one staging allocation: ids, rebased row pointers, windows, segments, text
    std::vector<uint32_t> rp(n + 1);
    for (uint32_t i = 0; i <= n; i++) rp[i] = seg_row_ptr[i] - seg_row_ptr[0];
    const size_t o_ids = 0, o_rp = o_ids + 4ull * n, o_mn = o_rp + 4ull * (n + 1), o_cs = o_mn + 4ull * n;
    const size_t o_sg = (o_cs + 4ull * n + 31) & ~size_t(31), o_tx = o_sg + sizeof(mt_load_seg) * n_segs;
    const size_t total = o_tx + text_bytes;
    uint8_t* buf = nullptr;
    if (hipMalloc(&buf, total ? total : 1) != hipSuccess) return MT_ERR_NOMEM;
    mt_status st = MT_OK;
    do {
        if (hipMemcpyAsync(buf + o_ids, doc_ids, 4ull * n, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
            hipMemcpyAsync(buf + o_rp, rp.data(), 4ull * (n + 1), hipMemcpyHostToDevice, e->stream) != hipSuccess ||
            hipMemcpyAsync(buf + o_mn, min_seq, 4ull * n, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
            hipMemcpyAsync(buf + o_cs, cur_seq, 4ull * n, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
            (n_segs && hipMemcpyAsync(buf + o_sg, segs + seg_row_ptr[0], sizeof(mt_load_seg) * n_segs,
                                      hipMemcpyHostToDevice, e->stream) != hipSuccess) ||
            (text_bytes && hipMemcpyAsync(buf + o_tx, text, text_bytes, hipMemcpyHostToDevice, e->stream) != hipSuccess)) {
            st = MT_ERR_HIP;
            break;
        }
        if (mt_launch_load(&e->g, n, reinterpret_cast<uint32_t*>(buf + o_ids), reinterpret_cast<uint32_t*>(buf + o_rp),
                           reinterpret_cast<mt_load_seg*>(buf + o_sg), buf + o_tx, reinterpret_cast<int32_t*>(buf + o_mn),
                           reinterpret_cast<int32_t*>(buf + o_cs), e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            st = MT_ERR_HIP;
    } while (0);
    hipFree(buf);
    return st;
}

mt_status mt_find_tiles(mt_engine* e, const mt_tile_query* q, uint32_t n, mt_tile_result* out) {
    static_assert(sizeof(mt_tile_query) == 48, "mt_tile_query is 48 bytes");
    if (!e || (n && (!q || !out))) return MT_ERR_ARG;
    for (uint32_t i = 0; i < n; i++)
        if (q[i].doc >= e->n_docs) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    HIP_OK(hipSetDevice(e->cfg.device));
    void* buf = nullptr;
    const size_t qb = (size_t)n * sizeof(mt_tile_query), rb = (size_t)n * sizeof(mt_tile_result);
    if (hipMalloc(&buf, qb + rb) != hipSuccess) return MT_ERR_NOMEM;
    auto* dq = static_cast<mt_tile_query*>(buf);
    auto* dr = reinterpret_cast<mt_tile_result*>(static_cast<uint8_t*>(buf) + qb);
    hipError_t r = hipMemcpyAsync(dq, q, qb, hipMemcpyHostToDevice, e->stream);
    if (r == hipSuccess) r = mt_launch_tiles(&e->g, dq, n, dr, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(out, dr, rb, hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(buf);
    return r == hipSuccess ? MT_OK : MT_ERR_HIP;
}

mt_status mt_resolve_positions(mt_engine* e, const mt_pos_query* q, uint32_t n, mt_pos_result* out) {
    static_assert(sizeof(mt_pos_query) == 16 && sizeof(mt_pos_result) == 16, "mt_pos_query / result are 16 bytes");
    if (!e || (n && (!q || !out))) return MT_ERR_ARG;
    for (uint32_t i = 0; i < n; i++)
        if (q[i].doc >= e->n_docs || q[i].kind > MT_POS_OF_ORDINAL) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    HIP_OK(hipSetDevice(e->cfg.device));
    void* buf = nullptr;
    const size_t qb = (size_t)n * sizeof(mt_pos_query), rb = (size_t)n * sizeof(mt_pos_result);
    if (hipMalloc(&buf, qb + rb) != hipSuccess) return MT_ERR_NOMEM;
    auto* dq = static_cast<mt_pos_query*>(buf);
    auto* dr = reinterpret_cast<mt_pos_result*>(static_cast<uint8_t*>(buf) + qb);
    hipError_t r = hipMemcpyAsync(dq, q, qb, hipMemcpyHostToDevice, e->stream);
    if (r == hipSuccess) r = mt_launch_resolve(&e->g, dq, n, e->n_docs, dr, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(out, dr, rb, hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(buf);
    return r == hipSuccess ? MT_OK : MT_ERR_HIP;
}

mt_status mt_resolve_positions_device(mt_engine* e, const mt_pos_query* d_q, uint32_t n, mt_pos_result* d_out) {
    if (!e || (n && (!d_q || !d_out))) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    HIP_OK(hipSetDevice(e->cfg.device));
    HIP_OK(mt_launch_resolve(&e->g, d_q, n, e->n_docs, d_out, e->stream));
    return MT_OK;
}

mt_status mt_segment_infos(mt_engine* e, const uint32_t* docs, const int32_t* ordinals, uint32_t n, mt_seg_info* out) {
    static_assert(sizeof(mt_seg_info) == 168, "mt_seg_info is 168 bytes");
    if (!e || (n && (!docs || !ordinals || !out))) return MT_ERR_ARG;
    for (uint32_t i = 0; i < n; i++)
        if (docs[i] >= e->n_docs) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    HIP_OK(hipSetDevice(e->cfg.device));
    void* buf = nullptr;
    const size_t db = (size_t)n * 4, ob = (size_t)n * sizeof(mt_seg_info);
    if (hipMalloc(&buf, 2 * db + ob) != hipSuccess) return MT_ERR_NOMEM;
    auto* dd = static_cast<uint32_t*>(buf);
    auto* dor = reinterpret_cast<int32_t*>(static_cast<uint8_t*>(buf) + db);
    auto* dout = reinterpret_cast<mt_seg_info*>(static_cast<uint8_t*>(buf) + 2 * db);
    hipError_t r = hipMemcpyAsync(dd, docs, db, hipMemcpyHostToDevice, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(dor, ordinals, db, hipMemcpyHostToDevice, e->stream);
    if (r == hipSuccess) r = mt_launch_seginfo(&e->g, dd, dor, n, dout, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(buf);
    return r == hipSuccess ? MT_OK : MT_ERR_HIP;
}

mt_status mt_segment_text(mt_engine* e, uint32_t doc, uint32_t toff, uint32_t len, uint16_t* out) {
    if (!e || doc >= e->n_docs || (len && !out)) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    mt_doc_scalars sc;
    HIP_OK(hipMemcpyAsync(&sc, e->g.sc + doc, sizeof sc, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    if ((uint64_t)toff + len > sc.text_top) return MT_ERR_ARG;
    if (!len) return MT_OK;
    const size_t base = ((size_t)doc * 2 + sc.text_half) * e->g.textcap;
    if (sc.wide & MT_WIDE_DOC) {
        HIP_OK(hipMemcpy(out, e->g.text + base + (size_t)toff * 2, (size_t)len * 2, hipMemcpyDeviceToHost));
        return MT_OK;
    }
    std::vector<uint8_t> b(len);
    HIP_OK(hipMemcpy(b.data(), e->g.text + base + toff, len, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < len; i++) out[i] = b[i];
    return MT_OK;
}

mt_status mt_regen_drain(mt_engine* e, uint32_t doc, mt_op_rec* recs, uint32_t cap, uint8_t* payload, uint32_t pcap,
                         uint32_t* n, uint32_t* pn) {
    if (!e || doc >= e->n_docs || !n || !pn) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HIP_OK(hipStreamSynchronize(e->stream));
    uint32_t cnt[2] = {0, 0};  // mt_loc::rgn, rgpn (adjacent)
    HIP_OK(hipMemcpy(cnt, &e->g.loc[doc].rgn, sizeof cnt, hipMemcpyDeviceToHost));
    *n = cnt[0];
    *pn = cnt[1];
    if (!recs) return MT_OK;  // sizes only
    // a drain takes everything or nothing: buffers too small leave the records in place
    if (cap < cnt[0] || (cnt[1] && (!payload || pcap < cnt[1]))) return MT_ERR_ARG;
    if (cnt[0])
        HIP_OK(hipMemcpy(recs, e->g.rg + (size_t)doc * MT_RG_RECS, cnt[0] * sizeof(mt_op_rec), hipMemcpyDeviceToHost));
    if (cnt[1]) HIP_OK(hipMemcpy(payload, e->g.rgp + (size_t)doc * MT_RG_BYTES, cnt[1], hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(&e->g.loc[doc].rgn, 0, sizeof cnt));
    return MT_OK;
}

mt_status mt_range_stacks(mt_engine* e, const mt_tile_query* q, uint32_t n, uint32_t cap, mt_stack_item* items,
                          uint32_t* depth) {
    static_assert(sizeof(mt_stack_item) == 12, "mt_stack_item is 12 bytes");
    if (!e || (n && (!q || !depth || (cap && !items)))) return MT_ERR_ARG;
    for (uint32_t i = 0; i < n; i++)
        if (q[i].doc >= e->n_docs) return MT_ERR_ARG;
    if (n == 0) return MT_OK;
    HIP_OK(hipSetDevice(e->cfg.device));
    void* buf = nullptr;
    const size_t qb = (size_t)n * sizeof(mt_tile_query), ib = (size_t)n * cap * sizeof(mt_stack_item),
                 db = (size_t)n * sizeof(uint32_t);
    if (hipMalloc(&buf, qb + ib + db) != hipSuccess) return MT_ERR_NOMEM;
    auto* dq = static_cast<mt_tile_query*>(buf);
    auto* di = reinterpret_cast<mt_stack_item*>(static_cast<uint8_t*>(buf) + qb);
    auto* dd = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(buf) + qb + ib);
    hipError_t r = hipMemcpyAsync(dq, q, qb, hipMemcpyHostToDevice, e->stream);
    if (r == hipSuccess) r = mt_launch_stacks(&e->g, dq, n, cap, di, dd, e->stream);
    if (r == hipSuccess && ib) r = hipMemcpyAsync(items, di, ib, hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(depth, dd, db, hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(buf);
    return r == hipSuccess ? MT_OK : MT_ERR_HIP;
}

mt_status mt_events_enable(mt_engine* e, uint32_t per_doc) {
    static_assert(sizeof(mt_event) == 96, "mt_event is 96 bytes");
    if (!e) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HIP_OK(hipStreamSynchronize(e->stream));
    if (e->g.ev) HIP_OK(hipFree(e->g.ev));
    if (e->g.evn) HIP_OK(hipFree(e->g.evn));
    e->g.ev = nullptr;
    e->g.evn = nullptr;
    e->g.evcap = 0;
    // the register engine records events in its own kernels (mtr::reg_apply_kernel_ev; its C64
    // documents on the LDS engine); MTGPU_EV_ENGINE=lds keeps every class on the LDS engine instead
    const char* evw = getenv("MTGPU_EV_ENGINE");
    e->use_reg = (per_doc && evw && strcmp(evw, "lds") == 0) ? false : e->reg_default;
    e->first_lds = e->use_reg ? kFirstLds : 0;
    if (!per_doc) return MT_OK;
    const size_t D = e->cfg.max_docs;
    if (hipMalloc(&e->g.ev, D * per_doc * sizeof(mt_event)) != hipSuccess ||
        hipMalloc(&e->g.evn, D * sizeof(uint32_t)) != hipSuccess) {
        if (e->g.ev) (void)hipFree(e->g.ev);
        e->g.ev = nullptr;
        e->g.evn = nullptr;
        e->use_reg = e->reg_default;
        e->first_lds = e->use_reg ? kFirstLds : 0;
        return MT_ERR_NOMEM;
    }
    e->g.evcap = per_doc;
    HIP_OK(hipMemset(e->g.evn, 0, D * sizeof(uint32_t)));
    return MT_OK;
}

mt_status mt_events_drain(mt_engine* e, mt_event* out, uint64_t cap, uint32_t* row_ptr, uint64_t* total) {
    if (!e || !row_ptr || !total || !e->g.ev) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HIP_OK(hipStreamSynchronize(e->stream));
    const uint32_t n = e->n_docs;
    std::vector<uint32_t> cnt(n);
    if (n) HIP_OK(hipMemcpy(cnt.data(), e->g.evn, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint64_t> off(n + 1, 0);
    for (uint32_t d = 0; d < n; d++) off[d + 1] = off[d] + std::min(cnt[d], e->g.evcap);
    if (off[n] >= (1ull << 32)) return MT_ERR_ARG;
    for (uint32_t d = 0; d <= n; d++) row_ptr[d] = (uint32_t)off[d];
    *total = off[n];
    if (!out) return MT_OK;
    if (cap < off[n]) return MT_ERR_ARG;
    if (off[n]) {
        uint64_t* d_off = nullptr;
        mt_event* d_out = nullptr;
        if (hipMalloc(&d_off, (n + 1) * sizeof(uint64_t)) != hipSuccess) return MT_ERR_NOMEM;
        if (hipMalloc(&d_out, off[n] * sizeof(mt_event)) != hipSuccess) {
            (void)hipFree(d_off);
            return MT_ERR_NOMEM;
        }
        mt_status st = MT_OK;
        if (hipMemcpyAsync(d_off, off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, e->stream) != hipSuccess ||
            mt_launch_events_pack(&e->g, n, d_off, d_out, e->stream) != hipSuccess ||
            hipMemcpyAsync(out, d_out, off[n] * sizeof(mt_event), hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            st = MT_ERR_HIP;
        (void)hipFree(d_off);
        (void)hipFree(d_out);
        if (st) return st;
    }
    HIP_OK(hipMemsetAsync(e->g.evn, 0, (size_t)n * sizeof(uint32_t), e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    return MT_OK;
}

mt_status mt_batch_upload(mt_engine* e, const mt_op_rec* ops, uint64_t n_ops, const uint8_t* payload,
                          uint64_t payload_bytes, const uint32_t* doc_row_ptr, mt_batch** out) {
    if (!e || !out || !doc_row_ptr) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    auto* b = new mt_batch();
    b->n_docs = e->n_docs;
    b->n_ops = n_ops;
    b->payload_bytes = payload_bytes;
    if (doc_row_ptr[b->n_docs] != n_ops) {
        delete b;
        return MT_ERR_ARG;
    }
    for (uint32_t d = 0; d < b->n_docs; d++) {
        if (doc_row_ptr[d + 1] < doc_row_ptr[d]) {
            delete b;
            return MT_ERR_ARG;
        }
        b->max_ops_per_doc = std::max(b->max_ops_per_doc, doc_row_ptr[d + 1] - doc_row_ptr[d]);
    }
    const int flags = scan_records(ops, n_ops, payload_bytes);
    if (flags & 1) {
        delete b;
        return MT_ERR_ARG;
    }
    b->wide = (flags & 2) != 0;
    if (hipMalloc(&b->ops, std::max<uint64_t>(1, n_ops) * sizeof(mt_op_rec)) != hipSuccess ||
        hipMalloc(&b->payload, std::max<uint64_t>(1, payload_bytes)) != hipSuccess ||
        hipMalloc(&b->row_ptr, (b->n_docs + 1) * sizeof(uint32_t)) != hipSuccess) {
        mt_batch_free(e, b);
        return MT_ERR_NOMEM;
    }
    HIP_OK(hipMemcpyAsync(b->ops, ops, n_ops * sizeof(mt_op_rec), hipMemcpyHostToDevice, e->stream));
    if (payload_bytes) HIP_OK(hipMemcpyAsync(b->payload, payload, payload_bytes, hipMemcpyHostToDevice, e->stream));
    HIP_OK(hipMemcpyAsync(b->row_ptr, doc_row_ptr, (b->n_docs + 1) * sizeof(uint32_t), hipMemcpyHostToDevice,
                          e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    *out = b;
    return MT_OK;
}

mt_status mt_batch_free(mt_engine* e, mt_batch* b) {
    if (!e || !b) return MT_ERR_ARG;
    hipSetDevice(e->cfg.device);
    hipStreamSynchronize(e->stream);
    if (b->ops) hipFree(b->ops);
    if (b->payload) hipFree(b->payload);
    if (b->row_ptr) hipFree(b->row_ptr);
    delete b;
    return MT_OK;
}

}  // extern "C"

// One apply call (mt_batch_apply, mt_submit_ticks) = apply_begin, the launches of one or more
// batches (apply_launches), apply_end: the statistics of mt_last_apply_stats cover the whole call.
static mt_status apply_begin(mt_engine* e) {
    e->gen++;
    e->last_launches = 0;
    HIP_OK(hipMemsetAsync(e->d_acc, 0, kBuckets * sizeof(unsigned long long), e->stream));
    e->kev_cls.clear();
    HIP_OK(hipEventRecord(e->ev0, e->stream));
    return MT_OK;
}

// The launches of one staged batch on the engine stream, in launches of ops_per_launch ops per
// document, then the window-assert fixup over the batch's records; nk counts the kernel events.
static mt_status apply_launches(mt_engine* e, const mt_batch* b, uint32_t& nk) {
    if (b->wide) {
        const mt_status ws = ensure_wide(e);
        if (ws) return ws;
    }
    const uint32_t per = e->cfg.ops_per_launch ? e->cfg.ops_per_launch : std::max<uint32_t>(1, b->max_ops_per_doc);
    const uint32_t ticks = (b->max_ops_per_doc + per - 1) / per;
    const int lds_base = e->n_classes + 1 + (e->n_classes > kFirstWide ? e->n_classes - kFirstWide : 0);
    for (uint32_t t = 0; t < ticks; t++) {
        const uint32_t lo = t * per;
        HIP_OK(hipMemsetAsync(e->d_counts, 0, kCounts * sizeof(uint32_t), e->stream));
        HIP_OK(mt_launch_bin(&e->g, b->row_ptr, b->n_docs, lo, per, e->d_classes, e->n_classes, e->first_lds,
                             kFirstWide, e->d_counts, e->d_ids, b->ops, b->payload, e->d_acc, e->stream));
        HIP_OK(hipMemcpyAsync(e->h_counts, e->d_counts, kCounts * sizeof(uint32_t), hipMemcpyDeviceToHost,
                              e->stream));
        HIP_OK(hipStreamSynchronize(e->stream));
        // the classes above 2048 segments keep each document's structure in an HBM workspace
        // (one region per class: their kernels may run concurrently)
        // (the wide documents' form keeps its structure in the workspace at every class)
        size_t ws_off[kNumClasses] = {}, wws_off[kNumClasses] = {}, need = 0;
        for (int c = kLdsClasses; c < e->n_classes; c++) {
            ws_off[c] = need;
            need += (size_t)e->h_counts[c] * mt_lds_bytes(kClasses[c]);
        }
        // (the LDS-staged wide classes take a region only when some document stages the extension)
        const int n_bk = lds_base + 2 * e->first_lds + kLocForms;
        for (int c = kFirstWide; c < e->n_classes; c++) {
            wws_off[c] = need;
            const bool xl_any = e->h_counts[n_bk + (c - kFirstWide)] != 0;
            if (kClasses[c] > 512 || xl_any)
                need += (size_t)e->h_counts[e->n_classes + 1 + (c - kFirstWide)] * mt_lds_bytes_wide(kClasses[c]);
        }
        size_t lws_off[kLocForms] = {};
        for (int q = 0; q < kLocForms; q++) {
            const uint32_t cnt = e->h_counts[lds_base + 2 * e->first_lds + q];
            if ((kLocCaps[q] <= MT_LOC_CAP && kLocGW[q] == 1) || !cnt) continue;
            const mt_status ls = assign_loc_rows(e, e->d_ids + (size_t)(lds_base + 2 * e->first_lds + q) * b->n_docs,
                                                 cnt, kLocCaps[q] > MT_LOC_CAP, kLocGW[q] > 1);
            if (ls) return ls;
            lws_off[q] = need;
            need += (size_t)cnt * mt_lds_bytes_loc(kLocCaps[q], kLocGW[q]);
        }
        if (need > e->ws_bytes) {
            HIP_OK(hipDeviceSynchronize());
            if (e->ws) HIP_OK(hipFree(e->ws));
            e->ws = nullptr;
            e->ws_bytes = 0;
            if (hipMalloc(&e->ws, need) != hipSuccess) return MT_ERR_NOMEM;
            e->ws_bytes = need;
        }
        if (e->concurrent) HIP_OK(hipEventRecord(e->fork_ev, e->stream));
        bool joined[kNumClasses] = {};
        // largest capacity first: a class's waves last longer the more segments its documents hold, and
        // the few documents of the upper classes would otherwise start once the bulk classes' waves had
        // all been dispatched -- the tick's tail.  Started first they run beside the bulk.
        for (int i = 0; i < e->n_classes; i++) {  // (h_counts[n_classes]: the editing bucket, below)
            const int c = e->desc_order ? e->n_classes - 1 - i : i;
            const uint32_t cnt = e->h_counts[c];
            if (!cnt) continue;
            hipStream_t st = e->stream;
            if (e->concurrent) {
                st = e->side[c];
                HIP_OK(hipStreamWaitEvent(st, e->fork_ev, 0));
                joined[c] = true;
            }
            while (e->kev.size() < 2 * (nk + 1)) {
                hipEvent_t ev;
                HIP_OK(hipEventCreate(&ev));
                e->kev.push_back(ev);
            }
            HIP_OK(hipEventRecord(e->kev[2 * nk], st));
            if (e->use_reg && kClasses[c] <= kRegMaxCap)
                HIP_OK(mt_launch_apply_reg(kClasses[c], e->g.ev ? 2 : 0, &e->g, b->ops, b->payload, b->row_ptr,
                                           e->d_ids + (size_t)c * b->n_docs, cnt, lo, per, st));
            else if (c >= kLdsClasses)
                HIP_OK(mt_launch_apply_big(kClasses[c], &e->g, b->ops, b->payload, b->row_ptr,
                                           e->d_ids + (size_t)c * b->n_docs, cnt, lo, per, e->ws + ws_off[c], st));
            else
                HIP_OK(mt_launch_apply(lds_cap(kClasses[c]), &e->g, b->ops, b->payload, b->row_ptr,
                                       e->d_ids + (size_t)c * b->n_docs, cnt, lo, per, st));
            HIP_OK(hipEventRecord(e->kev[2 * nk + 1], st));
            e->kev_cls.push_back(c);
            nk++;
        }
        // documents that need the LDS engine inside a register class (the LDS engine at that
        // class's capacity), then those with client ids above 32 (the register engine's C64 form),
        // on the class's stream after its register launch
        for (int q = 0; q < 2 * e->first_lds; q++) {
            const int c = q % e->first_lds;
            const bool c64 = q >= e->first_lds;
            if (c >= e->n_classes) continue;
            const uint32_t cnt = e->h_counts[lds_base + q];
            if (!cnt) continue;
            hipStream_t st = e->stream;
            if (e->concurrent) {
                st = e->side[c];
                if (!joined[c]) HIP_OK(hipStreamWaitEvent(st, e->fork_ev, 0));
                joined[c] = true;
            }
            while (e->kev.size() < 2 * (nk + 1)) {
                hipEvent_t ev;
                HIP_OK(hipEventCreate(&ev));
                e->kev.push_back(ev);
            }
            HIP_OK(hipEventRecord(e->kev[2 * nk], st));
            if (c64 && !e->g.ev)
                HIP_OK(mt_launch_apply_reg(kClasses[c], 1, &e->g, b->ops, b->payload, b->row_ptr,
                                           e->d_ids + (size_t)(lds_base + q) * b->n_docs, cnt, lo, per, st));
            else
                HIP_OK(mt_launch_apply(lds_cap(kClasses[c]), &e->g, b->ops, b->payload, b->row_ptr,
                                       e->d_ids + (size_t)(lds_base + q) * b->n_docs, cnt, lo, per, st));
            HIP_OK(hipEventRecord(e->kev[2 * nk + 1], st));
            e->kev_cls.push_back(kNumClasses + 1 + (c64 ? kFirstLds : 0) + c);
            nk++;
        }
        // wide documents: the LDS engine's wide form, per class, on the class's stream (disjoint
        // documents, their own workspace regions)
        for (int c = kFirstWide; c < e->n_classes; c++) {
            const int k = e->n_classes + 1 + (c - kFirstWide);
            const uint32_t cnt = e->h_counts[k];
            if (!cnt) continue;
            hipStream_t st = e->stream;
            if (e->concurrent) {
                st = e->side[c];
                if (!joined[c]) HIP_OK(hipStreamWaitEvent(st, e->fork_ev, 0));
                joined[c] = true;
            }
            while (e->kev.size() < 2 * (nk + 1)) {
                hipEvent_t ev;
                HIP_OK(hipEventCreate(&ev));
                e->kev.push_back(ev);
            }
            HIP_OK(hipEventRecord(e->kev[2 * nk], st));
            // (the extension's region only when one of the bucket's documents stages it)
            const bool xl = e->h_counts[lds_base + 2 * e->first_lds + kLocForms + (c - kFirstWide)] != 0;
            HIP_OK(mt_launch_apply_wide(kClasses[c], &e->g, b->ops, b->payload, b->row_ptr,
                                        e->d_ids + (size_t)k * b->n_docs, cnt, lo, per, e->ws + wws_off[c], xl ? 1 : 0,
                                        st));
            HIP_OK(hipEventRecord(e->kev[2 * nk + 1], st));
            e->kev_cls.push_back(kStatWide + (c - kFirstWide));
            nk++;
        }
        for (int c = 0; c < kNumClasses; c++) {  // join: the next tick's binning sees every class done
            if (!joined[c]) continue;
            HIP_OK(hipEventRecord(e->join_ev[c], e->side[c]));
            HIP_OK(hipStreamWaitEvent(e->stream, e->join_ev[c], 0));
        }
        // documents with an editing client (local edits + acks): the LDS engine's editing form
        // (the 1024-slot form's bucket at n_classes, the 256 / 512-slot forms' after the C64 buckets,
        // then the 2048 / 4096-slot HBM-workspace forms')
        for (int q = -1; q < kLocForms; q++) {
            const int bk = q < 0 ? e->n_classes : lds_base + 2 * e->first_lds + q;
            const uint32_t cnt = e->h_counts[bk];
            if (!cnt) continue;
            while (e->kev.size() < 2 * (nk + 1)) {
                hipEvent_t ev;
                HIP_OK(hipEventCreate(&ev));
                e->kev.push_back(ev);
            }
            HIP_OK(hipEventRecord(e->kev[2 * nk], e->stream));
            if (q >= 0 && (kLocCaps[q] > MT_LOC_CAP || kLocGW[q] > 1))
                HIP_OK(mt_launch_apply_loc_big(kLocCaps[q], kLocGW[q], &e->g, b->ops, b->payload, b->row_ptr,
                                               e->d_ids + (size_t)bk * b->n_docs, cnt, lo, per, e->ws + lws_off[q],
                                               e->stream));
            else
                HIP_OK(mt_launch_apply_loc(q < 0 ? MT_LOC_CAP : kLocCaps[q], &e->g, b->ops, b->payload, b->row_ptr,
                                           e->d_ids + (size_t)bk * b->n_docs, cnt, lo, per, e->stream));
            HIP_OK(hipEventRecord(e->kev[2 * nk + 1], e->stream));
            e->kev_cls.push_back(q < 0 ? kNumClasses : kNumClasses + 1 + 2 * kFirstLds + q);
            nk++;
        }
    }
    HIP_OK(mt_launch_fixup(&e->g, b->ops, b->n_docs, e->stream));  // error precedence, see mt_service.hip
    return MT_OK;
}

static mt_status apply_end(mt_engine* e, uint32_t nk) {
    const int lds_base = e->n_classes + 1 + (e->n_classes > kFirstWide ? e->n_classes - kFirstWide : 0);
    HIP_OK(hipEventRecord(e->ev1, e->stream));
    HIP_OK(hipEventSynchronize(e->ev1));
    float kms = 0.f;
    for (int c = 0; c < kStatClasses; c++) {
        e->cls_ms[c] = 0.f;
        e->cls_launches[c] = 0;
    }
    for (uint32_t k = 0; k < nk; k++) {
        float m = 0.f;
        HIP_OK(hipEventElapsedTime(&m, e->kev[2 * k], e->kev[2 * k + 1]));
        kms += m;
        e->cls_ms[e->kev_cls[k]] += m;
        e->cls_launches[e->kev_cls[k]]++;
    }
    HIP_OK(hipEventElapsedTime(&e->last_wall_ms, e->ev0, e->ev1));
    unsigned long long acc[kBuckets];
    HIP_OK(hipMemcpy(acc, e->d_acc, sizeof acc, hipMemcpyDeviceToHost));
    e->last_ms = kms;
    e->last_launches = nk;
    e->last_bytes = 0;
    for (int c = 0; c < kNumClasses; c++) {
        e->cls_bytes[c] = c < e->n_classes ? acc[c] : 0;
        e->last_bytes += e->cls_bytes[c];
    }
    e->cls_bytes[kNumClasses] = acc[e->n_classes];  // the editing bucket
    e->last_bytes += acc[e->n_classes];
    for (int q = 0; q < 2 * kFirstLds; q++) {
        const int c = q % kFirstLds;
        const bool on = e->first_lds == kFirstLds && c < e->n_classes;
        e->cls_bytes[kNumClasses + 1 + q] = on ? acc[lds_base + (q >= kFirstLds ? e->first_lds : 0) + c] : 0;
        e->last_bytes += e->cls_bytes[kNumClasses + 1 + q];
    }
    for (int q = 0; q < kLocForms; q++) {
        e->cls_bytes[kNumClasses + 1 + 2 * kFirstLds + q] = acc[lds_base + 2 * e->first_lds + q];
        e->last_bytes += acc[lds_base + 2 * e->first_lds + q];
    }
    for (int c = kFirstWide; c < kNumClasses; c++) {
        const uint64_t v = c < e->n_classes ? acc[e->n_classes + 1 + (c - kFirstWide)] : 0;
        e->cls_bytes[kStatWide + (c - kFirstWide)] = v;
        e->last_bytes += v;
    }
    return MT_OK;
}

extern "C" mt_status mt_deli_ticket_on_stream(mt_deli* dl, int32_t device, hipStream_t st, const mt_raw_msg* d_msgs,
                                              const uint32_t* d_row_ptr, uint32_t n_docs, mt_ticket* d_out,
                                              mt_op_rec* d_ops, uint64_t n_ops);

namespace {
// device slots of mt_submit_ticks: the copy stream runs up to kRing - 1 ticks ahead of the apply (a
// C5 tick is ~0.3 GB of records, messages and tickets: six slots are 2 GB of 288)
constexpr int kRing = 6;

// slot buffers of at least the given sizes (called with nothing in flight on the engine)
mt_status ring_reserve(mt_engine* e, uint64_t n_ops, uint64_t pay, uint64_t n_msgs) {
    // (the copy streams at the greatest priority: the runtime gives them a hardware queue of their own
    // where it keeps one per priority, so their packets never sit in front of the apply's)
    int lo_pri = 0, hi_pri = 0;
    if (hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri) != hipSuccess) hi_pri = 0;
    if (!e->h2d && hipStreamCreateWithPriority(&e->h2d, hipStreamNonBlocking, hi_pri) != hipSuccess) return MT_ERR_HIP;
    if (!e->d2h && hipStreamCreateWithPriority(&e->d2h, hipStreamNonBlocking, hi_pri) != hipSuccess) return MT_ERR_HIP;
    if (!e->d_scan) HIP_OK(hipMalloc(&e->d_scan, sizeof(uint32_t)));
    const size_t rp = ((size_t)e->cfg.max_docs + 1) * sizeof(uint32_t);
    for (auto& s : e->ring) {
        if (!s.ready) {
            for (hipEvent_t* ev : {&s.ready, &s.applied, &s.drained, &s.ticketed})
                if (hipEventCreateWithFlags(ev, hipEventDisableTiming) != hipSuccess) return MT_ERR_HIP;
            // (recorded once, so the first waits on them pass)
            HIP_OK(hipEventRecord(s.applied, e->stream));
            HIP_OK(hipEventRecord(s.drained, e->stream));
            HIP_OK(hipMalloc(&s.rp, rp));
            HIP_OK(hipMalloc(&s.mrp, rp));
        }
        if (s.ops_cap < n_ops) {
            if (s.ops) HIP_OK(hipFree(s.ops));
            s.ops = nullptr;
            s.ops_cap = 0;
            if (hipMalloc(&s.ops, n_ops * sizeof(mt_op_rec)) != hipSuccess) return MT_ERR_NOMEM;
            s.ops_cap = n_ops;
        }
        if (s.pay_cap < pay) {
            if (s.pay) HIP_OK(hipFree(s.pay));
            s.pay = nullptr;
            s.pay_cap = 0;
            if (hipMalloc(&s.pay, pay) != hipSuccess) return MT_ERR_NOMEM;
            s.pay_cap = pay;
        }
        if (s.msg_cap < n_msgs) {
            if (s.msgs) HIP_OK(hipFree(s.msgs));
            if (s.tk) HIP_OK(hipFree(s.tk));
            s.msgs = nullptr;
            s.tk = nullptr;
            s.msg_cap = 0;
            if (hipMalloc(&s.msgs, n_msgs * sizeof(mt_raw_msg)) != hipSuccess ||
                hipMalloc(&s.tk, n_msgs * sizeof(mt_ticket)) != hipSuccess)
                return MT_ERR_NOMEM;
            s.msg_cap = n_msgs;
        }
    }
    return MT_OK;
}

bool row_ptr_ok(const uint32_t* rp, uint32_t n_docs, uint64_t n, uint32_t* max_rows) {
    if (!rp || rp[0] != 0 || rp[n_docs] != n) return false;
    uint32_t mx = 0;
    for (uint32_t d = 0; d < n_docs; d++) {
        if (rp[d + 1] < rp[d]) return false;
        mx = std::max(mx, rp[d + 1] - rp[d]);
    }
    if (max_rows) *max_rows = mx;
    return true;
}

mt_status submit_ticks(mt_engine* e, mt_deli* dl, const mt_tick* ticks, uint32_t n) {
    if (!e || (n && !ticks)) return MT_ERR_ARG;
    const uint32_t D = e->n_docs;
    uint64_t mo = 1, mp = 1, mm = 1;
    for (uint32_t k = 0; k < n; k++) {
        const mt_tick& t = ticks[k];
        if (!t.doc_row_ptr || (t.n_ops && !t.ops) || (t.payload_bytes && !t.payload) || t.n_ops >= (1ull << 32) ||
            (t.n_msgs && (!dl || !t.msgs || !t.msg_row_ptr)) || t.n_msgs >= (1ull << 32))
            return MT_ERR_ARG;
        mo = std::max(mo, t.n_ops);
        mp = std::max(mp, t.payload_bytes);
        mm = std::max(mm, t.n_msgs);
    }
    HIP_OK(hipSetDevice(e->cfg.device));
    if (n == 0) return MT_OK;
    const auto t_start = std::chrono::steady_clock::now();
    HIP_OK(hipStreamSynchronize(e->stream));
    const auto t_synced = std::chrono::steady_clock::now();
    mt_status st = ring_reserve(e, mo, mp, mm);
    if (st) return st;
    const auto t_reserved = std::chrono::steady_clock::now();
    mt_batch bs[kRing];
    // (MTGPU_TICK_TRACE=1: the host's time in the checks and in the apply loop, to stderr)
    double t_check = 0, t_apply = 0, t_copy = 0, t_wait = 0, wait_k[64] = {}, check_k[64] = {};
    // tick k: checked on the host, then copied into its slot.  Every dependency between the copies and
    // the apply is kept by the host, not by a stream waiting on another stream's event: the streams
    // share the device's few hardware queues (GPU_MAX_HW_QUEUES), where such a wait holds up every
    // later packet of its queue -- a tick's apply then waited for the next ticks' copies.  The host
    // already synchronises once per tick (the bin counts), so the ordering costs nothing:
    //   * tick k is copied when its slot's previous tick (k - kRing) has applied and its tickets have
    //     gone back (both complete by then: the host issues the copy after tick k - kRing + 1's bin);
    //   * tick k applies once the host has seen its copy land (issued two ticks earlier).
    auto stage = [&](uint32_t k) -> mt_status {
        const mt_tick& t = ticks[k];
        auto& s = e->ring[k % kRing];
        mt_batch& b = bs[k % kRing];
        uint32_t mx = 0;
        const auto c0 = std::chrono::steady_clock::now();
        if (!row_ptr_ok(t.doc_row_ptr, D, t.n_ops, &mx) || (t.n_msgs && !row_ptr_ok(t.msg_row_ptr, D, t.n_msgs, nullptr)))
            return MT_ERR_ARG;
        // (tick 0: its records are checked on the device once they have landed, in the apply loop --
        // the host check would sit between the start and the first copy)
        const int flags = k == 0 ? 0 : scan_records(t.ops, t.n_ops, t.payload_bytes);
        if (flags & 1) return MT_ERR_ARG;
        const double ck = std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
        t_check += ck;
        if (k < 64) check_k[k] = ck;
        b = mt_batch();
        b.ops = s.ops;
        b.payload = s.pay;
        b.row_ptr = s.rp;
        b.n_ops = t.n_ops;
        b.payload_bytes = t.payload_bytes;
        b.n_docs = D;
        b.max_ops_per_doc = mx;
        b.wide = (flags & 2) != 0;
        const auto q0 = std::chrono::steady_clock::now();
        HIP_OK(hipEventSynchronize(s.applied));
        HIP_OK(hipEventSynchronize(s.drained));
        if (t.n_ops) HIP_OK(hipMemcpyAsync(s.ops, t.ops, t.n_ops * sizeof(mt_op_rec), hipMemcpyHostToDevice, e->h2d));
        if (t.payload_bytes) HIP_OK(hipMemcpyAsync(s.pay, t.payload, t.payload_bytes, hipMemcpyHostToDevice, e->h2d));
        HIP_OK(hipMemcpyAsync(s.rp, t.doc_row_ptr, (D + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, e->h2d));
        if (t.n_msgs) {
            HIP_OK(hipMemcpyAsync(s.msgs, t.msgs, t.n_msgs * sizeof(mt_raw_msg), hipMemcpyHostToDevice, e->h2d));
            HIP_OK(hipMemcpyAsync(s.mrp, t.msg_row_ptr, (D + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, e->h2d));
        }
        HIP_OK(hipEventRecord(s.ready, e->h2d));
        t_copy += std::chrono::duration<double>(std::chrono::steady_clock::now() - q0).count();
        return MT_OK;
    };
    if ((st = apply_begin(e))) return st;
    uint32_t nk = 0;
    // a tick that fails its checks ends the feed there: the ticks staged before it still apply
    uint32_t limit = n;
    mt_status refused = MT_OK;
    auto stage_or_stop = [&](uint32_t k) {
        if (k >= limit) return;
        if ((refused = stage(k))) limit = k;
    };
    // ticks 0 and 1 before the first apply (tick 1's check runs under tick 0's copy), then up to two per
    // tick (a check is ~1/3 of a copy: the copy stream stays busy, the host gets back to the next bin)
    uint32_t ns = 0;
    for (; ns < 2; ns++) stage_or_stop(ns);
    for (uint32_t k = 0; k < limit && !st; k++) {
        auto& s = e->ring[k % kRing];
        const mt_tick& t = ticks[k];
        const auto w0 = std::chrono::steady_clock::now();
        HIP_OK(hipEventSynchronize(s.ready));
        const double wk = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
        t_wait += wk;
        if (k < 64) wait_k[k] = wk;
        if (k == 0) {
            uint32_t f = 0;
            HIP_OK(mt_launch_scan_records(s.ops, t.n_ops, t.payload_bytes, e->d_scan, e->stream));
            HIP_OK(hipMemcpyAsync(&f, e->d_scan, sizeof f, hipMemcpyDeviceToHost, e->stream));
            HIP_OK(hipStreamSynchronize(e->stream));
            if (f & 1) {  // refused before anything of it ran: no tick applies
                refused = MT_ERR_ARG;
                limit = 0;
                break;
            }
            bs[0].wide = (f & 2) != 0;
        }
        if (t.n_msgs) {
            if ((st = mt_deli_ticket_on_stream(dl, e->cfg.device, e->stream, s.msgs, s.mrp, D, s.tk, s.ops, t.n_ops)))
                break;
            if (t.tickets) {
                HIP_OK(hipEventRecord(s.ticketed, e->stream));
                HIP_OK(hipStreamWaitEvent(e->d2h, s.ticketed, 0));
                HIP_OK(hipMemcpyAsync(t.tickets, s.tk, t.n_msgs * sizeof(mt_ticket), hipMemcpyDeviceToHost, e->d2h));
                HIP_OK(hipEventRecord(s.drained, e->d2h));
            }
        }
        const auto a0 = std::chrono::steady_clock::now();
        if ((st = apply_launches(e, &bs[k % kRing], nk))) break;
        t_apply += std::chrono::duration<double>(std::chrono::steady_clock::now() - a0).count();
        HIP_OK(hipEventRecord(s.applied, e->stream));
        // the next ticks' copies go out while this one applies (a slot is reused by tick k + kRing - 1 at
        // the latest; its tick, k - 1, is done: this tick's bin followed it on the engine stream)
        for (int j = 0; j < 2 && ns <= k + kRing - 1; j++, ns++) stage_or_stop(ns);
    }
    // (on an error the ticks in flight still land before the slots can be reused or freed)
    const mt_status se = apply_end(e, nk);
    HIP_OK(hipStreamSynchronize(e->h2d));
    HIP_OK(hipStreamSynchronize(e->d2h));
    if (const char* tv = getenv("MTGPU_TICK_TRACE"); tv && tv[0] == '1')
        fprintf(stderr, "mt_submit_ticks: %u ticks, %.2f ms: host checks %.2f ms, copy enqueue %.2f ms, waits for copies "
                "%.2f ms, apply loop %.2f ms, GPU wall %.2f ms\n", n,
                1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(),
                1e3 * t_check, 1e3 * t_copy, 1e3 * t_wait, 1e3 * t_apply, e->last_wall_ms);
    if (const char* tv = getenv("MTGPU_TICK_TRACE"); tv && tv[0] == '1') {
        fprintf(stderr, "  stream sync %.2f ms, ring %.2f ms; waits per tick (ms):",
                1e3 * std::chrono::duration<double>(t_synced - t_start).count(),
                1e3 * std::chrono::duration<double>(t_reserved - t_synced).count());
        for (uint32_t k = 0; k < std::min<uint32_t>(n, 64); k++) fprintf(stderr, " %.2f", 1e3 * wait_k[k]);
        fprintf(stderr, "; checks:");
        for (uint32_t k = 0; k < std::min<uint32_t>(n, 64); k++) fprintf(stderr, " %.2f", 1e3 * check_k[k]);
        fprintf(stderr, "\n");
    }
    return st ? st : se ? se : refused;
}
}  // namespace

extern "C" {

mt_status mt_batch_apply(mt_engine* e, const mt_batch* b) {
    if (!e || !b || b->n_docs != e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    mt_status st = apply_begin(e);
    uint32_t nk = 0;
    if (!st) st = apply_launches(e, b, nk);
    const mt_status se = apply_end(e, nk);
    return st ? st : se;
}

mt_status mt_submit_ticks(mt_engine* e, const mt_tick* ticks, uint32_t n_ticks) {
    if (e && ticks)
        for (uint32_t k = 0; k < n_ticks; k++)
            if (ticks[k].n_msgs) return MT_ERR_ARG;  // (raw messages need mt_submit_ticks_deli)
    return submit_ticks(e, nullptr, ticks, n_ticks);
}

mt_status mt_submit_ticks_deli(mt_engine* e, mt_deli* dl, const mt_tick* ticks, uint32_t n_ticks) {
    if (!dl) return MT_ERR_ARG;
    return submit_ticks(e, dl, ticks, n_ticks);
}

mt_status mt_log_to_ticks(const mt_op_rec* ops, uint64_t n_ops, const uint8_t* payload, uint64_t payload_bytes,
                          const uint32_t* doc_row_ptr, uint32_t n_docs, uint32_t per, const mt_raw_msg* msgs,
                          uint64_t n_msgs, const uint32_t* msg_row_ptr, mt_tick_layout* out) {
    return mt_log_to_ticks_ramp(ops, n_ops, payload, payload_bytes, doc_row_ptr, n_docs, per, per, msgs, n_msgs,
                                msg_row_ptr, out);
}

mt_status mt_log_to_ticks_ramp(const mt_op_rec* ops, uint64_t n_ops, const uint8_t* payload, uint64_t payload_bytes,
                               const uint32_t* doc_row_ptr, uint32_t n_docs, uint32_t per, uint32_t first,
                               const mt_raw_msg* msgs, uint64_t n_msgs, const uint32_t* msg_row_ptr,
                               mt_tick_layout* out) {
    if (!out || per == 0 || first == 0 || first > per || (n_ops && !ops) || (payload_bytes && !payload) ||
        (n_msgs && (!msgs || !msg_row_ptr)))
        return MT_ERR_ARG;
    uint32_t mx = 0;
    if (!row_ptr_ok(doc_row_ptr, n_docs, n_ops, &mx) || (msgs && !row_ptr_ok(msg_row_ptr, n_docs, n_msgs, nullptr)))
        return MT_ERR_ARG;
    // a ramp: tick t holds min(per, first << t) records of each document (first, 2 first, 4 first, ...,
    // then per): RT ramp ticks of [0, rs), then ticks of per
    uint32_t RT = 0;
    uint64_t rs = 0;
    while (((uint64_t)first << RT) < per) rs += (uint64_t)first << RT++;
    const uint32_t T = mx <= rs ? std::max<uint32_t>(1, [&] {
        uint32_t t = 0;
        for (uint64_t c = 0; c < mx; t++) c += (uint64_t)first << t;
        return t;
    }()) : RT + (uint32_t)((mx - rs + per - 1) / per);
    // documents in nt contiguous ranges; per range and tick: records, payload bytes, messages
    const unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 16u);
    const unsigned R = n_docs < 4096 ? 1u : nt;
    std::vector<uint64_t> cnt((size_t)R * T * 3, 0);
    std::atomic<bool> bad{false};
    auto tick_of = [&](uint32_t d, uint64_t rec) {
        const uint64_t l = rec - doc_row_ptr[d];
        if (l >= rs) return RT + (uint32_t)((l - rs) / per);
        uint32_t t = 0;  // (l < rs: inside the ramp, first * (2^(t+1) - 1) > l)
        while (((uint64_t)first << (t + 1)) - first <= l) t++;
        return t;
    };
    auto tick_start = [&](uint32_t t) {
        return t <= RT ? ((uint64_t)first << t) - first : rs + (uint64_t)(t - RT) * per;
    };
    // the tick of message i of document d (its record's, else the previous record's, else 0)
    auto run = [&](unsigned r, bool write, const std::vector<uint64_t>* base) {
        const uint32_t d0 = (uint32_t)((uint64_t)n_docs * r / R), d1 = (uint32_t)((uint64_t)n_docs * (r + 1) / R);
        uint64_t* c = cnt.data() + (size_t)r * T * 3;
        std::vector<uint64_t> o, p, m, start;  // write cursors per tick; a document's first record per tick
        if (write) {
            start.resize(T);
            o.resize(T);
            p.resize(T);
            m.resize(T);
            for (uint32_t t = 0; t < T; t++) {
                o[t] = (*base)[((size_t)r * T + t) * 3 + 0];
                p[t] = (*base)[((size_t)r * T + t) * 3 + 1];
                m[t] = (*base)[((size_t)r * T + t) * 3 + 2];
            }
        }
        for (uint32_t d = d0; d < d1; d++) {
            if (write) start = o;
            for (uint64_t i = doc_row_ptr[d]; i < doc_row_ptr[d + 1]; i++) {
                const uint32_t t = tick_of(d, i);
                const mt_op_rec& x = ops[i];
                if ((uint64_t)x.payload_off + x.payload_len > payload_bytes) {
                    bad = true;
                    return;
                }
                if (!write) {
                    c[t * 3 + 0]++;
                    c[t * 3 + 1] += x.payload_len;
                    continue;
                }
                mt_op_rec y = x;
                y.payload_off = (uint32_t)(p[t] - out->tick_payload[t]);
                memcpy(out->payload + p[t], payload + x.payload_off, x.payload_len);
                p[t] += x.payload_len;
                out->ops[o[t]++] = y;
            }
            if (write)
                for (uint32_t t = 0; t < T; t++) {
                    out->row_ptrs[(size_t)t * (n_docs + 1) + d + 1] = (uint32_t)(o[t] - out->tick_ops[t]);
                }
            if (!msgs) continue;
            uint32_t t = 0;
            uint64_t prev = 0;  // 1 + the last record a message of this document carried
            for (uint64_t i = msg_row_ptr[d]; i < msg_row_ptr[d + 1]; i++) {
                const mt_raw_msg& x = msgs[i];
                if (x.op_index) {
                    const uint64_t rec = x.op_index - 1;
                    // (a message carries a record of its own document, each record once and in stream
                    // order: a record behind the previous one would put its message in an earlier tick
                    // than the message before it, and deli would ticket the stream out of order)
                    if (rec < doc_row_ptr[d] || rec >= doc_row_ptr[d + 1] || x.op_index <= prev) {
                        bad = true;
                        return;
                    }
                    prev = x.op_index;
                    t = tick_of(d, rec);
                }
                if (!write) {
                    c[t * 3 + 2]++;
                    continue;
                }
                mt_raw_msg y = x;
                if (x.op_index) {
                    // the record's index inside its tick
                    const uint64_t rec = x.op_index - 1;
                    const uint64_t f = doc_row_ptr[d] + tick_start(t);  // the document's first record of tick t
                    y.op_index = (uint32_t)(start[t] - out->tick_ops[t] + (rec - f) + 1);
                }
                out->msgs[m[t]++] = y;
            }
            if (write)
                for (uint32_t tt = 0; tt < T; tt++)
                    out->msg_row_ptrs[(size_t)tt * (n_docs + 1) + d + 1] = (uint32_t)(m[tt] - out->tick_msgs[tt]);
        }
    };
    auto par = [&](bool write, const std::vector<uint64_t>* base) {
        if (R == 1) return run(0, write, base);
        std::vector<std::thread> th;
        for (unsigned r = 0; r < R; r++) th.emplace_back([&, r] { run(r, write, base); });
        for (auto& x : th) x.join();
    };
    par(false, nullptr);
    if (bad) return MT_ERR_ARG;
    // tick totals, and each range's first record / byte / message inside each tick
    std::vector<uint64_t> base((size_t)R * T * 3);
    std::vector<uint64_t> to(T + 1, 0), tp(T + 1, 0), tm(T + 1, 0);
    for (uint32_t t = 0; t < T; t++) {
        uint64_t a = to[t], b = tp[t], c = tm[t];
        for (unsigned r = 0; r < R; r++) {
            const uint64_t* q = cnt.data() + ((size_t)r * T + t) * 3;
            base[((size_t)r * T + t) * 3 + 0] = a;
            base[((size_t)r * T + t) * 3 + 1] = b;
            base[((size_t)r * T + t) * 3 + 2] = c;
            a += q[0];
            b += q[1];
            c += q[2];
        }
        to[t + 1] = a;
        tp[t + 1] = b;
        tm[t + 1] = c;
    }
    out->n_ticks = T;
    out->payload_bytes = tp[T];
    if (!out->ops) return MT_OK;  // (the sizing call)
    if (!out->payload && tp[T]) return MT_ERR_ARG;
    if (!out->row_ptrs || !out->tick_ops || !out->tick_payload ||
        (msgs && (!out->msgs || !out->msg_row_ptrs || !out->tick_msgs)))
        return MT_ERR_ARG;
    for (uint32_t t = 0; t <= T; t++) {
        out->tick_ops[t] = to[t];
        out->tick_payload[t] = tp[t];
        if (msgs) out->tick_msgs[t] = tm[t];
    }
    for (uint32_t t = 0; t < T; t++) {
        out->row_ptrs[(size_t)t * (n_docs + 1)] = 0;
        if (msgs) out->msg_row_ptrs[(size_t)t * (n_docs + 1)] = 0;
    }
    // (a document's row in tick t is written before its messages read it: one range writes both)
    par(true, &base);
    return bad ? MT_ERR_ARG : MT_OK;
}

static mt_status synth_generate(mt_engine* e, const mt_synth_cfg* cfg, uint32_t doc_id_base, const uint32_t* ids,
                                uint32_t payload_per_doc, mt_batch** out) {
    if (!e || !cfg || !out || cfg->n_clients == 0 || cfg->n_clients >= MT_MAX_CLIENTS || cfg->n_keys > MT_MAX_KEYS ||
        cfg->n_values > MT_MAX_VALUES)
        return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    e->gen++;
    const uint32_t n = e->n_docs, per = cfg->ops_per_doc;
    const uint64_t n_ops = (uint64_t)n * per;
    if (n_ops >= (1ull << 32) || (uint64_t)n * payload_per_doc >= (1ull << 32)) return MT_ERR_ARG;
    auto* b = new mt_batch();
    b->n_docs = n;
    b->n_ops = n_ops;
    b->payload_bytes = (uint64_t)n * payload_per_doc;
    b->max_ops_per_doc = per;
    std::vector<uint32_t> rp(n + 1);
    for (uint32_t d = 0; d <= n; d++) rp[d] = d * per;
    int32_t *cref = nullptr, *stall = nullptr;
    uint32_t *pay_used = nullptr, *gids = nullptr;
    if ((ids && hipMalloc(&gids, std::max<uint32_t>(1, n) * sizeof(uint32_t)) != hipSuccess) ||
        hipMalloc(&b->ops, std::max<uint64_t>(1, n_ops) * sizeof(mt_op_rec)) != hipSuccess ||
        hipMalloc(&b->payload, std::max<uint64_t>(1, b->payload_bytes)) != hipSuccess ||
        hipMalloc(&b->row_ptr, (n + 1) * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&cref, (size_t)n * 64 * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&stall, (size_t)n * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&pay_used, (size_t)n * sizeof(uint32_t)) != hipSuccess) {
        if (cref) (void)hipFree(cref);
        if (stall) (void)hipFree(stall);
        if (pay_used) (void)hipFree(pay_used);
        if (gids) (void)hipFree(gids);
        mt_batch_free(e, b);
        return MT_ERR_NOMEM;
    }
    mt_status st = MT_OK;
    hipError_t r = hipMemcpyAsync(b->row_ptr, rp.data(), (n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream);
    if (r == hipSuccess && gids)
        r = hipMemcpyAsync(gids, ids, n * sizeof(uint32_t), hipMemcpyHostToDevice, e->stream);
    if (r == hipSuccess) r = hipMemsetAsync(cref, 0, (size_t)n * 64 * sizeof(int32_t), e->stream);
    if (r == hipSuccess) r = hipMemsetAsync(stall, 0, (size_t)n * sizeof(int32_t), e->stream);
    if (r == hipSuccess) r = hipMemsetAsync(pay_used, 0, (size_t)n * sizeof(uint32_t), e->stream);
    const uint32_t tick = 64;
    for (uint32_t lo = 0; r == hipSuccess && lo < per; lo += tick) {
        r = hipMemsetAsync(e->d_counts, 0, kCounts * sizeof(uint32_t), e->stream);
        if (r == hipSuccess)
            r = mt_launch_bin(&e->g, b->row_ptr, n, lo, tick, e->d_classes, std::min(e->n_classes, kLdsClasses), 0,
                              kFirstWide, e->d_counts, e->d_ids, nullptr, nullptr, nullptr, e->stream);
        if (r == hipSuccess)
            r = hipMemcpyAsync(e->h_counts, e->d_counts, kNumClasses * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               e->stream);
        if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
        for (int c = 0; r == hipSuccess && c < std::min(e->n_classes, kLdsClasses); c++) {
            if (!e->h_counts[c]) continue;
            r = mt_launch_gen(lds_cap(kClasses[c]), &e->g, cfg, doc_id_base, gids, cref, stall, pay_used, payload_per_doc, b->ops,
                              b->payload, b->row_ptr, e->d_ids + (size_t)c * n, e->h_counts[c], lo, tick, e->stream);
        }
    }
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(cref);
    (void)hipFree(stall);
    (void)hipFree(pay_used);
    if (gids) (void)hipFree(gids);
    if (r != hipSuccess) {
        fprintf(stderr, "libmtgpu: mt_synth_generate: %s\n", hipGetErrorString(r));
        mt_batch_free(e, b);
        return MT_ERR_HIP;
    }
    *out = b;
    return st;
}

mt_status mt_synth_generate(mt_engine* e, const mt_synth_cfg* cfg, uint32_t doc_id_base, uint32_t payload_per_doc,
                            mt_batch** out) {
    return synth_generate(e, cfg, doc_id_base, nullptr, payload_per_doc, out);
}

mt_status mt_synth_generate_ids(mt_engine* e, const mt_synth_cfg* cfg, const uint32_t* doc_ids,
                                uint32_t payload_per_doc, mt_batch** out) {
    if (!doc_ids) return MT_ERR_ARG;
    return synth_generate(e, cfg, 0, doc_ids, payload_per_doc, out);
}

mt_status mt_batch_info(const mt_batch* b, uint64_t* n_ops, uint64_t* payload_bytes, uint32_t* max_ops_per_doc) {
    if (!b) return MT_ERR_ARG;
    if (n_ops) *n_ops = b->n_ops;
    if (payload_bytes) *payload_bytes = b->payload_bytes;
    if (max_ops_per_doc) *max_ops_per_doc = b->max_ops_per_doc;
    return MT_OK;
}

mt_status mt_batch_device_ptrs(const mt_batch* b, mt_op_rec** ops, uint8_t** payload, uint32_t** row_ptr) {
    if (!b) return MT_ERR_ARG;
    if (ops) *ops = b->ops;
    if (payload) *payload = b->payload;
    if (row_ptr) *row_ptr = b->row_ptr;
    return MT_OK;
}

mt_status mt_batch_copy_docs(mt_engine* e, const mt_batch* b, uint32_t d0, uint32_t d1, mt_op_rec* ops,
                             uint64_t* n_ops, uint8_t* payload, uint64_t* payload_bytes, uint32_t* row_ptr) {
    if (!e || !b || d0 > d1 || d1 > b->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    std::vector<uint32_t> rp(d1 - d0 + 1);
    HIP_OK(hipMemcpyAsync(rp.data(), b->row_ptr + d0, rp.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    const uint64_t cnt = rp.back() - rp.front();
    std::vector<mt_op_rec> tmp(cnt);
    if (cnt)
        HIP_OK(hipMemcpyAsync(tmp.data(), b->ops + rp.front(), cnt * sizeof(mt_op_rec), hipMemcpyDeviceToHost,
                              e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    uint64_t lo = ~0ull, hi = 0;
    for (const auto& o : tmp) {
        lo = std::min<uint64_t>(lo, o.payload_off);
        hi = std::max<uint64_t>(hi, (uint64_t)o.payload_off + o.payload_len);
    }
    if (!cnt) lo = hi = 0;
    if (n_ops) *n_ops = cnt;
    if (payload_bytes) *payload_bytes = hi - lo;
    if (row_ptr)
        for (size_t i = 0; i < rp.size(); i++) row_ptr[i] = rp[i] - rp.front();
    if (ops) {
        for (auto& o : tmp) o.payload_off -= (uint32_t)lo;
        memcpy(ops, tmp.data(), cnt * sizeof(mt_op_rec));
    }
    if (payload && hi > lo) {
        HIP_OK(hipMemcpyAsync(payload, b->payload + lo, hi - lo, hipMemcpyDeviceToHost, e->stream));
        HIP_OK(hipStreamSynchronize(e->stream));
    }
    return MT_OK;
}

mt_status mt_submit(mt_engine* e, const mt_op_rec* ops, uint64_t n_ops, const uint8_t* payload,
                    uint64_t payload_bytes, const uint32_t* doc_row_ptr) {
    mt_batch* b = nullptr;
    mt_status st = mt_batch_upload(e, ops, n_ops, payload, payload_bytes, doc_row_ptr, &b);
    if (st) return st;
    st = mt_batch_apply(e, b);
    mt_batch_free(e, b);
    return st;
}

mt_status mt_sync(mt_engine* e) {
    if (!e) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HIP_OK(hipStreamSynchronize(e->stream));
    return MT_OK;
}

mt_status mt_set_concurrent_classes(mt_engine* e, int on) {
    if (!e) return MT_ERR_ARG;
    e->concurrent = on != 0;
    return MT_OK;
}

mt_status mt_last_apply_stats(mt_engine* e, float* ms, float* wall_ms, uint32_t* launches, uint64_t* alg_bytes) {
    if (!e) return MT_ERR_ARG;
    if (ms) *ms = e->last_ms;
    if (wall_ms) *wall_ms = e->last_wall_ms;
    if (launches) *launches = e->last_launches;
    if (alg_bytes) *alg_bytes = e->last_bytes;
    return MT_OK;
}

mt_status mt_last_apply_class_stats(mt_engine* e, uint32_t cls, uint32_t* capacity, float* kernel_ms,
                                    uint32_t* launches, uint64_t* alg_bytes) {
    if (!e || cls >= (uint32_t)kStatClasses) return MT_ERR_ARG;
    if (capacity) {
        const uint32_t q = cls - kNumClasses - 1;  // (past the editing bucket)
        *capacity = cls >= (uint32_t)kStatWide          ? (MT_CLASS_WIDE | (uint32_t)kClasses[kFirstWide + cls - kStatWide])
                    : cls < (uint32_t)kNumClasses       ? (uint32_t)kClasses[cls]
                    : cls == (uint32_t)kNumClasses      ? (MT_CLASS_EDITING | MT_LOC_CAP)
                    : q < (uint32_t)kFirstLds           ? (MT_CLASS_LDS | (uint32_t)kClasses[q])
                    : q < (uint32_t)(2 * kFirstLds)     ? (MT_CLASS_C64 | (uint32_t)kClasses[q - kFirstLds])
                                                        : (MT_CLASS_EDITING | (kLocGW[q - 2 * kFirstLds] > 1 ? MT_CLASS_GROUPS : 0u) |
                                                           (uint32_t)kLocCaps[q - 2 * kFirstLds]);
    }
    if (kernel_ms) *kernel_ms = e->cls_ms[cls];
    if (launches) *launches = e->cls_launches[cls];
    if (alg_bytes) *alg_bytes = e->cls_bytes[cls];
    return MT_OK;
}

mt_status mt_class_kernel_name(mt_engine* e, uint32_t capacity, char* buf, uint64_t cap) {
    if (!e || !buf || !cap) return MT_ERR_ARG;
    char tmp[96];
    if ((capacity & MT_CLASS_EDITING) && (capacity & MT_CLASS_GROUPS))
        snprintf(tmp, sizeof tmp, "mt::apply_kernel_g<%u, false, true, %d>",
                 capacity & ~(uint32_t)(MT_CLASS_EDITING | MT_CLASS_GROUPS), MT_LOC_GW);
    else if ((capacity & MT_CLASS_EDITING) && (capacity & ~(uint32_t)MT_CLASS_EDITING) > MT_LOC_CAP)
        snprintf(tmp, sizeof tmp, "mt::apply_kernel_g<%u, false, true, 1>", capacity & ~(uint32_t)MT_CLASS_EDITING);
    else if (capacity & MT_CLASS_EDITING)
        snprintf(tmp, sizeof tmp, "mt::apply_kernel<%u, false, true>", capacity & ~(uint32_t)MT_CLASS_EDITING);
    else if ((capacity & MT_CLASS_WIDE) && (capacity & ~(uint32_t)MT_CLASS_WIDE) <= 512)
        snprintf(tmp, sizeof tmp, "mt::apply_kernel_wl<%u>", (capacity & ~(uint32_t)MT_CLASS_WIDE) <= 256 ? 256u : 512u);
    else if (capacity & MT_CLASS_WIDE)
        snprintf(tmp, sizeof tmp, "mt::apply_kernel_g<%u, true>",
                 std::max<uint32_t>(1024u, capacity & ~(uint32_t)MT_CLASS_WIDE));
    else if ((capacity & MT_CLASS_C64) && e->g.ev)
        snprintf(tmp, sizeof tmp, "mt::apply_kernel<%d, false>", lds_cap((int)(capacity & ~(uint32_t)MT_CLASS_C64)));
    else if (capacity & MT_CLASS_C64)
        snprintf(tmp, sizeof tmp, "mtr::reg_apply_kernel_c64<%u>", (capacity & ~(uint32_t)MT_CLASS_C64) / 64);
    else if (capacity & MT_CLASS_LDS)
        snprintf(tmp, sizeof tmp, "mt::apply_kernel<%d, false>", lds_cap((int)(capacity & ~(uint32_t)MT_CLASS_LDS)));
    else if (e->use_reg && capacity <= (uint32_t)kRegMaxCap)
        snprintf(tmp, sizeof tmp, e->g.ev ? "mtr::reg_apply_kernel_ev<%u>" : "mtr::reg_apply_kernel<%u>", capacity / 64);
    else if (capacity > 2048)
        snprintf(tmp, sizeof tmp, "mt::apply_kernel_g<%u>", capacity);
    else
        snprintf(tmp, sizeof tmp, "mt::apply_kernel<%d, false>", lds_cap((int)capacity));
    const size_t n = std::min<size_t>(cap - 1, strlen(tmp));
    memcpy(buf, tmp, n);
    buf[n] = 0;
    return MT_OK;
}

mt_status mt_checksums_device(mt_engine* e, uint64_t* d_out, uint32_t n_docs) {
    if (!e || !d_out || n_docs > e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    if (!n_docs) return MT_OK;
    HIP_OK(mt_launch_checksum(&e->g, n_docs, d_out, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    return MT_OK;
}

mt_status mt_checksums(mt_engine* e, uint64_t* out, uint32_t n_docs) {
    if (!e || !out || n_docs > e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    uint64_t* d = nullptr;
    HIP_OK(hipMalloc(&d, std::max<uint32_t>(1, n_docs) * sizeof(uint64_t)));
    hipError_t r = mt_launch_checksum(&e->g, n_docs, d, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(out, d, n_docs * sizeof(uint64_t), hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    hipFree(d);
    return r == hipSuccess ? MT_OK : MT_ERR_HIP;
}

mt_status mt_seg_counts(mt_engine* e, uint32_t* out, uint32_t n_docs) {
    if (!e || !out || n_docs > e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    std::vector<mt_doc_scalars> sc(n_docs);
    HIP_OK(hipMemcpyAsync(sc.data(), e->g.sc, n_docs * sizeof(mt_doc_scalars), hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    for (uint32_t d = 0; d < n_docs; d++) out[d] = (uint32_t)sc[d].nseg;
    return MT_OK;
}

mt_status mt_doc_error(mt_engine* e, uint32_t doc, int32_t* code, int32_t* seq) {
    if (!e || doc >= e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    mt_doc_scalars sc;
    HIP_OK(hipMemcpyAsync(&sc, e->g.sc + doc, sizeof sc, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    if (code) *code = sc.err;
    if (seq) *seq = sc.err_seq;
    return MT_OK;
}

}  // extern "C"

// ------------------------------------------------------------------- canonical readout
namespace {
// A document's state on the host, narrow or wide (mt_state.h): text as UTF-16 code units, props as
// a value id per key, overlap as a sorted client list
struct HostDoc {
    mt_doc_scalars sc;
    bool wide = false;
    std::vector<int32_t> seq, rseq;
    std::vector<uint32_t> len, toff;
    std::vector<uint64_t> ovl, props, ovx, ph, pxl, pxh, pxx;
    std::vector<uint8_t> client, rclient, flags;
    std::vector<uint16_t> chi;                 // (wide) the short ids' high bytes
    std::vector<uint16_t> text;                // the arena's current half, in code units
    std::vector<std::vector<uint8_t>> levels;  // per level child counts (level 0 = leaf blocks)
    uint32_t prop(int i, int k) const {
        const int sh = 8 * (k & 7);
        if (!wide) return k < 8 ? (uint32_t)((props[i] >> sh) & 0xFF) : 0u;
        if (k >= 16 && !(sc.wide & MT_WIDE_XKV)) return 0u;  // (no keys 16..31 stored)
        const uint64_t lo = k < 8 ? props[i] : k < 16 ? pxl[i] : pxx[4 * (size_t)i + 2 * ((k - 16) >> 3)];
        const uint64_t hi = k < 8 ? ph[i] : k < 16 ? pxh[i] : pxx[4 * (size_t)i + 2 * ((k - 16) >> 3) + 1];
        return (uint32_t)((lo >> sh) & 0xFF) | ((uint32_t)((hi >> sh) & 0xFF) << 8);
    }
    std::vector<int> overlap(int i) const {
        std::vector<int> v;
        for (int c = 0; c < 64; c++)
            if ((ovl[i] >> c) & 1) v.push_back(c);
        if (wide) {
            const uint64_t* x = ovx.data() + (size_t)MT_OVX_WORDS * i;
            for (int q = 0; q < MT_OVX_IDS; q++) {
                const int c = (int)mt_ovx_id2(x, (sc.wide & MT_WIDE_XOV) ? x + 4 : nullptr, q);
                if (!c) break;
                v.push_back(c);
            }
        }
        return v;
    }
    uint32_t client_of(int i) const { return client[i] | (wide ? (uint32_t)(chi[i] & 0xFF) << 8 : 0u); }
    uint32_t rclient_of(int i) const { return rclient[i] | (wide ? (uint32_t)(chi[i] >> 8) << 8 : 0u); }
    const uint16_t* units(int i) const { return text.data() + toff[i]; }
};

template <class T>
hipError_t fetch(std::vector<T>& v, const T* base, size_t off, size_t n, hipStream_t st) {
    v.resize(n);
    if (!n) return hipSuccess;
    return hipMemcpyAsync(v.data(), base + off, n * sizeof(T), hipMemcpyDeviceToHost, st);
}

// the current arena half of document d as code units (a narrow document's bytes widened)
mt_status fetch_text(mt_engine* e, uint32_t d, const mt_doc_scalars& sc, std::vector<uint16_t>& out) {
    const mt_gstate& g = e->g;
    const size_t base = ((size_t)d * 2 + sc.text_half) * g.textcap;
    if (sc.wide & MT_WIDE_DOC) {
        out.resize(sc.text_top);
        if (sc.text_top)
            HIP_OK(hipMemcpyAsync(out.data(), g.text + base, (size_t)sc.text_top * 2, hipMemcpyDeviceToHost, e->stream));
        HIP_OK(hipStreamSynchronize(e->stream));
        return MT_OK;
    }
    std::vector<uint8_t> b;
    HIP_OK(fetch(b, g.text, base, sc.text_top, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    out.assign(b.begin(), b.end());
    return MT_OK;
}

mt_status read_doc(mt_engine* e, uint32_t d, HostDoc& h) {
    const mt_gstate& g = e->g;
    HIP_OK(hipMemcpyAsync(&h.sc, g.sc + d, sizeof h.sc, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    h.wide = (h.sc.wide & MT_WIDE_DOC) != 0 && g.ovx;
    const size_t so = (size_t)d * g.segcap, n = (size_t)h.sc.nseg;
    HIP_OK(fetch(h.seq, g.seq, so, n, e->stream));
    HIP_OK(fetch(h.rseq, g.rseq, so, n, e->stream));
    HIP_OK(fetch(h.len, g.len, so, n, e->stream));
    HIP_OK(fetch(h.toff, g.toff, so, n, e->stream));
    HIP_OK(fetch(h.ovl, g.ovl, so, n, e->stream));
    HIP_OK(fetch(h.props, g.props, so, n, e->stream));
    if (h.wide) {
        HIP_OK(fetch(h.ovx, g.ovx, so * MT_OVX_WORDS, n * MT_OVX_WORDS, e->stream));
        HIP_OK(fetch(h.chi, g.chi, so, n, e->stream));
        HIP_OK(fetch(h.ph, g.ph, so, n, e->stream));
        HIP_OK(fetch(h.pxl, g.pxl, so, n, e->stream));
        HIP_OK(fetch(h.pxh, g.pxh, so, n, e->stream));
        HIP_OK(fetch(h.pxx, g.pxx, so * 4, n * 4, e->stream));
    }
    HIP_OK(fetch(h.client, g.client, so, n, e->stream));
    HIP_OK(fetch(h.rclient, g.rclient, so, n, e->stream));
    HIP_OK(fetch(h.flags, g.flags, so, n, e->stream));
    h.levels.resize(h.sc.nlev);
    for (int L = 0; L < h.sc.nlev; L++) {
        if (L == 0) HIP_OK(fetch(h.levels[0], g.lbcnt, (size_t)d * g.lbcap, h.sc.nb[0], e->stream));
        else HIP_OK(fetch(h.levels[L], g.ibcnt, ((size_t)d * (MT_MAXLEV - 1) + (L - 1)) * g.ibcap, h.sc.nb[L], e->stream));
    }
    HIP_OK(hipStreamSynchronize(e->stream));
    return fetch_text(e, d, h.sc, h.text);
}

// A JSON string of UTF-16 code units, ASCII only: printable ASCII as itself, \" \\ and the short
// forms JSON.stringify uses (ECMA-262 QuoteJSONString), every other unit -- non-ASCII and surrogate
// halves included -- as \uXXXX.  It parses to the same string the reference's JSON holds.
void json_units(std::string& o, const uint16_t* p, size_t n) {
    o += '"';
    for (size_t i = 0; i < n; i++) {
        const unsigned c = p[i];
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\b': o += "\\b"; break;
            case '\t': o += "\\t"; break;
            case '\n': o += "\\n"; break;
            case '\f': o += "\\f"; break;
            case '\r': o += "\\r"; break;
            default:
                if (c < 0x20 || c >= 0x7F) {
                    char buf[8];
                    snprintf(buf, sizeof buf, "\\u%04x", c);
                    o += buf;
                } else {
                    o += (char)c;
                }
        }
    }
    o += '"';
}

std::string state_json(const HostDoc& h) {
    std::string o = "{\"seq\":" + std::to_string(h.sc.cur_seq) + ",\"msn\":" + std::to_string(h.sc.min_seq) + ",\"segs\":[";
    for (int i = 0; i < h.sc.nseg; i++) {
        if (i) o += ',';
        o += '[';
        if (h.flags[i] & MT_SF_MARKER)  // a Marker: {"marker": refType}
            o += "{\"marker\":" + std::to_string(h.units(i)[0]) + "}";
        else
            json_units(o, h.units(i), h.len[i]);
        const bool rm = h.flags[i] & MT_SF_REMOVED;
        o += ',' + std::to_string(h.seq[i]) + ',' + std::to_string(mt_canon_client(h.client_of(i))) + ',';
        o += (rm ? std::to_string(h.rseq[i]) : "-1") + ',' + (rm ? std::to_string(h.rclient_of(i)) : "-1") + ",[";
        bool f = true;
        for (int c : h.overlap(i)) {
            if (!f) o += ',';
            f = false;
            o += std::to_string(c);
        }
        o += "],";
        if (!(h.flags[i] & MT_SF_PDEF)) {
            o += "null";
        } else {
            o += '{';
            bool f2 = true;
            for (int k = 0; k < MT_MAX_KEYS_WIDE; k++) {
                const unsigned v = h.prop(i, k);
                if (!v) continue;
                if (!f2) o += ',';
                f2 = false;
                o += "\"k" + std::to_string(k) + "\":" + std::to_string(v);
            }
            o += '}';
        }
        o += ']';
    }
    o += "],\"tree\":[";
    for (int depth = 0; depth < h.sc.nlev; depth++) {
        const auto& lv = h.levels[h.sc.nlev - 1 - depth];
        if (depth) o += ',';
        o += '[';
        for (size_t b = 0; b < lv.size(); b++) {
            if (b) o += ',';
            o += std::to_string(lv[b]);
        }
        o += ']';
    }
    o += "]}";
    return o;
}

// props as the reference's map: keys "k<id>" (interned key ids), values = interned value ids
void props_json(std::string& o, const HostDoc& h, int i) {
    o += '{';
    bool first = true;
    for (int k = 0; k < MT_MAX_KEYS_WIDE; k++) {
        const unsigned v = h.prop(i, k);
        if (!v) continue;
        if (!first) o += ',';
        first = false;
        o += "\"k" + std::to_string(k) + "\":" + std::to_string(v);
    }
    o += '}';
}

// TextSegment.toJSONObject (textSegment.ts:47-53) of `text` with the props of segment i;
// Marker.toJSONObject (mergeTree.ts:652-656) for a marker: {marker: {refType}, props?}
void seg_json(std::string& o, const HostDoc& h, int i, const std::vector<uint16_t>& text) {
    if (h.flags[i] & MT_SF_MARKER) {
        o += "{\"marker\":{\"refType\":" + std::to_string(h.units(i)[0]) + "}";
        if (h.flags[i] & MT_SF_PDEF) {
            o += ",\"props\":";
            props_json(o, h, i);
        }
        o += '}';
    } else if (h.flags[i] & MT_SF_PDEF) {
        o += "{\"text\":";
        json_units(o, text.data(), text.size());
        o += ",\"props\":";
        props_json(o, h, i);
        o += '}';
    } else {
        json_units(o, text.data(), text.size());
    }
}

std::string client_name(const char* const* names, uint32_t n_names, uint32_t c) {
    if (c == MT_CLIENT_NONCOLLAB) return "original";  // Client.getLongClientId of a negative id (client.ts:645-652)
    if (names && c < n_names && names[c]) return names[c];
    return std::to_string(c);
}

// SnapshotV1.emit (snapshotV1.ts:85-149) from the device's extraction specs: the tree entries as
// one JSON object {"header": chunk, "body_0": chunk, ...}
std::string snapshot_json(const HostDoc& h, const std::vector<uint32_t>& sp, uint32_t nspec, uint32_t chunk,
                          const char* const* names, uint32_t n_names) {
    std::vector<std::string> specs(nspec);
    std::vector<uint32_t> lens(nspec);
    for (uint32_t k = 0; k < nspec; k++) {
        const int pos = (int)sp[3 * k];
        const int cnt = (int)(sp[3 * k + 1] >> 1);
        const bool meta = sp[3 * k + 1] & 1u;
        std::vector<uint16_t> text;
        for (int i = pos; i < pos + cnt; i++) {
            // elided inside the run: removed at or below the MSN, or a pending local insert / removal
            if (h.seq[i] == -1 || ((h.flags[i] & MT_SF_REMOVED) && h.rseq[i] <= h.sc.min_seq)) continue;
            text.insert(text.end(), h.units(i), h.units(i) + h.len[i]);
        }
        lens[k] = sp[3 * k + 2];
        std::string& o = specs[k];
        if (!meta) {
            seg_json(o, h, pos, text);
            continue;
        }
        o += "{\"json\":";
        seg_json(o, h, pos, text);
        if (h.seq[pos] > h.sc.min_seq)
            o += ",\"seq\":" + std::to_string(h.seq[pos]) + ",\"client\":\"" + client_name(names, n_names, h.client_of(pos)) +
                 "\"";
        if (h.flags[pos] & MT_SF_REMOVED)
            o += ",\"removedSeq\":" + std::to_string(h.rseq[pos]) + ",\"removedClient\":\"" +
                 client_name(names, n_names, h.rclient_of(pos)) + "\"";
        o += '}';
    }
    // getSeqLengthSegs (:57-79): chunks of >= `chunk` characters
    struct Chunk { uint32_t start, count; uint64_t length; };
    std::vector<Chunk> chunks;
    uint32_t total_count = 0;
    uint64_t total_len = 0;
    do {
        Chunk c{total_count, 0, 0};
        while (c.length < chunk && c.start + c.count < nspec) c.length += lens[c.start + c.count++];
        chunks.push_back(c);
        total_count += c.count;
        total_len += c.length;
    } while (total_count < nspec);
    auto chunk_json = [&](const Chunk& c, bool header) {
        std::string o = "{\"version\":\"1\",\"segmentCount\":" + std::to_string(c.count) + ",\"length\":" +
                        std::to_string(c.length) + ",\"segments\":[";
        for (uint32_t k = 0; k < c.count; k++) {
            if (k) o += ',';
            o += specs[c.start + k];
        }
        o += "],\"startIndex\":" + std::to_string(c.start);
        if (header) {
            o += ",\"headerMetadata\":{\"minSequenceNumber\":" + std::to_string(h.sc.min_seq) +
                 ",\"sequenceNumber\":" + std::to_string(h.sc.cur_seq) + ",\"orderedChunkMetadata\":[{\"id\":\"header\"}";
            for (size_t b = 1; b < chunks.size(); b++) o += ",{\"id\":\"body_" + std::to_string(b - 1) + "\"}";
            o += "],\"totalLength\":" + std::to_string(total_len) + ",\"totalSegmentCount\":" +
                 std::to_string(total_count) + '}';
        }
        return o + '}';
    };
    std::string o = "{\"header\":" + chunk_json(chunks[0], true);
    for (size_t b = 1; b < chunks.size(); b++) o += ",\"body_" + std::to_string(b - 1) + "\":" + chunk_json(chunks[b], false);
    return o + '}';
}

// Documents [d0, d0 + n) to the host in one pass: every field of the range in one copy each, the
// text arenas per document, all asynchronous behind one synchronisation
mt_status read_range(mt_engine* e, uint32_t d0, uint32_t n, std::vector<HostDoc>& out) {
    const mt_gstate& g = e->g;
    std::vector<mt_doc_scalars> sc(n);
    HIP_OK(hipMemcpyAsync(sc.data(), g.sc + d0, n * sizeof(mt_doc_scalars), hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    const size_t S = (size_t)n * g.segcap, so = (size_t)d0 * g.segcap;
    std::vector<int32_t> seq, rseq;
    std::vector<uint32_t> len, toff;
    std::vector<uint64_t> ovl, props, ovx, ph, pxl, pxh, pxx;
    std::vector<uint8_t> client, rclient, flags, lb, ib;
    std::vector<uint16_t> chi;
    bool any_wide = false;
    for (uint32_t i = 0; i < n; i++) any_wide = any_wide || ((sc[i].wide & MT_WIDE_DOC) && g.ovx);
    HIP_OK(fetch(seq, g.seq, so, S, e->stream));
    HIP_OK(fetch(rseq, g.rseq, so, S, e->stream));
    HIP_OK(fetch(len, g.len, so, S, e->stream));
    HIP_OK(fetch(toff, g.toff, so, S, e->stream));
    HIP_OK(fetch(ovl, g.ovl, so, S, e->stream));
    HIP_OK(fetch(props, g.props, so, S, e->stream));
    if (any_wide) {
        HIP_OK(fetch(ovx, g.ovx, so * MT_OVX_WORDS, S * MT_OVX_WORDS, e->stream));
        HIP_OK(fetch(chi, g.chi, so, S, e->stream));
        HIP_OK(fetch(ph, g.ph, so, S, e->stream));
        HIP_OK(fetch(pxl, g.pxl, so, S, e->stream));
        HIP_OK(fetch(pxh, g.pxh, so, S, e->stream));
        HIP_OK(fetch(pxx, g.pxx, so * 4, S * 4, e->stream));
    }
    HIP_OK(fetch(client, g.client, so, S, e->stream));
    HIP_OK(fetch(rclient, g.rclient, so, S, e->stream));
    HIP_OK(fetch(flags, g.flags, so, S, e->stream));
    HIP_OK(fetch(lb, g.lbcnt, (size_t)d0 * g.lbcap, (size_t)n * g.lbcap, e->stream));
    HIP_OK(fetch(ib, g.ibcnt, (size_t)d0 * (MT_MAXLEV - 1) * g.ibcap, (size_t)n * (MT_MAXLEV - 1) * g.ibcap, e->stream));
    out.assign(n, HostDoc());
    HIP_OK(hipStreamSynchronize(e->stream));
    for (uint32_t i = 0; i < n; i++) {
        HostDoc& h = out[i];
        h.sc = sc[i];
        h.wide = (sc[i].wide & MT_WIDE_DOC) && g.ovx;
        mt_status st = fetch_text(e, d0 + i, sc[i], h.text);
        if (st) return st;
        const size_t a = (size_t)i * g.segcap, m = (size_t)h.sc.nseg;
        h.seq.assign(seq.begin() + a, seq.begin() + a + m);
        h.rseq.assign(rseq.begin() + a, rseq.begin() + a + m);
        h.len.assign(len.begin() + a, len.begin() + a + m);
        h.toff.assign(toff.begin() + a, toff.begin() + a + m);
        h.ovl.assign(ovl.begin() + a, ovl.begin() + a + m);
        h.props.assign(props.begin() + a, props.begin() + a + m);
        if (h.wide) {
            h.ovx.assign(ovx.begin() + a * MT_OVX_WORDS, ovx.begin() + (a + m) * MT_OVX_WORDS);
            h.chi.assign(chi.begin() + a, chi.begin() + a + m);
            h.ph.assign(ph.begin() + a, ph.begin() + a + m);
            h.pxl.assign(pxl.begin() + a, pxl.begin() + a + m);
            h.pxh.assign(pxh.begin() + a, pxh.begin() + a + m);
            h.pxx.assign(pxx.begin() + a * 4, pxx.begin() + (a + m) * 4);
        }
        h.client.assign(client.begin() + a, client.begin() + a + m);
        h.rclient.assign(rclient.begin() + a, rclient.begin() + a + m);
        h.flags.assign(flags.begin() + a, flags.begin() + a + m);
        h.levels.resize(h.sc.nlev);
        for (int L = 0; L < h.sc.nlev; L++) {
            const uint8_t* src = L == 0 ? lb.data() + (size_t)i * g.lbcap
                                        : ib.data() + ((size_t)i * (MT_MAXLEV - 1) + (L - 1)) * g.ibcap;
            h.levels[L].assign(src, src + h.sc.nb[L]);
        }
    }
    return MT_OK;
}

mt_status copy_out(const std::string& s, char* buf, uint64_t cap, uint64_t* len) {
    if (len) *len = s.size();
    if (buf && cap) {
        const uint64_t n = std::min<uint64_t>(cap - 1, s.size());
        memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return MT_OK;
}
}  // namespace

extern "C" {

mt_status mt_get_state(mt_engine* e, uint32_t doc, char* buf, uint64_t cap, uint64_t* len) {
    if (!e || doc >= e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HostDoc h;
    mt_status st = read_doc(e, doc, h);
    if (st) return st;
    return copy_out(state_json(h), buf, cap, len);
}

mt_status mt_get_snapshot(mt_engine* e, uint32_t doc, uint32_t chunk_size, const char* const* client_names,
                          uint32_t n_names, char* buf, uint64_t cap, uint64_t* len) {
    if (!e || doc >= e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HostDoc h;
    mt_status st = read_doc(e, doc, h);
    if (st) return st;
    const uint32_t scap = std::max<uint32_t>(1, (uint32_t)h.sc.nseg);
    uint32_t* d = nullptr;
    HIP_OK(hipMalloc(&d, (3 * (size_t)scap + 1) * sizeof(uint32_t)));
    std::vector<uint32_t> sp(3 * (size_t)scap);
    uint32_t nspec = 0;
    hipError_t r = mt_launch_snapshot(&e->g, doc, 1, scap, d + 1, d, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(&nspec, d, sizeof nspec, hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipMemcpyAsync(sp.data(), d + 1, sp.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream);
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
    (void)hipFree(d);
    if (r != hipSuccess) return MT_ERR_HIP;
    if (nspec > scap) return MT_ERR_STATE;
    return copy_out(snapshot_json(h, sp, nspec, chunk_size ? chunk_size : 10000u, client_names, n_names), buf, cap,
                    len);
}

mt_status mt_get_snapshots(mt_engine* e, uint32_t d0, uint32_t n, uint32_t chunk_size, const char* const* client_names,
                           uint32_t n_names, char* buf, uint64_t cap, uint64_t* offsets) {
    if (!e || !offsets || d0 > e->n_docs || n > e->n_docs - d0) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    // a sizing call (buf NULL) leaves its result for the copying call with the same arguments
    auto& c = e->snap_cache;
    const bool hit = c.valid && c.gen == e->gen && c.d0 == d0 && c.n == n && c.chunk == chunk_size && c.names == client_names &&
                     c.n_names == n_names;
    if (!hit) {
        c.valid = false;
        c.json.clear();
        c.off.assign(n + 1, 0);
        if (n) {
            std::vector<HostDoc> docs;
            mt_status st = read_range(e, d0, n, docs);
            if (st) return st;
            // the device extraction of every document in one launch
            const uint32_t scap = e->g.segcap;
            uint32_t *specs = nullptr, *counts = nullptr;
            if (hipMalloc(&specs, (size_t)n * scap * 3 * sizeof(uint32_t)) != hipSuccess) return MT_ERR_NOMEM;
            if (hipMalloc(&counts, (size_t)n * sizeof(uint32_t)) != hipSuccess) {
                (void)hipFree(specs);
                return MT_ERR_NOMEM;
            }
            std::vector<uint32_t> hc(n), hs((size_t)n * scap * 3);
            hipError_t r = mt_launch_snapshot(&e->g, d0, n, scap, specs, counts, e->stream);
            if (r == hipSuccess) r = hipMemcpyAsync(hc.data(), counts, n * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream);
            if (r == hipSuccess) r = hipMemcpyAsync(hs.data(), specs, hs.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream);
            if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
            (void)hipFree(specs);
            (void)hipFree(counts);
            if (r != hipSuccess) return MT_ERR_HIP;
            // the JSON of each document on the host cores, in parallel
            std::vector<std::string> parts(n);
            std::atomic<uint32_t> next{0};
            std::atomic<int> bad{0};
            const unsigned nt = std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), std::min(16u, n));
            auto work = [&] {
                for (uint32_t i; (i = next.fetch_add(1)) < n;) {
                    if (hc[i] > scap) {
                        bad = 1;
                        continue;
                    }
                    std::vector<uint32_t> sp(hs.begin() + (size_t)i * scap * 3, hs.begin() + ((size_t)i * scap + hc[i]) * 3);
                    parts[i] = snapshot_json(docs[i], sp, hc[i], chunk_size ? chunk_size : 10000u, client_names, n_names);
                }
            };
            std::vector<std::thread> th;
            for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
            work();
            for (auto& x : th) x.join();
            if (bad) return MT_ERR_STATE;
            for (uint32_t i = 0; i < n; i++) c.off[i + 1] = c.off[i] + parts[i].size();
            c.json.reserve(c.off[n]);
            for (auto& p : parts) c.json += p;
        }
        c.valid = true;
        c.gen = e->gen;
        c.d0 = d0;
        c.n = n;
        c.chunk = chunk_size;
        c.names = client_names;
        c.n_names = n_names;
    }
    for (uint32_t i = 0; i <= n; i++) offsets[i] = c.off[i];
    if (!buf) return MT_OK;
    if (cap < c.json.size()) return MT_ERR_ARG;
    memcpy(buf, c.json.data(), c.json.size());
    c.valid = false;  // consumed
    c.json.clear();
    c.json.shrink_to_fit();
    return MT_OK;
}

mt_status mt_snapshot_extract(mt_engine* e, uint32_t d0, uint32_t n, float* kernel_ms, uint64_t* n_specs) {
    if (!e || d0 > e->n_docs || n > e->n_docs - d0) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    if (n == 0) return MT_OK;
    const uint32_t cap = e->g.segcap;
    uint32_t *specs = nullptr, *counts = nullptr;
    if (hipMalloc(&specs, (size_t)n * cap * 3 * sizeof(uint32_t)) != hipSuccess) return MT_ERR_NOMEM;
    if (hipMalloc(&counts, (size_t)n * sizeof(uint32_t)) != hipSuccess) {
        (void)hipFree(specs);
        return MT_ERR_NOMEM;
    }
    hipError_t r = hipEventRecord(e->ev0, e->stream);
    if (r == hipSuccess) r = mt_launch_snapshot(&e->g, d0, n, cap, specs, counts, e->stream);
    if (r == hipSuccess) r = hipEventRecord(e->ev1, e->stream);
    if (r == hipSuccess) r = hipEventSynchronize(e->ev1);
    float ms = 0.f;
    if (r == hipSuccess) r = hipEventElapsedTime(&ms, e->ev0, e->ev1);
    std::vector<uint32_t> hc(n);
    if (r == hipSuccess) r = hipMemcpy(hc.data(), counts, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipFree(specs);
    (void)hipFree(counts);
    if (r != hipSuccess) return MT_ERR_HIP;
    uint64_t tot = 0;
    for (uint32_t c : hc) tot += c;
    if (kernel_ms) *kernel_ms = ms;
    if (n_specs) *n_specs = tot;
    return MT_OK;
}

mt_status mt_get_text(mt_engine* e, uint32_t doc, char* buf, uint64_t cap, uint64_t* len) {
    if (!e || doc >= e->n_docs) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HostDoc h;
    mt_status st = read_doc(e, doc, h);
    if (st) return st;
    std::string t;  // UTF-16 code units, little endian
    for (int i = 0; i < h.sc.nseg; i++)
        if (!(h.flags[i] & (MT_SF_REMOVED | MT_SF_MARKER)))  // gatherText: text segments only
            for (uint32_t q = 0; q < h.len[i]; q++) {
                t += (char)(h.units(i)[q] & 0xFF);
                t += (char)(h.units(i)[q] >> 8);
            }
    return copy_out(t, buf, cap, len);
}

mt_status mt_get_length(mt_engine* e, uint32_t doc, uint32_t* len) {
    if (!e || doc >= e->n_docs || !len) return MT_ERR_ARG;
    HIP_OK(hipSetDevice(e->cfg.device));
    HostDoc h;
    mt_status st = read_doc(e, doc, h);
    if (st) return st;
    uint32_t n = 0;
    for (int i = 0; i < h.sc.nseg; i++)
        if (!(h.flags[i] & MT_SF_REMOVED)) n += h.len[i];
    *len = n;
    return MT_OK;
}

}  // extern "C"
