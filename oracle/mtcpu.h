/* mtcpu.h -- C ABI of the CPU oracle (oracle/mtcpu.cpp).  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the
 * product library. */
#ifndef MTCPU_H
#define MTCPU_H
#include <stdint.h>
#include "../include/mtgpu.h"
#include "../fluidframework_amd/csrc/mt_synth.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mto_engine mto_engine;

mto_engine* mto_create(uint32_t n_docs);
void mto_destroy(mto_engine* e);
int mto_apply(mto_engine* e, const mt_op_rec* ops, const uint8_t* payload, const uint32_t* row_ptr,
              uint32_t n_docs, int n_threads);
void mto_checksums(mto_engine* e, uint64_t* out, uint32_t n_docs);
/* Client.findTile of one document: the tile's local position or -1 (labels = property `key`,
 * value ids in the 256-bit vmask) */
int32_t mto_find_tile(mto_engine* e, uint32_t doc, int32_t pos, uint32_t key, const uint8_t* vmask, int preceding);
uint64_t mto_doc_regen_json(mto_engine* e, uint32_t doc, char* buf, uint64_t cap);
uint32_t mto_stack_context(mto_engine* e, uint32_t doc, int32_t pos, uint32_t key, const uint8_t* vmask, int32_t* out,
                           uint32_t cap);
/* delta / maintenance events (mt_event form, include/mtgpu.h) of every document from now on */
void mto_record_events(mto_engine* e, int on);
uint64_t mto_events(mto_engine* e, uint32_t doc, mt_event* out, uint64_t cap);
int mto_doc_error(mto_engine* e, uint32_t doc, int32_t* seq);
/* SnapshotLoader.loadHeader of one document (reloadFromSegments + the collab window) */
int mto_load(mto_engine* e, uint32_t doc, const mt_load_seg* segs, uint32_t n_segs, const uint8_t* text,
             int32_t min_seq, int32_t cur_seq);
uint64_t mto_doc_state(mto_engine* e, uint32_t doc, char* buf, uint64_t cap);
uint64_t mto_doc_text(mto_engine* e, uint32_t doc, char* buf, uint64_t cap);
uint32_t mto_doc_nsegs(mto_engine* e, uint32_t doc);
uint32_t mto_doc_heap(mto_engine* e, uint32_t doc);
int mto_generate(const mt_synth_cfg* cfg, uint32_t d0, uint32_t n_docs, mt_op_rec* ops, uint8_t* payload,
                 uint32_t* row_ptr, uint64_t* pay_ptr, int n_threads);
uint64_t mto_seg_hash(uint64_t idx, uint64_t text_hash, int32_t seq, int32_t client, int32_t rseq,
                      int32_t rclient, uint64_t overlap, uint64_t props_lo, uint32_t props_defined);

#ifdef __cplusplus
}
#endif
#endif
