/* mtgpu_napi.c -- Node N-API addon over the C-ABI of libmtgpu.so (include/mtgpu.h).
 * Plain C, N-API 8 (node 12+).  js/batchClient.js is the JavaScript surface above it. */
#include <node_api.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mtgpu.h"

#define NAPI_CALL(env, call)                                                   \
    do {                                                                       \
        if ((call) != napi_ok) {                                               \
            napi_throw_error((env), NULL, "N-API call failed: " #call);        \
            return NULL;                                                       \
        }                                                                      \
    } while (0)

static napi_value throw_status(napi_env env, const char* what, mt_status st) {
    char buf[160];
    static const char* names[] = {"ok", "bad argument", "HIP error", "out of device memory", "bad state",
                                  "document error"};
    snprintf(buf, sizeof buf, "%s: %s", what, (unsigned)st < 6 ? names[st] : "unknown");
    napi_throw_error(env, NULL, buf);
    return NULL;
}

/* One engine + a FIFO turnstile.  libmtgpu's engine is not thread-safe (mtgpu.h), and
 * submitAsync runs mt_submit on a libuv pool thread while the JS thread stays free: every entry
 * point takes a ticket in call order on the JS thread and runs only when every earlier ticket
 * has finished, so batches apply in the order they were flushed and a readout sees every batch
 * flushed before it (a sync call blocks the JS thread until the async work ahead of it is done). */
typedef struct {
    mt_engine* e;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    uint64_t next, serving;
} engine_box;

static uint64_t take_ticket(engine_box* b) {
    pthread_mutex_lock(&b->mu);
    const uint64_t t = b->next++;
    pthread_mutex_unlock(&b->mu);
    return t;
}
static void wait_turn(engine_box* b, uint64_t t) {
    pthread_mutex_lock(&b->mu);
    while (b->serving != t) pthread_cond_wait(&b->cv, &b->mu);
    pthread_mutex_unlock(&b->mu);
}
static void end_turn(engine_box* b) {
    pthread_mutex_lock(&b->mu);
    b->serving++;
    pthread_cond_broadcast(&b->cv);
    pthread_mutex_unlock(&b->mu);
}
/* a synchronous entry point: its turn comes after every ticket handed out before it */
static engine_box* enter(engine_box* b) {
    if (b) wait_turn(b, take_ticket(b));
    return b;
}
static void leave(engine_box* b) {
    if (b) end_turn(b);
}

static engine_box* get_box(napi_env env, napi_value v) {
    void* p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok) return NULL;
    return (engine_box*)p;
}

static void finalize_engine(napi_env env, void* data, void* hint) {
    (void)env;
    (void)hint;
    engine_box* b = (engine_box*)data;
    if (!b) return;
    /* an external is finalized only when unreachable, i.e. after every pending job released it */
    enter(b);
    mt_engine_destroy(b->e);
    leave(b);
    pthread_cond_destroy(&b->cv);
    pthread_mutex_destroy(&b->mu);
    free(b);
}

static uint32_t get_u32(napi_env env, napi_value obj, const char* key, uint32_t dflt) {
    napi_value v;
    bool has = false;
    uint32_t out = dflt;
    if (napi_has_named_property(env, obj, key, &has) == napi_ok && has &&
        napi_get_named_property(env, obj, key, &v) == napi_ok) {
        napi_valuetype t;
        napi_typeof(env, v, &t);
        if (t == napi_number) napi_get_value_uint32(env, v, &out);
    }
    return out;
}

/* createEngine({device, maxDocs, segCapacity, textCapacity, heapCapacity, opsPerLaunch}) */
static napi_value create_engine(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    mt_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.device = (int32_t)get_u32(env, argv[0], "device", 0);
    cfg.max_docs = get_u32(env, argv[0], "maxDocs", 1);
    cfg.seg_capacity = get_u32(env, argv[0], "segCapacity", 0);
    cfg.text_capacity = get_u32(env, argv[0], "textCapacity", 0);
    cfg.heap_capacity = get_u32(env, argv[0], "heapCapacity", 0);
    cfg.ops_per_launch = get_u32(env, argv[0], "opsPerLaunch", 0);
    mt_engine* e = NULL;
    mt_status st = mt_engine_create(&cfg, &e);
    if (st) return throw_status(env, "mt_engine_create", st);
    st = mt_docs_init(e, cfg.max_docs);
    if (st) {
        mt_engine_destroy(e);
        return throw_status(env, "mt_docs_init", st);
    }
    engine_box* b = (engine_box*)calloc(1, sizeof *b);
    b->e = e;
    pthread_mutex_init(&b->mu, NULL);
    pthread_cond_init(&b->cv, NULL);
    NAPI_CALL(env, napi_create_external(env, b, finalize_engine, NULL, &out));
    return out;
}

/* rows of a CSR batch the engine will read: rowPtr must cover n_docs + 1 entries and ops whole
 * 32-byte records (mtgpu.h mt_batch_upload) */
static int batch_shape_ok(mt_engine* e, size_t nops, size_t nrow) {
    uint32_t n_docs = 0;
    if (mt_engine_info(e, &n_docs, NULL) != MT_OK) return 0;
    return nops % sizeof(mt_op_rec) == 0 && nrow >= 4 * ((size_t)n_docs + 1);
}

static void* buffer_data(napi_env env, napi_value v, size_t* len) {
    void* data = NULL;
    bool is_buf = false, is_ta = false;
    *len = 0;
    if (napi_is_buffer(env, v, &is_buf) == napi_ok && is_buf) {
        napi_get_buffer_info(env, v, &data, len);
        return data;
    }
    if (napi_is_typedarray(env, v, &is_ta) == napi_ok && is_ta) {
        napi_typedarray_type t;
        size_t n, off;
        napi_value ab;
        napi_get_typedarray_info(env, v, &t, &n, &data, &ab, &off);
        size_t el = (t == napi_uint32_array || t == napi_int32_array || t == napi_float32_array) ? 4
                    : (t == napi_uint16_array || t == napi_int16_array) ? 2
                    : (t == napi_float64_array || t == napi_bigint64_array || t == napi_biguint64_array) ? 8 : 1;
        *len = n * el;
        return data;
    }
    return NULL;
}

/* submit(engine, opsU8 (32-byte mt_op_rec rows), payloadU8, rowPtrU32): the batched applyMsg */
static napi_value submit(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = get_box(env, argv[0]);
    size_t nops, npay, nrow;
    const void* ops = buffer_data(env, argv[1], &nops);
    const void* pay = buffer_data(env, argv[2], &npay);
    const void* row = buffer_data(env, argv[3], &nrow);
    if (!b || (!ops && nops) || !row) {
        napi_throw_type_error(env, NULL, "submit(engine, ops, payload, rowPtr)");
        return NULL;
    }
    enter(b);
    mt_status st = batch_shape_ok(b->e, nops, nrow)
                       ? mt_submit(b->e, (const mt_op_rec*)ops, nops / sizeof(mt_op_rec), (const uint8_t*)pay, npay,
                                   (const uint32_t*)row)
                       : MT_ERR_ARG;
    leave(b);
    if (st) return throw_status(env, "mt_submit", st);
    return NULL;
}

/* submitAsync: the same on a libuv worker thread (napi_async_work); returns a Promise.  The
 * caller keeps the buffers alive until it settles. */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref refs[4];
    engine_box* b;
    uint64_t ticket;
    const void* ops;
    const void* pay;
    const void* row;
    size_t nops, npay;
    mt_status st;
} submit_job;

static void submit_execute(napi_env env, void* data) {
    (void)env;
    submit_job* j = (submit_job*)data;
    wait_turn(j->b, j->ticket);
    j->st = mt_submit(j->b->e, (const mt_op_rec*)j->ops, j->nops / sizeof(mt_op_rec), (const uint8_t*)j->pay, j->npay,
                      (const uint32_t*)j->row);
    end_turn(j->b);
}

static void submit_complete(napi_env env, napi_status status, void* data) {
    submit_job* j = (submit_job*)data;
    napi_value v;
    if (status == napi_ok && j->st == MT_OK) {
        napi_get_undefined(env, &v);
        napi_resolve_deferred(env, j->deferred, v);
    } else {
        napi_value msg;
        char buf[64];
        snprintf(buf, sizeof buf, "mt_submit failed (status %d)", (int)j->st);
        napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &v);
        napi_reject_deferred(env, j->deferred, v);
    }
    for (int i = 0; i < 4; i++) napi_delete_reference(env, j->refs[i]);
    napi_delete_async_work(env, j->work);
    free(j);
}

static napi_value submit_async(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4], promise, name;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    submit_job* j = (submit_job*)calloc(1, sizeof *j);
    j->b = get_box(env, argv[0]);
    j->ops = buffer_data(env, argv[1], &j->nops);
    j->pay = buffer_data(env, argv[2], &j->npay);
    size_t nrow;
    j->row = buffer_data(env, argv[3], &nrow);
    if (!j->b || !j->row || (!j->ops && j->nops)) {
        free(j);
        napi_throw_type_error(env, NULL, "submitAsync(engine, ops, payload, rowPtr)");
        return NULL;
    }
    /* the shape check reads only engine constants (n_docs), safe outside the turnstile */
    if (!batch_shape_ok(j->b->e, j->nops, nrow)) {
        free(j);
        return throw_status(env, "submitAsync", MT_ERR_ARG);
    }
    /* the engine external is referenced too: it cannot be finalized while the job is pending */
    for (int i = 0; i < 4; i++) napi_create_reference(env, argv[i], 1, &j->refs[i]);
    j->ticket = take_ticket(j->b);  /* call order = apply order */
    NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
    NAPI_CALL(env, napi_create_string_utf8(env, "mtgpu.submit", NAPI_AUTO_LENGTH, &name));
    NAPI_CALL(env, napi_create_async_work(env, NULL, name, submit_execute, submit_complete, j, &j->work));
    NAPI_CALL(env, napi_queue_async_work(env, j->work));
    return promise;
}

typedef mt_status (*string_fn)(mt_engine*, uint32_t, char*, uint64_t, uint64_t*);

static napi_value get_string(napi_env env, napi_callback_info info, string_fn fn, const char* what) {
    size_t argc = 2;
    napi_value argv[2], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = get_box(env, argv[0]);
    uint32_t doc = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    if (!b) return throw_status(env, what, MT_ERR_ARG);
    uint64_t n = 0;
    char* buf = NULL;
    enter(b);
    mt_status st = fn(b->e, doc, NULL, 0, &n);
    if (!st) {
        buf = (char*)malloc(n + 1);
        st = fn(b->e, doc, buf, n + 1, &n);
    }
    leave(b);
    if (st) {
        free(buf);
        return throw_status(env, what, st);
    }
    /* mt_get_text: UTF-16 code units (little endian, as x86 and gfx950 are); the state JSON: ASCII */
    napi_status ns = fn == mt_get_text ? napi_create_string_utf16(env, (const char16_t*)buf, n / 2, &out)
                                       : napi_create_string_latin1(env, buf, n, &out);
    free(buf);
    NAPI_CALL(env, ns);
    return out;
}

static napi_value get_text(napi_env env, napi_callback_info info) {
    return get_string(env, info, mt_get_text, "mt_get_text");
}
static napi_value get_state(napi_env env, napi_callback_info info) {
    return get_string(env, info, mt_get_state, "mt_get_state");
}

static napi_value get_length(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t doc = 0, len = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    engine_box* b = get_box(env, argv[0]);
    if (!b) return throw_status(env, "mt_get_length", MT_ERR_ARG);
    enter(b);
    mt_status st = mt_get_length(b->e, doc, &len);
    leave(b);
    if (st) return throw_status(env, "mt_get_length", st);
    NAPI_CALL(env, napi_create_uint32(env, len, &out));
    return out;
}

static napi_value doc_error(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out, a, bv;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t doc = 0;
    int32_t code = 0, seq = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    engine_box* b = get_box(env, argv[0]);
    if (!b) return throw_status(env, "mt_doc_error", MT_ERR_ARG);
    enter(b);
    mt_status st = mt_doc_error(b->e, doc, &code, &seq);
    leave(b);
    if (st) return throw_status(env, "mt_doc_error", st);
    NAPI_CALL(env, napi_create_array_with_length(env, 2, &out));
    NAPI_CALL(env, napi_create_int32(env, code, &a));
    NAPI_CALL(env, napi_create_int32(env, seq, &bv));
    NAPI_CALL(env, napi_set_element(env, out, 0, a));
    NAPI_CALL(env, napi_set_element(env, out, 1, bv));
    return out;
}

/* checksums(engine, nDocs) -> Buffer of nDocs little-endian u64 */
static napi_value checksums(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t n = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &n));
    void* data = NULL;
    NAPI_CALL(env, napi_create_buffer(env, (size_t)n * 8, &data, &out));
    engine_box* b = get_box(env, argv[0]);
    if (!b) return throw_status(env, "mt_checksums", MT_ERR_ARG);
    enter(b);
    mt_status st = mt_checksums(b->e, (uint64_t*)data, n);
    leave(b);
    if (st) return throw_status(env, "mt_checksums", st);
    return out;
}

/* findTiles(engine, queries (48-byte mt_tile_query rows)) -> Buffer of 8-byte mt_tile_result rows */
static napi_value find_tiles(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 2 ? get_box(env, argv[0]) : NULL;
    size_t nq = 0;
    const void* q = b ? buffer_data(env, argv[1], &nq) : NULL;
    if (!b || nq % sizeof(mt_tile_query)) {
        napi_throw_type_error(env, NULL, "findTiles(engine, queries)");
        return NULL;
    }
    const uint32_t n = (uint32_t)(nq / sizeof(mt_tile_query));
    void* data = NULL;
    NAPI_CALL(env, napi_create_buffer(env, n ? n * sizeof(mt_tile_result) : 1, &data, &out));
    enter(b);
    mt_status st = mt_find_tiles(b->e, (const mt_tile_query*)q, n, (mt_tile_result*)data);
    leave(b);
    if (st) return throw_status(env, "mt_find_tiles", st);
    return out;
}

/* resolvePositions(engine, queries (16-byte mt_pos_query rows)) -> Buffer of 16-byte mt_pos_result rows */
static napi_value resolve_positions(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 2 ? get_box(env, argv[0]) : NULL;
    size_t nq = 0;
    const void* q = b ? buffer_data(env, argv[1], &nq) : NULL;
    if (!b || nq % sizeof(mt_pos_query)) {
        napi_throw_type_error(env, NULL, "resolvePositions(engine, queries)");
        return NULL;
    }
    const uint32_t n = (uint32_t)(nq / sizeof(mt_pos_query));
    void* data = NULL;
    NAPI_CALL(env, napi_create_buffer(env, n ? n * sizeof(mt_pos_result) : 1, &data, &out));
    enter(b);
    mt_status st = mt_resolve_positions(b->e, (const mt_pos_query*)q, n, (mt_pos_result*)data);
    leave(b);
    if (st) return throw_status(env, "mt_resolve_positions", st);
    return out;
}

/* segmentInfos(engine, docs (uint32 rows), ordinals (int32 rows)) -> Buffer of 104-byte mt_seg_info rows */
static napi_value segment_infos(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 3 ? get_box(env, argv[0]) : NULL;
    size_t nd = 0, no = 0;
    const void* docs = b ? buffer_data(env, argv[1], &nd) : NULL;
    const void* ords = b ? buffer_data(env, argv[2], &no) : NULL;
    if (!b || nd % 4 || nd != no) {
        napi_throw_type_error(env, NULL, "segmentInfos(engine, docs, ordinals)");
        return NULL;
    }
    const uint32_t n = (uint32_t)(nd / 4);
    void* data = NULL;
    NAPI_CALL(env, napi_create_buffer(env, n ? n * sizeof(mt_seg_info) : 1, &data, &out));
    enter(b);
    mt_status st = mt_segment_infos(b->e, (const uint32_t*)docs, (const int32_t*)ords, n, (mt_seg_info*)data);
    leave(b);
    if (st) return throw_status(env, "mt_segment_infos", st);
    return out;
}

/* segmentText(engine, doc, toff, len) -> string of `len` UTF-16 code units */
static napi_value segment_text(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 4 ? get_box(env, argv[0]) : NULL;
    uint32_t doc = 0, toff = 0, len = 0;
    if (!b || napi_get_value_uint32(env, argv[1], &doc) != napi_ok || napi_get_value_uint32(env, argv[2], &toff) != napi_ok ||
        napi_get_value_uint32(env, argv[3], &len) != napi_ok) {
        napi_throw_type_error(env, NULL, "segmentText(engine, doc, toff, len)");
        return NULL;
    }
    uint16_t* u = (uint16_t*)malloc((len ? len : 1) * sizeof(uint16_t));
    if (!u) return throw_status(env, "segmentText", MT_ERR_NOMEM);
    enter(b);
    mt_status st = mt_segment_text(b->e, doc, toff, len, u);
    leave(b);
    if (st) {
        free(u);
        return throw_status(env, "mt_segment_text", st);
    }
    const napi_status ns = napi_create_string_utf16(env, (const char16_t*)u, len, &out);
    free(u);
    if (ns != napi_ok) return throw_status(env, "segmentText", MT_ERR_NOMEM);
    return out;
}

/* rangeStacks(engine, queries (48-byte mt_tile_query rows), cap) -> [Buffer of n*cap 12-byte mt_stack_item
 * rows, Buffer of n uint32 depth words (MT_STACK_TOUCHED | depth)] */
static napi_value range_stacks(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], out, ib, db;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 3 ? get_box(env, argv[0]) : NULL;
    size_t nq = 0;
    const void* q = b ? buffer_data(env, argv[1], &nq) : NULL;
    uint32_t cap = 0;
    if (!b || nq % sizeof(mt_tile_query) || napi_get_value_uint32(env, argv[2], &cap) != napi_ok) {
        napi_throw_type_error(env, NULL, "rangeStacks(engine, queries, cap)");
        return NULL;
    }
    const uint32_t n = (uint32_t)(nq / sizeof(mt_tile_query));
    void *items = NULL, *depth = NULL;
    const size_t ni = (size_t)n * cap;
    NAPI_CALL(env, napi_create_buffer(env, ni != 0 ? ni * sizeof(mt_stack_item) : 1, &items, &ib));
    NAPI_CALL(env, napi_create_buffer(env, n ? n * sizeof(uint32_t) : 1, &depth, &db));
    enter(b);
    mt_status st = mt_range_stacks(b->e, (const mt_tile_query*)q, n, cap, (mt_stack_item*)items, (uint32_t*)depth);
    leave(b);
    if (st) return throw_status(env, "mt_range_stacks", st);
    NAPI_CALL(env, napi_create_array_with_length(env, 2, &out));
    NAPI_CALL(env, napi_set_element(env, out, 0, ib));
    NAPI_CALL(env, napi_set_element(env, out, 1, db));
    return out;
}

/* regenDrain(engine, doc) -> [Buffer of 32-byte mt_op_rec rows, Buffer of their payload] (mt_regen_drain) */
static napi_value regen_drain(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out, rb, pb;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 2 ? get_box(env, argv[0]) : NULL;
    uint32_t doc = 0;
    if (!b || napi_get_value_uint32(env, argv[1], &doc) != napi_ok) {
        napi_throw_type_error(env, NULL, "regenDrain(engine, doc)");
        return NULL;
    }
    uint32_t n = 0, pn = 0;
    enter(b);
    mt_status st = mt_regen_drain(b->e, doc, NULL, 0, NULL, 0, &n, &pn);
    void *recs = NULL, *pay = NULL;
    if (!st && napi_create_buffer(env, n ? n * sizeof(mt_op_rec) : 1, &recs, &rb) == napi_ok &&
        napi_create_buffer(env, pn ? pn : 1, &pay, &pb) == napi_ok)
        st = mt_regen_drain(b->e, doc, (mt_op_rec*)recs, n, (uint8_t*)pay, pn, &n, &pn);
    leave(b);
    if (st) return throw_status(env, "mt_regen_drain", st);
    NAPI_CALL(env, napi_create_array_with_length(env, 2, &out));
    NAPI_CALL(env, napi_set_element(env, out, 0, rb));
    NAPI_CALL(env, napi_set_element(env, out, 1, pb));
    return out;
}

/* docsLoad(engine, docIdsU32, segRowPtrU32, segs (64-byte mt_load_seg rows), text, minSeqI32, curSeqI32):
 * SnapshotLoader.loadHeader for a batch of documents (mt_docs_load) */
static napi_value docs_load(napi_env env, napi_callback_info info) {
    size_t argc = 7;
    napi_value argv[7];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 7 ? get_box(env, argv[0]) : NULL;
    size_t nid = 0, nrow = 0, nseg = 0, ntext = 0, nmin = 0, ncur = 0;
    const void* ids = b ? buffer_data(env, argv[1], &nid) : NULL;
    const void* row = b ? buffer_data(env, argv[2], &nrow) : NULL;
    const void* segs = b ? buffer_data(env, argv[3], &nseg) : NULL;
    const void* text = b ? buffer_data(env, argv[4], &ntext) : NULL;
    const void* mn = b ? buffer_data(env, argv[5], &nmin) : NULL;
    const void* cs = b ? buffer_data(env, argv[6], &ncur) : NULL;
    const size_t n = nid / 4;
    if (!b || nid % 4 || nrow != 4 * (n + 1) || nmin != 4 * n || ncur != 4 * n || nseg % sizeof(mt_load_seg) ||
        (n && ((const uint32_t*)row)[n] - ((const uint32_t*)row)[0] != nseg / sizeof(mt_load_seg))) {
        napi_throw_type_error(env, NULL, "docsLoad(engine, docIds, segRowPtr, segs, text, minSeq, curSeq)");
        return NULL;
    }
    enter(b);
    mt_status st = mt_docs_load(b->e, (uint32_t)n, (const uint32_t*)ids, (const uint32_t*)row,
                                (const mt_load_seg*)segs, (const uint8_t*)text, ntext, (const int32_t*)mn,
                                (const int32_t*)cs);
    leave(b);
    if (st) return throw_status(env, "mt_docs_load", st);
    return NULL;
}

/* eventsEnable(engine, perDoc): record delta / maintenance callbacks (mt_events_enable) */
static napi_value events_enable(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t per = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &per));
    engine_box* b = get_box(env, argv[0]);
    if (!b) return throw_status(env, "mt_events_enable", MT_ERR_ARG);
    enter(b);
    mt_status st = mt_events_enable(b->e, per);
    leave(b);
    if (st) return throw_status(env, "mt_events_enable", st);
    return NULL;
}

/* eventsDrain(engine, nDocs) -> [Buffer of 64-byte mt_event rows, Buffer of nDocs+1 u32 row pointers] */
static napi_value events_drain(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out, rows, rp;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t n = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &n));
    engine_box* b = get_box(env, argv[0]);
    if (!b) return throw_status(env, "mt_events_drain", MT_ERR_ARG);
    uint32_t nd = 0;
    void* rpd = NULL;
    void* data = NULL;
    uint64_t total = 0;
    enter(b);
    mt_status st = mt_engine_info(b->e, &nd, NULL);
    if (!st && nd != n) st = MT_ERR_ARG;
    if (st) {
        leave(b);
        return throw_status(env, "mt_events_drain", st);
    }
    if (napi_create_buffer(env, (size_t)(n + 1) * 4, &rpd, &rp) != napi_ok) {
        leave(b);
        return NULL;
    }
    st = mt_events_drain(b->e, NULL, 0, (uint32_t*)rpd, &total);
    if (!st && napi_create_buffer(env, total ? total * sizeof(mt_event) : 1, &data, &rows) != napi_ok) {
        leave(b);
        return NULL;
    }
    if (!st && total) st = mt_events_drain(b->e, (mt_event*)data, total, (uint32_t*)rpd, &total);
    else if (!st) st = mt_events_drain(b->e, (mt_event*)data, 0, (uint32_t*)rpd, &total);
    leave(b);
    if (st) return throw_status(env, "mt_events_drain", st);
    NAPI_CALL(env, napi_create_array_with_length(env, 2, &out));
    NAPI_CALL(env, napi_set_element(env, out, 0, rows));
    NAPI_CALL(env, napi_set_element(env, out, 1, rp));
    return out;
}

static napi_value version(napi_env env, napi_callback_info info) {
    (void)info;
    napi_value out;
    NAPI_CALL(env, napi_create_string_utf8(env, mt_version(), NAPI_AUTO_LENGTH, &out));
    return out;
}

/* ---- deli (include/mtgpu.h "deli" section) ---------------------------------------------- */
static void finalize_deli(napi_env env, void* data, void* hint) {
    (void)env;
    (void)hint;
    if (data) mt_deli_destroy((mt_deli*)data);
}
static mt_deli* get_deli(napi_env env, napi_value v) {
    void* p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok) return NULL;
    return (mt_deli*)p;
}

/* createDeli({device, maxDocs}): new DeliLambda state for maxDocs documents (lambda.ts:112-171) */
static napi_value create_deli(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    mt_deli* dl = NULL;
    mt_status st = mt_deli_create((int32_t)get_u32(env, argv[0], "device", 0), get_u32(env, argv[0], "maxDocs", 1), &dl);
    if (st) return throw_status(env, "mt_deli_create", st);
    NAPI_CALL(env, napi_create_external(env, dl, finalize_deli, NULL, &out));
    return out;
}

/* deliTicket(deli, msgsU8 (16-byte mt_raw_msg rows), rowPtrU32) -> Buffer of 16-byte mt_ticket
 * rows: DeliLambda.ticket over every raw message of every document (lambda.ts:255-544) */
static napi_value deli_ticket(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3], out;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    mt_deli* dl = get_deli(env, argv[0]);
    size_t nmsg, nrow;
    const void* msgs = buffer_data(env, argv[1], &nmsg);
    const void* row = buffer_data(env, argv[2], &nrow);
    if (!dl || (!msgs && nmsg) || !row || nrow < 4 || nmsg % sizeof(mt_raw_msg) != 0 || nrow % 4 != 0) {
        napi_throw_type_error(env, NULL, "deliTicket(deli, msgs, rowPtr)");
        return NULL;
    }
    const uint64_t n = nmsg / sizeof(mt_raw_msg);
    void* data = NULL;
    NAPI_CALL(env, napi_create_buffer(env, n ? n * sizeof(mt_ticket) : 1, &data, &out));
    mt_status st = mt_deli_ticket(dl, (const mt_raw_msg*)msgs, n, (const uint32_t*)row,
                                  (uint32_t)(nrow / 4 - 1), (mt_ticket*)data);
    if (st) return throw_status(env, "mt_deli_ticket", st);
    return out;
}

/* deliError(deli, doc) -> [mt_deli_err, message index] */
static napi_value deli_error(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2], out, a, b;
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    uint32_t doc = 0;
    int32_t err = 0, idx = 0;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    mt_status st = mt_deli_doc_error(get_deli(env, argv[0]), doc, &err, &idx);
    if (st) return throw_status(env, "mt_deli_doc_error", st);
    NAPI_CALL(env, napi_create_array_with_length(env, 2, &out));
    NAPI_CALL(env, napi_create_int32(env, err, &a));
    NAPI_CALL(env, napi_create_int32(env, idx, &b));
    NAPI_CALL(env, napi_set_element(env, out, 0, a));
    NAPI_CALL(env, napi_set_element(env, out, 1, b));
    return out;
}

/* setLabelKeys(engine, doc, tileKey, rangeKey): mt_set_label_keys (-1: a key left as it is) */
static napi_value set_label_keys(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    engine_box* b = argc == 4 ? get_box(env, argv[0]) : NULL;
    if (!b) {
        napi_throw_type_error(env, NULL, "setLabelKeys(engine, doc, tileKey, rangeKey)");
        return NULL;
    }
    uint32_t doc = 0;
    int32_t tk = -1, rk = -1;
    NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
    NAPI_CALL(env, napi_get_value_int32(env, argv[2], &tk));
    NAPI_CALL(env, napi_get_value_int32(env, argv[3], &rk));
    mt_status st = mt_set_label_keys(b->e, doc, tk, rk);
    if (st) return throw_status(env, "mt_set_label_keys", st);
    return NULL;
}

static napi_value init(napi_env env, napi_value exports) {
    napi_property_descriptor d[] = {
        {"createEngine", NULL, create_engine, NULL, NULL, NULL, napi_default, NULL},
        {"submit", NULL, submit, NULL, NULL, NULL, napi_default, NULL},
        {"submitAsync", NULL, submit_async, NULL, NULL, NULL, napi_default, NULL},
        {"getText", NULL, get_text, NULL, NULL, NULL, napi_default, NULL},
        {"getState", NULL, get_state, NULL, NULL, NULL, napi_default, NULL},
        {"getLength", NULL, get_length, NULL, NULL, NULL, napi_default, NULL},
        {"docError", NULL, doc_error, NULL, NULL, NULL, napi_default, NULL},
        {"checksums", NULL, checksums, NULL, NULL, NULL, napi_default, NULL},
        {"version", NULL, version, NULL, NULL, NULL, napi_default, NULL},
        {"eventsEnable", NULL, events_enable, NULL, NULL, NULL, napi_default, NULL},
        {"docsLoad", NULL, docs_load, NULL, NULL, NULL, napi_default, NULL},
        {"findTiles", NULL, find_tiles, NULL, NULL, NULL, napi_default, NULL},
        {"setLabelKeys", NULL, set_label_keys, NULL, NULL, NULL, napi_default, NULL},
        {"rangeStacks", NULL, range_stacks, NULL, NULL, NULL, napi_default, NULL},
        {"resolvePositions", NULL, resolve_positions, NULL, NULL, NULL, napi_default, NULL},
        {"segmentInfos", NULL, segment_infos, NULL, NULL, NULL, napi_default, NULL},
        {"segmentText", NULL, segment_text, NULL, NULL, NULL, napi_default, NULL},
        {"regenDrain", NULL, regen_drain, NULL, NULL, NULL, napi_default, NULL},
        {"eventsDrain", NULL, events_drain, NULL, NULL, NULL, napi_default, NULL},
        {"createDeli", NULL, create_deli, NULL, NULL, NULL, napi_default, NULL},
        {"deliTicket", NULL, deli_ticket, NULL, NULL, NULL, napi_default, NULL},
        {"deliError", NULL, deli_error, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
