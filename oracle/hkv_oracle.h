/*
 * hkv_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline).
 *
 * A plain-C restatement of the HermesKV KVS batch path of A-Kokolis/Hermes:
 *   src/hermes/hermesKV.c:905-996  hermes_batch_ops_to_KVS  (3-pass lookup + exec)
 *   src/hermes/hermesKV.c:81-703   per-op exec functions (read/write/rmw/inv/ack/val/...)
 *   src/hermes/spacetime.c:17-68   init + populate
 *   src/mica-herd/mica.c:17-165    MICA index/log init, insert, key generation
 *   src/mica-herd/city.c:276-400   CityHash128 (CityMurmur path for short strings)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code, and only as the checker / the timed CPU baseline. The product path
 * (hermes_amd/, libhermeskv.so) never links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - CityHash128 is pinned against the reference's own city.c, compiled from
 *     /root/reference by oracle/Makefile into oracle/_ref/ (tests/golden/cityhash_ref.json).
 *   - The batch semantics are pinned against the known-answer outputs of the
 *     reference's hermes_batch_ops_to_KVS recorded in SURVEY.md section 4
 *     (tests/golden/known_answers.json). The reference batch path itself needs
 *     ibverbs/memcached headers that this image lacks, so it is unbuildable here.
 *
 * Byte layouts are the reference's (gcc, x86-64, little endian):
 *   op/inv (spacetime_op_t, spacetime.h:170-185): key 0-7, opcode 8, state|sender 9,
 *       val_len 10, ts.cid 11, ts.version 12-15, RMW_flag bit0 of 16, value 18..
 *   ack/val (spacetime_op_meta_t, spacetime.h:151-166): the first 16 bytes of the above.
 *   log entry (mica_op, mica.h:55-60): key 0-15 (key hash .first, .second), opcode 16,
 *       val_len 17, object meta 18-32, value 33..
 *   object meta (spacetime_object_meta, spacetime.h:138-148) at entry+18:
 *       state 0, ack_bv 1, RMW_flag bit0|last_writer_id bits1-7 2, op_buffer_index 3,
 *       lock 4, ts.cid 5, ts.version 6-9, llw.cid 10, llw.version 11-14.
 *   index bucket (mica_bkt, mica.h:62-70): 8 x u64 slots: in_use bit0, tag bits1-23,
 *       offset bits 24-63.
 */
#ifndef HKV_ORACLE_H
#define HKV_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hko_config {
    uint32_t big_objects;       /* USE_BIG_OBJECTS (hrd.h:36) */
    uint32_t extra_cache_lines; /* EXTRA_CACHE_LINES (hrd.h:37), used only when big_objects */
    uint32_t rmw_enabled;       /* ENABLE_RMWs (config.h:37) */
    uint32_t machine_id;        /* global machine_id (hrd.h:87) */
    uint64_t num_bkts;          /* SPACETIME_NUM_BKTS (spacetime.h:22), power of two */
    uint64_t log_cap;           /* SPACETIME_LOG_CAP (spacetime.h:23), power of two */
    uint32_t skew_flags;        /* bit 0: ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS (config.h:79),
                                   bit 1: ENABLE_WRITE_COALESCE_TO_THE_SAME_KEY_IN_SAME_NODE (config.h:80) */
    uint32_t pad;
} hko_config;

typedef struct hko_kvs hko_kvs;

/* derived sizes */
uint32_t hko_kvs_value_size(const hko_config *c); /* KVS_VALUE_SIZE (hrd.h:47) */
uint32_t hko_st_value_size(const hko_config *c);  /* ST_VALUE_SIZE  (spacetime.h:29) */
uint32_t hko_entry_size(const hko_config *c);     /* sizeof(struct mica_op) */
uint32_t hko_op_size(const hko_config *c);        /* sizeof(spacetime_op_t) */

/* CityHash128 of a short string (len < 128 handled; the path only uses len 4) */
void hko_cityhash128(const void *s, size_t len, uint64_t *first, uint64_t *second);
/* mica_gen_keys: .second of CityHash128(&i, 4) for i in [0, n) */
void hko_gen_keys(uint64_t *out_second, int64_t n);

hko_kvs *hko_create(const hko_config *c);                 /* mica_init */
void hko_destroy(hko_kvs *kv);
void hko_populate(hko_kvs *kv, int64_t n, int val_len);   /* spacetime_populate_fixed_len */
void hko_set_machine_id(hko_kvs *kv, uint32_t machine_id);

/* hermes_batch_ops_to_KVS; membership is the 8-byte spacetime_group_membership by value */
void hko_batch(hko_kvs *kv, int type, uint8_t *op_array, int op_num, uint16_t sizeof_op_elem,
               const uint8_t membership[8], int *node_suspected, uint8_t *read_write_ops);

/* B batches of the same type applied one after another (concatenation order).
 * Batch b owns elems [b*stride, b*stride + counts[b]) of op_array and the rw buffer
 * read_write_ops + b*rw_stride_bytes. node_suspected may be NULL or have B entries. */
void hko_batch_multi(hko_kvs *kv, int type, uint8_t *op_array, int n_batches, int stride,
                     const int32_t *counts, uint16_t sizeof_op_elem, const uint8_t membership[8],
                     int32_t *node_suspected, uint8_t *read_write_ops, int64_t rw_stride_bytes);

/* raw views for parity dumps */
uint8_t *hko_index(hko_kvs *kv);
uint8_t *hko_log(hko_kvs *kv);
uint64_t hko_log_head(hko_kvs *kv);
int64_t hko_num_index_evictions(hko_kvs *kv);

/* find a key's log entry (NULL on miss) -- the same lookup the batch path does */
uint8_t *hko_lookup(hko_kvs *kv, uint64_t key);

#ifdef __cplusplus
}
#endif
#endif
