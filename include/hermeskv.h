/*
 * hermeskv.h -- C ABI of libhermeskv.so, the MI355X-native HermesKV data path.
 *
 * Drop-in boundary: the three entry points the reference's worker links
 * against, with the reference's exact signatures and argument meaning:
 *
 *   hermes_batch_ops_to_KVS   replaces include/hermes/spacetime.h:228-230 (hermesKV.c:905-996)
 *   spacetime_init            replaces include/hermes/spacetime.h:211     (spacetime.c:25-30)
 *   spacetime_populate_fixed_len replaces include/hermes/spacetime.h:212  (spacetime.c:32-68)
 *
 * The MICA-herd index and log (mica.h:62-91) live in HBM; op arrays are caller-owned host
 * memory, mutated in place exactly as the reference mutates them. Errors the reference turns
 * into asserts make these three calls print a message and abort (fail loudly); the hkv_* calls
 * return a negative code instead and leave a message in hkv_last_error().
 *
 * The hkv_* extensions are the device-resident fast path: tables created explicitly,
 * op arrays already in HBM, many batches (one per virtual worker) concatenated into one
 * launch, asynchronous on a caller-supplied HIP stream. Their results are defined as the
 * reference applied to the batches one after another (concatenation order).
 *
 * Plain pointers and sizes only; no HIP or torch types appear in any signature
 * (streams are passed as void* and interpreted as hipStream_t; NULL is the HIP null stream).
 */
#ifndef HERMESKV_H
#define HERMESKV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HKV_ABI_VERSION 8

/* ------------------------------------------------------------------ reference types
 * Declared here only when the reference's own spacetime.h has not been included; the
 * layouts are the reference's (gcc, x86-64): see hermes_amd/layout.py for every offset. */
#ifndef HERMES_SPACETIME_H
enum hermes_batch_type_t {               /* spacetime.h:219-226 */
    local_ops,
    local_ops_after_membership_change,
    invs,
    acks,
    vals
};
typedef struct { uint8_t bit_array[1]; } bit_vector_t;               /* bit_vector.h:40-44 */
typedef struct { uint8_t lock; uint32_t version; } __attribute__((packed)) seqlock_t;
typedef struct {                          /* spacetime.h:188-195, 8 bytes, passed by value */
    volatile uint8_t num_of_alive_remotes;
    volatile bit_vector_t g_membership;
    volatile bit_vector_t w_ack_init;
    seqlock_t lock;
} spacetime_group_membership;
typedef struct hkv_spacetime_op spacetime_op_t; /* 56-byte spacetime_op_t, used by pointer */
struct spacetime_kv;                            /* opaque; only its address is passed */
#endif

/* ------------------------------------------------------------------ reference entry points */

/* spacetime.h:228-230. op_array holds op_num elements of sizeof_op_elem bytes (56 for local
 * ops and INVs, 16 for ACKs/VALs, 56 for ACKs in an RMW build). read_write_ops is the
 * caller's local-op buffer (hkv_config.rw_len elements), written by ACK completions.
 * node_suspected is written by INV batches that carry ST_OP_MEMBERSHIP_CHANGE. thread_id is
 * accepted for signature compatibility (the reference uses it for debug prints only). */
#ifndef HKV_IMPLEMENTATION
void hermes_batch_ops_to_KVS(enum hermes_batch_type_t type, uint8_t *op_array, int op_num,
                             uint16_t sizeof_op_elem, spacetime_group_membership curr_membership,
                             int *node_suspected, spacetime_op_t *read_write_ops, uint8_t thread_id);
#endif
/* ABI note: the reference's callers are built by gcc, which passes the 8-byte (packed)
 * spacetime_group_membership in one general-purpose register. clang classifies the same
 * packed struct as MEMORY (stack), so the library defines this entry point with the 8 bytes
 * received as a uint64_t (HKV_IMPLEMENTATION), matching what gcc-built callers pass. */

/* spacetime.h:211. Creates the default table in HBM (hkv_set_default_config, else the
 * reference defaults: 2^21 buckets, 1 GiB log) and populates hkv_config.num_keys keys
 * (default 1,000,000) exactly as the reference does. instance_id becomes machine_id unless
 * hkv_set_default_config set one. */
void spacetime_init(int instance_id);

/* spacetime.h:212. Populates the default table (creating it if needed); kv is accepted for
 * signature compatibility and may be &kv or NULL. */
void spacetime_populate_fixed_len(struct spacetime_kv *kv, int n, int val_len);

/* ------------------------------------------------------------------ hkv extensions */

typedef struct hkv_config {
    uint32_t abi_version;       /* HKV_ABI_VERSION */
    uint32_t machine_id;        /* reference global machine_id (hrd.h:87) */
    uint32_t rmw_enabled;       /* ENABLE_RMWs (config.h:37) */
    uint32_t big_objects;       /* USE_BIG_OBJECTS (hrd.h:36) */
    uint32_t extra_cache_lines; /* EXTRA_CACHE_LINES (hrd.h:37) */
    int32_t  device;            /* HIP device ordinal */
    uint32_t rw_len;            /* elements of read_write_ops (max_batch_size, default 250) */
    uint32_t skew_flags;        /* HKV_SKEW_*: the reference's opt-in skew optimisations (0 = off,
                                   the reference's default configuration) */
    uint64_t num_keys;          /* SPACETIME_NUM_KEYS (spacetime.h:21) */
    uint64_t num_bkts;          /* SPACETIME_NUM_BKTS (spacetime.h:22), power of two <= 2^31 */
    uint64_t log_cap;           /* SPACETIME_LOG_CAP (spacetime.h:23), power of two */
} hkv_config;

/* hkv_config.skew_flags: the exec-side skew optimisations of config.h:77-80, compile-time
 * switches in the reference and per table here. Both change only the op, never the key's meta.
 *   HKV_SKEW_READ_COMPLETE   ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS (config.h:79,
 *       hermesKV.c:224-238): a stalled GET records the key's timestamp the first time (its ts is
 *       (0, 0) after a refill) and completes, without copying a value, once the key's version is
 *       at least two above it (a write completed after the read was issued).
 *   HKV_SKEW_WRITE_COALESCE  ENABLE_WRITE_COALESCE_TO_THE_SAME_KEY_IN_SAME_NODE (config.h:80,
 *       hermesKV.c:196-221): a PUT stalling behind a local write records the key's version (16
 *       bits) when its own ts.version is 0, and completes (PUT_COMPLETE, no INV) once the key's
 *       version is at least two above it.
 * The refill-side flag (ENABLE_COALESCE_OF_HOT_REQS) is hkv_wl_refill's. */
#define HKV_SKEW_READ_COMPLETE  1u
#define HKV_SKEW_WRITE_COALESCE 2u

typedef struct hkv_table hkv_table;

/* One batch launch: n_batches batches of the same type, batch b owning elements
 * [b*stride, b*stride + counts[b]) of d_elems (HKV_BATCH_PACKED: see below), applied in
 * concatenation order. */
typedef struct hkv_batch_desc {
    int32_t  type;              /* enum hermes_batch_type_t */
    int32_t  n_batches;
    int32_t  stride;            /* elements reserved per batch */
    uint16_t elem_size;         /* sizeof_op_elem */
    uint16_t flags;             /* HKV_BATCH_*: which engine runs the launch (0 = by size) */
    uint8_t *d_elems;           /* device */
    const int32_t *d_counts;    /* device, n_batches entries; NULL = stride each */
    uint8_t *d_rw;              /* device base of batch 0's read_write_ops (ACK batches) */
    int64_t  rw_stride_bytes;   /* bytes between consecutive batches' read_write_ops */
    int32_t *d_node_suspected;  /* device, n_batches entries (INV batches); NULL = ignore */
    uint8_t  membership[8];     /* spacetime_group_membership by value */
    uint8_t *d_state_out;       /* device, local batches: receives each element's final state byte
                                   (op byte 9; n_batches * stride bytes), a mirror the worker loop's
                                   next passes can read instead of the ops; NULL = none (ABI 2) */
    const uint8_t *d_opcode_in; /* device, local batches: the caller's mirror of each element's opcode
                                   (op byte 8; n_batches * stride bytes), e.g. written by its refill
                                   (hkv_wl_refill); lets the launch find its PUTs without reading
                                   every op. A PUT the mirror misses raises error flag bit 3.
                                   NULL = read the ops (ABI 3). ACK batches with d_rw: the mirror of
                                   each read_write_ops slot's opcode (rw_stride_bytes / op size per
                                   batch), which a completion reads instead of the op; it must describe
                                   the ops (round 4) */
    const uint8_t *d_patch;     /* device, local batches: pending header writes, HKV_PATCH_BYTES per element
                                   (n_batches * stride), NULL = none (ABI 5). An element whose patch is
                                   valid first gets the patch's bytes, exactly as if the caller had written
                                   them into the op before the launch; hkv_wl_refill_plan writes a refill
                                   this way, so the launch's own write-back of every op replaces the
                                   refill's pass over the op slab. The mirrors (d_opcode_in) must already
                                   describe the patched ops. */
    uint8_t *d_rw_state;        /* device, ACK batches: a mirror of the read_write_ops' state bytes
                                   (rw_stride_bytes / op size per batch); every completion a launch writes
                                   into read_write_ops is also written here. NULL = none (ABI 5) */
    const uint64_t *d_put_keys; /* reserved, must be NULL (ABI 8; ABI 6-7: a PUT-key mirror for the local
                                   launch's prepass, measured slower and removed) */
    int32_t  n_rows;            /* HKV_BATCH_ROWS: rows of elements, applied row after row (ABI 6) */
    int32_t  skip_row;          /* HKV_BATCH_ROWS: a row that is not applied (-1: none) */
    int64_t  row_stride;        /* HKV_BATCH_ROWS: elements from one row to the next in d_elems */
    uint8_t *d_ack_out;         /* INV launches with HKV_BATCH_UNIQUE, 64-byte entries: element i's answer, as the
                                   worker's ACK callbacks make it (hermes_worker.c:69-118: an ACK from this
                                   machine for INV_SUCCESS, the element itself as INV-abort when ack_out_size holds
                                   it, else opcode ST_EMPTY), written to d_ack_out + i * ack_out_size by the launch
                                   itself, and each answered element leaves with opcode ST_EMPTY, as after the
                                   callbacks' send (ack_modify_elem_after_send). NULL = none (ABI 6)
                                   ACK launches with HKV_BATCH_ROWS, 16-byte ACKs and 64-byte entries: the VAL
                                   callbacks (hermes_worker.c:122-157) instead -- every row element of a batch
                                   whose result opcode is not ACK_SUCCESS, MEMBERSHIP_CHANGE or EMPTY is copied
                                   to d_ack_out + (r * row_stride + j) * 16 with opcode ST_OP_VAL and sender =
                                   this machine (val_copy_and_modify_elem), every other live position there
                                   gets opcode ST_EMPTY, and every non-empty element leaves with opcode
                                   ST_EMPTY (val_skip_or_get_sender_id, val_modify_elem_after_send);
                                   ack_out_size 16. Live positions are those of a batch's range in a row other
                                   than skip_row: the positions of skip_row and those past the last batch's
                                   end are not written (they keep what the buffer held), so a caller reads
                                   only live positions */
    uint32_t ack_out_size;
    const uint64_t *d_phys;     /* reserved, must be NULL (ABI 8; ABI 7: located entries that skipped the
                                   bucket read the reference makes, never the default, removed) */
} hkv_batch_desc;

/* d_patch layout (16 bytes per element): key 0..7, opcode 8, val_len 9, flags (RMW_flag | no_coales
 * << 1) 10..11, value fill byte 12 (0: the value is kept), ts reset 13 (1: ts bytes 11..15 := 0),
 * valid 14 (1: apply), 15 unused. Applying sets op bytes 0..7 = key, 8 = opcode, 9 = ST_NEW,
 * 10 = val_len, [11..15 = 0], 16..17 = flags and, with a fill byte, the ST_VALUE_SIZE value bytes. */
#define HKV_PATCH_BYTES 16

/* hkv_batch_desc.flags. By default launches of at most 4096 elements run as one single-workgroup
 * kernel and larger ones on the multi-kernel engine; both give the same bytes. */
#define HKV_BATCH_ENGINE 1u     /* always the multi-kernel engine */
#define HKV_BATCH_SMALL  2u     /* the single-workgroup kernel (launches of at most 4096 elements) */
/* INV, ACK and VAL batches stored back to back: d_counts holds n_batches + 1 element offsets (batch
 * b is elements [d_counts[b], d_counts[b+1]) of d_elems) and stride is the total, d_counts[n_batches];
 * an ACK batch b still completes into d_rw + b * rw_stride_bytes. Same results as the row layout;
 * no empty slots to launch over. */
#define HKV_BATCH_PACKED 4u
/* The caller guarantees that no key appears twice among the launch's elements (INV and ACK
 * launches): each element is then its key's only one and is applied to the entry in a single pass,
 * in any order. A replica's INV slab of one round has this property (a coordinator has at most one
 * write in flight per key: hermes_exec_write stalls while op_buffer_index is set,
 * hermesKV.c:331-344), and so have one peer's ACKs to it, so a receiver applies each peer's slab as
 * one such launch. A duplicate breaks the results; with HKV_CHECK_UNIQUE=1 in the environment every
 * launch checks and raises error flag bit 4. */
#define HKV_BATCH_UNIQUE 8u
/* With HKV_BATCH_UNIQUE, INV and ACK launches of 64-byte entries: n_rows (at most 8) launches of one
 * layout in one, applied in row order -- row r is the launch whose elements start at element
 * r * row_stride of d_elems (the same n_batches, stride, counts or offsets and read_write_ops for every
 * row), row skip_row excepted. Element j of every row carries the same key, or is a hole (opcode byte
 * 0: not an element of its row's batch; nothing of it is read or written). So each key is looked up
 * once and its elements applied one row after the other: a coordinator's ACKs from all its peers, lined
 * up with the INVs they answer, go in one launch, and so do INVs that peers sent for the same keys.
 * An element whose key differs from its position's raises error flag bit 4. d_node_suspected must be
 * NULL. */
#define HKV_BATCH_ROWS 16u   /* packed rows: elements past d_counts[n_batches] (<= stride) are in no batch */
/* Bits 5..7 are reserved (ABI 8; ABI 6-7: a local launch in two calls, HKV_BATCH_PREPASS / PREPASSED /
 * PREPASS_CANCEL, measured slower and removed): a launch that sets them fails. */
#define HKV_BATCH_RESERVED_FLAGS 0xE0u
#define HKV_MAX_ROWS 8
int  hkv_abi_version(void);
/* 1 when the library was built with work-skipping timing modes (-DHKV_DEBUG_MODES, HKV_DBG):
 * such a build is for timing experiments only and bench.py refuses to report from it. */
int  hkv_debug_modes(void);
const char *hkv_last_error(void);

int  hkv_table_create(const hkv_config *cfg, hkv_table **out);
int  hkv_table_destroy(hkv_table *t);
/* spacetime_populate_fixed_len on the device (reverse id order, MICA slot rules) */
int  hkv_table_populate(hkv_table *t, int64_t n, int val_len);
int  hkv_table_config(const hkv_table *t, hkv_config *out);
/* changes hkv_config.skew_flags of a table between launches (e.g. to time several policies on
 * one table); ordered after the launches already enqueued on the table's streams by the caller */
int  hkv_table_set_skew(hkv_table *t, uint32_t skew_flags);

/* device-resident batch path, asynchronous on `stream` (NULL = the HIP null stream). One
 * stream at a time per table: launches share the table's round scratch (entry ids, stages,
 * shadow images) and its per-log-line F/X/Y/T words. */
int  hkv_batch_async(hkv_table *t, const hkv_batch_desc *desc, void *stream);
int  hkv_sync(hkv_table *t, void *stream);

/* parity / debugging views of the HBM image (reference byte layout) */
int  hkv_copy_index(hkv_table *t, void *host_dst, uint64_t offset, uint64_t bytes);
int  hkv_copy_log(hkv_table *t, void *host_dst, uint64_t offset, uint64_t bytes);
uint64_t hkv_log_head(const hkv_table *t);
int64_t  hkv_num_index_evictions(const hkv_table *t);
void *hkv_device_index(hkv_table *t);
/* internal-consistency flags raised by the device path since the last call (0 = none);
 * bit 0: an element resolved in parallel (not a key's first mutating element) changed the meta;
 * bit 1: the ACK direct path completed a write from an unexpected state;
 * bit 2: a local launch's mutating element had not offered itself in its prepass;
 * bit 3: d_opcode_in missed a PUT;
 * bit 4: an HKV_BATCH_UNIQUE launch held a key twice (checked with HKV_CHECK_UNIQUE=1), or an
 *        HKV_BATCH_ROWS position's rows disagree on the key */
int  hkv_take_error_flags(hkv_table *t, uint32_t *out);
void *hkv_device_log(hkv_table *t);

/* default table used by the reference entry points */
int  hkv_set_default_config(const hkv_config *cfg);
hkv_table *hkv_default_table(void);

/* test hooks of the host entry point's combining submit: with a hold of n, the caller that
 * assembles the next launch first waits (up to 5 s) until n batches are queued, so a test can put
 * batches from several threads into one launch in a known order; 0 (default) = no hold. queued =
 * batches waiting in the default table's queue now. */
int  hkv_debug_host_hold(int n_batches);
int  hkv_debug_host_queued(void);

/* synthetic workload helpers (device kernels) */
/* keys_second[i] = CityHash128(&id_i, 4).second for ids[i] (mica_gen_keys, mica.c:149-165) */
int  hkv_hash_ids(const uint32_t *d_ids, uint64_t *d_keys_second, int64_t n, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HERMESKV_H */
