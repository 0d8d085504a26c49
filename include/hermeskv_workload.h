/*
 * hermeskv_workload.h -- device kernels around the batch path:
 * trace generation, refill with commit counting, and the message marshalling the worker
 * loop does between batch calls. They let a benchmark or a replica group keep batches in
 * HBM from one protocol round to the next.
 *
 *   hkv_wl_gen_trace      create_uni_trace / parse_trace, util.c:228-343 (seeded, Zipf or uniform)
 *   hkv_wl_refill         refill_ops, inline-util.h:149-303 (commit counting :205-217)
 *   hkv_wl_marshal_invs   inv_skip_or_get_sender_id / inv_modify_elem_after_send /
 *                         inv_copy_and_modify_elem, hermes_worker.c:12-65
 *   hkv_wl_marshal_acks   ack_skip_or_get_sender_id / ack_copy_and_modify_elem, :69-118
 *   hkv_wl_marshal_vals   val_skip_or_get_sender_id / val_copy_and_modify_elem, :122-157
 *   hkv_wl_marshal_memb_vals  memb_change_* callbacks, :163-203
 *   hkv_wl_peer_acks      the ACKs / INV-aborts `n_peers` replicas answer to a slab of INVs
 *                         (the remote side of hermes_worker.c:467-473)
 *   hkv_wl_gen_peer_round, hkv_wl_peer_ts
 *                         INVs + VALs written by virtual peer replicas (a coordinator's
 *                         inv_copy_and_modify_elem + val_copy_and_modify_elem)
 * All device pointers; stream = hipStream_t or NULL.
 */
#ifndef HERMESKV_WORKLOAD_H
#define HERMESKV_WORKLOAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hkv_table hkv_table;

typedef struct hkv_zipf {
    double theta;      /* 0 = uniform */
    double zetan;      /* sum_{i=1..n} 1/i^theta */
    double alpha;      /* 1 / (1 - theta) */
    double eta;        /* (1 - (2/n)^(1-theta)) / (1 - zeta(2)/zetan) */
    double half_pow;   /* 1 + 0.5^theta */
    uint64_t n;        /* number of key ids */
} hkv_zipf;

/* trace[w*len + j]: key = CityHash128(&id,4).second, op = ST_OP_PUT with probability
 * write_permille/1000 (then ST_OP_RMW with probability rmw_permille/1000 when RMWs are on),
 * else ST_OP_GET; ids drawn from zipf (seeded splitmix64 streams, one per worker) */
int hkv_wl_gen_trace(uint64_t *d_trace_key, uint8_t *d_trace_op, uint32_t *d_trace_id, int32_t n_workers,
                     int32_t len, const hkv_zipf *zipf, uint32_t write_permille, uint32_t rmw_permille,
                     uint64_t seed, void *stream);

/* refill_ops over n_workers buffers of `stride` ops (op_size bytes each). Slots that are
 * complete take the next trace command of their worker (all slots when first_iter); stalled ops
 * keep their slot and are retried, as in the reference. flags (HKV_WL_*):
 *   HKV_WL_REFILL_ALL    not the reference: stalled ops (GET/PUT/RMW stalls, ST_EMPTY, ST_NEW) are
 *                        dropped (counted) and take a fresh command too; ops in flight
 *                        (PUT/RMW/REPLAY_SUCCESS, IN_PROGRESS_*, *_COMPLETE_SEND_VALS, membership
 *                        change) always keep their slot;
 *   HKV_WL_READ_TS_RESET ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS (inline-util.h:268-272): a
 *                        refilled GET's timestamp becomes (0, 0) (pairs with HKV_SKEW_READ_COMPLETE);
 *   HKV_WL_COALESCE_HOT  ENABLE_COALESCE_OF_HOT_REQS (inline-util.h:237-257): GETs/PUTs on the 100
 *                        hottest ids are absorbed into the worker's last op of that id and opcode
 *                        (no_coales + 1; a completed op commits no_coales ops). Needs d_trace_id (the
 *                        trace's key ids, rank = id) and d_hot (2 * 100 bytes per worker, 0xFF
 *                        before the first refill: the n_hottest_keys_in_ops pointers as slot
 *                        indexes, hermes_worker.c:394-399); op_size * stride <= 56 KiB.
 * Counts completed-and-committed ops (everything complete except ST_MISS and ST_RMW_ABORT),
 * misses, completed writes, dropped stalled ops and RMW aborts (ST_RMW_ABORT) into
 * d_counters: HKV_WL_COUNTER_WORDS words, zeroed by the caller once, of which the words from
 * HKV_WL_STRIPE_BASE on are per-worker-group partial sums (one counter address hit by every
 * worker serialises in L2); hkv_wl_fold_counters adds them into d_counters[0..4] when the
 * caller reads the totals. d_opcode_out (NULL = none): every op's opcode byte after the refill,
 * the mirror hkv_batch_desc.d_opcode_in takes. */
#define HKV_WL_COUNTER_WORDS 4096
#define HKV_WL_STRIPE_BASE 64
#define HKV_WL_REFILL_ALL    1u
#define HKV_WL_READ_TS_RESET 2u
#define HKV_WL_COALESCE_HOT  4u
#define HKV_WL_HOT_KEYS      100
int hkv_wl_refill(uint8_t *d_ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint32_t st_value,
                  uint32_t shift, const uint64_t *d_trace_key, const uint8_t *d_trace_op, const uint32_t *d_trace_id,
                  int32_t trace_len, uint32_t *d_cursor, uint32_t machine_id, int32_t first_iter, uint32_t flags,
                  unsigned long long *d_counters, uint8_t *d_opcode_out, uint8_t *d_hot, void *stream);
/* refill_ops as a plan for the next local launch: the decisions, trace cursors and counts of
 * hkv_wl_refill (not on the first pass; flags HKV_WL_REFILL_ALL and HKV_WL_READ_TS_RESET), made from
 * d_states -- the ops' state bytes, kept by the round (the local launch's d_state_out, the INV and
 * membership marshals, the ACK launch's d_rw_state) -- instead of the ops. Each refilled op gets a
 * valid patch in d_patch (HKV_PATCH_BYTES per op, include/hermeskv.h), every other op an invalid one;
 * d_opcode (the opcode mirror) takes the refilled ops' opcodes. The ops themselves are untouched:
 * the next local launch, given d_patch, applies the patches as it reads them. (ABI 8: the PUT-key
 * mirror argument and hkv_wl_refill_plan_located are gone.) */
int hkv_wl_refill_plan(uint8_t *d_states, int32_t n_workers, int32_t stride, uint32_t st_value, uint32_t shift,
                       const uint64_t *d_trace_key, const uint8_t *d_trace_op, int32_t trace_len, uint32_t *d_cursor,
                       uint32_t machine_id, uint32_t flags, unsigned long long *d_counters, uint8_t *d_opcode,
                       uint8_t *d_patch, void *stream);
/* hkv_wl_refill for big ops (op_size > 64, refilled in place; not on the first pass, flags
 * HKV_WL_REFILL_ALL and HKV_WL_READ_TS_RESET), deciding from d_states, the state mirror
 * hkv_wl_refill_plan reads: an op that is not refilled is not touched, a refilled one is only
 * written (and its mirror byte set to ST_NEW); d_opcode takes the refilled ops' opcodes. */
int hkv_wl_refill_st(uint8_t *d_ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint32_t st_value,
                     uint32_t shift, const uint64_t *d_trace_key, const uint8_t *d_trace_op, int32_t trace_len,
                     uint32_t *d_cursor, uint32_t machine_id, uint32_t flags, unsigned long long *d_counters,
                     uint8_t *d_opcode, uint8_t *d_states, void *stream);
/* d_counters[0..4] += the refill stripes (which are cleared) */
int hkv_wl_fold_counters(unsigned long long *d_counters, void *stream);

/* INVs for this round's successful writes/RMWs/replays: per worker, compacted into
 * d_inv_out[w*stride ..] (op_size-byte spacetime_inv_t, sender = machine_id), count in
 * d_inv_count[w]; the ops move to ST_IN_PROGRESS_* */
int hkv_wl_marshal_invs(uint8_t *d_ops, int32_t n_workers, int32_t stride, uint32_t op_size,
                        uint8_t *d_inv_out, int32_t *d_inv_count, uint32_t machine_id, void *stream);

/* ACKs (or INV-aborts with RMWs) for a batch of received INVs: element i of the INV batch
 * produces element i of d_ack_out (ack_size bytes: 16, or op_size with RMWs), opcode
 * ST_EMPTY where nothing is sent; the INV elements become ST_EMPTY (ack_modify_elem_after_send) */
int hkv_wl_marshal_acks(uint8_t *d_invs, int64_t n, uint32_t op_size, uint8_t *d_ack_out, uint32_t ack_size,
                        uint32_t machine_id, void *stream);

/* VALs for ACK elements that completed a write: element i of d_val_out (16 bytes), ST_EMPTY
 * elsewhere; the ACK elements become ST_EMPTY. As val_skip_or_get_sender_id with the reference's
 * assertions off (config.h:83), every element that is not ST_ACK_SUCCESS, a membership change or
 * empty sends one (after an ACK batch: ST_LAST_ACK_SUCCESS, and ACKs of keys not in the table). */
int hkv_wl_marshal_vals(uint8_t *d_acks, int64_t n, uint32_t ack_size, uint8_t *d_val_out,
                        uint32_t machine_id, void *stream);

/* ---- virtual peer replicas (one-GPU rounds) ------------------------------------------
 * A virtual peer stands for a replica running the same workload. Per round it sends its
 * successful writes: at most one per key (a second local write of a key stalls on
 * op_buffer_index, hermesKV.c:314-356), timestamped by update_actions_n_unlock
 * (hermesKV.c:100-141) from the key's state at round start: version + 2 (+4 for a plain write
 * in an RMW build), cid = the peer. */

/* Draws `per_peer` Zipf keys per worker and peer for round index `round`, keeps each peer's
 * first occurrence of every key (in the peer's worker-major op order), and writes the kept
 * ones compacted per worker in peer order: d_invs / d_vals [n_workers][n_peers * per_peer]
 * (op_size-byte INVs with value 'a' + peer and RMW_flag drawn with rmw_permille; 16-B VALs),
 * d_peer_counts[w * n_peers + r] = how many of peer r's. The timestamps are filled in per
 * round by hkv_wl_peer_ts. d_scratch: hkv_wl_peer_round_scratch() bytes. */
size_t hkv_wl_peer_round_scratch(int32_t n_workers, int32_t per_peer, int32_t n_peers);
int hkv_wl_gen_peer_round(uint8_t *d_invs, uint8_t *d_vals, int32_t *d_peer_counts, int32_t n_workers,
                          int32_t per_peer, const uint8_t *d_peer_ids, int32_t n_peers, uint32_t op_size,
                          uint32_t st_value, uint32_t shift, const hkv_zipf *zipf, uint32_t rmw_permille,
                          uint32_t round, uint64_t seed, void *d_scratch, void *stream);

/* At the start of a round: the first d_counts[w] INVs of each worker's row (and their VALs) take
 * the timestamp the peer's write gives, read from table t. d_peer_ts (RMW builds, may be NULL;
 * hkv_wl_peer_ts_words() zeroed words: 8 per possible entry, log_cap / entry size + 1 of them)
 * records each peer's write per [entry][peer id] for hkv_wl_peer_acks. */
int hkv_wl_peer_ts(hkv_table *t, uint8_t *d_invs, uint8_t *d_vals, const int32_t *d_counts, int32_t n_workers,
                   int32_t stride, uint32_t op_size, unsigned long long *d_peer_ts, uint32_t round, void *stream);
uint64_t hkv_wl_peer_ts_words(const hkv_table *t);

/* The same for n INVs stored back to back (and their VALs), with each INV's entry located
 * beforehand: hkv_wl_peer_locate writes the log offset of every INV's key (~0 when absent) into
 * d_phys once per pre-drawn round index; hkv_wl_peer_ts_at reads one entry line per INV (an INV
 * whose entry no longer holds its key takes the full lookup). */
int hkv_wl_peer_locate(hkv_table *t, const uint8_t *d_invs, int64_t n, uint32_t op_size, uint64_t *d_phys,
                       void *stream);
int hkv_wl_peer_ts_at(hkv_table *t, uint8_t *d_invs, uint8_t *d_vals, const uint64_t *d_phys, int64_t n,
                      uint32_t op_size, unsigned long long *d_peer_ts, uint32_t round, void *stream);
/* hkv_wl_refill_plan and hkv_wl_peer_ts_at in one launch (round 6): the refill plan that ends a round and the
 * virtual peers' timestamps that start the next touch disjoint data, so one grid runs both side by side.
 * Same arguments and results as the two calls in that order. */
int hkv_wl_refill_plan_peer_ts(uint8_t *d_states, int32_t n_workers, int32_t stride, uint32_t st_value, uint32_t shift,
                               const uint64_t *d_trace_key, const uint8_t *d_trace_op, int32_t trace_len,
                               uint32_t *d_cursor, uint32_t machine_id, uint32_t flags,
                               unsigned long long *d_counters, uint8_t *d_opcode, uint8_t *d_patch, hkv_table *t,
                               uint8_t *d_invs, uint8_t *d_vals, const uint64_t *d_phys, int64_t n, uint32_t op_size,
                               unsigned long long *d_peer_ts, uint32_t round, void *stream);
/* The virtual peers' answers to this round's INVs: for INV j of worker w, the ack_size-byte
 * element d_acks[w*out_stride + j*n_peers + r] from peer_ids[r] is an ACK {key, ST_OP_ACK,
 * sender, ts = inv ts} (ack_copy_and_modify_elem, hermes_worker.c:100-118) -- or, with d_peer_ts
 * and an RMW INV below the peer's own write of the key this round, the INV-abort the peer's
 * hermes_exec_inv returns (hermesKV.c:566-576: the peer's RMW flag, timestamp and value). ack_size:
 * 16, or the op size in an RMW build; d_ack_count[w] = n_peers * d_inv_count[w]. out_stride is a
 * multiple of n_peers, at most inv_stride * n_peers, and the caller keeps every d_inv_count[w] <=
 * out_stride / n_peers (the N=1 round fits it to the round's largest count). d_out_off (may be
 * NULL): worker w's answers start at element d_out_off[w] instead (a packed ACK batch, offsets from
 * hkv_wl_ack_offsets); d_ack_count may then be NULL. */
int hkv_wl_peer_acks(hkv_table *t, const uint8_t *d_inv_out, const int32_t *d_inv_count, int32_t n_workers,
                     int32_t inv_stride, uint32_t op_size, uint8_t *d_acks, uint32_t ack_size, int32_t out_stride,
                     int32_t *d_ack_count, const uint8_t *peer_ids, int32_t n_peers,
                     const unsigned long long *d_peer_ts, uint32_t round, const int32_t *d_out_off, void *stream);

/* The same answers laid out peer-major, for one HKV_BATCH_UNIQUE ACK launch per peer: peer r's
 * answers to all INVs of the round form block r of T = d_inv_off[n_workers] elements, worker w's at
 * d_inv_off[w] within it (d_inv_off: the INV offsets, hkv_wl_ack_offsets with n_peers = 1).
 * max_invs >= every d_inv_count[w] (it sizes the grid). */
int hkv_wl_peer_acks_pm(hkv_table *t, const uint8_t *d_inv_out, const int32_t *d_inv_count, int32_t n_workers,
                        int32_t inv_stride, uint32_t op_size, uint8_t *d_acks, uint32_t ack_size, int32_t max_invs,
                        int32_t *d_ack_count, const uint8_t *peer_ids, int32_t n_peers,
                        const unsigned long long *d_peer_ts, uint32_t round, const int32_t *d_inv_off, void *stream);

/* Offsets of a packed ACK batch answering d_inv_count[0..n_workers) INVs from n_peers peers:
 * d_offsets[w] = n_peers * (INVs of workers before w), d_offsets[n_workers] = the total. h_out
 * (pinned host memory, 3 ints) receives the total and the largest d_inv_count: seq = 0, once
 * the stream passes this call (wait on an event); seq > 0, with h_out[2] = seq written after
 * them, for the host to spin on (no event, no fence on the stream). */
int hkv_wl_ack_offsets(const int32_t *d_inv_count, int32_t n_workers, int32_t n_peers, int32_t *d_offsets,
                       int32_t *h_out, int32_t seq, void *stream);

/* ---- replica groups (one replica per GPU, slabs exchanged over RCCL) ------------------ */

/* VALs of the writes/replays a membership change completed (memb_change_* callbacks,
 * hermes_worker.c:163-203): per worker w, ops in state PUT/RMW/REPLAY_COMPLETE_SEND_VALS are
 * compacted in op order into d_val_out[w*out_stride ...] (16-B VALs: the op's key and ts,
 * ST_OP_VAL, sender machine_id), d_count[w] = how many (at most out_stride); the ops become
 * PUT_COMPLETE / RMW_COMPLETE / ST_NEW. stride <= 256. d_states (may be NULL): the ops' state
 * mirror, updated the same way. */
int hkv_wl_marshal_memb_vals(uint8_t *d_ops, int32_t n_workers, int32_t stride, uint32_t op_size,
                             uint8_t *d_val_out, int32_t out_stride, int32_t *d_count, uint32_t machine_id,
                             uint8_t *d_states, void *stream);

/* *h_out = max(d_counts[0..n)), written by the kernel into pinned host memory (hipHostMalloc /
 * hipHostRegister; valid once the stream passes this call): a round's width without a copy. */
int hkv_wl_max_to_host(const int32_t *d_counts, int32_t n, int32_t *h_out, void *stream);

/* hkv_wl_marshal_invs with at most out_stride INVs per worker per round (d_inv_out rows of
 * out_stride); further sendable ops keep their state for a later round and are counted in
 * *d_held (may be NULL). d_states (may be NULL): the state mirror the local batch wrote
 * (hkv_batch_desc.d_state_out), read instead of each op's state byte, and updated with the states
 * the sent ops move to. */
int hkv_wl_marshal_invs_cap(uint8_t *d_ops, int32_t n_workers, int32_t stride, uint32_t op_size,
                            uint8_t *d_inv_out, int32_t out_stride, int32_t *d_inv_count, uint32_t machine_id,
                            unsigned long long *d_held, uint8_t *d_states, void *stream);

/* ACKs for `rows` rows of received INVs (row r: d_in_count[r] INVs at d_invs + r*C*op_size),
 * compacted to the front of row r of d_ack_out (row stride C), d_out_count[r] ACKs; INV
 * elements become ST_EMPTY as in hkv_wl_marshal_acks */
int hkv_wl_marshal_acks_rows(uint8_t *d_invs, const int32_t *d_in_count, int32_t rows, int32_t C,
                             uint32_t op_size, uint8_t *d_ack_out, uint32_t ack_size, int32_t *d_out_count,
                             uint32_t machine_id, void *stream);

/* rows [n_peers][n_workers][C] (counts [n_peers][n_workers]) -> per-worker batches
 * [n_workers][out_stride], the peers' elements back to back in peer order */
int hkv_wl_regroup(const uint8_t *d_in, const int32_t *d_counts, int32_t n_peers, int32_t n_workers, int32_t C,
                   uint32_t elem_size, uint8_t *d_out, int32_t out_stride, int32_t *d_out_count, void *stream);

/* VALs (16 B) for the ACK elements of per-worker ACK batches ([n_workers][stride], counts; or
 * packed, worker w at [d_offsets[w], d_offsets[w+1]) when d_offsets is not NULL) that completed a
 * write, compacted into [n_workers][C]; the ACK elements become ST_EMPTY as in
 * hkv_wl_marshal_vals. C must cover a worker's VALs (the N=1 round: its INV credits); any beyond
 * are counted in *d_held (may be NULL) -- the VAL-credit path (hkv_wl_vals_credit) carries them. */
int hkv_wl_collect_vals(uint8_t *d_acks, const int32_t *d_count, int32_t n_workers, int32_t stride,
                        uint32_t ack_size, uint8_t *d_val_out, int32_t C, int32_t *d_val_count,
                        uint32_t machine_id, unsigned long long *d_held, const int32_t *d_offsets, void *stream);
/* The same over n_blocks peer-major blocks (hkv_wl_peer_acks_pm's layout: block b holds
 * d_offsets[n_workers] elements, worker w's at d_offsets[w]); a worker's VALs in block order. */
int hkv_wl_collect_vals_blocks(uint8_t *d_acks, const int32_t *d_count, int32_t n_workers, int32_t stride,
                               uint32_t ack_size, uint8_t *d_val_out, int32_t C, int32_t *d_val_count,
                               uint32_t machine_id, unsigned long long *d_held, const int32_t *d_offsets,
                               int32_t n_blocks, void *stream);

/* The same over the ACK rows a replica-group coordinator receives (ReplicaRound: n_rows rows of
 * row_stride elements, row p from rank p, lined up with its packed INV slab): worker w's ACKs of
 * every row are [d_offsets[w], d_offsets[w+1]) of the row; empty slots (ST_EMPTY) send nothing. */
int hkv_wl_collect_vals_rows(uint8_t *d_acks, int32_t n_workers, int32_t n_rows, int64_t row_stride,
                             uint32_t ack_size, uint8_t *d_val_out, int32_t C, int32_t *d_val_count,
                             uint32_t machine_id, unsigned long long *d_held, const int32_t *d_offsets, void *stream);

/* ---- VAL credits and the outstanding-VAL gate (hermes_worker.c:479-503, wings.h:424-540, 862-916)
 * Per worker: an ACK queue (d_aq rows of q_stride elements of ack_size bytes, d_aq_n queued) and a
 * carried-VAL queue (d_vq rows of vq_stride 16-B VALs, d_vq_n carried).
 *
 * hkv_wl_marshal_invs_cap under INV credits: worker w may send at most
 * out_stride - d_aq_n[w] / r_alive INVs (INVs whose ACKs still wait in its queue hold theirs). */
int hkv_wl_marshal_invs_credits(uint8_t *d_ops, int32_t n_workers, int32_t stride, uint32_t op_size,
                                uint8_t *d_inv_out, int32_t out_stride, int32_t *d_inv_count, uint32_t machine_id,
                                unsigned long long *d_held, const int32_t *d_aq_n, int32_t r_alive, void *stream);

/* The virtual peers' ACKs (INV-aborts as in hkv_wl_peer_acks) appended to each worker's ACK queue;
 * d_ack_count[w] = the whole queue when d_vq_n[w] == 0, else 0 (the worker does not poll ACKs
 * while it has VALs outstanding). */
int hkv_wl_peer_acks_queue(hkv_table *t, const uint8_t *d_inv_out, const int32_t *d_inv_count, int32_t n_workers,
                           int32_t inv_stride, uint32_t op_size, uint8_t *d_aq, uint32_t ack_size, int32_t q_stride,
                           int32_t *d_aq_n, const int32_t *d_vq_n, int32_t *d_ack_count, const uint8_t *d_peer_ids,
                           int32_t n_peers, const unsigned long long *d_peer_ts, uint32_t round, void *stream);

/* After the ACK batch over the queues (counts d_ack_count): per worker, the carried VALs and then
 * the VALs of the queue's ST_LAST_ACK_SUCCESS elements (when it was applied), in that order; the
 * first min(v_credits, out_stride) go to d_val_out row w (d_val_count), the rest are carried in
 * d_vq. An applied queue's ACK/LAST_ACK/membership-change elements become ST_EMPTY and
 * d_aq_n[w] = 0. VALs that fit nowhere are counted in *d_overflow (may be NULL; 0 when
 * vq_stride >= the INV credits). */
int hkv_wl_vals_credit(uint8_t *d_aq, int32_t *d_aq_n, const int32_t *d_ack_count, int32_t n_workers,
                       int32_t q_stride, uint32_t ack_size, uint8_t *d_vq, int32_t *d_vq_n, int32_t vq_stride,
                       uint8_t *d_val_out, int32_t *d_val_count, int32_t out_stride, int32_t v_credits,
                       uint32_t machine_id, unsigned long long *d_overflow, void *stream);

/* Packed slabs of a replica group (one contiguous slab per rank instead of [W][C] rows):
 * rows [n_rows][C] x elem_size with d_counts[n_rows] -> d_packed, row w at d_offsets[w];
 * d_offsets[n_rows] = the total (d_offsets has n_rows + 1 entries) */
int hkv_wl_pack_rows(const uint8_t *d_rows, const int32_t *d_counts, int32_t n_rows, int32_t C,
                     uint32_t elem_size, uint8_t *d_packed, int32_t *d_offsets, void *stream);
/* This round's INVs (the INV callbacks of hermes_worker.c:12-65) straight into one packed slab of at
 * most `cap` INVs, so a replica group can size its collectives without reading anything back: worker
 * w sends its first min(sendable, C, what cap leaves after the workers before it) INVs to
 * d_out[d_offsets[w] ..] (d_offsets[n_workers] = the slab's total, d_count = sendable per worker,
 * d_sent = sent per worker; d_states is the state mirror, kept up to date). The INVs not sent keep
 * their state and are counted in *d_held. */
int hkv_wl_marshal_invs_packed(uint8_t *d_ops, int32_t n_workers, int32_t stride, uint32_t op_size, uint8_t *d_states,
                               int32_t C, int32_t cap, uint8_t *d_out, int32_t *d_offsets, int32_t *d_count,
                               int32_t *d_sent, uint32_t machine_id, unsigned long long *d_held, void *stream);

/* ACKs for received packed INV slabs ([rows][width], d_counts[rows] live per row), element i of
 * the output in the position of INV i: an ACK (with RMWs an INV-abort) where it applied,
 * ST_EMPTY elsewhere; the INVs become ST_EMPTY as in hkv_wl_marshal_acks */
int hkv_wl_marshal_acks_aligned(uint8_t *d_invs, const int32_t *d_counts, int32_t rows, int32_t width,
                                uint32_t op_size, uint8_t *d_ack_out, uint32_t ack_size, uint32_t machine_id,
                                void *stream);

/* ACK rows returned by the peers ([n_peers][width], lined up with the packed INV slab this
 * coordinator sent: worker w's INVs at d_offsets[w], d_counts[w] of them) -> per-worker ACK
 * batches [n_workers][out_stride], ST_EMPTY elements dropped, counts in d_out_count */
int hkv_wl_regroup_aligned(const uint8_t *d_in, int32_t n_peers, int32_t width, const int32_t *d_offsets,
                           const int32_t *d_counts, int32_t n_workers, uint32_t elem_size, uint8_t *d_out,
                           int32_t out_stride, int32_t *d_out_count, void *stream);

#ifdef __cplusplus
}
#endif
#endif
