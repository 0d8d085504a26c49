/* The reference's threading at the drop-in boundary: T worker threads (a gcc-built caller, like
 * the reference's run_worker threads, main.c:193-210) call hermes_batch_ops_to_KVS concurrently
 * on the default table with 250-op local batches, then ACK their own writes
 * (hermes_worker.c:451, 484).
 *
 *   capi_threads throughput T SECONDS WRITE_PERMILLE
 *       uniform keys over the 1M-key reference table; prints one JSON line with the aggregate
 *       rate of batch elements (local ops + ACKs) and of local ops.
 *   capi_threads trace T ROUNDS DIR
 *       thread k uses only key ids = k (mod T), so threads never share a key and any interleaving
 *       gives every key the same history; each thread writes its calls (inputs and outputs) to
 *       DIR/thread<k>.bin for tests/test_capi_threads.py to replay on the oracle.
 *   capi_threads shared ROUNDS DIR
 *       five threads on 32 shared hot keys, each round one call per thread, all five combined into
 *       one launch in thread order (hkv_debug_host_hold): a local batch, INVs from peers 1-2, the
 *       peers' ACKs of the previous round's writes (with that batch as read_write_ops), VALs of
 *       the previous round's INVs, and a second local batch. Every call is recorded to
 *       DIR/thread<k>.bin; replayed in round-major, thread order on the oracle they must match.
 *
 * Build (__graft_entry__.build): gcc -O2 -pthread -I include tools/capi_threads.c -L hermes_amd
 *   -lhermeskv -Wl,-rpath,'$ORIGIN/../hermes_amd' -o tools/capi_threads
 */
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hermeskv.h"

typedef struct {
    uint64_t key;
    uint8_t opcode, state, val_len, cid;
    uint32_t ver;
    uint16_t flags;
    uint8_t value[31];
    uint8_t pad[7];
} op56; /* spacetime_op_t (spacetime.h:170-185) */
typedef struct {
    uint64_t key;
    uint8_t opcode, sender, val_len, cid;
    uint32_t ver;
} msg16; /* spacetime_ack_t (spacetime.h:151-166) */

enum { S = 250, NKEYS = 1000000 };

static spacetime_group_membership g_mb;
static uint64_t *g_keys;  /* CityHash128(&id, 4).second, from the table itself via hkv_copy_log */
static int g_threads, g_rounds, g_write_pm;
static double g_seconds;
static const char *g_dir;
static pthread_barrier_t g_start;

typedef struct {
    int k;
    long elems, local;
    double secs;
} th_t;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static uint64_t sm64(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

static void rec(FILE *f, int type, const void *in, const void *out, int n, int esz, const void *rw_in,
                const void *rw_out)
{
    if (!f) return;
    int32_t h[3] = {type, n, esz};
    fwrite(h, 4, 3, f);
    fwrite(in, (size_t)esz, (size_t)n, f);
    fwrite(out, (size_t)esz, (size_t)n, f);
    int32_t has_rw = rw_in != NULL;
    fwrite(&has_rw, 4, 1, f);
    if (has_rw) {
        fwrite(rw_in, sizeof(op56), S, f);
        fwrite(rw_out, sizeof(op56), S, f);
    }
}

static void *worker(void *arg)
{
    th_t *th = (th_t *)arg;
    op56 *ops = calloc(S, sizeof(op56)), *in = calloc(S, sizeof(op56)), *rw_in = calloc(S, sizeof(op56));
    msg16 *ackbuf = calloc(2 * S, sizeof(msg16)), *ain = calloc(2 * S, sizeof(msg16));
    FILE *f = NULL;
    if (g_dir) {
        char path[512];
        snprintf(path, sizeof path, "%s/thread%d.bin", g_dir, th->k);
        f = fopen(path, "wb");
    }
    uint64_t rng = 0x5EED + (uint64_t)th->k * 7919;
    pthread_barrier_wait(&g_start);
    const double t0 = now_s();
    long elems = 0, local = 0;
    for (int round = 0;; ++round) {
        if (g_dir ? round >= g_rounds : now_s() - t0 >= g_seconds) break;
        for (int i = 0; i < S; i++) {  /* refill: a fresh batch each round */
            rng = sm64(rng);
            uint32_t id = (uint32_t)(rng % NKEYS);
            if (g_dir) id = id - id % (uint32_t)g_threads + (uint32_t)th->k;
            if (id >= NKEYS) id = (uint32_t)th->k;
            memset(&ops[i], 0, sizeof(op56));
            ops[i].key = g_keys[id];
            ops[i].state = 141;
            const int put = (uint32_t)((rng >> 40) % 1000u) < (uint32_t)g_write_pm;
            ops[i].opcode = put ? 112 : 111;
            if (put) {
                ops[i].val_len = 31;
                memset(ops[i].value, 'a' + (th->k % 20), 31);
            }
        }
        memcpy(in, ops, sizeof(op56) * S);
        hermes_batch_ops_to_KVS(local_ops, (uint8_t *)ops, S, sizeof(op56), g_mb, NULL, NULL, (uint8_t)th->k);
        rec(f, local_ops, in, ops, S, sizeof(op56), NULL, NULL);
        int na = 0;
        for (int i = 0; i < S; i++) {  /* the peers' ACKs for this batch's writes */
            if (ops[i].state != 122) continue;
            ops[i].state = 143;      /* inv_modify_elem_after_send */
            for (uint8_t p = 1; p <= 2; p++) {
                msg16 *a = &ackbuf[na++];
                a->key = ops[i].key;
                a->opcode = 115;
                a->sender = p;
                a->val_len = 0;
                a->cid = ops[i].cid;
                a->ver = ops[i].ver;
            }
        }
        elems += S;
        local += S;
        if (na) {
            memcpy(ain, ackbuf, sizeof(msg16) * na);
            memcpy(rw_in, ops, sizeof(op56) * S);
            hermes_batch_ops_to_KVS(acks, (uint8_t *)ackbuf, na, sizeof(msg16), g_mb, NULL, (spacetime_op_t *)ops,
                                    (uint8_t)th->k);
            rec(f, acks, ain, ackbuf, na, sizeof(msg16), rw_in, ops);
            elems += na;
        }
    }
    th->secs = now_s() - t0;
    th->elems = elems;
    th->local = local;
    if (f) fclose(f);
    free(ops); free(in); free(rw_in); free(ackbuf); free(ain);
    return NULL;
}

/* ---- shared mode: mixed batch types on shared keys in one combined launch */
enum { SH_T = 5, SH_KEYS = 32, SH_INVS = 64 };
static pthread_barrier_t g_round;
static op56 g_prev_local[S];     /* thread 0's output of the previous round */
static op56 g_prev_invs[SH_INVS];
static int g_prev_ninv;

static void *shared_worker(void *arg)
{
    th_t *th = (th_t *)arg;
    const int k = th->k;
    char path[512];
    snprintf(path, sizeof path, "%s/thread%d.bin", g_dir, k);
    FILE *f = fopen(path, "wb");
    op56 *ops = calloc(S, sizeof(op56)), *in = calloc(S, sizeof(op56));
    op56 *rw = calloc(S, sizeof(op56)), *rw_in = calloc(S, sizeof(op56));
    msg16 *msg = calloc(2 * S, sizeof(msg16)), *min_ = calloc(2 * S, sizeof(msg16));
    uint64_t rng = 0xC0FFEE + (uint64_t)k * 104729;
    for (int round = 0; round < g_rounds; ++round) {
        int n = 0, type = local_ops, esz = sizeof(op56), with_rw = 0;
        uint8_t *buf = (uint8_t *)ops;
        if (k == 0 || k == 4) {             /* local GET/PUT batch over the hot keys */
            n = S;
            for (int i = 0; i < S; i++) {
                rng = sm64(rng);
                memset(&ops[i], 0, sizeof(op56));
                ops[i].key = g_keys[rng % SH_KEYS];
                ops[i].state = 141;
                const int put = (uint32_t)((rng >> 40) % 1000u) < 300u;
                ops[i].opcode = put ? 112 : 111;
                if (put) {
                    ops[i].val_len = 31;
                    memset(ops[i].value, 'a' + k, 31);
                }
            }
        } else if (k == 1) {                /* INVs from peers 1 and 2 with small timestamps */
            type = invs;
            n = SH_INVS;
            for (int i = 0; i < n; i++) {
                rng = sm64(rng);
                memset(&ops[i], 0, sizeof(op56));
                ops[i].key = g_keys[rng % SH_KEYS];
                ops[i].opcode = 114;
                ops[i].state = (uint8_t)(1 + (rng >> 20) % 2);  /* sender */
                ops[i].cid = ops[i].state;
                ops[i].ver = (uint32_t)(2 * ((rng >> 30) % (uint64_t)(round + 3)));
                ops[i].val_len = 31;
                memset(ops[i].value, 'p' + ops[i].cid, 31);
            }
        } else if (k == 2) {                /* the peers' ACKs of thread 0's previous writes */
            type = acks;
            esz = sizeof(msg16);
            buf = (uint8_t *)msg;
            memcpy(rw, g_prev_local, sizeof(op56) * S);
            for (int i = 0; i < S && round > 0; i++) {
                if (rw[i].state != 122) continue;
                rw[i].state = 143;          /* inv_modify_elem_after_send */
                for (uint8_t p = 1; p <= 2; p++) {
                    msg16 *a = &msg[n++];
                    memset(a, 0, sizeof *a);
                    a->key = rw[i].key;
                    a->opcode = 115;
                    a->sender = p;
                    a->cid = rw[i].cid;
                    a->ver = rw[i].ver;
                }
            }
            if (n == 0) {                   /* round 0: one ACK no write waits for (ACK_SUCCESS) */
                memset(&msg[0], 0, sizeof msg[0]);
                msg[0].key = g_keys[0];
                msg[0].opcode = 115;
                msg[0].sender = 1;
                msg[0].ver = 0x7FFF;
                n = 1;
            }
            with_rw = 1;
        } else {                            /* VALs of thread 1's previous INVs */
            type = vals;
            esz = sizeof(msg16);
            buf = (uint8_t *)msg;
            for (int i = 0; i < g_prev_ninv && round > 0; i++) {
                msg16 *v = &msg[n++];
                memset(v, 0, sizeof *v);
                v->key = g_prev_invs[i].key;
                v->opcode = 116;
                v->sender = g_prev_invs[i].cid;
                v->cid = g_prev_invs[i].cid;
                v->ver = g_prev_invs[i].ver;
            }
            if (n == 0) {                   /* round 0: one VAL that matches nothing */
                memset(&msg[0], 0, sizeof msg[0]);
                msg[0].key = g_keys[1];
                msg[0].opcode = 116;
                msg[0].sender = 2;
                msg[0].ver = 0x7FFF;
                n = 1;
            }
        }
        memcpy(type == acks || type == vals ? (void *)min_ : (void *)in, buf, (size_t)n * esz);
        if (with_rw) memcpy(rw_in, rw, sizeof(op56) * S);
        pthread_barrier_wait(&g_round);
        /* queue in thread order: thread k calls once k batches are queued */
        while (hkv_debug_host_queued() < k) sched_yield();
        hermes_batch_ops_to_KVS(type, buf, n, (uint16_t)esz, g_mb, NULL, with_rw ? (spacetime_op_t *)rw : NULL,
                                (uint8_t)k);
        pthread_barrier_wait(&g_round);
        rec(f, type, type == acks || type == vals ? (void *)min_ : (void *)in, buf, n, esz, with_rw ? rw_in : NULL,
            with_rw ? rw : NULL);
        if (k == 0) memcpy(g_prev_local, ops, sizeof(op56) * S);
        if (k == 1) {
            memcpy(g_prev_invs, ops, sizeof(op56) * SH_INVS);
            g_prev_ninv = SH_INVS;
        }
        pthread_barrier_wait(&g_round);
    }
    fclose(f);
    free(ops); free(in); free(rw); free(rw_in); free(msg); free(min_);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 4 || (argc < 5 && strcmp(argv[1], "shared") != 0)) {
        fprintf(stderr, "usage: %s throughput T SECONDS WRITE_PERMILLE | trace T ROUNDS DIR | shared ROUNDS DIR\n",
                argv[0]);
        return 2;
    }
    const int trace = strcmp(argv[1], "trace") == 0, shared = strcmp(argv[1], "shared") == 0;
    g_threads = atoi(argv[2]);
    if (shared) {
        g_threads = SH_T;
        g_rounds = atoi(argv[2]);
        g_dir = argv[3];
    } else if (trace) {
        g_rounds = atoi(argv[3]);
        g_dir = argv[4];
        g_write_pm = 200;
    } else {
        g_seconds = atof(argv[3]);
        g_write_pm = atoi(argv[4]);
    }
    spacetime_init(0);  /* the reference defaults: 1M keys, 2^21 buckets, machine 0 */
    memset(&g_mb, 0, sizeof g_mb);
    g_mb.num_of_alive_remotes = 2;
    g_mb.g_membership.bit_array[0] = 0x07;
    g_mb.w_ack_init.bit_array[0] = 0xF9;
    /* key ids -> keys, read back from the populated log (ids n-1..0 were inserted in that order,
     * one 64-B entry each from offset 0: entry j holds id n-1-j) */
    hkv_table *t = hkv_default_table();
    uint8_t *log = malloc((size_t)NKEYS * 64);
    if (hkv_copy_log(t, log, 0, (uint64_t)NKEYS * 64)) {
        fprintf(stderr, "copy log: %s\n", hkv_last_error());
        return 1;
    }
    g_keys = malloc(sizeof(uint64_t) * NKEYS);
    for (int j = 0; j < NKEYS; j++) memcpy(&g_keys[NKEYS - 1 - j], log + (size_t)j * 64 + 8, 8);
    free(log);
    if (shared) {
        pthread_barrier_init(&g_round, NULL, SH_T);
        hkv_debug_host_hold(SH_T);
        pthread_t st[SH_T];
        th_t sh[SH_T];
        for (int k = 0; k < SH_T; k++) {
            sh[k].k = k;
            pthread_create(&st[k], NULL, shared_worker, &sh[k]);
        }
        for (int k = 0; k < SH_T; k++) pthread_join(st[k], NULL);
        hkv_debug_host_hold(0);
        printf("{\"shared_rounds\": %d}\n", g_rounds);
        return 0;
    }
    pthread_barrier_init(&g_start, NULL, (unsigned)g_threads);
    pthread_t *tid = calloc((size_t)g_threads, sizeof(pthread_t));
    th_t *th = calloc((size_t)g_threads, sizeof(th_t));
    for (int k = 0; k < g_threads; k++) {
        th[k].k = k;
        pthread_create(&tid[k], NULL, worker, &th[k]);
    }
    long elems = 0, local = 0;
    double secs = 0;
    for (int k = 0; k < g_threads; k++) {
        pthread_join(tid[k], NULL);
        elems += th[k].elems;
        local += th[k].local;
        if (th[k].secs > secs) secs = th[k].secs;
    }
    printf("{\"threads\": %d, \"seconds\": %.3f, \"elements_per_s\": %.1f, \"local_ops_per_s\": %.1f, "
           "\"write_permille\": %d}\n", g_threads, secs, elems / secs, local / secs, g_write_pm);
    return 0;
}
