/*
 * hkv_oracle_bench.c -- TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg.
 *
 * Times the CPU restatement (hkv_oracle.c) on the same workload shape as the GPU step, one worker
 * thread per core over one shared table as the reference runs (main.c:193-210): each thread runs
 * the reference worker loop (hermes_worker.c:438-546) over its workers' 250-op buffers:
 * refill (inline-util.h:149-303) -> local batch -> INV marshal (hermes_worker.c:12-65) ->
 * ACKs from the virtual peers -> incoming INV batch -> ACK batch (rw = the worker's ops) ->
 * VAL marshal -> incoming VAL batch. Traces and peer INV/VAL slabs are generated before the
 * timed loop with the same generators (splitmix64 streams, Gray/YCSB Zipf, CityHash keys).
 * refill flags (hkv_wl_refill's): 1 gives every worker a fresh batch each round (stalled ops
 * dropped), else stalled ops keep their slots as refill_ops does; 2 resets a refilled GET's
 * timestamp (ENABLE_READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS, inline-util.h:268-272); 4 coalesces
 * requests on the 100 hottest ids into the worker's live op of that id and opcode
 * (ENABLE_COALESCE_OF_HOT_REQS, inline-util.h:237-257; committed ops count no_coales each).
 * The table's skew_flags (hko_config) select the exec-side optimisations.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hkv_oracle.h"

typedef struct hko_zipf { double theta, zetan, alpha, eta, half_pow; uint64_t n; } hko_zipf;

enum { OPC_GET = 111, OPC_PUT = 112, OPC_INV = 114, OPC_ACK = 115, OPC_VAL = 116 };

static uint64_t sm64(uint64_t x)
{
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

static uint64_t zipf_draw(const hko_zipf *z, double u)
{
    if (z->theta <= 0) {
        uint64_t id = (uint64_t)(u * (double)z->n);
        return id < z->n ? id : z->n - 1;
    }
    double uz = u * z->zetan;
    if (uz < 1.0) return 0;
    if (uz < z->half_pow) return 1;
    uint64_t id = (uint64_t)((double)z->n * pow(z->eta * u - z->eta + 1.0, z->alpha));
    return id < z->n ? id : z->n - 1;
}

static uint64_t key_of(uint32_t id)
{
    uint64_t f, s;
    hko_cityhash128(&id, 4, &f, &s);
    return s;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

void hko_set_log_head(hko_kvs *kv, uint64_t head);
uint32_t hko_key_version(hko_kvs *kv, uint64_t key);

enum { BS = 250, BT = 8192, BP = 16 };   /* local batch, trace length, peer round indices */

typedef struct {
    hko_kvs *kv;
    uint32_t osz, sv;
    int n_peers, per_peer, rstride, refill_all, ts_reset, coalesce;
    uint8_t mid;
    uint8_t *ops;
    uint8_t *hot;   /* [n_workers][200]: n_hottest_keys_in_ops_get / _put as slot indexes, 255 = NULL */
    const uint64_t *tkey;
    const uint8_t *top;
    const uint32_t *tid;
    uint32_t *cursor;
    const uint8_t *rinv_pool, *rval_pool;
    const int32_t *rcount;
    int n_workers, w0, w1;
    double seconds;
    pthread_barrier_t *start;
    double *t0;
    int64_t committed, rounds;
    double t_end;
} bench_thread;

/* One worker thread of the reference (hermes_worker.c:438-546) per core, each over its own
 * workers' 250-op buffers; all threads share the table (concurrency control: hkv_oracle.c's
 * seqlock, concur_ctrl.h:144-224). */
static void *bench_worker(void *arg)
{
    bench_thread *b = (bench_thread *)arg;
    const uint32_t osz = b->osz, sv = b->sv;
    const int n_peers = b->n_peers, rstride = b->rstride, S = BS;
    uint8_t *inv_out = calloc(S, osz);
    uint8_t *acks = calloc((size_t)S * (n_peers ? n_peers : 1), 16);
    uint8_t *ack_out = calloc(rstride ? rstride : 1, 16);
    uint8_t *val_out = calloc((size_t)S * (n_peers ? n_peers : 1), 16);
    uint8_t *rinv = calloc(rstride ? rstride : 1, osz);
    uint8_t *rval = calloc(rstride ? rstride : 1, 16);
    uint8_t membership[8] = {2, 0x07, 0xF9, 0, 0, 0, 0, 0};
    const uint8_t mid = b->mid;
    int64_t committed = 0, rounds = 0;
    int first = 1;
    pthread_barrier_wait(b->start);
    const double t0 = *b->t0;
    double t = now_s();
    while (first || t - t0 < b->seconds) {
        for (int w = b->w0; w < b->w1; w++) {
            uint8_t *ow = b->ops + (size_t)w * S * osz;
            /* refill_ops (inline-util.h:149-303) */
            uint8_t *hp = b->hot + (size_t)w * 200;
            for (int i = 0; i < S; i++) {
                uint8_t *o = ow + (size_t)i * osz;
                uint8_t st = o[9];
                int complete = st == 130 || st == 128 || st == 138 || st == 137 || st == 119 || st == 121;
                /* in flight: PUT/RMW/REPLAY_SUCCESS, IN_PROGRESS_*, *_COMPLETE_SEND_VALS, membership change */
                int in_flight = st == 122 || st == 135 || st == 123 || st == 143 || st == 148 || st == 144 ||
                                st == 133 || st == 149 || st == 147 || st == 118;
                if (!first && complete && st != 130 && st != 138)
                    committed += b->coalesce ? (int64_t)((o[16] | o[17] << 8) >> 1) : 1;
                /* stalled ops retry unless refill_all; ops in flight always keep their slot */
                if (!(first || complete || (b->refill_all && !in_flight))) continue;
                if (!first) o[8] = o[9] = 140;   /* reset op bucket */
                int64_t ti = (int64_t)w * BT + b->cursor[w];
                if (b->coalesce && b->top[ti] != 113) {   /* a hot command joins the worker's live op */
                    uint32_t id;
                    int col;
                    for (;;) {
                        ti = (int64_t)w * BT + b->cursor[w];
                        id = b->tid[ti];
                        col = b->top[ti] == OPC_GET ? 0 : 100;
                        if (id < 100 && hp[col + id] != 255 && ow[(size_t)hp[col + id] * osz + 8] == b->top[ti]) {
                            uint8_t *t = ow + (size_t)hp[col + id] * osz;
                            uint16_t v = (uint16_t)(t[16] | t[17] << 8);
                            v = (uint16_t)((v & 1u) | ((((v >> 1) + 1u) & 0x7FFFu) << 1));
                            t[16] = (uint8_t)v;
                            t[17] = (uint8_t)(v >> 8);
                            b->cursor[w] = (b->cursor[w] + 1) % BT;
                        } else {
                            break;
                        }
                    }
                    if (id < 100) hp[col + id] = (uint8_t)i;
                }
                ti = (int64_t)w * BT + b->cursor[w];
                b->cursor[w] = (b->cursor[w] + 1) % BT;
                memcpy(o, &b->tkey[ti], 8);
                o[8] = b->top[ti];
                o[9] = 141;
                o[10] = b->top[ti] == OPC_GET ? 0 : (uint8_t)sv;
                if (b->top[ti] == OPC_GET && b->ts_reset) memset(o + 11, 0, 5);
                o[16] = first ? 0 : 2;   /* no_coales = 1 (not reset on the first pass), RMW_flag 0 */
                o[17] = 0;
                if (b->top[ti] != OPC_GET) memset(o + 18, 'a' + mid, sv);
            }
            hko_batch(b->kv, 0, ow, S, (uint16_t)osz, membership, NULL, NULL);
            /* INV marshalling (hermes_worker.c:12-65) + peers' ACKs */
            int ninv = 0;
            for (int i = 0; i < S; i++) {
                uint8_t *o = ow + (size_t)i * osz;
                if (o[9] != 122) continue;
                uint8_t *x = inv_out + (size_t)ninv * osz;
                memcpy(x, o, osz);
                x[9] = mid;
                x[8] = OPC_INV;
                o[9] = 143;
                for (int r = 0; r < n_peers; r++) {
                    uint8_t *a = acks + ((size_t)ninv * n_peers + r) * 16;
                    memcpy(a, x, 16);
                    a[8] = OPC_ACK;
                    a[9] = (uint8_t)(1 + r);
                }
                ninv++;
            }
            if (rstride) {
                size_t k = (size_t)(rounds % BP) * b->n_workers + w;
                const int rn = b->rcount[k];
                memcpy(rinv, b->rinv_pool + k * rstride * osz, (size_t)rn * osz);
                memcpy(rval, b->rval_pool + k * rstride * 16, (size_t)rn * 16);
                /* the peer's write: the key's current version + 2, cid = the peer (hermesKV.c:100-141) */
                for (int i = 0; i < rn; i++) {
                    uint64_t key;
                    memcpy(&key, rinv + (size_t)i * osz, 8);
                    const uint32_t ver = hko_key_version(b->kv, key) + 2;
                    memcpy(rinv + (size_t)i * osz + 12, &ver, 4);
                    memcpy(rval + (size_t)i * 16 + 12, &ver, 4);
                }
                int ns = -1;
                hko_batch(b->kv, 2, rinv, rn, (uint16_t)osz, membership, &ns, NULL);
                for (int i = 0; i < rn; i++) { /* ACKs back to the peers */
                    uint8_t *x = rinv + (size_t)i * osz, *a = ack_out + (size_t)i * 16;
                    if (x[8] == 124) { memcpy(a, x, 16); a[8] = OPC_ACK; a[9] = mid; }
                    x[8] = 140;
                }
                hko_batch(b->kv, 3, acks, ninv * n_peers, 16, membership, NULL, ow);
                for (int i = 0; i < ninv * n_peers; i++) { /* VALs for completed writes */
                    uint8_t *a = acks + (size_t)i * 16, *v = val_out + (size_t)i * 16;
                    if (a[8] == 126) { memcpy(v, a, 16); v[8] = OPC_VAL; v[9] = mid; }
                    a[8] = 140;
                }
                hko_batch(b->kv, 4, rval, rn, 16, membership, NULL, NULL);
            }
        }
        rounds++;
        first = 0;
        t = now_s();
    }
    /* harvest the last round's completions (counted by the next refill in the reference) */
    for (int64_t i = (int64_t)b->w0 * S; i < (int64_t)b->w1 * S; i++) {
        const uint8_t *o = b->ops + i * osz;
        if (o[9] == 128 || o[9] == 121 || o[9] == 137) committed += b->coalesce ? (int64_t)((o[16] | o[17] << 8) >> 1) : 1;
    }
    b->committed = committed;
    b->rounds = rounds;
    b->t_end = t;
    free(inv_out); free(acks); free(ack_out); free(val_out); free(rinv); free(rval);
    return NULL;
}

/* returns committed ops of all threads; rounds (per thread, the smallest) and seconds (the
 * slowest thread's) through out-params */
int64_t hko_bench_rounds(hko_kvs *kv, const hko_config *cfg, int n_workers, int n_threads, double seconds,
                         const hko_zipf *z, uint32_t write_pm, int n_peers, int per_peer, uint64_t seed,
                         int refill_flags, int64_t *out_rounds, double *out_secs)
{
    const int T = BT, P = BP;
    const uint32_t osz = hko_op_size(cfg), sv = hko_st_value_size(cfg);
    const int rstride = n_peers * per_peer;
    if (n_threads < 1) n_threads = 1;
    if (n_workers < n_threads) n_workers = n_threads;
    uint8_t *ops = calloc((size_t)n_workers * BS, osz);
    uint8_t *rinv_pool = calloc((size_t)n_workers * P * (rstride ? rstride : 1), osz);
    uint8_t *rval_pool = calloc((size_t)n_workers * P * (rstride ? rstride : 1), 16);
    uint64_t *tkey = malloc(sizeof(uint64_t) * (size_t)n_workers * T);
    uint8_t *top = malloc((size_t)n_workers * T);
    uint32_t *tid = malloc(sizeof(uint32_t) * (size_t)n_workers * T);
    uint8_t *hot = malloc((size_t)n_workers * 200);
    memset(hot, 255, (size_t)n_workers * 200);
    uint32_t *cursor = calloc(n_workers, 4);
    const uint8_t mid = (uint8_t)cfg->machine_id;
    /* traces (create_uni_trace / parse_trace shape) */
    for (int64_t g = 0; g < (int64_t)n_workers * T; g++) {
        uint64_t r1 = sm64(seed ^ (0x1000003ull * (uint64_t)g)), r2 = sm64(r1 ^ 0x5EEDull);
        uint32_t id = (uint32_t)zipf_draw(z, (double)(r1 >> 11) * (1.0 / 9007199254740992.0));
        tkey[g] = key_of(id);
        tid[g] = id;
        top[g] = (uint32_t)(r2 % 1000u) < write_pm ? OPC_PUT : OPC_GET;
    }
    /* peer INVs + VALs, P round indices deep: per round, each virtual peer's first write of a key
     * (in its worker-major op order), compacted per worker in peer order -- the GPU run's
     * hkv_wl_gen_peer_round. The timestamps are taken from the table when a round uses them. */
    int32_t *rcount = calloc((size_t)n_workers * P, sizeof(int32_t));
    {
        const int64_t per_round = (int64_t)n_workers * rstride;
        size_t hs = 1024;
        while (hs < 2 * (size_t)(per_round ? per_round : 1)) hs <<= 1;
        uint64_t *hk = malloc(hs * sizeof(uint64_t));
        uint32_t *ids = malloc(sizeof(uint32_t) * (size_t)(per_round ? per_round : 1));
        uint8_t *keep = malloc((size_t)(per_round ? per_round : 1));
        for (int k = 0; k < P && rstride; k++) {
            memset(hk, 0, hs * sizeof(uint64_t));
            for (int64_t g = 0; g < per_round; g++) {
                uint64_t r1 = sm64(seed ^ ((uint64_t)k << 40) ^ (0x9E37ull * (uint64_t)g));
                ids[g] = (uint32_t)zipf_draw(z, (double)(r1 >> 11) * (1.0 / 9007199254740992.0));
            }
            /* peer-major over the worker-major draws: a (peer, id) pair's first occurrence wins */
            for (int r = 0; r < n_peers; r++)
                for (int w = 0; w < n_workers; w++)
                    for (int j = 0; j < per_peer; j++) {
                        int64_t g = (int64_t)w * rstride + (int64_t)r * per_peer + j;
                        uint64_t key = (((uint64_t)r << 32) | ids[g]) + 1;
                        size_t h = (size_t)(sm64(key) & (hs - 1));
                        while (hk[h] != 0 && hk[h] != key) h = (h + 1) & (hs - 1);
                        keep[g] = hk[h] == 0;
                        hk[h] = key;
                    }
            for (int w = 0; w < n_workers; w++) {
                int cnt = 0;
                for (int r = 0; r < n_peers; r++)
                    for (int j = 0; j < per_peer; j++) {
                        int64_t g = (int64_t)w * rstride + (int64_t)r * per_peer + j;
                        if (!keep[g]) continue;
                        uint8_t peer = (uint8_t)(1 + r);
                        size_t o = ((size_t)k * n_workers + w) * rstride + cnt++;
                        uint8_t *x = rinv_pool + o * osz, *v = rval_pool + o * 16;
                        uint64_t key = key_of(ids[g]);
                        memcpy(x, &key, 8);
                        x[8] = OPC_INV; x[9] = peer; x[10] = (uint8_t)sv; x[11] = peer;
                        memset(x + 12, 0, 6);
                        memset(x + 18, 'a' + peer, sv);
                        memcpy(v, x, 16);
                        v[8] = OPC_VAL;
                    }
                rcount[(size_t)k * n_workers + w] = cnt;
            }
        }
        free(hk); free(ids); free(keep);
    }
    pthread_barrier_t start;
    pthread_barrier_init(&start, NULL, (unsigned)n_threads + 1);
    bench_thread *th = calloc((size_t)n_threads, sizeof(bench_thread));
    pthread_t *thr = calloc((size_t)n_threads, sizeof(pthread_t));
    double t0 = 0;
    for (int k = 0; k < n_threads; k++) {
        bench_thread *b = &th[k];
        b->kv = kv; b->osz = osz; b->sv = sv; b->n_peers = n_peers; b->per_peer = per_peer; b->rstride = rstride;
        b->refill_all = refill_flags & 1; b->ts_reset = (refill_flags & 2) != 0; b->coalesce = (refill_flags & 4) != 0;
        b->mid = mid; b->ops = ops; b->hot = hot; b->tkey = tkey; b->top = top; b->tid = tid; b->cursor = cursor;
        b->rinv_pool = rinv_pool; b->rval_pool = rval_pool; b->rcount = rcount; b->n_workers = n_workers;
        b->w0 = (int)((int64_t)n_workers * k / n_threads);
        b->w1 = (int)((int64_t)n_workers * (k + 1) / n_threads);
        b->seconds = seconds; b->start = &start; b->t0 = &t0;
        pthread_create(&thr[k], NULL, bench_worker, b);
    }
    t0 = now_s();
    pthread_barrier_wait(&start);
    int64_t committed = 0, rounds = -1;
    double t_end = t0;
    for (int k = 0; k < n_threads; k++) {
        pthread_join(thr[k], NULL);
        committed += th[k].committed;
        if (rounds < 0 || th[k].rounds < rounds) rounds = th[k].rounds;
        if (th[k].t_end > t_end) t_end = th[k].t_end;
    }
    pthread_barrier_destroy(&start);
    *out_rounds = rounds;
    *out_secs = t_end - t0;
    free(th); free(thr);
    free(ops); free(rinv_pool); free(rval_pool); free(tkey); free(top); free(tid); free(hot); free(cursor); free(rcount);
    return committed;
}
