// hkv_runtime.hip -- host runtime and C ABI of libhermeskv.so (include/hermeskv.h).
//
// Owns the HBM image of one MICA-herd table per hkv_table (index buckets + circular log,
// mica.h:62-91, byte layout identical to the reference), the per-launch scratch (sort keys,
// temp storage), and a HIP stream. The reference entry points run on a process-wide default
// table and block until the batch is applied, like the reference's synchronous C call.
#include <hip/hip_runtime.h>
#include <csetjmp>
#include <csignal>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sched.h>
#include <unistd.h>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <vector>
#include <string>

#define HKV_IMPLEMENTATION 1
#include "../../include/hermeskv.h"
#include "hkv_internal.h"

using namespace hkv;

// ---- combining submit for the host-pointer entry point
// The reference's worker threads call hermes_batch_ops_to_KVS concurrently on one table; its
// per-key seqlocks make the result some serial order of their batches (concur_ctrl.h:144-224,
// main.c:193-210). Here every caller queues its batch; whichever caller finds no combiner active
// becomes one: it takes the compatible batches at the head of the queue (same type, element size
// and membership), stages them into one of kHostSets pinned/device buffer sets, and enqueues the
// copy in, ONE multi-batch launch (hkv_batch_async, concatenation order) and the copy out on the
// table's stream. Each caller then waits for its set's event and copies its own results out.
// Launches on one stream run in order, so the combined result is the serial order of the sets'
// concatenations -- an order the reference could have produced. With several sets, the next
// combiner stages while the GPU runs the previous launch.
//
// Partitioned launches (64-B entries, the common case): each caller first stages its own batch in
// a pinned buffer of its thread, partition-major by key (part_of, hkv_internal.h), so the combiner
// copies nothing -- it writes one 48-byte header per batch and launches k_hpart, whose kPartG
// workgroups each own a partition of the keys and read their elements straight from the callers'
// buffers. A launch's latency is then that of one partition, whatever it combines. Batches that
// overflow a partition (one key hammered by more than kPartCap elements) and big objects take the
// single-workgroup kernel (k_small) or the multi-kernel engine as before.
constexpr int kHostSets = 4;
constexpr int kHostMaxBatches = 64;
constexpr int64_t kHostMaxElems = 32768;

enum { kModeEvent = 0, kModeSmall = 1, kModePart = 2 };

struct HostSet {
    uint8_t *h = nullptr;    // pinned, coherent: counts | node_suspected | ops | rw (or the part table)
    uint8_t *hd = nullptr;   // the same bytes as the device sees them
    uint8_t *d = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    uint32_t *flag = nullptr;   // pinned: k_small stores `seq` when its results are in h (flag[0]),
    uint32_t *flag_d = nullptr; // k_hpart's workgroup g into flag[g]
    uint32_t seq = 0;
    int mode = kModeEvent;   // how this launch signals completion
    int refs = 0;            // callers still to copy their results out
    bool busy = false;
};

// a caller thread's pinned staging for partitioned launches: elements | u16 positions | rw copy
struct CallerStage {
    uint8_t *h = nullptr, *d = nullptr;
    size_t cap = 0;
    // HKV_STAGE_VRAM=1: elements and positions written by the caller's CPU straight into
    // fine-grained device memory (through the BAR), so k_hpart reads them from HBM instead of over
    // PCIe; the results still come back to the pinned buffer h
    uint8_t *v = nullptr;
    size_t vcap = 0;
    bool vram_failed = false;     // its device buffer could not be allocated: pinned staging from then on
    std::vector<uint8_t> tmp;
    std::vector<uint32_t> perm;   // element i of the caller's batch sits at staged slot perm[i]
    // a caller returns only after its launch's flags arrived, so nothing reads the staging when its
    // thread exits. hipFree / hipHostFree synchronise the device, and the serving kernel may be busy
    // with other callers' launches for up to its lifetime limit: an exiting thread hands its buffers
    // to a process-wide list, freed at the next quiet point (hkv_sync with no serving kernel of any table
    // running, or hkv_table_destroy), so thread churn does not pile up pinned memory
    ~CallerStage();
};
static std::mutex g_stage_gy_mu;
static std::vector<std::pair<uint8_t *, bool>> g_stage_graveyard;   // (buffer, is device memory)
CallerStage::~CallerStage()
{
    std::lock_guard<std::mutex> g(g_stage_gy_mu);
    if (h) g_stage_graveyard.emplace_back(h, false);
    if (v) g_stage_graveyard.emplace_back(v, true);
}
static void free_stage_graveyard()
{
    std::vector<std::pair<uint8_t *, bool>> gy;
    {
        std::lock_guard<std::mutex> g(g_stage_gy_mu);
        gy.swap(g_stage_graveyard);
    }
    for (auto &b : gy) (void)(b.second ? hipFree(b.first) : hipHostFree(b.first));
}
static thread_local CallerStage t_stage;

struct HostReq {
    int type;
    uint8_t *ops;
    int n;
    uint16_t esz;
    uint64_t mb;
    int *ns;
    uint8_t *rw;
    HostSet *set = nullptr;
    size_t ops_off = 0, rw_off = 0, ns_off = 0, rw_bytes = 0;
    std::atomic<bool> launched{false};
    // partitioned: staged in the caller's t_stage (device addresses), partition g at [poff[g], poff[g+1])
    bool part = false;
    uint32_t pseq = 0;     // launched as partitioned launch pseq (0: in a set's launch)
    uint64_t st_elems = 0, st_pos = 0, st_rw = 0, st_out = 0, st_rwo = 0;
    uint16_t poff[kPartG + 1];
};

struct hkv_table {
    hkv_config cfg;
    Geometry geo;
    hipStream_t stream = nullptr;
    uint8_t *d_index = nullptr;
    uint8_t *d_log = nullptr;
    unsigned long long *d_evictions = nullptr;
    int64_t inserted = 0;
    uint32_t skip_key = 0;
    int key_bits = 0;
    // batch scratch (batch_carve)
    uint8_t *d_batch = nullptr;
    int64_t batch_cap = 0;
    unsigned long long *d_fw = nullptr;  // F words, one per 64-B log line (+ INV words X, Y, ACK words T)
    uint32_t epoch = 0;                // batch launches since d_fw was all-ones
    uint32_t scratch_gen = 0;          // d_batch reallocations
    // a local launch's prepass (HKV_BATCH_PREPASS) waiting for the rest of its launch
    struct {
        bool valid = false, done = false;
        uint32_t epoch = 0, scratch_gen = 0;
        int64_t n = 0;
        const uint8_t *elems = nullptr;
    } pre;
    unsigned int *d_error_flags = nullptr;
    int32_t *d_ns_idx = nullptr;
    int32_t ns_cap = 0;
    // the host-pointer reference API: concurrent callers' batches are combined into one launch
    // (see "combining submit" below)
    std::mutex hmu;
    std::condition_variable hcv;
    std::deque<HostReq *> hq;
    std::atomic<bool> combining{false};
    HostSet sets[kHostSets];
    // partitioned launches: workgroup g of launch n stores n into pflags[g] (pinned; launches run in
    // stream order, so each word only grows); pseq counts the launches
    uint32_t *pflags = nullptr, *pflags_d = nullptr;
    uint32_t pseq = 0;
    // the serving kernel (k_hserve): launches are published in a pinned ring instead of launched
    HostRingSlot *ring = nullptr, *ring_d = nullptr;
    uint32_t *srv_words = nullptr, *srv_words_d = nullptr;   // [0] stop, [32..63] exited per workgroup
    // with callers staging in device memory (HKV_STAGE_VRAM), the ring and the stop word live there
    // too: the serving kernel polls HBM instead of reading host memory over PCIe every iteration
    uint32_t *srv_stop = nullptr, *srv_stop_d = nullptr;
    bool ring_vram = false;
    uint32_t srv_epoch = 0;
    bool srv_running = false;
    hipEvent_t srv_ev = nullptr;
    std::mutex mu;
};

static void srv_stop(hkv_table *t);   // the serving kernel (see "combining submit") stopped
static bool stage_vram_usable();
static std::mutex g_srv_mu;                      // tables whose serving kernel was started (srv_atexit)
static std::vector<hkv_table *> g_srv_tables;
// the serving kernel's stop word (device memory: write-combined, so flushed at once)
static void srv_set_stop(hkv_table *t, uint32_t v)
{
    __atomic_store_n(t->srv_stop, v, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
}

static thread_local std::string g_err;
static const bool g_trace = getenv("HKV_TRACE") != nullptr;
#define TRACE(...)                                       \
    do {                                                 \
        if (g_trace) {                                   \
            fprintf(stderr, "[hkv] " __VA_ARGS__);       \
            fputc('\n', stderr);                         \
        }                                                \
    } while (0)
static std::mutex g_default_mu;
static hkv_table *g_default = nullptr;
static bool g_default_cfg_set = false;
static hkv_config g_default_cfg;

extern "C" {
// reference global `struct spacetime_kv kv` (spacetime.c:15): callers only take its address
struct spacetime_kv {
    void *handle;
    uint8_t pad[120];
} kv;
}

static int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) return fail(-5, "%s: %s", #expr, hipGetErrorString(e_));     \
    } while (0)

static bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

static hkv_config reference_defaults()
{
    hkv_config c;
    memset(&c, 0, sizeof c);
    c.abi_version = HKV_ABI_VERSION;
    c.machine_id = 0;
    c.rw_len = 250;                       // MAX_BATCH_KVS_OPS_SIZE, config.h:42
    c.num_keys = 1000 * 1000;             // SPACETIME_NUM_KEYS, spacetime.h:21
    c.num_bkts = 2 * 1024 * 1024;         // SPACETIME_NUM_BKTS, spacetime.h:22
    c.log_cap = 1024ull * 1024 * 1024;    // SPACETIME_LOG_CAP, spacetime.h:23
    return c;
}

static void make_geometry(const hkv_config &c, Geometry &g)
{
    uint32_t kvs_value = c.big_objects ? c.extra_cache_lines * 64u + 46u : 46u;  // hrd.h:47
    g.bkt_mask = c.num_bkts - 1;
    g.log_cap = c.log_cap;
    g.log_mask = c.log_cap - 1;
    g.log_head = 0;
    g.kvs_value = kvs_value;
    g.st_value = kvs_value - kObjMetaSize;
    g.entry_size = (kEntryMetaOff + kvs_value + 7u) & ~7u;
    g.shift = c.big_objects ? 3u : 0u;
    g.op_size = (kOpMetaSize + 2u + g.st_value + 7u) & ~7u;
    // entries start at multiples of entry_size from offset 0, modulo the power-of-two capacity: so
    // every offset is a multiple of the largest power of two dividing entry_size (64 for 320-B
    // entries), which keeps 32-bit entry ids valid up to 256 GiB of log
    const uint32_t low = g.entry_size & (~g.entry_size + 1u);
    g.entry_unit = (c.log_cap % g.entry_size == 0) ? g.entry_size : (low > 8u ? low : 8u);
    g.rmw_enabled = c.rmw_enabled ? 1u : 0u;
    g.machine_id = c.machine_id;
    g.skew = c.skew_flags & (kSkewReadComplete | kSkewWriteCoalesce);
}

static int bit_width(uint64_t x)
{
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

static int ensure_batch_scratch(hkv_table *t, int64_t n)
{
    if (!t->d_fw) {
        // F words, the INV words X and Y (batch_fw_words each), then the ACK words T (eight
        // epoch-tagged u64 per line), see hkv_batch.hip
        const size_t bytes = 8 * batch_fw_words(t->cfg.log_cap);
        HIP_TRY(hipMalloc(&t->d_fw, 11 * bytes));
        // F all-ones: every F word reads as stale for every epoch; X and Y zero (they are cleared
        // by the launch that sets them), T zero (older epochs read as empty). hipMemset runs on
        // the null stream, which does not order the table's non-blocking streams: wait for it here.
        HIP_TRY(hipMemset(t->d_fw, 0xFF, bytes));
        HIP_TRY(hipMemset(reinterpret_cast<uint8_t *>(t->d_fw) + bytes, 0, 10 * bytes));
        HIP_TRY(hipDeviceSynchronize());
        t->epoch = 0;
    }
    if (n <= t->batch_cap) return 0;
    const int64_t cap = n + n / 4 + 1024;
    hipFree(t->d_batch);
    t->d_batch = nullptr;
    t->batch_cap = 0;
    HIP_TRY(hipMalloc(&t->d_batch, batch_scratch_bytes(cap, t->geo.entry_size)));
    t->batch_cap = cap;
    ++t->scratch_gen;
    return 0;
}

// Virtual log offsets of a run of inserts (mica_insert_one, mica.c:119-145): the head advances
// by one entry per insert and wraps once, when fewer than MICA_MAX_VALUE + 32 bytes remain;
// after that the unsigned "remaining" test underflows and the head never wraps again.
static void plan_log(uint64_t h0, uint64_t cap, uint32_t e, uint32_t maxv, uint64_t n,
                     uint64_t &k, uint64_t &hw, uint64_t &final_head)
{
    const uint64_t T = (uint64_t)maxv + 32, mask = cap - 1;
    k = UINT64_MAX;
    hw = 0;
    if (h0 <= cap) {
        uint64_t lo = cap > T ? cap - T : 0;
        uint64_t kk = (h0 + e >= lo) ? 1 : (lo - h0 + e - 1) / e;
        if (h0 + kk * e <= cap) {
            k = kk;
            hw = (h0 + kk * e + cap) & ~mask;
        }
    }
    final_head = (n < k) ? h0 + n * e : hw + (n - k) * e;
}

namespace hkv {
int table_view(const hkv_table *t, TableView *out)
{
    if (!t || !out) return -1;
    out->g = t->geo;
    out->index = t->d_index;
    out->log = t->d_log;
    return 0;
}
}  // namespace hkv

extern "C" {

int hkv_abi_version(void) { return HKV_ABI_VERSION; }

int hkv_debug_modes(void)
{
#ifdef HKV_DEBUG_MODES
    return 1;
#else
    return 0;
#endif
}

const char *hkv_last_error(void) { return g_err.c_str(); }

int hkv_table_create(const hkv_config *cfg, hkv_table **out)
{
    if (!cfg || !out) return fail(-1, "null argument");
    if (cfg->abi_version != HKV_ABI_VERSION) return fail(-1, "abi_version %u != %d", cfg->abi_version, HKV_ABI_VERSION);
    if (!is_pow2(cfg->num_bkts) || cfg->num_bkts > (1ull << 31)) return fail(-1, "num_bkts must be a power of two <= 2^31");
    if (!is_pow2(cfg->log_cap) || cfg->log_cap < 4096) return fail(-1, "log_cap must be a power of two >= 4096");
    if (cfg->machine_id > 127) return fail(-1, "machine_id must be < 128");
    if (cfg->skew_flags & ~(HKV_SKEW_READ_COMPLETE | HKV_SKEW_WRITE_COALESCE))
        return fail(-1, "unknown skew_flags %#x", cfg->skew_flags);
    // 287 + 64 k value bytes in (k + 1) cache lines: val_len >> SHIFT_BITS must fit its byte and
    // the batch engine stages 128 entries of a launch in one workgroup's LDS
    if (cfg->big_objects && (cfg->extra_cache_lines < 1 || cfg->extra_cache_lines > 16))
        return fail(-1, "extra_cache_lines must be 1..16 with big objects");
    hkv_table *t = new hkv_table();
    t->cfg = *cfg;
    if (t->cfg.rw_len == 0) t->cfg.rw_len = 250;
    make_geometry(t->cfg, t->geo);
    uint64_t slots = t->geo.log_cap / t->geo.entry_unit;
    if (slots >= 0xFFFFFFFFull) {
        delete t;
        return fail(-1, "log too large for 32-bit entry ids");
    }
    t->skip_key = (uint32_t)slots;
    t->key_bits = bit_width(slots);
    int rc = 0;
    do {
        if (hipSetDevice(cfg->device) != hipSuccess) { rc = fail(-5, "hipSetDevice(%d) failed", cfg->device); break; }
        if (hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess) { rc = fail(-5, "stream"); break; }
        if (hipMalloc(&t->d_index, t->cfg.num_bkts * 64) != hipSuccess) { rc = fail(-6, "index alloc %llu B", (unsigned long long)(t->cfg.num_bkts * 64)); break; }
        if (hipMalloc(&t->d_log, t->cfg.log_cap + t->geo.entry_size) != hipSuccess) { rc = fail(-6, "log alloc %llu B", (unsigned long long)t->cfg.log_cap); break; }
        if (hipMalloc(&t->d_evictions, sizeof(unsigned long long)) != hipSuccess) { rc = fail(-6, "alloc"); break; }
        if (hipMalloc(&t->d_error_flags, sizeof(unsigned int)) != hipSuccess) { rc = fail(-6, "alloc"); break; }
        if (hipMemsetAsync(t->d_error_flags, 0, sizeof(unsigned int), t->stream) != hipSuccess) { rc = fail(-5, "memset"); break; }
        if (hipMemsetAsync(t->d_index, 0, t->cfg.num_bkts * 64, t->stream) != hipSuccess) { rc = fail(-5, "memset"); break; }
        if (hipMemsetAsync(t->d_log, 0, t->cfg.log_cap + t->geo.entry_size, t->stream) != hipSuccess) { rc = fail(-5, "memset"); break; }
        if (hipMemsetAsync(t->d_evictions, 0, sizeof(unsigned long long), t->stream) != hipSuccess) { rc = fail(-5, "memset"); break; }
        if (hipStreamSynchronize(t->stream) != hipSuccess) { rc = fail(-5, "sync"); break; }
    } while (0);
    if (rc) {
        hkv_table_destroy(t);
        return rc;
    }
    // whether callers can stage in device memory (a guarded store through the BAR) is probed once,
    // here on the creating thread, before any caller thread exists: its signal handlers are swapped
    // only while no other thread of the library runs
    (void)stage_vram_usable();
    *out = t;
    return 0;
}


int hkv_table_destroy(hkv_table *t)
{
    if (!t) return 0;
    if (t->stream) hipStreamSynchronize(t->stream);
    hipFree(t->d_index);
    hipFree(t->d_log);
    hipFree(t->d_evictions);
    hipFree(t->d_batch);
    hipFree(t->d_fw);
    hipFree(t->d_error_flags);
    hipFree(t->d_ns_idx);
    for (HostSet &hs : t->sets) {
        hipFree(hs.d);
        hipHostFree(hs.h);
        hipHostFree(hs.flag);
        if (hs.ev) hipEventDestroy(hs.ev);
    }
    if (t->srv_running) {
        srv_set_stop(t, 1u);
        hipEventSynchronize(t->srv_ev);
    }
    {
        std::lock_guard<std::mutex> lk(g_srv_mu);
        g_srv_tables.erase(std::remove(g_srv_tables.begin(), g_srv_tables.end(), t), g_srv_tables.end());
    }
    if (t->srv_ev) hipEventDestroy(t->srv_ev);
    free_stage_graveyard();   // staging buffers of caller threads that have exited
    if (t->ring) (void)(t->ring_vram ? hipFree(t->ring) : hipHostFree(t->ring));
    if (t->ring_vram && t->srv_stop) (void)hipFree(t->srv_stop);
    if (t->srv_words) hipHostFree(t->srv_words);
    if (t->pflags) hipHostFree(t->pflags);
    if (t->stream) hipStreamDestroy(t->stream);
    delete t;
    return 0;
}

int hkv_table_config(const hkv_table *t, hkv_config *out)
{
    if (!t || !out) return fail(-1, "null argument");
    *out = t->cfg;
    return 0;
}

int hkv_table_set_skew(hkv_table *t, uint32_t skew_flags)
{
    if (!t) return fail(-1, "null table");
    if (skew_flags & ~(HKV_SKEW_READ_COMPLETE | HKV_SKEW_WRITE_COALESCE)) return fail(-1, "unknown skew_flags %#x", skew_flags);
    srv_stop(t);   // it holds the geometry it was started with
    std::lock_guard<std::mutex> lk(t->mu);
    t->cfg.skew_flags = skew_flags;
    t->geo.skew = skew_flags;
    return 0;
}

int hkv_table_populate(hkv_table *t, int64_t n, int val_len)
{
    if (!t) return fail(-1, "null table");
    if (n <= 0) return fail(-1, "populate: n must be > 0");
    if (val_len <= 0 || (uint32_t)val_len > t->geo.kvs_value) return fail(-1, "populate: bad val_len %d", val_len);
    srv_stop(t);
    if (n > 0x7FFFFFFFll) return fail(-1, "populate: at most 2^31-1 keys (32-bit key ids)");
    std::lock_guard<std::mutex> lk(t->mu);
    HIP_TRY(hipSetDevice(t->cfg.device));
    int bbits = bit_width(t->cfg.num_bkts - 1);
    if (bbits == 0) bbits = 1;
    // populate temporaries: hashes, sort pairs and sort storage, freed before returning
    uint64_t *d_first = nullptr, *d_second = nullptr;
    uint32_t *d_pairs = nullptr;
    void *d_tmp = nullptr;
    const size_t tmp_bytes = sort_temp_bytes(n, bbits);
    auto release = [&]() {
        hipFree(d_first);
        hipFree(d_second);
        hipFree(d_pairs);
        hipFree(d_tmp);
    };
    if (hipMalloc(&d_first, n * 8) != hipSuccess || hipMalloc(&d_second, n * 8) != hipSuccess ||
        hipMalloc(&d_pairs, n * 16) != hipSuccess || hipMalloc(&d_tmp, tmp_bytes) != hipSuccess) {
        release();
        return fail(-6, "populate: temporary allocation of %lld keys failed", (long long)n);
    }
    PopulateLaunch pl;
    memset(&pl, 0, sizeof pl);
    pl.first = d_first;
    pl.second = d_second;
    pl.keys_a = d_pairs;
    pl.keys_b = d_pairs + n;
    pl.vals_a = d_pairs + 2 * n;
    pl.vals_b = d_pairs + 3 * n;
    pl.sort_tmp = d_tmp;
    pl.sort_tmp_bytes = tmp_bytes;
    pl.index = t->d_index;
    pl.log = t->d_log;
    pl.evictions = t->d_evictions;
    pl.n = n;
    pl.bkt_mask = t->geo.bkt_mask;
    pl.log_cap = t->geo.log_cap;
    pl.log_mask = t->geo.log_mask;
    pl.entry_size = t->geo.entry_size;
    pl.key_bits = bbits;
    pl.val_len_byte = (uint8_t)(val_len >> t->geo.shift);  // spacetime.c:45
    uint64_t final_head;
    pl.h0 = t->geo.log_head;
    plan_log(t->geo.log_head, t->geo.log_cap, t->geo.entry_size, t->geo.kvs_value, (uint64_t)n, pl.k, pl.hw, final_head);
    int rc = launch_populate(pl, t->stream);
    hipError_t se = hipStreamSynchronize(t->stream);
    release();
    if (rc) return fail(rc, "populate launch failed (%d): %s", rc, hipGetErrorString(hipGetLastError()));
    if (se != hipSuccess) return fail(-5, "populate: %s", hipGetErrorString(se));
    t->geo.log_head = final_head;
    t->inserted += n;
    return 0;
}

// The element rules every launch obeys, whichever entry point it comes through: a known type,
// elements of at least 16 bytes in 8-byte units (the engines move them in 8- and 16-byte words),
// room for the value where the exec functions read or write one, and at most 255 ops per local
// batch (op_buffer_index is a uint8, 255 = empty).
static int check_elems(const hkv_table *t, int type, uint32_t elem_size, int64_t per_batch)
{
    if (type < 0 || type > 4) return fail(-1, "bad batch type %d", type);
    if (elem_size < (uint32_t)kOpMetaSize || (elem_size & 7))
        return fail(-1, "elem_size %u must be >= 16 and a multiple of 8", elem_size);
    // ACK batches of an RMW table carry INV-aborts, which hermes_exec_inv applies with their value
    // (hermesKV.c:877-890): they need op-sized elements, as the reference worker sends them
    // (hermes_worker.c:332)
    const bool needs_value = type == kLocal || type == kLocalAfterMemb || type == kInvs ||
                             (type == kAcks && t->geo.rmw_enabled);
    if (needs_value && elem_size < kOpValueOff + t->geo.st_value)
        return fail(-1, "elem_size %u too small for %u-byte values", elem_size, t->geo.st_value);
    if (type == kLocal && per_batch > 255)
        return fail(-1, "local batches hold at most 255 ops (uint8 op_buffer_index)");
    return 0;
}

int hkv_batch_async(hkv_table *t, const hkv_batch_desc *d, void *stream)
{
    if (!t || !d) return fail(-1, "null argument");
    srv_stop(t);
    const bool packed = (d->flags & HKV_BATCH_PACKED) != 0;
    if (d->n_batches < 0 || d->stride < 0 || (d->stride == 0 && !packed)) return fail(-1, "bad batch geometry");
    if (int rc = check_elems(t, d->type, d->elem_size, packed ? 0 : d->stride)) return rc;
    // HKV_BATCH_PACKED: d_counts holds n_batches + 1 element offsets and stride the total
    if (packed && d->type != kInvs && d->type != kVals && d->type != kAcks)
        return fail(-1, "HKV_BATCH_PACKED applies to INV, ACK and VAL batches");
    if (packed && !d->d_counts) return fail(-1, "HKV_BATCH_PACKED needs the batch offsets in d_counts");
    int64_t n = packed ? (int64_t)d->stride : (int64_t)d->n_batches * d->stride;
    if (n == 0 || d->n_batches == 0) return 0;
    // 16-byte aligned slabs let the LDS-staged passes move whole 16-B words; a one-pass unique launch
    // reads each element on its own (its 8-byte alignment suffices), so a peer's slab can start at
    // any element of a larger buffer
    if ((uintptr_t)d->d_elems & ((d->flags & HKV_BATCH_UNIQUE) ? 7 : 15))
        return fail(-1, "d_elems must be 16-byte aligned (8 with HKV_BATCH_UNIQUE)");
    if (n > 0x7FFFFFFFll) return fail(-1, "too many elements in one launch");
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream, as in every HIP API
    int rc = ensure_batch_scratch(t, n);
    if (rc) return rc;
    int32_t *ns_idx = nullptr;
    if (d->type == kInvs && d->d_node_suspected) {
        if (d->n_batches > t->ns_cap) {
            hipFree(t->d_ns_idx);
            t->d_ns_idx = nullptr;
            t->ns_cap = 0;
            HIP_TRY(hipMalloc(&t->d_ns_idx, (size_t)d->n_batches * 4 + 64));
            t->ns_cap = d->n_batches;
        }
        HIP_TRY(hipMemsetAsync(t->d_ns_idx, 0xFF, (size_t)d->n_batches * 4, s));
        ns_idx = t->d_ns_idx;
    }
    BatchLaunch bl;
    memset(&bl, 0, sizeof bl);
    bl.g = t->geo;
    bl.elems = d->d_elems;
    bl.counts = packed ? nullptr : d->d_counts;
    bl.state_out = d->d_state_out;
    bl.opcode_in = d->type == kLocal || d->type == kAcks ? d->d_opcode_in : nullptr;
    bl.patch = d->type == kLocal ? d->d_patch : nullptr;
    bl.rw_state = d->type == kAcks ? d->d_rw_state : nullptr;
    if (bl.patch && ((uintptr_t)bl.patch & 15)) return fail(-1, "d_patch must be 16-byte aligned");
    // reserved since ABI 8 (the PUT-key mirror, located entries and the two-stage local launch were
    // measured, not adopted, and removed): a caller that sets them gets an error, not a silent no-op
    if (d->d_put_keys || d->d_phys) return fail(-1, "d_put_keys and d_phys are reserved (must be NULL)");
    if (d->flags & HKV_BATCH_RESERVED_FLAGS) return fail(-1, "hkv_batch_desc.flags: reserved bits set");
    bl.offsets = packed ? d->d_counts : nullptr;
    bl.index = t->d_index;
    bl.log = t->d_log;
    bl.rw = d->type == kAcks ? d->d_rw : nullptr;
    bl.rw_stride = d->rw_stride_bytes;
    bl.ns_idx = ns_idx;
    bl.node_suspected = d->d_node_suspected;
    batch_carve(bl, t->d_batch, t->batch_cap, t->geo.entry_size);
    bl.fw = t->d_fw;
    bl.fx = t->d_fw + batch_fw_words(t->cfg.log_cap);
    bl.fy = bl.fx + batch_fw_words(t->cfg.log_cap);
    bl.ft = bl.fy + batch_fw_words(t->cfg.log_cap);

    if (++t->epoch > batch_max_epoch()) {  // round tags would wrap: start the F and T words over
        HIP_TRY(hipMemsetAsync(t->d_fw, 0xFF, 8 * batch_fw_words(t->cfg.log_cap), s));
        HIP_TRY(hipMemsetAsync(bl.ft, 0, 64 * batch_fw_words(t->cfg.log_cap), s));
        t->epoch = 1;
    }
    bl.epoch = t->epoch;
    bl.error_flags = t->d_error_flags;
    bl.n = n;
    bl.n_batches = d->n_batches;
    bl.stride = d->stride;
    bl.esz = d->elem_size;
    bl.type = d->type;
    bl.g_membership = d->membership[1];
    bl.w_ack_init = d->membership[2];
    bl.path = (d->flags & HKV_BATCH_ENGINE) || packed ? kPathEngine
            : (d->flags & HKV_BATCH_SMALL) ? kPathSmall : kPathAuto;
    bl.unique = (d->flags & HKV_BATCH_UNIQUE) && (d->type == kInvs || d->type == kAcks) ? 1 : 0;
    if (d->d_ack_out && d->type == kAcks) {   // the VAL callbacks, by the ACK rows launch
        if (!(d->flags & HKV_BATCH_ROWS) || !bl.unique || d->elem_size != 16 || d->ack_out_size != 16 ||
            t->geo.entry_size != 64 || t->geo.st_value != 31 || ((uintptr_t)d->d_ack_out & 15))
            return fail(-1, "d_ack_out on an ACK launch: HKV_BATCH_ROWS unique launches of 16-byte ACKs and 64-byte "
                            "entries, 16-byte VALs, 16-byte aligned");
        bl.ack_out = d->d_ack_out;
        bl.ack_out_size = d->ack_out_size;
    } else if (d->d_ack_out) {
        const bool small_geo = t->geo.entry_size == 64 && t->geo.st_value == 31 && d->elem_size <= 64;
        const bool big_geo = t->geo.entry_size == 320 && t->geo.st_value == 287 && d->elem_size <= 320;
        if (d->type != kInvs || !bl.unique || d->n_rows > 1 || !(small_geo || big_geo) || d->ack_out_size < 16 ||
            (d->ack_out_size & 7) || ((uintptr_t)d->d_ack_out & 7))
            return fail(-1, "d_ack_out: unique INV launches of 64-byte entries and elements (or 320-byte big "
                            "objects), 16-byte ACKs or larger");
        bl.ack_out = d->d_ack_out;
        bl.ack_out_size = d->ack_out_size;
        bl.path = kPathEngine;
    }
    if (d->flags & HKV_BATCH_ROWS) {
        if (!bl.unique || t->geo.entry_size != 64 || t->geo.st_value != 31 || d->elem_size > 64)
            return fail(-1, "HKV_BATCH_ROWS: unique INV or ACK launches of 64-byte entries and elements only");
        if (d->n_rows < 1 || d->n_rows > HKV_MAX_ROWS || d->skip_row >= d->n_rows || d->d_node_suspected)
            return fail(-1, "HKV_BATCH_ROWS: 1..%d rows, a skip row among them (or -1), no node_suspected",
                        HKV_MAX_ROWS);
        if (d->n_rows > 1 && d->row_stride < n) return fail(-1, "HKV_BATCH_ROWS: rows overlap");
        bl.n_rows = d->n_rows;
        bl.skip_row = d->skip_row < 0 ? -1 : d->skip_row;
        bl.row_stride = d->row_stride;
        bl.path = kPathEngine;
    }
    TRACE("batch_async type=%d n=%lld", d->type, (long long)n);
    rc = launch_batch(bl, s);
    if (rc) return fail(rc, "batch launch failed (%d): %s", rc, hipGetErrorString(hipGetLastError()));
    return 0;
}

// The staging buffers of exited caller threads, freed when no table's serving kernel runs: hipFree waits for
// the device, and a persistent serving kernel may run for up to its 1-s lifetime (a server that starts after
// the check only makes the free wait, as at table destruction)
static bool srv_exited(const hkv_table *t);
static void free_stage_graveyard_if_quiet()
{
    {
        std::lock_guard<std::mutex> g(g_stage_gy_mu);
        if (g_stage_graveyard.empty()) return;
    }
    {
        std::lock_guard<std::mutex> lk(g_srv_mu);
        for (hkv_table *u : g_srv_tables)
            if (__atomic_load_n(&u->srv_running, __ATOMIC_ACQUIRE) && !srv_exited(u)) return;
    }
    free_stage_graveyard();
}

int hkv_sync(hkv_table *t, void *stream)
{
    if (!t) return fail(-1, "null table");
    srv_stop(t);
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize(t->stream));
    free_stage_graveyard_if_quiet();
    return 0;
}

int hkv_copy_index(hkv_table *t, void *dst, uint64_t off, uint64_t bytes)
{
    if (!t || !dst) return fail(-1, "null argument");
    if (off + bytes > t->cfg.num_bkts * 64) return fail(-1, "index range out of bounds");
    srv_stop(t);
    HIP_TRY(hipStreamSynchronize(t->stream));
    HIP_TRY(hipMemcpy(dst, t->d_index + off, bytes, hipMemcpyDeviceToHost));
    return 0;
}

int hkv_copy_log(hkv_table *t, void *dst, uint64_t off, uint64_t bytes)
{
    if (!t || !dst) return fail(-1, "null argument");
    if (off + bytes > t->cfg.log_cap + t->geo.entry_size) return fail(-1, "log range out of bounds");
    srv_stop(t);
    HIP_TRY(hipStreamSynchronize(t->stream));
    HIP_TRY(hipMemcpy(dst, t->d_log + off, bytes, hipMemcpyDeviceToHost));
    return 0;
}

uint64_t hkv_log_head(const hkv_table *t) { return t ? t->geo.log_head : 0; }

int64_t hkv_num_index_evictions(const hkv_table *t)
{
    if (!t) return -1;
    unsigned long long v = 0;
    if (hipMemcpy(&v, t->d_evictions, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (int64_t)v;
}

void *hkv_device_index(hkv_table *t) { return t ? t->d_index : nullptr; }

int hkv_take_error_flags(hkv_table *t, uint32_t *out)
{
    if (!t || !out) return fail(-1, "null argument");
    srv_stop(t);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, t->d_error_flags, sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(t->d_error_flags, 0, sizeof(uint32_t)));
    HIP_TRY(hipDeviceSynchronize());  // null-stream memset vs the non-blocking launch streams
    return 0;
}
void *hkv_device_log(hkv_table *t) { return t ? t->d_log : nullptr; }

int hkv_hash_ids(const uint32_t *d_ids, uint64_t *d_keys_second, int64_t n, void *stream)
{
    if (launch_hash_ids(d_ids, d_keys_second, n, (hipStream_t)stream)) return fail(-5, "hash launch failed");
    return 0;
}

int hkv_set_default_config(const hkv_config *cfg)
{
    std::lock_guard<std::mutex> lk(g_default_mu);
    if (g_default) return fail(-1, "default table already exists");
    g_default_cfg = *cfg;
    g_default_cfg_set = true;
    return 0;
}

hkv_table *hkv_default_table(void) { return g_default; }

// ------------------------------------------------------------------ reference entry points
[[noreturn]] static void die(const char *where)
{
    fprintf(stderr, "libhermeskv: %s: %s\n", where, g_err.c_str());
    abort();
}

static hkv_table *default_table_locked(int instance_id)
{
    if (!g_default) {
        hkv_config c = g_default_cfg_set ? g_default_cfg : reference_defaults();
        if (!g_default_cfg_set && instance_id >= 0) c.machine_id = (uint32_t)instance_id;
        if (hkv_table_create(&c, &g_default)) die("table create");
        kv.handle = g_default;
    }
    return g_default;
}

void spacetime_init(int instance_id)
{
    std::lock_guard<std::mutex> lk(g_default_mu);
    hkv_table *t = default_table_locked(instance_id);
    if (hkv_table_populate(t, (int64_t)t->cfg.num_keys, (int)t->geo.kvs_value)) die("spacetime_init populate");
}

void spacetime_populate_fixed_len(struct spacetime_kv *, int n, int val_len)
{
    std::lock_guard<std::mutex> lk(g_default_mu);
    hkv_table *t = default_table_locked(-1);
    if (hkv_table_populate(t, n, val_len)) die("spacetime_populate_fixed_len");
}

// HKV_HOST_STATS=1: launches and batches per launch of the combining submit, printed at exit
static const bool g_host_stats = getenv("HKV_HOST_STATS") != nullptr;
static std::atomic<long> g_hs_launches{0}, g_hs_batches{0};
static void host_stats_print()
{
    const long l = g_hs_launches.load(), b = g_hs_batches.load();
    fprintf(stderr, "[hkv] host submit: %ld launches, %ld batches, %.2f batches/launch\n", l, b, l ? (double)b / l : 0.0);
}
static void host_stats_note(int nb)
{
    static std::once_flag once;
    std::call_once(once, [] { atexit(host_stats_print); });
    g_hs_launches++;
    g_hs_batches += nb;
}


// HKV_HOST_TIMING=1: where a host-pointer call's time goes (staging, queue + launch + GPU, copy-out),
// averaged over the calls and printed at exit
static const bool g_host_timing = getenv("HKV_HOST_TIMING") != nullptr;
static std::atomic<long> g_ht_calls{0}, g_ht_stage{0}, g_ht_wait{0}, g_ht_out{0};
static std::atomic<long> g_hc_n{0}, g_hc_inflight{0}, g_hc_take{0}, g_hc_publish{0}, g_hc_flagwait{0};
static void host_timing_print()
{
    const long n = std::max(1L, g_ht_calls.load()), m = std::max(1L, g_hc_n.load());
    fprintf(stderr, "[hkv] host call timing (us, avg of %ld): stage %.2f wait %.2f (flags %.2f) copy-out %.2f\n", n,
            g_ht_stage.load() / 1e3 / n, g_ht_wait.load() / 1e3 / n, g_hc_flagwait.load() / 1e3 / n, g_ht_out.load() / 1e3 / n);
    fprintf(stderr, "[hkv] combiner (us, avg of %ld launches): in-flight wait %.2f take %.2f publish %.2f\n", m,
            g_hc_inflight.load() / 1e3 / m, g_hc_take.load() / 1e3 / m, g_hc_publish.load() / 1e3 / m);
}
static long now_ns()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000000000L + ts.tv_nsec;
}

static bool host_compatible(const HostReq *a, const HostReq *b)
{
    return a->type == b->type && a->esz == b->esz && a->mb == b->mb && (a->rw != nullptr) == (b->rw != nullptr) &&
           (a->ns != nullptr) == (b->ns != nullptr);
}

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// (re)allocates a staging set for `total` bytes: pinned coherent host memory the kernel reads and
// writes directly, and the device region it works in
static void host_set_reserve(HostSet *set, size_t total)
{
    if (total > set->cap) {
        hipFree(set->d);
        hipHostFree(set->h);
        set->d = set->h = set->hd = nullptr;
        const size_t cap = std::max(total + total / 2, (size_t)1 << 20);
        if (hipMalloc(&set->d, cap) != hipSuccess ||
            hipHostMalloc((void **)&set->h, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&set->hd, set->h, 0) != hipSuccess)
            die("staging alloc");
        set->cap = cap;
    }
    if (!set->ev && hipEventCreateWithFlags(&set->ev, hipEventDisableTiming) != hipSuccess) die("event");
    if (!set->flag) {
        if (hipHostMalloc((void **)&set->flag, 4 * kPartG, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&set->flag_d, set->flag, 0) != hipSuccess)
            die("flag alloc");
        for (int g = 0; g < kPartG; ++g) __atomic_store_n(set->flag + g, 0u, __ATOMIC_RELEASE);
    }
}

// The queued batches (any type, in queue order, as many as fit kSmallMaxElems elements and
// kSmallMaxBatches batches) as ONE mixed launch of the single-workgroup kernel: the region holds
// the batch headers, each batch's elements, each ACK batch's read_write_ops and each INV batch's
// node_suspected; the kernel copies it in, applies the batches in order, copies it back and
// stores the set's sequence number into set->flag. Called with t->hmu held.
static void host_launch_mixed(hkv_table *t, HostSet *set, std::unique_lock<std::mutex> &lk)
{
    std::vector<HostReq *> take;
    int64_t elems = 0;
    for (auto it = t->hq.begin(); it != t->hq.end() && (int)take.size() < kSmallMaxBatches;) {
        HostReq *r = *it;
        if (elems + r->n > kSmallMaxElems) {
            ++it;
            continue;
        }
        elems += r->n;
        take.push_back(r);
        it = t->hq.erase(it);
    }
    lk.unlock();
    const int nb = (int)take.size();
    const size_t rw_bytes = (size_t)t->cfg.rw_len * t->geo.op_size;
    size_t off = align16(sizeof(SmallBatch) * (size_t)nb);
    for (HostReq *r : take) {
        r->ops_off = off;
        off = align16(off + (size_t)r->n * r->esz);
    }
    for (HostReq *r : take) {
        r->rw_bytes = r->type == acks && r->rw ? rw_bytes : 0;
        r->rw_off = off;
        off = align16(off + r->rw_bytes);
        r->ns_off = off;
        if (r->type == invs && r->ns) off += 4;
    }
    const size_t total = align16(off);
    host_set_reserve(set, total);
    SmallBatch *hdr = reinterpret_cast<SmallBatch *>(set->h);
    for (int b = 0; b < nb; ++b) {
        HostReq *r = take[b];
        SmallBatch &h = hdr[b];
        memset(&h, 0, sizeof h);
        h.type = r->type;
        h.count = r->n;
        h.esz = r->esz;
        h.elem_off = (int32_t)r->ops_off;
        h.rw_off = r->rw_bytes ? (int32_t)r->rw_off : -1;
        h.ns_off = r->type == invs && r->ns ? (int32_t)r->ns_off : -1;
        h.g_membership = (uint8_t)(r->mb >> 8);
        h.w_ack_init = (uint8_t)(r->mb >> 16);
        memcpy(set->h + r->ops_off, r->ops, (size_t)r->n * r->esz);
        if (r->rw_bytes) memcpy(set->h + r->rw_off, r->rw, r->rw_bytes);
        if (h.ns_off >= 0) memcpy(set->h + r->ns_off, r->ns, 4);
    }
    BatchLaunch bl;
    memset(&bl, 0, sizeof bl);
    bl.g = t->geo;
    bl.index = t->d_index;
    bl.log = t->d_log;
    bl.error_flags = t->d_error_flags;
    bl.n = elems;
    bl.n_batches = nb;
    bl.stride = 1;
    bl.esz = 16;
    bl.type = take[0]->type;
    bl.g_membership = hdr[0].g_membership;
    bl.w_ack_init = hdr[0].w_ack_init;
    bl.path = kPathSmall;
    bl.host_src = set->hd;
    bl.host_dst = set->hd;
    bl.dev_region = set->d;
    bl.region_bytes = total;
    bl.done_flag = set->flag_d;
    bl.done_value = ++set->seq;
    bl.hdr = reinterpret_cast<const SmallBatch *>(set->d);
    set->mode = kModeSmall;
    if (g_host_stats) host_stats_note(nb);
    TRACE("mixed launch batches=%d elements=%lld", nb, (long long)elems);
    if (elems == 0) {
        // nothing to apply (callers never queue empty batches; kept as a guard): no kernel would
        // store the completion flag, so the host does
        __atomic_store_n(set->flag, bl.done_value, __ATOMIC_RELEASE);
    } else {
        // t->mu orders the launch against hkv_table_populate, which moves geo.log_head
        std::lock_guard<std::mutex> tl(t->mu);
        bl.g = t->geo;
        if (launch_batch(bl, t->stream)) die("hermes_batch_ops_to_KVS (small launch)");
    }
    lk.lock();
    set->busy = true;
    set->refs = nb;
    for (HostReq *r : take) {
        r->set = set;
        r->launched.store(true, std::memory_order_release);
    }
    t->combining = false;
    t->hcv.notify_all();
}

constexpr int kRingN = 16;   // ring slots of the serving kernel (launches in flight at most)
constexpr int kServeMerge = 4;   // published launches one serving-kernel pass may take together (HKV_SERVE_MERGE)

// The serving kernel has started leaving (some workgroup recorded the current epoch)
static bool srv_exited(const hkv_table *t)
{
    for (int g = 0; g < kPartG; ++g)
        if (__atomic_load_n(t->srv_words + 32 + g, __ATOMIC_ACQUIRE) == t->srv_epoch) return true;
    return false;
}

// With t->hmu held: every workgroup of the serving kernel gone (it may have left by itself already)
static void srv_stop_locked(hkv_table *t)
{
    if (!t->srv_running) return;
    srv_set_stop(t, 1u);
    if (hipEventSynchronize(t->srv_ev) != hipSuccess) die("serving kernel");
    srv_set_stop(t, 0u);
    t->srv_running = false;
}

static void srv_stop(hkv_table *t)
{
    std::lock_guard<std::mutex> lk(t->hmu);
    srv_stop_locked(t);
}

// Tables whose serving kernel was started: at process exit each is told to stop and waited for, so no
// persistent kernel is still running when the runtime tears down (it would leave after 2 ms idle anyway)
static void srv_atexit()
{
    std::lock_guard<std::mutex> lk(g_srv_mu);
    for (hkv_table *t : g_srv_tables)
        if (t->srv_running) {
            srv_set_stop(t, 1u);
            (void)hipEventSynchronize(t->srv_ev);
            t->srv_running = false;
        }
    g_srv_tables.clear();
}

// With t->hmu held, after a launch was published: a serving kernel will take it. If the running one
// is leaving (idle or lifetime limit), wait until it has gone and start another at every
// partition's first unfinished launch.
static void srv_ensure(hkv_table *t)
{
    if (t->srv_running && !srv_exited(t)) return;
    if (t->srv_running) {
        if (hipEventSynchronize(t->srv_ev) != hipSuccess) die("serving kernel");
        t->srv_running = false;
    }
    static const double idle_ms = getenv("HKV_SERVE_IDLE_MS") ? atof(getenv("HKV_SERVE_IDLE_MS")) : 2.0;
    HostServeLaunch sl;
    memset(&sl, 0, sizeof sl);
    {
        std::lock_guard<std::mutex> tl(t->mu);   // against hkv_table_populate (geo.log_head)
        sl.c.g = t->geo;
    }
    sl.c.index = t->d_index;
    sl.c.log = t->d_log;
    sl.c.error_flags = t->d_error_flags;
    sl.c.flags = t->pflags_d;
    sl.ring = t->ring_d;
    sl.ring_n = kRingN;
    sl.epoch = ++t->srv_epoch;
    sl.stop = t->srv_stop_d;
    sl.exited = t->srv_words_d + 32;
    sl.idle_ticks = (uint64_t)(idle_ms * 1e5);     // wall_clock64: 100 MHz
    sl.life_ticks = (uint64_t)1e8;                 // 1 s, then a fresh server
    static const int merge = getenv("HKV_SERVE_MERGE") ? std::max(1, atoi(getenv("HKV_SERVE_MERGE"))) : kServeMerge;
    sl.merge = std::min(merge, kRingN / 2);
    sl.spec = 1;   // the first launch's headers read beside the merge scan (round 5: 1 thread 7.2 -> 8.5 M)
    for (int g = 0; g < kPartG; ++g) sl.start[g] = __atomic_load_n(t->pflags + g, __ATOMIC_ACQUIRE) + 1;
    srv_set_stop(t, 0u);
    if (!t->srv_ev && hipEventCreateWithFlags(&t->srv_ev, hipEventDisableTiming) != hipSuccess) die("event");
    if (launch_host_serve(sl, t->stream) || hipEventRecord(t->srv_ev, t->stream) != hipSuccess) die("serving kernel launch");
    t->srv_running = true;
    {
        static std::once_flag once;
        std::call_once(once, [] { atexit(srv_atexit); });
        std::lock_guard<std::mutex> lk(g_srv_mu);
        if (std::find(g_srv_tables.begin(), g_srv_tables.end(), t) == g_srv_tables.end()) g_srv_tables.push_back(t);
    }
    TRACE("serving kernel epoch %u", sl.epoch);
}

// The last partitioned launch every workgroup has finished
static uint32_t part_done(const hkv_table *t)
{
    uint32_t m = __atomic_load_n(t->pflags, __ATOMIC_ACQUIRE);
    for (int g = 1; g < kPartG; ++g) {
        const uint32_t v = __atomic_load_n(t->pflags + g, __ATOMIC_ACQUIRE);
        if ((int32_t)(v - m) < 0) m = v;
    }
    return m;
}

// The queued partition-staged batches (in queue order, as many as keep every partition within
// kPartCap and the launch within kPartMaxB batches) as ONE k_hpart launch, its headers in the kernel
// arguments. At most HKV_PART_INFLIGHT (default 2) partitioned launches are in flight: a combiner
// first waits for the oldest, and batches queued meanwhile join its launch. Called with t->hmu held.
static void host_launch_part(hkv_table *t, std::unique_lock<std::mutex> &lk)
{
    // Serving kernel (k_hserve): launches are published to a ring that a persistent kernel polls,
    // instead of one k_hpart launch per combined batch. With the ring and the callers' batches in host
    // memory it ran at the launches' rates (round 3: the PCIe reads of descriptor and elements bound a
    // call); with both in device memory (stage_vram_usable) it is the default: same box, 3 reps each
    // (gpurun_out/r04z), 8.6-8.8 / 24.0-27.0 / 40.7-43.7 M local ops/s from 1 / 8 / 16 threads against
    // 6.1-6.9 / 23.0-26.0 / 35.6-44.1 M launched. HKV_HOST_SERVE=0 / 1 forces either.
    static const bool serve = getenv("HKV_HOST_SERVE") ? atoi(getenv("HKV_HOST_SERVE")) != 0 : stage_vram_usable();
    // One stream: launches round 4 streams, each partition's launches ordered on the device, were
    // measured (round 4) and ran 8 / 16 caller threads at 7.9-9.3 / 14.5-15.7 M local ops/s against
    // 20.4-21.0 / 34.9-36.0 M on the one table stream; that switch is gone (kept in git history)
    static const int inflight = std::min(kRingN, getenv("HKV_PART_INFLIGHT") ? std::max(1, atoi(getenv("HKV_PART_INFLIGHT")))
                                                                              : serve ? 4 : 2);
    if (!t->pflags) {
        // kPartG completion words (and one spare)
        if (hipHostMalloc((void **)&t->pflags, 4 * (kPartG + 1), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&t->pflags_d, t->pflags, 0) != hipSuccess)
            die("flag alloc");
        for (int g = 0; g <= kPartG; ++g) __atomic_store_n(t->pflags + g, 0u, __ATOMIC_RELEASE);
    }
    if (serve && !t->ring) {
        if (hipHostMalloc((void **)&t->srv_words, 4 * 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&t->srv_words_d, t->srv_words, 0) != hipSuccess)
            die("ring alloc");
        for (int k = 0; k < 64; ++k) __atomic_store_n(t->srv_words + k, 0u, __ATOMIC_RELEASE);
        t->ring_vram = stage_vram_usable();
        if (t->ring_vram) {   // under VRAM pressure the ring goes to pinned memory instead
            if (hipExtMallocWithFlags((void **)&t->ring, sizeof(HostRingSlot) * kRingN, hipDeviceMallocFinegrained) != hipSuccess ||
                hipExtMallocWithFlags((void **)&t->srv_stop, 64, hipDeviceMallocFinegrained) != hipSuccess) {
                (void)hipGetLastError();
                if (t->ring) (void)hipFree(t->ring);
                t->ring = nullptr;
                t->srv_stop = nullptr;
                t->ring_vram = false;
                TRACE("serving-kernel ring VRAM alloc failed: ring in pinned memory");
            }
        }
        if (t->ring_vram) {
            t->ring_d = t->ring;
            t->srv_stop_d = t->srv_stop;
        } else {
            if (hipHostMalloc((void **)&t->ring, sizeof(HostRingSlot) * kRingN, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
                hipHostGetDevicePointer((void **)&t->ring_d, t->ring, 0) != hipSuccess)
                die("ring alloc");
            t->srv_stop = t->srv_words;
            t->srv_stop_d = t->srv_words_d;
        }
        memset(t->ring, 0, sizeof(HostRingSlot) * kRingN);
        srv_set_stop(t, 0u);
    }
    const long c0 = g_host_timing ? now_ns() : 0;
    for (uint32_t spins = 0; (int32_t)(t->pseq - part_done(t)) >= inflight; ++spins) {
        if (serve && t->srv_running && srv_exited(t)) srv_ensure(t);   // a server that left has work to do
        lk.unlock();
        __builtin_ia32_pause();
        if ((spins & 255u) == 255u) sched_yield();
        lk.lock();
    }
    const long c1 = g_host_timing ? now_ns() : 0;
    HostPartLaunch pl;
    memset(&pl, 0, sizeof pl);
    std::vector<HostReq *> take;
    int tot[kPartG] = {0};
    for (auto it = t->hq.begin(); it != t->hq.end() && (int)take.size() < kPartMaxB;) {
        HostReq *r = *it;
        bool fits = r->part;
        for (int g = 0; fits && g < kPartG; ++g) fits = tot[g] + (r->poff[g + 1] - r->poff[g]) <= kPartCap;
        if (!fits) {  // taken later (another caller's batch: any order of callers is a serial order)
            ++it;
            continue;
        }
        for (int g = 0; g < kPartG; ++g) tot[g] += r->poff[g + 1] - r->poff[g];
        take.push_back(r);
        it = t->hq.erase(it);
    }
    const uint32_t seq = ++t->pseq;
    lk.unlock();
    const int nb = (int)take.size();
    for (int b = 0; b < nb; ++b) {
        const HostReq *r = take[b];
        HostPartHdr &h = pl.hdr[b];
        h.elems = r->st_elems;
        h.pos = r->st_pos;
        h.out = r->st_out;
        h.rw = r->st_rw;
        h.rwo = r->st_rwo;
        h.type = r->type;
        h.count = r->n;
        h.esz = r->esz;
        h.g_membership = (uint8_t)(r->mb >> 8);
        h.w_ack_init = (uint8_t)(r->mb >> 16);
        for (int g = 0; g <= kPartG; ++g) pl.part[g][b] = r->poff[g];
    }
    pl.c.index = t->d_index;
    pl.c.log = t->d_log;
    pl.c.error_flags = t->d_error_flags;
    pl.n_batches = nb;
    pl.c.flags = t->pflags_d;
    pl.seq = seq;
    if (g_host_stats) host_stats_note(nb);
    TRACE("partitioned launch %u batches=%d", seq, nb);
    const long c2 = g_host_timing ? now_ns() : 0;
    if (serve) {   // publish: the slot's contents, then its seq (x86 stores stay in order)
        HostRingSlot &slot = t->ring[seq % kRingN];
        slot.n_batches = nb;
        memcpy(slot.hdr, pl.hdr, sizeof(HostPartHdr) * (size_t)nb);
        memcpy(slot.part, pl.part, sizeof slot.part);
        __builtin_ia32_sfence();   // device memory is write-combined: the slot's bytes before its seq
        __atomic_store_n(&slot.seq, seq, __ATOMIC_RELEASE);
        __builtin_ia32_sfence();
        lk.lock();
        srv_ensure(t);
    } else {
        {
            std::lock_guard<std::mutex> tl(t->mu);   // against hkv_table_populate (geo.log_head)
            pl.c.g = t->geo;
            if (launch_host_part(pl, t->stream)) {
                die("hermes_batch_ops_to_KVS (partitioned launch)");
            }
        }
        lk.lock();
    }
    if (g_host_timing) {
        const long c3 = now_ns();
        g_hc_n += 1;
        g_hc_inflight += c1 - c0;
        g_hc_take += c2 - c1;
        g_hc_publish += c3 - c2;
    }
    for (HostReq *r : take) {
        r->pseq = seq;
        r->launched.store(true, std::memory_order_release);
    }
    t->combining = false;
}

// HKV_STAGE_VRAM (default 1): callers stage their batches in fine-grained device memory, written by
// the CPU through the PCIe BAR, so k_hpart reads them from HBM instead of over PCIe (same box, 3
// reps each: 8 threads 23.2-26.5 M local ops/s against 20.6-21.7 M; a lone call 17.4 against 19.3 us
// of wait). Whether the CPU can write device memory depends on the host (a resizable BAR): checked once
// with a guarded store, falling back to pinned staging when it faults.
static sigjmp_buf g_vram_jb;
static void vram_probe_fault(int) { siglongjmp(g_vram_jb, 1); }
static bool probe_vram()
{
    if (getenv("HKV_STAGE_VRAM") && atoi(getenv("HKV_STAGE_VRAM")) == 0) return false;
    void *p = nullptr;
    if (hipExtMallocWithFlags(&p, 4096, hipDeviceMallocFinegrained) != hipSuccess) return false;
    struct sigaction sa, old_segv, old_bus;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = vram_probe_fault;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_vram_jb, 1) == 0) {
        volatile uint64_t *v = reinterpret_cast<volatile uint64_t *>(p);
        v[0] = 0x5EED5EEDull;
        __builtin_ia32_sfence();
        ok = v[0] == 0x5EED5EEDull;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    (void)hipFree(p);
    TRACE("caller staging in device memory: %s", ok ? "yes" : "no (pinned)");
    return ok;
}
static bool stage_vram_usable()
{
    static const bool v = probe_vram();
    return v;
}

// Stages a caller's batch for a partitioned launch in its thread's pinned buffer (see "combining
// submit"): the elements partition-major, each with its position in the batch, and an ACK batch's
// read_write_ops. False when the table or the batch does not fit the partitioned kernel.
static bool host_stage_part(const hkv_table *t, HostReq &r)
{
    if (t->geo.entry_size != 64 || t->geo.st_value != 31 || r.esz > 64 || r.n > kPartG * kPartCap) return false;
    int cnt[kPartG] = {0};
    for (int i = 0; i < r.n; ++i) {
        const uint64_t key = *reinterpret_cast<const uint64_t *>(r.ops + (size_t)i * r.esz);
        if (++cnt[part_of(key)] > kPartCap) return false;
    }
    r.poff[0] = 0;
    for (int g = 0; g < kPartG; ++g) r.poff[g + 1] = (uint16_t)(r.poff[g] + cnt[g]);
    const size_t ebytes = align16((size_t)r.n * r.esz), pbytes = align16((size_t)r.n * 2);
    const size_t rw_bytes = r.type == acks && r.rw ? (size_t)t->cfg.rw_len * t->geo.op_size : 0;
    const size_t total = ebytes + pbytes + rw_bytes;
    CallerStage &st = t_stage;
    if (total > st.cap) {
        if (st.h) hipHostFree(st.h);
        st.h = st.d = nullptr;
        const size_t cap = std::max(total, (size_t)1 << 20);
        if (hipHostMalloc((void **)&st.h, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&st.d, st.h, 0) != hipSuccess) {
            if (st.h) (void)hipHostFree(st.h);
            st.h = st.d = nullptr;
            st.cap = 0;
            return false;   // the batch takes the staged-set path instead
        }
        st.cap = cap;
    }
    // device-memory staging when the BAR is writable and this caller's buffer could be allocated: under
    // VRAM pressure (torch in the same process) the caller stages in its pinned buffer instead
    bool vram = stage_vram_usable() && !st.vram_failed;
    // ACK batches in device memory: each read_write_ops slot's opcode beside the elements (hp_rw_ahead)
    size_t obytes = vram && rw_bytes ? align16((size_t)t->cfg.rw_len) : 0;
    if (vram && ebytes + pbytes + obytes > st.vcap) {
        if (st.v) (void)hipFree(st.v);
        st.v = nullptr;
        st.vcap = 0;
        const size_t cap = std::max(ebytes + pbytes + obytes, (size_t)1 << 20);
        if (hipExtMallocWithFlags((void **)&st.v, cap, hipDeviceMallocFinegrained) != hipSuccess) {
            (void)hipGetLastError();
            st.v = nullptr;
            st.vram_failed = true;
            vram = false;
            obytes = 0;
            TRACE("caller VRAM staging alloc failed: pinned staging for this caller");
        } else {
            st.vcap = cap;
        }
    }
    if ((int)st.perm.size() < r.n) st.perm.resize(r.n);
    uint16_t cur[kPartG];
    for (int g = 0; g < kPartG; ++g) cur[g] = r.poff[g];
    // built in a host buffer first when it goes to VRAM: one sequential copy, whole write-combined lines
    if (vram && st.tmp.size() < ebytes + pbytes + obytes) st.tmp.resize(ebytes + pbytes + obytes);
    uint8_t *sb = vram ? st.tmp.data() : st.h;
    uint16_t *pos = reinterpret_cast<uint16_t *>(sb + ebytes);
    for (int i = 0; i < r.n; ++i) {
        const uint8_t *x = r.ops + (size_t)i * r.esz;
        const uint32_t slot = cur[part_of(*reinterpret_cast<const uint64_t *>(x))]++;
        memcpy(sb + (size_t)slot * r.esz, x, r.esz);
        pos[slot] = (uint16_t)i;
        st.perm[i] = slot;
    }
    if (rw_bytes) memcpy(st.h + ebytes + pbytes, r.rw, rw_bytes);
    r.rw_bytes = rw_bytes;
    r.st_rwo = 0;
    if (obytes) {
        uint8_t *oc = sb + ebytes + pbytes;
        for (int k = 0; k < t->cfg.rw_len; ++k) oc[k] = r.rw[(size_t)k * t->geo.op_size + 8];
        r.st_rwo = (uint64_t)(uintptr_t)(st.v + ebytes + pbytes);
    }
    if (vram) {
        memcpy(st.v, sb, ebytes + pbytes + obytes);
        __builtin_ia32_sfence();   // the write-combined stores leave before the launch that reads them
        r.st_elems = (uint64_t)(uintptr_t)st.v;
        r.st_pos = (uint64_t)(uintptr_t)(st.v + ebytes);
        r.st_out = (uint64_t)(uintptr_t)st.d;
    } else {
        r.st_elems = (uint64_t)(uintptr_t)st.d;
        r.st_pos = (uint64_t)(uintptr_t)(st.d + ebytes);
        r.st_out = 0;
    }
    r.st_rw = rw_bytes ? (uint64_t)(uintptr_t)(st.d + ebytes + pbytes) : 0;
    r.rw_off = ebytes + pbytes;
    r.part = true;
    return true;
}

// Called with t->hmu held by a caller that found no combiner active: launches the compatible
// batches at the head of the queue as one multi-batch launch (see "combining submit" above).
// Test hook (hkv_debug_host_hold): a combiner first waits until this many batches are queued
// (or 5 s pass), so a test can put batches from several threads into one launch in a known order.
static std::atomic<int> g_host_hold{0};

static void host_combine(hkv_table *t, std::unique_lock<std::mutex> &lk)
{
    t->combining = true;
    if (const int hold = g_host_hold.load()) {
        for (int spins = 0; (int)t->hq.size() < hold && spins < 50000; ++spins) {
            lk.unlock();
            usleep(100);
            lk.lock();
        }
    }
    if (t->hq.front()->part) {  // partition-staged batches: one k_hpart launch, no staging set
        host_launch_part(t, lk);
        return;
    }
    srv_stop_locked(t);   // the launches below run on the table's stream, behind the serving kernel
    HostSet *set = nullptr;
    constexpr int n_sets = kHostSets;
    for (;;) {
        for (int k = 0; k < n_sets; ++k) {
            HostSet &hs = t->sets[k];
            if (!hs.busy) {
                set = &hs;
                break;
            }
        }
        if (set) break;
        t->hcv.wait(lk);
    }
    std::vector<HostReq *> take;
    int stride = 0;
    const HostReq *head = t->hq.front();
    if (head->n <= kSmallMaxElems) {  // batches of any type, one single-workgroup kernel
        host_launch_mixed(t, set, lk);
        return;
    }
    // a batch larger than the single-workgroup kernel takes: every queued batch of its kind on the
    // multi-kernel engine. Each caller has one batch queued at a time, so taking them out of queue
    // order still keeps every caller's own calls in program order.
    for (auto it = t->hq.begin(); it != t->hq.end() && (int)take.size() < kHostMaxBatches;) {
        HostReq *r = *it;
        const int st = std::max(stride, r->n);
        if (!host_compatible(head, r) || (!take.empty() && (int64_t)st * (int64_t)(take.size() + 1) > kHostMaxElems)) {
            ++it;
            continue;
        }
        stride = st;
        take.push_back(r);
        it = t->hq.erase(it);
    }
    lk.unlock();
    const int nb = (int)take.size();
    const HostReq *r0 = take[0];
    const bool with_rw = r0->type == acks && r0->rw != nullptr;
    const bool with_ns = r0->type == invs && r0->ns != nullptr;
    const size_t rw_bytes = with_rw ? (size_t)t->cfg.rw_len * t->geo.op_size : 0;
    const size_t ops_off = ((size_t)8 * nb + 255) & ~(size_t)255;
    const size_t ops_bytes = (size_t)nb * stride * r0->esz;
    const size_t rw_off = (ops_off + ops_bytes + 255) & ~(size_t)255;
    const size_t total = (rw_off + (size_t)nb * rw_bytes + 15) & ~(size_t)15;
    host_set_reserve(set, total);
    int32_t *h_counts = reinterpret_cast<int32_t *>(set->h);
    int32_t *h_ns = h_counts + nb;
    for (int b = 0; b < nb; ++b) {
        HostReq *r = take[b];
        h_counts[b] = r->n;
        h_ns[b] = with_ns ? *r->ns : -1;
        r->ops_off = ops_off + (size_t)b * stride * r->esz;
        r->ns_off = (size_t)4 * (nb + b);
        r->rw_off = rw_off + (size_t)b * rw_bytes;
        r->rw_bytes = rw_bytes;
        memcpy(set->h + r->ops_off, r->ops, (size_t)r->n * r->esz);
        if (with_rw) memcpy(set->h + r->rw_off, r->rw, rw_bytes);
    }
    hipStream_t s = t->stream;
    set->mode = kModeEvent;
    if (hipMemcpyAsync(set->d, set->h, total, hipMemcpyHostToDevice, s) != hipSuccess) die("copy in");
    hkv_batch_desc d;
    memset(&d, 0, sizeof d);
    d.type = r0->type;
    d.n_batches = nb;
    d.stride = stride;
    d.elem_size = r0->esz;
    d.d_elems = set->d + ops_off;
    d.d_counts = reinterpret_cast<const int32_t *>(set->d);
    d.d_rw = with_rw ? set->d + rw_off : nullptr;
    d.rw_stride_bytes = (int64_t)rw_bytes;
    d.d_node_suspected = with_ns ? reinterpret_cast<int32_t *>(set->d) + nb : nullptr;
    memcpy(d.membership, &r0->mb, 8);
    TRACE("combined launch type=%d batches=%d stride=%d", d.type, nb, stride);
    if (g_host_stats) host_stats_note(nb);
    {
        std::lock_guard<std::mutex> tl(t->mu);   // against hkv_table_populate (geo.log_head)
        if (hkv_batch_async(t, &d, s)) die("hermes_batch_ops_to_KVS");
    }
    if (hipMemcpyAsync(set->h, set->d, total, hipMemcpyDeviceToHost, s) != hipSuccess) die("copy out");
    if (hipEventRecord(set->ev, s) != hipSuccess) die("event record");
    lk.lock();
    set->busy = true;
    set->refs = nb;
    for (HostReq *r : take) {
        r->set = set;
        r->launched.store(true, std::memory_order_release);
    }
    t->combining = false;
    t->hcv.notify_all();
}

int hkv_debug_host_hold(int n_batches)
{
    if (n_batches < 0 || n_batches > kSmallMaxBatches) return fail(-1, "hold must be 0..%d", kSmallMaxBatches);
    g_host_hold.store(n_batches);
    return 0;
}

int hkv_debug_host_queued(void)
{
    hkv_table *t;
    {
        std::lock_guard<std::mutex> lk(g_default_mu);
        t = g_default;
    }
    if (!t) return 0;
    std::lock_guard<std::mutex> lk(t->hmu);
    return (int)t->hq.size();
}

// see the ABI note in hermeskv.h: curr_membership arrives as gcc passes the reference struct
void hermes_batch_ops_to_KVS(enum hermes_batch_type_t type, uint8_t *op_array, int op_num,
                             uint16_t sizeof_op_elem, uint64_t curr_membership,
                             int *node_suspected, spacetime_op_t *read_write_ops, uint8_t thread_id)
{
    static_assert(sizeof(spacetime_group_membership) == sizeof(uint64_t), "membership is 8 bytes");
    (void)thread_id;
    TRACE("hermes_batch_ops_to_KVS type=%d op_num=%d esz=%u rw=%p ns=%p", (int)type, op_num,
          (unsigned)sizeof_op_elem, (void *)read_write_ops, (void *)node_suspected);
    if (op_num <= 0) return;
    hkv_table *t;
    {
        std::lock_guard<std::mutex> lk(g_default_mu);
        t = g_default;
    }
    if (!t) {
        g_err = "spacetime_init was not called";
        die("hermes_batch_ops_to_KVS");
    }
    if ((int64_t)op_num > kHostMaxElems) {
        g_err = "more ops than a launch holds";
        die("hermes_batch_ops_to_KVS");
    }
    // the same element rules as hkv_batch_async, before anything is queued (either launch path)
    if (check_elems(t, (int)type, sizeof_op_elem, op_num)) die("hermes_batch_ops_to_KVS");
    if (hipSetDevice(t->cfg.device) != hipSuccess) die("hipSetDevice");
    HostReq r;
    r.type = (int)type;
    r.ops = op_array;
    r.n = op_num;
    r.esz = sizeof_op_elem;
    r.mb = curr_membership;
    r.ns = type == invs ? node_suspected : nullptr;
    r.rw = type == acks ? reinterpret_cast<uint8_t *>(read_write_ops) : nullptr;
    static const bool part_on = !getenv("HKV_HOST_PART") || atoi(getenv("HKV_HOST_PART")) != 0;
    const long t0 = g_host_timing ? now_ns() : 0;
    if (part_on) host_stage_part(t, r);   // else (or when it does not fit) the k_small / engine paths
    const long t1 = g_host_timing ? now_ns() : 0;
    {
        std::lock_guard<std::mutex> lk(t->hmu);
        t->hq.push_back(&r);
    }
    // until some combiner (maybe this caller) has launched the batch; spinning rather than sleeping
    // on a condition variable: a futex wake-up costs about as long as a whole launch
    for (uint32_t spins = 0; !r.launched.load(std::memory_order_acquire); ++spins) {
        if (!t->combining.load(std::memory_order_relaxed)) {
            std::unique_lock<std::mutex> lk(t->hmu);
            if (!r.launched.load(std::memory_order_acquire) && !t->combining.load()) host_combine(t, lk);
            continue;
        }
        __builtin_ia32_pause();
        if ((spins & 255u) == 255u) sched_yield();
    }
    HostSet *set = r.pseq ? nullptr : r.set;
    const int mode = set ? set->mode : kModePart;
    uint32_t seq = 0;
    if (set) {
        std::lock_guard<std::mutex> lk(t->hmu);
        seq = set->seq;
    }
    const long tl = g_host_timing ? now_ns() : 0;
    if (mode == kModePart) {  // every workgroup's flag at or past this launch (they only grow); yield
                              // now and then, so callers that outnumber the cores leave the combiner CPU time
        for (uint32_t spins = 0;; ++spins) {
            bool all = true;
            for (int g = 0; all && g < kPartG; ++g) all = (int32_t)(__atomic_load_n(t->pflags + g, __ATOMIC_ACQUIRE) - r.pseq) >= 0;
            if (all) break;
            __builtin_ia32_pause();
            if ((spins & 1023u) == 1023u) {
                sched_yield();
                std::lock_guard<std::mutex> lk(t->hmu);
                if (t->srv_running && srv_exited(t)) srv_ensure(t);   // it left before taking this launch
            }
        }
    } else if (mode == kModeSmall) {  // the kernel's completion flag in pinned memory
        for (uint32_t spins = 0; __atomic_load_n(set->flag, __ATOMIC_ACQUIRE) != seq; ++spins) {
            __builtin_ia32_pause();
            if ((spins & 1023u) == 1023u) sched_yield();
        }
    } else if (hipEventSynchronize(set->ev) != hipSuccess) {
        die("sync");
    }
    const long t2 = g_host_timing ? now_ns() : 0;
    if (g_host_timing) g_hc_flagwait += t2 - tl;
    if (mode == kModePart) {
        // results from this thread's staging, back in element order; node_suspected is
        // hermes_skip_inv's, a function of the elements alone: the last membership-change INV's
        // value[0] (hermesKV.c:735-744)
        const CallerStage &st = t_stage;
        for (int i = 0; i < op_num; ++i)
            memcpy(op_array + (size_t)i * sizeof_op_elem, st.h + (size_t)st.perm[i] * sizeof_op_elem, sizeof_op_elem);
        if (r.rw && r.rw_bytes) memcpy(r.rw, st.h + r.rw_off, r.rw_bytes);
        if (r.ns) {
            for (int i = op_num - 1; i >= 0; --i)
                if (op_array[(size_t)i * sizeof_op_elem + 8] == kOpMembChange) {
                    *r.ns = op_array[(size_t)i * sizeof_op_elem + kOpValueOff];
                    break;
                }
        }
    } else {
        memcpy(op_array, set->h + r.ops_off, (size_t)op_num * sizeof_op_elem);
        if (r.rw && r.rw_bytes) memcpy(r.rw, set->h + r.rw_off, r.rw_bytes);
        if (r.ns) memcpy(r.ns, set->h + r.ns_off, 4);
    }
    if (g_host_timing) {
        static std::once_flag once;
        std::call_once(once, [] { atexit(host_timing_print); });
        g_ht_calls++;
        g_ht_stage += t1 - t0;
        g_ht_wait += t2 - t1;
        g_ht_out += now_ns() - t2;
    }
    if (set) {
        std::lock_guard<std::mutex> lk(t->hmu);
        if (--set->refs == 0) {
            set->busy = false;
            t->hcv.notify_all();
        }
    }
    TRACE("done");
}

}  // extern "C"
