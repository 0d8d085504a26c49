// hkv_internal.h -- launch descriptors shared by the runtime and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "hkv_codes.h"

struct hkv_table;

namespace hkv {

struct BatchLaunch {
    Geometry g;
    uint8_t *elems;
    const int32_t *counts;
    const int32_t *offsets;      // packed INV/VAL launches: n_batches + 1 batch offsets (counts NULL)
    uint8_t *state_out;          // local launches: each element's final state byte (may be NULL)
    const uint8_t *opcode_in;    // local launches: the caller's mirror of each element's opcode (may be NULL)
    const uint8_t *patch;        // local launches: pending header writes, 16 B per element (may be NULL)
    uint8_t *rw_state;           // ACK launches: state-byte mirror of read_write_ops (may be NULL)
    const uint8_t *index;
    uint8_t *log;
    uint8_t *rw;
    int64_t rw_stride;
    int32_t *ns_idx;
    int32_t *node_suspected;
    // round state (see hkv_batch.hip): F words per log line (table-wide, all-ones when
    // allocated) and per-launch scratch carved by batch_carve
    unsigned long long *fw;
    unsigned long long *fx, *fy;              // INV words per log line (zero between launches)
    unsigned long long *ft;                   // ACK words, eight per log line (tagged with the epoch)
    unsigned long long *mem;
    uint32_t *ent, *fbl, *pf, *ctr;
    uint64_t *hx;                // [2 cap] patched headers of big local launches (BatchArgs::hx)
    uint16_t *fk;                // [cap] round-0 candidates' kinds of mutation (BatchArgs::fk)
    uint8_t *st, *shadow;
    uint32_t cap;                             // elements the scratch was carved for
    uint32_t epoch;                           // launch counter of the table, 1..batch_max_epoch()
    unsigned int *error_flags;                // checked builds: unsound would_mutate()
    int64_t n;
    int32_t n_batches;
    int32_t stride;
    int32_t esz;
    int32_t type;
    uint8_t g_membership;
    uint8_t w_ack_init;
    int32_t path;                             // kPath*: which engine runs the launch
    int32_t unique;                           // HKV_BATCH_UNIQUE: no key twice in the launch
    int32_t n_rows, skip_row;                 // HKV_BATCH_ROWS (n_rows 0: a plain launch)
    uint8_t *ack_out;                         // INV launches: the ACK marshal's output (hkv_batch_desc.d_ack_out)
    uint32_t ack_out_size;
    int64_t row_stride;
    // small launches staged in host memory (the combining submit of hermes_batch_ops_to_KVS): the
    // kernel first copies region_bytes from host_src to dev_region (where elems, counts, rw and
    // node_suspected point), at the end copies them back to host_dst, then stores done_value into
    // *done_flag at system scope. region_bytes = 0: everything already in device memory.
    const uint8_t *host_src;
    uint8_t *host_dst;
    uint8_t *dev_region;
    uint64_t region_bytes;
    uint32_t *done_flag;
    uint32_t done_value;
    // mixed small launches (host-staged): n_batches headers at dev_region, batches of any type and
    // element size back to back; elems/counts/stride/esz/type/rw/node_suspected unused
    const struct SmallBatch *hdr;
};

// One batch of a mixed small launch; offsets are bytes from the launch's device region.
struct SmallBatch {
    int32_t type, count, esz, elem_off;
    int32_t rw_off, ns_off;   // -1: none (rw: ACK batches' read_write_ops; ns: INV batches' node_suspected)
    uint8_t g_membership, w_ack_init, pad0, pad1;
    int32_t pad2;
};
constexpr int kSmallMaxBatches = 64;

// ---- partitioned host launches (the combining submit of hermes_batch_ops_to_KVS, 64-B entries):
// every element goes to the workgroup that owns its key, part_of(key) of kPartG, so workgroups
// never share a key and need no communication. Each caller stages its own batch, partition-major
// (elements in element order within a partition), in its own pinned buffer; the launch carries one
// HostPartHdr per batch and part[g][b]: batch b's elements of partition g are
// [part[g][b], part[g + 1][b]) of its staged array -- all in the kernel arguments, which the
// dispatch delivers with the launch (no PCIe round trip for them).
constexpr int kPartG = 32;       // workgroups of one launch
constexpr int kPartCap = 256;    // elements one workgroup takes
constexpr int kPartMaxB = 16;    // batches one launch combines
__host__ __device__ inline uint32_t part_of(uint64_t key)
{
    return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 59);   // kPartG = 32
}
struct HostPartHdr {
    uint64_t elems;   // device address: the staged elements, partition-major
    uint64_t pos;     // device address: u16 position in the batch of each staged element
    uint64_t rw;      // ACK batches: device address of the read_write_ops copy, else 0
    int32_t type, count, esz;
    uint8_t g_membership, w_ack_init, pad0, pad1;
    uint64_t out;     // device address the results go to (pinned), or 0: back into elems
    uint64_t rwo;     // ACK batches staged in device memory: each read_write_ops slot's opcode there, else 0
};
static_assert(sizeof(HostPartHdr) == 56, "HostPartHdr is seven 8-byte words");
struct HostPartCommon {
    Geometry g;
    const uint8_t *index;
    uint8_t *log;
    unsigned int *error_flags;
    uint32_t *flags;             // device address: kPartG words, workgroup g stores seq into flags[g]
    unsigned long long *prof;    // HKV_PART_PROF: workgroup 0's phase timestamps (debug), or NULL
};
struct HostPartLaunch {          // one launch, everything in the kernel arguments
    HostPartCommon c;
    uint32_t seq;
    int32_t n_batches;
    HostPartHdr hdr[kPartMaxB];
    uint16_t part[kPartG + 1][kPartMaxB];
};
// one launch published to the serving kernel (pinned ring slot; seq written last)
struct alignas(128) HostRingSlot {
    uint32_t seq;
    int32_t n_batches;
    uint32_t pad[2];
    HostPartHdr hdr[kPartMaxB];
    uint16_t part[kPartG + 1][kPartMaxB];
};
struct HostServeLaunch {
    HostPartCommon c;
    const HostRingSlot *ring;    // device address of ring_n slots (pinned); launch n in slot n % ring_n
    int32_t ring_n;
    uint32_t epoch;
    const uint32_t *stop;        // pinned: non-zero makes every workgroup leave between launches
    uint32_t *exited;            // pinned: workgroup g stores epoch into exited[g] when it leaves
    uint64_t idle_ticks, life_ticks;   // wall_clock64 ticks (100 MHz)
    int32_t merge;               // launches one workgroup pass may take together (HKV_SERVE_MERGE; 1: one at a time)
    uint32_t start[kPartG];      // the first launch each workgroup takes
    int32_t spec;                // the first launch's headers read beside the merge scan (HKV_SERVE_SPEC)
};
int launch_host_serve(const HostServeLaunch &sl, hipStream_t s);
int launch_host_part(const HostPartLaunch &pl, hipStream_t s);

enum : int32_t { kPathAuto = 0, kPathEngine = 1, kPathSmall = 2 };

struct PopulateLaunch {
    uint64_t *first, *second;
    uint32_t *keys_a, *keys_b, *vals_a, *vals_b;
    void *sort_tmp;
    size_t sort_tmp_bytes;
    uint8_t *index;
    uint8_t *log;
    unsigned long long *evictions;
    int64_t n;
    uint64_t bkt_mask;
    uint64_t log_cap, log_mask;
    uint64_t h0, k, hw;
    uint32_t entry_size;
    int32_t key_bits;
    uint8_t val_len_byte;
};

// A table's HBM image and geometry, for the workload kernels that read it (virtual peers take
// each key's current timestamp when they write it, hkv_workload.hip)
struct TableView {
    Geometry g;
    const uint8_t *index;
    const uint8_t *log;
};
int table_view(const hkv_table *t, TableView *out);

int launch_batch(BatchLaunch &bl, hipStream_t s);
constexpr int64_t kSmallMaxElems = 4096;   // launches the single-workgroup kernel can take
int launch_populate(const PopulateLaunch &pl, hipStream_t s);
int launch_hash_ids(const uint32_t *ids, uint64_t *out, int64_t n, hipStream_t s);
size_t sort_temp_bytes(int64_t n, int key_bits);
// batch scratch for launches of up to cap elements (size, carving into bl); the table-wide F
// words (one per 64-B log line, all-ones when allocated and whenever the epoch wraps)
size_t batch_scratch_bytes(int64_t cap, uint32_t entry_size);
void batch_carve(BatchLaunch &bl, uint8_t *base, int64_t cap, uint32_t entry_size);
size_t batch_fw_words(uint64_t log_cap);
uint32_t batch_max_epoch();

}  // namespace hkv
