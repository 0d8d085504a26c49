// hkv_internal.h -- launch descriptors shared by the runtime and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "hkv_codes.h"

namespace hkv {

struct BatchLaunch {
    Geometry g;
    uint8_t *elems;
    const int32_t *counts;
    const uint8_t *index;
    uint8_t *log;
    uint8_t *rw;
    int64_t rw_stride;
    int32_t *ns_idx;
    int32_t *node_suspected;
    uint32_t *keys_a, *keys_b, *vals_a, *vals_b;
    // long-segment round state (see hkv_kernels.hip, stage 3)
    uint32_t *seg_start, *seg_end, *seg_count, *seg_fallback, *seg_of;
    unsigned long long *seg_mut;              // epoch-tagged, all-ones when allocated
    void *seg_meta;
    uint8_t *seg_done, *seg_snap;
    uint64_t *seg_hdr;
    uint32_t seg_cap;
    uint32_t epoch;                           // launch counter of the table, >= 1
    unsigned int *error_flags;                       // checked builds: unsound would_mutate()
    void *sort_tmp;
    size_t sort_tmp_bytes;
    int64_t n;
    int32_t n_batches;
    int32_t stride;
    int32_t esz;
    int32_t type;
    uint32_t skip_key;
    int32_t key_bits;
    uint8_t g_membership;
    uint8_t w_ack_init;
};

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

int launch_batch(const BatchLaunch &bl, hipStream_t s);
int launch_populate(const PopulateLaunch &pl, hipStream_t s);
int launch_hash_ids(const uint32_t *ids, uint64_t *out, int64_t n, hipStream_t s);
size_t sort_temp_bytes(int64_t n, int key_bits);
// long-segment scratch for launches of up to n elements: size, and carving into bl.seg_*
size_t seg_scratch_bytes(int64_t n, uint32_t entry_size);
void seg_carve(BatchLaunch &bl, uint8_t *base, int64_t n, uint32_t entry_size);

}  // namespace hkv
