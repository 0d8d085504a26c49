// hkv_hades.cpp -- Hades membership agreement, driven one view-update period per call
// (include/hermeskv_hades.h). Host code: a replica group exchanges the views with one small
// collective per period and every replica runs the same agreement on what it received.
//
// Views are 4-byte hades_view_t images; bit vectors hold up to 8 nodes (bit_vector.h, one byte).

#include <cstdlib>
#include <cstring>
#include <new>

#include "../../include/hermeskv_hades.h"

namespace {

constexpr uint8_t kSameW = 1u;  // flags bit 0: same_w_local_membership; bits 1-7: have_ostracised_for_dst_node

inline bool bit(uint8_t bv, uint8_t i) { return (bv >> i) & 1u; }
inline int popcount8(uint8_t v) { return __builtin_popcount(v); }
inline uint8_t ostracised_for_dst(const hkv_hades_view &v) { return (uint8_t)(v.flags >> 1); }

}  // namespace

struct hkv_hades {
    uint8_t n = 0, me = 0;
    int arbitration = 1;
    hkv_hades_view last_local{}, intermediate{};
    uint8_t curr_g = 0;
    uint8_t recved[8] = {};
    hkv_hades_view remote[8] = {};
    uint8_t ostracized_for[8] = {};

    // majority_of_nodes, hades.c:62-67
    int majority() const { return n == 2 ? 2 : n / 2 + 1; }

    // skip_arbitration, hades.c:127-139
    bool skip(uint8_t i) const
    {
        if (i == me) return true;
        if (!recved[i]) return true;
        if (ostracised_for_dst(remote[i]) == 1) return true;  // it already ostracised someone for me
        if (!bit(remote[i].view, me)) return true;            // I am not in its view
        return false;
    }

    // view_arbitration_via_ostracism, hades.c:150-184: of two nodes that do not see each other,
    // the higher id is expelled -- unless the failure is one way and the higher one sees the
    // lower, which then goes
    void ostracism()
    {
        for (uint8_t i = 0; i < n; ++i) ostracized_for[i] = 0;
        for (uint8_t i = 0; i < n; ++i) {
            if (skip(i)) continue;
            for (uint8_t j = 0; j < n; ++j) {
                if (i >= j) continue;
                if (skip(j)) continue;
                const bool ivj = bit(remote[i].view, j), jvi = bit(remote[j].view, i);
                if (!ivj || !jvi) {
                    const uint8_t out = ivj ? i : j, fr = ivj ? j : i;
                    recved[out] = 0;
                    ostracized_for[fr] = 1;
                    intermediate.view &= (uint8_t)~(1u << out);
                }
            }
        }
    }

    // get_max_received_epoch_id, hades.c:186-195
    uint8_t max_received_epoch() const
    {
        uint8_t m = 0;
        for (uint8_t i = 0; i < n; ++i)
            if (recved[i] && remote[i].epoch_id > m) m = remote[i].epoch_id;
        return m;
    }

    // update_view_n_membership, hades.c:197-253 (the timer test is the caller's: one call, one period)
    bool update(int *maj)
    {
        const uint8_t before = curr_g;
        int agreeing = 1;  // always agree with my local view
        uint8_t same_w = 0;
        uint16_t max_epoch = intermediate.epoch_id;
        if (arbitration) ostracism();
        if (intermediate.view != curr_g || max_received_epoch() > intermediate.epoch_id) {
            for (uint8_t i = 0; i < n; ++i) {
                if (i == me || !recved[i]) continue;
                if (intermediate.view == remote[i].view) {
                    ++agreeing;
                    if (max_epoch < remote[i].epoch_id) {
                        max_epoch = remote[i].epoch_id;
                        same_w = remote[i].flags & kSameW;
                    }
                }
                recved[i] = 0;
            }
            if (agreeing >= majority()) {
                intermediate.epoch_id = (uint8_t)(max_epoch + (same_w == 1 ? 0 : 1));
                curr_g = intermediate.view;
            }
        }
        // check_if_majority_is_rechable (hades.c:70-86) only warns; report this period's view
        if (maj) *maj = popcount8(intermediate.view) >= majority();
        last_local = intermediate;
        last_local.flags = (uint8_t)((last_local.flags & ~kSameW) | (last_local.view == curr_g ? kSameW : 0));
        intermediate.view = (uint8_t)(1u << me);  // reset the local view
        return curr_g != before;
    }
};

extern "C" {

int hkv_hades_create(uint8_t max_nodes, uint8_t machine_id, int arbitration, hkv_hades **out)
{
    if (!out || max_nodes < 2 || max_nodes > 8 || machine_id >= max_nodes) return -1;
    hkv_hades *h = new (std::nothrow) hkv_hades;
    if (!h) return -1;
    // hades_ctx_init, hades.h:99-141: epoch 0, the membership and the local view hold this node only
    h->n = max_nodes;
    h->me = machine_id;
    h->arbitration = arbitration ? 1 : 0;
    h->intermediate.node_id = machine_id;
    h->intermediate.epoch_id = 0;
    h->intermediate.view = (uint8_t)(1u << machine_id);
    h->curr_g = (uint8_t)(1u << machine_id);
    h->last_local = h->intermediate;
    *out = h;
    return 0;
}

void hkv_hades_destroy(hkv_hades *h) { delete h; }

int hkv_hades_view_for(const hkv_hades *h, uint8_t dst, hkv_hades_view *out)
{
    if (!h || !out || dst >= h->n) return -1;
    // issue_heartbeats, hades.c:256-283: the last local view, stamped per destination
    *out = h->last_local;
    out->flags = (uint8_t)((out->flags & kSameW) | ((h->ostracized_for[dst] & 0x7Fu) << 1));
    return 0;
}

int hkv_hades_receive(hkv_hades *h, const hkv_hades_view *v)
{
    if (!h || !v) return -1;
    const uint8_t s = v->node_id;
    if (s == HKV_HADES_NO_VIEW || s >= h->n) return 0;
    // poll_for_remote_views, hades.c:296-331 (the rejoin branch resets transport credits only)
    h->recved[s] = 1;
    h->remote[s] = *v;
    h->intermediate.view |= (uint8_t)(1u << s);
    return 0;
}

int hkv_hades_update(hkv_hades *h, uint8_t membership_out[8], int *majority)
{
    if (!h) return -1;
    const bool changed = h->update(majority);
    if (membership_out) {
        // group_membership_update, inline-util.h:26-43
        std::memset(membership_out, 0, 8);
        membership_out[0] = (uint8_t)popcount8(h->curr_g);  // num_of_alive_remotes counts every member
        membership_out[1] = h->curr_g;
        membership_out[2] = (uint8_t)(~h->curr_g | (1u << h->me));
    }
    return changed ? 1 : 0;
}

int hkv_hades_state(const hkv_hades *h, uint8_t *g_membership, uint8_t *epoch_id)
{
    if (!h) return -1;
    if (g_membership) *g_membership = h->curr_g;
    if (epoch_id) *epoch_id = h->intermediate.epoch_id;
    return 0;
}

}  // extern "C"
