/*
 * hermeskv_hades.h -- Hades membership agreement for a replica group whose
 * rounds are driven by collectives rather than timers: the heartbeat view each replica sends to
 * every peer, the views it receives, and the periodic view update (ostracism arbitration, epochs,
 * the majority rule) that produces the spacetime_group_membership the batch calls take.
 *
 *   hkv_hades_create          hades_ctx_init, include/hades/hades.h:99-141
 *   hkv_hades_view_for        issue_heartbeats, src/hades/hades.c:256-283 (one view per destination)
 *   hkv_hades_receive         poll_for_remote_views, hades.c:296-331
 *   hkv_hades_update          update_view_n_membership, hades.c:197-253 (with
 *                             view_arbitration_via_ostracism :150-184, skip_arbitration :127-139,
 *                             get_max_received_epoch_id :186-195, majority_of_nodes :62-67,
 *                             check_if_majority_is_rechable :70-86) and group_membership_update,
 *                             include/hermes/inline-util.h:26-43
 *
 * One call of hkv_hades_update is one view-update period (the reference's
 * update_local_view_every_ms timer, which is also the lease: a membership is valid for the
 * period it was agreed in). The reference does not check leases on the read path (SURVEY.md 8(f),
 * "Failure detection" row), and neither does this library; it reports whether a majority was
 * reachable, and the membership it returns is what the next batches run under.
 */
#ifndef HERMESKV_HADES_H
#define HERMESKV_HADES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* hades_view_t (hades.h:47-55), 4 packed bytes as gcc lays out the bit fields:
 * byte 2 bit 0 = same_w_local_membership, bits 1-7 = have_ostracised_for_dst_node. */
typedef struct hkv_hades_view {
    uint8_t node_id;
    uint8_t epoch_id;
    uint8_t flags;
    uint8_t view;               /* bit_vector_t of up to 8 nodes */
} hkv_hades_view;

#define HKV_HADES_NO_VIEW 0xFFu /* node_id of an empty slot: nothing was received from that sender */

typedef struct hkv_hades hkv_hades;

/* max_nodes in 2..8, machine_id < max_nodes; arbitration = ENABLE_ARBITRATION (hades.h:37: 1) */
int  hkv_hades_create(uint8_t max_nodes, uint8_t machine_id, int arbitration, hkv_hades **out);
void hkv_hades_destroy(hkv_hades *h);

/* the heartbeat for destination dst: the last local view, carrying whether this node ostracised
 * someone for dst in its last arbitration */
int  hkv_hades_view_for(const hkv_hades *h, uint8_t dst, hkv_hades_view *out);

/* a received heartbeat (ignored when node_id is HKV_HADES_NO_VIEW or out of range) */
int  hkv_hades_receive(hkv_hades *h, const hkv_hades_view *v);

/* One view-update period. Returns 1 when curr_g_membership changed, 0 when not, < 0 on error.
 * membership_out (8 bytes, may be NULL) receives the spacetime_group_membership of the current
 * membership as group_membership_update builds it (num_of_alive_remotes = members, including
 * this node; w_ack_init = the complement of the membership plus this node). *majority
 * (may be NULL) = 1 when this period's view reached a majority of max_nodes. */
int  hkv_hades_update(hkv_hades *h, uint8_t membership_out[8], int *majority);

/* curr_g_membership and the epoch of the intermediate local view */
int  hkv_hades_state(const hkv_hades *h, uint8_t *g_membership, uint8_t *epoch_id);

#ifdef __cplusplus
}
#endif
#endif /* HERMESKV_HADES_H */
