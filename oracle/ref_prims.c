/*
 * ref_prims.c -- TEST INFRASTRUCTURE ONLY: exposes the reference's own L2 primitives to the
 * oracle tests. It holds no reference code: it #includes the reference headers where they lie
 * (-I /root/reference/include/utils, see oracle/Makefile) and wraps their static inline
 * functions in exported symbols, so tests/test_oracle.py can drive the unmodified reference
 * implementations against hkv_oracle.c's restatements:
 *
 *   concur_ctrl.h:144-213  cctrl_lock + cctrl_unlock_{dec,inc,inc_by_three,custom}_version
 *   concur_ctrl.h:63-75    timestamp_is_equal / timestamp_is_smaller
 *   concur_ctrl.h:217-224  cctrl_timestamp_is_same_and_valid
 *   bit_vector.h:403-481   bv_* (is_last_ack, spacetime.h:253-259, is bv_and + bv_are_equal;
 *                          group_membership_init, main.c:37-49, and group_membership_update,
 *                          inline-util.h:26-43, are bv_init/bit_set/copy/reverse/no_setted_bits)
 *   bit_vector.h:508-552   bv_unit_test, which runs dbv_unit_test (:341-384) first (both
 *                          defined by the reference, never called there)
 *
 * Built into oracle/_ref/libhkv_refprims.so only when /root/reference is present. Asserts stay
 * on (no -DNDEBUG): the reference's lock asserts (concur_ctrl.h:165-168) are part of what runs.
 */
#include <stdint.h>
#include <string.h>

#include "concur_ctrl.h"
#include "bit_vector.h"

/* cc: 6 bytes laid out as conc_ctrl_t {lock, ts.tie_breaker_id, ts.version}. Applies
 * cctrl_lock and then the unlock `variant` (0 dec, 1 inc, 2 inc_by_three, 3 custom(cid,
 * version)); returns the version reported through resp_version (inc variants) or 0. */
uint32_t hkr_cctrl_lock_unlock(uint8_t *cc, int variant, uint8_t cid, uint32_t version)
{
    conc_ctrl_t c;
    memcpy((void *)&c, cc, sizeof c);
    uint32_t resp = 0;
    cctrl_lock(&c);
    switch (variant) {
    case 0: cctrl_unlock_dec_version(&c); break;
    case 1: cctrl_unlock_inc_version(&c, cid, &resp); break;
    case 2: cctrl_unlock_inc_version_by_three(&c, cid, &resp); break;
    default: cctrl_unlock_custom_version(&c, cid, version); break;
    }
    memcpy(cc, (const void *)&c, sizeof c);
    return resp;
}

int hkr_conc_ctrl_size(void) { return (int)sizeof(conc_ctrl_t); }
int hkr_timestamp_size(void) { return (int)sizeof(timestamp_t); }

int hkr_ts_equal(uint32_t v1, uint8_t c1, uint32_t v2, uint8_t c2) { return timestamp_is_equal(v1, c1, v2, c2); }
int hkr_ts_smaller(uint32_t v1, uint8_t c1, uint32_t v2, uint8_t c2) { return timestamp_is_smaller(v1, c1, v2, c2); }

int hkr_cctrl_same_and_valid(const uint8_t *cc1, const uint8_t *cc2)
{
    conc_ctrl_t a, b;
    memcpy((void *)&a, cc1, sizeof a);
    memcpy((void *)&b, cc2, sizeof b);
    return cctrl_timestamp_is_same_and_valid(&a, &b);
}

/* is_last_ack (spacetime.h:253-259) on the reference bit vectors */
int hkr_is_last_ack(uint8_t ack_bv, uint8_t g_membership)
{
    bit_vector_t acks, g;
    acks.bit_array[0] = ack_bv;
    g.bit_array[0] = g_membership;
    bv_and(&acks, g);
    return bv_are_equal(acks, g);
}

/* the bit-vector steps of group_membership_init (main.c:37-49) for machines 0..machine_num-1:
 * out[0] g_membership, out[1] w_ack_init */
void hkr_membership_init(int machine_num, uint8_t machine_id, uint8_t *out)
{
    bit_vector_t g, w;
    bv_init(&g);
    for (uint8_t i = 0; i < machine_num; ++i) bv_bit_set(&g, i);
    bv_copy(&w, g);
    bv_reverse(&w);
    bv_bit_set(&w, machine_id);
    out[0] = g.bit_array[0];
    out[1] = w.bit_array[0];
}

/* the bit-vector steps of group_membership_update (inline-util.h:26-43) for a new g_membership:
 * out[0] g_membership, out[1] w_ack_init, out[2] num_of_alive_remotes (bv_no_setted_bits) */
void hkr_membership_update(uint8_t g_new, uint8_t machine_id, uint8_t *out)
{
    bit_vector_t src, g, w;
    src.bit_array[0] = g_new;
    bv_copy(&g, src);
    bv_copy(&w, g);
    bv_reverse(&w);
    bv_bit_set(&w, machine_id);
    out[0] = g.bit_array[0];
    out[1] = w.bit_array[0];
    out[2] = bv_no_setted_bits(g);
}

int hkr_bv_bit_get(uint8_t bv, int bit)
{
    bit_vector_t b;
    b.bit_array[0] = bv;
    return bv_bit_get(b, bit);
}

/* the reference's own static bit-vector unit test; aborts on failure */
void hkr_bv_unit_test(void) { bv_unit_test(); }
