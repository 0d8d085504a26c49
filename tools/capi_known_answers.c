/* Reference-side integration check in plain C: what a maintainer's worker would do after
 * replacing hermesKV.c/spacetime.c/mica.c with libhermeskv.so.
 * Build: gcc -O2 -I include tools/capi_known_answers.c -L hermes_amd -lhermeskv -Wl,-rpath,$PWD/hermes_amd */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "hermeskv.h"
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

static void on_segv(int sig, siginfo_t *si, void *ctx)
{
    (void)ctx;
    void *bt[64];
    int n = backtrace(bt, 64);
    fprintf(stderr, "signal %d at address %p\n", sig, si->si_addr);
    backtrace_symbols_fd(bt, n, 2);
    _exit(139);
}

/* layout of spacetime_op_t (spacetime.h:170-185) */
typedef struct { uint64_t key; uint8_t opcode, state, val_len, cid; uint32_t ver; uint16_t flags; uint8_t value[31]; uint8_t pad[7]; } op56;
typedef struct { uint64_t key; uint8_t opcode, sender, val_len, cid; uint32_t ver; } msg16;

/* CityHash128(&5,4).second and (&6,4).second from tests/golden/cityhash_ref.json */
int main(int argc, char **argv)
{
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, NULL);
    uint64_t k5 = strtoull(argv[1], 0, 10), k6 = strtoull(argv[2], 0, 10);
    spacetime_init(0);
    spacetime_group_membership m;
    memset(&m, 0, sizeof m);
    m.num_of_alive_remotes = 2; m.g_membership.bit_array[0] = 0x07; m.w_ack_init.bit_array[0] = 0xF9;
    op56 *ops = calloc(250, sizeof(op56));
    uint64_t keys[4] = {k5, k5, k5, k6};
    uint8_t codes[4] = {112, 111, 112, 111};
    for (int i = 0; i < 4; i++) {
        ops[i].key = keys[i]; ops[i].opcode = codes[i]; ops[i].state = 141;
        if (codes[i] == 112) { ops[i].val_len = 31; memset(ops[i].value, 'a', 31); }
    }
    hermes_batch_ops_to_KVS(local_ops, (uint8_t *)ops, 4, sizeof(op56), m, NULL, NULL, 0);
    printf("local: %u %u %u %u ts=(%u,%u) get6 len=%u v=%c\n", ops[0].state, ops[1].state, ops[2].state,
           ops[3].state, ops[0].ver, ops[0].cid, ops[3].val_len, ops[3].value[0]);
    int ok = ops[0].state == 122 && ops[1].state == 131 && ops[2].state == 132 && ops[3].state == 121 &&
             ops[0].ver == 2 && ops[3].val_len == 30 && ops[3].value[0] == 'g';
    op56 inv; memset(&inv, 0, sizeof inv);
    inv.key = k5; inv.opcode = 114; inv.state = 2; inv.val_len = 31; inv.ver = 2; inv.cid = 2; memset(inv.value, 'z', 31);
    int ns = -1;
    hermes_batch_ops_to_KVS(invs, (uint8_t *)&inv, 1, sizeof(op56), m, &ns, NULL, 0);
    msg16 ak[2] = {{k5, 115, 1, 0, 0, 2}, {k5, 115, 2, 0, 0, 2}};
    hermes_batch_ops_to_KVS(acks, (uint8_t *)ak, 2, sizeof(msg16), m, NULL, (spacetime_op_t *)ops, 0);
    msg16 val = {k5, 116, 2, 0, 2, 2};
    hermes_batch_ops_to_KVS(vals, (uint8_t *)&val, 1, sizeof(msg16), m, NULL, NULL, 0);
    op56 get; memset(&get, 0, sizeof get); get.key = k5; get.opcode = 111; get.state = 141;
    hermes_batch_ops_to_KVS(local_ops, (uint8_t *)&get, 1, sizeof(op56), m, NULL, NULL, 0);
    printf("inv=%u acks=%u,%u rw0=%u val=%u get=%u len=%u v=%c\n", inv.opcode, ak[0].opcode, ak[1].opcode,
           ops[0].state, val.opcode, get.state, get.val_len, get.value[0]);
    ok = ok && inv.opcode == 124 && ak[0].opcode == 125 && ak[1].opcode == 125 && ops[0].state == 128 &&
         val.opcode == 129 && get.state == 121 && get.val_len == 30 && get.value[0] == 'z';
    printf(ok ? "C-ABI known answers: OK\n" : "C-ABI known answers: MISMATCH\n");
    free(ops);
    return ok ? 0 : 1;
}
