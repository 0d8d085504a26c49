"""RCCL on the one GPU a test box has: a one-rank "nccl" process group (RCCL) carries every exchange
of a LoopbackGroup round (tests/test_rccl_gpu.py runs this file in a child process, so the process
group lives and dies with it).

The group's replicas share this process, so each collective of a round -- the INV totals and INV
slab all-gathers, the ACK all-to-all, the VAL totals and VAL slab all-gathers -- is staged exactly
as ReplicaGroupRound lays it out ([N][width] rows, row p = replica p) and then moved by RCCL
(all_gather_into_tensor / all_to_all_single over the one rank, async_op with the wait before the
consumer, on torch's stream), with the tensors, sizes and dtypes of a real round. With the per-peer
exchanges (HKV_GROUP_P2P, the default) every INV slab row and ACK row is one grouped isend/irecv
(batch_isend_irecv, to this rank itself) instead. Every batch launch
is mirrored into an oracle table and every key must converge. Prints one JSON line.
`--retry-skew`: bench.py's configuration (refill_ops' retry and the skew flags 3).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    from hermes_amd import layout as L
    from hermes_amd.kvs import HermesKV
    from hermes_amd.replica_group import LoopbackGroup, ReplicaRound
    from hermes_amd.workload import zipf_params
    from oracle.oracle import OracleKVS, gen_keys
    from tests.helpers import Mirror

    calls = {"all_gather_into_tensor": 0, "all_to_all_single": 0, "batch_isend_irecv": 0, "bytes": 0}

    class RcclLoopback(LoopbackGroup):
        """LoopbackGroup whose exchanges go through RCCL: the replicas' rows are staged in one
        tensor, which a one-rank all-gather / all-to-all moves into every replica's receive buffer."""

        @staticmethod
        def _gather(outs, ins):
            stage = torch.cat([x.reshape(-1) for x in ins])
            for o in outs:
                w = dist.all_gather_into_tensor(o.view(-1), stage, async_op=True)
                w.wait()
                calls["all_gather_into_tensor"] += 1
                calls["bytes"] += o.numel() * o.element_size()

        @staticmethod
        def _rows(pairs):
            # the per-peer exchanges (ReplicaGroupRound's p2p path): one grouped isend/irecv per row, here
            # a send to this one rank itself
            for snd, rcv in pairs:
                for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, snd.contiguous(), 0),
                                                 dist.P2POp(dist.irecv, rcv, 0)]):
                    w.wait()
                calls["batch_isend_irecv"] += 1
                calls["bytes"] += rcv.numel() * rcv.element_size()

        def _a2a(self, outs, ins):
            N = self.N
            for q, o in enumerate(outs):
                # row p of replica q's output is row q of replica p's input
                stage = torch.cat([x.view(N, -1)[q] for x in ins])
                w = dist.all_to_all_single(o.view(-1), stage, async_op=True)
                w.wait()
                calls["all_to_all_single"] += 1
                calls["bytes"] += o.numel() * o.element_size()

    retry_skew = "--retry-skew" in sys.argv
    skew = 3 if retry_skew else 0
    n_rep, n_keys, bkts, cap = 3, 4000, 8192, 1 << 20
    z = zipf_params(n_keys, 0.99)
    reps, mirrors = [], []
    for r in range(n_rep):
        g = HermesKV(n_keys, bkts, cap, machine_id=r, skew=skew)
        o = OracleKVS(bkts, cap, r, skew=skew)
        o.populate(n_keys, L.DEFAULT.kvs_value)
        mirrors.append(Mirror(g, o, f"replica {r}"))
        reps.append(ReplicaRound(g, 16, n_rep, r, z, 300, seed=99 + r, trace_len=512, retry_stalled=retry_skew))
    grp = RcclLoopback(reps)
    keys = gen_keys(n_keys)
    for _ in range(3):
        grp.step()
    torch.cuda.synchronize()
    # steady rounds at the planned width make no host synchronisation: 4 more rounds, unmirrored,
    # under torch.cuda.set_sync_debug_mode("error")
    for m in mirrors:
        m.g.batch = m._orig
    torch.cuda.set_sync_debug_mode("error")
    try:
        for _ in range(4):
            grp.step()
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    offs = [mirrors[0].o.lookup(int(k)) for k in keys]
    logs = [m.g.log_bytes() for m in mirrors]
    bad = 0
    for off in offs:
        if off is None:
            continue
        # state, timestamp (cid, version) and value must agree (the rest is each replica's own bookkeeping)
        img = [np.concatenate([lg[off + 18:off + 19], lg[off + 23:off + 28], lg[off + 33:off + 64]]) for lg in logs]
        if img[0][0] != L.State.VALID or any(not np.array_equal(x, img[0]) for x in img):
            bad += 1
    stats = [r.stats() for r in reps]
    dist.destroy_process_group()
    try:
        ver = list(torch.cuda.nccl.version())
    except Exception:   # noqa: BLE001 -- the version is informational
        ver = None
    print(json.dumps({"launches": [m.launches for m in mirrors], "calls": calls, "diverged_keys": bad,
                      "width": grp.plan.width if grp.plan else None,
                      "committed": [s["committed"] for s in stats], "rccl_version": ver, "skew": skew,
                      "retry": retry_skew}))


if __name__ == "__main__":
    main()
