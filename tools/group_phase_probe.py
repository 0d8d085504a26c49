"""Per-phase GPU time of an N-replica group round, all replicas on one GPU (LoopbackGroup): what one
replica of the RCCL run spends on local, INV, ACK and VAL phases (collectives excluded: here they
are tensor copies). python tools/group_phase_probe.py [N] [KEYS] [WORKERS] [ROUNDS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hermes_amd.kvs import HermesKV, sized_geometry  # noqa: E402
from hermes_amd.replica_group import LoopbackGroup, ReplicaRound  # noqa: E402
from hermes_amd.workload import zipf_params  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    keys = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
    workers = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    b, c = sized_geometry(keys)
    z = zipf_params(keys, 0.99)
    reps = [ReplicaRound(HermesKV(keys, b, c, machine_id=r, skew=3), workers, n, r, z, 200, seed=7 + r,
                         retry_stalled=True) for r in range(n)]
    grp = LoopbackGroup(reps)
    for _ in range(3):
        grp.step()
    torch.cuda.synchronize()
    names = ["start", "local", "invs", "acks", "vals", "end"]
    acc = {k: 0.0 for k in names[1:]}
    for _ in range(rounds):
        ev = {"start": torch.cuda.Event(enable_timing=True)}
        ev["start"].record()

        def seen(phase):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev[phase] = e
        grp.step(observer=seen)
        torch.cuda.synchronize()
        for a, bb in zip(names, names[1:]):
            acc[bb] += ev[a].elapsed_time(ev[bb])
    c0 = sum(r.fold_counters()[0].item() for r in reps)
    out = {k: round(v * 1e3 / rounds / n, 1) for k, v in acc.items()}
    out.update(replicas=n, keys=keys, workers=workers, unit="us per replica and round",
               committed_total=int(c0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
