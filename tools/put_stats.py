"""What the local launch's PUT prepass works on (diagnostics, not the bench): per round of the
one-GPU bench round, read right after the local launch (the ops then hold the patched batch and
their results):
* elements, PUT elements that were not skipped (opcode PUT, not IN_PROGRESS_*), distinct keys among them;
* the sum over 1024-element blocks of each block's distinct PUT keys (k_local_pre's lookups);
* distinct (block, key) pairs over all looked-up elements at blocks of 32 ... 4096 elements;
* PUTs that mutated (PUT_SUCCESS), elements whose key has a PUT in the launch (k_local_fused's tagged
  F loads), and the largest element count of one key.

  python tools/put_stats.py --steps 12 > gpurun_out/put_stats.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--skew", type=int, default=3)
    p.add_argument("--refill", choices=["retry", "fresh"], default="retry")
    p.add_argument("--steps", type=int, default=12)
    p.add_argument("--workers", type=int, default=16384)
    p.add_argument("--keys", type=int, default=100_000_000)
    p.add_argument("--seed", type=int, default=0x5EED)
    a = p.parse_args()
    import torch
    from hermes_amd import layout as L
    from hermes_amd.kvs import HermesKV, sized_geometry
    from hermes_amd.workload import Round, zipf_params

    bkts, cap = sized_geometry(a.keys, L.DEFAULT)
    kvs = HermesKV(a.keys, bkts, cap, machine_id=0, skew=a.skew)
    z = zipf_params(a.keys, 0.99)
    r = Round(kvs, a.workers, L.membership(3, 0), [1, 2], z, 200, 0, seed=a.seed, max_steps=a.steps + 4,
              retry_stalled=a.refill == "retry")
    torch.cuda.synchronize()
    ops = r.ops.view(-1, r.op)
    n = ops.shape[0]
    inprog = torch.tensor([int(x) for x in (L.Bucket.IN_PROGRESS_PUT, L.Bucket.IN_PROGRESS_REPLAY,
                                            L.Bucket.IN_PROGRESS_GET, L.Bucket.IN_PROGRESS_RMW)], device=ops.device)
    stats = []
    local = r.local_batch

    def probed_local():
        local()
        torch.cuda.synchronize()
        key = ops[:, :8].contiguous().view(torch.int64).view(-1)
        opc, st = ops[:, 8], ops[:, 9]
        put = (opc == int(L.Op.PUT)) & ~torch.isin(st, inprog)
        pk = key[put]
        uk = torch.unique(pk)
        blk = torch.nonzero(put).view(-1) // 1024
        # distinct (block, key) pairs
        pair = torch.unique(torch.stack([blk, pk]), dim=1).shape[1] if pk.numel() else 0
        on_put_key = int(torch.isin(key, uk).sum())
        _, cnt = torch.unique(key, return_counts=True)
        # distinct (block, key) pairs over every looked-up element (not skipped: IN_PROGRESS_* stay skipped)
        # at several block sizes: what a workgroup sharing its keys' lookups would fetch
        looked = ~torch.isin(st, inprog)
        lidx = torch.nonzero(looked).view(-1)
        lkey = key[lidx]
        shares = {}
        for bs in (32, 256, 512, 1024, 2048, 4096):
            shares[str(bs)] = torch.unique(torch.stack([lidx // bs, lkey]), dim=1).shape[1] if lidx.numel() else 0
        stats.append({"looked_up": int(lidx.numel()), "block_key_pairs_all": shares, "elements": n, "put_elems": int(put.sum()), "distinct_put_keys": int(uk.numel()),
                      "block_key_pairs": pair, "put_success": int((st == int(L.Resp.PUT_SUCCESS)).sum()),
                      "elems_on_put_keys": on_put_key, "distinct_keys": int(cnt.numel()),
                      "max_elems_one_key": int(cnt.max())})

    r.local_batch = probed_local
    for k in range(a.steps):
        r.step()
        torch.cuda.synchronize()
        print(json.dumps({"round": k, **stats[-1]}), flush=True)
    assert kvs.take_error_flags() == 0


if __name__ == "__main__":
    main()
