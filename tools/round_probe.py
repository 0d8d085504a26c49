"""Per-round dynamics of the one-GPU bench round (diagnostics, not the bench).

For each round: committed ops, RMW aborts, the op slots parked on stalled ops at the end of the
round (GET/PUT/RMW_STALL) and on how many distinct keys, and how many of the round's commits were
on keys that had parked slots when the round started. Answers two questions:
* does a configuration reach a steady state (configs[2] under retry: VERDICT r03 item 5)?
* what bounds refill_ops' retry policy without the skew flags: a key with parked slots commits
  the GETs before its first PUT plus that PUT per round (about 1 / write ratio), so the rate is
  about (1 / w) x parked keys / round time.

  python tools/round_probe.py --config cfg2 --skew 0 --steps 60 > gpurun_out/probe.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", choices=["cfg2", "cfg3"], default="cfg2")
    p.add_argument("--skew", type=int, default=3)
    p.add_argument("--refill", choices=["retry", "fresh"], default="retry")
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--workers", type=int, default=16384)
    p.add_argument("--keys", type=int, default=100_000_000)
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--audit-every", type=int, default=0, help="also print a CommitAudit every N rounds")
    a = p.parse_args()
    import torch
    from hermes_amd import layout as L
    from hermes_amd.kvs import HermesKV, sized_geometry
    from hermes_amd.workload import Round, zipf_params

    cfg3 = a.config == "cfg3"
    sizes = L.Sizes(True, 4) if cfg3 else L.DEFAULT
    bkts, cap = sized_geometry(a.keys, sizes)
    kvs = HermesKV(a.keys, bkts, cap, machine_id=0, rmw=cfg3, big_objects=cfg3,
                   extra_cache_lines=4 if cfg3 else 0, skew=a.skew)
    z = zipf_params(a.keys, 0.99)
    wp, rp = (500, 500) if cfg3 else (200, 0)
    r = Round(kvs, a.workers, L.membership(3, 0), [1, 2], z, wp, rp, seed=a.seed, max_steps=a.steps + 4,
              retry_stalled=a.refill == "retry")
    torch.cuda.synchronize()
    ops = r.ops.view(-1, r.op)
    stall = torch.tensor([int(L.Resp.GET_STALL), int(L.Resp.PUT_STALL), int(L.Resp.RMW_STALL)], device=ops.device)
    done = torch.tensor([int(L.Resp.GET_COMPLETE), int(L.Resp.PUT_COMPLETE), int(L.Resp.RMW_COMPLETE)],
                        device=ops.device)

    def keys_of(mask):
        return ops[mask, :8].contiguous().view(torch.int64).view(-1)

    parked_keys = torch.empty(0, dtype=torch.int64, device=ops.device)
    c_prev = r.fold_counters()[:5].clone()
    print(json.dumps({"config": a.config, "skew": a.skew, "refill": a.refill, "workers": a.workers, "keys": a.keys,
                      "slots": a.workers * r.LOCAL}), flush=True)
    for k in range(a.steps):
        # the round, with its refill held back so the end-of-round states can be read
        t0 = time.perf_counter()
        refill = r.refill
        r.refill = lambda *args, **kw: None
        r.step()
        r.refill = refill
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = ops[:, 9]
        is_stall = torch.isin(st, stall)
        is_done = torch.isin(st, done)
        dk = keys_of(is_done)
        on_parked = int(torch.isin(dk, parked_keys).sum()) if parked_keys.numel() else 0
        sk = keys_of(is_stall)
        uniq, cnt = torch.unique(sk, return_counts=True) if sk.numel() else (sk, sk)
        top = torch.topk(cnt, min(5, cnt.numel())).values.tolist() if cnt.numel() else []
        parked_keys = uniq
        r.refill()
        c = r.fold_counters()[:5].clone()
        d = (c - c_prev).tolist()
        c_prev = c
        line = {"round": k, "ms": dt * 1e3, "committed": d[0], "writes_completed": d[2], "rmw_aborts": d[4],
                "parked_slots": int(is_stall.sum()), "parked_keys": int(uniq.numel()),
                "parked_top5": top, "commits_on_parked_keys": on_parked,
                "get_stall": int((st == int(L.Resp.GET_STALL)).sum()),
                "put_stall": int((st == int(L.Resp.PUT_STALL)).sum()),
                "rmw_stall": int((st == int(L.Resp.RMW_STALL)).sum())}
        if a.audit_every and (k + 1) % a.audit_every == 0:
            line["audit"] = r.audit_rounds(3)
            c_prev = r.fold_counters()[:5].clone()
        print(json.dumps(line), flush=True)
    flags = kvs.take_error_flags()
    # under the timing modes (HKV_DBG, a -DHKV_DEBUG_MODES build) skipped work raises flags by design
    assert flags == 0 or os.environ.get("HKV_DBG"), flags


if __name__ == "__main__":
    main()
