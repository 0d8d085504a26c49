"""Replicated-KVS throughput of the MI355X HermesKV data path (BASELINE.json metric).

A step is one protocol round (hermes_worker.c:438-546) of every virtual worker of every
replica: refill -> local batch -> INV broadcast -> incoming INV batch -> ACK batch -> incoming
VAL batch, with the reference's commit counting (inline-util.h:189-217). value = committed
local ops (GET_COMPLETE + PUT_COMPLETE [+ RMW_COMPLETE]) of all ranks / max-over-ranks time.

N=1: configs[1] of BASELINE.json -- 100M keys, 31-byte values, Zipf 0.99, 20 % writes, INVs and
VALs from 2 virtual replicas that also ACK every local write. N>1 (torchrun): one replica per
GPU, INV/VAL slabs all-gathered and ACKs returned over RCCL (hermes_amd.replica_group).

Prints one JSON line on rank 0 (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
EVENT_EVERY = 4                # timed steps per sampled local-launch duration
PROBE_STEPS = 3                # untimed steps with every batch launch timed
AUDIT_STEPS = 6                # untimed steps whose commits are broken down by outcome (CommitAudit)
# algorithmic bytes per element, SURVEY.md 8(d): S_op (56, or 312 big), bucket 64, entry (64, or
# 320 big), S_msg 16 (ACKs carry S_op with RMWs)
def elem_bytes(op: int, entry: int, ack: int) -> dict:
    """Algorithmic HBM bytes per element: the element read and written, the bucket,
    the entry read (and written when it changes). ACKs and VALs touch only the entry's first
    64-B line (key and meta); GETs, PUTs and INVs the whole entry (value)."""
    meta = min(entry, 64)
    return {"get": op + 64 + entry + op, "put": op + 64 + 2 * entry + op, "inv": op + 64 + 2 * entry + op,
            "ack": ack + 64 + 2 * meta + ack, "val": 16 + 64 + 2 * meta + 16}


def table_digest(kvs, n_keys: int, chunk: int = 1 << 23) -> tuple[int, int]:
    """(digest, keys not VALID) of a replica's protocol state: each populated log entry's state,
    timestamp (cid, version) and value, position-weighted (the populated entries sit back to back
    in the same order on every replica). Equal digests on all replicas = the group converged."""
    import torch

    class _Dev:   # the log as a torch tensor without a copy (__cuda_array_interface__)
        def __init__(self, ptr, n):
            self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}
    e = kvs.sizes.entry
    cols = torch.tensor([18] + list(range(23, 28)) + list(range(33, 33 + min(31, kvs.sizes.st_value))),
                        device=f"cuda:{kvs.device}")
    w = (torch.arange(cols.numel(), device=cols.device, dtype=torch.int64) * 0x9E3779B1 + 0x7F4A7C15) | 1
    log = torch.as_tensor(_Dev(kvs.device_log(), n_keys * e), device=f"cuda:{kvs.device}").view(n_keys, e)
    dig = torch.zeros((), dtype=torch.int64, device=cols.device)
    bad = torch.zeros((), dtype=torch.int64, device=cols.device)
    for lo in range(0, n_keys, chunk):
        x = log[lo:lo + chunk].index_select(1, cols).to(torch.int64)
        h = (x * w).sum(1)
        pos = torch.arange(lo, lo + x.shape[0], device=cols.device, dtype=torch.int64) * 0x2545F491 + 1
        dig += ((h * pos) & 0xFFFFFFFFFFFF).sum()
        bad += (x[:, 0] != 1).sum()      # VALID_STATE
    return int(dig.item()), int(bad.item())


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--config", choices=["cfg2", "cfg3", "cfg5"], default="cfg2",
                   help="cfg2: BASELINE configs[1] (the metric's config); cfg3: configs[2], RMW-heavy "
                        "(RMWs on, 287-B values, 25%% PUT + 25%% RMW; one replica, virtual peers); "
                        "cfg5: configs[4] on one GPU, an 8-replica group of 7 virtual peers, the last "
                        "one dropped in the middle of the timed steps")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--keys", type=int, default=None,
                   help="keys per replica (default: 100M at N=1, configs[1]; 1B at N>1, configs[3])")
    p.add_argument("--workers", type=int, default=16384,
                   help="virtual workers (250-op buffers) per GPU (swept at 4096-32768 under retry+skew: "
                        "3.20 G ops/s at 16384, 3.23 G at 32768, 2.96 G at 8192)")
    p.add_argument("--zipf", type=float, default=0.99)
    p.add_argument("--write-permille", type=int, default=None, help="default 200 (cfg2), 500 (cfg3)")
    p.add_argument("--rmw-permille", type=int, default=None,
                   help="RMWs among the writes, permille (default 0 (cfg2), 500 (cfg3))")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample length (0 = skip)")
    p.add_argument("--cpu-workers", type=int, default=0,
                   help="CPU baseline 250-op buffers (0 = one per thread, as the reference's workers)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline worker threads (0 = one per usable core, at most 16)")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--host-api-seconds", type=float, default=1.0,
                   help="time the host-pointer entry point for this long (0 = skip; N=1 only)")
    p.add_argument("--no-fit-acks", action="store_true",
                   help="N=1: keep the ACK slab at its capacity stride (2C) instead of the round's largest count")
    p.add_argument("--val-credits", type=int, default=None,
                   help="N=1: VAL messages per worker and round (the VAL credits; 225 = the reference's 15 "
                        "credits x 15 coalesced messages); workers with VALs outstanding do not poll ACKs. "
                        "Default: credits that never bind (every ACK applied and every VAL sent each round)")
    p.add_argument("--refill", choices=["fresh", "retry"], default="retry",
                   help="retry: refill_ops (inline-util.h:149-303), stalled ops keep their slot, as the "
                        "reference; fresh: every worker gets a fresh batch per round, stalled ops dropped")
    p.add_argument("--retry", action="store_true", help="same as --refill retry")
    p.add_argument("--skew", type=int, default=3,
                   help="the reference's opt-in skew optimisations (config.h:77-80), a bit mask: 1 completes a "
                        "stalled GET once its key's version moved two on (READ_COMPLETE_AFTER_VAL_RECV_OF_HOT_REQS), "
                        "2 coalesces a stalled PUT into the local write in flight (WRITE_COALESCE_TO_THE_SAME_KEY_IN_"
                        "SAME_NODE); default 3, 0 = the reference's default build")
    p.add_argument("--coalesce-hot", action="store_true",
                   help="refill_ops' ENABLE_COALESCE_OF_HOT_REQS: requests on the 100 hottest ids join the worker's "
                        "live op of that id (committed ops count them)")
    p.add_argument("--inplace-refill", action="store_true",
                   help="N=1: refill the ops in place (hkv_wl_refill_st / hkv_wl_refill) instead of planning patches "
                        "that the next local launch writes into the ops (hkv_wl_refill_plan, the default; configs[2] "
                        "under retry refills in place anyway, where that is faster)")
    p.add_argument("--policy-steps", "--retry-steps", type=int, default=10, dest="policy_steps",
                   help="N=1: also time this many steps of each other refill policy on the same table and "
                        "report them under detail.policies (0 = skip)")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="torch.distributed backend for N>1 (nccl = RCCL; gloo lets several ranks share one "
                        "GPU in tests)")
    return p.parse_args()


def host_api_rate(seconds: float, threads=(1, 8)) -> dict:
    """The drop-in entry point hermes_batch_ops_to_KVS on host buffers, as the reference's worker
    threads call it (configs[0] shape: the default 1M-key table, uniform keys, 5 % PUTs, 250-op
    local batches, then the ACKs of each batch's writes): tools/capi_threads, a gcc-built caller,
    with 1 and 8 threads whose batches the library combines into shared launches. Every call
    copies its batch over PCIe and back. Reported beside `value`, never as it."""
    import subprocess
    tool = os.path.join(ROOT, "tools", "capi_threads")
    out = {"unit": "local ops/s", "what": "hermes_batch_ops_to_KVS from T gcc-built worker threads (PCIe round "
           "trip per call, concurrent callers combined), 1M keys, uniform, 5% PUT, + ACK batches"}
    for t in threads:
        p = subprocess.run([tool, "throughput", str(t), str(seconds), "50"], capture_output=True, text=True,
                           timeout=120)
        if p.returncode != 0:
            raise RuntimeError(f"capi_threads failed: {p.stderr[-500:]}")
        d = json.loads(p.stdout.strip().splitlines()[-1])
        out[f"threads_{t}"] = d["local_ops_per_s"]
    out["value"] = out[f"threads_{max(threads)}"]
    return out


def refuse_debug_modes():
    """A timing number measured with work skipped must never leave bench.py: HKV_DBG in the
    environment, or a library built with the work-skipping modes (-DHKV_DEBUG_MODES), ends the run
    with rc 4 and no JSON line."""
    if os.environ.get("HKV_DBG") is not None:
        print(f"bench.py: HKV_DBG={os.environ['HKV_DBG']!r} is set (work-skipping timing modes); no measurement "
              "is reported from such a run", file=sys.stderr, flush=True)
        raise SystemExit(4)
    from hermes_amd.lib import _L, LIB_PATH
    if _L.hkv_debug_modes():
        print(f"bench.py: {LIB_PATH} was built with -DHKV_DEBUG_MODES (work-skipping timing modes); no "
              "measurement is reported from it", file=sys.stderr, flush=True)
        raise SystemExit(4)


def main():
    a = parse()
    if os.environ.get("HKV_DBG") is not None:   # before anything runs (the library check follows torch)
        refuse_debug_modes()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # the host-pointer callers run first, before this process opens the GPU: with this process's queues
    # idle beside them they measured 6.2 / 23.9 M instead of 7.2-8.1 / 31-34 M (1 / 8 threads)
    host_api = host_api_rate(a.host_api_seconds) if rank == 0 and world == 1 and a.host_api_seconds > 0 else None
    import torch
    import torch.distributed as dist

    refuse_debug_modes()
    dev = local_rank % max(1, torch.cuda.device_count())   # gloo tests: several ranks on one GPU
    torch.cuda.set_device(dev)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")

    from hermes_amd import layout as L
    from hermes_amd.kvs import HermesKV, sized_geometry
    from hermes_amd.workload import Round, zipf_params

    cfg3 = a.config == "cfg3"
    cfg5 = a.config == "cfg5"
    if a.retry:
        a.refill = "retry"
    retry = a.refill == "retry"
    if a.keys is None:  # cfg3: configs[1]'s 100M keys in 320-B entries (a 32 GiB log)
        a.keys = 100_000_000 if world == 1 and not cfg5 else 1_000_000_000
    if cfg3 and world > 1:
        raise SystemExit("--config cfg3 runs on one GPU with virtual peers")
    if a.write_permille is None:
        a.write_permille = 500 if cfg3 else 200
    if a.rmw_permille is None:
        a.rmw_permille = 500 if cfg3 else 0
    if cfg3 or cfg5:
        a.cpu_seconds = 0.0       # the CPU restatement's bench driver runs configs[1]'s round only
    t0 = time.time()
    sizes = L.Sizes(True, 4) if cfg3 else L.DEFAULT
    bkts, cap = sized_geometry(a.keys, sizes)
    kvs = HermesKV(a.keys, bkts, cap, machine_id=rank if world > 1 else 0, device=dev, rmw=cfg3,
                   big_objects=cfg3, extra_cache_lines=4 if cfg3 else 0, skew=a.skew)
    BYTES = elem_bytes(kvs.sizes.op, kvs.sizes.entry, kvs.sizes.op if cfg3 else 16)
    torch.cuda.synchronize()
    t_pop = time.time() - t0
    z = zipf_params(a.keys, a.zipf)
    total_steps = a.warmup + a.steps
    cpu = None
    snaps = {}
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        # the CPU baseline runs on the freshly populated table image (copied out of HBM now), after
        # the GPU's timed region so that its threads never compete with the GPU run's host thread;
        # a second image runs the reference's shipped configuration (retry, no skew flags) beside it
        from oracle.cpu_baseline import TableSnapshot
        snaps["headline"] = TableSnapshot(kvs)
        if retry and a.skew and not a.coalesce_hot:
            snaps["retry"] = TableSnapshot(kvs, skew=0)

    if world > 1:
        from hermes_amd.replica_group import ReplicaGroupRound
        # cfg5: the membership comes from Hades agreement over per-round heartbeats (SURVEY 8(f)
        # row 4): the failed rank stops heartbeating and the survivors expel it when they agree
        rnd = ReplicaGroupRound(kvs, a.workers, z, a.write_permille, seed=a.seed, world=world, rank=rank,
                                retry_stalled=retry, hades=cfg5)
    else:
        machines = 8 if cfg5 else 3
        rnd = Round(kvs, a.workers, L.membership(machines, 0), list(range(1, machines)), z, a.write_permille,
                    a.rmw_permille, seed=a.seed,
                    max_steps=total_steps + 2, retry_stalled=retry, fit_ack_stride=not a.no_fit_acks,
                    val_credits=a.val_credits, hades=cfg5, coalesce_hot=a.coalesce_hot,
                    fused_refill=False if a.inplace_refill else None)
    torch.cuda.synchronize()

    for _ in range(a.warmup):
        rnd.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    c0 = rnd.fold_counters()[:4].clone()
    rnd.count_elems = False  # element bookkeeping runs in probe steps after the timed region
    events: dict = {}
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    drop_at = a.steps // 2 if cfg5 else -1   # cfg5: the last replica fails in this timed step
    drop_id = world - 1 if world > 1 else 7
    t = time.perf_counter()
    for k in range(a.steps):
        # HIP events around the local launch (the roofline's) on every EVENT_EVERY-th step: each
        # record costs ~5 us of GPU time between kernels; the other launches: probe steps below
        rnd.step(events if k % EVENT_EVERY == 0 else None, timed_batches=("local",),
                 drop=drop_id if k == drop_at else None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t
    c1 = rnd.fold_counters()[:4].clone()
    committed = int((c1[0] - c0[0]).item())
    writes = int((c1[2] - c0[2]).item())
    dropped = int((c1[3] - c0[3]).item())
    # probe steps (untimed): elements each batch launch applies and every launch's duration
    rnd.count_elems = True
    e0, inv0 = rnd.elem_totals.clone(), rnd.inv_total.clone()
    probe_events: dict = {}
    for _ in range(PROBE_STEPS):
        rnd.step(probe_events)
    torch.cuda.synchronize()
    n_inv, n_ack, n_val = ((rnd.elem_totals - e0).double() / PROBE_STEPS).tolist()
    puts_per_step = float((rnd.inv_total - inv0).item()) / PROBE_STEPS
    # how the committed ops completed (value-less GETs, coalesced PUTs: DESIGN.md section 5), over
    # untimed rounds that continue the timed ones
    audit = rnd.audit_rounds(AUDIT_STEPS) if world == 1 and not a.coalesce_hot else None
    flags = kvs.take_error_flags()

    convergence = None
    if world > 1:
        # every replica's table after the last round (no write in flight): the live replicas must
        # agree on every key's state, timestamp and value, and every key must be VALID again (cfg5:
        # INVALID only where the failed replica's last writes were never validated)
        digest, not_valid = table_digest(kvs, a.keys)
        tt = torch.tensor([committed, elapsed * 1e9, flags, not_valid], dtype=torch.float64, device="cuda")
        allc = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(allc, tt)
        dg = torch.tensor([digest], dtype=torch.int64, device="cuda")
        alld = [torch.zeros_like(dg) for _ in range(world)]
        dist.all_gather(alld, dg)
        committed_all = int(sum(x[0].item() for x in allc))
        elapsed_max = max(x[1].item() for x in allc) / 1e9
        flags_any = int(max(x[2].item() for x in allc))
        live = [r for r in range(world) if not (cfg5 and r == drop_id)]
        convergence = {"digests": [int(x.item()) for x in alld], "not_valid": [int(x[3].item()) for x in allc],
                       "live_ranks_agree": len({int(alld[r].item()) for r in live}) == 1}
    else:
        committed_all, elapsed_max, flags_any = committed, elapsed, flags

    # live kernel time of the local batch launch over the timed region (HIP events on the stream
    # the batches run on); every launch over the untimed probe steps
    def avg(v):
        return sum(s.elapsed_time(e) for s, e in v) / len(v)
    probe_ms = {k: avg(v) for k, v in probe_events.items()}
    ms = dict(probe_ms)
    ms.update({k: avg(v) for k, v in events.items()})
    W, S = a.workers, Round.LOCAL
    per_launch_bytes = {
        "local": W * S * BYTES["get"] + puts_per_step * (BYTES["put"] - BYTES["get"]),
        "invs": n_inv * BYTES["inv"],
        "acks": n_ack * BYTES["ack"],
        "vals": n_val * BYTES["val"],
    }
    units = {"local": W * S, "invs": n_inv, "acks": n_ack, "vals": n_val}
    launches = {}
    for k, b in per_launch_bytes.items():
        if k not in ms or ms[k] <= 0:
            continue
        gbs = b / (ms[k] / 1e3) / 1e9
        launches[k] = {"elements": units[k], "algorithmic_bytes": b, "ms": ms[k], "achieved": gbs,
                       "frac": gbs / HBM_PEAK_GBS}
    # the roofline is quoted on the local batch launch (configs[1]'s metric unit); every launch
    # and the whole step are in `launches` / `step`
    dom = "local" if "local" in ms else (max(ms, key=ms.get) if ms else "local")
    ach = per_launch_bytes[dom] / (ms[dom] / 1e3) / 1e9 if ms else 0.0
    value = committed_all / elapsed_max
    step_ms = elapsed_max * 1e3 / a.steps
    step_bytes = sum(per_launch_bytes.values())
    # HBM traffic per launch: rocprofv3 PMC passes of this bench (tools/pmc.sh, tools/pmc_local.py) are
    # committed under profiles/; counters cannot be read inside the timed run itself
    traffic, traffic_src, pmc_launches = None, None, {}
    pmc = os.path.join(ROOT, "profiles", "pmc_local_batch.json")
    want = {"workers": a.workers, "keys": a.keys, "refill": a.refill, "skew": a.skew}
    if world > 1 or cfg3 or cfg5 or dom != "local":
        traffic_src = (f"null: PMC counters are committed for configs[1] at N=1 only (profiles/pmc_local_batch.json); "
                       f"this run is {a.config} at N={world}")
    elif not os.path.exists(pmc):
        traffic_src = "null: profiles/pmc_local_batch.json is missing (tools/pmc.sh + tools/pmc_local.py write it)"
    else:
        with open(pmc) as f:
            pj = json.load(f)
        if pj.get("config") != want:   # only counters taken on this very configuration
            traffic_src = (f"null: profiles/pmc_local_batch.json holds counters of {pj.get('config')}, not of this "
                           f"run's {want}")
        else:
            traffic = pj["traffic_bytes"]
            pmc_launches = pj.get("launches", {})
            traffic_src = (f"profiles/pmc_local_batch.json ({pj.get('source', 'rocprofv3 --pmc')}: FETCH_SIZE x2 + "
                           f"WRITE_SIZE in separate rocprofv3 passes of this configuration, median of "
                           f"{pj.get('launches_counted', pj.get('launches'))} launches). Per-shape multipliers "
                           f"(profiles/r06_counter_calibration.txt, tools/calib_bench.hip): reads x2 for every shape -- "
                           f"random 8/16/64/128-B records and 16-B streaming lanes each cost one 128-B request, counted "
                           f"as 64 B (RDREQ = lines, RDREQ_32B = 0); writes x1 -- exact for 64-B and 128-B blocks, "
                           f"32-B granules below 64 B. Traffic = 128-B lines read + bytes written at the memory side")
    for k, v in launches.items():
        t = pmc_launches.get(k, {}).get("traffic_bytes")
        v["traffic"] = t
        v["traffic_ratio"] = t / v["algorithmic_bytes"] if t else None
    refill = a.refill
    out = {
        "metric": "replicated KVS ops/s (reads+writes committed)",
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": step_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded Zipf traces, CityHash keys, virtual or RCCL peers)",
        "config": {
            "workload": (f"cfg5: {world}x MI355X, {8 if world == 1 else world}-replica group "
                         f"({'7 virtual peers' if world == 1 else 'RCCL'}), {a.keys} keys/replica, 20% writes, "
                         f"replica {drop_id} fails in timed step {drop_at} (membership change"
                         " agreed by Hades heartbeats, write replays)"
                         if cfg5 else
                         f"cfg3: 1xMI355X RMW-heavy, {a.keys} keys, RMWs on, 287 B values, Zipf 0.99, 25% PUT + 25% RMW, "
                         "INV/ACK/VAL from 2 virtual replicas" if cfg3 else
                         "cfg2: 1xMI355X, 100M keys, 31 B values, Zipf 0.99, 20% writes, "
                         "INV/ACK/VAL from 2 virtual replicas" if world == 1 else
                         f"cfg4: {world}-replica Hermes group over {'RCCL' if a.dist_backend == 'nccl' else 'gloo'}, "
                         f"{a.keys} keys/replica"),
            "keys": a.keys, "buckets": bkts, "log_cap": cap, "workers_per_gpu": W,
            "local_batch": S, "zipf": a.zipf, "write_permille": a.write_permille,
            "rmw_permille_of_writes": a.rmw_permille,
            # retry: refill_ops (inline-util.h:149-303), stalled ops keep their slots, as the reference;
            # fresh: every worker gets a fresh 250-op batch each round, stalled ops (e.g. a GET on a
            # key being written) are dropped and counted in detail.dropped_per_step, never committed;
            # writes in flight keep their slots. detail.policies times the others at N=1.
            "refill": refill,
            # the reference's opt-in skew optimisations (config.h:77-80): skew_flags bit 0 read
            # completion, bit 1 write coalescing (hermesKV.c:196-238); coalesce_hot: refill_ops'
            # hot-request coalescing (inline-util.h:237-257)
            "skew_flags": a.skew, "coalesce_hot": a.coalesce_hot,
            # VAL credits per worker and round (null: never binding, hermes_worker.c:479's gate idle)
            "val_credits": getattr(rnd, "V", None),
            "remote_invs_per_worker": rnd.rstride, "parallelism": f"replicas{world}",
            "elements_per_step": {"inv": n_inv, "ack": n_ack, "val": n_val},
        },
        "roofline": {
            "bound": "hbm", "kernel": (f"{dom} batch launch (" + ("k_local_pre + k_local_fused + k_local_deferred + k_commit_w, the direct path" if dom == "local"
                                                  and not cfg3 else "k_lookup + element-order rounds, the refill patches "
                                                  "written by k_resolve0_direct" if cfg3 and getattr(rnd, "fused", False)
                                                  else "k_lookup + element-order rounds") + ", hkv_batch.hip)"),
            "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_source": traffic_src,
            "traffic_ratio": traffic / per_launch_bytes[dom] if traffic else None, "launch_ms": ms.get(dom),
            "launch_samples": len(events.get(dom, [])),
            "algorithmic_bytes_per_launch": per_launch_bytes[dom],
            "launches": launches,
            # all four batch launches' algorithmic bytes over the whole step's wall time (refill,
            # marshalling and host synchronisation included)
            "step": {"algorithmic_bytes": step_bytes, "ms": step_ms,
                     "achieved": step_bytes / (step_ms / 1e3) / 1e9,
                     "frac": step_bytes / (step_ms / 1e3) / 1e9 / HBM_PEAK_GBS},
        },
        "detail": {
            "committed_per_step_rank0": committed / a.steps, "writes_completed_rank0": writes,
            "dropped_per_step_rank0": dropped / a.steps,
            "issued_per_step_rank0": W * S,
            "puts_succeeded_per_step_rank0": puts_per_step, "populate_s": t_pop,
            "step_bytes_per_committed_op_model": 554,
            "error_flags": flags_any,
            "round_stats_rank0": rnd.stats(),
        },
    }
    if cfg3 and refill == "retry":
        # rounds 50-60 of configs[2] under retry: almost every slot is an RMW parked on a few thousand hot
        # keys, whose entry lines the launch finds on-die, so achieved / peak is no fraction of HBM bandwidth
        out["roofline"]["frac_kind"] = "on-die: parked hot keys' lines hit in cache; not an HBM roofline"
    if convergence is not None:
        out["detail"]["convergence"] = convergence
        plan = getattr(rnd, "plan", None)
        if plan is not None:   # slabs sized without a host read in all but every calib_every-th round
            out["detail"]["slab_width"] = {"width": plan.width, "calib_every": plan.calib_every, "slack": plan.slack,
                                           "rounds": plan.k}
    if audit is not None:
        out["detail"]["commit_breakdown"] = audit
        # committed ops excluding value-less GETs and PUTs completed by an inherited timestamp, at
        # the audited rounds' share of the timed rate
        out["detail"]["committed_strict"] = {
            "value": value * audit["strict_fraction"] if audit["strict_fraction"] is not None else None,
            "unit": "ops/s", "strict_fraction": audit["strict_fraction"],
            "what": "GET_COMPLETE with a value + PUT_COMPLETE by the PUT's own write or coalesced on a timestamp "
                    "the PUT recorded itself + RMW_COMPLETE, as a share of all commits over "
                    f"{audit['rounds']} audited rounds after the timed ones, times value"}
    if flags_any:
        print(json.dumps({"error": f"device consistency flags {flags_any:#x} raised", "partial": out}), flush=True)
        raise SystemExit(3)
    if cfg5:
        mb = rnd.mb if world == 1 else rnd.r.mb
        out["detail"]["membership"] = {"machines": 8 if world == 1 else world, "dropped": drop_id,
                                       "at_timed_step": drop_at, "g_membership_after": mb[1]}
        hz = rnd.hades[0] if world == 1 else (rnd.r.hades if not rnd.r.failed else None)
        out["detail"]["membership"].update(agreement="hades", epoch=hz.state()[1] if hz else None)
        if world == 1:
            out["detail"]["membership"]["agreed_at_round"] = [c[0] for c in rnd.hades_changes]
    if snaps:
        from oracle.cpu_baseline import host_cores, run_cpu_baseline
        from hermes_amd.workload import refill_flags
        cpu = run_cpu_baseline(kvs, z, a.write_permille, a.cpu_workers, a.cpu_seconds, a.seed,
                               refill_flags=refill_flags(kvs, retry, a.coalesce_hot), threads=a.cpu_threads,
                               snapshot=snaps["headline"])
        cpu.update(host_cores())
        if "retry" in snaps:   # refill_ops without skew flags: no GET timestamp reset either
            c0 = run_cpu_baseline(kvs, z, a.write_permille, a.cpu_workers, a.cpu_seconds, a.seed,
                                  refill_flags=0, threads=a.cpu_threads, snapshot=snaps["retry"])
            cpu["policies"] = {"retry": {k: c0[k] for k in ("value", "unit", "cores", "kind", "sample",
                                                           "probe_ops_per_s_by_threads")}}
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if world == 1 and a.policy_steps > 0 and not cfg5:
        # the policies start from the table this run leaves: every write of it must have completed,
        # which holds only when no INV was held back by the send credits (nothing else is in flight)
        assert int(rnd.held.item()) == 0, "INVs held back: writes in flight would skew the other policies"
        rnd.close()
        out["detail"]["policies"] = policy_rates(a, kvs, z, L, Round, (retry, a.skew, a.coalesce_hot))
    if host_api is not None:
        out["detail"]["host_api"] = host_api
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


# the refill policies bench.py can time: (name, retry, skew_flags, coalesce_hot, what)
POLICIES = [
    ("fresh", False, 0, False, "a fresh batch per worker and round, stalled ops dropped (not the reference)"),
    ("retry", True, 0, False, "refill_ops (inline-util.h:149-303): stalled ops keep their slots; the reference's "
                              "default configuration"),
    ("retry_skew", True, 3, False, "refill_ops with the reference's skew optimisations: read completion and write "
                                   "coalescing (config.h:79-80, hermesKV.c:196-238)"),
    ("retry_skew_hot", True, 3, True, "retry_skew plus hot-request coalescing in refill_ops (config.h:77-78, "
                                      "inline-util.h:237-257); committed ops count the coalesced requests"),
]


def policy_rates(a, kvs, z, L, Round, headline) -> dict:
    """Every other refill policy of POLICIES on the same table, after the headline run (each round
    leaves every write complete, so the table carries no state from one policy to the next): a
    fresh Round, max(warmup, 10) untimed steps (retry's stalls build up over rounds), then
    a.policy_steps timed steps."""
    import torch
    out = {}
    skew0 = kvs.skew
    # refill_ops' retry without the skew flags has no steady state for tens of rounds (DESIGN.md section 5:
    # slots drain into the hottest keys): it is timed over rounds RETRY_FROM..RETRY_FROM+policy_steps,
    # not over the first rounds' descent
    RETRY_FROM = 50
    # every policy starts from a table with no write in flight: the headline round's INVs all went
    # out (none held back by the send credits), so its last ACK batch completed every write
    for name, retry, skew, hot, what in POLICIES:
        if (retry, skew, hot) == headline:
            continue
        kvs.set_skew(skew)
        warm = RETRY_FROM if (retry, skew, hot) == (True, 0, False) else max(a.warmup, 10)
        r = Round(kvs, a.workers, L.membership(3, 0), [1, 2], z, a.write_permille, a.rmw_permille,
                  seed=a.seed + 1, max_steps=warm + a.policy_steps + 2, retry_stalled=retry, coalesce_hot=hot)
        for _ in range(warm):
            r.step()
        torch.cuda.synchronize()
        c0 = r.fold_counters()[:4].clone()
        t = time.perf_counter()
        for _ in range(a.policy_steps):
            r.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        c = (r.fold_counters()[:4] - c0).tolist()
        audit = r.audit_rounds(3) if not hot else None
        held = int(r.held.item())
        assert held == 0, f"policy {name}: INVs held back"   # the next policy needs a quiet table
        r.close()
        out[name] = {"value": c[0] / dt, "unit": "ops/s", "steps": a.policy_steps, "warmup": warm,
                     "rounds_from": warm, "rounds_to": warm + a.policy_steps,
                     "ms_per_step": dt * 1e3 / a.policy_steps, "committed_per_step": c[0] / a.policy_steps,
                     "writes_completed_per_step": c[2] / a.policy_steps, "dropped_per_step": c[3] / a.policy_steps,
                     "invs_held": held, "commit_breakdown": audit,
                     "committed_strict": c[0] / dt * audit["strict_fraction"] if audit and audit["strict_fraction"] else None,
                     "what": what}
        del r
    kvs.set_skew(skew0)
    return out


if __name__ == "__main__":
    main()
