"""Shared test helpers: build op/message arrays and drive the known-answer scenario."""
from __future__ import annotations

import json
import os

import numpy as np

from hermes_amd import layout as L

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def make_elems(spec: list, keys: np.ndarray, sizes: L.Sizes, msg: bool):
    dt = L.msg_dtype() if msg else L.op_dtype(sizes)
    a = np.zeros(len(spec), dtype=dt)
    for i, s in enumerate(spec):
        a[i]["key"] = keys[s["id"]]
        a[i]["opcode"] = int(getattr(L.Op, s["opcode"]))
        st = s.get("sender", int(L.Bucket.NEW))
        a[i]["sender" if msg else "state"] = st
        a[i]["ts_ver"] = s.get("ts_ver", 0)
        a[i]["ts_cid"] = s.get("ts_cid", 0)
        if not msg:
            if "value" in s:
                a[i]["value"][:] = ord(s["value"])
                a[i]["val_len"] = sizes.st_value >> sizes.shift
    return a


def check_fields(obj, expect: dict, what: str):
    for k, v in expect.items():
        if k in ("id", "index"):
            continue
        if k == "value":
            got = chr(int(obj["value"][0]))
            assert got == v, f"{what}: value {got!r} != {v!r}"
        elif k == "lwid":
            got = int(obj["rmw_lwid"]) >> 1
            assert got == v, f"{what}: lwid {got} != {v}"
        else:
            got = int(obj[k])
            assert got == v, f"{what}: {k} {got} != {v}"


def run_known_answers(engine, keys: np.ndarray):
    """engine: object with batch(btype, elems, membership, rw=None) and entry(key) -> entry record."""
    ka = load_golden("known_answers.json")
    cfg = ka["config"]
    mb = L.membership(cfg["machine_num"], cfg["machine_id"])
    step_elems = []
    for si, step in enumerate(ka["steps"]):
        btype = getattr(L.BatchType, step["batch"])
        msg = step["batch"] in ("acks", "vals")
        elems = make_elems(step["ops"], keys, L.DEFAULT, msg)
        rw = step_elems[step["rw_from_step"]] if "rw_from_step" in step else None
        engine.batch(btype, elems, mb, rw=rw)
        step_elems.append(elems)
        for j, exp in enumerate(step["expect_ops"]):
            check_fields(elems[j], exp, f"step {si} elem {j}")
        for exp in step.get("expect_rw", []):
            check_fields(rw[exp["index"]], exp, f"step {si} rw {exp['index']}")
        if "expect_key" in step:
            e = engine.entry(keys[step["expect_key"]["id"]])
            check_fields(e, step["expect_key"], f"step {si} key")
    miss = make_elems([{"id": i, "opcode": "GET"} for i in ka["always_miss_ids"]], keys, L.DEFAULT, False)
    engine.batch(L.BatchType.local_ops, miss, mb)
    assert (miss["state"] == int(L.Resp.MISS)).all()
