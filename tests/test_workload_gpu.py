"""The N=1 bench round (hermes_amd.workload.Round, virtual peers) on the GPU: every batch launch
of a Round over more than kLookupHead (8192) local elements -- so the split lookup, the
absorbing-state shortcut, the INV/ACK rounds and the fallback all run as in bench.py -- is
mirrored into an oracle table and must be bit-exact (elements, read_write_ops, index, log).
"""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hermes_amd import layout as L  # noqa: E402
from oracle.oracle import OracleKVS  # noqa: E402
from tests.helpers import Mirror  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("theta,workers,cfg3", [(0.99, 40, False), (0.0, 40, False), (0.99, 160, False),
                                                (0.99, 40, True)])
def test_bench_round_mirrored(theta, workers, cfg3):
    """cfg3: bench.py --config cfg3 (RMWs on, big objects, 25 % PUT + 25 % RMW): the rounds engine,
    op-sized ACKs from the virtual peers, RMW completions."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts = 60_000, 1 << 16
    cap = 1 << 25 if cfg3 else 1 << 23
    steps = 3                         # 10,000 / 40,000 local elements per launch
    g = HermesKV(n_keys, bkts, cap, machine_id=0, rmw=cfg3, big_objects=cfg3, extra_cache_lines=4 if cfg3 else 0)
    o = OracleKVS(bkts, cap, 0, cfg3, cfg3, 4 if cfg3 else 0)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "bench round")
    r = Round(g, workers, L.membership(3, 0), [1, 2], zipf_params(n_keys, theta), 500 if cfg3 else 200,
              500 if cfg3 else 0, seed=0x5EED, max_steps=8, trace_len=1024)
    for _ in range(steps):
        r.step()
    torch.cuda.synchronize()
    assert m.launches == steps * 4
    st = r.stats()
    assert st["committed"] > 0 and st["writes_completed"] > 0, st
    assert g.take_error_flags() == 0


class _DeviceBytes:
    """A device byte range as a torch tensor, without a copy (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def test_full_size_round_invariants():
    """BASELINE configs[1] at full size (100M keys, 8192 virtual workers, the bench's round):
    properties that hold at any size. After every round each key is VALID again (every local write
    was ACKed by both virtual peers and completed, every INV's VAL applied, no membership change),
    no INV was held back, writes completed, and the engine's consistency flags are clear."""
    from hermes_amd.kvs import HermesKV, sized_geometry
    from hermes_amd.workload import Round, zipf_params
    n_keys = 100_000_000
    bkts, cap = sized_geometry(n_keys)
    g = HermesKV(n_keys, bkts, cap, machine_id=0)
    r = Round(g, 8192, L.membership(3, 0), [1, 2], zipf_params(n_keys, 0.99), 200, seed=0x5EED, max_steps=4)
    entry = g.sizes.entry
    assert g.log_head == n_keys * entry       # populate wrote entries 0..n-1 back to back
    log = torch.as_tensor(_DeviceBytes(g.device_log(), n_keys * entry), device="cuda")
    state = log.view(n_keys, entry)[:, 18]    # object meta byte 0: state
    assert int((state != int(L.State.VALID)).sum()) == 0
    for step in range(3):
        r.step()
        torch.cuda.synchronize()
        bad = int((state != int(L.State.VALID)).sum())
        assert bad == 0, f"round {step}: {bad} keys not VALID"
    st = r.stats()
    assert st["invs_held"] == 0 and st["committed"] > 2_000_000 and st["writes_completed"] > 300_000, st
    assert g.take_error_flags() == 0


@pytest.mark.parametrize("machines", [3, 8])
def test_membership_change_round_mirrored(machines):
    """BASELINE configs[4] on one GPU: the last virtual peer fails in round 2 after sending its
    INVs (no ACKs, no VALs from it), the group drops it and every worker runs the
    after-membership-change batch (hermes_worker.c:526-542); later rounds replay the writes it
    left INVALID. Every launch, including the after-change batch, is mirrored into the oracle."""
    from hermes_amd.kvs import HermesKV
    from hermes_amd.workload import Round, zipf_params
    n_keys, bkts, cap = 60_000, 1 << 16, 1 << 23
    g = HermesKV(n_keys, bkts, cap, machine_id=0)
    o = OracleKVS(bkts, cap, 0)
    o.populate(n_keys, g.sizes.kvs_value)
    m = Mirror(g, o, "membership round")
    peers = list(range(1, machines))
    r = Round(g, 40, L.membership(machines, 0), peers, zipf_params(n_keys, 0.99), 200, seed=0x5EED,
              max_steps=8, trace_len=1024, remote_per_peer=20)
    op = g.sizes.op
    replays = []
    marshal = r.marshal_invs

    def counting_marshal():
        replays.append(int((r.ops.view(-1, op)[:, 9] == int(L.Resp.REPLAY_SUCCESS)).sum()))
        marshal()
    r.marshal_invs = counting_marshal
    for step in range(6):
        r.step(drop=peers[-1] if step == 2 else None)
    torch.cuda.synchronize()
    assert m.launches == 6 * 4 + 1
    assert r.mb[1] == ((1 << machines) - 1) & ~(1 << peers[-1]) and r.alive == machines - 2
    st = r.stats()
    assert st["committed"] > 0 and st["writes_completed"] > 0, st
    assert sum(replays[3:]) > 0, replays
    assert g.take_error_flags() == 0
