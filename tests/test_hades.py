"""Hades membership agreement (hades.c:150-331, inline-util.h:26-43):
libhermeskv's hkv_hades_* (hermes_amd/hades.py) against the CPU model oracle/hades_oracle.py,
period by period, plus the agreement's scenarios: bootstrap to the full group, a failed node
expelled by every survivor in the same period with a new epoch, the ostracism rule for two-way
and one-way link failures, and the majority rule. Host code only (no GPU)."""
import random

import pytest

from hermes_amd.hades import Hades, exchange_views
from oracle.hades_oracle import NO_VIEW, HadesModel, View


def _run_pair(n, periods, dead_at=None, lost=None, seed=0):
    """drive library and model replicas in lockstep; return per-period states of the library"""
    dead_at = dead_at or {}
    lost = lost or (lambda p, s, d: False)
    hs = [Hades(n, i) for i in range(n)]
    ms = [HadesModel(n, i) for i in range(n)]
    hist = []
    for p in range(periods):
        alive = [dead_at.get(i, periods + 1) > p for i in range(n)]
        states = []
        for i in range(n):
            if not alive[i]:
                states.append(None)
                continue
            ch, mb, maj = hs[i].update()
            mch, mmaj = ms[i].update()
            assert (ch, maj) == (mch, mmaj), f"period {p} node {i}"
            assert mb == ms[i].membership(), f"period {p} node {i}"
            g, e = hs[i].state()
            assert (g, e) == (ms[i].curr_g, ms[i].intermediate.epoch_id), f"period {p} node {i}"
            for d in range(n):
                assert hs[i].view_for(d) == ms[i].view_for(d).pack(), f"period {p} node {i} view for {d}"
            states.append((g, e, ch, maj))
        hist.append(states)
        exchange_views([h if alive[i] else None for i, h in enumerate(hs)], lambda s, d: lost(p, s, d))
        for d in range(n):          # the same messages into the model replicas
            if not alive[d]:
                continue
            for s in range(n):
                if s == d or not alive[s] or lost(p, s, d):
                    continue
                ms[d].receive(ms[s].view_for(d))
    return hist


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
def test_library_matches_model_random_faults(n):
    rng = random.Random(1000 + n)
    for trial in range(6):
        periods = 30
        dead_at = {}
        if n > 2 and rng.random() < 0.7:
            dead_at[rng.randrange(n)] = rng.randrange(4, 20)
        cuts = set()
        for _ in range(rng.randrange(0, 3)):
            a, b = rng.sample(range(n), 2)
            lo = rng.randrange(2, 20)
            for p in range(lo, lo + rng.randrange(1, 8)):
                cuts.add((p, a, b))
                if rng.random() < 0.5:
                    cuts.add((p, b, a))
        drops = {(p, s, d) for p in range(periods) for s in range(n) for d in range(n) if rng.random() < 0.02}
        _run_pair(n, periods, dead_at, lambda p, s, d: (p, s, d) in cuts or (p, s, d) in drops, seed=trial)


def _final(hist):
    return hist[-1]


def test_bootstrap_reaches_full_membership():
    """spin_until_all_nodes_are_in_membership (hermes_worker.c:245-259): from a membership of
    itself only, every node agrees on the whole group within a few periods"""
    n = 5
    hist = _run_pair(n, 6)
    full = (1 << n) - 1
    assert all(s[0] == full for s in _final(hist))
    assert len({s[1] for s in _final(hist)}) == 1       # one epoch everywhere


def test_failed_node_expelled_with_new_epoch():
    n, dead = 5, 3
    hist = _run_pair(n, 14, dead_at={dead: 6})
    full = (1 << n) - 1
    before = hist[5]
    assert all(s[0] == full for s in before)
    e0 = before[0][1]
    changed_at = {i: next(p for p in range(6, 14) if hist[p][i][2]) for i in range(n) if i != dead}
    assert len(set(changed_at.values())) == 1            # all survivors switch in the same period
    p = next(iter(changed_at.values()))
    assert p <= 6 + 2                                    # detection takes at most two periods
    for i in range(n):
        if i != dead:
            g, e, _, maj = hist[-1][i]
            assert g == full & ~(1 << dead) and e == e0 + 1 and maj


def test_two_way_link_failure_ostracises_the_higher_id():
    """view_arbitration_via_ostracism (hades.c:150-184): nodes 1 and 2 stop hearing each other;
    the majority expels max(1, 2) = 2"""
    n = 4
    cut = lambda p, s, d: p >= 6 and {s, d} == {1, 2}  # noqa: E731
    hist = _run_pair(n, 16, lost=cut)
    for i in (0, 1, 3):
        assert hist[-1][i][0] == 0b1011, (i, hist[-1][i])


def test_one_way_link_failure_ostracises_the_deaf_node():
    """one-way failure: 2 no longer receives 1's heartbeats but 1 still hears 2 -- so 1's view
    keeps 2 while 2's view lacks 1, and the arbitration expels the node that still sees the other
    (i_view_of_j == 1 -> ostracise i): node 1"""
    n = 4
    cut = lambda p, s, d: p >= 6 and (s, d) == (1, 2)  # noqa: E731
    hist = _run_pair(n, 16, lost=cut)
    for i in (0, 2, 3):
        assert hist[-1][i][0] == 0b1101, (i, hist[-1][i])


def test_minority_cannot_change_membership():
    """majority_of_nodes (hades.c:62-67): two of five nodes cut off from the rest keep the old
    membership (they never gather three agreeing views) and report no majority"""
    n = 5
    part = {3, 4}
    cut = lambda p, s, d: p >= 6 and ((s in part) != (d in part))  # noqa: E731
    hist = _run_pair(n, 16, lost=cut)
    full = (1 << n) - 1
    for i in part:
        g, _, _, maj = hist[-1][i]
        assert g == full and not maj
    for i in (0, 1, 2):
        assert hist[-1][i][0] == 0b00111 and hist[-1][i][3]


def test_view_image_layout():
    """hades_view_t is 4 packed bytes; same_w_local_membership in bit 0 of byte 2"""
    v = View(3, 7, 1, 1, 0b1011)
    assert v.pack() == bytes([3, 7, 0b11, 0b1011])
    assert View.unpack(v.pack()) == v
    h = Hades(4, 2)
    b = h.view_for(0)
    assert len(b) == 4 and b[0] == 2 and b[3] == 0b0100
    assert NO_VIEW == 0xFF
