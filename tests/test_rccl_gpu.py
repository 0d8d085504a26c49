"""RCCL itself on the test box's one GPU: a one-rank "nccl" process group carries every exchange
of a 3-replica round (tests/rccl_one_rank.py, in a child process), with every batch launch mirrored
into the oracle and every key converging. This is the RCCL execution possible before a multi-GPU
node runs bench.py --gpus N; the N-rank choreography itself is covered over gloo
(tests/test_replica_group_cpu.py) and on the GPU with several processes (test_dist_group_driver)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("args", [[], ["--retry-skew"]])
def test_one_rank_rccl_group_round(args):
    """args: [] the fresh policy; --retry-skew bench.py --gpus N's configuration (retry, skew flags 3)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_one_rank.py"), *args], capture_output=True,
                       text=True, timeout=170, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    print(d)
    assert d["launches"] == [15, 15, 15], d          # 3 rounds x (local, INV per peer (2), the ACK rows, VAL)
    assert d["diverged_keys"] == 0, d
    # per round and replica (3 mirrored rounds, then 4 steady ones under the sync check): INV totals, VAL
    # totals and VAL slabs gathered in the calibrating round, the VAL slab alone (carrying its total,
    # WidthPlan.fold) in the 6 steady ones; every INV slab row and ACK row one grouped isend/irecv
    # (3 replicas x 2 peers each, both directions: 12 per round)
    c = d["calls"]
    assert c["all_gather_into_tensor"] == (3 + 6 * 1) * 3 and c["all_to_all_single"] == 0, d
    assert c["batch_isend_irecv"] == 7 * 12, d
    assert d["width"] is not None
    assert min(d["committed"]) > 0
