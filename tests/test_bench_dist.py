"""Multi-rank bench logic on CPU (gloo, world_size 2): stream sharding and the max-over-ranks /
sum-over-ranks reductions bench.py uses for `value` (the data path itself has no collective)."""
from __future__ import annotations

import os
import socket
import sys

import torch.multiprocessing as mp

from conftest import ROOT


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import bench
    d = bench.Dist(world)
    elapsed = 1.0 + rank            # rank 1 is the slow one
    payload = 1000 * (rank + 1)
    d.barrier()
    out = (rank, bench.stream_base(rank), d.allmax(elapsed), d.allsum(payload))
    d.barrier()
    d.close()
    q.put(out)


def test_two_rank_reductions_and_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, base0, max0, sum0), (r1, base1, max1, sum1) = res
    assert (r0, r1) == (0, 1)
    assert max0 == max1 == 2.0          # value uses the slowest rank's time
    assert sum0 == sum1 == 3000         # and every rank's bytes
    import bench
    per = bench.STREAMS_PER_GPU
    assert base0 == 0 and base1 == per  # disjoint stream shards
    shards = [set(range(b, b + per)) for b in (base0, base1)]
    assert not (shards[0] & shards[1])


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` without a launcher starts two rank processes itself (no GPU is touched
    in --dry-run): they rendezvous over gloo and own disjoint 64-stream shards."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout          # rank 0 prints the one line, and nothing else reaches stdout
    j = json.loads(lines[0])                  # (gloo's connection messages go to stderr)
    assert j["n_gpus"] == 2
    ranks = j["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1] and [x["local_rank"] for x in ranks] == [0, 1]
    per = j["streams_per_gpu"]
    shards = [set(range(x["stream_base"], x["stream_base"] + per)) for x in ranks]
    assert not (shards[0] & shards[1]) and ranks[1]["stream_base"] == per
    # per-GPU entries (BASELINE.json configs[3]: per-GPU GiB/s beside the aggregate), one per rank
    pg = j["per_gpu"]
    assert len(pg) == j["n_gpus"] == 2
    assert [x["rank"] for x in pg] == [0, 1] and [x["stream_base"] for x in pg] == [0, per]
    assert all(set(x) >= {"value", "roofline_frac", "device_busy_frac", "ms_per_step"} for x in pg)


# A 2-socket 8-GPU node as the MI355X platform lays it out: GPUs 0-3 on socket 0 (cores 0-63,
# SMT siblings 128-191), GPUs 4-7 on socket 1 (64-127, 192-255); one CPU per core is usable.
NODE0 = ",".join(str(c) for c in range(64))
NODE1 = ",".join(str(c) for c in range(64, 128))
TOPOLOGY = [NODE0] * 4 + [NODE1] * 4


def test_cpu_share_eight_ranks_disjoint():
    """Each GPU's worker pool gets its own 16 cores of its socket: the 8 ranks' sets are
    disjoint, every set lies in its GPU's NUMA node, and together they cover the 128 cores."""
    import tonk_amd
    shares = [tonk_amd.cpu_share(TOPOLOGY, d, TOPOLOGY[d]) for d in range(8)]
    for d, s in enumerate(shares):
        assert len(s) == 16, (d, s)
        node = set(range(0, 64)) if d < 4 else set(range(64, 128))
        assert set(s) <= node
    flat = [c for s in shares for c in s]
    assert len(flat) == len(set(flat)) == 128


def test_cpu_share_edge_cases():
    import tonk_amd
    # one GPU per node keeps the whole node; an uneven split gives the remainder to the first
    assert tonk_amd.cpu_share(["0-7"], 0, "0-7") == list(range(8))
    three = [tonk_amd.cpu_share(["0-9"] * 3, d, "0-9") for d in range(3)]
    assert three == [[0, 1, 2, 3], [4, 5, 6], [7, 8, 9]]
    # more ranks than cores: no share is possible, every rank keeps the node (not pinned apart)
    assert tonk_amd.cpu_share(["0-1"] * 4, 3, "0-1") == [0, 1]
    # the override fixes the share when a launcher hides the other GPUs
    assert tonk_amd.cpu_share(["0-63"], 0, NODE0, "2/4") == list(range(32, 48))
    assert tonk_amd.cpu_share(["0-63"], 0, NODE0, "9/4") == list(range(64))  # invalid: ignored


def test_bench_dry_run_core_plan_disjoint():
    """`bench.py --gpus 2 --dry-run` on two GPUs of one socket: each rank reports its planned
    cores and the two lists are disjoint."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env["TONK_AMD_TOPOLOGY"] = ";".join(TOPOLOGY)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    c0, c1 = (x["host_cores"] for x in j["ranks"])
    assert c0 == list(range(16)) and c1 == list(range(16, 32))
    assert not set(c0) & set(c1)


# The same node with fewer usable cores: 48 per socket (the rest reserved), i.e. 12 per GPU.
SMALL0 = ",".join(str(c) for c in range(48))
SMALL1 = ",".join(str(c) for c in range(64, 112))
SMALL = [SMALL0] * 4 + [SMALL1] * 4


def test_cpu_share_fewer_cores_per_gpu():
    """Twelve usable cores per GPU: every rank's share is 12 cores of its own socket, disjoint."""
    import tonk_amd
    shares = [tonk_amd.cpu_share(SMALL, d, SMALL[d]) for d in range(8)]
    assert [len(s) for s in shares] == [12] * 8
    flat = [c for s in shares for c in s]
    assert len(flat) == len(set(flat)) == 96
    assert all(set(s) <= (set(range(48)) if d < 4 else set(range(64, 112))) for d, s in enumerate(shares))


def test_bench_dry_run_degrades_to_fewer_workers():
    """`bench.py --gpus 2 --dry-run` on a node with 12 usable cores per GPU: each rank plans 12
    workers (one per core of its share, never two on one core) instead of 16, and reports them."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env["TONK_AMD_TOPOLOGY"] = ";".join(SMALL)
    env["OMP_NUM_THREADS"] = "16"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    r0, r1 = j["ranks"]
    assert r0["host_cores"] == list(range(12)) and r1["host_cores"] == list(range(12, 24))
    # bench.host_threads: at most 16, and this process's CPUs split between the two ranks
    pool = max(1, min(16, len(os.sched_getaffinity(0)) // 2))
    assert r0["host_threads"] == r1["host_threads"] == min(pool, 12)
