"""The N>1 host path of bench.py on CPU: world_size-2 gloo processes share
the RCCL id from rank 0, size the per-rank fingerprint set and take the job
time as the max over ranks.  The device data path
(RCCL all-to-all-v between shards) is covered on one GPU by the virtual-shard
tests in test_gpu.py."""
import os
import re
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cid = bench.share_comm_id(rank, lambda: bytes(range(128)))
        t = bench.max_over_ranks(1.0 + rank, world)
        fpl = bench.fpset_log2_for(bench.SECONDARY, world)
        dist.barrier()
    finally:
        dist.destroy_process_group()
    out.put((rank, cid, t, fpl))


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_control_plane(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    assert [r[0] for r in res] == list(range(world))
    assert all(r[1] == bytes(range(128)) for r in res)      # every rank got rank 0's id
    assert all(r[2] == float(world) for r in res)           # max over ranks
    assert len({r[3] for r in res}) == 1


def test_fpset_per_rank_sizing():
    one = bench.fpset_log2_for(bench.SECONDARY, 1)
    assert one == 33
    distinct = 2_407_297_045  # the exhaust model
    for world in (1, 2, 4, 8):
        fpl = bench.fpset_log2_for(bench.SECONDARY, world)
        load = distinct / world / (1 << fpl)
        assert 0.2 < load < 0.3, (world, fpl, load)
        # parent records (0.75 x slots per shard, rtla_host.cpp) hold a shard's states
        assert distinct / world < 0.75 * (1 << fpl)
    assert bench.fpset_log2_for(bench.SECONDARY, 8, override=28) == 28
    # capped workloads at the oracle-pinned depth (the default) split the set
    # like any other; run to the depth that fits they keep the one-GPU set per
    # rank (more GPUs reach deeper levels)
    assert bench.fpset_log2_for("cfg2", 8) == bench.fpset_log2_for("cfg2", 1) - 3
    assert bench.fpset_log2_for("cfg2", 8, pinned=False) == bench.fpset_log2_for("cfg2", 1)


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts 2 ranks under
    torch.distributed.run as a child process; both reach the process group
    and receive rank 0's id (the GPU work is skipped with --dry-run)."""
    import subprocess
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=240,
                         env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stdout + out.stderr
    lines = sorted(re.findall(r"bench\.py rank \d of \d ready \(id [0-9a-f]+\)", out.stdout))
    assert lines == ["bench.py rank 0 of 2 ready (id 00010203)", "bench.py rank 1 of 2 ready (id 00010203)"], \
        out.stdout + out.stderr


def test_bench_rejects_world_mismatch():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr
