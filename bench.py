#!/usr/bin/env python3
"""bench.py -- distinct states/sec to exhaust a bounded 3-server Raft model.

A "step" is one complete model check of the workload: clear the fingerprint
set, Init, then BFS levels until no new state (TLC's "0 states left on
queue").  value = distinct states / mean wall time per step, the wall time
to exhaust being ms_per_step.  All inputs are device-resident (the search
starts from the Init row); nothing crosses PCIe inside a level except an
~100-byte counter read-back.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

N > 1 (launched by torch.distributed.run, one process per GPU): the search
is partitioned by fingerprint ownership -- each rank owns 1/N of the
fingerprint set, and every BFS level exchanges successor fingerprints with
their owners over RCCL (all-to-all-v on xGMI).  The model is fixed, so the
scaling is strong; value is the whole job's distinct states / wall time.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-tla_amd"))

# Feasible analogues of BASELINE.json configs (the reference's bounds give
# >1e11 states): name -> (N, V, MaxTerm, MaxLogLen, MaxCopies, MaxInFlight, invariants)
WORKLOADS = {
    "raft3_v2_t2_l2_m2": (3, 2, 2, 2, 1, 2, ("ElectionSafety", "LogMatching")),
    "raft3_v2_t2_l1_m3": (3, 2, 2, 1, 1, 3, ("ElectionSafety", "LogMatching")),
    "raft3_v2_t2_l1_m2": (3, 2, 2, 1, 1, 2, ("ElectionSafety", "LogMatching")),
    "raft3_v1_t2_l1_m2": (3, 1, 2, 1, 1, 2, ("NoTwoLeaders",)),
    "raft3_v1_t2_l1_m1": (3, 1, 2, 1, 1, 1, ("NoTwoLeaders",)),
}
DEFAULT = "raft3_v2_t2_l2_m2"
# fingerprint-set size per workload (distinct states: 2.41e9, 2.54e9, 1.45e8)
FPSET_LOG2 = {"raft3_v2_t2_l2_m2": 33, "raft3_v2_t2_l1_m3": 32, "raft3_v2_t2_l1_m2": 30}
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
# Random 8-byte fingerprint-set accesses into a 32 GiB table (far beyond the
# 256 MiB Infinity Cache), all CUs, measured on MI355X by tools/probe_calib.py
# (profiles/r01_v5/calib.log): CAS ~1.55e10/s (insert or
# present), load of a present key ~4.66e10/s.  The probe kernel loads the home
# slot and CASes only empty slots, so its ceiling for P probes of which D
# find new states is P / (P / LOAD + D / CAS).
CAS_PER_S = 1.55e10
LOAD_PER_S = 4.66e10


def load_traffic(workload, launches):
    """HBM bytes of the probe kernel per launch from the committed PMC profile
    (profiles/*/traffic.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes of this workload), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json"))):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if t.get("workload") == workload and t.get("kernel") == "k_expand_compact":
            best = t
            best["source"] = os.path.relpath(f, ROOT)
    return best


def fpset_log2_for(workload, world, override=0):
    """log2 fingerprint-set slots per rank: the workload's single-GPU size,
    divided by the next power of two >= world (each rank owns 1/world of the
    fingerprints, so the load stays ~28 %); an explicit override is per rank."""
    fpl = override or FPSET_LOG2.get(workload, 30)
    if not override and world > 1:
        fpl = max(24, fpl - (world - 1).bit_length())
    return fpl


def share_comm_id(rank, make_id):
    """Rank 0 creates the RCCL unique id, every rank receives it (gloo is the
    control plane only; the data path is the library's own communicator)."""
    import torch.distributed as dist
    box = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def max_over_ranks(x, world):
    """The job's time is the slowest rank's."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    tt = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def dist_env():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def cpu_baseline(shape, sample_states, threads):
    """The C oracle (oracle/raft_cpu.c, a 'port' of the spec) on a bounded
    prefix of the same BFS: distinct states/s on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import raft_cpu
    n, v, t, l, c, m, inv = shape
    r = raft_cpu.bfs(raft_cpu.cfg_of(n, v, t, l, c, m, inv, max_distinct=sample_states), threads=threads)
    return {"value": r["distinct"] / r["seconds"], "unit": "distinct states/s", "cores": threads,
            "kind": "port",
            "sample": "oracle/raft_cpu.c BFS of the same model, first %d levels (%d distinct, %d generated) in %.1f s"
                      % (len(r["levels"]), r["distinct"], r["generated"], r["seconds"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=DEFAULT, choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-sample", type=int, default=12_000_000, help="states in the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--fpset-log2", type=int, default=0,
                    help="log2 fingerprint-set slots per rank (TLC's -fpmem analogue); 0 = sized to the "
                         "workload (2^33 slots = 64 GiB for the 2.4e9-state default at 28%% load: 11%% faster "
                         "than 2^32 at 56%%, fewer long probe chains per wave, tools/fpset_sweep.sh; 2^34 leaves "
                         "too little HBM for the frontiers; fewer per rank when sharded)")
    ap.add_argument("--levels", action="store_true", help="print the per-level table to stderr")
    ap.add_argument("--shards", type=int, default=0,
                    help="diagnostic: split the search on one GPU into this many fingerprint-owned shards "
                         "(the multi-GPU exchange protocol with device copies as transport)")
    args = ap.parse_args()

    rank, world, local = dist_env()
    import rtla
    comm_id = None
    if world > 1:
        import torch.distributed as dist
        # gloo = control plane only (RCCL id broadcast, barriers, max-reduce of
        # times); the data path is the library's own RCCL communicator.
        dist.init_process_group("gloo")
        comm_id = share_comm_id(rank, rtla.comm_id)

    shape = WORKLOADS[args.workload]
    n, v, t, l, c, m, inv = shape
    fpl = fpset_log2_for(args.workload, world, args.fpset_log2)
    cfg = rtla.Config(n, v, t, l, c, m, inv, fpset_log2=fpl, shards=args.shards,
                      mem_budget=(200 << 30) if args.shards > 1 else 0)
    ck = rtla.Checker(cfg, rank=rank, world=world, comm_id=comm_id)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    def one_run():
        ck.reset()
        ck.run()
        if ck.status < 0 or ck.status == rtla.VIOLATION:
            raise SystemExit("model check ended with status %d" % ck.status)
        return ck.levels

    for _ in range(args.warmup):
        one_run()
    barrier()
    t0 = time.perf_counter()
    runs = []
    for _ in range(args.steps):
        runs.append(one_run())
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0, world)

    levels = runs[-1]
    distinct = sum(lv.new for lv in levels)
    generated = sum(lv.generated for lv in levels)
    depth = sum(1 for lv in levels if lv.new > 0)
    per_step = elapsed / args.steps
    value = distinct / per_step

    # Roofline of the dominant kernel, the probe kernel k_expand_compact, from
    # the last run's HIP-event times (expand_ms: the probe kernel alone; the
    # rest of kernel_ms is k_materialize building the new rows).
    # Algorithmic bytes of one launch over E frontier states: E*S (rows read)
    # + P*64 (one 64-B HBM transaction per fingerprint-set probe, P in-model
    # successors that differ from their parent) + D*8 (parent records).
    S = levels[0].row_bytes
    lv1 = levels[1:]
    launches = len(lv1)
    ems = sum(lv.expand_ms for lv in lv1)
    kms = sum(lv.kernel_ms for lv in lv1)
    E = sum(lv.frontier for lv in lv1)
    D = sum(lv.new for lv in lv1)
    P = sum(lv.probes for lv in lv1)
    probe_kernel_bytes = E * S + P * 64 + D * 8
    achieved = probe_kernel_bytes / world / (ems / 1e3) / 1e9   # per GPU
    mat_ms = kms - ems
    mat_bytes = D * (2 * S + 8)  # parent row read + record read + row written
    traffic = load_traffic(args.workload, launches) if world == 1 else None
    ra_ceiling = P / (P / LOAD_PER_S + D / CAS_PER_S) if P else LOAD_PER_S
    if args.levels and rank == 0:
        for lv in levels:
            print("level %3d frontier %12d new %12d generated %13d kernel %9.3f ms (probe %9.3f ms)" %
                  (lv.level, lv.frontier, lv.new, lv.generated, lv.kernel_ms, lv.expand_ms), file=sys.stderr)

    out = {
        "metric": "distinct states/sec (whole node) + wall time to exhaust, 3-server Raft",
        "value": value,
        "unit": "distinct states/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": per_step * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "exhaustive BFS from Init (no input data)",
        "config": {
            "workload": args.workload,
            "servers": n, "values": v, "max_term": t, "max_log": l, "max_copies": c, "max_in_flight": m,
            "invariants": list(inv), "distinct": distinct, "generated": generated, "depth": depth,
            "parallelism": "single" if world == 1 else "fp-sharded%d" % world,
            "fpset_slots_log2": fpl,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "traffic_source": traffic["source"] if traffic else None,
            "kernel": "k_expand_compact", "launches": launches, "kernel_ms_total": ems,
            "kernel_ms_avg": ems / max(1, launches),
            "bytes_per_launch": probe_kernel_bytes / max(1, launches),
            "bytes_per_frontier_state": probe_kernel_bytes / max(1, E),
            "model": "per launch: E*S rows read + 64 B per fingerprint-set probe + 8 B per new parent record",
            "random_access": {"probes_per_s": P / world / (ems / 1e3), "ceiling_per_s": ra_ceiling,
                              "frac": P / world / (ems / 1e3) / ra_ceiling,
                              "model": "load-first probes: P / (P / LOAD_PER_S + D / CAS_PER_S)",
                              "source": "tools/probe_calib.py on MI355X (profiles/r01_v5/calib.log)"},
            "k_materialize": {"ms_total": mat_ms, "bytes": mat_bytes,
                              "GB_per_s": mat_bytes / world / (mat_ms / 1e3) / 1e9 if mat_ms > 0 else None},
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(shape, args.cpu_sample, args.cpu_threads)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    ck.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
