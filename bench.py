#!/usr/bin/env python3
"""bench.py -- distinct states/sec of the BFS over raft.tla's Next on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

Workloads:

* ``cfg2`` (default) -- BASELINE.json configs[1] exactly as stated: 3 servers,
  Value = {v1, v2}, currentTerm <= 3, Len(log) <= 2, <= 1 copy per message,
  ElectionSafety + LogMatching, NO in-flight bound.  Its state space grows ~3x
  per BFS level and does not fit one GPU (nor TLC), so a timed step is a BFS
  from Init through a fixed number of complete levels: the levels the CPU
  oracle pins (tests/golden/bfs_counts.json: 17 levels, 525,432,784 states,
  every level's counts and state set checked by the -m gpu suite).
  ``capacity`` says what the device memory holds beyond them (arena rows,
  fingerprint-set load, whether the next level's estimated size fits).
  value = distinct states found / wall time per step; ``exhausted`` is false.
  Workloads without a pinned depth (configs[3]) run until device memory is
  full: a sizing run finds the deepest level whose next level no longer fits
  (reported, never truncated), then every timed step runs exactly those
  levels.
* ``cfg1`` -- BASELINE.json configs[0], the bounds of the reference's raft.cfg
  (3 servers, one value, term <= 2, log <= 1, 1 copy), NoTwoLeaders; capped
  the same way.
* ``raft3_v2_t2_l2_m2`` and friends -- exhaustible analogues with a
  MaxInFlight bound (specs/MC.tla): a step is a complete model check (TLC's
  "0 states left on queue"), ms_per_step is the wall time to exhaust.  The
  default run adds this as the secondary ``exhaust`` object.

A "step" starts from the Init row on the device: no input crosses PCIe
inside the timed region except ~200-byte counter read-backs per level.

N > 1: one process per GPU (bench.py re-launches itself under
torch.distributed.run when WORLD_SIZE is unset), the search partitioned by
fingerprint ownership over RCCL (all-to-all-v on xGMI every level).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-tla_amd"))

ES_LM = ("ElectionSafety", "LogMatching")
# name -> (N, V, MaxTerm, MaxLogLen, MaxCopies, MaxInFlight, invariants)
WORKLOADS = {
    "cfg2": (3, 2, 3, 2, 1, 0, ES_LM),                     # BASELINE.json configs[1]
    "cfg1": (3, 1, 2, 1, 1, 0, ("NoTwoLeaders",)),         # BASELINE.json configs[0] (raft.cfg bounds)
    "raft3_v2_t2_l2_m2": (3, 2, 2, 2, 1, 2, ES_LM),
    "raft3_v2_t2_l1_m3": (3, 2, 2, 1, 1, 3, ES_LM),
    "raft3_v2_t2_l1_m2": (3, 2, 2, 1, 1, 2, ES_LM),
    "raft3_v1_t2_l1_m2": (3, 1, 2, 1, 1, 2, ("NoTwoLeaders",)),
    "raft3_v1_t2_l1_m1": (3, 1, 2, 1, 1, 1, ("NoTwoLeaders",)),
}
# BASELINE.json configs[2] (dup/drop live: 2 copies per message) and configs[3]
# (5 servers under SYMMETRY Permutations(Server)), as stated; both are capped
# by device memory like cfg1/cfg2.  configs[3] names no invariant.
WORKLOADS["cfg3"] = (3, 2, 4, 3, 2, 0, ())
WORKLOADS["cfg4"] = (5, 1, 3, 2, 1, 0, ())
SYMMETRIC = {"cfg4"}
# BASELINE.json configs[4]: random valid packed states in the cfg-3 layout
# (SURVEY.md section 8(d)): 3 servers, 2 values, term <= 4, log <= 3, 2 copies
WORKLOADS["synthetic"] = (3, 2, 4, 3, 2, 0, ES_LM)
BASELINE_INDEX = {"cfg1": 0, "cfg2": 1, "cfg3": 2, "cfg4": 3, "synthetic": 4}
CAPPED = {"cfg1", "cfg2", "cfg3", "cfg4"}  # not exhaustible on one GPU
# Complete levels of each capped workload that the CPU oracle pins (per-level
# counts and state-set digests in tests/golden/bfs_counts.json): a timed step
# runs exactly these (--depth fit: as many as device memory holds instead).
PINNED_LEVELS = {"cfg1": 23, "cfg2": 17, "cfg3": 14, "cfg4": 15}
DEFAULT = "cfg2"
SECONDARY = "raft3_v2_t2_l2_m2"    # wall time to exhaust (the default run reports it too)
# Fingerprint-set size (log2 slots) per workload.  configs[0]-[2]: 2^32 slots
# (32 GiB; 7-14 % load at the pinned depth) -- fewer second-slot probes and
# CAS misses than 2^31 (12-28 %) beat clearing twice the bytes per step
# (configs[1] 197.2 -> 192.1 ms, configs[0] 300.9 -> 291.1, configs[2] 90.0 ->
# 88.4; 2^33: 194.9 ms, the clear grows faster; profiles/r04_v4/fpset_*.json).
FPSET_LOG2 = {"raft3_v2_t2_l2_m2": 33, "raft3_v2_t2_l1_m3": 32, "raft3_v2_t2_l1_m2": 30,
              "cfg2": 32, "cfg1": 32, "cfg3": 32, "cfg4": 30,
              # 1e9 inputs with a 1e8 pool find ~8.6e9 distinct successor fingerprints: 2^34 slots
              # (128 GiB, ~50 % load) on one GPU; N ranks each 1/N of the inputs in 2^34 / N
              "synthetic": 34}
# Bag slots per row for the unbounded-bag configs.  A state d BFS levels below
# Init holds at most d - 1 distinct messages (every action adds at most one),
# so this bounds the depth at which the row format -- not memory -- stops the
# search; a successor that needs more raises RTLA_CAP_ROW, never truncates.
BAG_CAP = {"cfg2": 18, "cfg1": 24, "cfg3": 20, "cfg4": 20, "synthetic": 12}
# Synthetic microbench: 1e9 input states over the whole job,
# half of them redrawn from a pool of 1e8 (so dedup has hits); states
# generated per device batch.
SYNTH_TOTAL = 1_000_000_000
SYNTH_POOL = 100_000_000
SYNTH_BATCH = 1 << 24
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
# Pure-stream rates of random 8-byte fingerprint-set accesses into a 32 GiB
# table, all CUs, measured on MI355X by tools/probe_calib.py
# (profiles/r01_v5/calib.log): CAS ~1.55e10/s, load of a present key
# ~4.66e10/s.  Only the fallback model P / (P / LOAD + D / CAS) when the live
# calibration is skipped (--no-calib): the random-access ceiling is MEASURED
# in the same run (calibrate_probes), on a mixed stream at the workload's own
# insert fraction.
CAS_PER_S = 1.55e10
LOAD_PER_S = 4.66e10


def load_traffic(workload):
    """HBM bytes of the level kernel per launch from the newest committed PMC
    profile of this workload (profiles/<round>/traffic*.json, written by
    tools/prof_summary.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3
    passes), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic*.json"))):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if t.get("workload") == workload and t.get("kernel") == "k_expand_compact":
            best = t
            best["source"] = os.path.relpath(f, ROOT)
    return best


def fpset_log2_for(workload, world, override=0, shards=0, pinned=True):
    """log2 fingerprint-set slots per rank (per shard): the workload's
    single-GPU size, divided by the next power of two >= world (each rank owns
    1/world of the fingerprints, so the load stays ~28 %); an explicit override
    is per rank.  A capped workload run to the depth that fits (--depth fit,
    not `pinned`) keeps the single-GPU size per rank: with more GPUs it
    reaches deeper levels.  Virtual shards on one GPU (--shards S) split the
    single-GPU set S ways, as S ranks would."""
    fpl = override or FPSET_LOG2.get(workload, 30)
    # (the synthetic microbench's ranks are replicas, each with its own set: its 2^34 slots stay per rank)
    if not override and world > 1 and (workload not in CAPPED or pinned) and workload != "synthetic":
        fpl = max(24, fpl - (world - 1).bit_length())
    if not override and shards > 1:
        fpl = max(24, fpl - (shards - 1).bit_length())
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


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc, argv):
    """--gpus N without a launcher: run N ranks of this script under
    torch.distributed.run as a CHILD process (nothing here has touched the
    GPU, and the parent never execs), relay its output and exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + argv
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cgroup v2
    cpu.max / v1 cfs quota), or None when unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def cpu_threads():
    """Host threads for the CPU baseline: every CPU this process may run on
    (affinity), capped by the cgroup's CPU quota -- on the GPU box nproc shows
    the whole machine but the job gets a share of it; more threads than the
    share only adds contention."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cpu_quota()
    if q:
        n = min(n, max(1, int(q + 0.999)))
    return n


def cpu_baseline(shape, sample_states, threads):
    """The C oracle (oracle/raft_cpu.c, a 'port' of the spec) on a bounded
    prefix of the same BFS: distinct states/s on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import raft_cpu
    n, v, t, l, c, m, inv = shape
    r = raft_cpu.bfs(raft_cpu.cfg_of(n, v, t, l, c, m, inv, max_distinct=sample_states), threads=threads)
    return {"value": r["distinct"] / r["seconds"], "unit": "distinct states/s", "cores": threads,
            "host_cpus": os.cpu_count(), "cgroup_cpu_quota": cpu_quota(), "kind": "port", "levels": len(r["levels"]),
            "sample": "prefix rate: oracle/raft_cpu.c level-synchronous BFS of the same model, first %d levels "
                      "(%d distinct, %d generated) in %.1f s on %d threads"
                      % (len(r["levels"]), r["distinct"], r["generated"], r["seconds"], threads)}


def cpu_baseline_synthetic(rtla, cfg, pool, threads, target_s=12.0):
    """The synthetic microbench's CPU leg: the same random input states
    (rtla_random_texts: the generator's rows printed as state text) parsed by
    the C oracle, then -- the timed phase -- run through Next + dedup into
    one seen set (oracle/raft_cpu.c orc_dedup_texts; the parse is untimed, as
    the GPU leg is handed packed rows) -- batches until ~target_s seconds of
    timed oracle work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import raft_cpu
    n, v, t, l, c, m, inv = WORKLOADS["synthetic"]
    d = raft_cpu.Dedup(raft_cpu.cfg_of(n, v, t, l, c, m, inv))
    first, batch = 0, 1 << 16
    while d.seconds < target_s and first < (16 << 20):
        d.batch(rtla.random_texts(cfg, first, batch, pool), batch, threads)
        first += batch
    gen, probes, new = d.counts
    d.close()
    return {"value": first / d.seconds, "unit": "input states/s", "cores": threads,
            "host_cpus": os.cpu_count(), "cgroup_cpu_quota": cpu_quota(), "kind": "port",
            "sample": "input states 0..%d of the same generator (pool %d), oracle/raft_cpu.c Next + dedup on %d "
                      "threads: %d generated, %d probes, %d new in %.1f s" % (first - 1, pool, threads, gen, probes,
                                                                             new, d.seconds)}


class Run:
    """A checker context for one workload, and how to time it."""

    def __init__(self, rtla, name, rank, world, comm_id, args, frontier_cap=0):
        self.rtla = rtla
        self.name = name
        self.shape = WORKLOADS[name]
        self.capped = name in CAPPED
        n, v, t, l, c, m, inv = self.shape
        self.fpl = fpset_log2_for(name, world, args.fpset_log2, args.shards,
                                  pinned=args.depth == "pinned" and name in PINNED_LEVELS)
        self.cfg = rtla.Config(n, v, t, l, c, m, inv, fpset_log2=self.fpl, shards=args.shards,
                               bag_cap=BAG_CAP.get(name, 0), frontier_cap=frontier_cap,
                               symmetry=name in SYMMETRIC, dedup_only=name == "synthetic",
                               mem_budget=(args.mem_budget << 30) if args.mem_budget else
                               (200 << 30) if args.shards > 1 else 0, chunk=args.chunk)
        self.ck = rtla.Checker(self.cfg, rank=rank, world=world, comm_id=comm_id)
        self.levels_cap = None   # complete levels a capped search reaches
        self.pinned = PINNED_LEVELS.get(name) if args.depth == "pinned" else None
        self.stop = None         # what stopped the sizing run
        self.exhausted = False

    def size(self):
        """Capped workloads: BFS until the next level does not fit; the timed
        steps then run exactly the complete levels before it."""
        ck = self.ck
        ck.reset()
        st = ck.init()
        while st == self.rtla.OK:
            try:
                st = ck.step()
                progress("%s sizing: level %d, %d distinct" % (self.name, len(ck.levels), ck.distinct))
            except self.rtla.RtlaError as e:
                if e.status != -3:  # only capacity may stop a capped search
                    raise
                self.stop = str(e)
                break
        if st == self.rtla.VIOLATION:
            raise SystemExit("%s: invariant violated" % self.name)
        self.levels_cap = len(ck.levels)
        self.exhausted = st == self.rtla.DONE

    def one(self):
        ck = self.ck
        ck.reset()
        if self.capped:
            st = ck.init()
            while st == self.rtla.OK and len(ck.levels) < self.levels_cap:
                st = ck.step()
        else:
            st = ck.run()
        if st < 0 or st == self.rtla.VIOLATION:
            raise SystemExit("%s: model check ended with status %d" % (self.name, st))
        return ck.levels


def progress(msg):
    """A progress line on stderr (long runs keep writing: a silent GPU job is taken to be hung)."""
    if dist_env()[0] == 0:
        print("bench.py: " + msg, file=sys.stderr, flush=True)


def timed(run, steps, warmup, world, barrier, cap_levels=0):
    if run.capped and cap_levels:
        run.levels_cap, run.exhausted, run.stop = cap_levels, False, "--cap-levels %d" % cap_levels
    elif run.capped and run.pinned:
        run.levels_cap, run.exhausted, run.stop = run.pinned, False, "oracle-pinned depth (%d levels)" % run.pinned
    elif run.capped:
        run.size()
    for w in range(warmup):
        run.one()
        progress("%s warmup %d/%d" % (run.name, w + 1, warmup))
    barrier()
    t0 = time.perf_counter()
    levels = None
    for _ in range(steps):
        levels = run.one()
    t1 = time.perf_counter()
    progress("%s timed %d steps: %.1f ms/step" % (run.name, steps, (t1 - t0) / steps * 1e3))
    barrier()
    return max_over_ranks(t1 - t0, world) / steps, levels


def calibrate_probes(fpl, n_present, probes, new):
    """The random-access ceiling, measured live (rtla_probe_bench3): a table
    of the workload's size (2^fpl slots) holding n_present keys -- what the
    fingerprint set holds when the run's largest level kernel starts -- then
    a timed stream of uniformly random load-first probes (load the home slot,
    CAS only an empty one), a fraction new / probes of them new keys: the
    level kernel's own mix.  Probes/s of that stream = the ceiling."""
    import rtla
    n = int(min(max(probes, 1 << 24), 1 << 30))
    q = new / probes if probes else 0.0
    n_present = int(min(n_present, (1 << fpl) // 2))
    sec, ins = rtla.probe_mixed(fpl, n_present, n, q)
    return {"ceiling_per_s": n / sec, "new_frac": q, "table_slots_log2": fpl, "present_keys": n_present,
            "probes": n, "inserted": ins, "seconds": sec,
            "source": "live: rtla_probe_bench3 (uniform random load-first probes, CAS on an empty slot, "
                      "this run, this GPU)"}


def calib_inputs(levels):
    """(keys in the set when the largest level kernel starts, probes, new) of a run."""
    lv1 = levels[1:]
    big = max(range(len(lv1)), key=lambda k: lv1[k].probes) if lv1 else 0
    present = sum(lv.new for lv in levels[:big + 1])
    return present, sum(lv.probes for lv in lv1), sum(lv.new for lv in lv1)


def roofline(levels, world, workload, calib=None):
    """Roofline of the dominant kernel -- k_expand_compact, the whole BFS
    level (expand, fingerprint, probe, insert, build the new rows) -- from
    the last run's HIP-event times around it (expand_ms).  Algorithmic bytes
    of one launch over E frontier states: E*S (rows read) + P*64 (one 64-B HBM
    transaction per fingerprint-set probe, P = in-model successors that differ
    from their parent) + D*(S+8) (new rows and their parent records written)."""
    S = levels[0].row_bytes
    lv1 = levels[1:]
    launches = len(lv1)
    ems = sum(lv.expand_ms for lv in lv1)
    E = sum(lv.frontier for lv in lv1)
    D = sum(lv.new for lv in lv1)
    P = sum(lv.probes for lv in lv1)
    kernel_bytes = E * S + P * 64 + D * (S + 8)
    achieved = kernel_bytes / world / (ems / 1e3) / 1e9   # per GPU
    traffic = load_traffic(workload) if world == 1 else None
    if calib:
        ra_ceiling, ra_model, ra_source = calib["ceiling_per_s"], "measured mixed stream (calibration)", calib["source"]
    else:
        ra_ceiling = P / (P / LOAD_PER_S + D / CAS_PER_S) if P else LOAD_PER_S
        ra_model = "load-first probes: P / (P / LOAD_PER_S + D / CAS_PER_S) (--no-calib fallback)"
        ra_source = "tools/probe_calib.py on MI355X (profiles/r01_v5/calib.log)"
    return {
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic["bytes_per_launch"] if traffic else None,
        "traffic_source": traffic["source"] if traffic else None,
        "kernel": "k_expand_compact", "launches": launches, "kernel_ms_total": ems,
        "kernel_ms_avg": ems / max(1, launches),
        "bytes_per_launch": kernel_bytes / max(1, launches),
        "bytes_per_frontier_state": kernel_bytes / max(1, E),
        "model": "per launch: E*S rows read + 64 B per fingerprint-set probe + D*(S+8) new rows and parent records",
        "random_access": {"probes_per_s": P / world / (ems / 1e3), "ceiling_per_s": ra_ceiling,
                          "frac": P / world / (ems / 1e3) / ra_ceiling,
                          "model": ra_model, "source": ra_source, "calibration": calib},
    }


def capacity(levels, info, fpl, parts=1):
    """What device memory holds beyond the timed levels: the frontier arena
    (current + next level share it), the fingerprint set's load, and whether
    the next level -- estimated from the last level's growth -- would fit.
    Arena rows and set slots are per shard (rank or virtual shard); the
    level counts are the job's, so they are split over the `parts` shards
    (fingerprint ownership and the level-end re-balancing keep the shards
    even)."""
    rows = info.get("frontier_cap") or 0
    last, prev = levels[-1].new, levels[-2].new if len(levels) > 1 else 1
    est_next = int(last * last / max(1, prev))
    distinct = sum(lv.new for lv in levels)
    per = lambda v: -(-v // max(1, parts))  # ceil(v / parts)
    return {"arena_rows": rows, "row_bytes": levels[0].row_bytes, "fpset_slots_log2": fpl, "shards": parts,
            "fpset_load": per(distinct) / float(1 << fpl), "last_level": last, "next_level_estimate": est_next,
            "next_level_fits_arena": rows >= ((per(last) + 63) // 64) * 64 + per(est_next),
            "fpset_load_after_next": per(distinct + est_next) / float(1 << fpl)}


def synthetic(run, args, rank, world, barrier):
    """BASELINE configs[4]: 1e9 input states over the job,
    each rank its own 1/N of the input numbering (input i is state
    synth_state_id(i): half of them redrawn from the job-wide 1e8 pool).  A
    step clears the rank's fingerprint set and runs every input through Next
    + fingerprint + dedup (level-kernel launches in dedup-only mode) into it.
    The inputs are generated on the device into the row arena in passes of
    as many rows as it holds (at N = 1 the 1e9 x 252 B do not fit HBM beside
    the set): each pass is generated OUTSIDE the timed region (a single pass
    once, before all steps), so every timed dedup runs over HBM-resident rows.
    With several ranks each deduplicates its own inputs (replicas: no
    exchange; 'parallelism' says so)."""
    n = args.synth_states // world
    first0 = rank * n
    rows = int(json.loads(run.ck.device_info())["frontier_cap"])
    per = min(n, rows) // 64 * 64
    passes = [(b, min(per, n - b)) for b in range(0, n, per)]

    def generate(b, m):
        for g in range(0, m, SYNTH_BATCH):
            run.ck.synthetic_generate(first0 + b + g, min(SYNTH_BATCH, m - g), args.synth_pool, at=g)

    if len(passes) == 1:
        generate(*passes[0])

    def one():
        t = time.perf_counter()
        run.ck.reset()
        timed_s = time.perf_counter() - t
        tot = {"generated": 0, "probes": 0, "new": 0, "kernel_ms": 0.0, "batches": len(passes)}
        for b, m in passes:
            if len(passes) > 1:
                generate(b, m)  # (untimed)
            t = time.perf_counter()
            lv = run.ck.synthetic_dedup(0, m)
            timed_s += time.perf_counter() - t
            tot["generated"] += lv.generated
            tot["probes"] += lv.probes
            tot["new"] += lv.new
            tot["kernel_ms"] += lv.kernel_ms
        return timed_s, tot

    for _ in range(args.warmup):
        one()
    barrier()
    timed = 0.0
    for _ in range(args.steps):
        dt, tot = one()
        timed += dt
    barrier()
    return max_over_ranks(timed, world) / args.steps, tot, n, per


def print_levels(name, levels):
    for lv in levels:
        print("%s level %3d frontier %12d new %12d generated %13d kernel %9.3f ms" %
              (name, lv.level, lv.frontier, lv.new, lv.generated, lv.expand_ms), file=sys.stderr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default=DEFAULT, choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="distinct states in the CPU baseline sample (0 = per workload, ~10-30 s of CPU work)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary wall-time-to-exhaust line of the default run")
    ap.add_argument("--fpset-log2", type=int, default=0,
                    help="log2 fingerprint-set slots per rank (TLC's -fpmem analogue); 0 = sized to the workload")
    ap.add_argument("--frontier-cap", type=int, default=0, help="rows of the frontier arena per rank (0 = auto)")
    ap.add_argument("--mem-budget", type=int, default=0,
                    help="device memory per rank in GiB (0 = 85 %% of what is free; several ranks sharing one GPU, "
                         "e.g. over RTLA_TRANSPORT=shm, need a share each)")
    ap.add_argument("--levels", action="store_true", help="print the per-level tables to stderr")
    ap.add_argument("--synth-states", type=int, default=SYNTH_TOTAL,
                    help="synthetic workload: input states of the whole job (split over the ranks)")
    ap.add_argument("--synth-pool", type=int, default=SYNTH_POOL,
                    help="synthetic workload: half the inputs are redrawn from a pool of this many states")
    ap.add_argument("--depth", choices=("pinned", "fit"), default="pinned",
                    help="capped workloads: the oracle-pinned levels (default), or as many as device memory holds")
    ap.add_argument("--cap-levels", type=int, default=0,
                    help="capped workloads: run exactly this many complete levels and skip the sizing run "
                         "(profiling; a level that does not fit is still an error)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / rendezvous check only: every rank joins the process group, receives rank 0's "
                         "RCCL-id payload, prints one line and exits (no GPU work; used by the CPU tests)")
    ap.add_argument("--no-calib", action="store_true",
                    help="skip the live random-access calibration (the ceiling then comes from the pure-stream model)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="multi-shard: frontier states per shard per exchange round (0 = sized from the budget)")
    ap.add_argument("--shards", type=int, default=0,
                    help="diagnostic: split the search on one GPU into this many fingerprint-owned shards "
                         "(the multi-GPU exchange protocol with device copies as transport)")
    args = ap.parse_args()

    rank, world, local = dist_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))

    if args.dry_run:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            cid = share_comm_id(rank, lambda: bytes(range(128)))
            dist.barrier()
            dist.destroy_process_group()
        else:
            cid = bytes(range(128))
        sys.stdout.write("bench.py rank %d of %d ready (id %s)\n" % (rank, world, cid[:4].hex()))  # one write per line
        sys.stdout.flush()
        return
    import rtla
    comm_id = None
    if world > 1:
        import torch.distributed as dist
        # gloo = control plane only (RCCL id broadcast, barriers, max-reduce of
        # times); the data path is the library's own RCCL communicator.
        dist.init_process_group("gloo")
        comm_id = share_comm_id(rank, rtla.comm_id)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    run = Run(rtla, args.workload, rank, world, comm_id, args, args.frontier_cap)
    info = json.loads(run.ck.device_info())
    if args.workload == "synthetic":
        per_step, tot, n, per = synthetic(run, args, rank, world, barrier)
        pool = args.synth_pool
        S = run.ck.levels[0].row_bytes if run.ck.levels else 4 * rtla.row_words(run.cfg)
        ems = tot["kernel_ms"]
        P, D = tot["probes"], tot["new"]
        kbytes = n * S + P * 64
        straffic = load_traffic("synthetic")
        run.ck.close()
        calib = None if args.no_calib else calibrate_probes(run.fpl, D // 2, P, D)
        ra = calib["ceiling_per_s"] if calib else (P / (P / LOAD_PER_S + D / CAS_PER_S) if P else LOAD_PER_S)
        out = {
            "metric": "random packed states/sec through Next + fingerprint + dedup (BASELINE configs[4])",
            "value": n * world / per_step, "unit": "input states/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": per_step * 1e3, "higher_is_better": True,
            "scaling": "strong",  # 1e9 inputs over the job at every N
            "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: counter-based PRNG (seed 0x5AF72025) valid random states, 1/2 redrawn from a "
                    "job-wide pool of %d" % pool,
            "config": {"workload": "synthetic", "baseline_config": 4, "layout": "cfg-3: N3 V2 T4 L3 C2, bag_cap 12",
                       "input_states": n * world, "input_states_per_gpu": n, "pool": pool,
                       "resident_rows_per_pass": per, "passes_per_step": tot["batches"],
                       "inputs": ("generated once before the timed steps, resident in HBM" if tot["batches"] == 1 else
                                  "generated on the device into the row arena before each dedup pass, outside the "
                                  "timed region (%d x %d B do not fit HBM beside the set): every timed pass runs "
                                  "over resident rows" % (n, S)),
                       "timed": "per step: the fingerprint-set clear + every dedup pass",
                       "launches_per_step": tot["batches"],
                       "generated": tot["generated"], "probes": P, "distinct_successors": D,
                       "successors_per_s": tot["generated"] * world / per_step, "row_bytes": S,
                       "fpset_slots_log2": run.fpl, "fpset_load": D / float(1 << run.fpl),
                       "parallelism": "single" if world == 1 else
                       "replicas%d (each rank deduplicates its own 1/N of the inputs; no exchange)" % world},
            "roofline": {"bound": "hbm", "achieved": kbytes / (ems / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": kbytes / (ems / 1e3) / 1e9 / HBM_PEAK_GBS,
                         "traffic": straffic["bytes_per_launch"] if straffic else None,
                         "traffic_source": straffic["source"] if straffic else None,
                         "kernel": "k_expand_compact (XF_DEDUP_ONLY)", "launches": tot["batches"],
                         "kernel_ms_total": ems, "kernel_ms_avg": ems / max(1, tot["batches"]),
                         "bytes_per_launch": kbytes / max(1, tot["batches"]),
                         "model": "per launch: E*S input rows read + 64 B per fingerprint-set probe",
                         "random_access": {"probes_per_s": P / (ems / 1e3), "ceiling_per_s": ra,
                                           "frac": P / (ems / 1e3) / ra, "calibration": calib}},
            "cpu_baseline": None,
        }
        if rank == 0 and world == 1 and not args.no_cpu:
            try:
                out["cpu_baseline"] = cpu_baseline_synthetic(rtla, run.cfg, pool, args.cpu_threads or cpu_threads())
            except Exception as e:  # reported, never fatal for the GPU number
                out["cpu_baseline"] = {"error": str(e)}
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    per_step, levels = timed(run, args.steps, args.warmup, world, barrier, args.cap_levels)
    distinct = sum(lv.new for lv in levels)
    generated = sum(lv.generated for lv in levels)
    depth = sum(1 for lv in levels if lv.new > 0)
    if args.levels and rank == 0:
        print_levels(args.workload, levels)
    n, v, t, l, c, m, inv = run.shape
    config = {
        "workload": args.workload,
        "baseline_config": BASELINE_INDEX.get(args.workload),
        "servers": n, "values": v, "max_term": t, "max_log": l, "max_copies": c, "max_in_flight": m,
        "invariants": list(inv), "distinct": distinct, "generated": generated, "depth": depth,
        "exhausted": (not run.capped) or bool(run.exhausted), "levels": len(levels),
        "parallelism": "single" if world == 1 else "fp-sharded%d" % world,
        "fpset_slots_log2": run.fpl, "bag_cap": run.cfg.bag_cap or None, "symmetry": run.cfg.symmetry,
        "frontier_arena_rows": info.get("frontier_cap"), "row_bytes": levels[0].row_bytes,
        "rccl_ranks": info.get("world"),
    }
    if world > 1 or args.shards > 1:  # the exchange over the whole run (warmup and timed steps, this rank)
        fin = json.loads(run.ck.device_info())
        config["exchange"] = {k: fin.get(k) for k in ("exchange_rounds", "records_sent", "overflowed_records",
                                                      "outbox_records_per_owner", "sent_cache_slots_log2",
                                                      "rebalanced_rows", "chunk")}
        config["exchange"]["steps_counted"] = args.steps + args.warmup
    if run.capped:
        config["stopped_by"] = run.stop
        config["oracle_pinned"] = bool(run.pinned) and not args.cap_levels
        config["capacity"] = capacity(levels, info, run.fpl, max(1, world) * max(1, args.shards))
    out = {
        "metric": "distinct states/sec (whole node) + wall time to exhaust, 3-server Raft",
        "value": distinct / per_step,
        "unit": "distinct states/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": per_step * 1e3,
        "higher_is_better": True,
        # the same levels at every GPU count (oracle-pinned / --cap-levels, or a
        # complete model check): strong scaling; --depth fit reaches deeper
        # levels with more GPUs' memory: weak
        "scaling": "weak" if run.capped and not run.pinned and not args.cap_levels else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "BFS from the Init row (no input data)" + (
            (", the oracle-pinned depth (%d complete levels, every level's counts and state set in "
             "tests/golden/bfs_counts.json)" % run.levels_cap) if run.capped and run.pinned and not args.cap_levels else
            (", %d complete levels (--cap-levels)" % run.levels_cap) if run.capped and args.cap_levels else
            ", capped at the deepest level that fits device memory" if run.capped else ", exhaustive"),
        "config": config,
        "cpu_baseline": None,
    }
    run.ck.close()
    calib = None if args.no_calib else calibrate_probes(run.fpl, *calib_inputs(levels))
    out["roofline"] = roofline(levels, world, args.workload, calib)

    if args.workload == DEFAULT and not args.no_secondary:
        sec = Run(rtla, SECONDARY, rank, world, comm_id, args)
        sec_step, sec_levels = timed(sec, args.steps, args.warmup, world, barrier)
        if args.levels and rank == 0:
            print_levels(SECONDARY, sec_levels)
        d2 = sum(lv.new for lv in sec_levels)
        out["exhaust"] = {"workload": SECONDARY, "shape": list(WORKLOADS[SECONDARY][:6]),
                          "wall_s_to_exhaust": sec_step, "distinct": d2,
                          "generated": sum(lv.generated for lv in sec_levels),
                          "depth": sum(1 for lv in sec_levels if lv.new > 0),
                          "distinct_per_s": d2 / sec_step}
        sec.ck.close()
        scal = None if args.no_calib else calibrate_probes(sec.fpl, *calib_inputs(sec_levels))
        out["exhaust"]["probe_kernel"] = roofline(sec_levels, world, SECONDARY, scal)

    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            sample = args.cpu_sample or (20_000_000 if run.capped else 12_000_000)
            cb = cpu_baseline(run.shape, sample, args.cpu_threads or cpu_threads())
            k = cb["levels"]  # the GPU's own rate over the same prefix of levels, for comparison
            if k <= len(levels):
                gsec = sum(lv.seconds for lv in levels[:k])
                cb["gpu_same_prefix_value"] = sum(lv.new for lv in levels[:k]) / gsec if gsec > 0 else None
            out["cpu_baseline"] = cb
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"error": str(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
