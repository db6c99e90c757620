"""One rank of a world-size-N BFS (test helper, run as a child process by
test_gpu.py::test_ranks_over_shm_transport_match_golden with
RTLA_TRANSPORT=shm, or over RCCL by tools/gpu_rccl_pair.sh): rank 0 writes the
RCCL unique id to a file, the other ranks poll for it -- the CLI's
rendezvous -- then every rank runs the golden model and rank 0 prints the
per-level counts as JSON.  Ranks share the device when the box has fewer
GPUs than ranks (device = rank % device count)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raft-tla_amd"))
import rtla  # noqa: E402


def main():
    rank, world, idfile, name = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bfs_counts.json")))[name]
    if rank == 0:
        cid = rtla.comm_id()
        with open(idfile + ".tmp", "wb") as f:
            f.write(cid)
        os.rename(idfile + ".tmp", idfile)
    else:
        t0 = time.time()
        while not os.path.exists(idfile):
            if time.time() - t0 > 60:
                raise SystemExit("rank %d: no RCCL id after 60 s" % rank)
            time.sleep(0.05)
        cid = open(idfile, "rb").read()
    log2 = max(16, (int(g["distinct"] * 2)).bit_length())
    # RCCL_PAIR_BUDGET_STEP: rank r gets r * STEP more bytes (ranks whose own
    # sizing differs must still agree on the exchange sizes)
    budget = (8 << log2) * 3 + (1 << 29) + rank * int(os.environ.get("RCCL_PAIR_BUDGET_STEP", "0"))
    cfg = rtla.Config(g["n_server"], g["n_value"], g["max_term"], g["max_log"], g["max_copies"], g["max_msgs"],
                      tuple(g["invariants"]), fpset_log2=log2, mem_budget=budget,
                      symmetry=bool(g.get("symmetry", False)), chunk=int(os.environ.get("RCCL_PAIR_CHUNK", "0")))
    levels = []
    if os.environ.get("RCCL_PAIR_MODE") == "recover_missing":
        # checkpoint after 3 levels, the last rank loses its file, every rank
        # recovers: all must fail, promptly (no rank left waiting)
        prefix = sys.argv[5]
        with rtla.Checker(cfg, rank=rank, world=world, comm_id=cid) as ck:
            ck.init()
            for _ in range(3):
                ck.step()
            ck.checkpoint(prefix)
            if rank == world - 1:
                os.remove("%s.shard%d.rtla" % (prefix, rank))
            t0 = time.time()
            try:
                ck.recover(prefix)
                out = {"rank": rank, "recover": 0}
            except rtla.RtlaError as e:
                out = {"rank": rank, "recover": e.status}
            out["seconds"] = time.time() - t0
        print(json.dumps(out), flush=True)
        return
    mode = os.environ.get("RCCL_PAIR_MODE", "")
    if mode.startswith("fault_"):
        # RTLA_FAULT=<where>:<rank> makes that rank's local work at <where>
        # fail: every rank must return an error from the same call, promptly
        # (the failure travels in the call's reductions)
        where = mode[len("fault_"):]
        out = {"rank": rank}
        with rtla.Checker(cfg, rank=rank, world=world, comm_id=cid) as ck:
            st = ck.init()
            t0 = time.time()
            try:
                while st == rtla.OK:
                    st = ck.step()
                out["step"] = st
            except rtla.RtlaError as e:
                out["step"] = e.status
            if where != "exchange":
                t0 = time.time()
                try:
                    if where == "coverage":
                        ck.coverage()
                    else:
                        ck.trace()
                    out[where] = 0
                except rtla.RtlaError as e:
                    out[where] = e.status
            out["seconds"] = time.time() - t0
        print(json.dumps(out), flush=True)
        return
    with rtla.Checker(cfg, rank=rank, world=world, comm_id=cid) as ck:
        st = ck.init()
        while st == rtla.OK:
            st = ck.step()
        levels = [[lv.new, lv.generated] for lv in ck.levels]
        trace = ck.trace() if st == rtla.VIOLATION else []  # collective: every rank walks it
        out = {"rank": rank, "levels": levels, "distinct": ck.distinct, "generated": ck.generated,
               "status": st, "trace": trace, "info": ck.device_info()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
