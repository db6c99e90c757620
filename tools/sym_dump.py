"""Sample configs[3] (SYMMETRY) states for the orbit-key statistics tool
(tools/symstat.cpp): BFS to --level, copy the frontier, draw --n parents at
random, generate their successors on the GPU (rtla_expand_batch), save
parents and in-model successors (with instance numbers) as .npy files."""
import argparse, ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raft-tla_amd"))
import rtla

ap = argparse.ArgumentParser()
ap.add_argument("--level", type=int, default=14)
ap.add_argument("--n", type=int, default=4000)
ap.add_argument("--out", default="gpurun_out/symdump")
a = ap.parse_args()
cfg = rtla.Config(n_server=5, n_value=1, max_term=3, max_log=2, max_copies=1, max_msgs=0, invariants=(),
                  symmetry=True, bag_cap=20, fpset_log2=30)
ck = rtla.Checker(cfg)
st = ck.init()
while len(ck.levels) < a.level:
    ck.step()
w = rtla.row_words(cfg)
n = C.c_size_t(0)
rtla._lib.rtla_frontier(ck._h, None, 0, C.byref(n))
buf = np.zeros(n.value * w, dtype=np.uint32)
rtla._check(rtla._lib.rtla_frontier(ck._h, buf.ctypes.data_as(C.POINTER(C.c_uint32)), n.value, C.byref(n)),
            "rtla_frontier")
rows = buf.reshape(-1, w)
rng = np.random.default_rng(1)
pick = rng.choice(rows.shape[0], size=min(a.n, rows.shape[0]), replace=False)
par = rows[np.sort(pick)]
succ = rtla.expand_batch(cfg, [list(map(int, r)) for r in par])
keep = [s for s in succ if s[3]]
os.makedirs(a.out, exist_ok=True)
np.save(os.path.join(a.out, "parents.npy"), par)
np.save(os.path.join(a.out, "succ.npy"), np.array([s[4] for s in keep], dtype=np.uint32))
np.save(os.path.join(a.out, "succ_info.npy"), np.array([(s[0], s[1], s[2]) for s in keep], dtype=np.int64))
print("level", a.level, "frontier", rows.shape[0], "parents", par.shape[0], "successors", len(keep))
