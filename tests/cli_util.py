"""Helpers for the tests of the TLC-style command line (raft-tla_amd/rtla)."""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "raft-tla_amd", "rtla")
REF = "/root/reference"   # only where present (this container); never on the GPU box

STRINGS = """    Follower = "Follower"
    Candidate = "Candidate"
    Leader = "Leader"
    Nil = "Nil"
    RequestVoteRequest = "RequestVoteRequest"
    RequestVoteResponse = "RequestVoteResponse"
    AppendEntriesRequest = "AppendEntriesRequest"
    AppendEntriesResponse = "AppendEntriesResponse"
"""


def model_dir(tmp, n, v, t, l, c, m, invariants, constraint=True, symmetry=False, extra=""):
    """A directory holding specs/MC.tla and MC.cfg for the given bounds."""
    os.makedirs(tmp, exist_ok=True)
    shutil.copy(os.path.join(ROOT, "specs", "MC.tla"), os.path.join(tmp, "MC.tla"))
    lines = ["SPECIFICATION Spec"]
    if constraint:
        lines.append("CONSTRAINT StateConstraint")
    if invariants:
        lines.append("INVARIANTS " + " ".join(invariants))
    if symmetry:
        lines.append("SYMMETRY Perms")
    lines.append("CONSTANTS")
    lines.append("    Server = {%s}" % ", ".join("r%d" % (i + 1) for i in range(n)))
    lines.append("    Value = {%s}" % ", ".join("x%d" % (i + 1) for i in range(v)))
    cfg = "\n".join(lines) + "\n" + STRINGS
    cfg += "    MaxTerm = %d\n    MaxLogLen = %d\n    MaxCopies = %d\n    MaxInFlight = %d\n" % (t, l, c, m)
    cfg += extra
    open(os.path.join(tmp, "MC.cfg"), "w").write(cfg)
    return os.path.join(tmp, "MC.tla"), os.path.join(tmp, "MC.cfg")


def run(args, timeout=300, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([CLI] + args, capture_output=True, text=True, timeout=timeout, env=e)
