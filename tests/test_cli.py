"""CPU tests of the TLC-style command line (raft-tla_amd/rtla): the parts of
TLC's contract that are decided before any GPU work -- spec identity (sha256
of raft.tla), cfg grammar and operator checks, exit codes -- and the -gpus
launcher.  Reference: raft.cfg:1-15 (the model), .vscode/settings.json:5
(the "-coverage 1" invocation)."""
import os
import shutil

import pytest

from cli_util import CLI, REF, model_dir, run

pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="build raft-tla_amd/rtla first")
HAVE_REF = os.path.exists(os.path.join(REF, "raft.tla"))


@pytest.mark.skipif(not HAVE_REF, reason="reference not mounted")
def test_reference_cfg_names_an_undefined_invariant():
    """raft.cfg:3 asks for INVARIANT NoTwoLeaders, which raft.tla never
    defines: TLC stops with this error, and so does rtla (after verifying the
    spec's identity, which the reference's own raft.tla passes)."""
    r = run(["-config", os.path.join(REF, "raft.cfg"), os.path.join(REF, "raft.tla")])
    assert r.returncode == 150, r.stdout + r.stderr
    assert "raft.tla sha256 683a120af29e... verified" in r.stdout
    assert ("Error: The invariant NoTwoLeaders specified in the configuration file is not defined in the "
            "specification.") in r.stdout


@pytest.mark.skipif(not HAVE_REF, reason="reference not mounted")
def test_modified_spec_is_refused(tmp_path):
    """The semantics are compiled in: any raft.tla but the reference's is refused."""
    text = open(os.path.join(REF, "raft.tla")).read()
    open(tmp_path / "raft.tla", "w").write(text + "\n\\* edited\n")
    shutil.copy(os.path.join(REF, "raft.cfg"), tmp_path / "raft.cfg")
    r = run(["-config", str(tmp_path / "raft.cfg"), str(tmp_path / "raft.tla")])
    assert r.returncode == 150 and "has sha256" in r.stdout, r.stdout


@pytest.mark.skipif(not HAVE_REF, reason="reference not mounted")
def test_wrapper_next_to_reference_spec_is_accepted_up_to_the_gpu(tmp_path):
    """specs/MC.tla EXTENDS raft: with raft.tla beside it the identity check
    passes and the cfg is accepted (the run itself then needs a GPU)."""
    tla, cfg = model_dir(str(tmp_path), 3, 1, 2, 1, 1, 1, ["NoTwoLeaders"])
    shutil.copy(os.path.join(REF, "raft.tla"), tmp_path / "raft.tla")
    r = run(["-config", cfg, tla])
    assert "verified" in r.stdout and "not defined" not in r.stdout, r.stdout
    assert r.returncode in (0, 255)  # 255 here: no GPU in this container


def test_no_constraint_is_refused(tmp_path):
    """Timeout (raft.tla:180) and Send (:106-110) are unbounded: without a
    CONSTRAINT the state space is infinite and rtla refuses to start."""
    tla, cfg = model_dir(str(tmp_path), 3, 1, 2, 1, 1, 1, ["NoTwoLeaders"], constraint=False)
    r = run(["-skip-spec-check", "-config", cfg, tla])
    assert r.returncode == 151 and "no CONSTRAINT" in r.stdout, r.stdout


def test_unknown_invariant_and_symmetry(tmp_path):
    tla, cfg = model_dir(str(tmp_path), 3, 1, 2, 1, 1, 1, ["TypeOK"])
    r = run(["-skip-spec-check", "-config", cfg, tla])
    assert r.returncode == 150 and "The invariant TypeOK specified" in r.stdout
    tla, cfg = model_dir(str(tmp_path / "b"), 3, 1, 2, 1, 1, 1, ["NoTwoLeaders"])
    open(cfg, "a").write("SYMMETRY Other\n")
    r = run(["-skip-spec-check", "-config", cfg, tla])
    assert r.returncode == 150 and "The symmetry Other specified" in r.stdout


def test_missing_bound_and_bad_strings(tmp_path):
    tla, cfg = model_dir(str(tmp_path), 3, 1, 2, 1, 1, 1, ["NoTwoLeaders"])
    txt = open(cfg).read()
    open(cfg, "w").write(txt.replace("    MaxTerm = 2\n", ""))
    r = run(["-skip-spec-check", "-config", cfg, tla])
    assert r.returncode == 151 and "constant MaxTerm is not assigned" in r.stdout
    open(cfg, "w").write(txt.replace('Leader = "Leader"', 'Leader = "Boss"'))
    r = run(["-skip-spec-check", "-config", cfg, tla])
    assert r.returncode == 151 and "constant Leader must be bound" in r.stdout


def test_usage_and_unknown_option():
    assert run([]).returncode == 255
    r = run(["-frobnicate", "1", "x.tla"])
    assert r.returncode == 255 and "unsupported option -frobnicate" in r.stderr


def test_gpus_flag_launches_one_process_per_rank():
    """-gpus 3: the launcher spawns three copies of itself, rank 0 publishes
    the RCCL id through the rendezvous file, every rank receives it (dry run:
    no GPU work)."""
    r = run(["-gpus", "3", "-config", "x.cfg", "x.tla"], env={"RTLA_CLI_DRYRUN": "1"})
    assert r.returncode == 0, r.stderr
    lines = sorted(l for l in r.stderr.splitlines() if l.startswith("rtla rank"))
    assert lines == ["rtla rank %d of 3 ready (id 00010203)" % k for k in range(3)]
