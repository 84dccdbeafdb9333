"""bench.py's per-leg watchdog (LegGuard): a leg that does not finish makes
rank 0 print the JSON line as it stands, with the leg named in
`legs_aborted`, and every rank leave with status 0 -- the headline survives a
hung sub-record (e.g. a collective that never completes on a new node)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, time
sys.path.insert(0, {root!r})
import bench
g = bench.LegGuard({rank})
if {rank} == 0:
    g.line = {{"metric": "m", "value": 1.0, "arc": None}}
g.start("churn_route_ready", 30.0)
g.start("arc", 0.2)   # replaces the first timer
time.sleep(20)
print("not reached")
"""


def _run(rank):
    return subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, rank=rank)],
                          capture_output=True, text=True, timeout=120)


def test_guard_rank0_prints_line_and_exits_zero():
    r = _run(0)
    assert r.returncode == 0, r.stderr
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["arc"] is None
    assert [a["leg"] for a in d["legs_aborted"]] == ["arc"]
    assert "did not finish" in r.stderr


def test_guard_other_rank_exits_zero_silently():
    r = _run(1)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == ""


CHILD_FAIL = r"""
import sys
sys.path.insert(0, {root!r})
import bench
g = bench.LegGuard({rank})
if {rank} == 0:
    g.line = {{"metric": "m", "value": 1.0, "arc": None}}
g.run("churn_route_ready", lambda: 7)
def bad():
    raise RuntimeError("collective failed")
g.run("arc", bad)
print("not reached")
"""


def test_guard_failed_leg_rank0_prints_line_and_exits_zero():
    """A leg that raises (e.g. an RCCL error on a new node): rank 0 prints the
    line with the leg and its error in `legs_failed`, status 0; another rank
    leaves silently with status 0 (its peers' watchdogs end their waits)."""
    r = subprocess.run([sys.executable, "-c", CHILD_FAIL.format(root=ROOT, rank=0)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout
    d = json.loads(lines[0])
    assert d["value"] == 1.0 and d["arc"] is None
    assert [(a["leg"], "collective failed" in a["error"]) for a in d["legs_failed"]] == \
        [("arc", True)]
    assert "failed" in r.stderr
    r1 = subprocess.run([sys.executable, "-c", CHILD_FAIL.format(root=ROOT, rank=1)],
                        capture_output=True, text=True, timeout=120)
    assert r1.returncode == 0, r1.stderr
    assert r1.stdout.strip() == ""
