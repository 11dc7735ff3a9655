"""The bounded backtracker (goregexp.cpp Machine::backtrack, Go's backtrack.go)
against the Pike VM: the confirmer's anchored leftmost-first matches with
submatches must not change.  Each side runs in its own process
(TSG_RE_NO_BACKTRACK=1 forces the VM) through tsg_scan_table_model (the
confirmer on the compiled plans, as on the GPU path) with the builtin rules
and with config 5's 500 custom rules (bounded and unbounded repeats, named
groups, allow rules, exclude blocks).  Random patterns: tests/test_lazy_dfa.py
compares match_at's anchored end (the backtracker for bounded patterns) with
the lazy DFA's."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, tempfile
sys.path.insert(0, %r)
from trivy_amd import secret as S
from workload import synth
out = {}
c = synth.generate(2_000_000, seed=21, sizes="lognormal", plant_rate=5e-3)
args = [S.ScanArgs(FilePath=c.paths[i], Content=c.file(i), Binary=False) for i in range(len(c.paths))]
out["builtin"] = S.scan_table_model(S.Scanner(None), args)
cfg5, plants = synth.config5(500, seed=3)
path = os.path.join(tempfile.mkdtemp(), "c5.yaml")
synth.write_yaml(cfg5, path)
c5 = synth.generate(1_500_000, seed=22, sizes="lognormal", plant_rate=2e-3)
synth.plant_custom(c5, plants, seed=3, rate=2e-3)
args5 = [S.ScanArgs(FilePath=c5.paths[i], Content=c5.file(i), Binary=False) for i in range(len(c5.paths))]
out["config5"] = S.scan_table_model(S.Scanner(S.ParseConfig(path)), args5)
print(json.dumps(out))
""" % ROOT


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    out = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout)


def test_backtracker_equals_pike_vm_on_rules():
    bt = _run({})
    vm = _run({"TSG_RE_NO_BACKTRACK": "1"})
    assert sum(len(s["Findings"]) for s in bt["builtin"]) > 20
    assert sum(len(s["Findings"]) for s in bt["config5"]) > 20
    assert bt["builtin"] == vm["builtin"]
    assert bt["config5"] == vm["config5"]
