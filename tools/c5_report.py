"""Compile the config-5 ruleset (500 custom rules + builtins) and print the
prefilter compile report summary.

  python tools/c5_report.py [n_rules]
"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trivy_amd import secret as S
from workload import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    cfg, _ = synth.config5(n)
    path = "/tmp/c5_%d.yaml" % n
    synth.write_yaml(cfg, path)
    t = time.time()
    sc = S.Scanner(S.ParseConfig(path))
    print("rules", len(sc.rule_ids), "parse+compile %.2fs" % (time.time() - t))
    t = time.time()
    rep = S.prefilter_report(sc)
    print("prefilter %.2fs" % (time.time() - t))
    lines = rep.splitlines()
    for ln in lines:
        if not (": anchored" in ln or ": FULL" in ln):
            print(ln)
    print(collections.Counter(ln.split(": ", 1)[1].split(" ")[0] for ln in lines if ": anchored" in ln or ": FULL" in ln))
    for ln in lines:
        if ": FULL" in ln:
            print(ln)


if __name__ == "__main__":
    main()
