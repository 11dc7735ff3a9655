"""Host-code sanitizer run (ASan + UBSan, or TSan with --thread) over the CPU entry points of the C-ABI.

Builds tools/asan_driver.cpp against the host sources of libtrivysecret
compiled with g++ -fsanitize=address,undefined (no recovery), linked with the
unsanitized HIP objects of trivy_amd/_build (the GPU kernels are not run:
there is no GPU here), then runs the driver over
  * a synthetic config-2-style corpus with dense planted secrets, near misses
    and invalid UTF-8 (builtin rules), and
  * a config-5 corpus (500 custom rules, allow rules, exclude blocks).
Each run must finish with no sanitizer report and host == table model.

  python tools/asan_check.py [--mb 8] [--out profiles/r3n_asan.log]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from trivy_amd import build as B  # noqa: E402
from workload import synth  # noqa: E402

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
TSAN = ["-fsanitize=thread", "-fno-omit-frame-pointer", "-g", "-O1"]


def build_driver(outdir, san):
    B.build()                                        # HIP objects in trivy_amd/_build
    common = ["-std=c++17", "-fPIC", "-I", B.CSRC, "-I", os.path.join(ROOT, "include")] + san
    objs = []
    jobs = []
    for s in B.HOST_SRCS:
        o = os.path.join(outdir, s + ".asan.o")
        jobs.append(subprocess.Popen(["g++", "-c", os.path.join(B.CSRC, s), "-o", o, "-march=x86-64-v2"] + common))
        objs.append(o)
    for j in jobs:
        if j.wait() != 0:
            raise SystemExit("sanitizer compile failed")
    exe = os.path.join(outdir, "asan_driver")
    hip_objs = [os.path.join(B.OBJ, s + ".o") for s in B.HIP_SRCS]
    subprocess.check_call(["g++", "-o", exe, os.path.join(ROOT, "tools", "asan_driver.cpp")] + objs + hip_objs +
                          common + ["-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lamdhip64", "-lpthread"])
    return exe


def write_case(d, corpus, cfg):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "config.json"), "w") as f:
        f.write(json.dumps(cfg) if cfg is not None else "")
    np.asarray(corpus.data[:corpus.nbytes], dtype=np.uint8).tofile(os.path.join(d, "data.bin"))
    np.asarray(corpus.offsets, dtype=np.uint64).tofile(os.path.join(d, "offsets.bin"))
    with open(os.path.join(d, "paths.txt"), "w") as f:
        f.write("".join(p + "\n" for p in corpus.paths))


class _Keep:
    def __init__(self, d):
        os.makedirs(d, exist_ok=True)
        self.d = d

    def __enter__(self):
        return self.d

    def __exit__(self, *exc):
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=8.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--thread", action="store_true", help="ThreadSanitizer instead of ASan + UBSan")
    ap.add_argument("--workdir", default="", help="keep the driver and inputs here")
    a = ap.parse_args()
    lines = []
    with (tempfile.TemporaryDirectory() if not a.workdir else _Keep(a.workdir)) as td:
        san = TSAN if a.thread else SAN
        exe = build_driver(td, san)
        nb = int(a.mb * 1e6)
        c2 = synth.generate(nb, seed=11, sizes="lognormal", plant_rate=2e-3, base_bytes=1 << 20)
        write_case(os.path.join(td, "c2"), c2, None)
        cfg5, plants = synth.config5(n_rules=500, seed=5)
        c5 = synth.generate(nb // 2, seed=12, sizes="lognormal", plant_rate=1e-3, base_bytes=1 << 20)
        synth.plant_custom(c5, plants, seed=5, rate=2e-3)
        write_case(os.path.join(td, "c5"), c5, cfg5)
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
                   TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
        rc_all = 0
        for case in ("c2", "c5"):
            p = subprocess.run([exe, os.path.join(td, case)], capture_output=True, text=True, env=env)
            lines.append("%s rc=%d %s%s" % (case, p.returncode, p.stdout, p.stderr[-4000:]))
            rc_all |= p.returncode
    text = "sanitizers: %s\n%s" % (" ".join(san), "".join(lines))
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    return rc_all


if __name__ == "__main__":
    sys.exit(main())
