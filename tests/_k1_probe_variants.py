"""Child process of tests/test_gpu_stress.py::test_k1_probe_variants_agree_gpu
(not collected by pytest): with TSG_LIB=libtrivysecret_probe.so, scans one
synthetic batch with each K1 measurement build ABL:CHUNK given on the
command line and checks it against the host confirmer run without the GPU
prefilter (tsg_scan_host_reference, in the same library)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from trivy_amd import secret as S  # noqa: E402
from workload import synth  # noqa: E402


def main():
    assert os.environ.get("TSG_LIB") == "libtrivysecret_probe.so"
    # large files plus ~21 KB files (a file boundary in most K1 lines' ranges:
    # the boundary-line builds) with non-ASCII text (the fold-special check)
    c = synth.generate(24_000_000, seed=31, sizes="loguniform", plant_rate=3e-3)
    d = synth.generate(8_000_000, seed=32, sizes="small", layout="image", plant_rate=3e-3)
    args = [S.ScanArgs(c.paths[i], c.file(i)) for i in range(len(c.paths))]
    args += [S.ScanArgs(d.paths[i], d.file(i)) for i in range(len(d.paths))]
    want = S.scan_host_reference(S.Scanner(None), args, threads=16)
    assert sum(len(w["Findings"]) for w in want) > 20
    for v in sys.argv[1].split(","):
        abl, chunk = v.split(":")
        os.environ["TSG_K1_ABL"] = abl
        os.environ["TSG_K1_CHUNK"] = chunk
        got, stats = S.Scanner(None).ScanBatch(args, with_stats=True)
        assert stats["chunk_bytes"] == int(chunk), (v, stats["chunk_bytes"])
        assert got == want, v
        print("K1 build %s chunk %s: agree" % (abl, chunk), flush=True)


if __name__ == "__main__":
    main()
