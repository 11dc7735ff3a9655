"""bench.k1_build: the hash that keys a committed HBM
traffic measurement (profiles/traffic_c*.json) to the K1 build it was taken
on must cover all of K1's device code -- the word steps, the line loop and
the kernel itself -- and nothing else."""
import json
import os
import re

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = open(os.path.join(ROOT, "trivy_amd", "csrc", "engine.hip"), "rb").read()


def _edit_inside(func_marker, src=SRC):
    """flip one byte of the first statement line after `func_marker`"""
    i = src.find(func_marker)
    assert i >= 0, func_marker
    j = src.find(b";\n", src.find(b"{", i)) - 1          # a byte just before a statement's ';'
    ch = src[j:j + 1]
    return src[:j] + (b" " if ch != b" " else b"\t") + src[j + 1:]


@pytest.mark.parametrize("marker", [
    b"__device__ __forceinline__ void k1_word_v3(",
    b"__device__ __forceinline__ void k1_word_c(",
    b"__device__ __forceinline__ v4u k1_load(",
    b"void tsg_k1_scan_v3(",
    b"__device__ __forceinline__ uint32_t k1_step(",
    b"constexpr int kK1Default",
])
def test_k1_edit_changes_build_hash(marker):
    assert bench.k1_build(_edit_inside(marker)) != bench.k1_build(SRC)


@pytest.mark.parametrize("marker", [
    b"void tsg_k2_verify(",
    b"bool Engine::run_segment(",
])
def test_k2_and_host_edits_keep_build_hash(marker):
    assert bench.k1_build(_edit_inside(marker)) == bench.k1_build(SRC)


def test_probe_only_variants_keep_build_hash():
    # the TSG_K1_PROBE variant list exists only in the probe library
    i = SRC.find(b"#ifdef TSG_K1_PROBE\n    TSG_K1_V3(")
    assert i > 0
    j = SRC.find(b"TSG_K1_V3(0)", i)
    edited = SRC[:j] + b"TSG_K1_V3(7) " + SRC[j:]
    assert bench.k1_build(edited) == bench.k1_build(SRC)


def test_markers_in_order():
    a, b, c = (SRC.find(m) for m in (b"\n// ==== K2 begin", b"\n// ==== K2 end", b"\n// ==== host side"))
    assert 0 < a < b < c
    k2 = SRC[a:b]
    assert b"tsg_k2_verify" in k2 and b"tsg_k1_scan_v3" not in k2
    assert b"void tsg_k1_scan_v3(" in SRC[b:c] and b"k1_word_v3(" in SRC[:a] + SRC[b:c]


def test_committed_traffic_files_match_current_k1():
    # the bench only cites a traffic file whose k1_build is the current one:
    # a stale file after a K1 edit must be re-measured (tools/pmc_traffic.sh)
    cur = bench.k1_build()
    for cfg in (1, 2, 3, 5):
        tj = json.load(open(os.path.join(ROOT, "profiles", "traffic_c%d.json" % cfg)))
        assert tj["k1_build"] == cur, (cfg, tj["k1_build"], cur)
