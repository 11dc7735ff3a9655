"""tsg_result_free hands results of >= 4096 files to a background thread
(capi.cpp Reaper): many frees, from several Python threads and from a forked
child, all complete and the process exits cleanly."""
import ctypes
import json
import os
import subprocess
import sys
import threading

from trivy_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _big_result(n):
    secrets = [{"FilePath": "f%d.txt" % i, "Findings": []} for i in range(n)]
    secrets[7] = {"FilePath": "x.env", "Findings": [{"RuleID": "aws-access-key-id", "Category": "AWS",
                                                      "Severity": "CRITICAL", "Title": "AWS Access Key ID",
                                                      "StartLine": 1, "EndLine": 1, "Code": {"Lines": []},
                                                      "Match": "AWS_ACCESS_KEY_ID=********************"}]}
    js = json.dumps(secrets).encode()
    h = ctypes.c_void_p()
    _lib.check(_lib.lib().tsg_result_from_json(js, len(js), ctypes.byref(h)))
    return h


def test_reaper_frees_from_threads():
    L = _lib.lib()
    def work():
        for _ in range(5):
            L.tsg_result_free(_big_result(5000))
            L.tsg_result_free(_big_result(10))        # inline path
    ts = [threading.Thread(target=work) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


def test_reaper_process_exit_and_fork():
    # a child process frees through the reaper, forks, frees again in the
    # forked grandchild and in itself, and exits: no hang, status 0
    code = r"""
import os, sys
sys.path.insert(0, %r)
from tests.test_result_reaper import _big_result
from trivy_amd import _lib
L = _lib.lib()
L.tsg_result_free(_big_result(6000))
pid = os.fork()
if pid == 0:
    L.tsg_result_free(_big_result(6000))
    L.tsg_result_free(_big_result(6000))
    sys.exit(0)
L.tsg_result_free(_big_result(6000))
_, st = os.waitpid(pid, 0)
assert os.WIFEXITED(st) and os.WEXITSTATUS(st) == 0, st
print("ok")
""" % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"
