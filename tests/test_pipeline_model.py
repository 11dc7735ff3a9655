"""The one-engine, many-device mode (cgo NewScanner's default, device_mask 0 =
every GPU) without more hardware: the
engine's segment pipeline (trivy_amd/csrc/pipeline.h, DriverPipeline -- the
code Engine::scan runs its device drivers on) driven by 8 simulated devices
(tsg_test_multi_driver_model).  A device driver failing mid-batch -- an error
return as a HIP error gives, or a thrown bad_alloc -- or the confirming thread
throwing must fail the whole call (no partial result), stop the other drivers
within the segment each is running, return every lane to its pool and leave
no driver running; without a failure every segment is confirmed exactly once.
Reference: the goroutine fan-out this replaces, pkg/fanal/analyzer/analyzer.go:429-451."""
import ctypes

import pytest

from trivy_amd import _lib


def _run(ndev, nseg, fail_dev=-1, fail_at=0, mode=0, seg_us=300, confirm_us=100):
    st = _lib.TsgModelPipelineStats()
    L = _lib.lib()
    rc = L.tsg_test_multi_driver_model(ndev, nseg, fail_dev, fail_at, mode, seg_us, confirm_us, ctypes.byref(st))
    err = L.tsg_last_error().decode() if rc else ""
    return rc, err, {k: getattr(st, k) for k, _ in st._fields_}


@pytest.mark.parametrize("ndev", [1, 2, 8])
def test_all_segments_confirmed_once(ndev):
    rc, err, st = _run(ndev, 400)
    assert rc == 0, err
    assert st["segments_started"] == st["segments_pushed"] == st["segments_confirmed"] == 400
    assert st["segments_confirmed_twice"] == 0
    assert st["lanes_outstanding"] == 0 and st["drivers_alive"] == 0
    assert st["lanes_created"] == ndev                   # one lane per driver, one driver per device


@pytest.mark.parametrize("mode,what", [(1, "injected device failure"), (2, "out of memory|bad_alloc|host exception")])
@pytest.mark.parametrize("fail_dev,fail_at", [(0, 0), (5, 3), (7, 10)])
def test_device_failure_mid_batch_fails_call(mode, what, fail_dev, fail_at):
    import re
    nseg = 2000
    rc, err, st = _run(8, nseg, fail_dev, fail_at, mode)
    assert rc != 0 and re.search(what, err), (rc, err)
    # the other 7 drivers each finish at most the segment they were running
    assert st["started_after_failure"] <= 8, st
    assert st["segments_started"] < nseg // 4, st
    assert st["segments_confirmed"] < st["segments_started"], st       # the call did not run to the end
    assert st["lanes_outstanding"] == 0 and st["drivers_alive"] == 0, st
    assert st["fail_to_return_ms"] < 200, st                           # no hang: ~one segment's time


def test_confirm_failure_stops_drivers():
    rc, err, st = _run(8, 2000, fail_at=20, mode=3)
    assert rc != 0 and "host exception" in err, err
    assert st["segments_started"] < 500, st
    assert st["lanes_outstanding"] == 0 and st["drivers_alive"] == 0, st
    assert st["fail_to_return_ms"] < 200, st


def test_failure_with_full_queue_wakes_blocked_drivers():
    # a slow confirmer: the queue fills (2 x 8 + 2 jobs) and drivers block in
    # push; a failing driver's abort must wake them all
    rc, err, st = _run(8, 3000, fail_dev=2, fail_at=6, mode=1, seg_us=50, confirm_us=3000)
    assert rc != 0 and "injected device failure" in err
    assert st["lanes_outstanding"] == 0 and st["drivers_alive"] == 0, st
    assert st["fail_to_return_ms"] < 500, st
