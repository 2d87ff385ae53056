"""The capture-topology invariant (monst3r_slam_amd.capture, DESIGN §5 "Capture topology") on
CPU: the vector-clock bookkeeping that decides, before capture_end, whether every side
stream forked into a capture is joined back, whether an event crosses the capture boundary,
and whether the capture is wider than the HIP runtime's hardware queues allow.  The launch /
event hooks themselves run on the GPU (tests/test_gpu_sequence.py)."""
import types

import pytest

from monst3r_slam_amd.capture import CaptureTopology, TopologyError, max_capture_streams

CAP, A, B, C = 0x100, 0x200, 0x300, 0x400


def _topo(max_streams=5):
    return CaptureTopology(types.SimpleNamespace(cuda_stream=CAP), max_streams=max_streams)


def _ev():
    return types.SimpleNamespace()


def _fork(t, src, dst):
    e = _ev()
    t.record(e, src)
    t.wait(dst, e)


def test_fork_join_ok():
    t = _topo()
    _fork(t, CAP, A)          # side.wait_stream(main)
    t.tick(A)                 # side work
    t.tick(CAP)               # main work meanwhile
    _fork(t, A, CAP)          # main.wait_stream(side)
    t.check()
    assert sorted(t.streams()) == [CAP, A]


def test_unjoined_side_stream_raises():
    t = _topo()
    _fork(t, CAP, A)
    t.tick(A)
    e = _ev()
    t.record(e, A)            # joined mid-way ...
    t.wait(CAP, e)
    t.tick(A)                 # ... but more work after the join point
    with pytest.raises(TopologyError, match="not joined"):
        t.check()


def test_forked_idle_stream_must_rejoin():
    t = _topo()
    _fork(t, CAP, A)          # a fork with no work still puts A into the capture
    assert any("not joined" in p for p in t.problems())


def test_transitive_join_through_another_stream():
    t = _topo()
    _fork(t, CAP, A)
    t.tick(A)
    _fork(t, A, B)            # B waits on A
    t.tick(B)
    _fork(t, B, CAP)          # main waits on B only: A's work is ordered before it
    t.check()


def test_event_recorded_outside_the_capture():
    t = _topo()
    foreign = _ev()           # never recorded under this topology
    t.wait(CAP, foreign)
    with pytest.raises(TopologyError, match="outside the capture"):
        t.check()


def test_width_limit():
    t = _topo(max_streams=3)
    for s in (A, B, C):
        _fork(t, CAP, s)
        t.tick(s)
        _fork(t, s, CAP)
    with pytest.raises(TopologyError, match="4 streams"):
        t.check()
    t2 = _topo(max_streams=3)
    for s in (A, B):
        _fork(t2, CAP, s)
        t2.tick(s)
        _fork(t2, s, CAP)
    t2.check()


def test_budget_follows_hw_queues(monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "2")
    assert max_capture_streams() == 3
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    assert max_capture_streams() == 4        # five streams over four queues crashed (round 5)
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    assert max_capture_streams() == 4


def test_self_wait_raises():
    """s.wait_stream(s) inside a capture (round 5: capture_end segfaulted on it)."""
    t = _topo()
    _fork(t, CAP, A)
    t.tick(A)
    _fork(t, A, A)            # the stream waits on its own event
    _fork(t, A, CAP)
    with pytest.raises(TopologyError, match="recorded itself"):
        t.check()
