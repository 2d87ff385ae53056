"""HIP graph capture of the tracking step with a host-side check of its stream topology.

The step is captured once per feature parity (bench.py, SequenceLoop) and replayed per frame.
Work issued on side streams joins the capture through events: a side stream enters the
capture when it waits on an event recorded on a capturing stream (the fork), and the capture
is well formed only if the capture stream, before capture_end, has waited on an event
recorded on every such side stream after its last work (the join).  On this ROCm stack a
malformed or over-wide capture does not fail cleanly: hipStreamEndCapture / the graph
instantiate segfaulted (profiles/r03_capture_segfault.txt) when more streams took part than
the HIP runtime has hardware queues to spare (measured: 6 and 5 streams over
GPU_MAX_HW_QUEUES=4 and 4 streams over 2 crash; 4 streams over 3 or 4 queues capture; DESIGN §5
"Capture topology"), and when a stream waited on an event recorded on itself (round 5: a
fork / join whose two ends were the same stream crashed every capture that had it, at 3 and
4 streams alike).  CaptureTopology records the fork/join graph while the step is issued — a
vector clock per stream, advanced by every native launch (_lib.stream) and every entry into
a stream context — and raises TopologyError before capture_end when

  * a side stream's last work is not ordered before the end of the capture stream
    (an unjoined fork: CUDA semantics return cudaErrorStreamCaptureUnjoined, HIP crashed);
  * an event waited on inside the capture was recorded outside it (a cross-capture edge);
  * a stream waits on an event it recorded itself (e.g. s.wait_stream(s));
  * more streams take part than min(GPU_MAX_HW_QUEUES + 1, 4).

Host-only bookkeeping at capture time; replays are untouched.
"""
from __future__ import annotations

import os

import torch

from . import _lib


class TopologyError(RuntimeError):
    pass


def hw_queues() -> int:
    """Hardware queues per process the HIP runtime may use (GPU_MAX_HW_QUEUES, default 4)."""
    try:
        return max(1, int(os.environ.get("GPU_MAX_HW_QUEUES", "4")))
    except ValueError:
        return 4


def max_capture_streams() -> int:
    """Widest capture this stack survives: one stream more than its hardware queues, and
    never more than four (five over four queues crashed, round 5)."""
    return min(hw_queues() + 1, 4)


class CaptureTopology:
    """Context manager recording the fork / join structure of the work issued inside it
    (see module doc).  `capture_stream` is the stream the graph is captured on."""

    def __init__(self, capture_stream: torch.cuda.Stream, max_streams: int | None = None):
        self.cap = int(capture_stream.cuda_stream)
        self.max_streams = max_streams or max_capture_streams()
        self.vc: dict[int, dict[int, int]] = {self.cap: {self.cap: 1}}
        self.errors: list[str] = []
        self._saved = None

    # ---- clock operations ----
    def _clock(self, h):
        return self.vc.setdefault(h, {h: 0})

    def tick(self, h):
        c = self._clock(h)
        c[h] = c.get(h, 0) + 1

    def record(self, ev, h):
        ev._m3s_vc = (id(self), dict(self._clock(h)), h)

    def wait(self, h, ev):
        tag = getattr(ev, "_m3s_vc", None)
        if tag is None or tag[0] != id(self):
            self.errors.append(f"stream {h:#x} waits on an event recorded outside the capture")
            return
        if tag[2] == h:
            self.errors.append(f"stream {h:#x} waits on an event it recorded itself (a fork / "
                               "join onto the same stream: capture_end segfaults)")
            return
        c = self._clock(h)
        for k, v in tag[1].items():
            if c.get(k, 0) < v:
                c[k] = v
        self.tick(h)   # a fork puts the stream into the capture: it must be joined back

    # ---- patching ----
    def __enter__(self):
        topo = self
        ev_record = torch.cuda.Event.record
        ev_wait = torch.cuda.Event.wait
        ctx_enter = torch.cuda.StreamContext.__enter__
        lib_stream = _lib.stream

        def _cur():
            return int(torch.cuda.current_stream().cuda_stream)

        def record(ev, stream=None):
            h = int(stream.cuda_stream) if stream is not None else _cur()
            ev_record(ev, stream)
            topo.record(ev, h)

        def ev_wait_(ev, stream=None):
            h = int(stream.cuda_stream) if stream is not None else _cur()
            ev_wait(ev, stream)
            topo.wait(h, ev)

        def enter(ctx):
            r = ctx_enter(ctx)
            topo.tick(_cur())
            return r

        def stream(device=None):
            s = lib_stream(device)
            topo.tick(int(s.value or 0))
            return s

        # (Stream.wait_event / wait_stream go through Event.wait / Event.record)
        self._saved = (ev_record, ev_wait, ctx_enter, lib_stream)
        torch.cuda.Event.record = record
        torch.cuda.Event.wait = ev_wait_
        torch.cuda.StreamContext.__enter__ = enter
        _lib.stream = stream
        return self

    def __exit__(self, *exc):
        ev_record, ev_wait, ctx_enter, lib_stream = self._saved
        torch.cuda.Event.record = ev_record
        torch.cuda.Event.wait = ev_wait
        torch.cuda.StreamContext.__enter__ = ctx_enter
        _lib.stream = lib_stream
        return False

    # ---- the invariant ----
    def streams(self):
        """Streams that took part (launched, entered, or were forked into the capture)."""
        return [h for h, c in self.vc.items() if c.get(h, 0) > 0]

    def problems(self):
        out = list(self.errors)
        end = self.vc[self.cap]
        for h in self.streams():
            if h == self.cap:
                continue
            own = self.vc[h].get(h, 0)
            if end.get(h, 0) < own:
                out.append(f"stream {h:#x}: its last work (clock {own}) is not joined into the "
                           f"capture stream (joined up to {end.get(h, 0)})")
        n = len(self.streams())
        if n > self.max_streams:
            out.append(f"{n} streams take part in the capture, more than the {self.max_streams} "
                       "this stack survives (min(GPU_MAX_HW_QUEUES + 1, 4): the HIP runtime "
                       "segfaults at capture_end past that width, DESIGN §5)")
        return out

    def check(self):
        p = self.problems()
        if p:
            raise TopologyError("malformed graph capture: " + "; ".join(p))


def _join_all(topo: CaptureTopology, s: torch.cuda.Stream):
    """Make the capture stream wait on every stream that took part (closes the graph)."""
    for h in topo.streams():
        if h != topo.cap:
            other = torch.cuda.ExternalStream(h)
            s.wait_stream(other)


def check_topology(fn, dev, check: bool = True):
    """Run fn once eagerly on a fresh stream under CaptureTopology and raise TopologyError on
    a malformed fork / join structure or a capture wider than the hardware queues allow —
    the pre-capture check of `capture_graph(warmup=True)`, for callers that warm up
    separately (bench.step_timeline) and then capture with warmup=False.  A width violation
    found only DURING a capture cannot be kept from capture_end (torch's graph context always
    ends the capture), so a capture without this eager pass in front is unchecked for width."""
    s = torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)
    s.wait_stream(cur)
    topo = CaptureTopology(s)
    with topo, torch.cuda.stream(s):
        fn()
    cur.wait_stream(s)
    torch.cuda.synchronize(dev)
    if check:
        topo.check()
    return topo


def capture_graph(fn, dev, warmup: bool = True, check: bool = True):
    """Capture fn into a torch.cuda.CUDAGraph on a fresh stream, its stream topology checked.

    warmup: fn first runs once eagerly on that stream (allocations, lazy state) under the same
    CaptureTopology, and a malformed topology raises TopologyError there — before any capture
    begins, so a graph the runtime would crash on is never handed to capture_end.  The capture
    itself is traced again; should it differ and fail, every participating stream is joined
    into the capture stream before capture_end and the error is raised after it.
    Returns the graph (attribute m3s_streams: the streams that took part)."""
    if warmup:
        check_topology(fn, dev, check)
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    topo = CaptureTopology(s)
    bad = None
    with torch.cuda.graph(g, stream=s):
        with topo:
            fn()
        if check and topo.problems():
            bad = topo.problems()
            _join_all(topo, s)
    if bad:
        raise TopologyError("malformed graph capture: " + "; ".join(bad))
    torch.cuda.synchronize(dev)
    g.m3s_streams = len(topo.streams())
    return g
