"""Phase tracing (SURVEY.md §5 "Tracing"): every product phase — collect (policy + env
steps), gae, episodes (the cross-rank episode bookkeeping), train (epochs of minibatch
updates) — is a roctx range (torch.cuda.nvtx on ROCm), so `rocprofv3 --marker-trace` shows
them on the timeline; with timers enabled, each phase also records HIP events on the launch
stream (torch's current stream, where libppox launches) and the host clock, so
bench.py reports the per-phase GPU time next to the host time spent issuing it.  The
reference only times the whole loop by wall clock (ppo.py:277,290-291)."""
import contextlib
import functools
import time

import torch

_timers = None          # name -> list of (start event, end event, host seconds)
_nvtx = None            # resolved on first use: torch.cuda.nvtx, or False when unusable


def _ranges():
    global _nvtx
    if _nvtx is None:
        try:
            torch.cuda.nvtx.range_push("ppox")
            torch.cuda.nvtx.range_pop()
            _nvtx = torch.cuda.nvtx
        except Exception:  # no roctx in this build: phases still time, just unnamed on the trace
            _nvtx = False
    return _nvtx


def enable_timers(on=True):
    """Start (or stop) recording per-phase HIP events; clears what was recorded."""
    global _timers
    _timers = {} if on else None


@contextlib.contextmanager
def phase(name):
    nv = _ranges()
    if nv:
        nv.range_push(name)
    rec = _timers is not None and torch.cuda.is_available()
    if rec:
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        h0 = time.perf_counter()
    try:
        yield
    finally:
        if rec:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            _timers.setdefault(name, []).append((s, e, time.perf_counter() - h0))
        if nv:
            nv.range_pop()


def traced(name):
    """Decorator form of phase()."""
    def wrap(fn):
        @functools.wraps(fn)
        def inner(*a, **k):
            with phase(name):
                return fn(*a, **k)
        return inner
    return wrap


def summary():
    """{phase: {"gpu_ms", "host_ms", "count"}} totals since enable_timers(); synchronises.
    gpu_ms is the stream time from the phase's first to its last launch boundary (events
    on the launch stream), host_ms the host time spent inside the phase."""
    if not _timers:
        return {}
    torch.cuda.synchronize()
    out = {}
    for k, v in _timers.items():
        out[k] = {"gpu_ms": round(sum(s.elapsed_time(e) for s, e, _ in v), 3),
                  "host_ms": round(sum(h for _, _, h in v) * 1e3, 3), "count": len(v)}
    return out
