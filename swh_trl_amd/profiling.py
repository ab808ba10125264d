"""Live per-kernel timing with HIP events (torch.cuda.Event records on the
same stream the C-ABI kernels are launched on).  Off by default; bench.py
switches it on for the timed region.  Replaces the reference's wall-clock
`profiling_context` (trl/extras/profiling.py:31-100) for device work."""
from __future__ import annotations

import sys
import time
from collections import defaultdict
from contextlib import contextmanager

import torch

_enabled = False
_events: dict[str, list] = defaultdict(list)
_bytes: dict[str, float] = defaultdict(float)


def enable(on: bool = True):
    global _enabled
    _enabled = on


def reset():
    _events.clear()
    _bytes.clear()


@contextmanager
def kernel(name: str, nbytes: float = 0.0):
    if not _enabled:
        yield
        return
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    _events[name].append((s, e))
    _bytes[name] += nbytes


def summary() -> dict:
    """{name: {launches, total_ms, avg_us, bytes_per_launch}} (synchronises)."""
    torch.cuda.synchronize()
    out = {}
    for k, ev in _events.items():
        tot = sum(s.elapsed_time(e) for s, e in ev)
        out[k] = {"launches": len(ev), "total_ms": tot, "avg_us": 1000.0 * tot / max(1, len(ev)),
                  "bytes_per_launch": _bytes[k] / max(1, len(ev))}
    return out


_TRACE = [False]
_T0 = [time.time()]


def set_trace(on: bool) -> None:
    """Synchronised phase timings on stderr (diagnostics only; tools and bench.py
    turn it on, e.g. from SWH_TRACE=1)."""
    _TRACE[0] = bool(on)
    _T0[0] = time.time()


def trace(msg: str):
    """A phase line when tracing is on (`set_trace`)."""
    if _TRACE[0]:
        import torch
        torch.cuda.synchronize()
        now = time.time()
        print(f"[swh {now - _T0[0]:8.3f}s] {msg}", file=sys.stderr, flush=True)
