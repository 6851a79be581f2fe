"""Tracing / profiling hooks.

* roctx ranges (``libroctx64``) around every phase of a training step -- visible in
  ``rocprofv3 --marker-trace`` timelines next to the HIP kernels;
* ``PhaseTimer`` collects per-phase wall time and (on the GPU) device time from HIP
  events without synchronising inside the step; resolved once per epoch into the
  ``progress.txt`` columns (RolloutMs, LearnMs, ...);
* ``torch_profiler`` wraps torch.profiler for the Python glue.

The reference's profiling hooks (Cargo feature ``profile`` = flamegraph +
console-subscriber) broke the build; nothing here changes the code path
when tracing is off.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict
from typing import Dict, List

_ROCTX = None
_ROCTX_TRIED = False


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if _ROCTX_TRIED:
        return _ROCTX
    _ROCTX_TRIED = True
    if os.environ.get("RRL_ROCTX", "1") == "0":
        return None
    cands = ["libroctx64.so", "/opt/rocm/lib/libroctx64.so"]
    try:
        import torch

        cands.insert(0, os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"))
    except Exception:
        pass
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _ROCTX = lib
            break
        except OSError:
            continue
    return _ROCTX


def roctx_available() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def roctx_mark(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Per-phase wall (host) and device (HIP events) time, resolved lazily."""

    def __init__(self, device=None, enabled: bool = True):
        self.enabled = enabled
        self.device = device
        self.cuda = False
        try:
            import torch

            self.cuda = device is not None and torch.device(device).type == "cuda"
        except Exception:
            pass
        self.wall: Dict[str, float] = defaultdict(float)
        self.count: Dict[str, int] = defaultdict(int)
        self._events: List = []
        self.device_ms: Dict[str, float] = defaultdict(float)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        ev0 = ev1 = None
        if self.cuda:
            import torch

            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        t0 = time.perf_counter()
        with roctx_range(name):
            yield
        self.wall[name] += time.perf_counter() - t0
        self.count[name] += 1
        if self.cuda:
            import torch

            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._events.append((name, ev0, ev1))

    def resolve(self) -> Dict[str, float]:
        """Device milliseconds per phase since the last resolve (synchronises once)."""
        if self._events:
            self._events[-1][2].synchronize()
            for name, a, b in self._events:
                self.device_ms[name] += a.elapsed_time(b)
            self._events.clear()
        return dict(self.device_ms)

    def columns(self, prefix: str = "") -> Dict[str, float]:
        dev = self.resolve()
        out = {}
        for k, v in self.wall.items():
            out[f"{prefix}{k}WallMs"] = 1e3 * v
        for k, v in dev.items():
            out[f"{prefix}{k}Ms"] = v
        return out

    def per_step(self, steps: int) -> Dict[str, float]:
        """Device ms per step of every phase (wall ms where no device time exists: CPU / gloo),
        and the number of calls per step -- e.g. 81 AllReduce calls per learner epoch."""
        dev = self.resolve()
        out = {}
        for k in self.wall:
            v = dev.get(k, 1e3 * self.wall[k])
            out[f"{k}Ms"] = round(v / max(steps, 1), 4)
            out[f"{k}Calls"] = round(self.count[k] / max(steps, 1), 2)
        return out

    def reset(self):
        self.resolve()
        self.wall.clear()
        self.count.clear()
        self.device_ms.clear()


@contextlib.contextmanager
def torch_profiler(path: str, cuda: bool = True):
    """torch.profiler trace (chrome json) of the enclosed block."""
    import torch

    acts = [torch.profiler.ProfilerActivity.CPU]
    if cuda and torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    prof.export_chrome_trace(path)


@contextlib.contextmanager
def gc_paused():
    """No automatic garbage collection inside the block: a hipGraph capture must not run
    finalizers that destroy HIP events / streams of unrelated, unreachable objects (a collection
    triggered by an allocation inside the capture aborted a capture once)."""
    import gc

    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
