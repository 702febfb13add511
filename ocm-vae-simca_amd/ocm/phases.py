"""Per-phase timing of the fit / score path (bench.py's phase breakdown).

``PhaseTimer.mark(name)`` records a timing hipEvent on the current (launch)
stream and the host clock; phase ``name`` is the interval since the previous
mark.  Installed with ``engine.set_phase_timer``; with no timer installed the
marks cost nothing.  GPU intervals include any idle gap while the host was
still issuing, so they add up to the step's wall time on the stream.
"""
from __future__ import annotations

import time
from collections import defaultdict

import torch


class PhaseTimer:
    def __init__(self, device):
        self.device = device
        self._marks = []

    def mark(self, name: str):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self._marks.append((name, ev, time.perf_counter()))

    def reset(self):
        self._marks = []

    def intervals(self) -> list[tuple[str, float, float]]:
        """[(phase, gpu_ms, host_ms)] between consecutive marks ("start" opens a step)."""
        torch.cuda.synchronize(self.device)
        out = []
        for (_, e0, h0), (name, e1, h1) in zip(self._marks, self._marks[1:]):
            if name == "start":
                continue
            out.append((name, e0.elapsed_time(e1), (h1 - h0) * 1e3))
        return out

    def summary(self, steps: int) -> dict:
        """Mean GPU / host milliseconds per phase over ``steps`` steps."""
        g, h = defaultdict(float), defaultdict(float)
        order = []
        for name, gm, hm in self.intervals():
            if name not in g:
                order.append(name)
            g[name] += gm
            h[name] += hm
        return {name: {"gpu_ms": round(g[name] / steps, 4), "host_ms": round(h[name] / steps, 4)} for name in order}
