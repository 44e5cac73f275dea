"""Run observability: reference-format stdout line, JSONL metrics stream, event file,
and a phase profiler (roctx ranges + CUDA-event timing).

stdout keeps the reference's line (train.py:205-208)::

    {global_step}/{total} (epoch {e}), train_loss = {loss:.3f}, time/batch = {t:.3f}

followed by ``, chars/sec = N`` (node aggregate).
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from collections import defaultdict
from typing import Dict, Optional

import torch

from .tfevents import EventWriter


class MetricsLogger:
    def __init__(self, log_dir: Optional[str], enabled: bool = True,
                 jsonl_path: Optional[str] = None, events: bool = True):
        self.enabled = enabled
        self.run_dir = None
        self._jsonl = None
        self.events: Optional[EventWriter] = None
        if not enabled or log_dir is None:
            return
        self.run_dir = os.path.join(log_dir, time.strftime("%Y-%m-%d-%H-%M-%S"))
        os.makedirs(self.run_dir, exist_ok=True)
        self._jsonl = open(jsonl_path or os.path.join(self.run_dir, "metrics.jsonl"), "a")
        if events:
            self.events = EventWriter(self.run_dir)

    def log(self, record: Dict) -> None:
        if self._jsonl is not None:
            self._jsonl.write(json.dumps(record) + "\n")
            self._jsonl.flush()

    def scalar(self, tag: str, value: float, step: int) -> None:
        if self.events is not None:
            self.events.scalar(tag, value, step)

    def histogram(self, tag: str, values, step: int) -> None:
        if self.events is not None:
            self.events.histogram(tag, values, step)

    def close(self) -> None:
        if self._jsonl is not None:
            self._jsonl.close()
            self._jsonl = None
        if self.events is not None:
            self.events.close()


def progress_line(global_step: int, total: int, epoch: int, loss: float, dt: float,
                  chars_per_sec: Optional[float] = None) -> str:
    s = "{}/{} (epoch {}), train_loss = {:.3f}, time/batch = {:.3f}".format(
        global_step, total, epoch, loss, dt)
    if chars_per_sec is not None:
        s += ", chars/sec = {:.0f}".format(chars_per_sec)
    return s


class PhaseProfiler:
    """Per-phase GPU timing via events + roctx ranges (visible in rocprofv3 --marker-trace).
    Disabled => zero overhead context managers."""

    def __init__(self, enabled: bool = False, device: Optional[torch.device] = None):
        self.enabled = enabled and device is not None and device.type == "cuda"
        self.device = device
        self._pending = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        torch.cuda.nvtx.range_push(name)
        s.record()
        try:
            yield
        finally:
            e.record()
            torch.cuda.nvtx.range_pop()
            self._pending.append((name, s, e))

    def collect(self):
        if not self.enabled or not self._pending:
            return
        torch.cuda.synchronize(self.device)
        for name, s, e in self._pending:
            self.totals[name] += s.elapsed_time(e)
            self.counts[name] += 1
        self._pending.clear()

    def table(self) -> str:
        self.collect()
        if not self.totals:
            return ""
        tot = sum(self.totals.values())
        lines = [f"{'phase':<28}{'calls':>8}{'ms/call':>12}{'share':>8}"]
        for k, v in sorted(self.totals.items(), key=lambda kv: -kv[1]):
            lines.append(f"{k:<28}{self.counts[k]:>8}{v / max(1, self.counts[k]):>12.3f}"
                         f"{100 * v / tot:>7.1f}%")
        return "\n".join(lines)
