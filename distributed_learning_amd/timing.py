"""Per-phase step timers with the reference's CSV schema, plus device-accurate timers.

Reference (/root/reference/src/timing.py:3-40): module-global dicts, ``start_timer``/``end_timer``
on ``time.time()*1000`` with no device synchronisation, ``end_timing_experiment`` appends one row
(per-timer mean for the batch + extra fields) and ``writeout_timer`` writes
``experiment_name, <timers in first-end order>, <extra fields>`` with a ``", "`` separator
(SURVEY.md Appendix A). That format is kept byte-compatible here so the reference's
``measurements/collect_data.py`` style analysis reads our files unchanged.

Additions:
* ``Timers(sync=True)`` synchronises the device at every boundary, so each phase's column is the
  real device time of that phase (the reference smears GPU time into whichever phase blocks next,
  SURVEY.md §5.1).
* ``EventTimers`` records HIP events on the current stream without any host sync and resolves them
  once per step — the headline-safe way to get per-phase device time.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Tuple

import torch

from .utils import trace


class Timers:
    def __init__(self, sync: bool = False):
        self.sync = sync and torch.cuda.is_available()
        self.collected: List[Tuple[str, Dict[str, float]]] = []
        self._starts: Dict[str, float] = {}
        self._sums: Dict[str, float] = {}
        self._counts: Dict[str, int] = {}

    def _now(self) -> float:
        if self.sync:
            torch.cuda.synchronize()
        return time.time() * 1000.0

    def start(self, name: str) -> None:
        trace.push(name)  # roctx range per phase when DLA_TRACE=1
        self._starts[name] = self._now()

    def end(self, name: str) -> None:
        trace.pop()
        dt = self._now() - self._starts[name]
        self._sums[name] = self._sums.get(name, 0.0) + dt
        self._counts[name] = self._counts.get(name, 0) + 1

    def end_experiment(self, experiment_name: str, extra_fields: Optional[Dict] = None) -> None:
        row = {k: v / self._counts[k] for k, v in self._sums.items()}
        row.update(extra_fields or {})
        self.collected.append((experiment_name, row))
        self._sums, self._counts, self._starts = {}, {}, {}

    def rows(self) -> List[Tuple[str, Dict[str, float]]]:
        return list(self.collected)

    def writeout(self, filename: str) -> None:
        if not self.collected:
            return
        keys = list(self.collected[0][1].keys())
        with open(filename, "w") as f:
            f.write("experiment_name, " + ", ".join(keys) + "\n")
            for name, row in self.collected:
                f.write(name + ", " + ", ".join(str(row[k]) for k in keys) + "\n")
        self.collected = []


class EventTimers:
    """Per-phase device time from HIP events (no host synchronisation inside the step)."""

    def __init__(self):
        self._pending: List[Tuple[str, "torch.cuda.Event", "torch.cuda.Event"]] = []
        self._open: Dict[str, "torch.cuda.Event"] = {}
        self.collected: List[Tuple[str, Dict[str, float]]] = []

    def start(self, name: str) -> None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._open[name] = ev

    def end(self, name: str) -> None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._pending.append((name, self._open.pop(name), ev))

    def end_experiment(self, experiment_name: str, extra_fields: Optional[Dict] = None) -> None:
        # events are resolved lazily (at writeout) so the training loop never blocks on the GPU
        self.collected.append((experiment_name, (list(self._pending), dict(extra_fields or {}))))
        self._pending = []

    def _resolve(self) -> None:
        out = []
        for name, item in self.collected:
            if isinstance(item, dict):
                out.append((name, item))
                continue
            events, extra = item
            row: Dict[str, float] = {}
            for ph, a, b in events:
                b.synchronize()
                row[ph] = row.get(ph, 0.0) + a.elapsed_time(b)
            row.update(extra)
            out.append((name, row))
        self.collected = out

    def writeout(self, filename: str) -> None:
        self._resolve()
        if not self.collected:
            return
        keys = list(self.collected[0][1].keys())
        with open(filename, "w") as f:
            f.write("experiment_name, " + ", ".join(keys) + "\n")
            for name, row in self.collected:
                f.write(name + ", " + ", ".join(str(row.get(k, "")) for k in keys) + "\n")
        self.collected = []


# ---- module-level API identical to the reference's timing.py --------------------------------
_GLOBAL = Timers()


def start_timer(name: str) -> None:
    _GLOBAL.start(name)


def end_timer(name: str) -> None:
    _GLOBAL.end(name)


def end_timing_experiment(experiment_name: str, extra_fields: Optional[Dict] = None) -> None:
    _GLOBAL.end_experiment(experiment_name, extra_fields)


def writeout_timer(filename: str) -> None:
    _GLOBAL.writeout(filename)
