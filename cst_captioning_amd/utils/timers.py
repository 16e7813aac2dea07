"""Per-phase timers (rollout, reward, backward, all-reduce, optimizer).

On a GPU the phases are bracketed with HIP events recorded on the current
stream, so timing does not add host synchronisation inside the step; the
elapsed times are read once, at log time.  On CPU it falls back to wall
clock.  The reference only logs a per-iteration wall time
(``/root/reference/train.py:101,224,244``).
"""
import time
from collections import OrderedDict

import torch


class PhaseTimer:
    def __init__(self, enabled=True):
        self.enabled = enabled
        self.cuda = torch.cuda.is_available()
        self._marks = []

    def reset(self):
        self._marks = []

    def mark(self, name):
        if not self.enabled:
            return
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._marks.append((name, ev))
        else:
            self._marks.append((name, time.perf_counter()))

    def summary(self):
        """{phase: ms} where phase i spans mark i-1 .. mark i."""
        out = OrderedDict()
        if len(self._marks) < 2:
            return out
        if self.cuda:
            self._marks[-1][1].synchronize()
        for (_, a), (name, b) in zip(self._marks[:-1], self._marks[1:]):
            if self.cuda:
                out[name] = a.elapsed_time(b)
            else:
                out[name] = (b - a) * 1e3
        return out
