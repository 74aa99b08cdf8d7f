"""Interpreter garbage-collector handling around an experiment.

Everything alive when an experiment starts — datasets, models, engines, the logger's stores — lives
for the whole run, yet every full (generation-2) collection walks it again: a single one measured
95 ms on the headline setup, 50 rounds' worth of device work (``bench.py`` prints the pauses).
With ``Settings.GC_FREEZE`` the objects alive at the start move to the permanent generation
(``gc.freeze``), so collections during the run only look at what the run itself allocates; the
experiment's end unfreezes them again. Driven by the node state's experiment lifecycle
(``NodeState.set_experiment`` / ``clear``), per node: the freeze lasts while any local node runs.
"""

from __future__ import annotations

import gc
import threading

from myfyp_amd.settings import Settings

_lock = threading.Lock()
_active: set = set()


def experiment_started(node: str) -> None:
    if not Settings.GC_FREEZE:
        return
    with _lock:
        if not _active:
            gc.freeze()
        _active.add(node)


def experiment_finished(node: str) -> None:
    with _lock:
        if node not in _active:
            return
        _active.discard(node)
        if not _active:
            gc.unfreeze()
