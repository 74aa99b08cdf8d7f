"""GC freeze across the experiment lifecycle (``myfyp_amd/utils/gc_tuning.py``)."""

import gc

from myfyp_amd.node_state import NodeState
from myfyp_amd.settings import Settings


def test_freeze_lasts_while_any_node_runs(monkeypatch):
    monkeypatch.setattr(Settings, "GC_FREEZE", True)
    gc.unfreeze()
    base = gc.get_freeze_count()
    a, b = NodeState("gc-a"), NodeState("gc-b")
    a.set_experiment("exp", 2)
    assert gc.get_freeze_count() > base
    b.set_experiment("exp", 2)
    a.clear()
    assert gc.get_freeze_count() > base  # b still runs
    b.clear()
    assert gc.get_freeze_count() == 0
    b.clear()  # a second clear is harmless
    assert gc.get_freeze_count() == 0


def test_no_freeze_when_disabled(monkeypatch):
    monkeypatch.setattr(Settings, "GC_FREEZE", False)
    gc.unfreeze()
    s = NodeState("gc-c")
    s.set_experiment("exp", 1)
    assert gc.get_freeze_count() == 0
    s.clear()
