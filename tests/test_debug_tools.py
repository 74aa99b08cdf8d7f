"""Debug subsystems: lock-order checking and roctx tracing ranges."""

import threading
import time

import pytest

from myfyp_amd.management import tracing
from myfyp_amd.settings import Settings
from myfyp_amd.utils import lockcheck


@pytest.fixture
def lock_check():
    old = Settings.LOCK_CHECK
    Settings.LOCK_CHECK = True
    lockcheck.reset()
    yield
    Settings.LOCK_CHECK = old
    lockcheck.reset()


def test_inversion_is_recorded_without_a_deadlock(lock_check):
    a, b = lockcheck.make_lock("T.a"), lockcheck.make_lock("T.b")
    assert isinstance(a, lockcheck.CheckedLock)
    with a:
        with b:
            pass
    assert lockcheck.violations() == []

    def other():  # opposite order, later in time: the schedule never deadlocks, the order does
        with b:
            with a:
                pass

    t = threading.Thread(target=other)
    t.start()
    t.join()
    v = lockcheck.violations()
    assert len(v) == 1 and v[0][:2] == ("T.b", "T.a")
    assert lockcheck.lock_graph() == {"T.a": ["T.b"], "T.b": ["T.a"]}


def test_raise_mode_reentrancy_and_same_name_nesting(lock_check):
    Settings.LOCK_CHECK = "raise"
    r = lockcheck.make_lock("T.r", reentrant=True)
    with r:
        with r:  # re-entry is not an edge
            assert r.locked()
    assert not r.locked()
    x1, x2 = lockcheck.make_lock("T.same"), lockcheck.make_lock("T.same")
    with x1, x2:  # two instances of one lock class
        pass
    a, b, c = (lockcheck.make_lock(n) for n in ("T.p", "T.q", "T.s"))
    with a, b:
        pass
    with b, c:
        pass
    with pytest.raises(lockcheck.LockOrderError):
        with c:
            with a:  # closes p -> q -> s -> p
                pass
    assert not c.locked()


def test_plain_locks_when_off():
    assert Settings.LOCK_CHECK is False
    assert not isinstance(lockcheck.make_lock("T.off"), lockcheck.CheckedLock)


def test_gossip_experiment_has_consistent_lock_order(lock_check):
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.node import Node
    from myfyp_amd.utils.utils import wait_convergence, wait_to_finish

    old_bs, old_trace = Settings.BATCH_SIZE, Settings.TRACE_MARKERS
    Settings.BATCH_SIZE, Settings.TRACE_MARKERS = 32, True  # tracing on too: ranges must balance
    nodes = []
    try:
        parts = synthetic_mnist(900, 150, seed=11).generate_partitions(3, RandomIIDPartitionStrategy)
        exp = f"lock-{time.time_ns()}"
        nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"lk-{i}-{time.time_ns()}", exp_name=exp) for i in range(3)]
        assert isinstance(nodes[0].aggregator._agg_lock, lockcheck.CheckedLock)
        for nd in nodes:
            nd.start()
        nodes[0].connect(nodes[1].addr)
        nodes[1].connect(nodes[2].addr)
        wait_convergence(nodes, 2, only_direct=False, wait=10)
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_to_finish(nodes, timeout=120)
    finally:
        for nd in nodes:
            nd.stop()
        Settings.BATCH_SIZE, Settings.TRACE_MARKERS = old_bs, old_trace
    assert lockcheck.violations() == [], lockcheck.violations()
    assert lockcheck.lock_graph() is not None


def test_trace_ranges_nest_and_are_noops_when_off():
    old = Settings.TRACE_MARKERS
    try:
        Settings.TRACE_MARKERS = False
        assert tracing.trace_range("x") is tracing.trace_range("y")  # shared null context
        Settings.TRACE_MARKERS = True
        if not tracing.enabled():
            pytest.skip("roctx library not available")
        with tracing.trace_range("outer"):
            with tracing.trace_range("inner"):
                assert tracing.depth() == 2
        assert tracing.depth() == 0

        class Peer:
            _self_addr = "peer-7"

            @tracing.traced("work")
            def work(self):
                return tracing.depth()

        assert Peer().work() == 1
        tracing.mark("done")
    finally:
        Settings.TRACE_MARKERS = old
