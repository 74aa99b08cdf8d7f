"""Simulation device pool (reference: test/simulation/actor_pool_test.py,
test/simulation/virtual_node_learner_test.py).

The reference drives a real local Ray cluster and patches ``ray.get``/``ray.wait``; the pool here is
in-process (device worker threads), so the tests run it for real on CPU workers with fake learners:
singleton, sizing from resources, idle/pending submission, per-address results, dead-worker
removal, pool shrinking, and a two-node federated run whose learners go through the pool.
"""

import threading
import time

import pytest

from myfyp_amd.learning.frameworks.simulation import (
    ActorDiedError,
    SuperActorPool,
    VirtualLearnerActor,
    VirtualNodeLearner,
    check_client_resources,
    pool_size_from_resources,
    try_init_learner_with_ray,
)
from myfyp_amd.learning.frameworks.simulation.utils import pool_devices
from myfyp_amd.settings import Settings

CPU8 = {"CPU": 8, "GPU": 0}


@pytest.fixture(autouse=True)
def fresh_pool():
    SuperActorPool.reset()
    yield
    SuperActorPool.reset()


class FakeLearner:
    """Records concurrency; ``fit`` returns a per-learner model object."""

    active = 0
    peak = 0
    lock = threading.Lock()

    def __init__(self, name, delay=0.02, fail=None):
        self.name = name
        self.delay = delay
        self.fail = fail
        self.model = object()
        self.fits = 0
        self.interrupted = False
        self.epochs = 1

    def fit(self):
        with FakeLearner.lock:
            FakeLearner.active += 1
            FakeLearner.peak = max(FakeLearner.peak, FakeLearner.active)
        try:
            time.sleep(self.delay)
            if self.fail is not None:
                raise self.fail
            self.fits += 1
            return self.model
        finally:
            with FakeLearner.lock:
                FakeLearner.active -= 1

    def evaluate(self):
        return {"test_acc": 0.5, "who": self.name}

    def get_model(self):
        return self.model

    def set_model(self, m):
        self.model = m

    def set_epochs(self, e):
        self.epochs = e

    def interrupt_fit(self):
        self.interrupted = True

    def get_framework(self):
        return "pytorch"


def _fit(actor, addr, learner):
    return actor.fit(addr, learner)


def test_resources_and_pool_size():
    assert check_client_resources(None) == {"num_cpus": 1, "num_gpus": 0.0}
    assert check_client_resources({"num_gpus": 0.5})["num_cpus"] == 1
    with pytest.raises(ValueError):
        check_client_resources({"num_cpus": 0})
    assert pool_size_from_resources({"num_cpus": 2}, CPU8) == 4
    assert pool_size_from_resources({"num_cpus": 1, "num_gpus": 0.25}, {"CPU": 64, "GPU": 2}) == 8
    assert pool_size_from_resources({"num_cpus": 4, "num_gpus": 0.25}, {"CPU": 8, "GPU": 2}) == 2
    with pytest.raises(ValueError):
        pool_size_from_resources({"num_cpus": 1, "num_gpus": 1}, CPU8)  # needs a GPU, none visible
    with pytest.raises(ValueError):
        pool_size_from_resources({"num_cpus": 16}, CPU8)
    assert pool_devices({"num_cpus": 1, "num_gpus": 0.5}, 4, {"CPU": 8, "GPU": 2}) == ["cuda:0", "cuda:1", "cuda:0", "cuda:1"]
    assert pool_devices({"num_cpus": 1}, 2, CPU8) == ["cpu", "cpu"]


def test_singleton_and_initialisation():
    p = SuperActorPool({"num_cpus": 4}, inventory=CPU8)
    assert p is SuperActorPool() and p.num_actors == 2 and len(p._idle_actors) == 2
    assert p.devices() == ["cpu"]
    p.add_actor(1)
    assert p.num_actors == 3 and len(p._idle_actors) == 3


def test_jobs_bounded_by_pool_size_and_results_per_address():
    p = SuperActorPool({"num_cpus": 4}, inventory=CPU8)  # 2 workers
    FakeLearner.active = FakeLearner.peak = 0
    learners = {f"n{i}": FakeLearner(f"n{i}") for i in range(5)}
    for a, lr in learners.items():
        p.submit_learner_job(_fit, (a, lr))
    assert len(p._pending_submits) >= 1  # more jobs than workers: the rest wait
    for a, lr in learners.items():
        addr, model = p.get_learner_result(a, timeout=10)
        assert addr == a and model is lr.model and lr.fits == 1
    assert FakeLearner.peak <= 2
    assert not p.has_next()
    assert len(p._idle_actors) == 2
    with pytest.raises(StopIteration):
        p.process_unordered_future(timeout=0.1)


def test_ordinary_failure_keeps_worker():
    p = SuperActorPool({"num_cpus": 8}, inventory=CPU8)  # 1 worker
    p.submit_learner_job(_fit, ("bad", FakeLearner("bad", fail=ValueError("boom"))))
    with pytest.raises(ValueError):
        p.get_learner_result("bad", timeout=10)
    assert p.num_actors == 1
    p.submit_learner_job(_fit, ("ok", FakeLearner("ok")))
    assert p.get_learner_result("ok", timeout=10)[0] == "ok"


def test_dead_worker_is_removed_and_queue_moves_on():
    p = SuperActorPool({"num_cpus": 4}, inventory=CPU8)  # 2 workers
    dying = FakeLearner("dying", fail=RuntimeError("HIP error: an illegal memory access was encountered"))
    p.submit_learner_job(_fit, ("dying", dying))
    with pytest.raises(ActorDiedError):
        p.get_learner_result("dying", timeout=10)
    assert p.num_actors == 1 and len(p._actors) == 1
    for i in range(3):
        p.submit_learner_job(_fit, (f"s{i}", FakeLearner(f"s{i}")))
    for i in range(3):
        assert p.get_learner_result(f"s{i}", timeout=10)[0] == f"s{i}"
    # the last worker dies too: queued work fails instead of hanging
    p.submit_learner_job(_fit, ("d2", FakeLearner("d2", fail=ActorDiedError("x"))))
    with pytest.raises(ActorDiedError):
        p.get_learner_result("d2", timeout=10)
    assert p.num_actors == 0
    p.submit_learner_job(_fit, ("late", FakeLearner("late")))
    with pytest.raises(ActorDiedError):
        p.get_learner_result("late", timeout=10)


def test_flagged_worker_removed_on_next_use_and_pool_shrinks():
    a, b = VirtualLearnerActor("cpu"), VirtualLearnerActor("cpu")
    p = SuperActorPool({"num_cpus": 1}, actor_list=[a, b], inventory=CPU8)
    p._flag_actor_for_removal(a.actor_id)
    assert p._check_and_remove_actor_from_pool(a) is False and p.num_actors == 1
    assert p._check_and_remove_actor_from_pool(b) is True
    p._inventory = {"CPU": 0, "GPU": 0}  # the host lost its CPUs: the pool must shrink
    assert p._check_actor_fits_in_pool() is False and p.num_actors == 0


def test_timeout_and_unordered_processing():
    p = SuperActorPool({"num_cpus": 8}, inventory=CPU8)
    p.submit_learner_job(_fit, ("slow", FakeLearner("slow", delay=0.5)))
    with pytest.raises(TimeoutError):
        p.get_learner_result("slow", timeout=0.05)
    with pytest.raises(TimeoutError):
        p.process_unordered_future(timeout=0.01)
    p.process_unordered_future(timeout=5)
    assert p.get_learner_result("slow", timeout=5)[0] == "slow"


def test_device_placement_is_sticky_and_balanced():
    p = SuperActorPool({"num_cpus": 1}, actor_list=[VirtualLearnerActor("cpu") for _ in range(2)], inventory=CPU8)
    assert p.place("x") == "cpu" and p.place("x") == "cpu"
    # a learner pinned to a device with no worker may use any worker
    lr = FakeLearner("g")
    lr.device = "cuda:3"
    p.submit_learner_job(_fit, ("g", lr))
    assert p.get_learner_result("g", timeout=10)[1] is lr.model


def test_virtual_node_learner_delegates_and_fits_through_pool():
    SuperActorPool({"num_cpus": 4}, inventory=CPU8)
    inner = FakeLearner("v")
    v = VirtualNodeLearner(inner, "v")
    v.set_epochs(3)
    assert inner.epochs == 3 and v.epochs == 3
    m = object()
    v.set_model(m)
    assert v.get_model() is m and v.model is m
    assert v.fit() is m and inner.fits == 1
    assert v.evaluate()["who"] == "v"
    assert v.get_framework() == "pytorch"
    v.interrupt_fit()
    assert inner.interrupted
    assert not hasattr(v, "_engine") and not hasattr(v, "fit_request")
    inner.fail = ValueError("nope")
    with pytest.raises(ValueError):
        v.fit()


def test_try_init_learner_with_ray_wraps_only_when_enabled():
    sentinel = object()
    assert try_init_learner_with_ray(sentinel) is sentinel
    old = Settings.SIMULATION_POOL, Settings.SIMULATION_RESOURCES
    Settings.SIMULATION_POOL, Settings.SIMULATION_RESOURCES = True, {"num_cpus": 4}
    try:
        lr = FakeLearner("w")
        v = try_init_learner_with_ray(lr, addr="w")
        assert isinstance(v, VirtualNodeLearner) and v.learner is lr
    finally:
        Settings.SIMULATION_POOL, Settings.SIMULATION_RESOURCES = old


@pytest.mark.gpu
def test_pool_gpu_workers_train_four_peers():
    """Four peers share one MI355X through two pool workers (two HIP streams)."""
    import torch

    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.node import Node
    from myfyp_amd.utils.utils import check_equal_models, wait_convergence, wait_to_finish

    old = Settings.SIMULATION_POOL, Settings.BATCH_SIZE
    Settings.SIMULATION_POOL, Settings.BATCH_SIZE = True, 64
    nodes = []
    try:
        pool = SuperActorPool({"num_cpus": 1, "num_gpus": 0.5}, inventory={"CPU": 16, "GPU": 1})
        assert pool.devices() == ["cuda:0"] and pool.num_actors == 2
        parts = synthetic_mnist(4000, 400, seed=7).generate_partitions(4, RandomIIDPartitionStrategy)
        exp = f"poolgpu-{time.time_ns()}"
        nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"pg-{i}-{time.time_ns()}", exp_name=exp) for i in range(4)]
        assert all(str(nd.learner.device) == "cuda:0" for nd in nodes)
        for nd in nodes:
            nd.start()
        for i in range(1, 4):
            nodes[0].connect(nodes[i].addr)
        wait_convergence(nodes, 3, only_direct=False, wait=10)
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_to_finish(nodes, timeout=100)
        check_equal_models(nodes)
        assert all(a.device.type == "cuda" and a.jobs_done > 0 for a in pool._actors.values())
        assert torch.cuda.is_available()
    finally:
        for nd in nodes:
            nd.stop()
        Settings.SIMULATION_POOL, Settings.BATCH_SIZE = old


def test_two_nodes_train_through_the_pool():
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.node import Node
    from myfyp_amd.utils.utils import check_equal_models, wait_convergence, wait_to_finish

    old = Settings.SIMULATION_POOL, Settings.SIMULATION_RESOURCES, Settings.BATCH_SIZE
    Settings.SIMULATION_POOL, Settings.SIMULATION_RESOURCES, Settings.BATCH_SIZE = True, {"num_cpus": 8}, 32
    nodes = []
    try:
        parts = synthetic_mnist(1200, 200, seed=5).generate_partitions(2, RandomIIDPartitionStrategy)
        exp = f"pool-{time.time_ns()}"
        SuperActorPool({"num_cpus": 8}, inventory=CPU8)  # the nodes below pick up this instance
        nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"pool-{i}-{time.time_ns()}", exp_name=exp) for i in range(2)]
        assert all(isinstance(nd.learner, VirtualNodeLearner) for nd in nodes)
        pool = SuperActorPool()
        assert pool.num_actors == 1  # one worker: the two peers' fits are serialised
        for nd in nodes:
            nd.start()
        nodes[0].connect(nodes[1].addr)
        wait_convergence(nodes, 1, only_direct=True, wait=10)
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_to_finish(nodes, timeout=120)
        check_equal_models(nodes)
        assert sum(a.jobs_done for a in pool._actors.values()) >= 4  # 2 peers x 2 rounds of fits (+ evaluations)
    finally:
        for nd in nodes:
            nd.stop()
        Settings.SIMULATION_POOL, Settings.SIMULATION_RESOURCES, Settings.BATCH_SIZE = old
