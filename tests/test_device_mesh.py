"""In-process device mesh (``parallel/device_mesh.py``): host collectives and the mesh workflow on CPU.

The reference runs every peer of a simulation in one process (``test/node_test.py:79-132``); the
device mesh keeps that process model across G devices. On CPU the members are ``cpu`` devices and
the collectives are :class:`HostMesh` torch ops; the RCCL implementation is covered on the GPU
(``tests/test_device_mesh_gpu.py``).
"""

from __future__ import annotations

import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
from myfyp_amd.learning.aggregators import FedAvg, FedMedian, FedProx, NeighborAvg, Scaffold
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.management.logger import logger
from myfyp_amd.models import MLP
from myfyp_amd.node import Node
from myfyp_amd.parallel.device_mesh import HostMesh, MeshError
from myfyp_amd.parallel.federation import Federation, mesh_devices
from myfyp_amd.settings import Settings
from myfyp_amd.utils.utils import check_equal_models, wait_to_finish

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cpu_mesh(g: int) -> HostMesh:
    return HostMesh([torch.device("cpu")] * g)


def test_host_mesh_collectives():
    m = _cpu_mesh(3)
    ts = [torch.full((5,), float(i + 1)) for i in range(3)]
    m.all_reduce_(ts)
    assert all(torch.equal(t, torch.full((5,), 6.0)) for t in ts)
    ts = [torch.tensor([1.0, 5.0]), torch.tensor([3.0, 2.0]), torch.tensor([2.0, 4.0])]
    m.all_reduce_(ts, op="max")
    assert all(t.tolist() == [3.0, 5.0] for t in ts)
    ts = [torch.arange(4.0) * (i + 1) for i in range(3)]
    m.broadcast_(ts, root=2)
    assert all(torch.equal(t, torch.arange(4.0) * 3) for t in ts)
    ins = [torch.full((2,), float(i)) for i in range(3)]
    outs = [torch.empty(6) for _ in range(3)]
    m.all_gather_(outs, ins)
    assert all(o.tolist() == [0, 0, 1, 1, 2, 2] for o in outs)
    a, b = torch.arange(3.0), torch.zeros(3)
    m.p2p_([("send", 0, 2, a), ("recv", 2, 0, b)])
    assert torch.equal(a, b)
    with pytest.raises(MeshError):
        m.p2p_([("recv", 1, 0, torch.zeros(3))])
    with pytest.raises(ValueError):
        m.all_reduce_([torch.zeros(2)] * 2)


def test_host_mesh_fedavg_matches_numpy():
    """rmesh_fedavg semantics: Σ_i Σ_p w x / Σ w into the masked rows of every group."""
    rng = np.random.default_rng(0)
    m = _cpu_mesh(2)
    n, ld = 10, 12
    P = [3, 2]
    params = [torch.from_numpy(rng.standard_normal((p, ld)).astype(np.float32)) for p in P]
    w = np.array([1.0, 0.0, 3.0, 2.0, 4.0], dtype=np.float32)
    mask = np.array([1, 1, 0, 1, 1], dtype=np.float32)
    rows = np.concatenate([p.numpy()[:, :n] for p in params])
    want = (w[:, None] * rows).sum(0) / w.sum()
    keep = [p.clone() for p in params]
    bufs = [torch.zeros(n + 1) for _ in P]
    m.fedavg_stacked(params, bufs, P, n, [ld, ld], w, mask)
    flat_mask = mask.astype(bool)
    allrows = torch.cat(params).numpy()
    allkeep = torch.cat(keep).numpy()
    np.testing.assert_allclose(allrows[flat_mask, :n], np.broadcast_to(want, (int(flat_mask.sum()), n)), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(allrows[~flat_mask], allkeep[~flat_mask])  # unmasked row untouched
    np.testing.assert_array_equal(allrows[:, n:], allkeep[:, n:])  # padding untouched


def test_host_mesh_shrink():
    m = _cpu_mesh(4)
    m.shrink([0, 2, 3])
    assert m.size == 3 and m.shrinks == 1


def test_mesh_devices_spec(monkeypatch):
    assert mesh_devices(None) is None and mesh_devices(1) is None
    assert mesh_devices(3) == [torch.device("cpu")] * 3  # CPU host: cpu members


@pytest.fixture
def data():
    return synthetic_mnist(1600, 400, seed=11, similarity=0.3, noise=0.5)


def _run(nodes, rounds, timeout=240):
    nodes[0].set_start_learning(rounds=rounds, epochs=1)
    wait_to_finish(nodes, timeout=timeout)


def _mesh_federation(data, aggregator, g: int, n: int, rounds: int = 2):
    Settings.BATCH_SIZE = 16
    Settings.TRAIN_SET_SIZE = n
    from myfyp_amd.utils.seed import set_seed

    set_seed(7)
    Federation.reset()
    fed = Federation.init(devices=g) if g > 1 else Federation.init()
    parts = data.generate_partitions(n, RandomIIDPartitionStrategy)
    exp = f"mesh-{g}-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"m{g}-{i}-{time.time_ns()}", aggregator=aggregator(), protocol=CollectiveCommunicationProtocol,
                  exp_name=exp) for i in range(n)]
    for nd in nodes:
        nd.start()
    try:
        fed.finalize()
        _run(nodes, rounds)
        params = [np.concatenate([p.ravel() for p in nd.learner.get_model().get_parameters()]) for nd in nodes]
        return fed, nodes, exp, params
    finally:
        for nd in nodes:
            nd.stop()


@pytest.mark.parametrize("aggregator", [FedAvg, FedMedian, lambda: Scaffold(global_lr=1.0), FedProx, lambda: NeighborAvg(topology="ring")],
                         ids=["fedavg", "fedmedian", "scaffold", "fedprox", "neighbor-ring"])
def test_mesh_workflow_matches_single_device(data, aggregator):
    """4 peers on a 2-device CPU mesh (round-robin placement, mesh collectives) end where the same
    federation on one device ends (the reduction order differs: fp32 tolerance)."""
    try:
        fed, nodes, exp, mesh_params = _mesh_federation(data, aggregator, 2, 4)
        assert fed.mesh is not None and fed.mesh.calls > 0
        assert [nd.learner.mesh_rank for nd in nodes] == [0, 1, 0, 1]
        assert all(nd.learning_workflow.history.count("RoundFinishedStage") == 2 for nd in nodes)
        if not isinstance(nodes[0].aggregator, NeighborAvg):
            for p in mesh_params[1:]:
                np.testing.assert_allclose(p, mesh_params[0], atol=1e-5)
        Federation.reset()
        _, _, _, solo_params = _mesh_federation(data, aggregator, 1, 4)
        for a, b in zip(mesh_params, solo_params):
            # Adam's step is ~lr whatever the gradient's size, so a reduction-order ulp that flips
            # the sign of a near-zero gradient moves that coordinate by ~lr (1e-3) per later step:
            # the bound is on the mean deviation, with a loose cap on the largest one
            d = np.abs(a - b)
            assert d.mean() < 1e-4 and d.max() < 0.05, (float(d.mean()), float(d.max()))
    finally:
        Federation.reset()


def test_mesh_learns_and_drops_an_empty_device(data):
    """A peer that stops mid-experiment takes its device out of the mesh (abort + init-all over
    the survivors); the others finish and agree."""
    Settings.BATCH_SIZE = 16
    Settings.TRAIN_SET_SIZE = 3
    Federation.reset()
    fed = Federation.init(devices=3)
    parts = data.generate_partitions(3, RandomIIDPartitionStrategy)
    exp = f"meshdrop-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"md-{i}-{time.time_ns()}", protocol=CollectiveCommunicationProtocol, exp_name=exp)
             for i in range(3)]
    for nd in nodes:
        nd.start()
    try:
        fed.finalize()
        from myfyp_amd.fault_injection import kill_at

        kill_at(nodes[2], "TrainStage", round=1)
        _run(nodes[:2], 4)
        assert fed.mesh_members == [0, 1] and fed.mesh.shrinks == 1
        check_equal_models(nodes[:2], atol=1e-5)
        logs = logger.get_global_logs()[exp]
        acc = dict(logs[nodes[0].addr]["test_metric"])
        assert acc[max(acc)] > 0.5, acc
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()


def test_bench_refuses_missing_gpus():
    """``bench.py --gpus 8`` with no launcher and no GPUs exits non-zero (never a 1-GPU number)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "0"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode != 0
    assert "GPU" in (r.stderr + r.stdout)


def test_bench_virtual_mesh_cpu():
    """``--mesh-virtual``: 4 mesh ranks on the CPU run the mesh path and report 0 physical GPUs."""
    import json

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--mesh-virtual", "--steps", "2", "--warmup", "1", "--n-train", "2000",
                        "--n-test", "400"], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 0 and out["config"]["peers_per_gpu"] == 2
    assert "mesh" in out["config"]["collective"]


def test_bench_torchrun_mesh_parks_other_ranks_cpu():
    """The driver's launch shape (``torch.distributed.run --nproc-per-node 2 bench.py --gpus 2``) with
    ``--launch mesh --mesh-virtual`` on the CPU: rank 0 drives the two-member mesh, rank 1 parks on
    the gloo barrier, both exit 0, and exactly one JSON line is printed."""
    import json

    from _ports import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
           str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch", "mesh", "--mesh-virtual", "--steps", "2", "--warmup", "1",
           "--n-train", "2000", "--n-test", "400"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["config"]["peers_per_gpu"] == 4 and "mesh" in out["config"]["collective"]


def test_mesh_falls_back_to_host_when_rccl_init_fails(monkeypatch):
    """An RCCL mesh that cannot be created (auto backend) leaves a host mesh over the same devices,
    reported as ``kind == "host"``; an explicitly requested backend still raises."""
    from myfyp_amd.parallel import device_mesh

    def broken(devs, backend=None):
        raise MeshError("ncclCommInitAll failed (test)")

    monkeypatch.setattr(device_mesh, "make_mesh", broken)
    Federation.reset()
    try:
        fed = Federation._init_mesh([torch.device("cpu"), torch.device("cpu")], None)
        assert fed.mesh.kind == "host" and fed.mesh_size == 2
        Federation.reset()
        with pytest.raises(MeshError):
            Federation._init_mesh([torch.device("cpu"), torch.device("cpu")], "rccl")
    finally:
        Federation.reset()
