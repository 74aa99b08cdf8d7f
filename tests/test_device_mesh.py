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


# ---------------------------------------------------------------------------------------------
# mesh guard (parallel/mesh_guard.py): deadline, async-error poll, abort, rebuild, aggregate what
# arrived (reference: aggregator.py:177-208, wait_agg_models_stage.py:40-67)
# ---------------------------------------------------------------------------------------------
@pytest.fixture
def short_timeouts():
    saved = (Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT, Settings.COLLECTIVE_FAILOVER)
    Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT, Settings.COLLECTIVE_FAILOVER = 0.3, 0.2, True
    yield
    Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT, Settings.COLLECTIVE_FAILOVER = saved


def _stacked_fedavg(fed, params, P, n, ld, w, mask):
    """The stacked path of weights_plane._mesh_mean on explicit rows (out of place + guarded)."""
    bufs = [torch.zeros(n + 1) for _ in P]
    outs = [torch.zeros(n + 1) for _ in P]
    offs = np.concatenate([[0], np.cumsum(P)])
    fed.mesh.fedavg_stacked(params, bufs, P, n, ld, w, mask, outs=outs)

    def retry():
        live = list(fed.mesh_members)
        fed.mesh.fedavg_retry([params[r] for r in live], [bufs[r] for r in live], [outs[r] for r in live], [P[r] for r in live], n,
                              [ld[r] for r in live], np.concatenate([mask[offs[r] : offs[r + 1]] for r in live]))

    fed.mesh_track("fedavg", retry)


def _want(rows, w, members_rows):
    sel = np.concatenate(members_rows)
    return (w[sel, None] * rows[sel]).sum(0) / w[sel].sum()


def test_mesh_guard_stalled_member_aggregates_survivors(short_timeouts):
    """A mesh member that never completes the FedAvg: the deadline expires, the watchdog aborts the
    mesh, the confirmation probes the devices, rebuilds over the two that answer, drops the third,
    and re-runs the all-reduce from the survivors' retained partial sums: their rows end at the
    survivors' weighted average (the models that arrived), not the three-member one."""
    rng = np.random.default_rng(3)
    Federation.reset()
    try:
        fed = Federation._init_mesh([torch.device("cpu")] * 3, "host")
        n, ld, P = 9, 12, [2, 1, 2]
        params = [torch.from_numpy(rng.standard_normal((p, ld)).astype(np.float32)) for p in P]
        rows = np.concatenate([p.numpy()[:, :n] for p in params])
        w = np.array([1.0, 2.0, 3.0, 4.0, 5.0], dtype=np.float32)
        mask = np.ones(5, dtype=np.float32)
        fed.mesh.stall(2)  # device 2 hangs: its completion markers and probes never fire
        _stacked_fedavg(fed, params, P, n, [ld] * 3, w, mask)
        time.sleep(0.5)  # past the deadline: the watchdog aborts the mesh
        assert fed.mesh_guard.aborted and fed.mesh.aborted
        assert fed.mesh_confirm() is True
        assert fed.mesh_members == [0, 1] and fed.mesh_guard.lost == [2] and fed.mesh_guard.recoveries == 1
        want = _want(rows, w, [np.arange(0, 2), np.arange(2, 3)])
        got = np.concatenate([params[0].numpy()[:, :n], params[1].numpy()[:, :n]])
        np.testing.assert_allclose(got, np.broadcast_to(want, got.shape), rtol=1e-5, atol=1e-6)
        fed.mesh.check()  # healthy again
        assert fed.mesh_confirm() is False  # the retry's own collective confirmed
    finally:
        Federation.reset()


def test_mesh_guard_async_error_reinit_keeps_every_member(short_timeouts):
    """An asynchronous error reported by the mesh (fault hook) on a collective that did complete:
    abort, every device answers the probe, the mesh is re-initialised over all of them and the
    FedAvg re-run from the retained partials gives exactly the undisturbed result."""
    rng = np.random.default_rng(4)
    Federation.reset()
    try:
        fed = Federation._init_mesh([torch.device("cpu")] * 2, "host")
        n, ld, P = 7, 8, [2, 2]
        params = [torch.from_numpy(rng.standard_normal((p, ld)).astype(np.float32)) for p in P]
        ref = [p.clone() for p in params]
        w = np.array([1.0, 0.0, 3.0, 2.0], dtype=np.float32)
        mask = np.array([1, 1, 0, 1], dtype=np.float32)
        _stacked_fedavg(fed, ref, P, n, [ld] * 2, w, mask)
        assert fed.mesh_confirm() is False
        _stacked_fedavg(fed, params, P, n, [ld] * 2, w, mask)
        fed.mesh.inject_error(1)
        assert fed.mesh_confirm() is True
        assert fed.mesh_members == [0, 1] and fed.mesh_guard.lost == [] and fed.mesh.shrinks == 1
        for a, b in zip(params, ref):
            assert torch.equal(a, b)
    finally:
        Federation.reset()


def test_mesh_workflow_survives_a_hung_device(data, short_timeouts):
    """3 peers on a 3-device CPU mesh; device 2 hangs in round 1. Its peer leaves, the survivors
    finish every round over the rebuilt two-device mesh and agree."""
    from myfyp_amd.fault_injection import StageFault

    Settings.BATCH_SIZE = 16
    Settings.TRAIN_SET_SIZE = 3
    Federation.reset()
    fed = Federation.init(devices=3)
    parts = data.generate_partitions(3, RandomIIDPartitionStrategy)
    exp = f"meshhang-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"mh-{i}-{time.time_ns()}", protocol=CollectiveCommunicationProtocol, exp_name=exp)
             for i in range(3)]
    for nd in nodes:
        nd.start()
    try:
        fed.finalize()
        assert [nd.learner.mesh_rank for nd in nodes] == [0, 1, 2]
        StageFault(nodes[2], "TrainStage", lambda n: fed.mesh.stall(2), round=1)
        _run(nodes[:2], 4)
        assert fed.mesh_members == [0, 1] and fed.mesh_guard.recoveries >= 1 and fed.mesh_guard.lost == [2]
        assert nodes[2].addr not in fed.local_nodes
        assert all(nd.learning_workflow.history.count("RoundFinishedStage") == 4 for nd in nodes[:2])
        check_equal_models(nodes[:2], atol=1e-5)
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()


def test_bench_refuses_a_host_mesh_on_physical_gpus():
    """``--gpus N`` over physical GPUs must run on the RCCL mesh: a host-copy mesh is refused (a
    virtual rehearsal is not)."""
    from types import SimpleNamespace

    from myfyp_amd.utils import launch

    fed = SimpleNamespace(mesh=SimpleNamespace(kind="host"), mesh_size=2)
    with pytest.raises(SystemExit, match="RCCL"):
        launch.check_mesh(fed, 2, virtual=False)
    launch.check_mesh(fed, 2, virtual=True)
    launch.check_mesh(SimpleNamespace(mesh=SimpleNamespace(kind="rccl"), mesh_size=2), 2, virtual=False)
    with pytest.raises(SystemExit):
        launch.check_mesh(SimpleNamespace(mesh=None, mesh_size=1), 2, virtual=False)


def test_torchrun_defaults_to_one_process_per_gpu(monkeypatch):
    """Under torchrun ``--launch auto`` is one process per GPU; one process started
    with ``--gpus N`` drives a mesh."""
    from myfyp_amd.utils import launch

    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "2")
    assert launch.plan_launch(4, "auto") == "ranks"
    assert launch.plan_launch(4, "mesh", mesh_virtual=True) == "park"
    monkeypatch.setenv("RANK", "0")
    assert launch.plan_launch(4, "mesh", mesh_virtual=True) == "mesh"
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert launch.plan_launch(3, "auto", mesh_virtual=True) == "mesh"
    assert launch.plan_launch(1, "auto") == "single"


# ---------------------------------------------------------------------------------------------
# bucketed, overlapped mesh FedAvg (rmesh_fedavg_bucketed semantics)
# ---------------------------------------------------------------------------------------------
def _bucketed_case(seed: int, P=(3, 2), n=10, ld=12):
    rng = np.random.default_rng(seed)
    params = [torch.from_numpy(rng.standard_normal((p, ld)).astype(np.float32)) for p in P]
    rows = np.concatenate([p.numpy()[:, :n] for p in params])
    return list(P), n, ld, params, rows


@pytest.mark.parametrize("bucket", [4, 8, 1 << 20])
def test_host_mesh_bucketed_fedavg_matches_numpy(bucket):
    """Partial sums [Σw, pad x3 | Σ w x] retained in ``keeps``, per-bucket all-reduce into ``outs``,
    the mean applied to the masked rows; unmasked rows and padding untouched; every bucket size
    (one float4 per bucket up to one bucket) gives the same rows."""
    P, n, ld, params, rows = _bucketed_case(0)
    m = _cpu_mesh(2)
    w = np.array([1.0, 0.0, 3.0, 2.0, 4.0], dtype=np.float32)
    mask = np.array([1, 1, 0, 1, 1], dtype=np.float32)
    before = [p.clone() for p in params]
    keeps = [torch.zeros(n + 4) for _ in P]
    outs = [torch.zeros(n + 4) for _ in P]
    m.fedavg_bucketed(params, keeps, outs, P, n, [ld, ld], w, mask, [None, None], bucket, apply=True)
    want = (w[:, None] * rows).sum(0) / w.sum()
    allrows, allbefore = torch.cat(params).numpy(), torch.cat(before).numpy()
    fm = mask.astype(bool)
    np.testing.assert_allclose(allrows[fm, :n], np.broadcast_to(want, (int(fm.sum()), n)), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(allrows[~fm], allbefore[~fm])
    np.testing.assert_array_equal(allrows[:, n:], allbefore[:, n:])
    # each member keeps its own partial sum (the retry input); outs hold the global one
    np.testing.assert_allclose(keeps[0][4:].numpy(), (w[:3, None] * rows[:3]).sum(0), rtol=1e-6)
    assert float(keeps[1][0]) == 6.0 and float(outs[0][0]) == float(outs[1][0]) == float(w.sum())


def test_host_mesh_delayed_averaging_lands_a_round_later():
    """Delayed averaging on the mesh: round r's snapshot is exchanged with no apply; at round r + 1
    every masked row lands x += avg_r - snap_r (its local progress since the snapshot kept) and is
    snapshotted again."""
    P, n, ld, params, rows = _bucketed_case(1, P=(2, 2), n=6, ld=8)
    m = _cpu_mesh(2)
    w = np.array([1.0, 2.0, 3.0, 4.0], dtype=np.float32)
    mask = np.ones(4, dtype=np.float32)
    snaps = [torch.zeros(p * n) for p in P]
    keeps = [torch.zeros(n + 4) for _ in P]
    outs = [torch.zeros(n + 4) for _ in P]
    m.delayed_land(params, snaps, outs, P, n, [ld, ld], n, mask, False)  # first round: snapshot only
    m.fedavg_bucketed(snaps, keeps, outs, P, n, [n, n], w, mask, [None, None], 4, apply=False)
    avg = (w[:, None] * rows).sum(0) / w.sum()
    assert np.array_equal(torch.cat(params).numpy()[:, :n], rows)  # nothing applied yet
    step = [torch.full_like(p, 0.25) for p in params]  # the next local epoch's progress
    for p, d in zip(params, step):
        p.add_(d)
    m.delayed_land(params, snaps, outs, P, n, [ld, ld], n, mask, True)
    got = torch.cat(params).numpy()[:, :n]
    np.testing.assert_allclose(got, np.broadcast_to(avg + 0.25, got.shape), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(torch.cat([s.view(p, n) for s, p in zip(snaps, P)]).numpy(), got, rtol=0, atol=0)


def _bucketed_guarded(fed, params, P, n, ld, w, mask, bucket=4):
    keeps = [torch.zeros(n + 4) for _ in P]
    outs = [torch.zeros(n + 4) for _ in P]
    offs = np.concatenate([[0], np.cumsum(P)])
    fed.mesh.fedavg_bucketed(params, keeps, outs, P, n, ld, w, mask, [None] * len(P), bucket, apply=True)

    def retry():
        live = list(fed.mesh_members)
        fed.mesh.fedavg_bucketed_retry([params[r] for r in live], [keeps[r] for r in live], [outs[r] for r in live], [P[r] for r in live], n,
                                       [ld[r] for r in live], np.concatenate([mask[offs[r] : offs[r + 1]] for r in live]))

    fed.mesh_track("fedavg", retry)


def test_mesh_guard_bucketed_stalled_member_aggregates_survivors(short_timeouts):
    """The stalled-device recovery on the bucketed exchange: the survivors' retained [Σw | Σ w x]
    are all-reduced again over the rebuilt mesh and applied — the average of what arrived."""
    rng = np.random.default_rng(7)
    Federation.reset()
    try:
        fed = Federation._init_mesh([torch.device("cpu")] * 3, "host")
        n, ld, P = 9, 12, [2, 1, 2]
        params = [torch.from_numpy(rng.standard_normal((p, ld)).astype(np.float32)) for p in P]
        rows = np.concatenate([p.numpy()[:, :n] for p in params])
        w = np.array([1.0, 2.0, 3.0, 4.0, 5.0], dtype=np.float32)
        mask = np.ones(5, dtype=np.float32)
        fed.mesh.stall(2)
        _bucketed_guarded(fed, params, P, n, [ld] * 3, w, mask)
        time.sleep(0.5)
        assert fed.mesh_confirm() is True
        assert fed.mesh_members == [0, 1] and fed.mesh_guard.lost == [2]
        want = _want(rows, w, [np.arange(0, 2), np.arange(2, 3)])
        got = np.concatenate([params[0].numpy()[:, :n], params[1].numpy()[:, :n]])
        np.testing.assert_allclose(got, np.broadcast_to(want, got.shape), rtol=1e-5, atol=1e-6)
        assert fed.mesh_confirm() is False
    finally:
        Federation.reset()
