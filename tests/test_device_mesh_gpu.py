"""Device mesh on the GPU: the C++ RCCL wrapper (``csrc/runtime/rccl_mesh.hip``) and the mesh
workflow on the fused MLP engine.

The box has one MI355X, so the RCCL mesh runs at G = 1 (``ncclCommInitAll`` over one device: the
whole wrapper path — init-all, grouped collectives, the fused FedAvg call, async-error polling,
abort and re-init — with RCCL's single-rank copy in place of the xGMI transfer). The N-device logic
(placement, one engine group per device, per-device launches) runs as a *virtual* mesh: G members
on cuda:0 with host-side collectives.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
from myfyp_amd.learning.aggregators import FedAvg
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.management.logger import logger
from myfyp_amd.models import MLP
from myfyp_amd.node import Node
from myfyp_amd.ops import _native
from myfyp_amd.parallel.device_mesh import MeshError, RcclMesh
from myfyp_amd.parallel.federation import Federation
from myfyp_amd.parallel.mlp_engine import MLPGroup
from myfyp_amd.settings import Settings
from myfyp_amd.utils.utils import check_equal_models, wait_to_finish

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = torch.device("cuda", 0)


def _mesh() -> RcclMesh:
    return RcclMesh([DEV])


def test_rccl_mesh_g1_collectives_abort_reinit():
    m = _mesh()
    try:
        assert m.kind == "rccl" and m.size == 1
        t = torch.arange(1000, dtype=torch.float32, device=DEV)
        m.all_reduce_([t])
        m.broadcast_([t], root=0)
        out = torch.empty(1000, dtype=torch.float32, device=DEV)
        m.all_gather_([out], [t])
        torch.cuda.synchronize()
        assert torch.equal(t, torch.arange(1000, dtype=torch.float32, device=DEV))
        assert torch.equal(out, t)
        m.check()
        m.abort()
        with pytest.raises(MeshError):
            m.all_reduce_([t])
        m.shrink([0])  # fresh ncclCommInitAll over the survivor
        t2 = torch.ones(64, dtype=torch.bfloat16, device=DEV)
        m.all_reduce_([t2], op="max")
        torch.cuda.synchronize()
        m.check()
        assert torch.equal(t2, torch.ones(64, dtype=torch.bfloat16, device=DEV))
        assert m.shrinks == 1
    finally:
        m.close()


def test_rccl_mesh_refuses_duplicate_devices():
    with pytest.raises(ValueError):
        RcclMesh([DEV, DEV])


@pytest.mark.parametrize("P", [1, 3, 8])
def test_rccl_mesh_fedavg_bit_equal_to_local_kernel(P):
    """``rmesh_fedavg`` (reduce → grouped all-reduce → apply) writes exactly what the single-device
    ``k_fedavg_local`` launch writes, before and after an abort + re-init."""
    lib = _native.load(required=True)
    n = 235146
    S = (n + 63) // 64 * 64
    g = torch.Generator(device="cpu").manual_seed(P)
    base = torch.randn(P, S, generator=g).to(DEV)
    w = np.arange(1, P + 1, dtype=np.float32) * 37.0
    w[0] = 0.0 if P > 1 else w[0]  # a non-trainer row (weight 0) still receives the mean
    mask = np.ones(P, dtype=np.float32)
    if P > 2:
        mask[2] = 0.0  # a row outside the group (stopped peer) is left alone
    ref = base.clone()
    stream = torch.cuda.current_stream(DEV).cuda_stream
    _native.check(lib.myfyp_fedavg_stacked_local(ref.data_ptr(), P, n, S, w.ctypes.data, mask.ctypes.data, stream), "fedavg_local")
    m = _mesh()
    try:
        for attempt in range(2):
            got = base.clone()
            buf = torch.empty(n + 1, dtype=torch.float32, device=DEV)
            m.fedavg_stacked([got], [buf], [P], n, [S], w, mask)
            torch.cuda.synchronize()
            assert torch.equal(got, ref), f"attempt {attempt}: max diff {(got - ref).abs().max().item()}"
            m.check()
            if attempt == 0:
                m.abort()
                m.shrink([0])
    finally:
        m.close()


def _mesh_run(devices, backend, n=4, rounds=3, virtual=False, aggregator=FedAvg):
    from myfyp_amd.utils.seed import set_seed

    Settings.BATCH_SIZE = 64
    Settings.TRAIN_SET_SIZE = n
    Settings.GANG_WINDOW = 5.0
    Settings.MESH_VIRTUAL = virtual
    set_seed(11)
    MLPGroup.reset_all()
    Federation.reset()
    fed = Federation.init(devices=devices, mesh_backend=backend) if devices is not None else Federation.init()
    parts = synthetic_mnist(8000, 800, seed=5).generate_partitions(n, RandomIIDPartitionStrategy)
    exp = f"mg-{backend}-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"mg-{i}-{time.time_ns()}", aggregator=aggregator(), protocol=CollectiveCommunicationProtocol,
                  exp_name=exp) for i in range(n)]
    try:
        for nd in nodes:
            nd.start()
        assert all(nd.learner._engine is not None for nd in nodes)
        fed.finalize()
        nodes[0].set_start_learning(rounds=rounds, epochs=1)
        wait_to_finish(nodes, timeout=120)
        check_equal_models(nodes, atol=1e-5)
        logs = logger.get_global_logs()[exp]
        final = [dict(logs[nd.addr]["test_metric"])[rounds] for nd in nodes]
        groups = {id(nd.learner._engine.group) for nd in nodes}
        params = nodes[0].learner.flat_params().detach().cpu().clone()
        calls = fed.mesh.calls if fed.mesh is not None else 0
        return final, len(groups), params, calls, [nd.learning_workflow.history for nd in nodes]
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()
        MLPGroup.reset_all()
        Settings.MESH_VIRTUAL = False


def test_mesh_workflow_rccl_g1_matches_single_group():
    """4 fused peers on a one-GPU RCCL mesh: the round driver aggregates through ``rmesh_fedavg``
    and ends bit-equal to the same federation without a mesh (``k_fedavg_local``)."""
    final, ngroups, mesh_params, calls, hist = _mesh_run(["cuda:0"], "rccl")
    assert ngroups == 1 and calls >= 3
    assert min(final) > 0.75, final
    _, _, solo_params, _, _ = _mesh_run(None, None)
    assert torch.equal(mesh_params, solo_params), (mesh_params - solo_params).abs().max()


@pytest.mark.parametrize("agg", ["scaffold", "fedmedian", "fedprox"])
def test_mesh_workflow_rccl_g1_aggregators_match_single_group(agg):
    """the mesh variants of SCAFFOLD (``_mesh_scaffold``: packed reduction,
    one RCCL all-reduce, apply), FedMedian (``_mesh_median``: RCCL all-gather + median kernel) and
    FedProx (``rmesh_fedavg`` with the proximal term in the fused step) on the one-GPU RCCL mesh,
    pinned to the same federation without a mesh: 4 fused peers, 3 rounds, the final parameters
    equal to fp32 reduction-order tolerance, and every peer learns."""
    from myfyp_amd.learning.aggregators import FedMedian, FedProx, Scaffold

    make = {"scaffold": lambda: Scaffold(global_lr=1.0), "fedmedian": FedMedian, "fedprox": lambda: FedProx(proximal_mu=0.01)}[agg]
    final, ngroups, mesh_params, calls, _ = _mesh_run(["cuda:0"], "rccl", aggregator=make)
    assert ngroups == 1 and calls >= 3, calls
    assert min(final) > 0.75, final
    _, _, solo_params, _, _ = _mesh_run(None, None, aggregator=make)
    d = (mesh_params - solo_params).abs()
    scale = solo_params.abs().mean()
    # the mesh and the single-group path reduce in different orders: fp32 ulps, amplified by Adam's
    # sign-sensitivity on near-zero gradients over 3 local epochs (cf. test_device_mesh.py)
    assert d.mean() < 1e-4 * max(1.0, float(scale)) and d.max() < 0.05, (float(d.mean()), float(d.max()))


@pytest.mark.parametrize("g", [2, 4])
def test_mesh_workflow_virtual_devices(g):
    """G virtual mesh ranks on cuda:0: one engine group per rank (the N-GPU layout), host
    collectives; models agree and learn."""
    final, ngroups, _, calls, hist = _mesh_run(g, "host", n=4, virtual=True)
    assert ngroups == g and calls >= 3
    assert min(final) > 0.75, final
    assert all(h.count("RoundFinishedStage") == 3 for h in hist)


def test_bench_virtual_mesh_gpu():
    """``bench.py --gpus 2 --mesh-virtual`` on one GPU: the mesh path of the headline, fused engine,
    reports the one physical GPU it used."""
    env = dict(os.environ)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mesh-virtual", "--steps", "10", "--warmup", "3"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and out["config"]["peers_per_gpu"] == 4
    assert out["config"]["engine"].startswith("fused-hip")
    assert out["value"] > 50, out


def test_bench_torchrun_mesh_virtual_gpu():
    """The driver's multi-GPU launch shape on one GPU with the mesh asked for explicitly (torchrun's
    default is one process per GPU): ``torch.distributed.run --nproc-per-node 2 bench.py --gpus 2
    --launch mesh --mesh-virtual``. Rank 0 drives the two-member mesh; rank 1 parks on the gloo
    barrier and exits cleanly; exactly one JSON line comes out."""
    from _ports import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch", "mesh", "--mesh-virtual", "--steps", "10", "--warmup",
           "3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=dict(os.environ))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["peers_per_gpu"] == 4 and out["value"] > 50, out


def _stacked_case(P: int, seed: int):
    n = 235146
    S = (n + 63) // 64 * 64
    g = torch.Generator(device="cpu").manual_seed(seed)
    base = torch.randn(P, S, generator=g).to(DEV)
    w = np.arange(1, P + 1, dtype=np.float32) * 11.0
    mask = np.ones(P, dtype=np.float32)
    ref = base.clone()
    lib = _native.load(required=True)
    _native.check(lib.myfyp_fedavg_stacked_local(ref.data_ptr(), P, n, S, w.ctypes.data, mask.ctypes.data, torch.cuda.current_stream(DEV).cuda_stream),
                  "fedavg_local")
    return n, S, base, w, mask, ref


def _guarded_fedavg(fed, rows, P, n, S, w, mask):
    buf = torch.empty(n + 1, dtype=torch.float32, device=DEV)
    out = torch.empty(n + 1, dtype=torch.float32, device=DEV)
    fed.mesh.fedavg_stacked([rows], [buf], [P], n, [S], w, mask, outs=[out])

    def retry():
        fed.mesh.fedavg_retry([rows], [buf], [out], [P], n, [S], mask)

    fed.mesh_track("fedavg", retry)
    return buf, out


def test_rccl_mesh_async_error_recovers_bit_equal():
    """An asynchronous RCCL error (fault hook: ``rmesh_check`` reports one) after a grouped FedAvg:
    the round driver's confirmation aborts the mesh, probes the device, re-initialises RCCL and
    re-runs the all-reduce from the retained partial sums; the rows end bit-equal to
    ``k_fedavg_local`` over the same rows."""
    saved = (Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT)
    Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT = 30.0, 10.0
    Federation.reset()
    try:
        fed = Federation.init(devices=["cuda:0"], mesh_backend="rccl")
        assert fed.mesh.kind == "rccl"
        P = 8
        n, S, base, w, mask, ref = _stacked_case(P, 5)
        rows = base.clone()
        _guarded_fedavg(fed, rows, P, n, S, w, mask)
        fed.mesh.inject_error(0)
        assert fed.mesh_confirm() is True
        torch.cuda.synchronize()
        assert fed.mesh_guard.recoveries == 1 and fed.mesh_members == [0] and fed.mesh.shrinks == 1
        assert torch.equal(rows, ref), (rows - ref).abs().max()
        fed.mesh.check()
        # the rebuilt mesh keeps working, and a clean round confirms without a recovery
        rows2 = base.clone()
        _guarded_fedavg(fed, rows2, P, n, S, w, mask)
        assert fed.mesh_confirm() is False
        torch.cuda.synchronize()
        assert torch.equal(rows2, ref)
    finally:
        Federation.reset()
        Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT = saved


def test_rccl_mesh_rebuild_right_after_enqueued_fedavg():
    """a healthy-mesh rebuild (a device's last peer left) issued right after a grouped
    FedAvg was enqueued drains the devices first and destroys (not aborts) the communicators, so
    the queued all-reduce and apply complete: the rows are exactly ``k_fedavg_local``'s."""
    Federation.reset()
    try:
        fed = Federation.init(devices=["cuda:0"], mesh_backend="rccl")
        P = 3
        n, S, base, w, mask, ref = _stacked_case(P, 9)
        rows = base.clone()
        torch.cuda._sleep(50_000_000)  # keep the device busy so the FedAvg is still queued
        _guarded_fedavg(fed, rows, P, n, S, w, mask)
        fed._mesh_rebuild([0])
        assert fed.mesh.shrinks == 1
        torch.cuda.synchronize()
        assert torch.equal(rows, ref), (rows - ref).abs().max()
        fed.mesh.check()
    finally:
        Federation.reset()


def test_mesh_workflow_rccl_g1_async_error_mid_experiment():
    """4 fused peers on the one-GPU RCCL mesh; an asynchronous RCCL error is injected in round 1.
    The next weights section recovers (abort, re-init, retained-partial re-run), every peer
    finishes every round, and the models agree and learn."""
    saved = (Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT)
    Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT = 30.0, 10.0
    Settings.BATCH_SIZE = 64
    Settings.TRAIN_SET_SIZE = 4
    Settings.GANG_WINDOW = 5.0
    MLPGroup.reset_all()
    Federation.reset()
    fed = Federation.init(devices=["cuda:0"], mesh_backend="rccl")
    parts = synthetic_mnist(8000, 800, seed=5).generate_partitions(4, RandomIIDPartitionStrategy)
    exp = f"mgerr-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"mge-{i}-{time.time_ns()}", aggregator=FedAvg(), protocol=CollectiveCommunicationProtocol,
                  exp_name=exp) for i in range(4)]
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        # a round hook (the lock-step round driver stays in use): after round 1's FedAvg
        fed.round_hooks.append(lambda r, f: f.mesh.inject_error(0) if r == 1 else None)
        nodes[0].set_start_learning(rounds=4, epochs=1)
        wait_to_finish(nodes, timeout=120)
        assert fed.mesh_guard.recoveries == 1, fed.mesh_guard.recoveries
        assert all(nd.learning_workflow.history.count("RoundFinishedStage") == 4 for nd in nodes)
        check_equal_models(nodes, atol=1e-5)
        logs = logger.get_global_logs()[exp]
        assert min(dict(logs[nd.addr]["test_metric"])[4] for nd in nodes) > 0.75
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()
        MLPGroup.reset_all()
        Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT = saved


# ---------------------------------------------------------------------------------------------
# bucketed, overlapped mesh FedAvg (rmesh_fedavg_bucketed / rmesh_delayed_land)
# ---------------------------------------------------------------------------------------------
BUCKET = 60000  # floats: 4 buckets over the MLP's 235146 parameters


@pytest.mark.parametrize("P", [1, 3, 8])
def test_rccl_mesh_bucketed_fedavg_bit_equal_to_local_kernel(P):
    """Reduce on the comm stream, per-bucket grouped all-reduce, per-bucket apply on the compute
    stream behind a bucket event: the rows end exactly as ``k_fedavg_local`` writes them, with the
    compute stream still busy when the call is enqueued (the comm stream must wait for it), and
    again after an abort + re-init."""
    from myfyp_amd.parallel.weights_plane import comm_stream

    n, S, base, w, mask, ref = _stacked_case(P, 20 + P)
    m = _mesh()
    try:
        for attempt in range(2):
            got = base.clone()
            keep = torch.zeros(n + 4, dtype=torch.float32, device=DEV)
            out = torch.zeros(n + 4, dtype=torch.float32, device=DEV)
            torch.cuda._sleep(20_000_000)  # the compute stream is busy: the reduce must wait for it
            got.mul_(1.0)
            m.fedavg_bucketed([got], [keep], [out], [P], n, [S], w, mask, [comm_stream(DEV)], BUCKET, apply=True)
            torch.cuda.synchronize()
            assert torch.equal(got, ref), f"attempt {attempt}: max diff {(got - ref).abs().max().item()}"
            assert float(keep[0]) == float(np.sum(w, dtype=np.float64))
            m.check()
            if attempt == 0:
                m.abort()
                m.shrink([0])
    finally:
        m.close()


def test_rccl_mesh_bucketed_async_error_recovers_bit_equal():
    """The guard's recovery on the bucketed exchange: async error → abort → re-init → all-reduce of
    the retained [Σw | Σ w x] → apply; the rows end exactly as ``k_fedavg_local`` writes them."""
    from myfyp_amd.parallel.weights_plane import comm_stream

    saved = (Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT)
    Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT = 30.0, 10.0
    Federation.reset()
    try:
        fed = Federation.init(devices=["cuda:0"], mesh_backend="rccl")
        P = 8
        n, S, base, w, mask, ref = _stacked_case(P, 31)
        rows = base.clone()
        keep = torch.zeros(n + 4, dtype=torch.float32, device=DEV)
        out = torch.zeros(n + 4, dtype=torch.float32, device=DEV)
        fed.mesh.fedavg_bucketed([rows], [keep], [out], [P], n, [S], w, mask, [comm_stream(DEV)], BUCKET)
        fed.mesh_track("fedavg", lambda: fed.mesh.fedavg_bucketed_retry([rows], [keep], [out], [P], n, [S], mask))
        fed.mesh.inject_error(0)
        assert fed.mesh_confirm() is True
        torch.cuda.synchronize()
        assert fed.mesh_guard.recoveries == 1 and fed.mesh_members == [0]
        assert torch.equal(rows, ref), (rows - ref).abs().max()
    finally:
        Federation.reset()
        Settings.COLLECTIVE_TIMEOUT, Settings.FAILURE_TIMEOUT = saved


def test_rccl_mesh_delayed_averaging_lands_next_round():
    """Delayed averaging on the RCCL mesh: snapshot, exchange on the comm stream with no apply
    (the compute stream keeps training: a local step is added meanwhile), then the land launch
    waits on the exchange and writes x + avg - snap, the snapshot following."""
    from myfyp_amd.parallel.weights_plane import comm_stream

    P = 4
    n, S, base, w, mask, ref = _stacked_case(P, 41)  # ref: the weighted mean in every row
    m = _mesh()
    try:
        rows = base.clone()
        snap = torch.zeros(P * n, dtype=torch.float32, device=DEV)
        keep = torch.zeros(n + 4, dtype=torch.float32, device=DEV)
        out = torch.zeros(n + 4, dtype=torch.float32, device=DEV)
        m.delayed_land([rows], [snap], [out], [P], n, [S], n, mask, False)
        m.fedavg_bucketed([snap], [keep], [out], [P], n, [n], w, mask, [comm_stream(DEV)], BUCKET, apply=False)
        rows[:, :n].add_(0.125)  # the next local epoch, beside the exchange
        m.delayed_land([rows], [snap], [out], [P], n, [S], n, mask, True)
        torch.cuda.synchronize()
        want = ref[:, :n] + 0.125
        assert torch.allclose(rows[:, :n], want, rtol=1e-5, atol=1e-5), (rows[:, :n] - want).abs().max()
        assert torch.equal(snap.view(P, n), rows[:, :n])
        assert torch.equal(rows[:, n:], base[:, n:])
        m.check()
    finally:
        m.close()


def test_virtual_mesh_bucketed_fedavg_matches_float64():
    """Two virtual members on cuda:0 (HostMesh, GPU members): the bucketed exchange's launches with
    a stream-ordered sum in place of RCCL give the float64 weighted mean of both members' rows."""
    from myfyp_amd.parallel.device_mesh import HostMesh
    from myfyp_amd.parallel.weights_plane import comm_stream

    m = HostMesh([DEV, DEV])
    n, S, b0, w0, mask0, _ = _stacked_case(3, 51)
    _, _, b1, _, _, _ = _stacked_case(2, 52)
    w = np.array([1.0, 2.0, 0.0, 4.0, 5.0], dtype=np.float32)
    mask = np.ones(5, dtype=np.float32)
    keeps = [torch.zeros(n + 4, device=DEV) for _ in range(2)]
    outs = [torch.zeros(n + 4, device=DEV) for _ in range(2)]
    r0, r1 = b0.clone(), b1.clone()
    m.fedavg_bucketed([r0, r1], keeps, outs, [3, 2], n, [S, S], w, mask, [comm_stream(DEV)] * 2, BUCKET)
    torch.cuda.synchronize()
    allr = torch.cat([b0[:, :n], b1[:, :n]]).double()
    want = (torch.from_numpy(w).double().to(DEV)[:, None] * allr).sum(0) / float(w.sum())
    for r in (r0, r1):
        assert torch.allclose(r[:, :n].double(), want.expand(r.shape[0], n), rtol=1e-5, atol=1e-5)


def test_mesh_workflow_rccl_g1_delayed_averaging_learns():
    """4 fused peers on the one-GPU RCCL mesh with DELAYED_AVERAGING: every round's exchange runs on
    the comm stream beside the next local epoch and lands a round later (the last round aggregates
    exactly); the models agree at the end and learn."""
    saved = Settings.DELAYED_AVERAGING
    Settings.DELAYED_AVERAGING = True
    try:
        final, ngroups, _, calls, hist = _mesh_run(["cuda:0"], "rccl", rounds=4)
    finally:
        Settings.DELAYED_AVERAGING = saved
    assert ngroups == 1 and calls >= 4
    assert min(final) > 0.75, final
    assert all(h.count("RoundFinishedStage") == 4 for h in hist)
