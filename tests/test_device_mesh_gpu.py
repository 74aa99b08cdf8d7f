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


def _mesh_run(devices, backend, n=4, rounds=3, virtual=False):
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
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"mg-{i}-{time.time_ns()}", aggregator=FedAvg(), protocol=CollectiveCommunicationProtocol,
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
    """The driver's multi-GPU launch shape on one GPU: ``torch.distributed.run --nproc-per-node 2
    bench.py --gpus 2 --mesh-virtual``. Rank 0 drives the two-member mesh; rank 1 parks on the gloo
    barrier and exits cleanly; exactly one JSON line comes out."""
    from _ports import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mesh-virtual", "--steps", "10", "--warmup", "3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=dict(os.environ))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["peers_per_gpu"] == 4 and out["value"] > 50, out
