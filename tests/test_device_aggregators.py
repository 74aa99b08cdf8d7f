"""SCAFFOLD and FedMedian on the collective plane (``weights_plane.aggregate_scaffold`` /
``aggregate_median``) against the host aggregators (reference math:
``p2pfl/learning/aggregators/scaffold.py:76-111``, ``fedmedian.py:56-62``) in float64 numpy.

The device path never builds wire models: Δy/Δc stay device flats in the SCAFFOLD callback and are
reduced with one all-reduce; FedMedian packs the trainers' rows, all-gathers them and runs the
``coordinate_median`` kernel. CPU (gloo / in-process) here, the same checks on ``cuda:0`` under
the gpu marker (fused MLP engine rows), and a 2-rank gloo run through ``tests/workers``.
"""

import os
import subprocess
import sys
import time

import numpy as np
import pytest

from _ports import free_port
import torch

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
from myfyp_amd.learning.aggregators import FedMedian, Scaffold
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.models import MLP
from myfyp_amd.node import Node
from myfyp_amd.parallel import weights_plane
from myfyp_amd.parallel.federation import Federation
from myfyp_amd.settings import Settings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _nodes(make_agg, k, hidden):
    data = synthetic_mnist(200, 50)
    tag = time.time_ns()
    model = (lambda i: MLP(seed=i)) if hidden is None else (lambda i: MLP(hidden_sizes=hidden, seed=i))
    return [Node(TorchModel(model(i)), data, address=f"dev{tag}-{i}", aggregator=make_agg(), protocol=CollectiveCommunicationProtocol) for i in range(k)]


def _flat64(t):
    return t.detach().double().cpu().numpy().ravel()


def _scaffold_case(device, hidden):
    Settings.DEVICE = device
    Federation.reset()
    fed = Federation.init()
    weights = [10.0, 0.0, 30.0, 20.0]
    nodes = _nodes(lambda: Scaffold(global_lr=0.7), len(weights), hidden)
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        g = torch.Generator().manual_seed(5)
        n = nodes[0].learner.flat_params().numel()
        x0 = torch.randn(n, generator=g)
        dys, dcs = [], []
        for nd in nodes:
            lr = nd.learner
            cb = weights_plane._scaffold_cb(lr)
            with torch.no_grad():
                lr.flat_params().copy_(x0)
            dys.append(torch.randn(n, generator=g) * 0.1)
            dcs.append(torch.randn(n, generator=g))
            dev = lr.flat_params().device
            cb.x0 = x0.to(dev)
            cb.delta_y, cb.delta_c = dys[-1].to(dev), dcs[-1].to(dev)
        tr = [i for i, w in enumerate(weights) if w > 0]
        tot = sum(weights[i] for i in tr)
        x_exp = x0.double().numpy() + 0.7 * sum(weights[i] * dys[i].double().numpy() for i in tr) / tot
        c_exp = sum(dcs[i].double().numpy() for i in tr) / len(tr)
        # the host aggregator on the same models (wire path, built before the device step
        # overwrites the live weights) agrees with the closed form
        host = Scaffold(global_lr=0.7)
        wire = []
        for i in tr:
            lr = nodes[i].learner
            m = lr.get_model().build_copy(params=[p.copy() for p in lr.get_model().get_parameters()], num_samples=int(weights[i]), contributors=[nodes[i].addr])
            m.add_info("scaffold", {"delta_y_i": [t.cpu().numpy() for t in lr.split_flat(dys[i].to(lr.flat_params().device))],
                                    "delta_c_i": [t.cpu().numpy() for t in lr.split_flat(dcs[i].to(lr.flat_params().device))]})
            m.set_parameters([a + d for a, d in zip(lr.get_model().get_parameters(), m.get_info("scaffold")["delta_y_i"])])
            wire.append(m)
        out = host.aggregate(wire)
        host_x = np.concatenate([np.asarray(p, dtype=np.float64).ravel() for p in out.get_parameters()])
        host_c = np.concatenate([np.asarray(c, dtype=np.float64).ravel() for c in out.get_info("scaffold")["global_c"]])
        np.testing.assert_allclose(host_x, x_exp, rtol=0, atol=1e-6)
        np.testing.assert_allclose(host_c, c_exp, rtol=0, atol=1e-6)
        agg = nodes[0].aggregator
        weights_plane.aggregate_scaffold(fed, {nd.addr: (w, None) for nd, w in zip(nodes, weights)}, agg)
        for nd in nodes:
            np.testing.assert_allclose(_flat64(nd.learner.flat_params()), x_exp, rtol=0, atol=1e-6)
            gc = nd.learner.get_model().get_info("scaffold")["global_c"]
            np.testing.assert_allclose(np.concatenate([_flat64(t) for t in gc]), c_exp, rtol=0, atol=1e-6)
            assert gc[0].device.type == nd.learner.flat_params().device.type  # stayed on the device
        # second round: the control variate accumulates on the device
        for nd in nodes:
            cb = weights_plane._scaffold_cb(nd.learner)
            cb.x0 = nd.learner.flat_params().detach().clone()
        weights_plane.aggregate_scaffold(fed, {nd.addr: (w, None) for nd, w in zip(nodes, weights)}, agg)
        gc = nodes[2].learner.get_model().get_info("scaffold")["global_c"]
        np.testing.assert_allclose(np.concatenate([_flat64(t) for t in gc]), 2 * c_exp, rtol=0, atol=2e-6)
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()
        Settings.DEVICE = "auto"


def _median_case(device, hidden, k=5):
    Settings.DEVICE = device
    Federation.reset()
    fed = Federation.init()
    weights = [1.0, 0.0, 2.0, 3.0, 4.0][:k]
    nodes = _nodes(FedMedian, len(weights), hidden)
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        g = torch.Generator().manual_seed(9)
        rows = []
        for nd in nodes:
            with torch.no_grad():
                f = nd.learner.flat_params()
                r = torch.randn(f.numel(), generator=g)
                f.copy_(r)
            rows.append(r.double().numpy())
        tr = [i for i, w in enumerate(weights) if w > 0]
        wire = [nodes[i].learner.get_model().build_copy(params=[p.copy() for p in nodes[i].learner.get_model().get_parameters()], num_samples=1, contributors=[nodes[i].addr]) for i in tr]
        host = FedMedian().aggregate(wire)
        host_flat = np.concatenate([np.asarray(p, dtype=np.float64).ravel() for p in host.get_parameters()])
        weights_plane.aggregate_median(fed, {nd.addr: (w, None) for nd, w in zip(nodes, weights)})
        exp = np.median(np.stack([rows[i] for i in tr]), axis=0)
        np.testing.assert_allclose(host_flat[: exp.size], exp, rtol=0, atol=1e-6)
        for nd in nodes:
            np.testing.assert_allclose(_flat64(nd.learner.flat_params()), exp, rtol=0, atol=1e-6)
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()
        Settings.DEVICE = "auto"


def test_scaffold_device_plane_cpu():
    _scaffold_case("cpu", [8, 8])


@pytest.mark.parametrize("k", [4, 5])
def test_median_device_plane_cpu(k):
    _median_case("cpu", [8, 8], k)


@pytest.mark.gpu
def test_scaffold_device_plane_gpu():
    _scaffold_case("cuda", None)  # default MLP: rows of the fused engine's stacked buffer


@pytest.mark.gpu
@pytest.mark.parametrize("k", [4, 5])
def test_median_device_plane_gpu(k):
    _median_case("cuda", None, k)


@pytest.mark.slow
def test_scaffold_median_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "tests", "workers", "device_agg_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    assert res.stdout.count("OK") == 2


@pytest.mark.gpu
def test_scaffold_median_two_ranks_gpu():
    """2 ranks x 2 peers on the fused engine (one MI355X: gloo carries the cross-rank collectives,
    RCCL refuses two ranks per device)."""
    env = dict(os.environ, MYFYP_DIST_BACKEND="gloo", AGG_DEVICE="cuda", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "tests", "workers", "device_agg_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    assert res.stdout.count("OK") == 2
