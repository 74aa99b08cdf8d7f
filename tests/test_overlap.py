"""Side-stream bucketed FedAvg and opt-in delayed averaging (SURVEY §7.4 hard part 4; VERDICT r1
item 3): bucket layout, closed-form numerics in-process (CPU), 2-rank gloo on CPU, and the same on
the fused engine's stacked rows on one MI355X (gpu marker)."""

import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from _ports import free_port
from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.management.logger import logger
from myfyp_amd.models import MLP
from myfyp_amd.node import Node
from myfyp_amd.parallel import weights_plane
from myfyp_amd.parallel.federation import Federation
from myfyp_amd.settings import Settings
from myfyp_amd.utils.utils import check_equal_models, wait_to_finish

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bucket_ranges_cover_and_align():
    for n in (1, 3, 4, 17, 4096, 100003):
        for bb in (16, 64, 1000, 1 << 20):
            r = weights_plane.bucket_ranges(n, bb)
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert all(b0 % 4 == 0 for b0, _ in r)


def _delayed_in_process(device, hidden):
    Settings.DEVICE = device
    Federation.reset()
    fed = Federation.init()
    nodes = [Node(TorchModel(MLP(hidden_sizes=hidden)), synthetic_mnist(200, 50), address=f"dl{time.time_ns()}-{i}", protocol=CollectiveCommunicationProtocol) for i in range(3)]
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        Settings.DELAYED_AVERAGING = True
        fl = [nd.learner.flat_params() for nd in nodes]
        n = fl[0].numel()
        g = torch.Generator().manual_seed(1)
        x0 = [torch.randn(n, generator=g) for _ in fl]
        w = [2.0, 0.0, 6.0]
        arrived = {nd.addr: (wt, None) for nd, wt in zip(nodes, w)}
        with torch.no_grad():
            for f, x in zip(fl, x0):
                f.copy_(x.to(f.device))
        weights_plane.aggregate_mean(fed, arrived, final=False)
        for f, x in zip(fl, x0):
            assert torch.equal(f.detach().cpu(), x)  # local weights kept
        d = [torch.randn(n, generator=g) * 0.01 for _ in fl]
        with torch.no_grad():
            for f, dd in zip(fl, d):
                f.add_(dd.to(f.device))
        avg0 = sum(wt * x.double() for wt, x in zip(w, x0)) / sum(w)
        weights_plane.aggregate_mean(fed, arrived, final=False)
        y = [x.double() + dd.double() + avg0 - x.double() for x, dd in zip(x0, d)]
        for f, yy in zip(fl, y):
            np.testing.assert_allclose(f.detach().cpu().double().numpy(), yy.numpy(), atol=1e-5)
        weights_plane.aggregate_mean(fed, arrived, final=True)
        avg1 = sum(wt * yy for wt, yy in zip(w, y)) / sum(w)
        for f in fl:
            np.testing.assert_allclose(f.detach().cpu().double().numpy(), avg1.numpy(), atol=1e-5)
    finally:
        Settings.DELAYED_AVERAGING = False
        Settings.DEVICE = "auto"
        for nd in nodes:
            nd.stop()
        Federation.reset()


def test_delayed_averaging_closed_form_cpu():
    _delayed_in_process("cpu", [8, 8])


@pytest.mark.gpu
def test_delayed_averaging_closed_form_stacked_gpu():
    _delayed_in_process("cuda", [256, 128])  # fused engine rows: k_fedavg_delayed_land + side-stream reduce


def test_delayed_averaging_workflow_converges_equal():
    Settings.BATCH_SIZE = 16
    Settings.TRAIN_SET_SIZE = 4
    Settings.DELAYED_AVERAGING = True
    Federation.reset()
    fed = Federation.init()
    data = synthetic_mnist(4000, 400, seed=3, similarity=0.3)
    parts = data.generate_partitions(4, RandomIIDPartitionStrategy)
    exp = f"delayed-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"{exp}-{i}", protocol=CollectiveCommunicationProtocol, exp_name=exp) for i in range(4)]
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        nodes[0].set_start_learning(rounds=3, epochs=1)
        wait_to_finish(nodes, timeout=120)
        check_equal_models(nodes, atol=1e-5)  # the last round aggregates exactly
        logs = logger.get_global_logs()[exp]
        assert max(logs[nd.addr]["test_metric"][-1][1] for nd in nodes) > 0.5
    finally:
        Settings.DELAYED_AVERAGING = False
        for nd in nodes:
            nd.stop()
        Federation.reset()


def _two_ranks(device):
    env = dict(os.environ, AGG_DEVICE=device, HSA_ENABLE_IPC_MODE_LEGACY="0")
    if device == "cuda":
        env["MYFYP_DIST_BACKEND"] = "gloo"  # RCCL refuses two ranks on one device
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "tests", "workers", "overlap_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    assert res.stdout.count("OK") == 2


@pytest.mark.slow
def test_overlap_and_delayed_two_ranks_gloo():
    _two_ranks("cpu")


@pytest.mark.gpu
def test_overlap_and_delayed_two_ranks_gpu():
    _two_ranks("cuda")
