"""Decentralised neighbour averaging (BASELINE config 3): mixing matrix, in-process and 2-rank P2P."""

import os
import subprocess
import sys
import time

import numpy as np
import pytest

from _ports import free_port
import torch

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
from myfyp_amd.learning.aggregators.neighbor_avg import NeighborAvg
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.management.logger import logger
from myfyp_amd.models import MLP
from myfyp_amd.node import Node
from myfyp_amd.parallel import weights_plane
from myfyp_amd.parallel.federation import Federation
from myfyp_amd.utils.utils import wait_to_finish

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("topology", ["ring", "line", "star", "full"])
def test_mixing_matrix_doubly_stochastic(topology):
    w = NeighborAvg(topology=topology).mixing_matrix(6)
    np.testing.assert_allclose(w.sum(0), 1.0)
    np.testing.assert_allclose(w.sum(1), 1.0)
    np.testing.assert_allclose(w, w.T)
    assert (w >= 0).all()


def test_ring_mixing_in_process():
    Federation.reset()
    fed = Federation.init()
    agg = NeighborAvg(topology="ring")
    data = synthetic_mnist(200, 50)
    tag = time.time_ns()
    nodes = [Node(TorchModel(MLP(hidden_sizes=[8, 8])), data, address=f"nb{tag}-{i}", aggregator=agg, protocol=CollectiveCommunicationProtocol) for i in range(5)]
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        peers = fed.all_peers()
        for nd in nodes:
            with torch.no_grad():
                nd.learner.flat_params().fill_(float(peers.index(nd.addr)))
        weights_plane.aggregate_neighbors(fed, {nd.addr: None for nd in nodes}, agg)
        w = agg.mixing_matrix(5)
        for nd in nodes:
            i = peers.index(nd.addr)
            expect = float(w[i] @ np.arange(5, dtype=np.float64))
            torch.testing.assert_close(nd.learner.flat_params(), torch.full_like(nd.learner.flat_params(), expect))
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()


def test_neighbor_avg_workflow_learns():
    from myfyp_amd.settings import Settings

    Settings.BATCH_SIZE = 32
    Federation.reset()
    fed = Federation.init()
    data = synthetic_mnist(4000, 800, seed=5, similarity=0.3)
    parts = data.generate_partitions(4, RandomIIDPartitionStrategy)
    exp = f"nbavg-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"{exp}-{i}", aggregator=NeighborAvg("ring"), protocol=CollectiveCommunicationProtocol, exp_name=exp) for i in range(4)]
    try:
        for nd in nodes:
            nd.start()
        fed.finalize()
        nodes[0].set_start_learning(rounds=3, epochs=1)
        wait_to_finish(nodes, timeout=120)
        for nd in nodes:
            assert nd.learning_workflow.history.count("TrainStage") == 3  # everyone trains every round
        logs = logger.get_global_logs()[exp]
        assert min(logs[nd.addr]["test_metric"][-1][1] for nd in nodes) > 0.5
        # consensus is approached: peers are closer to each other than at the start
        p = [np.concatenate([a.ravel() for a in nd.learner.get_model().get_parameters()]) for nd in nodes]
        spread = max(np.abs(p[i] - p[0]).max() for i in range(1, 4))
        assert spread < 1.0
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()


@pytest.mark.slow
def test_ring_p2p_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "tests", "workers", "neighbor_avg_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    assert res.stdout.count("OK") == 2
