"""BASELINE config 5 in small: non-IID Dirichlet(0.5) partitions, ResNet-18, FedProx, on the fused
HIP CNN engine (bf16 operands) against the torch autograd fp32 learner on the SAME partitions.

Round 3 logged config 5 at chance for its 3 timed rounds; the round-4 bisect
(``profiles/r4a_config5_bisect``) showed that the torch fp32 learner on identical partitions stays
at chance for the same ~5 rounds before it climbs, and so does FedAvg on the same split without
dropout: a slow start of this non-IID problem, not an engine defect. This test pins that the engine
trains the same problem as torch: per-round mean training loss within the spread of two torch runs
that differ only in their batch shuffle (the engine shuffles differently again), plus a margin for
bf16. Reference semantics: the Dirichlet partitioner (/root/reference/p2pfl/learning/dataset/
partition_strategies.py:161-430), FedAvg-style aggregation of what arrived (aggregator.py:191-208).
"""

import sys
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(fused: bool, seed: int, rounds: int = 3, peers: int = 3):
    from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
    from myfyp_amd.learning.aggregators import FedProx
    from myfyp_amd.learning.dataset.partition_strategies import DirichletPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.management.logger import logger
    from myfyp_amd.models import ResNet18
    from myfyp_amd.node import Node
    from myfyp_amd.parallel.cnn_engine import CNNGroup
    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.seed import set_seed
    from myfyp_amd.utils.utils import wait_to_finish

    saved = (Settings.USE_FUSED_KERNELS, Settings.BATCH_SIZE, Settings.TRAIN_SET_SIZE, Settings.GANG_WINDOW)
    Settings.USE_FUSED_KERNELS = fused
    Settings.BATCH_SIZE = 64
    Settings.TRAIN_SET_SIZE = peers
    Settings.GANG_WINDOW = 30.0
    set_seed(seed)
    CNNGroup.reset_all()
    Federation.reset()
    fed = Federation.init()
    data = synthetic_cifar10(1024 * peers, 256 * peers, seed=7, similarity=0.85, noise=1.2, modes=4, label_noise=0.1)
    parts = data.generate_partitions(peers, DirichletPartitionStrategy, alpha=0.5)
    exp = f"c5-{int(fused)}-{seed}-{time.time_ns()}"
    nodes = [
        Node(TorchModel(ResNet18(seed=100 + g)), parts[g], address=f"c5-{int(fused)}-{seed}-{g}-{time.time_ns()}", protocol=CollectiveCommunicationProtocol,
             aggregator=FedProx(proximal_mu=0.01), exp_name=exp, learner_kwargs={"batch_size": 64})
        for g in range(peers)
    ]
    try:
        for nd in nodes:
            nd.start()
        assert all((nd.learner._engine is not None) == fused for nd in nodes)
        fed.finalize()
        nodes[0].set_start_learning(rounds=rounds, epochs=1)
        wait_to_finish(nodes, timeout=600)
        local = logger.get_local_logs()[exp]
        loss = []
        for r in range(rounds):
            vals = [local[r][nd.addr]["train_loss"][-1][1] for nd in nodes if nd.addr in local.get(r, {}) and local[r][nd.addr].get("train_loss")]
            loss.append(float(np.mean(vals)))
        logs = logger.get_global_logs()[exp]
        acc = float(np.mean([dict(logs[nd.addr]["test_metric"])[rounds] for nd in nodes]))
        return loss, acc
    finally:
        for nd in nodes:
            nd.stop()
        Federation.reset()
        CNNGroup.reset_all()
        Settings.USE_FUSED_KERNELS, Settings.BATCH_SIZE, Settings.TRAIN_SET_SIZE, Settings.GANG_WINDOW = saved


def test_config5_engine_trains_like_torch_on_dirichlet_fedprox():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    eng, acc_e = _run(True, 1)
    t1, acc_1 = _run(False, 1)
    t2, acc_2 = _run(False, 2)
    print(f"[config5] engine loss {eng} acc {acc_e:.3f} | torch(1) {t1} acc {acc_1:.3f} | torch(2) {t2} acc {acc_2:.3f}", file=sys.stderr)
    for r in range(len(eng)):
        ref = 0.5 * (t1[r] + t2[r])
        spread = abs(t1[r] - t2[r])
        assert np.isfinite(eng[r]), eng
        # shuffle spread of torch itself, plus 15 % of the loss for bf16 operands and the engine's
        # own batch order
        assert abs(eng[r] - ref) <= 2 * spread + 0.15 * ref, (r, eng, t1, t2)
    assert eng[-1] < eng[0], eng  # the local objective goes down over the rounds
