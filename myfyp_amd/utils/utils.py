"""Test/experiment helpers (parity: ``p2pfl/utils/utils.py:39-145``)."""

from __future__ import annotations

import time
from typing import List, Optional, Sequence, Union

import numpy as np

from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings


def set_test_settings() -> None:
    """Fast timers for tests (reference ``set_test_settings``), event-driven gossip."""
    Settings.GRPC_TIMEOUT = 2
    Settings.HEARTBEAT_PERIOD = 0.5
    Settings.HEARTBEAT_TIMEOUT = 2
    Settings.GOSSIP_PERIOD = 0
    Settings.TTL = 10
    Settings.GOSSIP_MESSAGES_PER_PERIOD = 100
    Settings.AMOUNT_LAST_MESSAGES_SAVED = 100
    Settings.GOSSIP_MODELS_PERIOD = 1
    Settings.GOSSIP_MODELS_PER_ROUND = 4
    Settings.GOSSIP_EXIT_ON_X_EQUAL_ROUNDS = 4
    Settings.TRAIN_SET_SIZE = 4
    Settings.VOTE_TIMEOUT = 60
    Settings.AGGREGATION_TIMEOUT = 60
    Settings.WAIT_HEARTBEATS_CONVERGENCE = 0.2 * Settings.HEARTBEAT_TIMEOUT
    Settings.LOG_LEVEL = "INFO"
    logger.set_level(Settings.LOG_LEVEL)


def set_standalone_settings() -> None:
    """Long-running experiment preset (reference ``examples/mnist.py:43-70``)."""
    Settings.GRPC_TIMEOUT = 0.5
    Settings.HEARTBEAT_PERIOD = 5
    Settings.HEARTBEAT_TIMEOUT = 40
    Settings.GOSSIP_PERIOD = 1
    Settings.TTL = 40
    Settings.GOSSIP_MESSAGES_PER_PERIOD = 9999999999
    Settings.AMOUNT_LAST_MESSAGES_SAVED = 10000
    Settings.GOSSIP_MODELS_PERIOD = 1
    Settings.GOSSIP_MODELS_PER_ROUND = 4
    Settings.GOSSIP_EXIT_ON_X_EQUAL_ROUNDS = 10
    Settings.TRAIN_SET_SIZE = 4
    Settings.VOTE_TIMEOUT = 60
    Settings.AGGREGATION_TIMEOUT = 60
    Settings.WAIT_HEARTBEATS_CONVERGENCE = 0.2 * Settings.HEARTBEAT_TIMEOUT
    Settings.LOG_LEVEL = "INFO"
    logger.set_level(Settings.LOG_LEVEL)


def wait_convergence(nodes: Sequence, n_neis: int, wait: Union[int, float] = 5, only_direct: bool = False) -> None:
    """Wait until every node sees ``n_neis`` neighbours (AssertionError on timeout)."""
    deadline = time.time() + wait
    while True:
        if all(len(n.get_neighbors(only_direct=only_direct)) == n_neis for n in nodes):
            return
        if time.time() > deadline:
            raise AssertionError(f"Convergence timeout: {[len(n.get_neighbors(only_direct=only_direct)) for n in nodes]} != {n_neis}")
        time.sleep(0.05)


def full_connection(node, nodes: Sequence) -> None:
    for n in nodes:
        node.connect(n.addr)


def wait_to_finish(nodes: Sequence, timeout: float = 60) -> None:
    """Wait until every node's workflow finished (TimeoutError otherwise)."""
    start = time.time()
    while True:
        if all(n.learning_workflow.finished for n in nodes):
            return
        time.sleep(0.02)
        if time.time() - start > timeout:
            raise TimeoutError("Timeout waiting for nodes to finish")


def check_equal_models(nodes: Sequence, atol: float = 1e-1) -> None:
    """All nodes hold (approximately) the same parameters."""
    ref: Optional[List[np.ndarray]] = None
    for node in nodes:
        params = node.learner.get_model().get_parameters()
        if ref is None:
            ref = params
            continue
        for a, b in zip(ref, params):
            assert np.allclose(a, b, atol=atol)
