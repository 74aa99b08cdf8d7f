"""Per-node mutable learning state (parity: ``p2pfl/node_state.py:26-136``).

Differences from the reference, on purpose:

* ``experiment name`` is configurable (reference hard-codes ``"experiment"``,
  ``start_learning_stage.py:59``) — default unchanged.
* ``votes_event`` wakes the vote aggregator the instant a vote arrives (the reference polls with a
  2 s lock timeout, ``vote_train_set_stage.py:171``). ``wait_votes_ready_lock`` is kept for parity.
"""

from __future__ import annotations

import threading
from typing import Dict, List, Optional

from myfyp_amd.experiment import Experiment
from myfyp_amd.utils.lockcheck import make_lock


class NodeState:
    """Status, experiment, votes, train set and the synchronisation primitives of one node."""

    def __init__(self, addr: str, simulation: bool = False) -> None:
        self.addr = addr
        self.status = "Idle"
        self.simulation = simulation
        self.experiment_config = None
        self.fused_round = False  # collective workflow: this round runs as one fused gang op
        self.models_aggregated: Dict[str, List[str]] = {}
        self.nei_status: Dict[str, int] = {}
        self.train_set: List[str] = []
        self.train_set_votes: Dict[str, Dict[str, int]] = {}
        # votes keyed by the round they were cast for: a fast peer's vote for round r+1 must not be
        # consumed by round r's tally (reference keys by source only and then stalls VOTE_TIMEOUT)
        self.round_votes: Dict[int, Dict[str, Dict[str, int]]] = {}
        self.experiment: Optional[Experiment] = None

        self.train_set_votes_lock = make_lock("NodeState.train_set_votes")
        self.start_thread_lock = make_lock("NodeState.start_thread")
        self.wait_votes_ready_lock = threading.Lock()
        self.votes_event = threading.Event()
        self.model_initialized_lock = threading.Lock()
        self.model_initialized_lock.acquire()
        self.aggregated_model_event = threading.Event()
        self.aggregated_model_event.set()
        # wakes gossip loops whenever a peer's status changes (nei_status / models_aggregated)
        self.status_changed = threading.Condition()

    @property
    def round(self) -> Optional[int]:
        return self.experiment.round if self.experiment is not None else None

    @property
    def total_rounds(self) -> Optional[int]:
        return self.experiment.total_rounds if self.experiment is not None else None

    @property
    def exp_name(self) -> Optional[str]:
        return self.experiment.exp_name if self.experiment is not None else None

    def set_experiment(self, exp_name: str, total_rounds: int, start_round: int = 0) -> None:
        from myfyp_amd.utils import gc_tuning

        self.status = "Learning"
        self.experiment = Experiment(exp_name, total_rounds)
        self.experiment.round = start_round  # > 0 when resuming from a checkpoint
        gc_tuning.experiment_started(self.addr)  # long-lived objects out of the collector's way

    def increase_round(self) -> None:
        if self.experiment is None:
            raise ValueError("Experiment not initialized")
        self.experiment.increase_round()
        self.models_aggregated = {}

    def notify_status(self) -> None:
        """Wake any loop waiting on peer status changes."""
        with self.status_changed:
            self.status_changed.notify_all()

    def wait_status(self, timeout: float) -> None:
        """Block until a peer status change or ``timeout`` seconds."""
        with self.status_changed:
            self.status_changed.wait(timeout)

    def clear(self) -> None:
        """Reset the state (keeps the address, like the reference ``clear``)."""
        from myfyp_amd.utils import gc_tuning

        gc_tuning.experiment_finished(self.addr)
        # wake anybody blocked on the old primitives before replacing them
        self.votes_event.set()
        self.aggregated_model_event.set()
        self.notify_status()
        init_lock = self.model_initialized_lock
        type(self).__init__(self, self.addr, self.simulation)
        # a StartLearningStage still waiting for the initial model holds on to the OLD lock: release
        # it so that stage wakes, sees the cleared round and ends the workflow (a stop that arrived
        # before the initial model otherwise left it blocked for good)
        if init_lock.locked():
            try:
                init_lock.release()
            except RuntimeError:
                pass

    def __str__(self) -> str:
        return (
            f"NodeState(addr={self.addr}, status={self.status}, exp_name={self.exp_name}, "
            f"round={self.round}, total_rounds={self.total_rounds}, simulation={self.simulation}, "
            f"models_aggregated={self.models_aggregated}, nei_status={self.nei_status}, "
            f"train_set={self.train_set}, train_set_votes={self.train_set_votes})"
        )
