"""Node facade (parity: ``p2pfl/node.py:89-413``).

Same public API: ``Node(model, data, address, learner, aggregator, protocol, simulation)``,
``start/stop/connect/disconnect/get_neighbors``, ``set_start_learning(rounds, epochs)``,
``set_stop_learning``, ``set_learner/set_model/set_data``, ``get_model/get_data``, ``.state``,
``.learning_workflow``, ``.learner``, ``.aggregator``, ``.addr``.

MI355X additions:

* the protocol decides the workflow flavour: gossip protocols (in-memory, gRPC) run the
  reference stages; ``CollectiveCommunicationProtocol`` runs the same-named collective stages whose
  weights plane is RCCL over xGMI;
* ``learner_kwargs`` (e.g. ``batch_size``) reach the learner; ``exp_name`` names the experiment
  (reference hard-codes ``"experiment"``);
* ``set_start_learning`` returns the experiment name (the FYP scripts expect it,
  ``exp_SAVE3.txt:107``).
"""

from __future__ import annotations

import contextlib
import threading
import traceback
from typing import Any, Dict, Optional, Type

from myfyp_amd.communication.commands.message.metrics_command import MetricsCommand
from myfyp_amd.communication.commands.message.model_initialized_command import ModelInitializedCommand
from myfyp_amd.communication.commands.message.models_agregated_command import ModelsAggregatedCommand
from myfyp_amd.communication.commands.message.models_ready_command import ModelsReadyCommand
from myfyp_amd.communication.commands.message.start_learning_command import StartLearningCommand
from myfyp_amd.communication.commands.message.stop_learning_command import StopLearningCommand
from myfyp_amd.communication.commands.message.vote_train_set_command import VoteTrainSetCommand
from myfyp_amd.communication.commands.weights.full_model_command import FullModelCommand
from myfyp_amd.communication.commands.weights.init_model_command import InitModelCommand
from myfyp_amd.communication.commands.weights.partial_model_command import PartialModelCommand
from myfyp_amd.communication.protocols.communication_protocol import CommunicationProtocol
from myfyp_amd.communication.protocols.memory.memory_communication_protocol import InMemoryCommunicationProtocol
from myfyp_amd.exceptions import LearnerRunningException, NodeRunningException, ZeroRoundsException
from myfyp_amd.learning.aggregators.aggregator import Aggregator
from myfyp_amd.learning.aggregators.fedavg import FedAvg
from myfyp_amd.learning.frameworks.learner import Learner
from myfyp_amd.learning.frameworks.learner_factory import LearnerFactory
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel
from myfyp_amd.learning.frameworks.simulation import try_init_learner_with_ray
from myfyp_amd.management.logger import logger
from myfyp_amd.node_state import NodeState
from myfyp_amd.settings import Settings
from myfyp_amd.stages.workflows import LearningWorkflow


class Node:
    """A federated-learning peer."""

    def __init__(
        self,
        model: P2PFLModel,
        data: Any = None,
        address: str = "",
        learner: Optional[Type[Learner]] = None,
        aggregator: Optional[Aggregator] = None,
        protocol: Type[CommunicationProtocol] = InMemoryCommunicationProtocol,
        simulation: bool = False,
        learner_kwargs: Optional[Dict[str, Any]] = None,
        exp_name: str = "experiment",
        **kwargs: Any,
    ) -> None:
        self._communication_protocol = protocol(address) if isinstance(protocol, type) else protocol
        self.addr = self._communication_protocol.get_address()
        self.aggregator = FedAvg() if aggregator is None else aggregator
        self.aggregator.set_node_name(self.addr)
        if learner is None:
            learner = LearnerFactory.create_learner(model)
        # a process driving a device mesh places its peers round-robin over the devices
        place = getattr(self._communication_protocol, "placement", None)
        if place is not None and "device" not in (learner_kwargs or {}):
            where = place()
            if where is not None:
                import inspect

                params = inspect.signature(learner).parameters
                learner_kwargs = dict(learner_kwargs or {})
                if "device" in params:
                    learner_kwargs["device"] = where[0]
                if "mesh_rank" in params:
                    learner_kwargs["mesh_rank"] = where[1]
        # plain learner, or (Settings.SIMULATION_POOL) one pinned to a device of the simulation pool
        self.learner: Learner = try_init_learner_with_ray(learner, model, data, self.addr, self.aggregator, **(learner_kwargs or {}))
        self.exp_name = exp_name
        self._running = False
        self.state = NodeState(self.addr, simulation=simulation)
        self.simulation = simulation
        self.learning_workflow = LearningWorkflow(getattr(self._communication_protocol, "workflow", "gossip"))
        self._learning_thread: Optional[threading.Thread] = None
        self._communication_protocol.add_command(
            [
                StartLearningCommand(self._start_learning_thread),
                StopLearningCommand(self.state, self.aggregator, self.learner),
                ModelInitializedCommand(self.state),
                VoteTrainSetCommand(self.state),
                ModelsAggregatedCommand(self.state),
                ModelsReadyCommand(self.state),
                MetricsCommand(self.state),
                InitModelCommand(self.state, self.stop, self.aggregator, self.learner),
                PartialModelCommand(self.state, self.stop, self.aggregator, self._communication_protocol, self.learner),
                FullModelCommand(self.state, self.stop, self.aggregator, self.learner),
            ]
        )
        if hasattr(self._communication_protocol, "bind_node"):
            self._communication_protocol.bind_node(self)

    @property
    def communication_protocol(self) -> CommunicationProtocol:
        return self._communication_protocol

    # ------------------------------------------------------------------ neighbourhood
    def connect(self, addr: str) -> bool:
        self.assert_running(True)
        return self._communication_protocol.connect(addr)

    def get_neighbors(self, only_direct: bool = False) -> Dict[str, Any]:
        return self._communication_protocol.get_neighbors(only_direct)

    def disconnect(self, addr: str) -> None:
        self.assert_running(True)
        logger.info(self.addr, f"Removing {addr}...")
        self._communication_protocol.disconnect(addr, disconnect_msg=True)

    # ------------------------------------------------------------------ lifecycle
    def assert_running(self, running: bool) -> None:
        if self._running != running:
            raise NodeRunningException(f"Node is {'not ' if self._running else ''}running.")

    def start(self, wait: bool = False) -> None:
        self.assert_running(False)
        self._running = True
        logger.register_node(self.addr, self.simulation)
        self._communication_protocol.start()
        if Settings.ENGINE_PREWARM:
            prewarm = getattr(self.learner, "prewarm", None)
            if prewarm is not None:
                prewarm()  # fused engine: capture the epoch graph now, not in round 0
        if wait:
            self._communication_protocol.wait_for_termination()
            logger.info(self.addr, "Protocol terminated.")

    def stop(self) -> None:
        logger.info(self.addr, "Stopping node...")
        with contextlib.suppress(Exception):
            self.learner.interrupt_fit()
        with contextlib.suppress(Exception):
            self._communication_protocol.stop()
        self._running = False
        self.state.clear()
        with contextlib.suppress(Exception):
            self.aggregator.clear()
        with contextlib.suppress(Exception):
            logger.unregister_node(self.addr)
        close = getattr(self.learner, "close", None)
        if close is not None:
            with contextlib.suppress(Exception):
                close()  # frees a grouped-engine slot: co-located peers stop waiting for this one

    # ------------------------------------------------------------------ learning setters/getters
    def set_learner(self, learner: Learner) -> None:
        if self.state.round is not None:
            raise LearnerRunningException("Learner cannot be set after learning is started.")
        self.learner = learner

    def set_model(self, model: P2PFLModel) -> None:
        if self.state.round is not None:
            raise LearnerRunningException("Data cannot be set after learner is set.")
        self.learner.set_model(model)

    def set_data(self, data: Any) -> None:
        if self.state.round is not None:
            raise LearnerRunningException("Data cannot be set after learner is set.")
        self.learner.set_data(data)

    def set_epochs(self, epochs: int) -> None:
        """Documented by the reference (``docs/.../node.md:103``) but missing there."""
        self.learner.set_epochs(epochs)

    def get_model(self) -> P2PFLModel:
        return self.learner.get_model()

    def get_data(self) -> Any:
        return self.learner.get_data()

    # ------------------------------------------------------------------ network learning
    def _start_learning_thread(self, rounds: int, epochs: int, start_round: int = 0) -> None:
        with self.state.start_thread_lock:
            if self._learning_thread is not None and self._learning_thread.is_alive():
                return
            self.learning_workflow.finished = False
            t = threading.Thread(target=self._start_learning, args=(rounds, epochs, start_round), name=f"learning_thread-{self.addr}", daemon=True)
            self._learning_thread = t
            t.start()

    def set_start_learning(self, rounds: int = 1, epochs: int = 1, start_round: int = 0) -> Optional[str]:
        """Start network-wide learning. ``start_round > 0`` resumes an experiment whose first
        ``start_round`` rounds are already done (restore models with
        :func:`myfyp_amd.management.checkpoint.restore_node` first)."""
        self.assert_running(True)
        if rounds < 1:
            raise ZeroRoundsException("Rounds must be greater than 0.")
        if not 0 <= start_round < rounds:
            raise ValueError(f"start_round must be in [0, {rounds}), got {start_round}")
        if self.state.round is not None:
            logger.info(self.addr, "Learning already started")
            return None
        logger.info(self.addr, "🚀 Broadcasting start learning...")
        proto = self._communication_protocol
        args = [str(rounds), str(epochs)] + ([str(start_round)] if start_round else [])
        proto.broadcast(proto.build_msg(StartLearningCommand.get_name(), args))
        self.state.model_initialized_lock.release()
        proto.broadcast(proto.build_msg(ModelInitializedCommand.get_name()))
        self._start_learning_thread(rounds, epochs, start_round)
        return self.exp_name

    def set_stop_learning(self) -> None:
        if self.state.round is None:
            logger.info(self.addr, "Learning already stopped")
            return
        self._communication_protocol.broadcast(self._communication_protocol.build_msg(StopLearningCommand.get_name()))
        self._stop_learning()

    def _start_learning(self, rounds: int, epochs: int, start_round: int = 0) -> None:
        try:
            self.learning_workflow.run(
                rounds=rounds,
                epochs=epochs,
                start_round=start_round,
                state=self.state,
                learner=self.learner,
                communication_protocol=self._communication_protocol,
                aggregator=self.aggregator,
                exp_name=self.exp_name,
                node=self,
            )
        except Exception as e:
            if getattr(e, "fault_injected", False):
                logger.warning(self.addr, f"learning thread ended by fault injection: {e}")
            else:
                logger.error(self.addr, f"Error {type(e).__name__}: {e}\n{traceback.format_exc()}")
            self.stop()

    def _stop_learning(self) -> None:
        logger.info(self.addr, "Stopping learning")
        self.learner.interrupt_fit()
        self.aggregator.clear()
        self.state.clear()
        logger.experiment_finished(self.addr)
        with contextlib.suppress(Exception):
            self.state.wait_votes_ready_lock.release()
