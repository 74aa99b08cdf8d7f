"""Start learning (parity: ``stages/base_node/start_learning_stage.py:44-112``)."""

import time
from typing import Any, List, Optional, Type

from myfyp_amd.communication.commands.message.model_initialized_command import ModelInitializedCommand
from myfyp_amd.communication.commands.weights.init_model_command import InitModelCommand
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings
from myfyp_amd.stages.stage import Stage
from myfyp_amd.stages.stage_factory import StageFactory


class StartLearningStage(Stage):
    """Set the experiment, wait for the initial model, gossip it to uninitialised neighbours."""

    @staticmethod
    def name() -> str:
        return "StartLearningStage"

    @staticmethod
    def execute(rounds=None, epochs=None, state=None, learner=None, communication_protocol=None, aggregator=None, exp_name: str = "experiment", **kwargs) -> Optional[Type[Stage]]:
        if rounds is None or epochs is None or state is None or learner is None or communication_protocol is None or aggregator is None:
            raise Exception("Invalid parameters on StartLearningStage.")
        with state.start_thread_lock:
            state.set_experiment(exp_name, rounds, start_round=int(kwargs.get("start_round", 0) or 0))
            learner.set_epochs(epochs)
            logger.experiment_started(state.addr, state.experiment)
        begin = time.time()
        logger.info(state.addr, "⏳ Waiting initialization.")
        lock = state.model_initialized_lock
        lock.acquire()
        # learning stopped while waiting for the initial model (NodeState.clear released the lock
        # it replaced). Test the lock's identity too: a new experiment may already have set a round
        # on the cleared state before this thread ran, and this stale stage must not join it
        # 
        if state.round is None or state.model_initialized_lock is not lock:
            logger.info(state.addr, "Learning stopped before the model was initialized.")
            return None
        communication_protocol.broadcast(communication_protocol.build_msg(ModelInitializedCommand.get_name()))
        logger.info(state.addr, "🗣️ Gossiping model initialization.")
        StartLearningStage._gossip_model(state, communication_protocol, learner)
        wait_time = Settings.WAIT_HEARTBEATS_CONVERGENCE - (time.time() - begin)
        if wait_time > 0:
            time.sleep(wait_time)
        return StageFactory.get_stage("VoteTrainSetStage")

    @staticmethod
    def _gossip_model(state, communication_protocol, learner) -> None:
        def candidates() -> List[str]:
            return [n for n in communication_protocol.get_neighbors(only_direct=True) if n not in state.nei_status]

        def model_fn(_: str) -> Any:
            if state.round is None:
                raise Exception("Round not initialized.")
            return communication_protocol.build_weights(InitModelCommand.get_name(), state.round, learner.get_model().encode_parameters())

        communication_protocol.gossip_weights(lambda: state.round is None, candidates, candidates, model_fn, wait_fn=state.wait_status)
