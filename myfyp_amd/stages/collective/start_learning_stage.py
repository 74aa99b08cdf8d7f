"""Collective start (parity target: ``stages/base_node/start_learning_stage.py:44-112``).

The reference gossips the initiator's pickled model until every neighbour is initialised; here
every co-located peer joins one gang op whose leader broadcasts the reference weights over RCCL
(deterministic source: the first peer of the federation) — bit-identical initial models everywhere.
"""

from typing import Optional, Type

from myfyp_amd.management.logger import logger
from myfyp_amd.parallel import weights_plane
from myfyp_amd.stages.collective._common import fed
from myfyp_amd.stages.stage import Stage
from myfyp_amd.stages.stage_factory import StageFactory


class StartLearningStage(Stage):
    @staticmethod
    def name() -> str:
        return "StartLearningStage"

    @staticmethod
    def execute(rounds=None, epochs=None, state=None, learner=None, communication_protocol=None, aggregator=None, exp_name: str = "experiment", **kwargs) -> Optional[Type[Stage]]:
        if rounds is None or epochs is None or state is None or learner is None or communication_protocol is None or aggregator is None:
            raise Exception("Invalid parameters on StartLearningStage.")
        f = fed()
        with state.start_thread_lock:
            state.set_experiment(exp_name, rounds, start_round=int(kwargs.get("start_round", 0) or 0))
            learner.set_epochs(epochs)
            logger.experiment_started(state.addr, state.experiment)
        if not f.finalized.is_set():
            f.finalized.wait()
        initiator = f.all_peers()[0]
        f.gang_run(state.addr, None, lambda arrived: weights_plane.sync_initial_model(f, arrived, initiator))
        logger.info(state.addr, "🤖 Initial model synchronised (RCCL broadcast).")
        return StageFactory.get_stage("VoteTrainSetStage", "collective")
