"""Collective round end (parity: ``stages/base_node/round_finished_stage.py:42-91``)."""

from typing import Optional, Type

from myfyp_amd.management.checkpoint import maybe_checkpoint
from myfyp_amd.management.logger import logger
from myfyp_amd.stages.collective._common import fed, set_gang_expectations
from myfyp_amd.stages.stage import Stage
from myfyp_amd.stages.stage_factory import StageFactory


class RoundFinishedStage(Stage):
    @staticmethod
    def name() -> str:
        return "RoundFinishedStage"

    @staticmethod
    def execute(state=None, learner=None, communication_protocol=None, aggregator=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None or aggregator is None or learner is None:
            raise Exception("Invalid parameters on RoundFinishedStage.")
        aggregator.clear()
        state.increase_round()
        logger.round_finished(state.addr)
        logger.debug(state.addr, f"🎉 Round {state.round} of {state.total_rounds} finished.")
        if state.round is None or state.total_rounds is None:
            raise ValueError("Round or total rounds not set.")
        maybe_checkpoint(state, learner)
        if state.round < state.total_rounds:
            return StageFactory.get_stage("VoteTrainSetStage", "collective")
        f = fed()
        f.gang_run(state.addr, None, lambda arrived: set_gang_expectations(f, set(), None))
        results = learner.evaluate()
        logger.info(state.addr, f"📈 Final evaluation: {results}")
        state.clear()
        logger.experiment_finished(state.addr)
        return None
