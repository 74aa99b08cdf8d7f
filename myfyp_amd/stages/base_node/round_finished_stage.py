"""Round bookkeeping (parity: ``stages/base_node/round_finished_stage.py:42-91``)."""

from typing import Optional, Type

from myfyp_amd.management.checkpoint import maybe_checkpoint
from myfyp_amd.management.logger import logger
from myfyp_amd.stages.base_node.train_stage import broadcast_metrics
from myfyp_amd.stages.stage import Stage
from myfyp_amd.stages.stage_factory import StageFactory


class RoundFinishedStage(Stage):
    """Clear the aggregator, advance the round; final evaluation after the last round."""

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
        logger.info(state.addr, f"🎉 Round {state.round} of {state.total_rounds} finished.")
        if state.round is None or state.total_rounds is None:
            raise ValueError("Round or total rounds not set.")
        maybe_checkpoint(state, learner)
        if state.round < state.total_rounds:
            return StageFactory.get_stage("VoteTrainSetStage")
        logger.info(state.addr, "🔬 Evaluating...")
        results = learner.evaluate()
        logger.info(state.addr, f"📈 Evaluated. Results: {results}")
        broadcast_metrics(state, communication_protocol, results)
        state.clear()
        logger.experiment_finished(state.addr)
        logger.info(state.addr, "😋 Training finished!!")
        return None
