"""Diffuse the aggregate (parity: ``stages/base_node/gossip_model_stage.py:41-87``)."""

from typing import Any, List, Optional, Type

from myfyp_amd.communication.commands.weights.full_model_command import FullModelCommand
from myfyp_amd.management.logger import logger
from myfyp_amd.stages.stage import Stage, check_early_stop
from myfyp_amd.stages.stage_factory import StageFactory


class GossipModelStage(Stage):
    """Send the full model to direct neighbours that have not reported this round's model."""

    @staticmethod
    def name() -> str:
        return "GossipModelStage"

    @staticmethod
    def execute(state=None, communication_protocol=None, aggregator=None, learner=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or aggregator is None or communication_protocol is None or learner is None:
            raise Exception("Invalid parameters on GossipModelStage.")
        logger.info(state.addr, "🗣️ Gossiping aggregated model.")
        fixed_round = state.round
        if fixed_round is None:
            return None

        def candidates() -> List[str]:
            return [n for n in communication_protocol.get_neighbors(only_direct=True) if state.nei_status.get(n, -1) < fixed_round]

        encoded: dict = {}

        def model_fn(_: str) -> Any:
            if state.round is None:
                raise Exception("Round not initialized")
            if "m" not in encoded:  # encode once per stage, not once per send
                encoded["m"] = learner.get_model().encode_parameters()
            return communication_protocol.build_weights(FullModelCommand.get_name(), state.round, encoded["m"])

        communication_protocol.gossip_weights(lambda: check_early_stop(state, raise_exception=False), candidates, candidates, model_fn, wait_fn=state.wait_status)
        return StageFactory.get_stage("RoundFinishedStage")
