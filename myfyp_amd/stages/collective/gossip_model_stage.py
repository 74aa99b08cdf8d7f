"""Collective "gossip" (parity target: ``stages/base_node/gossip_model_stage.py``): after the
all-reduce every peer already holds the aggregate, so diffusion is a no-op."""

from typing import Optional, Type

from myfyp_amd.stages.stage import Stage
from myfyp_amd.stages.stage_factory import StageFactory


class GossipModelStage(Stage):
    @staticmethod
    def name() -> str:
        return "GossipModelStage"

    @staticmethod
    def execute(state=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or state.round is None:
            return None
        return StageFactory.get_stage("RoundFinishedStage", "collective")
