"""Wait for the aggregate (parity: ``stages/base_node/wait_agg_models_stage.py:40-67``)."""

from typing import Optional, Type

from myfyp_amd.communication.commands.message.models_ready_command import ModelsReadyCommand
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings
from myfyp_amd.stages.stage import Stage
from myfyp_amd.stages.stage_factory import StageFactory


class WaitAggregatedModelsStage(Stage):
    """Non-trainers block (≤ ``AGGREGATION_TIMEOUT``) until a full model arrives."""

    @staticmethod
    def name() -> str:
        return "WaitAggregatedModelsStage"

    @staticmethod
    def execute(state=None, communication_protocol=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None:
            raise Exception("Invalid parameters on WaitAggregatedModelsStage.")
        state.aggregated_model_event.clear()
        logger.info(state.addr, "⏳ Waiting aggregation.")
        if state.aggregated_model_event.wait(timeout=Settings.AGGREGATION_TIMEOUT):
            logger.info(state.addr, "✅ Aggregation event received.")
        else:
            logger.warning(state.addr, "⏰ Aggregation timeout occurred.")
        if state.round is None:
            return None
        communication_protocol.broadcast(communication_protocol.build_msg(ModelsReadyCommand.get_name(), [], round=state.round))
        return StageFactory.get_stage("GossipModelStage")
