"""Train + aggregate (parity: ``stages/base_node/train_stage.py:44-187``)."""

import time
from typing import Any, List, Optional, Set, Type

from myfyp_amd.communication.commands.message.metrics_command import MetricsCommand
from myfyp_amd.communication.commands.message.models_agregated_command import ModelsAggregatedCommand
from myfyp_amd.communication.commands.message.models_ready_command import ModelsReadyCommand
from myfyp_amd.communication.commands.weights.partial_model_command import PartialModelCommand
from myfyp_amd.learning.aggregators.aggregator import NoModelsToAggregateError
from myfyp_amd.management.logger import logger
from myfyp_amd.stages.stage import EarlyStopException, Stage, check_early_stop
from myfyp_amd.stages.stage_factory import StageFactory


def broadcast_metrics(state, communication_protocol, results: dict) -> None:
    if results:
        flat = [str(x) for kv in results.items() for x in kv]
        communication_protocol.broadcast(communication_protocol.build_msg(MetricsCommand.get_name(), flat, round=state.round))


class TrainStage(Stage):
    """Evaluate → fit → add own model → gossip partial aggregates → wait → install aggregate."""

    @staticmethod
    def name() -> str:
        return "TrainStage"

    @staticmethod
    def execute(state=None, communication_protocol=None, learner=None, aggregator=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None or aggregator is None or learner is None:
            raise Exception("Invalid parameters on TrainStage.")
        try:
            check_early_stop(state)
            aggregator.set_nodes_to_aggregate(state.train_set)
            check_early_stop(state)
            logger.info(state.addr, "🔬 Evaluating...")
            results = learner.evaluate()
            logger.info(state.addr, f"📈 Evaluated. Results: {results}")
            broadcast_metrics(state, communication_protocol, results)
            check_early_stop(state)
            logger.info(state.addr, "🏋️‍♀️ Training...")
            learner.fit()
            check_early_stop(state)
            models_added = aggregator.add_model(learner.get_model())
            communication_protocol.broadcast(communication_protocol.build_msg(ModelsAggregatedCommand.get_name(), models_added, round=state.round))
            TrainStage._gossip_model_aggregation(state, communication_protocol, aggregator)
            check_early_stop(state)
            t0 = time.time()
            agg_model = aggregator.wait_and_get_aggregation()
            learner.set_model(agg_model)
            logger.log_timing(state.addr, "aggregate", time.time() - t0)
            communication_protocol.broadcast(communication_protocol.build_msg(ModelsReadyCommand.get_name(), [], round=state.round))
            return StageFactory.get_stage("GossipModelStage")
        except EarlyStopException:
            return None

    @staticmethod
    def _aggregated(node: str, state) -> List[str]:
        return state.models_aggregated.get(node, [])

    @staticmethod
    def _remaining(node: str, state) -> Set[str]:
        return set(state.train_set) - set(TrainStage._aggregated(node, state))

    @staticmethod
    def _gossip_model_aggregation(state, communication_protocol, aggregator) -> None:
        def candidates() -> List[str]:
            return [n for n in set(state.train_set) - {state.addr} if TrainStage._remaining(n, state)]

        def status() -> Any:
            return [(n, TrainStage._aggregated(n, state)) for n in communication_protocol.get_neighbors(only_direct=False) if n in state.train_set]

        def model_fn(node: str) -> Any:
            try:
                model = aggregator.get_model(TrainStage._aggregated(node, state))
            except NoModelsToAggregateError:
                logger.info(state.addr, f"❔ No models to aggregate from {node}.")
                return None
            if state.round is None:
                raise Exception("Round not initialized.")
            return communication_protocol.build_weights(
                PartialModelCommand.get_name(), state.round, model.encode_parameters(), model.get_contributors(), model.get_num_samples()
            )

        communication_protocol.gossip_weights(lambda: state.round is None, candidates, status, model_fn, create_connection=True, wait_fn=state.wait_status)
