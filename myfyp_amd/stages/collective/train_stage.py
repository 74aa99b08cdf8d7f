"""Collective train (parity target: ``stages/base_node/train_stage.py:44-187``).

Evaluate → fit (co-located trainers ganged into one fused launch sequence) → join the round's
aggregation collective with weight ``n_i``. No partial-model gossip: one weighted RCCL all-reduce
leaves every peer of every rank holding the FedAvg result.
"""

import time
from typing import Optional, Type

from myfyp_amd.management.logger import logger
from myfyp_amd.stages.collective import fused_round
from myfyp_amd.stages.collective.wait_agg_models_stage import join_aggregation
from myfyp_amd.stages.stage import EarlyStopException, Stage, check_early_stop
from myfyp_amd.stages.stage_factory import StageFactory


class TrainStage(Stage):
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
            if getattr(state, "fused_round", False):
                fused_round.join(state, learner, aggregator, trainer=True)
                return StageFactory.get_stage("GossipModelStage", "collective")
            # metrics are only logged here (reference: train_stage.py:104-117), so the evaluation is
            # enqueued and its results are filed under this round when they land — no GPU wait
            if hasattr(learner, "evaluate_async"):
                learner.evaluate_async()
            else:
                logger.debug(state.addr, f"📈 Evaluated. Results: {learner.evaluate()}")
            check_early_stop(state)
            learner.fit()
            check_early_stop(state)
            t0 = time.time()
            join_aggregation(state, learner, aggregator, trainer=True)
            logger.log_timing(state.addr, "aggregate", time.time() - t0)
            return StageFactory.get_stage("GossipModelStage", "collective")
        except EarlyStopException:
            return None
