"""Lazy stage lookup (parity: ``p2pfl/stages/stage_factory.py:26-59``).

``get_stage(name, flavor)``: ``flavor="gossip"`` returns the reference-semantics stages
(message gossip, partial aggregates); ``flavor="collective"`` returns the MI355X collective stages
(same names, same transitions, RCCL data plane) used with ``CollectiveCommunicationProtocol``.
"""

import importlib
from typing import Type

from myfyp_amd.stages.stage import Stage

_STAGES = {
    "StartLearningStage": "start_learning_stage",
    "VoteTrainSetStage": "vote_train_set_stage",
    "TrainStage": "train_stage",
    "WaitAggregatedModelsStage": "wait_agg_models_stage",
    "GossipModelStage": "gossip_model_stage",
    "RoundFinishedStage": "round_finished_stage",
}


class StageFactory:
    """Maps stage names to classes without import cycles."""

    @staticmethod
    def get_stage(stage_name: str, flavor: str = "gossip") -> Type[Stage]:
        mod = _STAGES.get(stage_name)
        if mod is None:
            raise Exception("Invalid stage name.")
        pkg = "base_node" if flavor == "gossip" else "collective"
        return getattr(importlib.import_module(f"myfyp_amd.stages.{pkg}.{mod}"), stage_name)
