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

    @staticmethod
    def preload(flavor: str = "gossip") -> None:
        """Import every stage module of ``flavor`` now (workflow construction), not on the first
        transition: a first import inside a running experiment held the import lock for several ms
        while all eight peer threads queued on it between StartLearning and the first vote
        (``scripts/probes/start_sampler.py``, ``profiles/r5_start``)."""
        for name in _STAGES:
            StageFactory.get_stage(name, flavor)
        if flavor != "gossip":
            importlib.import_module("myfyp_amd.stages.collective.driver")
