"""Collective vote (parity target: ``stages/base_node/vote_train_set_stage.py:43-184``).

Each peer still casts its own ``TRAIN_SET_SIZE`` weighted votes (same sampling rule), but votes are
all-gathered in one collective, so every rank tallies the identical vote set and the train set is
consistent by construction — a precondition for RCCL collectives (SURVEY §7.4 hard part 1).
"""

from typing import Optional, Type

from myfyp_amd.management.logger import logger
from myfyp_amd.parallel import weights_plane
from myfyp_amd.stages.base_node.vote_train_set_stage import make_votes, tally_votes
from myfyp_amd.stages.collective import driver, fused_round
from myfyp_amd.stages.collective._common import fed, set_gang_expectations
from myfyp_amd.stages.stage import Stage, check_early_stop
from myfyp_amd.stages.stage_factory import StageFactory


class VoteTrainSetStage(Stage):
    @staticmethod
    def name() -> str:
        return "VoteTrainSetStage"

    @staticmethod
    def execute(state=None, communication_protocol=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None:
            raise Exception("Invalid parameters on VoteTrainSetStage.")
        if check_early_stop(state, raise_exception=False):
            return None
        logger.round_started(state.addr, state.experiment)
        f = fed()
        votes = make_votes(state.addr, f.all_peers(), state.round)
        aggregator = kwargs.get("aggregator")
        everyone = bool(getattr(aggregator, "all_peers_train", False))

        def leader(arrived):
            allv = weights_plane.gather_votes(f, arrived)
            # decentralised mixing (NeighborAvg): every live peer trains; the gather still runs so
            # ranks learn who is alive
            train_set = sorted(allv, key=lambda a: f.all_peers().index(a)) if everyone else tally_votes(allv)
            set_gang_expectations(f, set(train_set), set(train_set))
            for hook in list(f.round_start_hooks):
                hook(state.round, f)
            return train_set, fused_round.eligible(f, aggregator), driver.eligible(f, aggregator)

        train_set, state.fused_round, drive = f.gang_run(state.addr, votes, leader)
        state.train_set = list(train_set)
        if drive:
            # the remaining rounds of every co-located peer run on one driver thread (driver.py);
            # this peer's workflow ends when its experiment does
            f.round_driver().enter(dict(kwargs, state=state, communication_protocol=communication_protocol))
            return None
        logger.info(state.addr, f"🚂 Train set of {len(state.train_set)} nodes: {state.train_set}")
        if state.addr in state.train_set:
            return StageFactory.get_stage("TrainStage", "collective")
        return StageFactory.get_stage("WaitAggregatedModelsStage", "collective")
