"""Vote the round's train set (parity: ``stages/base_node/vote_train_set_stage.py:43-184``).

Differences: the vote wait wakes on each vote (``votes_event``) instead of 2 s polling; the vote RNG
is seeded from ``Settings.SEED`` + node + round when a seed is set (reproducible train sets, SURVEY
§2.11 #14); ``_validate_train_set`` does not mutate the list it iterates (#5).
"""

import math
import random
import time
from typing import Dict, List, Optional, Type

from myfyp_amd.communication.commands.message.vote_train_set_command import VoteTrainSetCommand
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings
from myfyp_amd.stages.stage import EarlyStopException, Stage, check_early_stop
from myfyp_amd.stages.stage_factory import StageFactory


def vote_rng(addr: str, round_: Optional[int]) -> random.Random:
    if Settings.SEED is None:
        return random.Random()
    return random.Random(f"{Settings.SEED}-{addr}-{round_}")


def make_votes(addr: str, candidates: List[str], round_: Optional[int]) -> Dict[str, int]:
    """``min(TRAIN_SET_SIZE, |candidates|)`` peers with weights ``floor(randint(0,1000)/(i+1))``."""
    rng = vote_rng(addr, round_)
    samples = min(Settings.TRAIN_SET_SIZE, len(candidates))
    nodes = rng.sample(sorted(candidates), samples)
    weights = [math.floor(rng.randint(0, 1000) / (i + 1)) for i in range(samples)]
    return dict(zip(nodes, weights))


def tally_votes(votes: Dict[str, Dict[str, int]]) -> List[str]:
    """Sum weights, order by (votes desc, name desc), keep the top ``TRAIN_SET_SIZE``."""
    results: Dict[str, int] = {}
    for node_vote in votes.values():
        for k, v in node_vote.items():
            results[k] = results.get(k, 0) + v
    ordered = sorted(results.items(), key=lambda x: x[0], reverse=True)
    ordered = sorted(ordered, key=lambda x: x[1], reverse=True)
    return [k for k, _ in ordered[: min(len(ordered), Settings.TRAIN_SET_SIZE)]]


class VoteTrainSetStage(Stage):
    """Vote, gather everybody's votes (or time out), keep the top-K live nodes."""

    @staticmethod
    def name() -> str:
        return "VoteTrainSetStage"

    @staticmethod
    def execute(state=None, communication_protocol=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None:
            raise Exception("Invalid parameters on VoteTrainSetStage.")
        logger.round_started(state.addr, state.experiment)
        try:
            VoteTrainSetStage._vote(state, communication_protocol)
            state.train_set = VoteTrainSetStage._validate_train_set(VoteTrainSetStage._aggregate_votes(state, communication_protocol), state, communication_protocol)
            logger.info(state.addr, f"🚂 Train set of {len(state.train_set)} nodes: {state.train_set}")
            if state.addr in state.train_set:
                return StageFactory.get_stage("TrainStage")
            return StageFactory.get_stage("WaitAggregatedModelsStage")
        except EarlyStopException:
            return None

    @staticmethod
    def _vote(state, communication_protocol) -> None:
        candidates = list(communication_protocol.get_neighbors(only_direct=False))
        if state.addr not in candidates:
            candidates.append(state.addr)
        votes = make_votes(state.addr, candidates, state.round)
        with state.train_set_votes_lock:
            state.train_set_votes[state.addr] = votes
            state.round_votes.setdefault(state.round, {})[state.addr] = votes
        logger.debug(state.addr, f"🪞🗳️ Self Vote: {votes}")
        communication_protocol.broadcast(
            communication_protocol.build_msg(VoteTrainSetCommand.get_name(), [str(x) for kv in votes.items() for x in kv], round=state.round)
        )

    @staticmethod
    def _aggregate_votes(state, communication_protocol) -> List[str]:
        deadline = time.time() + Settings.VOTE_TIMEOUT
        while True:
            check_early_stop(state)
            state.votes_event.clear()
            members = set(communication_protocol.get_neighbors(only_direct=False)) | {state.addr}
            with state.train_set_votes_lock:
                nc_votes = {k: v for k, v in state.round_votes.get(state.round, {}).items() if k in members}
            ready = members == set(nc_votes)
            timeout = time.time() > deadline
            if ready or timeout:
                if timeout and not ready:
                    logger.info(state.addr, f"Timeout for vote aggregation. Missing votes from {members - set(nc_votes)}")
                with state.train_set_votes_lock:
                    # drop this round's votes, keep those already cast for the next round
                    state.train_set_votes = {}
                    for r in [r for r in state.round_votes if state.round is not None and r <= state.round]:
                        del state.round_votes[r]
                logger.info(state.addr, f"🔢 Computed {len(nc_votes)} votes.")
                return tally_votes(nc_votes)
            state.votes_event.wait(timeout=min(0.5, max(0.0, deadline - time.time())))

    @staticmethod
    def _validate_train_set(train_set: List[str], state, communication_protocol) -> List[str]:
        members = set(communication_protocol.get_neighbors(only_direct=False))
        return [n for n in train_set if n in members or n == state.addr]
