"""``vote_train_set`` (parity: ``message/vote_train_set_command.py:28-74``)."""

import contextlib

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.management.logger import logger


class VoteTrainSetCommand(Command):
    """Stores ``(node, weight)*`` votes for the current (or next) round and wakes the voter."""

    def __init__(self, state) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "vote_train_set"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        st = self.state
        if st.round is None:
            logger.error(st.addr, "Vote received when learning is not running")
            return
        if round not in (st.round, st.round + 1):
            logger.error(st.addr, f"Vote received in a late round. Ignored. {round} != {st.round} / {st.round + 1}")
            return
        votes = {args[i]: int(args[i + 1]) for i in range(0, len(args) - 1, 2)}
        with st.train_set_votes_lock:
            st.train_set_votes[source] = votes
            st.round_votes.setdefault(round, {})[source] = votes
        st.votes_event.set()
        with contextlib.suppress(Exception):
            st.wait_votes_ready_lock.release()
