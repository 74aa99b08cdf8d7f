"""``stop_learning`` (parity: ``message/stop_learning_command.py:30-64``)."""

import contextlib

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.management.logger import logger


class StopLearningCommand(Command):
    """Interrupt fit, clear the aggregator and the state, wake the vote waiter."""

    def __init__(self, state, aggregator, learner) -> None:
        self.state = state
        self.aggregator = aggregator
        self.learner = learner

    @staticmethod
    def get_name() -> str:
        return "stop_learning"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        logger.info(self.state.addr, "Stopping learning received")
        self.learner.interrupt_fit()
        self.aggregator.clear()
        self.state.clear()
        logger.experiment_finished(self.state.addr)
        with contextlib.suppress(Exception):
            self.state.wait_votes_ready_lock.release()
