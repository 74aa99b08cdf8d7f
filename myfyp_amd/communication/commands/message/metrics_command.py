"""``metrics`` (parity: ``message/metrics_command.py:26-53``)."""

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.management.logger import logger


class MetricsCommand(Command):
    """Logs ``(key, value)*`` evaluation metrics of the sender as global metrics."""

    def __init__(self, state) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "metrics"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        for i in range(0, len(args) - 1, 2):
            logger.log_metric(source, args[i], float(args[i + 1]), round=round)
