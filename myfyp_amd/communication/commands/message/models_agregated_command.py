"""``models_aggregated`` (parity: ``message/models_agregated_command.py:26-56``)."""

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.management.logger import logger


class ModelsAggregatedCommand(Command):
    """Records which contributions the sender already aggregated (same round only)."""

    def __init__(self, state) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "models_aggregated"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        if round == self.state.round:
            self.state.models_aggregated[source] = list(args)
            self.state.notify_status()
        else:
            logger.debug(self.state.addr, f"Models Aggregated from {source} in a late round. Ignored. {round} != {self.state.round}")
