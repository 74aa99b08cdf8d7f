"""``model_initialized`` (parity: ``message/model_initialized_command.py:25-48``)."""

from myfyp_amd.communication.commands.command import Command


class ModelInitializedCommand(Command):
    """Marks the sender as initialised (``nei_status[src] = -1``)."""

    def __init__(self, state) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "model_initialized"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        self.state.nei_status[source] = -1
        self.state.notify_status()
