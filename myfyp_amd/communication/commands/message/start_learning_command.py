"""``start_learning`` (parity: ``message/start_learning_command.py:26-60``)."""

from typing import Callable, Optional

from myfyp_amd.communication.commands.command import Command


class StartLearningCommand(Command):
    """Spawns the node's learning thread with the broadcast rounds/epochs."""

    def __init__(self, start_learning_fn: Callable[..., None]) -> None:
        self._start_learning_fn = start_learning_fn

    @staticmethod
    def get_name() -> str:
        return "start_learning"

    def execute(self, source: str, round: int, learning_rounds: Optional[str] = None, learning_epochs: Optional[str] = None, *args, **kwargs) -> None:
        if learning_rounds is None or learning_epochs is None:
            raise ValueError("Learning rounds and epochs are required")
        # optional 3rd arg (extension): round to resume from; reference peers send only two
        start_round = int(args[0]) if args else 0
        self._start_learning_fn(int(learning_rounds), int(learning_epochs), start_round)
