"""Command interface (parity: ``p2pfl/communication/commands/command.py:24-43``)."""

import abc


class Command(abc.ABC):
    """A named message handler registered on a protocol."""

    @staticmethod
    def get_name() -> str:
        raise NotImplementedError

    @abc.abstractmethod
    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        """Handle a message from ``source`` tagged with ``round``."""
        raise NotImplementedError
