"""``models_ready`` (parity: ``message/models_ready_command.py:26-62``)."""

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.management.logger import logger


class ModelsReadyCommand(Command):
    """The sender holds the aggregated model of ``round`` (``nei_status[src] = round``)."""

    def __init__(self, state) -> None:
        self.state = state

    @staticmethod
    def get_name() -> str:
        return "models_ready"

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        st = self.state
        if st.round is None:
            logger.warning(st.addr, "Models ready received when learning is not running")
            return
        if round in (st.round - 1, st.round):
            st.nei_status[source] = st.round
            st.notify_status()
        else:
            logger.error(st.addr, f"Models ready from {source} in a late round. Ignored. {round} != {st.round} / {st.round - 1}")
