"""``add_model`` (parity: ``weights/full_model_command.py:31-89``)."""

from typing import Callable, Optional

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.learning.frameworks.exceptions import DecodingParamsError, ModelNotMatchingError
from myfyp_amd.management.logger import logger


class FullModelCommand(Command):
    """Installs a fully aggregated model on a node that is waiting for one."""

    def __init__(self, state, stop: Callable[[], None], aggregator, learner) -> None:
        self.state = state
        self.stop = stop
        self.aggregator = aggregator
        self.learner = learner

    @staticmethod
    def get_name() -> str:
        return "add_model"

    def execute(self, source: str, round: int, weights: Optional[bytes] = None, *args, **kwargs) -> None:
        if weights is None:
            raise ValueError("Weights are required")
        st = self.state
        if st.round is None:
            logger.debug(st.addr, "❌ Tried to add a model while learning is not running")
            return
        if round != st.round:
            logger.debug(st.addr, f"Model reception in a late round ({round} != {st.round}).")
            return
        if st.aggregated_model_event.is_set():
            logger.debug(st.addr, "😲 Aggregated model not expected.")
            return
        try:
            logger.info(st.addr, "📦 Aggregated model received.")
            self.learner.set_model(weights)
            st.aggregated_model_event.set()
        except (DecodingParamsError, ModelNotMatchingError) as e:
            logger.error(st.addr, f"❌ Invalid aggregated model from {source}: {e}")
