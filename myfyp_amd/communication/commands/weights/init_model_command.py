"""``init_model`` (parity: ``weights/init_model_command.py:31-97``)."""

from typing import Callable, Optional

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.learning.frameworks.exceptions import DecodingParamsError, ModelNotMatchingError
from myfyp_amd.management.logger import logger


class InitModelCommand(Command):
    """Loads the initiator's weights and releases ``model_initialized_lock``."""

    def __init__(self, state, stop: Callable[[], None], aggregator, learner) -> None:
        self.state = state
        self.stop = stop
        self.aggregator = aggregator
        self.learner = learner

    @staticmethod
    def get_name() -> str:
        return "init_model"

    def execute(self, source: str, round: int, weights: Optional[bytes] = None, *args, **kwargs) -> None:
        st = self.state
        if weights is None:
            logger.error(st.addr, "Invalid InitModelCommand message")
            return
        if st.round is None:
            logger.debug(st.addr, "Tried to add a model while learning is not running")
            return
        if round != st.round:
            logger.debug(st.addr, f"Model initialization in a late round ({round} != {st.round}).")
            return
        if not st.model_initialized_lock.locked():
            logger.debug(st.addr, "Model initialization message when the model is already initialized. Ignored.")
            return
        try:
            self.learner.set_model(weights)
            st.model_initialized_lock.release()
            logger.info(st.addr, "🤖 Model Weights Initialized")
        except (DecodingParamsError, ModelNotMatchingError) as e:
            logger.error(st.addr, f"Invalid initial model: {e}")
            self.stop()
        except RuntimeError:
            pass  # released concurrently by another sender
