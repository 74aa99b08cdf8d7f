"""``partial_model`` (parity: ``weights/partial_model_command.py:33-112``)."""

from typing import Callable, List, Optional

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.communication.commands.message.models_agregated_command import ModelsAggregatedCommand
from myfyp_amd.learning.frameworks.exceptions import DecodingParamsError, ModelNotMatchingError
from myfyp_amd.management.logger import logger


class PartialModelCommand(Command):
    """Adds a (partial) aggregate from a train-set peer and announces the new contributor set."""

    def __init__(self, state, stop: Callable[[], None], aggregator, comm_proto, learner) -> None:
        self.state = state
        self.stop = stop
        self.aggregator = aggregator
        self.communication_protocol = comm_proto
        self.learner = learner

    @staticmethod
    def get_name() -> str:
        return "partial_model"

    def execute(
        self,
        source: str,
        round: int,
        weights: Optional[bytes] = None,
        contributors: Optional[List[str]] = None,
        num_samples: Optional[int] = None,
        *args,
        **kwargs,
    ) -> None:
        if weights is None or contributors is None or num_samples is None:
            raise ValueError("Weights, contributors and weight are required")
        st = self.state
        if st.round is None:
            logger.debug(st.addr, "Tried to add a model while learning is not running")
            return
        if round != st.round:
            logger.debug(st.addr, f"Model reception in a late round ({round} != {st.round}).")
            return
        if len(st.train_set) == 0:
            logger.error(st.addr, "Model Reception when there is no trainset")
            return
        try:
            model = self.learner.get_model().build_copy(params=weights, num_samples=num_samples, contributors=list(contributors))
            models_added = self.aggregator.add_model(model)
            if models_added:
                self.communication_protocol.broadcast(
                    self.communication_protocol.build_msg(ModelsAggregatedCommand.get_name(), models_added, round=st.round)
                )
        except (DecodingParamsError, ModelNotMatchingError) as e:
            # reference stops the node (partial_model_command.py:98-107); a malformed payload from one
            # peer should not take this node down (SURVEY §5.3 DoS note): drop it and log.
            logger.error(st.addr, f"Invalid partial model from {source}: {e}")
