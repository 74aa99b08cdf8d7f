"""Stage base + early stop (parity: ``p2pfl/stages/stage.py:26-66``)."""

from typing import Optional, Type

from myfyp_amd.management.logger import logger


class Stage:
    """A step of the learning workflow; ``execute(**kw)`` returns the next stage or ``None``."""

    @staticmethod
    def name() -> str:
        raise NotImplementedError("Stage name not implemented.")

    @staticmethod
    def execute(**kwargs) -> Optional[Type["Stage"]]:
        raise NotImplementedError("Stage execute not implemented.")


class EarlyStopException(Exception):
    """Learning was stopped while a stage was running."""


def check_early_stop(state, raise_exception: bool = True) -> bool:
    if state.round is None:
        logger.info(state.addr, "Stopping Workflow.")
        if raise_exception:
            raise EarlyStopException("Early stopping.")
        return True
    return False
