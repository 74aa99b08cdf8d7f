"""Workflow runner (parity: ``p2pfl/stages/workflows.py:28-60``).

``history`` records every executed stage name (tests pin the pattern); ``finished`` flips when the
workflow ends. Each stage's wall time is recorded with ``logger.log_timing``.
"""

import time
from typing import Any, Callable, Dict, List, Optional, Type

from myfyp_amd.management.logger import logger
from myfyp_amd.management.tracing import trace_range
from myfyp_amd.stages.stage import Stage, check_early_stop
from myfyp_amd.stages.stage_factory import StageFactory


class StageWokflow:
    """Runs stages until one returns ``None`` or learning stops."""

    def __init__(self, first_stage: Type[Stage]) -> None:
        self.first_stage = first_stage
        self.current_stage = first_stage
        self.history: List[str] = []
        self.finished = False
        # called as hook(stage_name, kwargs) before each stage (fault injection, tracing)
        self.hooks: List[Callable[[str, Dict[str, Any]], None]] = []

    def run(self, **kwargs) -> None:
        self.finished = False
        self.current_stage = self.first_stage
        state = kwargs.get("state")
        if state is None:
            raise ValueError("State not found in kwargs")
        try:
            while True:
                logger.debug(state.addr, f"🏃 Running stage: {self.current_stage.name()}")
                self.history.append(self.current_stage.name())
                for hook in list(self.hooks):
                    hook(self.current_stage.name(), kwargs)
                t0 = time.time()
                with trace_range(f"{self.current_stage.name()}/{state.addr}"):
                    next_stage: Optional[Type[Stage]] = self.current_stage.execute(**kwargs)
                logger.log_timing(state.addr, self.current_stage.name(), time.time() - t0)
                if next_stage is None or check_early_stop(state, raise_exception=False):
                    break
                self.current_stage = next_stage
        finally:
            self.finished = True


StageWorkflow = StageWokflow


class LearningWorkflow(StageWokflow):
    """Federated-learning workflow; ``flavor`` selects gossip or collective stages."""

    def __init__(self, flavor: str = "gossip") -> None:
        self.flavor = flavor
        StageFactory.preload(flavor)
        super().__init__(StageFactory.get_stage("StartLearningStage", flavor))
