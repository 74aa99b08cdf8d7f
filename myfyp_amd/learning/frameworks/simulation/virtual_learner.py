"""Learner decorator that runs fit/evaluate on the simulation device pool.

Parity: ``p2pfl/learning/frameworks/simulation/virtual_learner.py:31-141``. Setters and getters
go straight to the wrapped learner; ``fit``/``evaluate`` become pool jobs (``SuperActorPool``) that
run the learner in place on a device worker's HIP stream, so V simulated peers share the node's
GPUs with at most ``pool size`` of them training at once.

Difference from the reference: the wrapped learner lives in this process, so ``interrupt_fit``
reaches it (the reference raises ``NotImplementedError`` because its learner is inside a Ray actor).
Attribute reads not defined here fall through to the wrapped learner, except the fused-engine
entry points (``_engine``, ``fit_request``, ``evaluate_async``): a pooled peer always trains through
its own pool job rather than the grouped fast paths.
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Union

import numpy as np

from myfyp_amd.learning.frameworks.learner import Learner
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel
from myfyp_amd.learning.frameworks.simulation.actor_pool import SuperActorPool
from myfyp_amd.management.logger import logger

_NOT_FORWARDED = frozenset({"_engine", "fit_request", "evaluate_async"})


class VirtualNodeLearner(Learner):
    """Wraps a learner; fit/evaluate run as device-pool jobs."""

    def __init__(self, learner: Learner, addr: Optional[str] = None, pool: Optional[SuperActorPool] = None) -> None:
        # Learner.__init__ is not called: all state belongs to the wrapped learner
        self.__dict__["learner"] = learner
        self.actor_pool = pool if pool is not None else SuperActorPool()
        self.addr = addr if addr is not None else getattr(learner, "_self_addr", "unknown-node")

    def __getattr__(self, name: str) -> Any:
        if name in _NOT_FORWARDED or name.startswith("__") or "learner" not in self.__dict__:
            raise AttributeError(name)
        return getattr(self.__dict__["learner"], name)

    # state owned by the wrapped learner (the base class reads these attributes directly)
    @property
    def model(self) -> P2PFLModel:
        return self.learner.model

    @model.setter
    def model(self, value: P2PFLModel) -> None:
        self.learner.model = value

    @property
    def data(self) -> Any:
        return self.learner.data

    @data.setter
    def data(self, value: Any) -> None:
        self.learner.data = value

    @property
    def callbacks(self) -> List[Any]:
        return self.learner.callbacks

    @property
    def epochs(self) -> int:
        return self.learner.epochs

    # ------------------------------------------------------------------ delegation
    def set_addr(self, addr: str) -> None:
        self.learner.set_addr(addr)
        self.addr = addr

    def set_model(self, model: Union[P2PFLModel, List[np.ndarray], bytes]) -> None:
        self.learner.set_model(model)

    def get_model(self) -> P2PFLModel:
        return self.learner.get_model()

    def set_data(self, data: Any) -> None:
        self.learner.set_data(data)

    def get_data(self) -> Any:
        return self.learner.get_data()

    def set_epochs(self, epochs: int) -> None:
        self.learner.set_epochs(epochs)

    def update_callbacks_with_model_info(self) -> None:
        self.learner.update_callbacks_with_model_info()

    def add_callback_info_to_model(self) -> None:
        self.learner.add_callback_info_to_model()

    def get_framework(self) -> str:
        return self.learner.get_framework()

    # ------------------------------------------------------------------ pool jobs
    def fit(self) -> P2PFLModel:
        try:
            self.actor_pool.submit_learner_job(lambda actor, addr, learner: actor.fit(addr, learner), (str(self.addr), self.learner))
            model: P2PFLModel = self.actor_pool.get_learner_result(str(self.addr), None)[1]
        except Exception as ex:
            logger.error(str(self.addr), f"An error occurred during pooled fit: {ex}")
            raise
        if model is not self.learner.get_model():  # the job trained in place; only foreign results are copied in
            self.learner.set_model(model)
        return model

    def interrupt_fit(self) -> None:
        self.learner.interrupt_fit()

    def evaluate(self) -> Dict[str, float]:
        try:
            self.actor_pool.submit_learner_job(lambda actor, addr, learner: actor.evaluate(addr, learner), (str(self.addr), self.learner))
            return self.actor_pool.get_learner_result(str(self.addr), None)[1]
        except Exception as ex:
            logger.error(str(self.addr), f"An error occurred during pooled evaluation: {ex}")
            raise
