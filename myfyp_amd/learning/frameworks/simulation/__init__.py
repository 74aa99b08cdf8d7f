"""Simulation entry points (parity: ``p2pfl/learning/frameworks/simulation/__init__.py:16-33``).

The reference wraps every learner in a Ray ``VirtualNodeLearner`` and ships the whole pickled
learner (model + dataset) to an actor pool each round. On MI355X the equivalent
— many simulated peers sharing devices — is the grouped device engines: co-located peers of one
architecture train in a single launch sequence (``parallel/mlp_engine.py``, ``parallel/cnn_engine.py``)
and never leave the GPU. ``try_init_learner_with_ray`` is kept so reference code keeps working; it
returns the learner unchanged (Ray is not used; ``Settings.DISABLE_RAY`` is honoured).
"""

from __future__ import annotations

from myfyp_amd.management.logger import logger
from myfyp_amd.utils.check_ray import ray_installed


def try_init_learner_with_ray(learner):
    """Return ``learner``; simulated peers are batched by the grouped device engines instead."""
    if ray_installed():
        logger.debug(getattr(learner, "_self_addr", "simulation"), "Ray is installed but not used: grouped device engines batch co-located peers")
    return learner


class VirtualNodeLearner:
    """Name kept for API parity; wrapping is a no-op (see module docstring)."""

    def __new__(cls, learner, *args, **kwargs):
        return learner
