"""Simulation entry points (parity: ``p2pfl/learning/frameworks/simulation/__init__.py:16-33``).

The reference wraps every learner in a Ray ``VirtualNodeLearner`` whenever Ray is importable and
ships the whole pickled learner (model + dataset) to an actor pool each round.
Here two MI355X-native mechanisms cover the same ground:

* grouped device engines (default): co-located peers of one architecture train in a single launch
  sequence (``parallel/mlp_engine.py``, ``parallel/cnn_engine.py``) and never leave HBM;
* the device pool (``Settings.SIMULATION_POOL = True``): every peer is pinned to one GPU of this
  process (``SuperActorPool.place``) and its fit/evaluate run as jobs on per-device worker streams,
  at most ``pool size`` at once — the reference's resource-bounded actor pool, without processes
  or serialisation (``actor_pool.py``, ``virtual_learner.py``).
"""

from __future__ import annotations

import inspect
from typing import Any, Optional

from myfyp_amd.learning.frameworks.simulation.actor_pool import ActorDiedError, SuperActorPool, VirtualLearnerActor
from myfyp_amd.learning.frameworks.simulation.utils import check_client_resources, pool_size_from_resources
from myfyp_amd.learning.frameworks.simulation.virtual_learner import VirtualNodeLearner
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings
from myfyp_amd.utils.check_ray import ray_installed

__all__ = [
    "ActorDiedError",
    "SuperActorPool",
    "VirtualLearnerActor",
    "VirtualNodeLearner",
    "check_client_resources",
    "pool_enabled",
    "pool_size_from_resources",
    "simulation_pool",
    "try_init_learner_with_ray",
]


def pool_enabled() -> bool:
    return bool(Settings.SIMULATION_POOL) or ray_installed()


def simulation_pool() -> SuperActorPool:
    """The process-wide pool, sized from ``Settings.SIMULATION_RESOURCES`` or, when GPUs are
    visible, ``SIMULATION_WORKERS_PER_GPU`` streams per device."""
    if SuperActorPool._instance is not None and getattr(SuperActorPool._instance, "initialized", False):
        return SuperActorPool._instance
    res = Settings.SIMULATION_RESOURCES
    if res is None:
        from myfyp_amd.learning.frameworks.simulation.utils import host_inventory

        if host_inventory()["GPU"] > 0:
            res = {"num_cpus": 1, "num_gpus": 1.0 / max(1, int(Settings.SIMULATION_WORKERS_PER_GPU))}
    return SuperActorPool(res)


def _accepts_device(cls: Any) -> bool:
    try:
        return "device" in inspect.signature(cls).parameters
    except (TypeError, ValueError):
        return False


def try_init_learner_with_ray(learner: Any, model: Any = None, data: Any = None, addr: Optional[str] = None, aggregator: Any = None, **learner_kwargs: Any) -> Any:
    """Build the node's learner (``learner`` may be a class or an instance) and, when the device
    pool is enabled, pin it to a pool device and wrap it in :class:`VirtualNodeLearner`.
    With the pool disabled the learner is returned unwrapped."""
    enabled = pool_enabled()
    if isinstance(learner, type):
        kwargs = dict(learner_kwargs)
        if enabled and addr is not None and "device" not in kwargs and _accepts_device(learner):
            kwargs["device"] = simulation_pool().place(addr)
        inst = learner(model, data, addr if addr is not None else "unknown-node", aggregator, **kwargs)
    else:
        inst = learner
    if not enabled:
        return inst
    name = addr if addr is not None else getattr(inst, "_self_addr", "unknown-node")
    logger.debug(name, f"Learner runs on the simulation device pool ({getattr(inst, 'device', 'cpu')})")
    return VirtualNodeLearner(inst, name, pool=simulation_pool())
