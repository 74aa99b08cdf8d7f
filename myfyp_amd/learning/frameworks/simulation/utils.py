"""Resource sizing for the simulation device pool.

Parity: ``p2pfl/learning/frameworks/simulation/utils.py:33-96`` (``check_client_resources``,
``pool_size_from_resources``). The reference asks Ray for each cluster node's CPU/GPU count; here
the pool lives in this process, so the inventory is this host's CPU affinity set and the GPUs
visible to it. ``num_gpus`` is a fraction of one MI355X per virtual client: 0.25 puts four pool
workers (each with its own HIP stream) on every device.
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional, Union

from myfyp_amd.management.logger import logger

Resources = Dict[str, Union[int, float]]


def host_inventory() -> Dict[str, int]:
    """CPUs usable by this process and GPUs visible to it (``device_count`` does not initialise
    the HIP runtime)."""
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover - non-Linux
        cpus = os.cpu_count() or 1
    gpus = 0
    try:
        import torch

        gpus = torch.cuda.device_count()
    except Exception:  # pragma: no cover
        gpus = 0
    return {"CPU": cpus, "GPU": gpus}


def check_client_resources(client_resources: Optional[Resources]) -> Resources:
    """Validate per-virtual-client resources; ``None`` means one CPU and no GPU, as in the
    reference. A missing ``num_cpus`` defaults to 1."""
    if client_resources is None:
        logger.info("ActorPool", "No `client_resources` specified. Using minimal resources for clients.")
        client_resources = {"num_cpus": 1, "num_gpus": 0.0}
    else:
        client_resources = dict(client_resources)
    if "num_cpus" not in client_resources:
        logger.debug("ActorPool", "No `num_cpus` in `client_resources`: using one CPU per client.")
        client_resources["num_cpus"] = 1
    if client_resources["num_cpus"] <= 0:
        raise ValueError("client_resources['num_cpus'] must be positive")
    if client_resources.get("num_gpus", 0.0) < 0:
        raise ValueError("client_resources['num_gpus'] must be >= 0")
    logger.info("ActorPool", f"Resources for each Virtual Client: {client_resources}")
    return client_resources


def pool_size_from_resources(client_resources: Resources, inventory: Optional[Dict[str, int]] = None) -> int:
    """Number of pool workers that fit on this host: CPUs / num_cpus, capped by GPUs / num_gpus
    when clients need a GPU. Raises ``ValueError`` when not even one fits (reference behaviour)."""
    inv = inventory or host_inventory()
    n = int(inv["CPU"] / client_resources["num_cpus"])
    need_gpu = float(client_resources.get("num_gpus", 0.0) or 0.0)
    if need_gpu > 0.0:
        n = min(n, int(inv["GPU"] / need_gpu + 1e-9)) if inv["GPU"] else 0
    if n <= 0:
        logger.debug(
            "ActorPool",
            f"The ActorPool is empty: CPUs={inv['CPU']}, GPUs={inv['GPU']} cannot host one client with {client_resources}.",
        )
        raise ValueError("ActorPool is empty. Stopping Simulation. Check 'client_resources'")
    return n


def pool_devices(client_resources: Resources, num_actors: int, inventory: Optional[Dict[str, int]] = None) -> List[str]:
    """Device of each pool worker: GPU clients are spread round-robin over the visible devices
    (worker i → ``cuda:i % G``) so every device gets the same number of streams; CPU clients run
    on ``cpu``."""
    inv = inventory or host_inventory()
    if float(client_resources.get("num_gpus", 0.0) or 0.0) > 0.0 and inv["GPU"] > 0:
        return [f"cuda:{i % inv['GPU']}" for i in range(num_actors)]
    return ["cpu"] * num_actors
