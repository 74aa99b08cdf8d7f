"""Process model of a multi-GPU run on one node, decided BEFORE anything touches a GPU.

``--gpus N`` of the benchmarks (``bench.py``, ``benchmarks/bench_cnn.py``) and ``devices: N`` of a
YAML experiment must use N GPUs whatever the launcher:

* **mesh** (default): ONE process drives the N GPUs (in-process RCCL device mesh,
  ``parallel/device_mesh.py``) — started directly (``python bench.py --gpus 8``) or as rank 0 of a
  ``torchrun --nproc-per-node N`` job, whose other ranks only wait for rank 0 on a CPU (gloo) group;
* **ranks**: one process per GPU under ``torchrun`` (``parallel/federation.py``'s multi-rank plane).

A run that cannot form the N-GPU federation it was asked for exits non-zero: it never reports a
one-GPU number as an N-GPU one.
"""

from __future__ import annotations

import datetime
import os
from typing import Tuple


def env_world() -> Tuple[int, int]:
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))


def plan_launch(gpus: int, launch: str = "auto", mesh_virtual: bool = False) -> str:
    """"single" (one GPU), "mesh" (this process drives ``gpus`` devices), "park" (a torchrun rank
    other than 0 in mesh mode) or "ranks" (one process per GPU)."""
    import torch

    world, rank = env_world()
    if launch == "ranks":
        if gpus != world:
            raise SystemExit(f"--launch ranks needs one process per GPU: --gpus {gpus} but WORLD_SIZE={world}")
        return "ranks" if world > 1 else "single"
    if world > 1 and gpus != world:
        raise SystemExit(f"launched with {world} ranks but --gpus {gpus}")
    if gpus <= 1:
        return "single"
    if world > 1 and launch == "auto" and torch.cuda.device_count() == 0:
        return "ranks"  # CPU host under torchrun (gloo rehearsal): one process per rank
    if world > 1 and rank != 0:
        return "park"
    have = torch.cuda.device_count()  # does not initialise the GPU on this image
    if gpus > have and not mesh_virtual:
        raise SystemExit(f"--gpus {gpus} but {have} GPU(s) visible (use --mesh-virtual for a one-device rehearsal)")
    return "mesh"


def cpu_group() -> None:
    """Join the torchrun job's CPU-only (gloo) group (mesh mode: rank 0 and the waiting ranks)."""
    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group("gloo", timeout=datetime.timedelta(hours=2))


def park() -> None:
    """torchrun rank > 0 in mesh mode: rank 0 drives every GPU; wait for it, then leave."""
    import torch.distributed as dist

    cpu_group()
    dist.barrier()
    dist.destroy_process_group()


def release_parked() -> None:
    """Rank 0 of a mesh-mode torchrun job, at the end: let the waiting ranks go."""
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
