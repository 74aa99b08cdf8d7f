"""Process model of a multi-GPU run on one node, decided BEFORE anything touches a GPU.

``--gpus N`` of the benchmarks (``bench.py``, ``benchmarks/bench_cnn.py``) and ``devices: N`` of a
YAML experiment must use N GPUs whatever the launcher:

* **ranks** (default under ``torchrun``): one process per GPU, ``torch.distributed`` over RCCL
  (``parallel/federation.py``'s multi-rank plane). Every process runs the same single-device code
  as a one-GPU run, on its own ``LOCAL_RANK`` device, and the host work of a round is spread over
  the N processes (the one-process mesh stays opt-in until an N >= 2 run has pinned it to
  this path);
* **mesh** (default for ONE process started with ``--gpus N``; ``--launch mesh`` under torchrun):
  one process drives the N GPUs (in-process RCCL device mesh, ``parallel/device_mesh.py``); under
  torchrun rank 0 drives them and the other ranks only wait on a CPU (gloo) group.

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
    if world > 1 and launch == "auto":
        return "ranks"  # torchrun: one process per GPU (also the CPU gloo rehearsal)
    if world > 1 and rank != 0:
        return "park"
    have = torch.cuda.device_count()  # does not initialise the GPU on this image
    if gpus > have and not mesh_virtual:
        raise SystemExit(f"--gpus {gpus} but {have} GPU(s) visible (use --mesh-virtual for a one-device rehearsal)")
    return "mesh"


def check_mesh(fed, gpus: int, virtual: bool, who: str = "bench") -> None:
    """A physical N-GPU mesh must be the RCCL one: a run whose RCCL mesh could not form must not
    report a host-copy "mesh" as an N-GPU number."""
    if fed.mesh is None or fed.mesh_size != gpus:
        raise SystemExit(f"{who}: device mesh of {gpus} not formed (got {fed.mesh_size})")
    if not virtual and gpus > 1 and fed.mesh.kind != "rccl":
        raise SystemExit(f"{who}: --gpus {gpus} asked for a physical mesh, but it runs on the {fed.mesh.kind!r} backend (RCCL did not form)")


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
