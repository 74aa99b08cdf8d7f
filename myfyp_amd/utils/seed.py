"""Seeding (the FYP scripts import ``p2pfl.utils.seed``, ``mlp_pytorch.txt:29``)."""

import os
import random

import numpy as np


_GENERATION = 0


def seed_generation() -> int:
    """Bumped by every :func:`set_seed`: state drawn from the RNG ahead of time (the fused MLP
    engine's next-epoch shuffle key) is dropped when it changes."""
    return _GENERATION


def set_seed(seed: int = 666, deterministic: bool = False) -> None:
    """Seed python, numpy and torch (CPU + every GPU); also ``Settings.SEED`` for vote RNGs."""
    global _GENERATION
    from myfyp_amd.settings import Settings

    _GENERATION += 1
    Settings.SEED = seed
    random.seed(seed)
    np.random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    try:
        import torch

        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(seed)
        if deterministic:
            torch.use_deterministic_algorithms(True, warn_only=True)
    except Exception:  # pragma: no cover
        pass
