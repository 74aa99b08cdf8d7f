"""Seeding (the FYP scripts import ``p2pfl.utils.seed``, ``mlp_pytorch.txt:29``)."""

import os
import random

import numpy as np


def set_seed(seed: int = 666, deterministic: bool = False) -> None:
    """Seed python, numpy and torch (CPU + every GPU); also ``Settings.SEED`` for vote RNGs."""
    from myfyp_amd.settings import Settings

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
