"""Byzantine attacks and fault injection (FYP harness ``exp_SAVE3.txt``).

The FYP harness poisons one node's *initial* weights before learning starts: a sign flip
``w ← −w`` (``exp_SAVE3.txt:91-100``) or additive Gaussian noise ``w ← w + σ·N(0,1)``, σ = 0.1
(``exp_SAVE3.txt:214-223``). Here the same attacks run in place on the learner's device-resident
parameters through the ``scale_add_noise`` HIP kernel (K14) — no host round trip — and can also be
installed as *persistent* model poisoning (applied after every local fit, i.e. to every model the
node contributes).

Crash/delay faults hook the stage workflow (``StageWokflow.hooks``): ``kill_at`` stops a node when
it reaches a given stage of a given round (BASELINE config 5: 1-peer dropout), ``delay_at`` stalls
it. Survivors keep going: gossip peers evict it by heartbeat / send failure, collective gangs drop
it as soon as it unregisters (``Federation.unregister_local``).
"""

from __future__ import annotations

import os
import sys
import threading
import time
from typing import Any, Callable, Dict, List, Optional

import torch

from myfyp_amd import ops
from myfyp_amd.management.logger import logger

ATTACKS = ("sign_flip", "gaussian_noise", "scale")


def _learner(target):
    return getattr(target, "learner", target)


def _param_tensors(learner) -> List[torch.Tensor]:
    """Device tensors holding the model: flat trainable vector (+ floating buffers)."""
    out = [learner.flat_params()]
    module = learner.get_model().get_model()
    for b in module.buffers():
        if b.is_floating_point():
            out.append(b)
    return out


@torch.no_grad()
def apply_attack(target, kind: str = "sign_flip", sigma: float = 0.1, factor: float = -1.0, seed: int = 0) -> None:
    """Poison the parameters of ``target`` (a Node or a Learner) in place.

    * ``sign_flip``       — ``w ← −w``
    * ``gaussian_noise``  — ``w ← w + σ·N(0,1)`` (counter-based RNG, deterministic in ``seed``)
    * ``scale``           — ``w ← factor·w``
    """
    lr = _learner(target)
    if kind not in ATTACKS:
        raise ValueError(f"unknown attack {kind!r}; choose from {ATTACKS}")
    scale, sig = {"sign_flip": (-1.0, 0.0), "gaussian_noise": (1.0, float(sigma)), "scale": (float(factor), 0.0)}[kind]
    for i, t in enumerate(_param_tensors(lr)):
        if t.is_contiguous() and t.dtype == torch.float32:
            ops.scale_add_noise(t, scale, sig, seed=seed * 1000003 + i)
        else:
            tmp = t.detach().float().contiguous()
            ops.scale_add_noise(tmp, scale, sig, seed=seed * 1000003 + i)
            t.copy_(tmp.to(t.dtype))
    logger.info(getattr(lr, "_self_addr", "?"), f"☠️ attack applied: {kind} (σ={sig}, scale={scale})")


def sign_flip(target) -> None:
    apply_attack(target, "sign_flip")


def gaussian_noise(target, sigma: float = 0.1, seed: int = 0) -> None:
    apply_attack(target, "gaussian_noise", sigma=sigma, seed=seed)


class ModelPoisoning:
    """Persistent attack: poison the node's model after every local ``fit`` (its contributions)."""

    def __init__(self, target, kind: str = "sign_flip", sigma: float = 0.1, factor: float = -1.0, seed: int = 0) -> None:
        self.learner = _learner(target)
        self.kind, self.sigma, self.factor, self.seed = kind, sigma, factor, seed
        self._orig_fit = self.learner.fit
        self.count = 0

        def fit_then_poison():
            model = self._orig_fit()
            apply_attack(self.learner, self.kind, self.sigma, self.factor, self.seed + self.count)
            self.count += 1
            return model

        self.learner.fit = fit_then_poison  # type: ignore[method-assign]

    def remove(self) -> None:
        self.learner.fit = self._orig_fit  # type: ignore[method-assign]


class StageFault:
    """Run ``action(node)`` once when ``node`` enters ``stage`` in ``round`` (None = any round)."""

    def __init__(self, node, stage: str, action: Callable[[Any], None], round: Optional[int] = None) -> None:
        self.node, self.stage, self.round, self.action = node, stage, round, action
        self.fired = threading.Event()
        node.learning_workflow.hooks.append(self._hook)

    def _hook(self, stage_name: str, kwargs: Dict[str, Any]) -> None:
        if self.fired.is_set() or stage_name != self.stage:
            return
        if self.round is not None and self.node.state.round != self.round:
            return
        self.fired.set()
        self.action(self.node)

    def remove(self) -> None:
        try:
            self.node.learning_workflow.hooks.remove(self._hook)
        except ValueError:
            pass


class _Crash(Exception):
    """Raised inside the victim's learning thread so it ends immediately (a crash)."""

    fault_injected = True


def kill_at(node, stage: str = "TrainStage", round: Optional[int] = 1) -> StageFault:
    """Crash ``node`` when it reaches ``stage`` of ``round``: the node stops (protocol down, heartbeats
    stop, collective gangs drop it) and its learning thread ends without finishing the stage."""

    def crash(n) -> None:
        logger.warning(n.addr, f"💥 fault injection: killing node at {stage} (round {n.state.round})")
        n.stop()
        raise _Crash(f"{n.addr} killed at {stage}")

    return StageFault(node, stage, crash, round)


def crash_process_at(node, stage: str = "TrainStage", round: Optional[int] = 1, code: int = 0) -> StageFault:
    """Kill the whole PROCESS when ``node`` reaches ``stage`` of ``round`` — no shutdown, no
    departure notice, heartbeats just stop (a crashed rank). The other ranks must evict it by
    heartbeat staleness (``Settings.FAILURE_TIMEOUT``). ``code`` 0 keeps ``torchrun`` from tearing
    down the surviving workers, as a node-level crash on another host would."""

    def crash(n) -> None:
        logger.warning(n.addr, f"💥 fault injection: process crash at {stage} (round {n.state.round})")
        sys.stdout.flush()
        os._exit(code)

    return StageFault(node, stage, crash, round)


class CollectiveFault:
    """Kill the whole PROCESS right before it issues a weight collective (after the reduce of its
    local rows, after the pre-collective membership agreement) in ``round``: the other ranks are
    already inside the collective — the case the collective guard (``Federation.await_works``)
    must survive without waiting out ``COLLECTIVE_TIMEOUT``."""

    def __init__(self, fed, node, round: Optional[int] = 1, kinds=("all_reduce", "all_reduce_async"), code: int = 0) -> None:
        self.fed, self.node, self.round, self.kinds, self.code = fed, node, round, tuple(kinds), code
        self.fired = threading.Event()
        fed.pre_collective_hooks.append(self._hook)

    def _hook(self, kind: str) -> None:
        if self.fired.is_set() or kind not in self.kinds:
            return
        if self.round is not None and self.node.state.round != self.round:
            return
        self.fired.set()
        logger.warning(self.node.addr, f"💥 fault injection: process crash inside {kind} (round {self.node.state.round})")
        sys.stdout.flush()
        os._exit(self.code)

    def remove(self) -> None:
        try:
            self.fed.pre_collective_hooks.remove(self._hook)
        except ValueError:
            pass


def crash_in_collective(fed, node, round: Optional[int] = 1, code: int = 0) -> CollectiveFault:
    return CollectiveFault(fed, node, round, code=code)


def delay_at(node, stage: str, seconds: float, round: Optional[int] = None) -> StageFault:
    """Stall ``node`` for ``seconds`` before ``stage`` (straggler injection)."""
    return StageFault(node, stage, lambda n: time.sleep(seconds), round)
