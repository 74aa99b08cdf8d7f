"""Callback registry (parity: ``frameworks/callback_factory.py:32-101``)."""

from __future__ import annotations

from typing import Callable, Dict, List

from myfyp_amd.learning.frameworks.callback import P2PFLCallback


class CallbackFactory:
    """``(framework, name) → callback class`` registry."""

    _registry: Dict[str, Dict[str, Callable[[], P2PFLCallback]]] = {}

    @classmethod
    def register_callback(cls, learner: str, callback: Callable[[], P2PFLCallback]) -> None:
        cls._registry.setdefault(learner, {})[callback.get_name()] = callback  # type: ignore[attr-defined]

    @classmethod
    def create_callbacks(cls, framework: str, aggregator) -> List[P2PFLCallback]:
        required = aggregator.get_required_callbacks()
        _ensure_builtin_callbacks()
        out: List[P2PFLCallback] = []
        for name in required:
            cb = cls._registry.get(framework, {}).get(name)
            if cb is None:
                raise ValueError(f"No callback {name!r} registered for framework {framework!r}")
            out.append(cb())
        return out


def _ensure_builtin_callbacks() -> None:
    # imported lazily to avoid import cycles; registration happens at import time
    import myfyp_amd.learning.frameworks.torch.callbacks  # noqa: F401
