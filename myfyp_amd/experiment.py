"""Experiment descriptor (parity: ``p2pfl/experiment.py:21-74``)."""

from typing import Any, Optional


class Experiment:
    """Name, total rounds and current round of a running experiment."""

    def __init__(self, exp_name: str, total_rounds: int) -> None:
        self.exp_name = exp_name
        self.total_rounds = total_rounds
        self.round: Optional[int] = 0

    def increase_round(self) -> None:
        """Advance to the next round."""
        if self.round is None:
            raise ValueError("Round not initialized")
        self.round += 1

    def self(self, param_name: str, param_val: Any = None) -> Any:
        """Generic getter/setter kept for API parity (``p2pfl/experiment.py:55-70``)."""
        if param_val is None:
            return getattr(self, param_name)
        setattr(self, param_name, param_val)
        return param_val

    def __str__(self) -> str:
        return f"Experiment(exp_name={self.exp_name}, total_rounds={self.total_rounds}, round={self.round})"
