"""Placeholder; replaced by the grouped fused MLP engine."""


class MLPEngineHandle:
    @staticmethod
    def supports(module) -> bool:
        return False
