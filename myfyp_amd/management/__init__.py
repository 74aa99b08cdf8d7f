"""Observability: logger, metric storage, resource monitor, web dashboard client."""
