"""Parallel runtime: flat parameter buffers, co-located peer groups (grouped fused engine),
process groups and the RCCL weights plane."""
