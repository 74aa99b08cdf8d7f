"""MI355X collective (RCCL/xGMI) stages: same names and transitions as base_node."""
