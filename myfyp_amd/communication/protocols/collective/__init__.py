"""RCCL/xGMI collective data plane protocol."""
