"""myfyp_amd — an MI355X-native decentralized federated-learning engine.

Capabilities of p2pfl (PrivEimantas/myFYP fork): Node/Learner API, stage workflow, gossip +
in-memory/gRPC transports, FedAvg/SCAFFOLD/FedMedian/FedProx aggregators, IID/Dirichlet data
partitioning, pickle-compatible model format — with a PyTorch-ROCm + hand-written HIP (gfx950)
compute path and an RCCL-over-xGMI weights plane.
"""

__version__ = "0.1.0"
