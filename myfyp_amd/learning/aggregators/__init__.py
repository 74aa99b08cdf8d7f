"""Aggregators: FedAvg, FedMedian, SCAFFOLD, FedProx, robust (Krum, trimmed mean), decentralised NeighborAvg."""

from myfyp_amd.learning.aggregators.aggregator import Aggregator, NoModelsToAggregateError
from myfyp_amd.learning.aggregators.fedavg import FedAvg
from myfyp_amd.learning.aggregators.fedmedian import FedMedian
from myfyp_amd.learning.aggregators.fedprox import FedProx
from myfyp_amd.learning.aggregators.krum import Krum
from myfyp_amd.learning.aggregators.neighbor_avg import NeighborAvg
from myfyp_amd.learning.aggregators.scaffold import Scaffold
from myfyp_amd.learning.aggregators.trimmed_mean import TrimmedMean

__all__ = ["Aggregator", "NoModelsToAggregateError", "FedAvg", "FedMedian", "FedProx", "Krum", "NeighborAvg", "Scaffold", "TrimmedMean"]
