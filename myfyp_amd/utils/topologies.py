"""Topologies (parity: ``p2pfl/utils/topologies.py:30-93``).

Adjacency matrices for STAR/FULL/LINE/RING (+ GRID and RANDOM here), used both to wire gossip
connections and, on the collective plane, to define neighbour averaging over xGMI.
"""

from __future__ import annotations

import time
from enum import Enum
from typing import List, Sequence

import numpy as np


class TopologyType(Enum):
    STAR = "star"
    FULL = "full"
    LINE = "line"
    RING = "ring"
    GRID = "grid"
    RANDOM = "random"


class TopologyFactory:
    """Builds adjacency matrices and connects nodes accordingly."""

    @staticmethod
    def generate_matrix(topology_type: TopologyType, num_nodes: int, p: float = 0.5, seed: int = 0) -> np.ndarray:
        t = TopologyType(topology_type)
        m = np.zeros((num_nodes, num_nodes), dtype=int)
        if t == TopologyType.STAR:
            m[0, 1:] = 1
            m[1:, 0] = 1
        elif t == TopologyType.FULL:
            m = np.ones((num_nodes, num_nodes), dtype=int) - np.eye(num_nodes, dtype=int)
        elif t == TopologyType.LINE:
            for i in range(num_nodes - 1):
                m[i, i + 1] = m[i + 1, i] = 1
        elif t == TopologyType.RING:
            for i in range(num_nodes - 1):
                m[i, i + 1] = m[i + 1, i] = 1
            if num_nodes > 2:
                m[0, num_nodes - 1] = m[num_nodes - 1, 0] = 1
        elif t == TopologyType.GRID:
            side = int(np.ceil(np.sqrt(num_nodes)))
            for i in range(num_nodes):
                r, c = divmod(i, side)
                for j in (i + 1, i + side):
                    if j < num_nodes and (j == i + side or divmod(j, side)[0] == r):
                        m[i, j] = m[j, i] = 1
        elif t == TopologyType.RANDOM:
            rng = np.random.default_rng(seed)
            upper = np.triu((rng.random((num_nodes, num_nodes)) < p).astype(int), 1)
            m = upper + upper.T
            for i in range(num_nodes - 1):  # keep it connected
                m[i, i + 1] = m[i + 1, i] = 1
        return m

    @staticmethod
    def connect_nodes(adjacency_matrix: np.ndarray, nodes: Sequence, delay: float = 0.0) -> None:
        """Connect node i → j for each edge of the upper triangle (reference sleeps 0.1 s per edge)."""
        n = len(nodes)
        for i in range(n):
            for j in range(i + 1, n):
                if adjacency_matrix[i, j] == 1:
                    nodes[i].connect(nodes[j].addr)
                    if delay:
                        time.sleep(delay)

    @staticmethod
    def neighbors(adjacency_matrix: np.ndarray, i: int) -> List[int]:
        return [int(j) for j in np.nonzero(adjacency_matrix[i])[0]]
