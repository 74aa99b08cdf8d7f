"""Datasets: ``P2PFLDataset`` wrapper, partition strategies, synthetic generators."""
