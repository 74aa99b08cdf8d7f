"""Aggregation math (reference: test/learning/aggregator_test.py, scaffold_test.py)."""

import threading

import numpy as np
import pytest
import torch

from myfyp_amd.learning.aggregators import FedAvg, FedMedian, FedProx, Krum, NoModelsToAggregateError, Scaffold, TrimmedMean
from myfyp_amd.learning.frameworks.p2pfl_model import NumpyModel


def M(params, n=1, contributors=("a",), info=None):
    return NumpyModel(None, params=[np.asarray(p, dtype=np.float64) for p in params], num_samples=n, contributors=list(contributors), additional_info=info)


def test_fedavg_simple():
    agg = FedAvg()
    out = agg.aggregate([M([[1, 2, 3]], 1, ["a"]), M([[4, 5, 6]], 1, ["b"]), M([[7, 8, 9]], 1, ["c"])])
    assert np.allclose(out.get_parameters()[0], [4, 5, 6])
    assert sorted(out.get_contributors()) == ["a", "b", "c"] and out.get_num_samples() == 3


def test_fedavg_weighted_and_torch_tensors():
    agg = FedAvg()
    out = agg.aggregate([M([[0.0], [[1.0, 1.0]]], 1, ["a"]), M([[4.0], [[3.0, 3.0]]], 3, ["b"])])
    assert np.allclose(out.get_parameters()[0], [3.0]) and np.allclose(out.get_parameters()[1], [[2.5, 2.5]])
    from myfyp_amd.learning.aggregators._math import weighted_mean

    res = weighted_mean([[torch.ones(3)], [torch.zeros(3)]], [1, 3])
    assert torch.allclose(res[0], torch.full((3,), 0.25))


def test_fedavg_complex_perturbation():
    rng = np.random.default_rng(0)
    base = [rng.normal(size=(20, 10)), rng.normal(size=10)]
    models = [M([b + 1 for b in base], 1, ["a"]), M([b - 1 for b in base], 1, ["b"])]
    out = FedAvg().aggregate(models)
    for o, b in zip(out.get_parameters(), base):
        assert np.allclose(o, b)


def test_aggregator_lifecycle_and_partial():
    agg = FedAvg(node_name="n0")
    agg.set_nodes_to_aggregate(["a", "b", "c"])
    with pytest.raises(Exception):
        agg.set_nodes_to_aggregate(["a"])  # running
    assert agg.add_model(M([[1.0]], 1, ["a"])) == ["a"]
    assert agg.add_model(M([[1.0]], 1, ["a"])) == []  # duplicate contributor
    assert agg.add_model(M([[1.0]], 1, ["z"])) == []  # not in train set
    assert agg.get_missing_models() == {"b", "c"}
    partial = agg.get_model(except_nodes=["b"])
    assert partial.get_contributors() == ["a"]
    assert sorted(agg.add_model(M([[3.0]], 1, ["b", "c"]))) == ["a", "b", "c"]
    out = agg.wait_and_get_aggregation(timeout=1)
    assert np.allclose(out.get_parameters()[0], [2.0])
    agg.clear()
    agg.set_nodes_to_aggregate(["x"])
    t0 = threading.Event()
    out = None
    with pytest.raises(NoModelsToAggregateError):
        agg.wait_and_get_aggregation(timeout=0.05)  # timeout + nothing arrived


def test_fedmedian_and_trimmed_mean():
    ms = [M([[v, -v]], 1, [c]) for v, c in zip([1.0, 2.0, 100.0, 3.0, 4.0], "abcde")]
    assert np.allclose(FedMedian().aggregate(ms).get_parameters()[0], [3.0, -3.0])
    assert np.allclose(TrimmedMean(beta=0.2).aggregate(ms).get_parameters()[0], [3.0, -3.0])
    even = ms[:4]
    assert np.allclose(FedMedian().aggregate(even).get_parameters()[0], [2.5, -2.5])


def test_krum_rejects_outlier():
    good = [M([[1.0 + 0.01 * i, 1.0]], 1, [f"g{i}"]) for i in range(4)]
    bad = M([[100.0, -100.0]], 1, ["bad"])
    out = Krum(num_byzantine=1).aggregate(good + [bad])
    assert abs(out.get_parameters()[0][0] - 1.0) < 0.1


def test_scaffold_server_math():
    aggr = Scaffold(node_name="n", global_lr=0.1)
    aggr.global_model_params = [np.zeros(2), np.zeros(2)]
    aggr.c = [np.zeros(2), np.zeros(2)]
    m1 = M([[1.0, 1.0], [1.0, 1.0]], 10, ["c1"], {"scaffold": {"delta_y_i": [np.ones(2), np.ones(2)], "delta_c_i": [np.ones(2), np.ones(2)]}})
    m2 = M([[2.0, 2.0], [2.0, 2.0]], 20, ["c2"], {"scaffold": {"delta_y_i": [2 * np.ones(2)] * 2, "delta_c_i": [2 * np.ones(2)] * 2}})
    out = aggr.aggregate([m1, m2])
    assert np.allclose(out.get_parameters()[0], 0.1 * (10 + 40) / 30)
    assert np.allclose(out.get_info("scaffold")["global_c"][0], 1.5)
    with pytest.raises(NoModelsToAggregateError):
        aggr.aggregate([])
    with pytest.raises(ValueError):
        aggr.aggregate([M([[1.0]], 1, ["x"], {"scaffold": {"delta_y_i": [np.ones(1)]}})])
    fresh = Scaffold(global_lr=1.0)
    out2 = fresh.aggregate([M([[3.0]], 1, ["a"], {"scaffold": {"delta_y_i": [np.ones(1)], "delta_c_i": [np.zeros(1)]}})])
    assert np.allclose(out2.get_parameters()[0], [3.0])  # x = y - dy = 2, + 1.0 * dy = 3


def test_fedprox_ships_mu():
    out = FedProx(proximal_mu=0.3).aggregate([M([[1.0]], 1, ["a"])])
    assert out.get_info("fedprox") == {"mu": 0.3}
    assert FedProx().get_required_callbacks() == ["fedprox"]
