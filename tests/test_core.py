"""Settings, experiment/state, logger + metric storage (reference: settings.py, node_state.py,
management/metric_storage.py, management/logger/logger.py)."""

import numpy as np
import pytest

from myfyp_amd.experiment import Experiment
from myfyp_amd.management.logger import logger
from myfyp_amd.management.metric_storage import GlobalMetricStorage, LocalMetricStorage
from myfyp_amd.node_state import NodeState
from myfyp_amd.settings import Settings


def test_settings_flat_and_nested_aliases(tmp_path):
    Settings.general.SEED = 42
    assert Settings.SEED == 42
    Settings.HEARTBEAT_PERIOD = 3
    assert Settings.heartbeat.PERIOD == 3
    with pytest.raises(AttributeError):
        Settings.general.NOPE = 1
    Settings.update({"TRAIN_SET_SIZE": 7, "gossip": {"TTL": 3}})
    assert Settings.TRAIN_SET_SIZE == 7 and Settings.TTL == 3
    cfg = tmp_path / "exp.yaml"
    cfg.write_text("settings:\n  VOTE_TIMEOUT: 12\n  training:\n    BATCH_SIZE: 16\nexperiment:\n  rounds: 2\n")
    doc = Settings.from_yaml(str(cfg))
    assert Settings.VOTE_TIMEOUT == 12 and Settings.BATCH_SIZE == 16 and doc["experiment"]["rounds"] == 2
    assert "HEARTBEAT_TIMEOUT" in Settings.snapshot()


def test_experiment_and_state():
    e = Experiment("exp", 3)
    assert e.round == 0
    e.increase_round()
    assert e.round == 1 and e.self("total_rounds") == 3
    st = NodeState("a")
    assert st.round is None and st.model_initialized_lock.locked()
    st.set_experiment("x", 2)
    st.models_aggregated["b"] = ["b"]
    st.increase_round()
    assert st.round == 1 and st.models_aggregated == {}
    st.clear()
    assert st.round is None and st.addr == "a"


def test_metric_storage_shapes():
    loc = LocalMetricStorage()
    loc.add_log("e", 0, "loss", "n1", 1.0, 1)
    loc.add_log("e", 0, "loss", "n1", 0.5, 2)
    assert loc.get_experiment_round_node_logs("e", 0, "n1") == {"loss": [(1, 1.0), (2, 0.5)]}
    glob = GlobalMetricStorage()
    glob.add_log("e", 0, "acc", "n1", 0.1)
    glob.add_log("e", 0, "acc", "n1", 0.9)  # same round: first value kept
    glob.add_log("e", 1, "acc", "n1", 0.5)
    assert glob.get_experiment_node_logs("e", "n1") == {"acc": [(0, 0.1), (1, 0.5)]}


def test_logger_metrics_require_registration():
    addr = "logger-test-node"
    logger.log_metric(addr, "m", 1.0)  # not registered: silently dropped
    logger.register_node(addr, True)
    try:
        logger.log_metric(addr, "m", 1.0)  # no experiment yet: dropped
        exp = Experiment("logger-exp", 2)
        logger.experiment_started(addr, exp)
        logger.log_metric(addr, "acc", 0.5)
        logger.log_metric(addr, "loss", 2.0, step=3)
        assert logger.get_global_logs()["logger-exp"][addr]["acc"] == [(0, 0.5)]
        assert logger.get_local_logs()["logger-exp"][0][addr]["loss"] == [(3, 2.0)]
        with pytest.raises(Exception):
            logger.register_node(addr, True)
        events = []
        hook = lambda ev, node, ex: events.append(ev)  # noqa: E731
        logger.add_round_hook(hook)
        logger.round_started(addr, exp)
        logger.round_finished(addr)
        logger.remove_round_hook(hook)
        assert events == ["round_started", "round_finished"]
    finally:
        logger.unregister_node(addr)
