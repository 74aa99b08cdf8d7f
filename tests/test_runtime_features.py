"""Checkpoint/resume, Byzantine attacks, fault injection (dropout), YAML runner and CLI (CPU)."""

import os
import time

import numpy as np
import pytest

from _ports import free_port
import torch

from myfyp_amd import fault_injection
from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
from myfyp_amd.learning.aggregators.fedavg import FedAvg
from myfyp_amd.learning.aggregators.scaffold import Scaffold
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.management import checkpoint as ckpt
from myfyp_amd.management.logger import logger
from myfyp_amd.models import MLP
from myfyp_amd.node import Node
from myfyp_amd.parallel.federation import Federation
from myfyp_amd.settings import Settings
from myfyp_amd.utils.utils import check_equal_models, wait_to_finish


@pytest.fixture(scope="module")
def data():
    return synthetic_mnist(4000, 800, seed=11, similarity=0.3)


def _collective_nodes(parts, n, exp, aggregator=FedAvg):
    Federation.reset()
    fed = Federation.init()
    nodes = [Node(TorchModel(MLP(seed=i)), parts[i], address=f"{exp}-{i}", aggregator=aggregator(), protocol=CollectiveCommunicationProtocol, exp_name=exp) for i in range(n)]
    for nd in nodes:
        nd.start()
    fed.finalize()
    return nodes


def _stop(nodes):
    for nd in nodes:
        nd.stop()
    Federation.reset()


# ------------------------------------------------------------------------------------------ checkpoint
def test_checkpoint_roundtrip_is_wire_format(tmp_path, data):
    nd = Node(TorchModel(MLP(seed=3)), data, address=f"ck-{time.time_ns()}")
    path = ckpt.save_checkpoint(nd.learner, str(tmp_path), "exp", nd.addr, round=2, total_rounds=5, epochs=1)
    assert os.path.exists(path) and ckpt.latest_checkpoint(str(tmp_path), "exp", nd.addr) == path
    params, info, meta = ckpt.load_checkpoint(path)
    assert meta["round"] == 2 and meta["total_rounds"] == 5 and meta["format"] == "p2pfl-pickle-v1"
    # the .bin is exactly a P2PFL weights message
    with open(path, "rb") as f:
        dec, _ = P2PFLModel(None).decode_parameters(f.read())
    for a, b in zip(dec, nd.learner.get_model().get_parameters()):
        np.testing.assert_array_equal(a, b)
    other = Node(TorchModel(MLP(seed=4)), data, address=f"ck2-{time.time_ns()}")
    ckpt.restore_node(other, path, restore_rng=True)
    for a, b in zip(other.learner.get_model().get_parameters(), params):
        np.testing.assert_array_equal(a, b)


def test_checkpoint_rejects_code(tmp_path):
    import pickle

    p = tmp_path / "evil.bin"
    p.write_bytes(pickle.dumps({"params": [], "additional_info": {"x": os.system}}))
    with pytest.raises(Exception):
        ckpt.load_checkpoint(str(p))


def test_scaffold_state_in_checkpoint(tmp_path, data):
    Settings.BATCH_SIZE = 32
    nd = Node(TorchModel(MLP(seed=1)), data, address=f"sc-{time.time_ns()}", aggregator=Scaffold())
    nd.learner.set_epochs(1)
    nd.learner.fit()
    cb = [c for c in nd.learner.callbacks if c.get_name() == "scaffold"][0]
    path = ckpt.save_checkpoint(nd.learner, str(tmp_path), "e", nd.addr, 1)
    nd2 = Node(TorchModel(MLP(seed=2)), data, address=f"sc2-{time.time_ns()}", aggregator=Scaffold())
    ckpt.restore_node(nd2, path)
    cb2 = [c for c in nd2.learner.callbacks if c.get_name() == "scaffold"][0]
    torch.testing.assert_close(cb2.c_i, cb.c_i.cpu())


def test_auto_checkpoint_and_resume(tmp_path, data):
    Settings.BATCH_SIZE = 32
    Settings.TRAIN_SET_SIZE = 4
    Settings.CHECKPOINT_DIR = str(tmp_path)
    n = 3
    parts = data.generate_partitions(n, RandomIIDPartitionStrategy)
    exp = f"resume-{time.time_ns()}"
    nodes = _collective_nodes(parts, n, exp)
    try:
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_to_finish(nodes, timeout=120)
        final = [p.copy() for p in nodes[0].learner.get_model().get_parameters()]
    finally:
        _stop(nodes)
    for r in (1, 2):
        assert os.path.exists(os.path.join(ckpt.node_dir(str(tmp_path), exp, f"{exp}-0"), f"round_{r}.bin"))
    # resume: fresh nodes (different init), restore round 2, run to round 3
    Settings.CHECKPOINT_DIR = None
    nodes = _collective_nodes(parts, n, exp)
    try:
        metas = [ckpt.restore_node(nd, directory=str(tmp_path), exp_name=exp) for nd in nodes]
        assert {m["round"] for m in metas} == {2}
        for a, b in zip(nodes[0].learner.get_model().get_parameters(), final):
            np.testing.assert_array_equal(a, b)
        nodes[0].set_start_learning(rounds=3, epochs=1, start_round=2)
        wait_to_finish(nodes, timeout=120)
        hist = nodes[0].learning_workflow.history
        assert hist.count("VoteTrainSetStage") == 1  # exactly one more round
        logs = logger.get_global_logs()[exp][nodes[0].addr]["test_metric"]
        assert max(r for r, _ in logs) == 3
        check_equal_models(nodes, atol=1e-5)
    finally:
        _stop(nodes)
        Settings.CHECKPOINT_DIR = None


# ------------------------------------------------------------------------------------------ attacks
def test_sign_flip_and_noise(data):
    nd = Node(TorchModel(MLP(seed=5)), data, address=f"att-{time.time_ns()}")
    before = [p.copy() for p in nd.learner.get_model().get_parameters()]
    fault_injection.sign_flip(nd)
    for a, b in zip(nd.learner.get_model().get_parameters(), before):
        np.testing.assert_allclose(a, -b)
    fault_injection.sign_flip(nd)
    fault_injection.gaussian_noise(nd, sigma=0.1, seed=3)
    diff = np.concatenate([(a - b).ravel() for a, b in zip(nd.learner.get_model().get_parameters(), before)])
    assert abs(diff.std() - 0.1) < 0.01 and abs(diff.mean()) < 0.01


def test_persistent_poisoning(data):
    Settings.BATCH_SIZE = 64
    nd = Node(TorchModel(MLP(seed=5)), data, address=f"poi-{time.time_ns()}")
    nd.learner.set_epochs(1)
    poison = fault_injection.ModelPoisoning(nd, "scale", factor=0.0)
    nd.learner.fit()
    assert all(np.all(p == 0) for p in nd.learner.get_model().get_parameters())
    poison.remove()
    assert poison.count == 1


# ------------------------------------------------------------------------------------------ dropout
def test_collective_peer_dropout(data):
    Settings.BATCH_SIZE = 32
    Settings.TRAIN_SET_SIZE = 4
    n = 4
    parts = data.generate_partitions(n, RandomIIDPartitionStrategy)
    exp = f"drop-{time.time_ns()}"
    nodes = _collective_nodes(parts, n, exp)
    try:
        fault = fault_injection.kill_at(nodes[2], "TrainStage", round=1)
        t0 = time.time()
        nodes[0].set_start_learning(rounds=3, epochs=1)
        wait_to_finish(nodes, timeout=120)
        assert time.time() - t0 < 60  # survivors did not wait for an aggregation timeout
        assert fault.fired.is_set()
        survivors = [nodes[i] for i in (0, 1, 3)]
        for nd in survivors:
            assert nd.learning_workflow.history.count("RoundFinishedStage") == 3
        check_equal_models(survivors, atol=1e-5)
        logs = logger.get_global_logs()[exp]
        assert max(v for _, v in logs[nodes[0].addr]["test_metric"]) > 0.5
    finally:
        _stop(nodes)


def test_gossip_peer_dropout(data):
    Settings.BATCH_SIZE = 32
    Settings.TRAIN_SET_SIZE = 3
    Settings.AGGREGATION_TIMEOUT = 4
    Settings.VOTE_TIMEOUT = 6
    n = 3
    parts = data.generate_partitions(n, RandomIIDPartitionStrategy)
    exp = f"gdrop-{time.time_ns()}"
    nodes = [Node(TorchModel(MLP(seed=1)), parts[i], address=f"{exp}-{i}", exp_name=exp) for i in range(n)]
    for nd in nodes:
        nd.start()
    try:
        for i in range(n):
            for j in range(i + 1, n):
                nodes[i].connect(nodes[j].addr)
        time.sleep(0.5)
        fault_injection.kill_at(nodes[2], "TrainStage", round=1)
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_to_finish(nodes[:2], timeout=90)
        for nd in nodes[:2]:
            assert nd.learning_workflow.history.count("RoundFinishedStage") == 2
        check_equal_models(nodes[:2])
    finally:
        for nd in nodes:
            nd.stop()


# ------------------------------------------------------------------------------------------ runner / CLI
@pytest.mark.parametrize("devices", [None, 3], ids=["one-device", "mesh3"])
def test_yaml_runner(tmp_path, devices):
    """``devices: N`` runs the experiment on an N-device mesh in one process (CPU members here)."""
    import yaml

    from myfyp_amd.parallel.federation import Federation

    cfg = {
        "experiment": {
            "name": f"yaml-{time.time_ns()}",
            "rounds": 2,
            "epochs": 1,
            "seed": 3,
            "dataset": {"source": "synthetic", "name": "mnist", "n_train": 6000, "n_test": 900, "batch_size": 32, "similarity": 0.3},
            "model": {"name": "MLP"},
            "aggregator": {"package": "p2pfl.learning.aggregators.fedavg", "aggregator": "FedAvg"},
            "attack": {"node": 1, "kind": "gaussian_noise", "sigma": 0.05},
        },
        "network": {"protocol": "collective", "nodes": 3, **({"devices": devices} if devices else {})},
        "settings": {"training": {"TRAIN_SET_SIZE": 3}},
    }
    Federation.reset()
    p = tmp_path / "exp.yaml"
    p.write_text(yaml.safe_dump(cfg))
    from myfyp_amd.runner import run_experiment

    res = run_experiment(str(p), verbose=False)
    assert Settings.TRAIN_SET_SIZE == 3
    assert set(res["global_logs"]) == set(res["nodes"])
    for h in res["histories"].values():
        assert h.count("RoundFinishedStage") == 2
    accs = [m["test_metric"][-1][1] for m in res["global_logs"].values()]
    assert min(accs) > 0.5


def test_cli_lists_and_helps():
    from typer.testing import CliRunner

    from myfyp_amd.cli import app

    r = CliRunner().invoke(app, ["experiment", "list"])
    assert r.exit_code == 0 and "mnist" in r.output and "fyp_attack" in r.output
    r = CliRunner().invoke(app, ["experiment", "help", "mnist"])
    assert r.exit_code == 0 and "--protocol" in r.output
    r = CliRunner().invoke(app, ["experiment", "run", "does-not-exist"])
    assert r.exit_code == 1


@pytest.mark.slow
def test_yaml_runner_split_over_two_ranks():
    """run_experiment under torchrun: each rank hosts its block of peers, the attack lands on the
    owning rank only, and the metric stores are merged so every rank sees all four peers."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(root, "tests", "workers", "runner_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert res.returncode == 0, res.stderr[-3000:] + res.stdout[-2000:]
    assert res.stdout.count(" OK ") == 2, res.stdout


@pytest.mark.slow
def test_central_log_relay_two_ranks_gloo():
    """Rank 0 sees the other rank's peers' metrics while the job runs (no end-of-run merge)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(root, "tests", "workers", "central_log_worker.py")]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root)
    assert res.returncode == 0, res.stderr[-3000:]
    assert res.stdout.count("OK") == 2


def test_node_monitor_reports_comm_stats():
    """Weight-plane traffic shows up in the node monitor (bytes, rate, latency per kind)."""
    from myfyp_amd.management.node_monitor import NodeMonitor
    from myfyp_amd.parallel.federation import Federation

    Federation.reset()
    fed = Federation.init()
    try:
        mon = NodeMonitor("mon", lambda *a: None)
        fed.comm.host("all_reduce", 4_000_000, 250e-6)
        s1 = mon.sample()
        assert s1["comm_all_reduce_mb"] == pytest.approx(4.0) and s1["comm_all_reduce_us"] == pytest.approx(250.0)
        fed.comm.host("all_reduce", 6_000_000, 100e-6)
        time.sleep(0.01)
        s2 = mon.sample()
        assert s2["comm_all_reduce_mb"] == pytest.approx(10.0) and s2["comm_all_reduce_mb_s"] > 0
    finally:
        Federation.reset()


@pytest.mark.gpu
def test_device_telemetry_reads_the_gpu():
    """Power / HBM / activity of the training GPU through AMD SMI (or sysfs)."""
    from myfyp_amd.management.device_telemetry import DeviceTelemetry

    tel = DeviceTelemetry(0)
    s = tel.sample()
    print(tel.source, s)
    assert tel.source in ("amdsmi", "sysfs"), "no telemetry source on the GPU box"
    assert s.get("hbm_total_gb", 0) > 200  # MI355X: 288 GB HBM3E
    assert "gpu_power_w" in s or "gpu_busy_pct" in s
