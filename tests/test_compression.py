"""Wire compression of model payloads (``myfyp_amd/learning/compression.py``): the FYP's
``model_build_fn(..., compression=)`` (``/root/reference/mlp_pytorch.txt:148-151``). The reference
tree ships no implementation, so the encoding is ours (parity unpinned); what is pinned is that the
uncompressed format is the reference's, every technique round-trips within its stated error, the
restricted unpickler decodes every payload, and compressed peers federate."""

import pickle

import numpy as np
import pytest
import torch

from myfyp_amd.learning import compression as comp
from myfyp_amd.learning.frameworks.p2pfl_model import safe_loads
from myfyp_amd.learning.frameworks.torch import TorchModel
from myfyp_amd.models import MLP


def _params(seed=0):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal((64, 32)).astype(np.float32), rng.standard_normal(32).astype(np.float32), np.arange(5, dtype=np.int64)]


def test_uncompressed_is_reference_format():
    ps = _params()
    data = comp.encode(ps, {"a": 1}, None)
    loaded = pickle.loads(data)
    assert set(loaded) == {"params", "additional_info"}
    out, info = comp.decode(data, safe_loads)
    assert info == {"a": 1} and all(np.array_equal(a, b) for a, b in zip(ps, out))


def test_zlib_is_lossless_and_smaller_on_redundant_data():
    ps = [np.zeros((256, 256), np.float32), np.ones(100, np.float32), np.arange(4, dtype=np.int32)]
    data = comp.encode(ps, {}, comp.validate({"zlib": {"level": 9}}))
    assert data.startswith(comp.MAGIC)
    assert len(data) < len(comp.encode(ps, {}, None)) / 20
    out, _ = comp.decode(data, safe_loads)
    assert all(np.array_equal(a, b) and a.dtype == b.dtype for a, b in zip(ps, out))


@pytest.mark.parametrize("dtype,tol", [("float16", 1e-3), ("bfloat16", 8e-3), ("int8", 1.0 / 127)])
def test_ptq_roundtrip_error(dtype, tol):
    ps = _params(1)
    data = comp.encode(ps, {}, comp.validate({"ptq": {"dtype": dtype}}))
    out, _ = comp.decode(data, safe_loads)
    for a, b in zip(ps, out):
        assert a.shape == b.shape and a.dtype == b.dtype
        if np.issubdtype(a.dtype, np.floating):
            assert np.max(np.abs(a - b)) <= tol * np.max(np.abs(a)), dtype
        else:
            assert np.array_equal(a, b)
    assert len(data) < len(comp.encode(ps, {}, None)) * (0.35 if dtype == "int8" else 0.55)  # pickle framing on small tensors


def test_topk_keeps_largest():
    ps = _params(2)
    out, _ = comp.decode(comp.encode(ps, {}, comp.validate({"topk": {"k": 0.1}})), safe_loads)
    a, b = ps[0], out[0]
    kept = b != 0
    assert kept.sum() == round(0.1 * a.size)
    assert np.array_equal(a[kept], b[kept])
    assert np.abs(a[~kept]).max() <= np.abs(a[kept]).min()


def test_combined_techniques_and_validation():
    ps = _params(3)
    c = comp.validate({"topk": {"k": 0.5}, "ptq": {"dtype": "float16"}, "zlib": {}})
    out, _ = comp.decode(comp.encode(ps, {"x": [1, 2]}, c), safe_loads)
    kept = out[0] != 0
    assert abs(kept.mean() - 0.5) < 0.01
    assert np.allclose(out[0][kept], ps[0][kept], rtol=1e-3, atol=1e-3)
    for bad in ({"gzip": {}}, {"topk": {"k": 0}}, {"ptq": {"dtype": "int4"}}, [("zlib", {})]):
        with pytest.raises(ValueError):
            comp.validate(bad)


def test_model_encode_decode_and_build_copy_keep_compression():
    m = TorchModel(MLP(seed=0), compression={"ptq": {"dtype": "bfloat16"}, "zlib": {}})
    data = m.encode_parameters()
    cp = m.build_copy(params=data, num_samples=3, contributors=["a"])
    assert cp.compression == m.compression
    for a, b in zip(m.get_parameters(), cp.get_parameters()):
        assert np.allclose(a, b, rtol=8e-3, atol=1e-6)
    plain = TorchModel(MLP(seed=0))
    assert plain.compression is None
    out, _ = plain.decode_parameters(data)  # a non-compressing peer decodes a compressed payload
    assert len(out) == len(m.get_parameters())


def test_fyp_model_build_fn_and_yaml_runner():
    from myfyp_amd.examples.mlp_pytorch import model_build_fn
    from myfyp_amd.learning.frameworks.pytorch.lightning_model import LightningModel
    from myfyp_amd.runner import build_model

    m = model_build_fn(hidden_sizes=[32, 16], compression={"zlib": {"level": 1}})
    assert isinstance(m, LightningModel) and m.compression == {"zlib": {"level": 1}}
    assert [p.shape for p in m.get_parameters()][:2] == [(32, 784), (32,)]
    m2 = build_model({"package": "myfyp_amd.examples.mlp_pytorch", "model_build_fn": "model_build_fn",
                      "params": {"compression": {"ptq": {"dtype": "float16"}}}})
    assert m2.compression == {"ptq": {"dtype": "float16"}}
    m3 = build_model({"name": "MLP", "params": {"compression": {"topk": {"k": 0.2}}}}, seed=1)
    assert m3.compression == {"topk": {"k": 0.2}}


def test_compressed_peers_federate_over_memory_protocol():
    """Two peers whose payloads go over the wire (memory protocol: encode → decode), float16 + zlib:
    they finish and agree to within the float16 transport error."""
    from myfyp_amd.communication.protocols.memory.memory_communication_protocol import InMemoryCommunicationProtocol
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.node import Node
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.utils import wait_convergence, wait_to_finish

    saved = Settings.USE_FUSED_KERNELS
    Settings.USE_FUSED_KERNELS = False
    try:
        data = synthetic_mnist(512, 128, seed=3)
        parts = data.generate_partitions(2, RandomIIDPartitionStrategy)
        nodes = [Node(TorchModel(MLP(seed=g), compression={"ptq": {"dtype": "float16"}, "zlib": {}}), parts[g], protocol=InMemoryCommunicationProtocol)
                 for g in range(2)]
        for nd in nodes:
            nd.start()
        nodes[0].connect(nodes[1].addr)
        wait_convergence(nodes, 1, only_direct=True, wait=10)
        nodes[0].set_start_learning(rounds=2, epochs=1)
        wait_to_finish(nodes, timeout=120)
        a, b = (nd.learner.get_model().get_parameters() for nd in nodes)
        for x, y in zip(a, b):
            assert np.allclose(x, y, rtol=2e-3, atol=2e-3)
    finally:
        for nd in nodes:
            nd.stop()
        Settings.USE_FUSED_KERNELS = saved


def test_newer_upstream_protobuff_import_paths():
    """``exp_SAVE3.txt:9`` imports ``p2pfl.communication.protocols.protobuff.memory``."""
    from myfyp_amd.communication.protocols.memory.memory_communication_protocol import InMemoryCommunicationProtocol
    from myfyp_amd.communication.protocols.protobuff.grpc import GrpcCommunicationProtocol
    from myfyp_amd.communication.protocols.protobuff.memory import MemoryCommunicationProtocol
    from myfyp_amd.runner import resolve_protocol

    assert MemoryCommunicationProtocol is InMemoryCommunicationProtocol
    assert GrpcCommunicationProtocol.__name__ == "GrpcCommunicationProtocol"
    assert resolve_protocol({"package": "p2pfl.communication.protocols.protobuff.memory", "protocol": "MemoryCommunicationProtocol"}) is InMemoryCommunicationProtocol


def test_yaml_example_with_fyp_model_and_compression():
    """``examples/configs/mnist_fyp_compressed_memory.yaml``: the FYP model builder with float16 +
    zlib payloads over the in-memory gossip protocol finishes and learns."""
    import os

    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.runner import run_experiment
    from myfyp_amd.settings import Settings

    saved = Settings.USE_FUSED_KERNELS
    try:
        Federation.reset()
        cfg = os.path.join(os.path.dirname(__file__), "..", "myfyp_amd", "examples", "configs", "mnist_fyp_compressed_memory.yaml")
        res = run_experiment(cfg, verbose=False)
        for h in res["histories"].values():
            assert h.count("RoundFinishedStage") == 3
        accs = [m["test_metric"][-1][1] for m in res["global_logs"].values()]
        assert min(accs) > 0.5, accs
    finally:
        Settings.USE_FUSED_KERNELS = saved
        Federation.reset()


def test_decode_refuses_bombs_and_bad_shapes():
    """peer-supplied compressed payloads are bounded by the receiving model — a zlib
    bomb, a tensor shape the model does not have, and out-of-range or unsorted top-k indices are
    refused before anything large is allocated."""
    import pickle
    import zlib

    from myfyp_amd.learning import compression as C
    from myfyp_amd.learning.frameworks.p2pfl_model import safe_loads

    shapes = [(4, 3), (3,)]
    params = [np.arange(12, dtype=np.float32).reshape(4, 3), np.ones(3, np.float32)]
    good = C.encode(params, {}, C.validate({"topk": {"k": 0.5}, "zlib": {}}))
    out, _ = C.decode(good, safe_loads, shapes)
    assert [o.shape for o in out] == shapes
    bomb = C.MAGIC + zlib.compress(b"\0" * (64 << 20), 9)  # 64 MiB of zeros in ~64 KB
    with pytest.raises(ValueError, match="inflates"):
        C.decode(bomb, safe_loads, shapes)
    huge = pickle.dumps({"params": [{"shape": np.array([1 << 20, 1 << 20]), "dtype": "float32", "idx": np.array([0]), "v": np.ones(1, np.float32)}],
                         "additional_info": {}, "compression": ["topk"]})
    with pytest.raises(ValueError):
        C.decode(huge, safe_loads, [(4, 3)])
    with pytest.raises(ValueError, match="exceeds"):
        C.decode(huge, safe_loads)  # no model shapes: the global element bound still holds
    for idx in (np.array([0, 12]), np.array([5, 2]), np.array([-1, 3])):
        bad = pickle.dumps({"params": [{"shape": np.array([4, 3]), "dtype": "float32", "idx": idx, "v": np.ones(2, np.float32)}],
                            "additional_info": {}, "compression": ["topk"]})
        with pytest.raises(ValueError, match="indices"):
            C.decode(bad, safe_loads, [(4, 3)])
