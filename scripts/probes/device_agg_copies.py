"""Device SCAFFOLD / FedMedian aggregation on cuda:0 in a timed window: prints the window
(CLOCK_MONOTONIC ns, the clock rocprofv3 stamps with) and per-call wall times, so
scripts/tools/copies_in_window.py can show which copies and kernels fall inside it.

    rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/agg -o run -- python3 scripts/probes/device_agg_copies.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.aggregators import FedMedian, Scaffold  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.models import MLP  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.parallel import weights_plane  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402

ITERS = 50


def run(kind: str, k: int = 8) -> dict:
    Federation.reset()
    fed = Federation.init()
    data = synthetic_mnist(256, 64)
    make = (lambda: Scaffold(global_lr=1.0)) if kind == "scaffold" else FedMedian
    nodes = [Node(TorchModel(MLP(seed=i)), data, address=f"{kind}-{i}", aggregator=make(), protocol=CollectiveCommunicationProtocol) for i in range(k)]
    for nd in nodes:
        nd.start()
    fed.finalize()
    n = nodes[0].learner.flat_params().numel()
    for i, nd in enumerate(nodes):
        f = nd.learner.flat_params()
        if kind == "scaffold":
            cb = weights_plane._scaffold_cb(nd.learner)
            cb.x0 = f.detach().clone()
            cb.delta_y = torch.randn(n, device=f.device) * 1e-3
            cb.delta_c = torch.randn(n, device=f.device) * 1e-3
    arrived = {nd.addr: (float(1 + i), None) for i, nd in enumerate(nodes)}
    agg = nodes[0].aggregator
    call = (lambda: weights_plane.aggregate_scaffold(fed, arrived, agg)) if kind == "scaffold" else (lambda: weights_plane.aggregate_median(fed, arrived))
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    t0 = time.monotonic_ns()
    w0 = time.perf_counter()
    for _ in range(ITERS):
        call()
    torch.cuda.synchronize()
    w1 = time.perf_counter()
    t1 = time.monotonic_ns()
    for nd in nodes:
        nd.stop()
    Federation.reset()
    return {"kind": kind, "peers": k, "numel": n, "iters": ITERS, "window_ns": [t0, t1], "us_per_call": round((w1 - w0) / ITERS * 1e6, 1)}


if __name__ == "__main__":
    out = [run("scaffold"), run("median")]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/device_agg_windows.json", "w") as f:
        json.dump(out, f)
    print(json.dumps(out))
