"""Side-stream FedAvg concurrent with evaluation kernels on one MI355X (8 ResNet-18 peers on the
CNN engine). Delayed averaging: aggregate_mean(final=False) snapshots on the compute stream and
launches the bucketed reduce on the side stream; the next round's evaluation is launched right
behind it on the compute stream and does not wait for it. Run under
    rocprofv3 --kernel-trace -d gpurun_out/ovlp -o run -- python3 scripts/probes/overlap_probe.py
then  python3 scripts/tools/kernel_overlap.py gpurun_out/ovlp/run_results.db fedavg
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_cifar10  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.models import ResNet18  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.parallel import weights_plane  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402


def main() -> None:
    Settings.BATCH_SIZE = 128
    Settings.BUCKET_BYTES = 4 << 20  # several buckets per aggregation
    fed = Federation.init()
    parts = synthetic_cifar10(8 * 512, 8 * 2048, seed=7).generate_partitions(8, RandomIIDPartitionStrategy)
    nodes = [Node(TorchModel(ResNet18(seed=i)), parts[i], address=f"ovl-{i}", protocol=CollectiveCommunicationProtocol, learner_kwargs={"batch_size": 128})
             for i in range(8)]
    for nd in nodes:
        nd.start()
    fed.finalize()
    group = nodes[0].learner._engine.group
    slots = {nd.learner._engine.slot: () for nd in nodes}
    arrived = {nd.addr: (1.0, None) for nd in nodes}
    group._run_eval_batch(slots)  # warm: eager run, then graph capture
    group._run_eval_batch(slots)
    for mode in ("delayed", "exact"):
        Settings.DELAYED_AVERAGING = mode == "delayed"
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(4):
            weights_plane.aggregate_mean(fed, arrived, final=(mode == "exact"))
            group._run_eval_batch(slots)
        torch.cuda.synchronize()
        print(f"{mode}: {1000 * (time.perf_counter() - t0) / 4:.2f} ms per (aggregate + eval of 8x2048 images)", flush=True)
    weights_plane.aggregate_mean(fed, arrived, final=True)  # flush the pending delayed average
    torch.cuda.synchronize()
    for nd in nodes:
        nd.stop()
    fed.shutdown()


if __name__ == "__main__":
    main()
