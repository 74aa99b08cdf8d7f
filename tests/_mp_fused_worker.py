"""Worker of tests/test_multiproc_gpu.py: one rank of a 2-rank job on ONE GPU (gloo weights plane:
RCCL refuses two ranks per device). Each rank hosts 2 peers on the fused MLP engine; 3 collective
FedAvg rounds; rank 0 prints a JSON line with the max parameter difference over all 4 peers and the
max deviation of the last round's aggregate from the host float64 weighted mean of the 4 peers'
pre-aggregation rows (the FedAvg math pinned as in the reference's aggregator_test.py:68-113)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch

    from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.node import Node
    from myfyp_amd.parallel import weights_plane
    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.utils import wait_to_finish

    Settings.BATCH_SIZE = 64
    Settings.TRAIN_SET_SIZE = 4
    Settings.GANG_WINDOW = 5.0
    Settings.MLP_PRECISION = os.environ.get("MP_PRECISION", "fp32")
    fed = Federation.init()
    rank, world = fed.rank, fed.world
    parts = synthetic_mnist(4000, 800, seed=11).generate_partitions(2 * world, RandomIIDPartitionStrategy)
    nodes = [Node(TorchModel(MLP(seed=rank * 2 + j)), parts[rank * 2 + j], address=f"mp-{rank}-{j}", protocol=CollectiveCommunicationProtocol,
                  learner_kwargs={"batch_size": 64}) for j in range(2)]
    for n in nodes:
        n.start()
    fed.finalize()
    fused = all(getattr(n.learner, "_engine", None) is not None for n in nodes)
    # probe the last round's aggregation: every local peer's row (and sample weight) going in, and out
    probe = {}
    orig = weights_plane.aggregate_mean

    def probed(f, arrived, final=True):
        if not final:
            return orig(f, arrived, final=final)
        torch.cuda.synchronize()
        probe["pre"] = {a: (float(arrived[a][0]), weights_plane._pack(f.local_nodes[a].learner).double().cpu().numpy()) for a in arrived}
        out = orig(f, arrived, final=final)
        torch.cuda.synchronize()
        probe["post"] = {a: weights_plane._pack(f.local_nodes[a].learner).double().cpu().numpy() for a in arrived}
        return out

    weights_plane.aggregate_mean = probed
    if rank == 0:
        nodes[0].set_start_learning(rounds=3, epochs=1)
    wait_to_finish(nodes, timeout=300)
    flats = [torch.cat([p.detach().flatten().cpu() for p in n.learner.model.get_model().parameters()]) for n in nodes]
    gathered = fed.all_gather_object([f.numpy() for f in flats])
    allf = [torch.from_numpy(a) for per_rank in gathered for a in per_rank]
    diff = max(float((allf[0] - f).abs().max()) for f in allf)
    moved = float((allf[0] - torch.cat([p.detach().flatten() for p in MLP(seed=0).parameters()])).abs().max())
    probes = fed.all_gather_object(probe)
    pre = [v for pr in probes for v in pr["pre"].values()]
    wsum = sum(w for w, _ in pre)
    host = sum(w * row for w, row in pre) / wsum
    fedavg_err = max(float(abs(row - host).max()) for pr in probes for row in pr["post"].values())
    fedavg_scale = float(abs(host).max())
    for n in nodes:
        n.stop()
    if rank == 0:
        print(json.dumps({"world": world, "peers": len(allf), "fused": fused, "max_diff": diff, "moved": moved, "fedavg_err": fedavg_err,
                          "fedavg_scale": fedavg_scale, "n_pre": len(pre), "wsum": wsum}), flush=True)
    fed.shutdown()


if __name__ == "__main__":
    main()
