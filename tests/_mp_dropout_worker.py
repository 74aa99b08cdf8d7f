"""Worker of tests/test_fault_tolerance.py: one rank (one peer) of a W-rank collective job; the
peer of rank KILL_RANK is killed at TrainStage of round 1. Survivors must finish every round with
equal models; every rank prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch

    from myfyp_amd import fault_injection
    from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol
    from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.node import Node
    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.utils import wait_to_finish

    rounds = int(os.environ.get("ROUNDS", "3"))
    kill_rank = int(os.environ.get("KILL_RANK", "2"))
    Settings.BATCH_SIZE = 32
    Settings.GANG_WINDOW = 5.0
    Settings.FAILURE_TIMEOUT = float(os.environ.get("FAILURE_TIMEOUT", "10"))
    fed = Federation.init()
    rank, world = fed.rank, fed.world
    Settings.TRAIN_SET_SIZE = world
    parts = synthetic_mnist(600 * world, 200, seed=5, similarity=0.3).generate_partitions(world, RandomIIDPartitionStrategy)
    node = Node(TorchModel(MLP(seed=rank)), parts[rank], address=f"ft-{rank}", protocol=CollectiveCommunicationProtocol,
                learner_kwargs={"batch_size": 32})
    node.start()
    fed.finalize()
    mode = os.environ.get("KILL_MODE", "stop")
    fault = None
    if rank == kill_rank:
        fault = (fault_injection.crash_process_at if mode == "crash" else fault_injection.kill_at)(node, "TrainStage", round=1)
    t0 = time.time()
    if rank == 0:
        node.set_start_learning(rounds=rounds, epochs=1)
    wait_to_finish([node], timeout=300)
    elapsed = time.time() - t0
    flat = torch.cat([p.detach().flatten().cpu() for p in node.learner.model.get_model().parameters()])
    hist = node.learning_workflow.history
    out = {"rank": rank, "killed": fault is not None and fault.fired.is_set(), "departed": fed.departed, "members": fed.members,
           "finished_rounds": hist.count("RoundFinishedStage"), "elapsed": elapsed, "checksum": float(flat.double().sum()),
           "absmax": float(flat.abs().max())}
    node.stop()
    print(json.dumps(out), flush=True)
    fed.shutdown()


if __name__ == "__main__":
    main()
