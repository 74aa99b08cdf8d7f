"""Worker of tests/test_fault_tolerance.py::test_rank_dies_inside_the_all_reduce: one rank (one
peer) of a 3-rank collective job; rank KILL_RANK's process exits right before it issues the FedAvg
all-reduce of round KILL_ROUND — after the reduce of its local rows and after the pre-collective
membership agreement, so the survivors are already inside the collective. Every rank records the
rows that entered and left each round's aggregation; survivors print one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    from myfyp_amd.parallel import weights_plane
    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.settings import Settings
    from myfyp_amd.utils.utils import wait_to_finish

    rounds = int(os.environ.get("ROUNDS", "3"))
    kill_rank = int(os.environ.get("KILL_RANK", "2"))
    kill_round = int(os.environ.get("KILL_ROUND", "1"))
    Settings.BATCH_SIZE = 32
    Settings.GANG_WINDOW = 5.0
    Settings.FAILURE_TIMEOUT = float(os.environ.get("FAILURE_TIMEOUT", "20"))
    fed = Federation.init()
    rank, world = fed.rank, fed.world
    Settings.TRAIN_SET_SIZE = world
    parts = synthetic_mnist(600 * world, 200, seed=5, similarity=0.3).generate_partitions(world, RandomIIDPartitionStrategy)
    node = Node(TorchModel(MLP(hidden_sizes=[32, 16], seed=rank)), parts[rank], address=f"cc-{rank}", protocol=CollectiveCommunicationProtocol,
                learner_kwargs={"batch_size": 32})
    node.start()
    fed.finalize()
    if rank == kill_rank:
        fault_injection.crash_in_collective(fed, node, round=kill_round)

    # record what enters / leaves every aggregation of this rank's peer
    trace = {}
    orig = weights_plane.aggregate_mean

    def probed(f, arrived, final=True):
        r = node.state.round
        lr = node.learner
        pre = weights_plane._pack(lr).detach().cpu().double()
        w = float(arrived[node.addr][0]) if node.addr in arrived else 0.0
        out = orig(f, arrived, final=final)
        post = weights_plane._pack(lr).detach().cpu().double()
        trace[r] = {"pre": pre.tolist(), "w": w, "post": post.tolist()}
        return out

    weights_plane.aggregate_mean = probed
    t0 = time.time()
    if rank == 0:
        node.set_start_learning(rounds=rounds, epochs=1)
    wait_to_finish([node], timeout=300)
    elapsed = time.time() - t0
    hist = node.learning_workflow.history
    out = {"rank": rank, "members": fed.members, "recoveries": fed.recoveries, "finished_rounds": hist.count("RoundFinishedStage"),
           "elapsed": elapsed, "trace": {str(k): v for k, v in trace.items() if k == kill_round}}
    node.stop()
    # rows are long: a file per rank (torchrun interleaves long stdout lines of concurrent ranks)
    with open(os.path.join(os.environ["OUT_DIR"], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    fed.shutdown()


if __name__ == "__main__":
    main()
