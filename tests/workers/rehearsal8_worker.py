"""Worker of tests/test_rehearsal8.py and of ``scripts/probes/control_plane8.py``: one rank of an
8-rank collective job on the CPU (gloo weights plane + the shared-memory control plane), one
small-MLP peer per rank — the headline's process layout at N = 8 (8 peers, one per
GPU), rehearsed without GPUs. Optionally rank KILL_RANK's process dies right before it issues the
FedAvg all-reduce of round KILL_ROUND (inside the collective, after the pre-collective agreement).

Every surviving rank writes rank<r>.json: finished rounds, members, recoveries, elapsed time, a
parameter checksum, and the host time of each control-plane primitive (median and total over the
run): the vote / model gather, the pre-collective ``sync_members``, the post-collective ``_agree``
and the deferred-collective confirmation."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main() -> None:
    import faulthandler

    # a rank stuck for 90 s prints every thread's stack and exits (a test failure with a diagnosis,
    # not a 300 s subprocess timeout)
    hang = open(os.path.join(os.environ["OUT_DIR"], f"hang_{os.environ.get('LOCAL_RANK', '0')}.txt"), "w")
    faulthandler.dump_traceback_later(float(os.environ.get("HANG_DUMP_S", "90")), exit=True, file=hang)
    import numpy as np
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

    torch.set_num_threads(1)
    rounds = int(os.environ.get("ROUNDS", "5"))
    kill_rank = int(os.environ.get("KILL_RANK", "-1"))
    kill_round = int(os.environ.get("KILL_ROUND", "2"))
    Settings.BATCH_SIZE = 32
    Settings.GANG_WINDOW = 5.0
    Settings.FAILURE_TIMEOUT = float(os.environ.get("FAILURE_TIMEOUT", "20"))
    fed = Federation.init()
    rank, world = fed.rank, fed.world
    Settings.TRAIN_SET_SIZE = world
    parts = synthetic_mnist(200 * world, 50 * world, seed=5, similarity=0.3).generate_partitions(world, RandomIIDPartitionStrategy)
    node = Node(TorchModel(MLP(hidden_sizes=[32, 16], seed=rank)), parts[rank], address=f"r8-{rank}", protocol=CollectiveCommunicationProtocol,
                learner_kwargs={"batch_size": 32})
    node.start()
    fed.finalize()

    def dump_shm_state() -> None:  # diagnostics of a stuck run: control-plane generations
        if fed.shm is not None:
            gen, st = fed.shm.state()
            hang.write(f"shm gen {gen} status {st} members {fed.members}\n")
            hang.flush()

    t_dump = threading.Timer(float(os.environ.get("HANG_DUMP_S", "90")) - 5, dump_shm_state)
    t_dump.daemon = True
    t_dump.start()
    if rank == kill_rank:
        fault_injection.crash_in_collective(fed, node, round=kill_round)
    t0 = time.time()
    if rank == 0:
        node.set_start_learning(rounds=rounds, epochs=1)
    wait_to_finish([node], timeout=300)
    elapsed = time.time() - t0
    flat = torch.cat([p.detach().flatten().cpu() for p in node.learner.model.get_model().parameters()])
    hist = node.learning_workflow.history
    cp = {}
    for k, v in fed.stats.items():
        if k.startswith("cp_") and v:
            cp[k] = {"n": len(v), "median_us": round(1e6 * float(np.median(v)), 1), "p90_us": round(1e6 * float(np.percentile(v, 90)), 1),
                     "total_ms": round(1e3 * float(np.sum(v)), 3)}
    out = {"rank": rank, "world": world, "members": fed.members, "recoveries": fed.recoveries, "finished_rounds": hist.count("RoundFinishedStage"),
           "elapsed": elapsed, "checksum": float(flat.double().sum()), "absmax": float(flat.abs().max()), "control_plane": cp}
    node.stop()
    with open(os.path.join(os.environ["OUT_DIR"], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    fed.shutdown()


if __name__ == "__main__":
    main()
