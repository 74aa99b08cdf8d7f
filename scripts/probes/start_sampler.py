"""Stack sampler over the first ~30 ms after set_start_learning (headline setup, 8 peers): every
0.25 ms, the innermost myfyp_amd frame of every thread. Prints, per 1 ms bucket, the most common
frames (who is busy or waiting where) — finds host-side latency before the first epochs."""

import collections
import os
import sys
import threading
import time
import traceback

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))

from myfyp_amd.communication.protocols.collective.collective_protocol import CollectiveCommunicationProtocol  # noqa: E402
from myfyp_amd.learning.dataset.partition_strategies import RandomIIDPartitionStrategy  # noqa: E402
from myfyp_amd.learning.dataset.synthetic import synthetic_mnist  # noqa: E402
from myfyp_amd.learning.frameworks.torch import TorchModel  # noqa: E402
from myfyp_amd.models import MLP  # noqa: E402
from myfyp_amd.node import Node  # noqa: E402
from myfyp_amd.parallel.federation import Federation  # noqa: E402
from myfyp_amd.settings import Settings  # noqa: E402
from myfyp_amd.utils.utils import wait_to_finish  # noqa: E402

Settings.BATCH_SIZE = 64
fed = Federation.init()
data = synthetic_mnist(60000, 10000, seed=2024, similarity=0.75, noise=1.0)
parts = data.generate_partitions(8, RandomIIDPartitionStrategy)
nodes = [Node(TorchModel(MLP(seed=100 + g)), parts[g], address=f"peer-{g}", protocol=CollectiveCommunicationProtocol, learner_kwargs={"batch_size": 64})
         for g in range(8)]
for nd in nodes:
    nd.start()
fed.finalize()
samples = []
stop = threading.Event()
me = threading.get_ident()


def where(frame):
    st = traceback.extract_stack(frame)
    own = [f for f in st if "myfyp_amd" in f.filename]
    inner = st[-1]
    o = own[-1] if own else inner
    return f"{os.path.basename(o.filename)}:{o.lineno}:{o.name} <- {os.path.basename(inner.filename)}:{inner.name}"


def sampler(t0):
    while not stop.is_set():
        t = time.perf_counter() - t0
        if t > 0.045:
            break
        fr = sys._current_frames()
        for tid, f in fr.items():
            if tid in (me, threading.get_ident()):
                continue
            samples.append((t, tid, where(f)))
        time.sleep(0.00025)


t0 = time.perf_counter()
th = threading.Thread(target=sampler, args=(t0,), daemon=True)
th.start()
nodes[0].set_start_learning(rounds=12, epochs=1)
wait_to_finish(nodes, timeout=120)
stop.set()
th.join()
byb = collections.defaultdict(collections.Counter)
for t, tid, w in samples:
    if "threading.py:wait" in w and "queue" not in w and "pending" not in w:
        pass
    byb[int(t * 1000)][w] += 1
for b in sorted(byb):
    top = byb[b].most_common(6)
    print(f"--- {b} ms")
    for w, c in top:
        print(f"   {c:4d} {w}")
for nd in nodes:
    nd.stop()
Federation.reset()
