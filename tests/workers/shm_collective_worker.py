"""torchrun worker: shared-memory control-plane gathers vs gloo (run by tests/test_shm_collective.py)."""

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch.distributed as dist  # noqa: E402

from myfyp_amd.parallel.federation import Federation  # noqa: E402

fed = Federation.init()
rank, world = fed.rank, fed.world
assert fed.shm is not None, "single-host job should get the shared-memory control plane"
# small payloads: votes-like dicts, many generations (parity slots reused)
for g in range(200):
    got = fed.all_gather_object({"r": rank, "g": g, "votes": {f"peer-{rank}": g * 10 + rank}})
    assert [x["r"] for x in got] == list(range(world)), got
    assert all(x["g"] == g for x in got), got
    assert got[(rank + 1) % world]["votes"] == {f"peer-{(rank + 1) % world}": g * 10 + (rank + 1) % world}
# one rank overflows its slot: every rank must fall back to gloo in the same call and still agree
big = b"x" * (200_000 if rank == 1 else 10)
got = fed.all_gather_object(big)
assert [len(x) for x in got] == [200_000 if r == 1 else 10 for r in range(world)]
# and the shared path keeps working afterwards
got = fed.all_gather_object(rank * 7)
assert got == [r * 7 for r in range(world)]
fed.shm.barrier()
t = time.perf_counter()
for _ in range(500):
    fed.all_gather_object(("vote", rank))
dt = (time.perf_counter() - t) / 500
print(f"rank {rank} OK shm gather {dt * 1e6:.1f} us", flush=True)
fed.shutdown()
assert not dist.is_initialized()
