"""Worker of tests/test_fault_tolerance.py::test_clean_leave_with_a_deferred_all_reduce:
3 gloo ranks start a deferred (asynchronously confirmed) weight all-reduce; rank 2 then departs
cleanly — its last local peer stopped — before the others confirm it. The survivors' confirmation
must accept the departure (no recovery, no retry), keep the departed rank's share in the result and
continue over ranks [0, 1]. Each survivor writes one JSON file."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch

    from myfyp_amd.parallel.federation import Federation
    from myfyp_amd.settings import Settings

    Settings.FAILURE_TIMEOUT = 20.0
    fed = Federation.init()
    fed.finalize()
    rank = fed.rank
    retried = []
    t = torch.full((8,), float(rank + 1))
    with fed.weights_section():
        w = fed.all_reduce_async(t)
        fed.defer_confirm([w], lambda: retried.append(1))
    if rank == 2:
        fed.depart()  # clean leave: completes its side of the pending all-reduce first
        fed.shutdown()
        return
    fed.confirm_collectives()
    members = fed.sync_members()
    u = torch.full((4,), float(rank + 1))
    fed.all_reduce_(u)  # the next collective runs over the survivors only
    out = {"rank": rank, "recoveries": fed.recoveries, "retried": len(retried), "result": t.tolist(), "members": members, "next": u.tolist()}
    with open(os.path.join(os.environ["OUT_DIR"], f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    fed.shutdown()


if __name__ == "__main__":
    main()
