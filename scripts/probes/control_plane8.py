"""Control-plane cost of the headline's 8-rank layout, on this host's CPUs:
  1. the shared-memory gather primitive alone: 8 ranks, back-to-back ``all_gather_object`` of a
     vote-sized payload (tests/workers/shm_collective_worker.py), median per gather;
  2. the collective workflow at 8 ranks (tests/workers/rehearsal8_worker.py, ROUNDS rounds): per
     rank and round, the host time inside the vote / model gathers, ``sync_members``, every
     post-collective ``_agree`` and the deferred-collective confirmation.
Writes a markdown summary to stdout (profiles/r4_control_plane8/README.md)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _ports import free_port  # noqa: E402


def torchrun(script, env_extra, nproc=8):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), script]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    if res.returncode != 0:
        raise SystemExit(res.stdout[-2000:] + res.stderr[-4000:])
    return res.stdout


def main() -> None:
    rounds = int(os.environ.get("ROUNDS", "30"))
    out = torchrun(os.path.join(ROOT, "tests", "workers", "shm_collective_worker.py"), {})
    gathers = [float(l.split()[-2]) for l in out.splitlines() if "shm gather" in l]
    print("# Control plane at 8 ranks (CPU rehearsal)\n")
    print(f"Host: {os.cpu_count()} CPUs. 8 processes, one per would-be GPU.\n")
    print("## Shared-memory gather primitive\n")
    print(f"Back-to-back `all_gather_object` of a vote-sized payload, 500 per rank: median over ranks "
          f"**{np.median(gathers):.1f} us** per gather (min {min(gathers):.1f}, max {max(gathers):.1f}).\n")
    for label, extra in (("no fault", {}), ("rank 5 dies inside round 2's all-reduce", {"KILL_RANK": "5", "KILL_ROUND": "2"})):
        with tempfile.TemporaryDirectory() as d:
            torchrun(os.path.join(ROOT, "tests", "workers", "rehearsal8_worker.py"), {"ROUNDS": str(rounds), "OUT_DIR": d, **extra})
            ranks = [json.load(open(os.path.join(d, f))) for f in sorted(os.listdir(d))]
        print(f"## Collective workflow, {rounds} rounds, {label}\n")
        print(f"Survivors: {len(ranks)}; finished rounds {sorted({r['finished_rounds'] for r in ranks})}; "
              f"recoveries {sorted({r['recoveries'] for r in ranks})}; elapsed {np.median([r['elapsed'] for r in ranks]):.2f} s (median rank).\n")
        keys = sorted({k for r in ranks for k in r["control_plane"]})
        print("| primitive | calls per rank | median us | p90 us | host ms per round (median rank) |")
        print("|---|---|---|---|---|")
        per_round = []
        for k in keys:
            calls = [r["control_plane"][k]["n"] for r in ranks if k in r["control_plane"]]
            med = [r["control_plane"][k]["median_us"] for r in ranks if k in r["control_plane"]]
            p90 = [r["control_plane"][k]["p90_us"] for r in ranks if k in r["control_plane"]]
            tot = [r["control_plane"][k]["total_ms"] / rounds for r in ranks if k in r["control_plane"]]
            per_round.append(np.median(tot))
            print(f"| `{k}` | {int(np.median(calls))} | {np.median(med):.1f} | {np.median(p90):.1f} | {np.median(tot):.3f} |")
        tot_rank = [sum(r["control_plane"][k]["total_ms"] for k in r["control_plane"]) / rounds for r in ranks]
        print(f"\nAll primitives: **{np.median(tot_rank):.3f} ms per round** (median rank; max {max(tot_rank):.3f}).\n")


if __name__ == "__main__":
    main()
