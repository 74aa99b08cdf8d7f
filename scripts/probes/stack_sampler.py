"""Sampling profiler for the bench's host threads: runs bench.py in-process and every 0.5 ms records
each thread's innermost frames; prints the hottest (file:line function) stacks per thread role.

    python scripts/probes/stack_sampler.py --steps 20 --warmup 3
"""
import collections
import os
import sys
import threading
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

samples = collections.Counter()
stop = False


def sampler():
    me = threading.get_ident()
    while not stop:
        names = {t.ident: t.name for t in threading.enumerate()}
        for tid, frame in sys._current_frames().items():
            if tid == me:
                continue
            st = traceback.extract_stack(frame)[-4:]
            key = (names.get(tid, "?").split("-")[0], " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in reversed(st)))
            samples[key] += 1
        time.sleep(0.0005)


if __name__ == "__main__":
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    sys.argv = ["bench.py"] + sys.argv[1:]
    import runpy

    try:
        runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
    finally:
        stop = True
        th.join()
        tot = collections.Counter()
        for (role, _), n in samples.items():
            tot[role] += n
        for role, n in tot.most_common(8):
            print(f"== {role}: {n} samples", file=sys.stderr)
            for (r, st), k in samples.most_common():
                if r == role and k >= max(3, n // 100):
                    print(f"  {k:6d} {st}", file=sys.stderr)
