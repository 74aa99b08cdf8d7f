"""Profile the Python side of bench.py: every thread runs under its own cProfile; merged stats printed."""
import cProfile
import io
import os
import pstats
import sys
import threading

sys.path.insert(0, os.getcwd())
profiles = []
_orig_run = threading.Thread.run


def _run(self):
    p = cProfile.Profile()
    profiles.append(p)
    p.enable()
    try:
        _orig_run(self)
    finally:
        p.disable()


threading.Thread.run = _run
sys.argv = ["bench.py"] + sys.argv[1:]
import bench  # noqa: E402

main_prof = cProfile.Profile()
main_prof.enable()
bench.main()
main_prof.disable()
profiles.append(main_prof)
s = io.StringIO()
st = pstats.Stats(profiles[0], stream=s)
for p in profiles[1:]:
    st.add(p)
out = os.environ.get("PSTATS_OUT")
if out:
    st.dump_stats(out)
st.sort_stats("tottime").print_stats(40)
st.sort_stats("cumulative").print_stats("myfyp_amd", 60)
print(s.getvalue()[:12000], file=sys.stderr)
