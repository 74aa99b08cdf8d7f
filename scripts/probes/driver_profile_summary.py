"""Summarise a cProfile dump of the round driver thread (MYFYP_PROFILE_DRIVER=<path>)."""
import pstats
import sys

st = pstats.Stats(sys.argv[1])
st.sort_stats("tottime").print_stats(int(sys.argv[2]) if len(sys.argv) > 2 else 40)
st.sort_stats("cumulative").print_stats(int(sys.argv[2]) if len(sys.argv) > 2 else 40)
