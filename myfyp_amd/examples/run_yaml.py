"""Run an experiment described by a YAML file (see myfyp_amd/examples/configs/)."""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from myfyp_amd.runner import run_experiment  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="Run a YAML experiment.")
    ap.add_argument("config", help="path to the YAML file")
    run_experiment(ap.parse_args().config)
