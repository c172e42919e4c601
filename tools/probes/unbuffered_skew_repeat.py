"""Failure rate of the UNBUFFERED skew repro (tools/probes/unbuffered_skew.py) over
repeated runs, per distribution."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from unbuffered_skew import run  # noqa: E402

if __name__ == "__main__":
    for seed in range(12):
        run((2, 64, 5), [1.0, 0.0], [0.0, 1.0], "UNBUFFERED", seed=seed)
    for seed in range(6):
        run((8, 8, 8), [1.0, 0.0], [0.0, 1.0], "UNBUFFERED", seed=seed)
        run((2, 64, 5), [1.0, 1.0], [0.0, 1.0], "UNBUFFERED", seed=seed)
