"""Run the map-lifetime GPU tests several times in one process (run-to-run
determinism evidence for the release path: tests/test_lifetime_gpu.py checks
every scan's counters and the whole root map against the oracle, and two lone
runs against each other bit for bit).

    python scripts/repeat_lifetime.py [repeats]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("vina-slam_amd/py", "oracle", "tests", ""):
    sys.path.insert(0, os.path.join(REPO, p))

import oracle  # noqa: E402
import test_lifetime_gpu as t  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    oracle.build()
    for r in range(n):
        for name in ("test_release_matches_oracle", "test_release_runs_are_bit_identical",
                     "test_small_capacity_completes_with_release"):
            t0 = time.time()
            f = getattr(t, name)
            f(oracle) if f.__code__.co_argcount else f()
            print("repeat %d %s ok (%.1f s)" % (r, name, time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
