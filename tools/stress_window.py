"""Run the two-rank relay -> queues -> window test (tests/test_comm_gpu.py) N times in one process
and report each failure (diagnosing an intermittent SHD_ERR_INVALID from shd_equeue_advance)."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_comm_gpu as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
fails = 0
for i in range(n):
    for dyn in (True, False):
        try:
            T.test_local_two_ranks_relay_into_queues_with_window(None, dyn)
        except Exception as e:  # noqa: BLE001
            fails += 1
            print(f"iter {i} dynamic={dyn}: FAIL {type(e).__name__}: {e}", flush=True)
            traceback.print_exc(limit=3)
    print(f"iter {i} done, fails so far {fails}", flush=True)
print(f"STRESS fails={fails} of {2 * n}")
