"""Timing-only probe (outputs wrong): bench.py --chain wideband with one stage of the wideband step
made a no-op -- WB_SKIP=waterfall prices k_waterfall's place in the three-stream step (the upper
bound of forming the waterfall frames inside the analysis).
usage: WB_SKIP=waterfall python tools/probes/wb_skip.py --chain wideband --no-cpu"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))
from tetraear.signal import wideband  # noqa: E402

if os.environ.get("WB_SKIP") == "waterfall":
    wideband.BenchStep._waterfall = lambda self, c: None
import bench  # noqa: E402

sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[1:]
sys.exit(bench.main())
