"""The bench's C3 1% crash leg alone (bench.crash_leg), one JSON line:
  python tools/crash_leg.py [N]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.argv = sys.argv[:2]
import bench  # noqa: E402  (puts the package on sys.path)
import gossipsim as gs  # noqa: E402

print(json.dumps(bench.crash_leg(gs, int(sys.argv[1]) if len(sys.argv) > 1 else 65536)))
