"""One bench.py rank with tests/benchfake/fake_gossipsim.py standing in for
gossipsim (CPU plumbing test only): python rank.py <bench.py arguments>."""
import pathlib
import sys

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parents[1]))
import fake_gossipsim  # noqa: E402

sys.modules["gossipsim"] = fake_gossipsim
sys.argv = ["bench.py"] + sys.argv[1:]
import bench  # noqa: E402

bench.main()
