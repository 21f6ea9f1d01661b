"""bench.py's argument handling and its one-JSON-line contract at
--gpus 1 and --gpus 2 (gloo, world 2, launched as the driver does:
torch.distributed.run, 127.0.0.1), with a stand-in engine
(tests/benchfake/fake_gossipsim.py) so that it runs on CPU. Pins the schema
of the N > 1 line: whole-job value = rounds / max-over-ranks time, every
rank's k_round roofline, and the multi-GPU legs (the row layout's exchange
over xGMI; config 4's N=262,144 column leg at 8 GPUs or with --c4)."""
import json
import os
import pathlib
import socket
import subprocess
import sys

REPO = pathlib.Path(__file__).resolve().parents[1]
RANK = REPO / "tests" / "benchfake" / "rank.py"
TOP = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
       "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}
ROOF = {"bound", "achieved", "peak", "unit", "frac", "traffic", "avg_launch_ms", "bytes_per_launch"}


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def one_line(out):
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def check_common(d, n_gpus, steps, warmup):
    assert TOP <= d.keys(), TOP - d.keys()
    assert d["metric"] == json.loads((REPO / "BASELINE.json").read_text())["metric"]
    assert (d["n_gpus"], d["steps"], d["warmup"], d["unit"], d["dtype"]) == (n_gpus, steps, warmup, "rounds/s",
                                                                             "int32")
    assert d["value"] > 0 and abs(d["value"] - 1e3 / d["ms_per_step"]) < 1e-6 * d["value"]
    assert ROOF <= d["roofline"].keys()
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["unit"] == "GB/s"
    assert abs(d["roofline"]["avg_launch_ms"] - 1.5) < 1e-9  # the stand-in's launch time
    assert len(d["roofline_per_rank"]) == n_gpus
    assert "workload" in d["config"]


def test_bench_line_one_gpu():
    r = subprocess.run([sys.executable, str(RANK), "--steps", "4", "--warmup", "1", "--no-secondary",
                        "--no-cpu-baseline", "--files", "0"], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 0, r.stderr
    d = one_line(r.stdout)
    check_common(d, 1, 4, 1)
    assert d["config"]["parallelism"] == "single" and d["cpu_baseline"] is None
    # k_round covers all N x N cells: 2 B per cell on the 4-bit tier
    assert d["roofline"]["bytes_per_launch"] == 2.0 * 65536 * 65536


def test_bench_line_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), str(RANK), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--c4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=REPO,
                       env={**os.environ, "OMP_NUM_THREADS": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = one_line(r.stdout)
    check_common(d, 2, 3, 1)
    assert d["scaling"] == "strong" and d["cpu_baseline"] is None and d["placement"] is None
    assert d["config"]["parallelism"].startswith("column-shard x2")
    # each column shard's k_round covers all rows x its N/2 columns
    for i, pr in enumerate(d["roofline_per_rank"]):
        assert pr["rank"] == i and pr["cols"] == 32768 and pr["bytes_per_launch"] == 2.0 * 65536 * 32768
    sec = d["secondary"]
    assert set(sec) == {"rows", "c4_n262144"}
    rows = sec["rows"]
    assert rows["layout"] == "rows" and len(rows["roofline_per_rank"]) == 2
    for pr in rows["roofline_per_rank"]:  # each row shard: N/2 rows x all N columns, and its exchange
        assert pr["rows"] == 32768 and pr["cols"] == 65536
        assert pr["exchange"]["bytes_in"] > 0 and pr["xgmi_in_gbs"] > 0
    c4 = sec["c4_n262144"]
    assert c4["n_members"] == 262144 and c4["layout"] == "columns"
    assert [pr["cols"] for pr in c4["roofline_per_rank"]] == [131072, 131072]
