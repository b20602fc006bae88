"""bench.py's multi-GPU entry point (config 3's scaling leg): ``--gpus N`` starts N ranks
through torch.distributed.run before any GPU call, and a launcher whose WORLD_SIZE differs
from ``--gpus`` is refused.  CPU only: the launch command is composed, not run, and the
check is the pure function the entry point calls first."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_command_composes_one_rank_per_gpu():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = bench.launch_command(argv, 8, 29555)
    assert cmd[0] == sys.executable
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv            # every bench argument reaches every rank


def test_check_world():
    assert bench.check_world(1, {}) == "run"                     # the N=1 line is unchanged
    assert bench.check_world(4, {}) == "launch"                  # spawn 4 ranks
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == "run"    # a rank of the driver's launch
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(SystemExit):
        bench.check_world(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "2"})


def test_free_port_is_bindable():
    import socket
    p = bench.free_port()
    with socket.socket() as s:
        s.bind(("127.0.0.1", p))


def test_gpus_2_launches_two_ranks_end_to_end():
    """`bench.py --gpus 2 --dry-run` from a plain shell: the parent spawns torch.distributed.run,
    two ranks rendezvous on 127.0.0.1 over gloo, rank 0's JSON line reaches our stdout."""
    import json
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert lines == [{"dry_run": True, "n_gpus": 2, "ranks_seen": 2}]


def test_graph_streams_env():
    """bench.py sets the HIP graph executor's stream count (2) before torch loads the runtime, for
    one GPU and for every rank of an N-GPU run; CMX_GRAPH_STREAMS picks another count (0 = the
    runtime's own), an explicit DEBUG_HIP_FORCE_GRAPH_QUEUES is kept.  The count never exceeds
    GPU_MAX_HW_QUEUES: clamped, and an explicit larger setting is refused."""
    import bench
    for argv, e in ((["--steps", "5"], {}), (["--gpus", "2"], {}), (["--gpus=8"], {}), ([], {"WORLD_SIZE": "4"})):
        bench._graph_streams_env(argv, e)
        assert e["DEBUG_HIP_FORCE_GRAPH_QUEUES"] == "2", (argv, e)
    e = {"CMX_GRAPH_STREAMS": "0"}
    bench._graph_streams_env([], e)
    assert "DEBUG_HIP_FORCE_GRAPH_QUEUES" not in e
    e = {"DEBUG_HIP_FORCE_GRAPH_QUEUES": "3"}
    bench._graph_streams_env([], e)
    assert e["DEBUG_HIP_FORCE_GRAPH_QUEUES"] == "3"
    e = {"CMX_GRAPH_STREAMS": "3"}
    bench._graph_streams_env([], e)
    assert e["DEBUG_HIP_FORCE_GRAPH_QUEUES"] == "3"
    for hwq, want in (("1", "1"), ("2", "2"), ("3", "2"), ("8", "2")):
        e = {"GPU_MAX_HW_QUEUES": hwq}
        bench._graph_streams_env([], e)
        assert e["DEBUG_HIP_FORCE_GRAPH_QUEUES"] == want, (hwq, e)
    e = {"GPU_MAX_HW_QUEUES": "2", "CMX_GRAPH_STREAMS": "0"}
    bench._graph_streams_env([], e)
    assert e["DEBUG_HIP_FORCE_GRAPH_QUEUES"] == "2"
    with pytest.raises(SystemExit):
        bench._graph_streams_env([], {"GPU_MAX_HW_QUEUES": "1", "DEBUG_HIP_FORCE_GRAPH_QUEUES": "2"})
