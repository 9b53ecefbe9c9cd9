"""bench.py --gpus N's launcher (lac_amd/launch.py), on CPU: N children under
torch.distributed.run get RANK / LOCAL_RANK / WORLD_SIZE, rank 0's one JSON line is
relayed, a failing child fails the run, and nccl ranks beyond the GPUs are refused."""
import io
import json
import os
import subprocess
import sys

import pytest

from lac_amd import launch

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = os.path.join(HERE, "helpers", "rank_child.py")
REPO = os.path.dirname(HERE)


def _envs(text):
    return sorted((json.loads(l[4:]) for l in text.splitlines() if l.startswith("env ")), key=lambda d: d["rank"])


@pytest.mark.parametrize("n", [2, 4])
def test_children_get_rank_env_and_one_line(n):
    out = io.StringIO()
    rc, lines = launch.run_ranks(n, CHILD, ["--gpus", str(n), "--steps", "3"], out=out)
    assert rc == 0
    envs = _envs(out.getvalue())
    assert [e["rank"] for e in envs] == list(range(n))
    assert [e["local_rank"] for e in envs] == list(range(n))
    assert all(e["world"] == n and e["master_addr"] == "127.0.0.1" for e in envs)
    assert all(e["argv"] == ["--gpus", str(n), "--steps", "3"] for e in envs)
    results = [d for d in lines if "metric" in d]
    assert len(results) == 1 and results[0]["n_gpus"] == n


def test_failing_child_fails_the_run():
    env = dict(os.environ, LAC_TEST_FAIL_RANK="1")
    rc, lines = launch.run_ranks(2, CHILD, [], env=env, out=io.StringIO())
    assert rc != 0


def test_relay_status(monkeypatch):
    monkeypatch.setenv("LAC_TEST_FAIL_RANK", "0")
    assert launch.relay(2, CHILD, []) != 0
    monkeypatch.delenv("LAC_TEST_FAIL_RANK")
    assert launch.relay(2, CHILD, []) == 0


def test_nccl_ranks_beyond_gpus_refused():
    with pytest.raises(launch.LaunchError):
        launch.check_devices(8, "nccl", 1)
    with pytest.raises(launch.LaunchError):
        launch.check_devices(0, "gloo", 1)
    launch.check_devices(8, "nccl", 8)
    launch.check_devices(2, "gloo", 1)           # gloo rehearsals may share a GPU


def test_bench_refuses_more_gpus_than_visible():
    """bench.py itself, no GPU here: --gpus 2 under nccl exits 2 before any rank starts."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["LAC_DIST_BACKEND"] = "nccl"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr
    assert "needs 2 GPUs" in p.stderr


def test_workload_labels_follow_baseline_configs():
    """bench.py names the BASELINE.json config a run measures: c2..c5 by
    vocab, streams per GPU and GPU count -- `--gpus 8 --vocab 128256` is c5."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.workload_name(32000, 1, 1) == "c2"
    assert bench.workload_name(32000, 4096, 1) == "c3"
    assert bench.workload_name(32000, 4096, 8).startswith("c3 weak-scaled over 8")
    assert bench.workload_name(128256, 4096, 1) == "c4"
    assert bench.workload_name(128256, 4096, 8) == "c5"
    assert bench.workload_name(128256, 4096, 2).startswith("c5 shape on 2 GPUs")
    assert bench.workload_name(1000, 7, 1) == "custom"
