"""`bench.py --gpus N` starts its own N ranks when no launcher set WORLD_SIZE
(bench.launch_ranks), the way the reference's multi-GPU example spawns one
process per device (examples/pytorch/graphsage/train_sampling_multi_gpu.py:
193-200,336).  CPU only: the ranks run the launcher stub (gloo, no GPU), which
goes through the same side-line / print / exit-status path as the real run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(*argv, env_extra=None, timeout=200):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH, *argv], capture_output=True, text=True,
                       timeout=timeout, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


def test_launches_n_ranks():
    code, lines, err = _run("--gpus", "3", "--launcher-stub", "ok")
    assert code == 0, err[-3000:]
    assert len(lines) == 1, (lines, err[-3000:])
    res = json.loads(lines[0])
    assert res["n_gpus"] == 3
    assert sorted(r[0] for r in res["ranks"]) == [0, 1, 2]
    assert [r[1] for r in sorted(res["ranks"])] == [0, 1, 2]  # LOCAL_RANK = rank
    assert len({r[2] for r in res["ranks"]}) == 3  # three processes
    assert res["c4"] == {"value": 3.0}
    assert "side_line_errors" not in res


def test_single_gpu_runs_in_process():
    code, lines, err = _run("--gpus", "1", "--launcher-stub", "ok")
    assert code == 0, err[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and len(res["ranks"]) == 1
    assert "launcher:" not in err


def test_world_size_mismatch_is_an_error():
    code, lines, err = _run("--gpus", "4", "--launcher-stub", "ok",
                            env_extra={"WORLD_SIZE": "2", "RANK": "0"})
    assert code == 2 and not lines
    assert "WORLD_SIZE=2" in err


def test_same_device_refused_from_three_ranks():
    code, lines, err = _run("--gpus", "3", "--same-device", "--launcher-stub", "ok")
    assert code == 2 and not lines
    assert "refused" in err


def test_rank_crash_propagates_status():
    # rank 1 exits 7 before joining; its peers wait in the rendezvous until the
    # launcher's grace period ends and it kills them
    code, lines, err = _run("--gpus", "2", "--launch-grace", "3", "--launcher-stub", "crash1")
    assert code == 7, err[-3000:]
    assert not lines
    assert "rank 1 exited with status 7" in err


def test_side_line_failure_sets_status_and_list():
    code, lines, err = _run("--gpus", "2", "--launcher-stub", "side1")
    assert code == 3, err[-3000:]  # bench.SIDE_LINE_RC
    assert len(lines) == 1, (lines, err[-3000:])
    res = json.loads(lines[0])
    assert res["value"] == 1.0 and res["n_gpus"] == 2
    assert "injected side-line failure" in res["c4"]["error"]
    assert [e["line"] for e in res["side_line_errors"]] == ["c4"]
