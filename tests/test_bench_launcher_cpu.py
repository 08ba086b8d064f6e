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


import pytest


@pytest.mark.parametrize("n", [3, 8])
def test_launches_n_ranks(n):
    """N stub ranks (8: the driver's node), one JSON line, LOCAL_RANK = rank, N processes,
    the side line's all-reduce over all of them."""
    code, lines, err = _run("--gpus", str(n), "--launcher-stub", "ok")
    assert code == 0, err[-3000:]
    assert len(lines) == 1, (lines, err[-3000:])
    res = json.loads(lines[0])
    assert res["n_gpus"] == n
    assert sorted(r[0] for r in res["ranks"]) == list(range(n))
    assert [r[1] for r in sorted(res["ranks"])] == list(range(n))  # LOCAL_RANK = rank
    assert len({r[2] for r in res["ranks"]}) == n  # n processes
    assert res["c4"] == {"value": float(n)}
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
    """Full-size --same-device runs with N >= 3 are refused (look-back-sort stall); a
    reduced-size rehearsal of the 8-rank topology is let through to the launcher."""
    code, lines, err = _run("--gpus", "3", "--same-device", "--launcher-stub", "ok")
    assert code == 2 and not lines
    assert "refused" in err
    code, lines, err = _run("--gpus", "8", "--same-device", "--edges-per-gpu", "250000",
                            "--c4-edges", "2000000", "--c5-edges", "2000000",
                            "--launcher-stub", "ok", timeout=240)
    assert code == 0, err[-3000:]
    assert json.loads(lines[0])["n_gpus"] == 8


def test_rank_crash_propagates_status():
    # rank 1 exits 7 before joining; its peers wait in the rendezvous until the
    # launcher's grace period ends and it kills them
    code, lines, err = _run("--gpus", "2", "--launch-grace", "3", "--launcher-stub", "crash1")
    assert code == 7, err[-3000:]
    assert not lines
    assert "rank 1 exited with status 7" in err


@pytest.mark.parametrize("n,bad", [(2, 1), (8, 7), (8, 0)])
def test_side_line_failure_sets_status_and_list(n, bad):
    """A side line raising on one rank (the last of 8, or rank 0 itself): the headline
    line still prints once, with the error under the line and in side_line_errors, and
    the job exits SIDE_LINE_RC."""
    code, lines, err = _run("--gpus", str(n), "--launcher-stub", "side%d" % bad)
    assert code == 3, err[-3000:]  # bench.SIDE_LINE_RC
    assert len(lines) == 1, (lines, err[-3000:])
    res = json.loads(lines[0])
    assert res["value"] == 1.0 and res["n_gpus"] == n
    assert "injected side-line failure" in res["c4"]["error"]
    assert [e["line"] for e in res["side_line_errors"]] == ["c4"]


def test_rank_crash_of_eight_propagates_status():
    """Rank 5 of 8 exits 7 before joining: the launcher kills the other seven after its
    grace period and reports rank 5's status."""
    code, lines, err = _run("--gpus", "8", "--launch-grace", "3", "--launcher-stub", "crash5",
                            timeout=240)
    assert code == 7, err[-3000:]
    assert not lines
    assert "rank 5 exited with status 7" in err


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_pmc_child_env_pins_the_rank_gpu(monkeypatch):
    """The PMC child of rank r sees only rank r's GPU, through the chain of visibility
    variables the rank itself sees (ROCR_VISIBLE_DEVICES, then HIP_/CUDA_VISIBLE_DEVICES)."""
    b = _bench()
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "2")
    env = b._child_device_env(2)
    assert env["ROCR_VISIBLE_DEVICES"] == "2" and "WORLD_SIZE" not in env and "RANK" not in env
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "4,5,6,7")
    assert b._child_device_env(1)["ROCR_VISIBLE_DEVICES"] == "5"
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3,2")
    env = b._child_device_env(0)
    assert env["ROCR_VISIBLE_DEVICES"] == "7" and "HIP_VISIBLE_DEVICES" not in env


def test_pmc_phases_by_dispatch_order():
    """Each pass: 3 M1 launch pairs (reduce + fixup) then 3 calibration pairs; the
    phases come from dispatch order, whatever the grid sizes."""
    b = _bench()
    rows = []
    for p in range(2):
        d = 100 * p
        for phase_val in (10.0, 1.0):            # m1 launches, then calibration
            for _ in range(3):
                rows.append((p, d, True, "FETCH_SIZE", phase_val))
                rows.append((p, d + 1, False, "FETCH_SIZE", phase_val / 10))
                d += 2
    vals = b.pmc_phase_values(rows, 2)
    assert sorted(vals[("m1", "FETCH_SIZE")]) == sorted([10.0] * 6 + [1.0] * 6)
    assert sorted(vals[("cal", "FETCH_SIZE")]) == sorted([1.0] * 6 + [0.1] * 6)


def test_configs_run_isolated(tmp_path):
    """measure_configs: every config in a child process of its own under a time limit --
    a crash, a stall or garbage is recorded under its key and the others still run."""
    b = _bench()
    stub = tmp_path / "stub.py"
    stub.write_text(
        "import json, sys, time\n"
        "name = sys.argv[sys.argv.index('--configs') + 1]\n"
        "if name == 'crash': raise RuntimeError('boom')\n"
        "if name == 'hang': time.sleep(60)\n"
        "print(json.dumps({'config': name, 'ms': 1.0}))\n")
    t0 = __import__("time").time()
    out = b.measure_configs("cpu", budgets=(("crash", 20), ("hang", 3), ("ok", 20)),
                            script=str(stub))
    assert "boom" in out["crash"]["error"]
    assert out["hang"]["error"] == "exceeded 3 s"
    assert out["ok"]["config"] == "ok" and out["ok"]["ms"] == 1.0
    assert __import__("time").time() - t0 < 40
