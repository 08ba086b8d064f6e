"""bench.py at N > 1: a side line (with-exchange, C4) that fails or stalls on one
rank must not take the headline line down (SideLineGuard).  gloo, two CPU ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(mode, budget=300, nproc=2):
    env = dict(os.environ, BUDGET=str(budget), OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % nproc,
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "guard_worker.py"), mode]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, lines, p.stderr


@pytest.mark.parametrize("mode,nproc", [("ok", 2), ("raise", 2), ("raise0", 2), ("ok", 8),
                                         ("raise", 8), ("raiselast", 8), ("raise0", 8)])
def test_side_line_failure_keeps_headline(mode, nproc):
    """World 2 and the driver's 8 ranks: a raise on rank 1, on the last rank or on rank 0
    (the watchdog's own rank) leaves one line with the error while the peers wait in an
    all-reduce."""
    code, lines, err = _run(mode, nproc=nproc)
    # a failed side line keeps the line but not a zero exit status (torchrun
    # reports the ranks' SIDE_LINE_RC as its own failure)
    assert (code == 0) == (mode == "ok"), err[-2000:]
    assert len(lines) == 1, (lines, err[-2000:])
    res = json.loads(lines[0])
    assert res["value"] == 1.0
    if mode == "ok":
        assert res["c4"] == {"value": float(nproc)}
        assert "side_line_errors" not in res
    else:
        assert "injected failure" in res["c4"]["error"]
        assert res["side_line_errors"][0]["line"] == "c4"


@pytest.mark.parametrize("nproc", [2, 8])
def test_side_line_stall_hits_budget(nproc):
    code, lines, err = _run("stall", budget=3, nproc=nproc)
    assert code != 0
    assert len(lines) == 1, err[-2000:]
    assert "exceeded" in json.loads(lines[0])["c4"]["error"]
