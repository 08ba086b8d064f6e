"""Examples as tests (the reference's task_example_test.sh runs the
GCN example on Cora): the GCN and GAT training examples on the synthetic Cora
stand-in train to well above chance (7 classes), fused and unfused GAT alike."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, *args):
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "examples", script)] +
                                  list(args), timeout=600)
    return json.loads(out.decode().strip().splitlines()[-1])


def test_gcn_example_learns():
    r = _run("gcn_train.py", "--epochs", "100")
    assert r["test_acc"] > 0.6, r


@pytest.mark.parametrize("unfused", [False, True])
def test_gat_example_learns(unfused):
    r = _run("gat_train.py", "--epochs", "60", *(["--unfused"] if unfused else []))
    assert r["test_acc"] > 0.6, r


@pytest.mark.parametrize("model", ["gat", "rgcn"])
def test_dist_train_example_runs(model):
    """examples/dist_train.py (configs C3 / C5, partition-parallel modules) at 2 %
    of the config size, one process: trains and reports a finite loss."""
    r = _run("dist_train.py", "--model", model, "--scale", "0.02", "--epochs", "2",
             "--warmup", "1")
    assert r["n_gpus"] == 1 and r["epoch_ms"] > 0 and 0 < r["loss"] < 10, r
