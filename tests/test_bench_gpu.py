"""Regression check of bench.py's own multi-rank path:
the N > 1 branch of train_line and launch_ranks are exactly what the driver's
8-GPU SCALE run executes (`bench.py --gpus N` under torch.distributed.run).
Here two ranks share the one GPU of the box over gloo (RCCL needs one GPU per
rank); the collective sequence, the gradient buckets, the barrier and the
max-over-ranks timing are the production ones.  Reference: the commented-out
MirroredStrategy line, audiomodel.py:498-500."""
import json
import math
import os
import re
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_two_ranks_gloo():
    if torch.cuda.device_count() < 1:  # counting devices does not initialise HIP
        pytest.skip("no GPU")
    env = dict(os.environ, ACFE_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "2", "--batch", "32", "--steps", "3",
           "--warmup", "1", "--no-cpu-baseline", "--no-extra"]
    r = subprocess.run(cmd, cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints ONE JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 64 and out["steps"] == 3 and out["warmup"] == 1
    assert len(out["per_rank_s"]) == 2 and all(v > 0 for v in out["per_rank_s"])
    # value = all ranks' clips / the slowest rank's time
    assert out["value"] == pytest.approx(64 * 3 / max(out["per_rank_s"]), rel=2e-3)
    ga = out["grad_allreduce"]
    assert ga is not None and ga["buckets"] >= 3 and ga["overlapped_with_backward"]
    assert math.isfinite(out["final_loss"])
    m = re.search(r"bench rank 1/2: .* loss (\S+)", r.stderr)
    assert m, r.stderr[-2000:]
    assert math.isfinite(float(m.group(1)))
    assert out["switches"]["env"].get("ACFE_DIST_BACKEND") == "gloo"
