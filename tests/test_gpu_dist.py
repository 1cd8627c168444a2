"""Multi-rank bench path on the one-GPU box: ``bench.py --gpus 2`` (which starts
``torch.distributed.run`` on itself) with two ranks sharing cuda:0 over the gloo backend (the device exchange buffers are all-reduced through
host staging; the 8-GPU RCCL run is the driver's).  The 2-rank run shards 2x500 farmer scenarios
with the reference's slicing; its PH trajectory must match a 1-rank run of the same 1000 scenarios
(conv to 1e-9 relative: only the node-sum summation order differs)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "3", "--warmup", "2", "--conv-iters", "0", "--cpu-seconds", "0", "--cm", "2"]


def _run(cmd, env):
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    # the driver reads stdout: exactly one line, the JSON (RCCL's version banner goes to stderr)
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    return json.loads(lines[0])


def test_two_ranks_match_one_rank():
    env = dict(os.environ, PHG_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    one = _run([sys.executable, "bench.py", "--scen", "1000"] + ARGS, env)
    # bench.py starts torch.distributed.run on itself for --gpus 2 (the driver's N-GPU command)
    two = _run([sys.executable, "bench.py", "--gpus", "2", "--scen", "500"] + ARGS, env)
    assert two["n_gpus"] == 2 and two["config"]["scenarios"] == 1000
    assert len(two["per_rank"]["pdhg_ms_per_step"]) == 2
    assert one["config"]["scenarios"] == 1000
    assert two["value"] > 0
    c1, c2 = one["conv_at_end"], two["conv_at_end"]
    assert abs(c1 - c2) <= 1e-9 * max(1.0, abs(c1)), (c1, c2)


def test_rccl_backend_single_rank_matches():
    """The production multi-GPU code path -- nccl (= RCCL) process group, TorchComm, the packed
    device exchange all-reduced by RCCL on torch's stream, the conv run's collectives -- on ONE rank
    (PHG_FORCE_DIST=1: a one-GPU box cannot hold two RCCL ranks).  A one-rank SUM is the identity,
    so the PH trajectory equals the single-GPU path's bit for bit."""
    args = ["--steps", "3", "--warmup", "2", "--conv-iters", "400", "--cpu-seconds", "0", "--cm", "2",
            "--scen", "1000"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("PHG_DIST_BACKEND", None)
    plain = _run([sys.executable, "bench.py"] + args, env)
    forced = _run([sys.executable, "bench.py"] + args, dict(env, PHG_FORCE_DIST="1"))
    assert forced["n_gpus"] == 1 and forced["config"]["scenarios"] == 1000
    assert forced["conv_at_end"] == plain["conv_at_end"]
    tp, tf = plain["time_to_conv"], forced["time_to_conv"]
    assert tf["ph_iters"] == tp["ph_iters"] and tf["conv"] == tp["conv"] and tf["Eobj"] == tp["Eobj"]
