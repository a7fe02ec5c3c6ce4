"""bench.py's modes on MI355X, checked end to end (each run compares its own output with the
oracle before timing and reports `verified_vs_oracle`).

The dependent-chain mode (--chain) is the multi-GPU path with an
exchange on the dependency path: run here with one rank, and rehearsed with two ranks on
the one GPU of the box (H264R_BENCH_REHEARSE=1: gloo in place of RCCL, which refuses two
ranks on one device) -- the exchange moves real bands between processes, and chain 0's
pictures after two exchanges must equal the oracle's chain."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out: str) -> dict:
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def _run(cmd, env=None):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, cwd=ROOT,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return _last_json(r.stdout)


def test_gpu_bench_chain_one_rank():
    d = _run([sys.executable, "bench.py", "--config", "4", "--chain", "4", "--steps", "2", "--warmup", "1"])
    assert d["verified_vs_oracle"] is True
    assert d["config"]["mode"] == "chain" and d["config"]["chains"] == 4 and d["value"] > 0


def test_gpu_bench_chain_two_ranks_rehearsal():
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", "29517", "bench.py", "--gpus", "2", "--config", "4",
              "--chain", "4", "--steps", "2", "--warmup", "1"], env={"H264R_BENCH_REHEARSE": "1"})
    assert d["verified_vs_oracle"] is True
    assert d["n_gpus"] == 2 and d["config"]["bands"] == [[0, 34], [34, 68]]
    assert d["exchange_per_step"]["collectives"] == 3
