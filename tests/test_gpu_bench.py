"""bench.py's modes on MI355X, checked end to end (each run compares its own output with the
oracle before timing and reports `verified_vs_oracle`).

The dependent-chain mode is the multi-GPU path with an exchange on the
dependency path: run here with one rank, and rehearsed with two ranks on the one GPU of the box
(H264R_BENCH_REHEARSE=1: gloo in place of RCCL, which refuses two ranks on one device) -- the
exchange moves real rows between processes, and chain 0's second picture (which read its first
through the exchange) must equal the oracle's chain.  The default is one group of chains per step;
`--chain-groups 2` overlaps one group's exchange with the next one's decode.  `bench.py --gpus 2` with no launcher starts
its two ranks itself; its default line is the headline workload as replicas with the slice-sharded chain line beside it."""
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
              "--chain", "4", "--chain-groups", "2", "--steps", "2", "--warmup", "1", "--no-n1"],
             env={"H264R_BENCH_REHEARSE": "1"})
    assert d["verified_vs_oracle"] is True
    assert d["n_gpus"] == 2 and d["config"]["bands"] == [[0, 34], [34, 68]]
    assert d["config"]["chain_groups"] == 2          # the exchange of one group beside the next one's decode
    assert d["exchange"]["mode"] == "halo" and d["exchange"]["halo_mb_rows"] >= 1
    # the library's exchange (include/h264r_group.h): one send and one receive per peer and group
    assert d["exchange"]["impl"] == "abi" and d["exchange"]["ops_per_step"] == 4


def test_gpu_bench_gpus2_spawns_its_ranks():
    """`bench.py --gpus 2` with no torchrun: the default N > 1 line -- the headline workload
    (config 3) as replicas, with the slice-sharded config-5 chain line beside it (`slice_sharded`,
    its one-GPU line of the same mode and the CPU baseline of that workload)."""
    d = _run([sys.executable, "bench.py", "--gpus", "2", "--batch", "8", "--chains-per-gpu", "2", "--steps", "2",
              "--warmup", "1", "--latency-pictures", "0", "--cpu-seconds", "1"],
             env={"H264R_BENCH_REHEARSE": "1"})
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "replicas2" and d["config"]["survey_config"] == 3
    assert d["config"]["pictures_per_step"] == 16 and d["verified_vs_oracle"] is True
    assert d["distributed"]["ranks"] == 2 and d["distributed"]["backend"] == "gloo"
    s = d["slice_sharded"]
    assert s["config"]["survey_config"] == 5 and s["config"]["mode"] == "chain" and s["config"]["chains"] == 4
    assert s["config"]["parallelism"] == "slices2" and s["exchange"]["ops_per_step"] == 2   # a send and a receive
    assert s["verified_vs_oracle"] is True and "slice-sharded" in s["metric"]
    assert s["same_mode_n1"]["verified_vs_oracle"] is True and s["same_mode_n1"]["chains"] == 2
    assert s["same_mode_n1"]["cpu_baseline"]["kind"] == "port" and s["scaling_vs_same_mode_n1"] > 0


def test_gpu_bench_chain_four_ranks_rehearsal():
    """Config 4's slice-sharded shape at 4 ranks (its 4 slices, one band each; the two interior
    ranks exchange halo rows with two peers), rehearsed on the box's one GPU (gloo for RCCL)."""
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "4",
              "--master-addr", "127.0.0.1", "--master-port", "29519", "bench.py", "--gpus", "4", "--config", "4",
              "--chain", "8", "--steps", "2", "--warmup", "1", "--no-n1"],
             env={"H264R_BENCH_REHEARSE": "1"})
    assert d["verified_vs_oracle"] is True
    assert d["n_gpus"] == 4 and d["config"]["bands"] == [[0, 17], [17, 34], [34, 51], [51, 68]]
    assert d["exchange"]["mode"] == "halo" and d["exchange"]["halo_mb_rows"] >= 1


def test_gpu_bench_chain_allgather_rehearsal():
    d = _run([sys.executable, "bench.py", "--gpus", "2", "--mode", "chain", "--config", "4", "--chains-per-gpu", "2",
              "--exchange", "allgather", "--steps", "2", "--warmup", "1", "--no-n1"], env={"H264R_BENCH_REHEARSE": "1"})
    assert d["verified_vs_oracle"] is True and d["exchange"]["mode"] == "allgather"
