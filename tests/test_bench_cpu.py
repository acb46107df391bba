"""CPU: bench.py's multi-GPU launch contract (no GPU is touched).

* ``--gpus N`` that disagrees with the launcher's WORLD_SIZE fails non-zero before anything
  initialises the GPU;
* ``--gpus N`` without torchrun's env re-launches itself as an N-rank
  ``python -m torch.distributed.run`` child (a subprocess; the parent never touches the GPU)
  and returns the child's exit code;
* the host record of the CPU baseline names the CPU model and both core counts.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_world_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-budget", "0",
                        "--mappo", ""], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_launch_ranks_starts_torchrun_child(monkeypatch):
    import bench

    seen = {}

    def fake_call(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "5"])

    class A:
        gpus, cpu_budget = 4, 0.0

    assert bench.launch_ranks(A()) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]
    assert os.path.basename(cmd[-5]) == "bench.py"
    assert "MARLSAT_BENCH_CPU_JSON" not in seen["env"]  # cpu_budget 0: no baseline file


def test_host_cpu_record(monkeypatch):
    import bench

    monkeypatch.setenv("MARLSAT_CPU_BASELINE_CORES", "3")
    h = bench.host_cpu()
    assert h["cpu_model"] and h["affinity_cores"] >= 1
    assert h["cores"] == min(3, h["affinity_cores"]) and h["cap_source"] == "MARLSAT_CPU_BASELINE_CORES"
    monkeypatch.delenv("MARLSAT_CPU_BASELINE_CORES")
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    h = bench.host_cpu()
    assert h["cores"] == min(2, h["affinity_cores"]) and h["cap_source"] == "OMP_NUM_THREADS"
