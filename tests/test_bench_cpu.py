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
    # the cgroup's CPU quota bounds the cores reported, however many the affinity mask shows (the GPU box:
    # 256 in the mask, 16 in the quota)
    monkeypatch.delenv("OMP_NUM_THREADS")
    monkeypatch.setattr(bench, "cgroup_cpus", lambda: 1.0)
    h = bench.host_cpu()
    assert h["cores"] == 1 and h["cgroup_cpus"] == 1.0
    assert h["cap_source"] == ("cgroup quota" if h["affinity_cores"] > 1 else "affinity")


def test_world_from_torchrun_without_gpus_flag():
    """torchrun --nproc-per-node N bench.py (no --gpus) takes N from WORLD_SIZE; only an explicit --gpus that
    disagrees is an error; without torchrun's env, --gpus N > 1 launches the ranks."""
    import bench

    assert bench.resolve_world(None, {"WORLD_SIZE": "8"}) == 8
    assert bench.resolve_world(8, {"WORLD_SIZE": "8"}) == 8
    assert bench.resolve_world(2, {"WORLD_SIZE": "8"}) is None
    assert bench.resolve_world(None, {}) == 1
    assert bench.resolve_world(1, {}) == 1
    assert bench.resolve_world(4, {}) == "launch"


def test_side_legs_fit_the_driver_tail():
    """The env side legs and two compact MAPPO legs at 8 ranks close the line within the driver's
    2,000-character tail, which also carries the run's stderr (progress lines, ~350 characters)."""
    import json

    import bench

    kern = "gru_ln_fused_fwd_h2s_kernel (fp16x2, + x3r fixup launch)"
    full = {"metric": "MAPPO updates/sec", "value": 1 / 27.6123456, "unit": "updates/s", "s_per_update": 27.6123456,
            "s_per_update_cycles": [27.6123456, 27.7123456, 27.5123456],
            "samples_per_s": 296.712345, "adam_steps_per_s": 0.579123,
            "phase_ms": {"rollout": 1618.1123, "gae": 122.7123, "ppo_update": 25631.7123, "metrics": 244.5123},
            "config": {"workload": "uf200-860", "num_agents": 25, "max_vars_per_agent": 8, "envs_per_gpu": 4096,
                       "NUM_STEPS": 2, "UPDATE_EPOCHS": 4, "MINIBATCH_SIZE": 2048, "GNN_HIDDEN_DIM": 128,
                       "GNN_NUM_MESSAGE_PASSING_STEPS": 16,
                       "parallelism": "dp8 (env shards; RCCL gradient all-reduce per minibatch)"},
            "roofline": {"bound": "hbm", "achieved": 3107.123456, "peak": 8000.0, "unit": "GB/s", "frac": 0.3884123,
                         "traffic": 3.6e9 * 1.17123, "kernel": kern, "kernel_ms": 1.3168123,
                         "mfma": {"frac": 0.27123}, "per_rank_kernel_ms": [1.3168123 + i * 1e-3 for i in range(8)]},
            "params_check": {"finite": True, "identical": True, "checksum": [123.4567890123, 1234567890123456789]}}
    leg = bench.compact_leg(full, "gpurun_out/bench_mappo_uf200-860_n8_rank0.json")
    env = [{"workload": w, "envs_per_gpu": b, "value": bench._sig(1.234567e8), "kernel_ms": bench._sig(0.0267123),
            "frac": bench._sig(0.612345, 3), "sclk_mhz": 2103.4} for w, b in (("uf50-218", 1024), ("uf100-430", 4096), ("mixed", 1024),
                                                          ("mixed", 8192))]
    tail = json.dumps({"env_other_legs": env, "mappo_other_legs": [leg], "mappo": leg})
    assert len(tail) < 1600, len(tail)
    assert leg["roofline"]["kernel"] == "gru_ln_fused_fwd_h2s_kernel" and leg["config"].endswith(" dp8")
    assert leg["s_min_med_max"] == [27.51, 27.61, 27.71]
