"""Which fp16x2 kernel carries the default path's train-cycle error (verdict r05 item 1)?  Runs the headline-shape
teacher-forced train cycle (tests/test_mappo_gpu.py, uf100 A = 10 m = 10 H = 128 L = 16, two Adam steps) with one
fp16x2 kernel family at a time switched to its bf16x3 form, printing the per-step margins of each run.

    python profiles/parity_switch_probe.py [case ...]    (cases: default gru dgrad wgrad planes0; default all)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from marlsat.learners.gnn import GNNActorCritic  # noqa: E402
from test_mappo_gpu import test_train_cycle_every_adam_step_matches_oracle as cycle  # noqa: E402

CASES = {  # label: the switches that differ from the fp16x2 default
    "default": {},
    "gru": {"use_gru_h2": False},  # GRU forward in bf16x3
    "dgrad": {"use_dgrad_h2": False},  # data gradients in bf16x3
    "wgrad": {"use_wgrad_h2": False},  # weight gradients in bf16x3
    "planes0": {"use_planes": False},  # packed rows stored fp32, split by each consumer
}
SHAPE = (100, 430, 10, 128, 16, 0, (2, 4, 4, 1))

if __name__ == "__main__":
    for label in sys.argv[1:] or list(CASES):
        saved = {k: getattr(GNNActorCritic, k) for k in CASES[label]}
        for k, v in CASES[label].items():
            setattr(GNNActorCritic, k, v)
        try:
            print(f"=== {label}: {CASES[label]}", flush=True)
            cycle(*SHAPE, precision_path=f"fp16x2-{label}")
            print(f"=== {label}: passed", flush=True)
        except AssertionError as e:
            print(f"=== {label}: FAILED {str(e)[:300]}", flush=True)
        finally:
            for k, v in saved.items():
                setattr(GNNActorCritic, k, v)
