"""Which fp16x2 kernel carries the default path's train-cycle error (verdict r05 item 1)?  Runs the headline-shape
teacher-forced train cycle (tests/test_mappo_gpu.py, uf100 A = 10 m = 10 H = 128 L = 16, two Adam steps) with one
fp16x2 kernel family at a time switched to its bf16x3 form, printing the per-step margins of each run.

    python profiles/parity_switch_probe.py [--seeds 4,5,6,7] [case ...]
        (cases: default gru dgrad wgrad planes0 bf16x3; default all; seeds: the test's network / RNG seeds --
        the margin of one run depends on the whole trajectory, so each case is sampled over several)
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
    "bf16x3": {"use_gru_h2": False, "use_dgrad_h2": False, "use_wgrad_h2": False},  # the whole bf16x3 path
    "fp32": "fp32",  # MARLSAT_PRECISION=fp32's path (gnn.set_precision): fp32 MFMA, the reference's order
}
SHAPE = (100, 430, 10, 128, 16, 0, (2, 4, 4, 1))

if __name__ == "__main__":
    from marlsat import _lib
    from marlsat.learners import gnn

    args = sys.argv[1:]
    seeds = [4]
    if args and args[0] == "--seeds":
        seeds = [int(x) for x in args[1].split(",")]
        args = args[2:]
    for label in args or list(CASES):
        if isinstance(CASES[label], str):  # a whole precision path
            prev = gnn.set_precision(CASES[label])
            saved = {k: v for k, v in prev.items() if k != "_code"}
        else:
            saved = {k: getattr(GNNActorCritic, k) for k in CASES[label]}
            for k, v in CASES[label].items():
                setattr(GNNActorCritic, k, v)
            if not GNNActorCritic.use_wgrad_h2:  # the library's weight-gradient path follows
                _lib.check(_lib.lib.msat_set_precision(gnn.PRECISION_CODES["bf16x3"]), "msat_set_precision")
        try:
            for sd in seeds:
                try:
                    print(f"=== {label} seed {sd}: {CASES[label]}", flush=True)
                    cycle(*SHAPE, precision_path=f"fp16x2-{label}-s{sd}", seed=sd)
                    print(f"=== {label} seed {sd}: passed", flush=True)
                except AssertionError as e:
                    print(f"=== {label} seed {sd}: FAILED {str(e)[:300]}", flush=True)
        finally:
            for k, v in saved.items():
                setattr(GNNActorCritic, k, v)
            _lib.check(_lib.lib.msat_set_precision(gnn.PRECISION_CODES[gnn.PRECISION]), "msat_set_precision")
