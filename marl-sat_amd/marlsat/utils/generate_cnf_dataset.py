"""Planted-solution random k-SAT instances (host-side data producer).

Restates ``generate_sat_cnf`` / ``generate_cnf_dataset_sat`` of the reference
(``src/utils/generate_cnf_dataset.py:5-57``) so that the same seed yields the
byte-identical DIMACS text (pinned by tests/golden/generator.json, produced
from the reference function itself).  Unlike the reference module, importing
this one has no side effects (the reference writes 1000 files at import,
``:60-64``).

Algorithm (stdlib Mersenne Twister, draw order matters):
  1. hidden solution: one coin per var 1..V, in order;
  2. per clause: k distinct vars (``sample``), the index of the literal forced
     to agree with the hidden solution (``randrange``), then one coin per
     other literal for its sign.
"""
from __future__ import annotations

import os
import random
from typing import List, Optional

import numpy as np


def _planted_clauses(num_vars: int, num_clauses: int, k: int, rnd) -> List[List[int]]:
    assert 1 <= k <= num_vars
    hidden = {v: rnd.choice([True, False]) for v in range(1, num_vars + 1)}
    out = []
    for _ in range(num_clauses):
        picked = rnd.sample(range(1, num_vars + 1), k)
        anchor = rnd.randrange(k)
        clause = []
        for pos, v in enumerate(picked):
            positive = hidden[v] if pos == anchor else rnd.choice([True, False])
            clause.append(v if positive else -v)
        out.append(clause)
    return out


def generate_sat_cnf(num_vars: int, num_clauses: int, clause_size: int = 3, seed: Optional[int] = None) -> str:
    """DIMACS text of one guaranteed-satisfiable instance (no trailing newline, like the reference)."""
    rnd = random.Random(seed) if seed is not None else random
    clauses = _planted_clauses(num_vars, num_clauses, clause_size, rnd)
    body = [f"p cnf {num_vars} {num_clauses}"] + [" ".join(map(str, c)) + " 0" for c in clauses]
    return "\n".join(body)


def generate_sat_clauses(num_vars: int, num_clauses: int, clause_size: int = 3,
                         seed: Optional[int] = None) -> np.ndarray:
    """Same instance as ``generate_sat_cnf`` as an int32 (C, k) literal array."""
    rnd = random.Random(seed) if seed is not None else random
    return np.asarray(_planted_clauses(num_vars, num_clauses, clause_size, rnd), dtype=np.int32)


def has_isolated_variable(clauses: np.ndarray, num_vars: int) -> bool:
    """True when some variable 1..num_vars occurs in no clause of the (C, k) literal array."""
    return bool((np.bincount(np.abs(np.asarray(clauses)).ravel() - 1, minlength=num_vars) == 0).any())


def generate_problem_pool(num_vars: int, num_clauses: int, num_problems: int, size_id: int = 0,
                          clause_size: int = 3, skip_isolated: bool = False) -> np.ndarray:
    """(N, C, k) int32 pool with seed = 1000*size_id + i (BASELINE.md §2 input spec).

    skip_isolated: pass over the seeds whose instance leaves a variable in no clause (the generator allows
    it: uf200-860 seed 3090 leaves variable 126 unused) and take the next ones.  Such a variable, assigned
    0, is an all-zero row through every layer of the network while the biases are at their zero init:
    each LayerNorm (learner:27-82, eps 1e-6) then scales its gradient by rsqrt(1e-6) = 1000, and at 16
    layers the reference's gradient reaches ~1e44 (float64 oracle), past fp32 range -- the first Adam
    step of a run that samples it is non-finite in the reference and here alike.
    """
    out, seed = [], 1000 * size_id
    while len(out) < num_problems:
        cl = generate_sat_clauses(num_vars, num_clauses, clause_size, seed)
        seed += 1
        if skip_isolated and has_isolated_variable(cl, num_vars):
            continue
        out.append(cl)
    return np.stack(out)


def generate_cnf_dataset_sat(num_files: int, num_vars: int, num_clauses: int, save_dir: str,
                             seed: Optional[int] = None) -> None:
    """Writes uf{V}-{i:03d}.cnf files; per-file seeds drawn from one master RNG (reference :45-57)."""
    os.makedirs(save_dir, exist_ok=True)
    rnd = random.Random(seed) if seed is not None else random
    for i in range(1, num_files + 1):
        text = generate_sat_cnf(num_vars, num_clauses, clause_size=3, seed=rnd.randrange(1 << 30))
        with open(os.path.join(save_dir, f"uf{num_vars}-{i:03d}.cnf"), "w") as f:
            f.write(text)
