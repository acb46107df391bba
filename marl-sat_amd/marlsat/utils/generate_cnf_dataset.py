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


def generate_problem_pool(num_vars: int, num_clauses: int, num_problems: int, size_id: int = 0,
                          clause_size: int = 3) -> np.ndarray:
    """(N, C, k) int32 pool with seed = 1000*size_id + i (BASELINE.md §2 input spec)."""
    return np.stack([generate_sat_clauses(num_vars, num_clauses, clause_size, 1000 * size_id + i)
                     for i in range(num_problems)])


def generate_cnf_dataset_sat(num_files: int, num_vars: int, num_clauses: int, save_dir: str,
                             seed: Optional[int] = None) -> None:
    """Writes uf{V}-{i:03d}.cnf files; per-file seeds drawn from one master RNG (reference :45-57)."""
    os.makedirs(save_dir, exist_ok=True)
    rnd = random.Random(seed) if seed is not None else random
    for i in range(1, num_files + 1):
        text = generate_sat_cnf(num_vars, num_clauses, clause_size=3, seed=rnd.randrange(1 << 30))
        with open(os.path.join(save_dir, f"uf{num_vars}-{i:03d}.cnf"), "w") as f:
            f.write(text)
