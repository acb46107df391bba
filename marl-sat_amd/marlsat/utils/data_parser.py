"""DIMACS CNF input (drop-in for src/utils/data_parser.py) + size-class grouping for the device pool.

``parse_cnf`` / ``parse_sol`` / ``load_cnf_problems`` return what the reference's functions
return (data_parser.py:8-42, :44-56, :59-72) for every file the reference accepts:
``(num_vars, num_clauses, clauses)`` with each clause line's trailing ``0`` dropped, and
``[{"num_vars", "num_clauses", "clauses", "name"}]`` over the sorted ``*.cnf`` names.
Two deliberate differences, both on inputs the reference mishandles:
  * a SATLIB ``%`` trailer line ends the clause section (the reference raises
    ``ValueError: invalid literal for int()`` on the ``%``);
  * blank lines are skipped (the reference appends an empty clause for each).

``group_problems`` replaces the reference's ``jnp.stack`` of the whole set
(runner:114-118), which requires every problem to share (V, C): problems are grouped
into size classes by exact (num_vars, num_clauses), each an (N_g, C, K) int32 array ready
for ``SATEnv.make_pool`` / ``MixedSATEnv``.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, List, Sequence, Tuple

import numpy as np


def parse_cnf(file_path: str) -> Tuple[int, int, List[List[int]]]:
    """data_parser.py:8-42."""
    clauses: List[List[int]] = []
    num_vars = num_clauses = 0
    with open(file_path, "r") as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line.startswith("c"):
                continue
            if line.startswith("%"):
                break  # SATLIB trailer: "%" then "0"
            if line.startswith("p"):
                parts = line.split()
                num_vars, num_clauses = int(parts[2]), int(parts[3])
                continue
            lits = [int(x) for x in line.split()]
            clauses.append(lits[:-1])  # drop the terminating 0 (one clause per line, as the reference)
    return num_vars, num_clauses, clauses


def parse_sol(file_path: str) -> np.ndarray:
    """data_parser.py:44-56: first line of whitespace-separated 0/1 values -> int32 array."""
    with open(file_path, "r") as f:
        line = f.readline()
    return np.array([int(x) for x in line.strip().split()], dtype=np.int32)


def load_cnf_problems(cnf_data_dir: str) -> List[Dict]:
    """data_parser.py:59-72 (sorted *.cnf names)."""
    names = sorted(f for f in os.listdir(cnf_data_dir) if f.endswith(".cnf"))
    problems = []
    for fname in names:
        v, c, clauses = parse_cnf(os.path.join(cnf_data_dir, fname))
        problems.append({"num_vars": v, "num_clauses": c, "clauses": clauses, "name": fname})
    return problems


def write_cnf(file_path: str, num_vars: int, clauses: Sequence[Sequence[int]], comment: str = "") -> None:
    """DIMACS writer (header + one zero-terminated clause per line)."""
    with open(file_path, "w") as f:
        if comment:
            f.write(f"c {comment}\n")
        f.write(f"p cnf {num_vars} {len(clauses)}\n")
        for cl in clauses:
            f.write(" ".join(str(int(l)) for l in cl) + " 0\n")


def clauses_array(problem: Dict) -> np.ndarray:
    """One problem's clause list -> (C, K) int32 (the reference's jnp.array of the list)."""
    cl = problem["clauses"]
    widths = {len(c) for c in cl}
    if len(widths) != 1:
        raise ValueError(f"{problem.get('name', '?')}: clauses of different widths {sorted(widths)} "
                         "(the reference stacks them into one rectangular array)")
    arr = np.asarray(cl, dtype=np.int32)
    if arr.shape[0] != problem["num_clauses"]:
        raise ValueError(f"{problem.get('name', '?')}: header says {problem['num_clauses']} clauses, "
                         f"found {arr.shape[0]}")
    return arr


def group_problems(problems: Sequence[Dict]) -> "OrderedDict[Tuple[int, int], Dict]":
    """Size classes keyed by (num_vars, num_clauses), in first-seen order:
    {(V, C): {"clauses": (N_g, C, K) int32, "names": [...], "index": [positions in `problems`]}}."""
    out: "OrderedDict[Tuple[int, int], Dict]" = OrderedDict()
    for i, p in enumerate(problems):
        key = (int(p["num_vars"]), int(p["num_clauses"]))
        g = out.setdefault(key, {"clauses": [], "names": [], "index": []})
        g["clauses"].append(clauses_array(p))
        g["names"].append(p.get("name", str(i)))
        g["index"].append(i)
    for key, g in out.items():
        widths = {a.shape[1] for a in g["clauses"]}
        if len(widths) != 1:
            raise ValueError(f"size class {key} mixes clause widths {sorted(widths)}")
        g["clauses"] = np.stack(g["clauses"])
    return out


def split_train_eval(n: int, seed: int, train_frac: float = 0.8):
    """runner:100-108: np.random.RandomState(seed).shuffle(arange(n)); first 80 % train."""
    idx = np.arange(n)
    np.random.RandomState(seed).shuffle(idx)
    k = int(n * train_frac)
    return idx[:k], idx[k:]
