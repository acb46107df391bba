"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Runs only in the build container (it reads /root/reference, which never travels
to the GPU box).  Executes the three pieces of the reference that are
importable without JAX:

  * ``generate_sat_cnf``   src/utils/generate_cnf_dataset.py:5-42
      (loaded through ``ast``: importing the module would write 1000 files,
      :60-64) -> generator.json: DIMACS text SHA-256 per (V, C, k, seed)
      plus the full text of the small cases;
  * ``check_satisfiability`` src/utils/check_sat.py:4-43 and
  * ``verify_solution`` / ``parse_cnf_file`` src/test/verify_solutions.py:5-81
      -> clause_truth.npz: per-clause truth (each clause checked alone),
      formula satisfiability and verify_solution verdicts for random and
      satisfying assignments; parse_cnf.json: parsed clause lists;
  * ``SATEnv._find_factors`` / ``_create_agent_groups`` / ``_calculate_obs_dim``
      src/envs/multi_agent_sat_env.py:286-343 (pure Python methods, loaded
      through ``ast`` from the class body -- the module imports jax) ->
      agent_groups.json: the partition of every V in 1..256 for the explicit
      VARS_PER_AGENT values and the auto mode, and the obs dim;
  * ``parse_cnf`` src/utils/data_parser.py:8-42 (pure Python, loaded through
      ``ast`` without the module's jax import) -> data_parser.json: the
      clauses it returns for DIMACS texts the reference accepts.

Usage:  python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import ast
import hashlib
import importlib.util
import itertools
import json
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# (V, C, k, seed): the BASELINE.json sizes with the BASELINE.md seed rule
# seed = 1000*size_id + i, plus small/odd shapes.
GEN_CASES = (
    [(20, 91, 3, s) for s in range(8)]
    + [(50, 218, 3, 1000 + i) for i in range(4)]
    + [(100, 430, 3, 2000 + i) for i in range(4)]
    + [(200, 860, 3, 3000 + i) for i in range(4)]
    + [(8, 20, 3, 7), (5, 9, 2, 11), (3, 4, 1, 5), (35, 149, 3, 42)]
)


def load_generator(ref: str):
    path = os.path.join(ref, "src/utils/generate_cnf_dataset.py")
    tree = ast.parse(open(path).read(), path)
    keep = [n for n in tree.body if isinstance(n, (ast.Import, ast.ImportFrom))
            or (isinstance(n, ast.FunctionDef) and n.name == "generate_sat_cnf")]
    ns: dict = {}
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return ns["generate_sat_cnf"]


def load_defs(ref: str, rel: str, names, cls=None):
    """Function definitions ``names`` (of class ``cls``'s body when given) compiled alone: none of the
    module's imports run.  ``math`` and ``typing`` names are provided for their bodies / annotations."""
    import math
    import typing

    path = os.path.join(ref, rel)
    tree = ast.parse(open(path).read(), path)
    body = tree.body if cls is None else next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls).body
    keep = [n for n in body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert len(keep) == len(names), [n.name for n in keep]
    ns: dict = {"math": math, **{k: getattr(typing, k) for k in ("Tuple", "List", "Dict", "Optional")}}
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return [ns[n] for n in names]


def load_module(ref: str, rel: str, name: str):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ref, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def parse_dimacs(text: str):
    return [[int(t) for t in ln.split()[:-1]] for ln in text.splitlines() if ln and ln[0] not in "cp"]


def brute_force_solution(clauses, V):
    """One satisfying assignment of a small instance (numpy exhaustive search)."""
    cl = np.asarray(clauses)
    idx = np.abs(cl) - 1
    for start in range(0, 1 << V, 1 << 16):
        xs = ((np.arange(start, min(start + (1 << 16), 1 << V))[:, None] >> np.arange(V)) & 1)
        vals = xs[:, idx]
        sat = (((cl > 0) & (vals == 1)) | ((cl < 0) & (vals == 0))).any(-1).all(-1)
        hit = np.nonzero(sat)[0]
        if hit.size:
            return xs[hit[0]].astype(np.uint8)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    gen = load_generator(args.reference)
    chk = load_module(args.reference, "src/utils/check_sat.py", "ref_check_sat")
    ver = load_module(args.reference, "src/test/verify_solutions.py", "ref_verify_solutions")

    # ---- generator ------------------------------------------------------
    gen_out = []
    for (V, C, k, seed) in GEN_CASES:
        text = gen(V, C, k, seed=seed)
        rec = {"V": V, "C": C, "k": k, "seed": seed, "sha256": hashlib.sha256(text.encode()).hexdigest()}
        if V <= 50:
            rec["text"] = text
        gen_out.append(rec)
    with open(os.path.join(HERE, "generator.json"), "w") as f:
        json.dump(gen_out, f, indent=0)

    # ---- clause truth ---------------------------------------------------
    rng = np.random.default_rng(20251031)
    cases = {}
    for ci, (V, C, k, seed) in enumerate([(20, 91, 3, 0), (20, 91, 3, 1), (8, 20, 3, 7), (5, 9, 2, 11),
                                          (50, 218, 3, 1000), (100, 430, 3, 2000), (200, 860, 3, 3000)]):
        clauses = parse_dimacs(gen(V, C, k, seed=seed))
        xs = [rng.integers(0, 2, size=V).astype(np.uint8) for _ in range(6)]
        if V <= 20:
            sol = brute_force_solution(clauses, V)
            assert sol is not None
            xs.append(sol)
            # flip one var of the solution: typically breaks a clause
            bad = sol.copy()
            bad[0] ^= 1
            xs.append(bad)
        xs = np.stack(xs)
        per_clause = np.array([[chk.check_satisfiability([c], x) for c in clauses] for x in xs], dtype=np.uint8)
        formula = np.array([chk.check_satisfiability(clauses, x) for x in xs], dtype=np.uint8)
        verify = np.array([ver.verify_solution(clauses, "".join(map(str, x)))[0] for x in xs], dtype=np.uint8)
        cases[f"c{ci}_clauses"] = np.asarray(clauses, dtype=np.int32)
        cases[f"c{ci}_x"] = xs
        cases[f"c{ci}_clause_sat"] = per_clause
        cases[f"c{ci}_formula_sat"] = formula
        cases[f"c{ci}_verify"] = verify
        cases[f"c{ci}_dims"] = np.array([V, C, k], dtype=np.int32)
    # a hand-built instance with a literal 0 slot and repeated vars (reference quirks)
    quirk = [[1, -2, 0], [3, 3, -1], [-4, 2, 4], [0, 0, 0], [-3, -1, 2]]
    xs = np.array(list(itertools.product([0, 1], repeat=4)), dtype=np.uint8)
    cases["quirk_clauses"] = np.asarray(quirk, dtype=np.int32)
    cases["quirk_x"] = xs
    cases["quirk_clause_sat"] = np.array([[chk.check_satisfiability([c], x) for c in quirk] for x in xs], np.uint8)
    cases["quirk_formula_sat"] = np.array([chk.check_satisfiability(quirk, x) for x in xs], np.uint8)
    np.savez_compressed(os.path.join(HERE, "clause_truth.npz"), **cases)

    # ---- DIMACS parsing (verify_solutions.parse_cnf_file) --------------
    text = "c generated for the golden fixtures\n" + gen(20, 91, 3, seed=3) + "\n"
    with tempfile.NamedTemporaryFile("w", suffix=".cnf", delete=False) as f:
        f.write(text)
        tmp = f.name
    try:
        parsed = ver.parse_cnf_file(tmp)
    finally:
        os.unlink(tmp)
    with open(os.path.join(HERE, "parse_cnf.json"), "w") as f:
        json.dump({"text": text, "clauses": parsed}, f)
    # ---- agent partitions (SATEnv._create_agent_groups, env:286-343) ------------------------------
    import contextlib
    import io

    find_factors, create_groups, obs_dim = load_defs(
        args.reference, "src/envs/multi_agent_sat_env.py",
        ["_find_factors", "_create_agent_groups", "_calculate_obs_dim"], cls="SATEnv")

    class _Env:  # the methods' `self`: only the attributes they read
        _find_factors = find_factors
        _create_agent_groups = create_groups
        _calculate_obs_dim = obs_dim

    parts = []
    for V in range(1, 257):
        for vpa in (None, 1, 2, 3, 4, 5, 7, 8, 10, 12, 16, 25, 64):
            e = _Env()
            with contextlib.redirect_stdout(io.StringIO()):  # the reference prints its mode
                groups = e._create_agent_groups(V, vpa)
            assert list(groups) == [f"agent_{i}" for i in range(len(groups))]
            flat = [v for i in range(len(groups)) for v in groups[f"agent_{i}"]]
            assert flat == list(range(V)), (V, vpa)  # contiguous, in agent order: the sizes say it all
            runs = []  # run-length encoded group sizes [[size, count], ...]
            for i in range(len(groups)):
                n = len(groups[f"agent_{i}"])
                if runs and runs[-1][0] == n:
                    runs[-1][1] += 1
                else:
                    runs.append([n, 1])
            parts.append({"V": V, "vpa": vpa, "runs": runs})
    e = _Env()
    e.num_vars, e.num_clauses = 200, 860
    with open(os.path.join(HERE, "agent_groups.json"), "w") as f:
        json.dump({"partitions": parts, "obs_dim_uf200": e._calculate_obs_dim(),
                   "factors": {str(n): e._find_factors(n) for n in (1, 12, 36, 97, 200, 256)}}, f,
                  separators=(",", ":"))

    # ---- data_parser.parse_cnf (data_parser.py:8-42) ------------------------------------------------
    (ref_parse,) = load_defs(args.reference, "src/utils/data_parser.py", ["parse_cnf"])
    texts = ["c two comments\nc here\n" + gen(20, 91, 3, seed=5) + "\n",
             gen(8, 20, 3, seed=7),  # no trailing newline
             "p cnf 5 3\n  1 -2 3 0  \n-4 5 0\n c indented comment\n2 0\n",  # ragged clauses, spaces
             "c x\np  cnf  3  2 \n1 2 -3 0\n-1 -2 3 0\n"]
    out = []
    for text in texts:
        with tempfile.NamedTemporaryFile("w", suffix=".cnf", delete=False) as f:
            f.write(text)
            tmp = f.name
        try:
            V, C, clauses = ref_parse(tmp)
        finally:
            os.unlink(tmp)
        out.append({"text": text, "num_vars": V, "num_clauses": C, "clauses": clauses})
    with open(os.path.join(HERE, "data_parser.json"), "w") as f:
        json.dump(out, f)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    sys.exit(main())
