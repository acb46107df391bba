"""Host-side pieces around the hot path (no GPU): DIMACS input (data_parser.py), the
80/20 split, size-class grouping, the flax-msgpack checkpoint codec, config overrides
and the test_solutions.txt line format."""
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN


def test_parse_cnf_matches_reference_parser_fixture(tmp_path):
    """tests/golden/parse_cnf.json holds a DIMACS text and the clause lists the reference's own
    parser (src/test/verify_solutions.py parse_cnf_file) returned for it."""
    from marlsat.utils.data_parser import parse_cnf

    g = json.load(open(os.path.join(GOLDEN, "parse_cnf.json")))
    p = tmp_path / "a.cnf"
    p.write_text(g["text"])
    V, C, clauses = parse_cnf(str(p))
    assert clauses == g["clauses"]
    head = [l for l in g["text"].splitlines() if l.startswith("p")][0].split()
    assert (V, C) == (int(head[2]), int(head[3]))


def test_parse_cnf_satlib_trailer_and_blank_lines(tmp_path):
    from marlsat.utils.data_parser import parse_cnf

    p = tmp_path / "uf3.cnf"
    p.write_text("c SATLIB style\nc second comment\np cnf 3 2\n 1 -2 3 0\n\n-1 2 -3 0\n%\n0\n\n")
    assert parse_cnf(str(p)) == (3, 2, [[1, -2, 3], [-1, 2, -3]])


def test_generator_files_roundtrip_and_loader(tmp_path):
    from marlsat.utils.data_parser import group_problems, load_cnf_problems, write_cnf
    from marlsat.utils.generate_cnf_dataset import generate_cnf_dataset_sat, generate_sat_clauses

    generate_cnf_dataset_sat(5, 20, 91, str(tmp_path), seed=7)
    write_cnf(str(tmp_path / "z50.cnf"), 50, generate_sat_clauses(50, 218, seed=3).tolist(), comment="x")
    probs = load_cnf_problems(str(tmp_path))
    assert [p["name"] for p in probs] == sorted(os.listdir(tmp_path))
    groups = group_problems(probs)
    assert list(groups) == [(20, 91), (50, 218)]
    assert groups[(20, 91)]["clauses"].shape == (5, 91, 3)
    np.testing.assert_array_equal(groups[(50, 218)]["clauses"][0], generate_sat_clauses(50, 218, seed=3))


def test_split_is_the_reference_split():
    from marlsat.utils.data_parser import split_train_eval

    idx = np.arange(37)
    np.random.RandomState(42).shuffle(idx)
    tr, ev = split_train_eval(37, 42)
    np.testing.assert_array_equal(tr, idx[:29])
    np.testing.assert_array_equal(ev, idx[29:])


def test_checkpoint_codec_layout_and_roundtrip(tmp_path):
    """flax serialization rules: arrays -> ExtType(1, packb((shape, dtype name, C bytes))),
    numpy scalars -> ExtType(3, ...), nested dicts stay maps."""
    import msgpack

    from marlsat.utils import checkpoints as ck

    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    tree = {"step": np.asarray(3, np.int32), "params": {"enc": {"kernel": a}},
            "opt_state": {"0": {"count": np.asarray(3, np.int32)}, "1": {}}}
    raw = ck.to_bytes(tree)
    # decode with plain msgpack: the array leaf is ext type 1 holding (shape, "float32", bytes)
    plain = msgpack.unpackb(raw, raw=False)
    ext = plain["params"]["enc"]["kernel"]
    assert isinstance(ext, msgpack.ExtType) and ext.code == 1
    shape, name, buf = msgpack.unpackb(ext.data, raw=False)
    assert shape == [2, 3] and name == "float32" and buf == a.tobytes()
    back = ck.from_bytes(raw)
    np.testing.assert_array_equal(back["params"]["enc"]["kernel"], a)
    assert back["opt_state"]["1"] == {} and int(back["step"]) == 3
    path = ck.save_checkpoint(str(tmp_path / "ckpt"), tree, 0, "latest_model_")
    assert os.path.basename(path) == "latest_model_0"
    got = ck.restore_checkpoint(str(tmp_path / "ckpt"), "latest_model_", None)
    np.testing.assert_array_equal(got["params"]["enc"]["kernel"], a)
    assert ck.restore_checkpoint(str(tmp_path / "missing")) is None


def test_flax_tree_nesting_matches_param_layout():
    from marlsat.learners import params as P
    from marlsat.utils import checkpoints as ck

    flat = P.to_flax(P.init_flat(64, 2, 3, 4, 0, seed=1), 64, 2, 3, 4, 0)
    tree = ck.nest(flat)
    assert set(tree) >= {"encoder", "critic_dense_0", "actor_flip_head_dense", "agent_id_embedding"}
    assert tree["encoder"]["update_c"]["ir"]["kernel"].shape == (128, 64)
    assert "LayerNorm_5" in tree["encoder"]
    back = P.from_flax(ck.flatten(tree), 64, 2, 3, 4, 0)
    np.testing.assert_array_equal(back, P.init_flat(64, 2, 3, 4, 0, seed=1))


def test_config_overrides_and_solution_line(tmp_path):
    from marlsat.runners.mappo_runner import flat_config, load_config, solution_line

    cfg = load_config(os.path.join(os.path.dirname(__file__), "..", "configs", "MAPPO_CONFIG.yaml"),
                      ["training.NUM_UPDATES=3", "loading.inject_bc_model_path=models/bc", "SEED=7"])
    assert cfg["training"]["NUM_UPDATES"] == 3 and cfg["SEED"] == 7
    assert cfg["loading"]["inject_bc_model_path"] == "models/bc"
    fc = flat_config(cfg)
    assert fc["NUM_VARS"] == 35 and fc["GNN_HIDDEN_DIM"] == 128 and fc["MINIBATCH_SIZE"] == 256
    line = solution_line("uf20-01.cnf", True, 17, np.array([1, 0, 1], np.uint8))
    m = re.search(r"Problem: ([\w.-]+), Solved: True, .* Solution: ([01]+)", line.strip())  # verify_solutions.py:107
    assert m.groups() == ("uf20-01.cnf", "101")
    assert solution_line("b.cnf", False, 0, None) == "Problem: b.cnf, Solved: False\n"


@pytest.mark.parametrize("cfg", [
    {"ANNEAL_LR": True, "NUM_UPDATES": 300, "LEARNING_RATE": 1e-4, "LR_START_FACTOR": 1.0, "LR_END_FLOOR": 2e-5},
    {"ANNEAL_LR": True, "NUM_UPDATES": 7, "LEARNING_RATE": 3e-3, "LR_START_FACTOR": 0.5, "LR_END_FLOOR": 1e-5},
    {"ANNEAL_LR": False, "LEARNING_RATE": 5e-4, "NUM_UPDATES": 10},
])
def test_learning_rate_schedule_matches_oracle(cfg):
    from marlsat.learners.mappo_gnn_sat_learner import learning_rate_at
    from oracle import mappo as om

    for count in list(range(0, 20)) + [cfg["NUM_UPDATES"] - 1, cfg["NUM_UPDATES"], 10 * cfg["NUM_UPDATES"]]:
        assert learning_rate_at(count, cfg) == pytest.approx(om.learning_rate(count, cfg), rel=1e-12, abs=0)


@pytest.mark.parametrize("cfg", [
    {"ANNEAL_ENT": True, "NUM_UPDATES": 300, "ENT_COEF": 0.01, "ENT_COEF_END": 0.001, "ANNEAL_ENT_FRAC": 0.333},
    {"ANNEAL_ENT": True, "NUM_UPDATES": 12, "ENT_COEF": 0.05},
    {"ANNEAL_ENT": False, "NUM_UPDATES": 12, "ENT_COEF": 0.005},
])
def test_entropy_schedule_matches_oracle(cfg):
    from marlsat.learners.mappo_gnn_sat_learner import ent_coef_at
    from oracle import mappo as om

    for u in range(0, cfg["NUM_UPDATES"] + 3):
        assert ent_coef_at(u, cfg) == pytest.approx(om.ent_coef(u, cfg), rel=1e-12, abs=1e-15)


def test_agent_partitions_match_reference_fixture():
    """tests/golden/agent_groups.json: SATEnv._create_agent_groups / _find_factors / _calculate_obs_dim
    (env:286-343) run from the reference's own source for every V in 1..256 and each VARS_PER_AGENT
    (None = the auto mode): the build's partition and the oracle's, group for group."""
    import math

    from marlsat.envs.multi_agent_sat_env import _find_factors, create_agent_groups
    from oracle.sat_env import create_agent_groups as oracle_groups

    g = json.load(open(os.path.join(GOLDEN, "agent_groups.json")))
    for rec in g["partitions"]:
        V, vpa = rec["V"], rec["vpa"]
        want, start = {}, 0
        for n, count in rec["runs"]:
            for _ in range(count):
                want[f"agent_{len(want)}"] = list(range(start, start + n))
                start += n
        assert create_agent_groups(V, vpa) == want, (V, vpa)
        assert oracle_groups(V, vpa) == want, (V, vpa)
    for n, f in g["factors"].items():
        assert _find_factors(int(n)) == f
    assert g["obs_dim_uf200"] == 2 * 200 + 860
    # the BASELINE configs: uf200 with VARS_PER_AGENT 8 -> 25 agents of 8
    uf200 = next(r for r in g["partitions"] if r["V"] == 200 and r["vpa"] == 8)
    assert uf200["runs"] == [[8, 25]] and math.ceil(200 / 8) == 25


def test_parse_cnf_matches_reference_data_parser_fixture(tmp_path):
    """tests/golden/data_parser.json: the reference's own ``parse_cnf`` (data_parser.py:8-42) on texts it
    accepts (comments, no trailing newline, ragged clauses, extra spaces in the header and lines)."""
    from marlsat.utils.data_parser import parse_cnf

    for i, rec in enumerate(json.load(open(os.path.join(GOLDEN, "data_parser.json")))):
        p = tmp_path / f"t{i}.cnf"
        p.write_text(rec["text"])
        assert parse_cnf(str(p)) == (rec["num_vars"], rec["num_clauses"], rec["clauses"]), i
