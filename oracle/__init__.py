"""CPU oracle for the marl-sat hot path — TEST INFRASTRUCTURE ONLY.

This package restates the reference algorithms of kongqg/marl-sat
(snapshot 2025-10-31) in NumPy / plain Python so the HIP implementation in
``marl-sat_amd/`` can be checked against them.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker (or the timed CPU baseline) — never as the thing
measured or shipped.  The product path (``marlsat``) never imports this package.

Pinning:
  * clause truth / satisfied status is pinned against the reference's own
    pure-Python checkers ``src/utils/check_sat.py:4-43`` and
    ``src/test/verify_solutions.py:38-81`` (fixtures in tests/golden/);
  * the instance generator is pinned byte-for-byte against the reference
    ``generate_sat_cnf`` (``src/utils/generate_cnf_dataset.py:5-42``), loaded by
    AST in this container only (fixtures in tests/golden/);
  * env obs / masks / rewards / GAE / PPO follow the reference source
    line by line but JAX/Flax are absent here, so those parts are
    hand-checked known-answer tests ("parity pinned by KATs", not by
    reference execution).
"""
