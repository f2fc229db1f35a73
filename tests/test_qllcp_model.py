"""The soundness argument of SAS_ALGO_QUAD_LLCP (k_sa_quad_llcp, csrc/sas_search.hip) on the CPU:
tools/qllcp_model.py restates the kernel's routing invariants (leaf k of the first suffix whose
16-char key is >= K16, the leaf of K16 + 1), its leaf counts, L0 / U / s0 / kappa and the LLCP
walk with its substituted lcps; every tie compare asserts that the chars it skips equal q's,
and every answer equals the oracle's binary_search (sas/sa_search.rs:98-112).  Random, all-A,
periodic, planted-repeat and substituted-copy texts; the repetitive ones must reach the walk."""
import importlib.util
import os

import numpy as np
import pytest


def _model():
    path = os.path.join(os.path.dirname(__file__), "..", "tools", "qllcp_model.py")
    spec = importlib.util.spec_from_file_location("qllcp_model", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("next_mode", [0, 1, 2])
def test_quad_llcp_model_matches_oracle(next_mode):
    """next_mode: the kernel's SAS_QLLCP_NEXT (the entry after leaf k never read / always /
    only when just leaf k's last entry shares K16, the shipped policy)."""
    M = _model()
    M.NEXT_MODE = next_mode
    rng = np.random.default_rng(3)
    blk = rng.integers(0, 4, 700, dtype=np.uint8)
    st = M.run("random", rng.integers(0, 4, 3000, dtype=np.uint8))
    assert st["one"] > 0
    st = M.run("all_A", np.zeros(2000, np.uint8), nq=100)
    assert st["reads"] > 0
    M.run("period_7", np.tile(rng.integers(0, 4, 7, dtype=np.uint8), 400), nq=150)
    st = M.run("repeats", np.concatenate([blk, rng.integers(0, 4, 30, dtype=np.uint8), blk, blk[:500], blk]))
    assert st["reads"] > 0 and st["kU_descents"] > 0
    sub = np.tile(rng.integers(0, 4, 300, dtype=np.uint8), 8)
    sub[rng.integers(0, len(sub), 25)] = rng.integers(0, 4, 25)
    st = M.run("copies_subst", sub)
    assert st["reads"] > 0
