"""Host logic of bench.py (no GPU): the phase-stagger schedule and the algorithmic byte and
FLOP figures its roofline blocks are built on."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("cfg,stagger", [("config3", 4800), ("config5", 32000), ("config4", 40000)])
def test_stagger_marks_stay_on_the_search_grid(bench, cfg, stagger):
    n, B, sims = bench.CONFIGS[cfg]
    ratio = bench.GENBU_ARGS["ratio_fullMCTS"]
    marks = bench.stagger_marks(stagger, 16, sims, ratio)
    its = [i for i, _ in marks]
    assert [j for _, j in marks] == list(range(1, 16))
    assert all(i % (sims // ratio) == 0 for i in its)        # restarts on search boundaries
    assert its == sorted(set(its)) and 0 < its[0] and its[-1] < stagger
    assert its[-1] + its[0] >= stagger - 16 * (sims // ratio)   # spread over ~the whole span


def test_stagger_marks_empty_when_too_short(bench):
    assert bench.stagger_marks(100, 16, 100, 5) == []
    assert bench.stagger_marks(0, 16, 100, 5) == []


def test_algorithmic_figures(bench):
    assert bench.bytes_per_board_step(2) == 846                  # SURVEY §8(d), 2 players
    assert round(bench.bytes_per_rollout(2, 4.8)) == 3698        # ~3.7 KB per simulation
    assert bench.nn_flops_per_eval(2) == 2 * 595328              # 1.19 MFLOP per leaf
