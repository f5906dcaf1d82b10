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


def _run_bench(argv, env_extra=None, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_flag_launches_that_many_ranks():
    """`bench.py --gpus 2` without torch.distributed.run starts 2 ranks itself (gloo dry run:
    barrier, max over ranks) and rank 0 prints ONE JSON line with n_gpus 2."""
    import json
    r = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_reporting"] == 2 and out["steps"] == 3 and out["dry_run"]


def test_gpus_flag_must_match_world_size():
    r = _run_bench(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE 1" in r.stderr


@pytest.mark.parametrize("workload", ["config4", "all"])
def test_config4_multi_rank_dry_run(workload):
    """BASELINE config 4 at N = 2: the run measures config 4's per-GPU shard
    on every rank (65,536 games in all) with its own prefill / stagger / window, and its
    window's example all-gather runs over the ranks (gloo here, RCCL on the GPUs)."""
    import json
    r = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--workload", workload, "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    c4 = out["selfplay"] if workload == "config4" else out["config4_shard"]
    assert out["n_gpus"] == 2 and c4["n_gpus"] == 2 and c4["global_games"] == 65536
    assert c4["window"]["examples_gathered"] == 3 + 4          # rank 0: 3 examples, rank 1: 4
    assert (c4["window"]["prefill"], c4["window"]["stagger"], c4["window"]["window"]) == (84000, 80000, 4000)
    if workload == "all":
        assert out["selfplay"]["global_games"] == 65536 and out["selfplay"]["numMCTSSims"] == 100


def test_phase_defaults_per_workload(bench):
    assert bench.PHASES["config3"] == dict(prefill=6000, stagger=4800, window=10000)
    assert bench.PHASES["config4"]["prefill"] == 84000 and bench.PHASES["config5"]["prefill"] == 40000


def test_window_counters_are_wrap_safe():
    """the per-tree 32-bit header counters (depth_sum wraps after ~40 M simulations
    of a long-lived tree) are differenced per tree modulo 2^32 before summing."""
    import numpy as np
    from splendor.selfplay import SelfPlay
    before = {"depth_sum": np.array([2**32 - 10, 5, 2**31 - 1], np.uint32)}
    after = {"depth_sum": np.array([20, 9, 2**31 + 99], np.uint32)}
    assert SelfPlay.counter_delta(before, after) == {"depth_sum": 30 + 4 + 100}
