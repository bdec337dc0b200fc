"""Split-UNet stage placement (parallel/sd_split.py): the FLOP model orders the SDXL
stages as the measured per-rank compute does (profiles/r4_bench_n4_shared_1gpu.json), and
the cost-balanced split is contiguous, covers every stage and minimises the largest rank."""
import itertools

from cake_amd.models.sd.config import get_config
from cake_amd.parallel.sd_split import split_stages, stage_costs


def test_stage_costs_match_measured_shape():
    cfg = get_config("xl")
    c = stage_costs(cfg.unet, cfg.height // 8, cfg.width // 8)
    assert list(c) == ["down.0", "down.1", "down.2", "mid", "up.0", "up.1", "up.2"]
    tot = sum(c.values())
    # measured on one MI355X (4-rank rehearsal): down.0 4 %, down.1+2 27 %, mid+up.0 47 %,
    # up.1+2 22 % of the step's UNet compute
    for keys, frac in ((("down.0",), 0.04), (("down.1", "down.2"), 0.27),
                       (("mid", "up.0"), 0.47), (("up.1", "up.2"), 0.22)):
        assert abs(sum(c[k] for k in keys) / tot - frac) < 0.05, (keys, sum(c[k] for k in keys) / tot)


def test_split_is_contiguous_and_minimax():
    cfg = get_config("xl")
    c = stage_costs(cfg.unet, 128, 128)
    stages = list(c)
    for n in range(1, 9):
        runs = split_stages(stages, n, c)
        assert [r for r, _ in runs] == list(range(min(n, len(stages))))
        assert [s for _, names in runs for s in names] == stages
        assert all(names for _, names in runs)
        worst = max(sum(c[s] for s in names) for _, names in runs)
        # brute force over every contiguous split into the same number of runs
        k = len(runs)
        best = min(max(sum(c[s] for s in stages[a:b]) for a, b in zip((0,) + cuts, cuts + (len(stages),)))
                   for cuts in itertools.combinations(range(1, len(stages)), k - 1))
        assert abs(worst - best) < 1e-6 * best
    # no costs: balanced by count (the old rule)
    assert split_stages(stages, 2) == [(0, stages[:3]), (1, stages[3:])]
