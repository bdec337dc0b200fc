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


def test_split_plan_routes_each_skip_once_to_its_consumer():
    """SplitPlan (the split-UNet's message plan): the feature map follows the runs and
    comes back to rank 0, every skip goes exactly once from the rank that pushes it to
    the rank that pops it, and a step over the plan pops the same skips per stage as the
    whole UNet on one rank (labels instead of tensors)."""
    from cake_amd.models.sd.unet import UNet2DConditionModel
    from cake_amd.parallel.sd_split import SplitPlan, skip_counts
    for version in ("xl", "v1-5"):
        cfg = get_config(version)
        model = UNet2DConditionModel(cfg.unet)
        stages = model.stage_names()
        counts = skip_counts(model)
        assert sum(p for p, _ in counts.values()) == sum(q for _, q in counts.values())
        c = stage_costs(cfg.unet, cfg.height // 8, cfg.width // 8)
        ref = None
        for n in range(1, 9):
            runs = split_stages(stages, n, c)
            plan = SplitPlan(stages, counts, runs)
            order = plan.order
            # x: run j -> run j + 1, last -> rank 0
            xs = [k for k, items in plan.channels.items() if "x" in items]
            assert sorted(xs) == sorted(list(zip(order[:-1], order[1:])) +
                                        ([(order[-1], order[0])] if len(order) > 1 else []))
            # every skip exactly once, producer -> consumer, never relayed
            seen = [i for items in plan.channels.values() for i in items if i != "x"]
            assert len(seen) == len(set(seen))
            for i in seen:
                assert (plan.producer[i], plan.consumer[i]) in plan.channels
                assert i in plan.channels[(plan.producer[i], plan.consumer[i])]
            local = [i for i in plan.producer if plan.producer[i] == plan.consumer[i]]
            assert sorted(seen + local) == sorted(plan.producer)
            # one step with labels: same pops per stage as one rank
            popped = _run_labels(plan, stages, counts)
            if ref is None:
                ref = popped
            assert popped == ref, (version, n)


def _run_labels(plan, stages, counts):
    owner = {n: r for r, names in plan.runs for n in names}
    boxes = {k: [] for k in plan.channels}
    popped = {}

    def runner(rank):
        names = [n for n in stages if owner[n] == rank]

        def run(x, skips):
            k = plan.base.get(rank, 0)
            skips = list(skips)
            for n in names:
                push, pop = counts[n]
                popped[n] = [skips.pop() for _ in range(pop)]
                for _ in range(push):
                    skips.append(k)
                    k += 1
                x = x + [n]
            return x, skips
        return run

    def recv_of(rank):
        return lambda a: boxes[(a, rank)].pop(0)

    def send_of(rank):
        def send(b, items, tensors):
            for it, t in zip(items, tensors):
                assert it == "x" or it == t, (it, t)
            boxes[(rank, b)].append(dict(zip(items, tensors)))
        return send

    first = plan.order[0]
    if len(plan.order) == 1:
        out = plan.step(first, [], runner(first), recv_of(first), send_of(first))
    else:
        # rank 0's step receives the output last: run it with a recv that first lets
        # the other ranks run (the sequential pipeline of one step)
        def recv0(a):
            for r in plan.order[1:]:
                plan.step(r, None, runner(r), recv_of(r), send_of(r))
            return boxes[(a, first)].pop(0)
        out = plan.step(first, [], runner(first), recv0, send_of(first))
    assert out == stages  # the feature map went through every stage in order
    assert all(not v for v in boxes.values())
    return popped
