"""Step-by-step equivalence of a multi-rank token stream against the single-GPU model.

The multi-rank path (tensor parallel, layer-sharded pipeline) generated `tokens`
(prompt + continuation).  The single-GPU model is teacher-forced on that very stream:
at every generated position it computes the logits (HIP kernels, f32 residual) and the
reference's selection (repeat penalty over the last `last_n` tokens, argmax).  Each
multi-rank token must equal that argmax, or the reference's top-2 margin at that step
must be within `tol` (a near-tie that the other path's different reduction order or
bf16 hop rounding may legitimately flip).  Teacher forcing means a late divergence is
checked at EVERY later step too, instead of ending the comparison.
"""
from __future__ import annotations

import torch


def teacher_forced_check(model, tokens: list[int], prompt_len: int, penalty: float,
                         last_n: int, tol: float) -> dict:
    from cake_amd.ops import reference as R
    model.reset()
    logits = model.forward(tokens[:prompt_len], 0)
    exact = near = 0
    bad = []
    for i in range(prompt_len, len(tokens)):
        lp = R.apply_repeat_penalty(logits.float(), penalty, tokens[max(0, i - last_n):i]) \
            if penalty != 1.0 else logits.float()
        top2 = torch.topk(lp, 2)
        ref = int(top2.indices[0])
        margin = float(top2.values[0] - top2.values[1])
        got = tokens[i]
        if got == ref:
            exact += 1
        elif float(lp[ref] - lp[got]) <= tol:
            near += 1  # the multi-rank pick is within tol of the reference's best
        else:
            bad.append((i, got, ref, margin, float(lp[ref] - lp[got])))
        if i + 1 < len(tokens):
            logits = model.forward([got], i)
    return {"steps": len(tokens) - prompt_len, "exact": exact, "near_ties": near, "bad": bad}
