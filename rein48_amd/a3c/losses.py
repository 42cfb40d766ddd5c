"""A3C losses over a batch of variable-length rollout segments (time-major [T, n]).

Reference semantics (algorithm/a3c/a3c.py:99-123), per segment of length B:
    td     = target - V                                     [B,1]
    critic = mean(td^2)
    actor  = mean(-(beta*H + log_prob*td))  with the TF shapes taken literally: the action
             placeholder is [B,1] (:57), so one_hot is [B,1,4] and log(p)[B,4]*one_hot broadcasts to
             [B,B,4]. Reduced exactly (oracle/a3c_ref.py):
             actor = -beta*mean(H) - (sum_z td_z) * (sum_k c_k S_k) / (4 B^2),
             S_k = sum_y log p[y,k], c_k = #{x : a_x = k}, H = -sum p log(p + 1e-5).
Textbook: actor = mean(-(beta*H + td*log p[a])), critic = mean(td^2).
In both, the actor's td is a constant for the actor (TF differentiates actor_loss only w.r.t.
actor params, :127-132), hence td.detach() below.

Both losses are sums over time steps of per-step terms once the per-segment scalars
(B, sum td, c_k) are known, so the update runs in time chunks (bounded memory at 2^20 boards x
100 steps) with exactly the same gradient. The batch loss is the mean over segments (each
segment is one reference worker update; the synchronous batch averages them).
"""
import torch

ENTROPY_BETA = 0.001  # a3c.py:21


def segment_stats(values, targets, actions, mask):
    """Per-segment constants from a no-grad pass. values/targets/mask [T,n], actions [T,n] int.
    Returns dict(B [n], td_sum [n], counts [n,4])."""
    m = mask.to(values.dtype)
    B = m.sum(0).clamp(min=1.0)
    td_sum = ((targets - values) * m).sum(0)
    counts = torch.zeros(values.shape[1], 4, dtype=values.dtype, device=values.device)
    counts.scatter_add_(1, actions.long().t(), m.t().contiguous())
    return {"B": B, "td_sum": td_sum, "counts": counts}


def chunk_loss(logits, v, actions, targets, mask, stats, mode="reference", beta=ENTROPY_BETA):
    """Loss contribution of time chunk [t0, t1) for all segments: logits [t,n,4], v/targets/mask [t,n].
    Summing over chunks gives the full batch loss (mean over segments). Returns (actor, critic)."""
    m = mask.to(v.dtype)
    n = v.shape[1]
    B = stats["B"]
    logp = torch.log_softmax(logits if logits.dtype in (torch.float32, torch.float64) else logits.float(), dim=-1)
    p = logp.exp()
    H = -(p * torch.log(p + 1e-5)).sum(-1)                         # a3c.py:114
    td = targets - v
    w = m / B                                                       # per-step weight 1/B within the segment
    if mode == "reference":
        coef = (stats["td_sum"] / (4.0 * B * B)).detach()           # (sum_z td_z) / (4 B^2)
        s_a = (logp * stats["counts"].unsqueeze(0)).sum(-1)         # sum_k c_k log p[y,k]
        actor = (-beta * H * w - coef * s_a * m).sum()
    elif mode == "textbook":
        lp_a = logp.gather(-1, actions.long().unsqueeze(-1))[..., 0]
        actor = (-(beta * H + td.detach() * lp_a) * w).sum()
    else:
        raise ValueError("mode must be 'reference' or 'textbook'")
    critic = (td * td * w).sum()
    return actor / n, critic / n
