"""float64 numpy restatement of the reference A3C maths -- TEST INFRASTRUCTURE ONLY.

nevertiree/Rein48 algorithm/a3c/a3c.py cannot run (a3c.py:8 imports the missing
game.game_cli; TensorFlow 1.x is not installed), so the TF parts of this restatement (net,
losses, optimiser) are "parity unpinned": they follow the reference's formulas line by line,
and tests/test_a3c.py checks the product (PyTorch-ROCm + HIP kernels) against them within fp32
tolerance. Two parts ARE pinned (tests/golden/a3c_golden.json, tests/golden/make_a3c_golden.py):
target_values by the reference's own _get_target_value_list executed on 48 seeded reward lists,
and choose_action by numpy's np.random.choice in the a3c.py:89-93 call form.

  net_forward        a3c.py:136-169  actor 16->64 relu6 ->(dropout = identity)-> 64->4 relu -> softmax;
                                      critic 16->64 relu6 -> 64->1; input = raw tile values
  target_values      a3c.py:246-256  reverse discounted scan, gamma 0.9, LAST REWARD DROPPED
  loss_literal       a3c.py:99-123   the TF graph's shapes taken literally: action [B,1] ->
                                      one_hot [B,1,4] broadcasts log(p)[B,4] to [B,B,4] (survey §8 a14)
  loss_textbook      the usual -mean(beta*H + td*log p[a]) and mean(td^2)
  rmsprop_tf1        a3c.py:264-265  tf.train.RMSPropOptimizer(1e-3): decay .9, momentum 0,
                                      eps 1e-10 inside the sqrt, ms slot initialised to ONES
  choose_action      a3c.py:89-93    np.random.choice over the softmax: first k with cdf > u
"""
import numpy as np

ENTROPY_BETA = 0.001  # a3c.py:21
GAMMA = 0.9           # a3c.py:247


def relu6(x):
    return np.minimum(np.maximum(x, 0.0), 6.0)


def softmax(z):
    z = z - z.max(axis=-1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=-1, keepdims=True)


def board_values(boards):
    """int8 exponent boards [B,16] -> raw tile values [B,16] float64 (a3c.py:139 feeds raw values)."""
    b = np.asarray(boards).astype(np.int64)
    return np.where(b > 0, np.left_shift(1, b), 0).astype(np.float64)


def net_forward(params, x):
    """params: dict of a_w1[16,64] a_b1[64] a_w2[64,4] a_b2[4] c_w1[16,64] c_b1[64] c_w2[64,1] c_b2[1]."""
    h = relu6(x @ params["a_w1"] + params["a_b1"])
    logits = np.maximum(h @ params["a_w2"] + params["a_b2"], 0.0)  # ReLU before the softmax (:150-154)
    probs = softmax(logits)
    hc = relu6(x @ params["c_w1"] + params["c_b1"])
    v = hc @ params["c_w2"] + params["c_b2"]
    return probs, v


def target_values(rewards, last_target, gamma=GAMMA, drop_last=True):
    """a3c.py:246-256: targets[T-1] = last_target; targets[t] = r_t + gamma*targets[t+1].
    drop_last=False is the textbook n-step return (targets[t] includes r_{T-1})."""
    r = list(rewards)
    if drop_last:
        out = [last_target]
        for rew in r[:-1][::-1]:
            last_target = rew + gamma * last_target
            out.append(last_target)
        out.reverse()
        return np.asarray(out, np.float64)
    out = []
    for rew in r[::-1]:
        last_target = rew + gamma * last_target
        out.append(last_target)
    out.reverse()
    return np.asarray(out, np.float64)


def loss_literal(probs, v, actions, targets, beta=ENTROPY_BETA):
    """a3c.py:99-123 with the TF broadcasting taken literally (explicit [B,B,4] tensors)."""
    B = probs.shape[0]
    td = targets.reshape(B, 1) - v.reshape(B, 1)                         # [B,1]
    critic = np.mean(td ** 2)
    onehot = np.eye(4)[np.asarray(actions).reshape(B, 1)]               # tf.one_hot([B,1]) -> [B,1,4]
    log_prob = np.sum(np.log(probs) * onehot, axis=1, keepdims=True)    # [B,4]*[B,1,4] -> [B,B,4] -> [B,1,4]
    exp_v = log_prob * td                                               # [B,1,4]*[B,1] -> [B,B,4]
    entropy = -np.sum(probs * np.log(probs + 1e-5), axis=1, keepdims=True)  # [B,1]
    exp_v = beta * entropy + exp_v                                      # -> [B,B,4]
    actor = np.mean(-exp_v)
    return actor, critic


def loss_literal_closed(probs, v, actions, targets, beta=ENTROPY_BETA):
    """Same value in O(B): -beta*mean(H) - (sum_z td_z)(sum_x S[a_x]) / (4 B^2), S[k] = sum_y log p[y,k]."""
    B = probs.shape[0]
    td = targets.reshape(B) - v.reshape(B)
    S = np.log(probs).sum(axis=0)
    H = -np.sum(probs * np.log(probs + 1e-5), axis=1)
    actor = -beta * H.mean() - td.sum() * S[np.asarray(actions).reshape(B)].sum() / (4.0 * B * B)
    return actor, np.mean(td ** 2)


def loss_textbook(probs, v, actions, targets, beta=ENTROPY_BETA):
    B = probs.shape[0]
    td = targets.reshape(B) - v.reshape(B)
    lp = np.log(probs[np.arange(B), np.asarray(actions).reshape(B)])
    H = -np.sum(probs * np.log(probs + 1e-5), axis=1)
    return np.mean(-(beta * H + td * lp)), np.mean(td ** 2)


def rmsprop_tf1(var, grad, ms, mom, lr=1e-3, decay=0.9, momentum=0.0, eps=1e-10):
    """One ApplyRMSProp step (TF1). ms starts at ONES, mom at zeros. Returns (var, ms, mom)."""
    ms = decay * ms + (1.0 - decay) * grad * grad
    mom = momentum * mom + lr * grad / np.sqrt(ms + eps)
    return var - mom, ms, mom


def choose_action(probs, u):
    """np.random.choice(range(4), p=probs) given its uniform u: first k with cdf(k) > u."""
    cdf = np.cumsum(probs, axis=-1)
    return np.minimum((cdf <= np.asarray(u)[..., None]).sum(axis=-1), probs.shape[-1] - 1)


def xavier_uniform(rng, fan_in, fan_out):
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out))


def init_params(seed=0):
    """a3c.py:138 xavier-uniform kernels, TF-default zero biases."""
    rng = np.random.default_rng(seed)
    return {"a_w1": xavier_uniform(rng, 16, 64), "a_b1": np.zeros(64), "a_w2": xavier_uniform(rng, 64, 4),
            "a_b2": np.zeros(4), "c_w1": xavier_uniform(rng, 16, 64), "c_b1": np.zeros(64),
            "c_w2": xavier_uniform(rng, 64, 1), "c_b2": np.zeros(1)}
