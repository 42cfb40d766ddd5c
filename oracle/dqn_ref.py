"""TEST INFRASTRUCTURE ONLY -- float64 numpy restatement of the config-5 value-based pieces.

No reference code exists for DQN or the ResNet (README.md:15-17 only names "ResNet + ReLU +
Batch Normalization"; BASELINE config 5 names "ResNet-10 policy bf16, DQN replay"), so parity
here is UNPINNED against the reference: these functions restate the textbook definitions the
build implements, and the GPU path is tested against them.
  onehot        board exponents -> [n, 16, 18] planes
  conv3x3       3x3 convolution, padding 1, on [n, 4, 4, C] (explicit taps)
  resnet10_q    the ResNet10Q forward (rein48_amd/dqn/nets.py) with eval-mode BatchNorm
  td_target     r + gamma (1 - done) Q'(s', argmax)   (DQN / double DQN)
  huber         smooth L1 with delta 1 (torch.nn.functional.smooth_l1_loss, mean)
  egreedy       u < eps -> random action, else the first argmax
"""
import numpy as np

PLANES = 18


def onehot(boards):
    b = np.asarray(boards, np.int64).reshape(-1, 16)
    out = np.zeros((b.shape[0], 16, PLANES))
    np.put_along_axis(out, b[:, :, None], 1.0, axis=2)
    return out


def conv3x3(x, w, b):
    """x [n, 4, 4, ci], w [co, ci, 3, 3], b [co] -> [n, 4, 4, co]."""
    n = x.shape[0]
    xp = np.zeros((n, 6, 6, x.shape[3]))
    xp[:, 1:5, 1:5] = x
    out = np.zeros((n, 4, 4, w.shape[0])) + b
    for dr in range(3):
        for dc in range(3):
            out += np.einsum("nrci,oi->nrco", xp[:, dr:dr + 4, dc:dc + 4], w[:, :, dr, dc])
    return out


def batchnorm_eval(x, p, eps=1e-5):
    return (x - p["mean"]) / np.sqrt(p["var"] + eps) * p["gamma"] + p["beta"]


def resnet10_q(params, boards):
    """params: {"convs": [(w, b), ...9], "bns": [dict(mean, var, gamma, beta)] or None,
    "head": (w [4, 16C], b [4])}. Returns Q [n, 4]."""
    x = onehot(boards).reshape(-1, 4, 4, PLANES)
    relu = lambda t: np.maximum(t, 0.0)
    bn = (lambda k, t: batchnorm_eval(t, params["bns"][k])) if params.get("bns") else (lambda k, t: t)
    convs = params["convs"]
    h = relu(bn(0, conv3x3(x, *convs[0])))
    for blk in range((len(convs) - 1) // 2):
        y = relu(bn(1 + 2 * blk, conv3x3(h, *convs[1 + 2 * blk])))
        h = relu(bn(2 + 2 * blk, conv3x3(y, *convs[2 + 2 * blk])) + h)
    hw, hb = params["head"]
    return h.reshape(h.shape[0], -1) @ hw.T + hb       # flatten position-major, channel-minor


def td_target(reward, done, q_next_target, q_next_online=None, gamma=0.99):
    qt = np.asarray(q_next_target, np.float64)
    a = np.argmax(qt if q_next_online is None else np.asarray(q_next_online), axis=1)
    boot = qt[np.arange(qt.shape[0]), a]
    d = np.zeros(qt.shape[0]) if done is None else np.asarray(done, np.float64)
    return np.asarray(reward, np.float64) + gamma * (1.0 - d) * boot


def huber(x, y):
    d = np.abs(np.asarray(x, np.float64) - np.asarray(y, np.float64))
    return float(np.mean(np.where(d < 1.0, 0.5 * d * d, d - 0.5)))


def egreedy(q, u, rand_action, eps):
    q = np.asarray(q)
    return np.where(np.asarray(u) < eps, np.asarray(rand_action), np.argmax(q, axis=1))
