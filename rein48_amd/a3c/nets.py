"""Policy/value networks (PyTorch-ROCm).

ActorCriticMLP  -- the reference network, algorithm/a3c/a3c.py:136-169:
    actor:  Dense 16->64 ReLU6 -> Dropout(0.4) -> Dense 64->4 ReLU -> softmax
    critic: Dense 16->64 ReLU6 -> Dropout(0.4) -> Dense 64->1
    tf.layers.dropout defaults to training=False, so the dropout is the identity; kernels
    xavier-uniform (a3c.py:138), biases zero (TF default). Input = the 16 raw tile values.
ActorCriticCNN  -- BASELINE config 3's "2-layer CNN policy", the trunk of the reference's only CNN
    (algorithm/ddpg/actor.py:51-85: conv 2x2 valid x32 ReLU -> conv 2x2 valid x64 ReLU -> 256),
    with an actor head (256->4, softmax) and a critic head (256->1). Xavier init as in a3c.py
    (the DDPG actor's N(1, 2) init saturates on raw tile values). Both convolutions are written
    as patch-gather + GEMM so the batch (millions of boards) lands on hipBLASLt/MFMA as two large
    GEMMs instead of MIOpen convolutions over 4x4 images.
forward(x[B,16]) returns (logits[B,4], value[B]); logits are what the softmax / the sampling
kernel consume (for the MLP already through the ReLU of a3c.py:153).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _xavier_(layer):
    nn.init.xavier_uniform_(layer.weight)
    nn.init.zeros_(layer.bias)
    return layer


class ActorCriticMLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.a1 = _xavier_(nn.Linear(16, 64))
        self.a2 = _xavier_(nn.Linear(64, 4))
        self.c1 = _xavier_(nn.Linear(16, 64))
        self.c2 = _xavier_(nn.Linear(64, 1))

    def forward(self, x):
        h = F.relu6(self.a1(x))
        logits = F.relu(self.a2(h))
        v = self.c2(F.relu6(self.c1(x)))[..., 0]
        return logits, v

    @torch.no_grad()
    def load_reference_params(self, p):
        """p: oracle/a3c_ref.py layout (kernels [in, out], TF style)."""
        for name, lay in (("a_w1", self.a1), ("a_w2", self.a2), ("c_w1", self.c1), ("c_w2", self.c2)):
            lay.weight.copy_(torch.as_tensor(p[name]).t())
            lay.bias.copy_(torch.as_tensor(p[name.replace("w", "b")]))

    def reference_params(self):
        out = {}
        for name, lay in (("a_w1", self.a1), ("a_w2", self.a2), ("c_w1", self.c1), ("c_w2", self.c2)):
            out[name] = lay.weight.detach().t().double().cpu().numpy()
            out[name.replace("w", "b")] = lay.bias.detach().double().cpu().numpy()
        return out


# patch indices: conv1 (2x2 valid on 4x4 -> 3x3) and conv2 (2x2 valid on 3x3 -> 2x2)
def _patches(h, k):
    out = h - k + 1
    idx = []
    for r in range(out):
        for c in range(out):
            idx.append([(r + dr) * h + (c + dc) for dr in range(k) for dc in range(k)])
    return torch.tensor(idx, dtype=torch.long)


class ActorCriticCNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Linear(4, 32)      # 2x2x1 -> 32
        self.conv2 = nn.Linear(4 * 32, 64)  # 2x2x32 -> 64
        self.actor = nn.Linear(4 * 64, 4)
        self.critic = nn.Linear(4 * 64, 1)
        for lay in (self.conv1, self.conv2, self.actor, self.critic):
            _xavier_(lay)
        self.register_buffer("p1", _patches(4, 2), persistent=False)   # [9, 4]
        self.register_buffer("p2", _patches(3, 2), persistent=False)   # [4, 4]

    def forward(self, x):
        B = x.shape[0]
        h1 = F.relu(self.conv1(x[:, self.p1]))                          # [B, 9, 32]
        h2 = F.relu(self.conv2(h1[:, self.p2].reshape(B, 4, 4 * 32)))   # [B, 4, 64]
        h = h2.reshape(B, 4 * 64)
        return self.actor(h), self.critic(h)[..., 0]


def make_net(kind):
    return {"mlp": ActorCriticMLP, "cnn": ActorCriticCNN}[kind]()
