"""Whole-episode evaluation of a policy: main.py's play() loop (nevertiree/Rein48 main.py:11-48) on
many boards at once -- every board starts from Game.reset (GameClient.py:33-38), is stepped with the
policy's action until game over (no auto-reset; a finished board keeps its final state: a game-over
board has no move that changes it, so later steps leave it as it is, GameClient.py:48-51), and is
scored by its tile sum, np.sum(state_matrix) (main.py:48, a3c.py:214).

policy(boards int8 [n, 16], t) -> actions int8 [n] on the env's device. The reference's own random
policy (control/rand.py) has the fingerprint tests/golden/fingerprint.json (20,000 reference
episodes: mean score 265.1, mean length 142.4), the yardstick for "does a trained policy learn".
"""
import torch

from .env import VecGame


def random_policy(seed=0):
    """Uniform actions (control/rand.py:9-11) from a torch generator on the boards' device."""
    gen = {}

    def policy(boards, t):
        g = gen.get(boards.device)
        if g is None:
            g = gen[boards.device] = torch.Generator(device=boards.device).manual_seed(seed)
        return torch.randint(0, 4, (boards.shape[0],), generator=g, device=boards.device, dtype=torch.int8)
    return policy


@torch.no_grad()
def play_episodes(policy, n_boards, device="cuda:0", seed=0, max_steps=20_000, check_every=50):
    """Play n_boards episodes to game over (or max_steps). Returns a dict: mean / max score (tile
    sum), mean episode length, the fraction that finished, and the distribution of the largest
    tile (exponent -> fraction of boards)."""
    env = VecGame(n_boards, device=device, seed=seed)
    env.reset()
    length = torch.zeros(n_boards, dtype=torch.int32, device=env.boards.device)
    alive = torch.ones(n_boards, dtype=torch.bool, device=env.boards.device)
    t = 0
    while t < max_steps:
        _, _, done = env.step(policy(env.boards, t))
        length += alive.int()
        alive &= done == 0
        t += 1
        if t % check_every == 0 and not bool(alive.any()):
            break
    score = env.score().double()
    top = env.boards.max(dim=1).values.long()
    hist = torch.bincount(top, minlength=18).double() / n_boards
    return {"boards": n_boards, "mean_score": float(score.mean()), "max_score": float(score.max()),
            "mean_length": float(length.double().mean()), "finished": float((~alive).double().mean()),
            "steps_run": t, "max_tile_exponent_hist": {int(e): float(f) for e, f in enumerate(hist) if f > 0}}
