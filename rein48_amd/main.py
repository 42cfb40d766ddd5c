"""Drop-in for nevertiree/Rein48 main.py: `python -m rein48_amd.main -c rand -v y`.

play() is the reference's episode loop (main.py:11-48) over the drop-in Game (GPU kernels);
the score is the tile-value sum (main.py:48). The CLI keeps the reference's flags (main.py:55-71).
"""
import argparse

from .control.hand import Hand
from .control.rand import Rand
from .game.GameClient import Game

# hand-mode banner, the same text main.py:22-33 prints (a "2048" in ASCII art + the key help)
_ART = (r"    ---         ------           /|       /-------\  ",
        r"  /     \     /        \        / |      |         | ",
        r" |       |   |          |      /  |      |         | ",
        r"        /    |          |     /   |       \_______/  ",
        r"      /      |          |    /    |       /       \  ",
        r"    /        |          |   /_____|_____ |         | ",
        r"  /           \        /          |      |         | ",
        r" ---------      ------            |       \_______/  ")
BANNER = "\n".join(("#" * 53,) + _ART + (
    "PLEASE INPUT [ACTION DIRECTION] TO PLAY THIS GAME.",
    "Left: [L] or [l] ", "Right:[R] or [r] ", "Up:   [U] or [u] ", "Down: [D] or [d] ", "#" * 53))


def play(game, control="hand", show_state=False, show_result=True):
    strategy = {"rand": Rand.random_action, "hand": Hand.hand_control}[control]
    if control == "hand":
        show_state, show_result = True, True
        print(BANNER)
    done = False
    while not done:
        if show_state:
            Game.print_terminal(game.state_matrix)
        _, _, done = game.step(strategy(game.state_matrix))
    if show_result:
        Game.print_terminal(game.state_matrix)
    return sum(sum(row) for row in game.state_matrix)


def parse(argv=None):
    ap = argparse.ArgumentParser(description="Play terminal 2048...")
    ap.add_argument("-c", "--control", type=str, dest="control", default="hand", help="Auto-control or hand-control")
    ap.add_argument("-v", "--visual", type=str, dest="visual", default="y")
    args = ap.parse_args(argv)
    control = "rand" if args.control in ("rand", "Rand", "RAND", "r", "R") else "hand"
    visual = args.visual in ("Y", "y", "Yes", "yes")
    return control, visual


def main(argv=None):
    control, visual = parse(argv)
    return play(game=Game(), control=control, show_result=visual)


if __name__ == "__main__":
    main()
