"""Drop-in CLI / Hand policy (main.py:51-75, control/hand.py:7-21): host logic, no GPU."""
import builtins

from rein48_amd.control.hand import Hand
from rein48_amd.main import parse


def test_cli_flags_like_reference():
    assert parse(["-c", "rand", "-v", "y"]) == ("rand", True)
    assert parse(["-c", "R", "-v", "n"]) == ("rand", False)
    assert parse([]) == ("hand", True)
    assert parse(["--control", "whatever"]) == ("hand", True)


def test_hand_reprompts_until_valid(monkeypatch, capsys):
    answers = iter(["x", "", "up"])
    monkeypatch.setattr(builtins, "input", lambda *a: next(answers))
    assert Hand.hand_control([[0]]) == "up"
    assert capsys.readouterr().out.count("[Error]") == 2
