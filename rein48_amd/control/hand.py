"""Drop-in for nevertiree/Rein48 control/hand.py (class Hand): the interactive stdin policy.

Hand.hand_control(*args) prompts on stdout and reads lines from stdin until one is an action
alias the env accepts (the string aliases of GameClient.py:140-230; control/hand.py:7-21), then
returns that string unchanged. The prompt and the error banner are the reference's text, so a
user driving main.py by hand sees the same screen.
"""

_DIRECTIONS = ("UP", "DOWN", "LEFT", "RIGHT")
# every spelling per direction: full upper, capitalised, first letter, lower, first letter lower
VALID = tuple(a for d in _DIRECTIONS for a in (d, d.capitalize(), d[0], d.lower(), d[0].lower()))

_PROMPT = "Input action direction, then press ENTER button: "
_INVALID = ("\n##########[Error]########## \n"
            "Input action signal is invalid, you must input valid value...\n"
            "########################### \n")


class Hand:

    @staticmethod
    def hand_control(*args):
        print(_PROMPT, end="")
        line = input()
        while line not in VALID:
            print(_INVALID)
            line = input()
        return line
