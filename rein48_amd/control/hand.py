"""Drop-in for nevertiree/Rein48 control/hand.py (class Hand): the interactive stdin policy.
Prompts until the line is one of the action aliases GameClient accepts (control/hand.py:7-21)."""

VALID = ("UP", "Up", "U", "up", "u", "DOWN", "Down", "D", "down", "d",
         "LEFT", "Left", "L", "left", "l", "RIGHT", "Right", "R", "right", "r")


class Hand:

    @staticmethod
    def hand_control(*args):
        print("Input action direction, then press ENTER button: ", end="")
        action = input()
        while action not in VALID:
            print("\n##########[Error]########## \n"
                  "Input action signal is invalid, you must input valid value...\n"
                  "########################### \n")
            action = input()
        return action
