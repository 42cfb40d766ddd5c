from .GameClient import Game  # noqa: F401
