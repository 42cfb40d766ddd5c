from .hand import Hand  # noqa: F401
from .rand import Rand  # noqa: F401
