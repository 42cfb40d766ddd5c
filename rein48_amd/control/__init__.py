from .rand import Rand  # noqa: F401
