from .segment import Segment  # noqa: F401
