from .simple import SimpleStrategy

__all__ = ["SimpleStrategy"]
