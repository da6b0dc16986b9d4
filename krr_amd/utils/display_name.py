"""Registry names for plugins (reference robusta_krr/utils/display_name.py:6-20).

A class decorated with ``add_display_name(postfix="Strategy")`` reports
``__display_name__`` = its class name without the postfix (``SimpleStrategy`` ->
``Simple``) unless a subclass sets ``__display_name__`` itself.
"""
from __future__ import annotations

from typing import Callable, TypeVar

_T = TypeVar("_T")


class _NameFromClass:
    def __init__(self, postfix: str):
        self._postfix = postfix

    def __get__(self, instance, owner) -> str:
        name = owner.__name__
        n = len(self._postfix)
        return name[:-n] if n and name.lower().endswith(self._postfix.lower()) else name


def add_display_name(*, postfix: str) -> Callable[[type[_T]], type[_T]]:
    def decorate(cls: type[_T]) -> type[_T]:
        cls.__display_name__ = _NameFromClass(postfix)  # type: ignore[attr-defined]
        return cls

    return decorate
