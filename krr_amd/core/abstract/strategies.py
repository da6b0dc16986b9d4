"""Strategy plugin API — same names, signatures and registry rules as the reference
(robusta_krr/core/abstract/strategies.py:14-89).

  ResourceRecommendation  strategies.py:14-16
  StrategySettings        strategies.py:19-31
  ResourceHistoryData / HistoryData / RunResult   strategies.py:35-37
  BaseStrategy            strategies.py:42-77  (run 54-56, find 58-66,
                          get_all 68-73: DIRECT subclasses only, get_settings_type 75-77)

Addition (optional, not required of plugins): a strategy may implement
``run_batch(histories, objects) -> list[RunResult]``.  The batched runner
(krr_amd.core.runner) calls it once for the whole fleet; strategies without it
get the reference's per-object ``run()`` loop, so custom strategies written
against the reference keep working unchanged.
"""
from __future__ import annotations

import abc
import datetime
from decimal import Decimal
from typing import Generic, Optional, Sequence, TypeVar, get_args

import pydantic.v1 as pd

from krr_amd.core.models.allocations import ResourceType
from krr_amd.core.models.objects import K8sObjectData
from krr_amd.utils.display_name import add_display_name


class ResourceRecommendation(pd.BaseModel):
    request: Optional[Decimal]
    limit: Optional[Decimal]


class StrategySettings(pd.BaseModel):
    history_duration: float = pd.Field(
        24 * 7 * 2, ge=1, description="The duration of the history data to use (in hours)."
    )
    timeframe_duration: float = pd.Field(15, ge=1, description="The step for the history data (in minutes).")

    @property
    def history_timedelta(self) -> datetime.timedelta:
        return datetime.timedelta(hours=self.history_duration)

    @property
    def timeframe_timedelta(self) -> datetime.timedelta:
        return datetime.timedelta(minutes=self.timeframe_duration)


_StrategySettings = TypeVar("_StrategySettings", bound=StrategySettings)
ResourceHistoryData = dict[str, list[Decimal]]
HistoryData = dict[ResourceType, ResourceHistoryData]
RunResult = dict[ResourceType, ResourceRecommendation]

Self = TypeVar("Self", bound="BaseStrategy")


@add_display_name(postfix="Strategy")
class BaseStrategy(abc.ABC, Generic[_StrategySettings]):
    __display_name__: str

    settings: _StrategySettings

    def __init__(self, settings: _StrategySettings):
        self.settings = settings

    def __str__(self) -> str:
        return self.__display_name__.title()

    @abc.abstractmethod
    def run(self, history_data: HistoryData, object_data: K8sObjectData) -> RunResult:
        """Run the strategy to calculate the recommendation"""

    @classmethod
    def find(cls: type[Self], name: str) -> type[Self]:
        """Get a strategy from its name (case-insensitive)."""
        strategies = cls.get_all()
        key = name.lower()
        if key in strategies:
            return strategies[key]
        raise ValueError(f"Unknown strategy name: {name}. Available strategies: {', '.join(strategies)}")

    @classmethod
    def get_all(cls: type[Self]) -> dict[str, type[Self]]:
        from krr_amd import strategies as _  # noqa: F401  (registers the built-in strategies)

        return {sub.__display_name__.lower(): sub for sub in cls.__subclasses__()}

    @classmethod
    def get_settings_type(cls) -> type[StrategySettings]:
        return get_args(cls.__orig_bases__[0])[0]  # type: ignore[attr-defined]


def _defined_in(cls: type, name: str) -> Optional[type]:
    for k in cls.__mro__:
        if name in k.__dict__:
            return k
    return None


def supports_batch(strategy: BaseStrategy) -> bool:
    """True if the strategy's fleet-wide ``run_batch`` hook computes what its ``run()`` does.

    The hook must come from the class that defines ``run()`` or from a subclass of it:
    a user subclass of SimpleStrategy that overrides only ``run()`` inherits
    ``run_batch`` but must still get its own ``run()`` per object, as the reference's
    Runner always calls ``strategy.run()`` (runner.py:106)."""
    if not callable(getattr(strategy, "run_batch", None)):
        return False
    cls = type(strategy)
    rb, r = _defined_in(cls, "run_batch"), _defined_in(cls, "run")
    return rb is not None and (r is None or issubclass(rb, r))


def supports_packed(strategy: BaseStrategy) -> bool:
    """True if the strategy takes the packed-fleet path (kernel + native rounding)."""
    if not supports_batch(strategy) or not callable(getattr(strategy, "format_packed", None)):
        return False
    cls = type(strategy)
    fp, r = _defined_in(cls, "format_packed"), _defined_in(cls, "run")
    return fp is not None and (r is None or issubclass(fp, r))


def run_each(strategy: BaseStrategy, histories: Sequence[HistoryData],
             objects: Sequence[K8sObjectData]) -> list[RunResult]:
    """The reference's per-object loop (runner.py:88-107 minus the I/O)."""
    return [strategy.run(h, o) for h, o in zip(histories, objects)]


AnyStrategy = BaseStrategy[StrategySettings]

__all__ = [
    "AnyStrategy",
    "BaseStrategy",
    "StrategySettings",
    "HistoryData",
    "K8sObjectData",
    "ResourceType",
    "ResourceRecommendation",
    "ResourceHistoryData",
    "RunResult",
]
