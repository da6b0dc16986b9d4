"""Config fields the hot path reads (reference robusta_krr/core/models/config.py:18-65).

Only what the strategy boundary and the rounding need is mirrored: the two
minimum values (config.py:26-27, settable by env var as in the reference,
since this is a pydantic BaseSettings) and ``create_strategy`` (config.py:48-51).
Cluster discovery / Prometheus connection settings are accepted and carried,
but this build does not talk to clusters (out of scope).
"""
from __future__ import annotations

from typing import Any, Literal, Optional, Union

import pydantic.v1 as pd

from krr_amd.core.abstract.strategies import AnyStrategy, BaseStrategy


class Config(pd.BaseSettings):
    quiet: bool = pd.Field(False)
    verbose: bool = pd.Field(False)

    clusters: Union[list[str], Literal["*"], None] = None
    namespaces: Union[list[str], Literal["*"]] = pd.Field("*")

    cpu_min_value: int = pd.Field(5, ge=0)  # millicores
    memory_min_value: int = pd.Field(10, ge=0)  # megabytes

    prometheus_url: Optional[str] = pd.Field(None)
    prometheus_auth_header: Optional[str] = pd.Field(None)
    prometheus_ssl_enabled: bool = pd.Field(False)

    format: str = "table"
    strategy: str = "simple"
    log_to_stderr: bool = False

    other_args: dict[str, Any] = pd.Field(default_factory=dict)

    @pd.validator("namespaces")
    def _empty_means_all(cls, v):
        return "*" if v == [] else v

    @pd.validator("strategy")
    def _known_strategy(cls, v: str) -> str:
        BaseStrategy.find(v)  # raises for unknown names
        return v

    def create_strategy(self) -> AnyStrategy:
        strategy_type = AnyStrategy.find(self.strategy)
        settings_type = strategy_type.get_settings_type()
        return strategy_type(settings_type(**self.other_args))  # type: ignore[call-arg]
