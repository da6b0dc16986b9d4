"""ResourceType / RecommendationValue / ResourceAllocations
(reference robusta_krr/core/models/allocations.py:13-51).

ResourceType's member ORDER (CPU, then Memory) is part of the contract: the
runner gathers and reports resources in enum order (runner.py:91-102).
"""
from __future__ import annotations

import enum
from decimal import Decimal
from typing import Literal, Optional, Union

import pydantic.v1 as pd

from krr_amd.utils import resource_units


class ResourceType(str, enum.Enum):
    CPU = "cpu"
    Memory = "memory"


RecommendationValue = Union[Decimal, Literal["?"], None]


def _to_recommendation_value(value: Union[Decimal, str, None]) -> RecommendationValue:
    if value is None:
        return None
    if isinstance(value, str):
        return resource_units.parse(value)
    if value.is_nan():  # NaN (no data) is shown as "?" (allocations.py:40-41)
        return "?"
    return value


class ResourceAllocations(pd.BaseModel):
    requests: dict[ResourceType, RecommendationValue]
    limits: dict[ResourceType, RecommendationValue]

    @pd.validator("requests", "limits", pre=True)
    def _normalise(cls, value: dict[ResourceType, Optional[Union[Decimal, str]]]) -> dict:
        return {rt: _to_recommendation_value(v) for rt, v in value.items()}

    @classmethod
    def from_container(cls, container) -> "ResourceAllocations":
        """From a V1Container-like object (``.resources.requests/.limits`` dicts)."""
        res = getattr(container, "resources", None)
        req = getattr(res, "requests", None) or {}
        lim = getattr(res, "limits", None) or {}
        return cls(
            requests={ResourceType.CPU: req.get("cpu"), ResourceType.Memory: req.get("memory")},
            limits={ResourceType.CPU: lim.get("cpu"), ResourceType.Memory: lim.get("memory")},
        )
