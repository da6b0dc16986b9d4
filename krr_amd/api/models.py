"""Public model surface (reference robusta_krr/api/models.py:1-17)."""
from krr_amd.core.abstract.strategies import HistoryData, ResourceRecommendation, RunResult
from krr_amd.core.models.allocations import RecommendationValue, ResourceAllocations, ResourceType
from krr_amd.core.models.objects import K8sObjectData
from krr_amd.core.models.result import ResourceScan, Result, Severity

__all__ = [
    "ResourceType",
    "ResourceAllocations",
    "RecommendationValue",
    "K8sObjectData",
    "ResourceRecommendation",
    "HistoryData",
    "RunResult",
    "Result",
    "Severity",
    "ResourceScan",
]
