"""Public model surface (reference robusta_krr/api/models.py:1-17).

Result / Severity / ResourceScan (the downstream O(objects) bookkeeping,
SURVEY.md §8f "next" rank 3) are not part of this build yet.
"""
from krr_amd.core.abstract.strategies import HistoryData, ResourceRecommendation, RunResult
from krr_amd.core.models.allocations import RecommendationValue, ResourceAllocations, ResourceType
from krr_amd.core.models.objects import K8sObjectData

__all__ = [
    "ResourceType",
    "ResourceAllocations",
    "RecommendationValue",
    "K8sObjectData",
    "ResourceRecommendation",
    "HistoryData",
    "RunResult",
]
