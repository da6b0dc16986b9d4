"""K8sObjectData (reference robusta_krr/core/models/objects.py:8-21).

``pods`` fixes the order in which an object's pod series are concatenated into
its segment — the REF_INDEX result depends on it.
"""
from __future__ import annotations

from typing import Optional

import pydantic.v1 as pd

from krr_amd.core.models.allocations import ResourceAllocations


class K8sObjectData(pd.BaseModel):
    cluster: Optional[str]
    name: str
    container: str
    pods: list[str]
    namespace: str
    kind: Optional[str]
    allocations: ResourceAllocations

    def __str__(self) -> str:
        return f"{self.kind} {self.namespace}/{self.name}/{self.container}"

    def __hash__(self) -> int:
        return hash(str(self))
