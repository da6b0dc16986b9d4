"""Public plugin-author surface (reference robusta_krr/api/strategies.py:1-3)."""
from krr_amd.core.abstract.strategies import BaseStrategy, StrategySettings

__all__ = ["BaseStrategy", "StrategySettings"]
