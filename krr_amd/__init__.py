"""krr_amd — MI355X-native KRR SimpleStrategy hot path.

The reference's plugin surface (BaseStrategy / StrategySettings / RunResult /
ResourceRecommendation / ResourceType / K8sObjectData) is mirrored under
krr_amd.core and re-exported from krr_amd.api; the per-container CPU
percentile and memory max run as fleet-wide segmented HIP kernels behind the C
ABI in include/krr_amd.h (bound by krr_amd._native).
"""
__version__ = "0.1.0"
REFERENCE_VERSION = "1.0.0"  # yonahd/krr snapshot this mirrors (pyproject.toml:3)
