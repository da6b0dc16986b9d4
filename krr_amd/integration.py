"""Reference-side drop-in: route the reference Runner's fleet fan-out to the HIP path.

The reference's ``Runner`` (robusta_krr/core/runner.py:17-137) holds ``self._strategy``,
built by ``Config.create_strategy()`` (core/models/config.py:48-51) from the strategy
registry (core/abstract/strategies.py:58-73): the reference's own pure-Python
``SimpleStrategy`` (strategies/simple.py:39-49).  Handing that object to
``krr_amd.core.runner.BatchedRunner`` would run ``simple.py:42-49`` per object, so this
module does the translation a maintainer needs:

* ``hip_strategy(reference_strategy)`` — the reference's ``SimpleStrategy`` (exactly that
  class; a subclass overriding ``run()`` is the user's own code) becomes
  ``krr_amd.strategies.simple.SimpleStrategy`` with the SAME settings values.  Only the
  fields the caller set are copied (pydantic v1 ``__fields_set__``), so the two numeric
  paths of SURVEY §0.4 survive: the CLI path (every field set, Decimals) and the
  int-default path (nothing set: ``99`` / ``5`` stay ``int``).
* ``gather_objects_recommendations(runner, objects)`` — replaces
  ``Runner._gather_objects_recommendations`` (runner.py:109-120): the reference's loaders
  fetch every object's history exactly as ``_calculate_object_recommendations``
  (runner.py:88-102) does, then ONE packed kernel pass + native exact-decimal rounding
  (runner.py:49-86) run for the whole fleet, and the reference's own
  ``ResourceAllocations`` come back (NaN -> "?" by its validator, allocations.py:40-41).
  Any other strategy takes the reference's own per-object path unchanged.
* ``install(Runner)`` — patches that method on the reference's ``Runner`` class.

Nothing here falls back to CPU arithmetic: without ``libkrr_amd.so`` or a HIP device the
kernel call raises ``krr_amd._native.NativeUnavailable``.
"""
from __future__ import annotations

import asyncio
import sys
from typing import Any, Optional, Sequence

from krr_amd.core.models.allocations import ResourceType as HipResourceType
from krr_amd.core.runner import BatchedRunner
from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

REFERENCE_SIMPLE = ("robusta_krr.strategies.simple", "SimpleStrategy")
_ORIGINAL_ATTR = "_krr_amd_original_gather"


def hip_strategy(reference_strategy: Any) -> Optional[SimpleStrategy]:
    """The HIP-backed SimpleStrategy equivalent to the reference's, or None for any other
    strategy (custom plugins keep the reference's per-object ``run()``)."""
    cls = type(reference_strategy)
    if (cls.__module__, cls.__name__) != REFERENCE_SIMPLE:
        return None
    settings = reference_strategy.settings
    explicit = {name: getattr(settings, name) for name in getattr(settings, "__fields_set__", ())}
    return SimpleStrategy(SimpleStrategySettings(**explicit))


def _reference_types(runner: Any):
    """The reference's ResourceType / ResourceAllocations, as its runner module imported them
    (runner.py:11), so the results are the reference's own model objects."""
    mod = sys.modules[type(runner).__module__]
    return mod.ResourceType, mod.ResourceAllocations


async def gather_objects_recommendations(runner: Any, objects: Sequence[Any]) -> list:
    """Drop-in body of the reference's ``Runner._gather_objects_recommendations``."""
    RefResourceType, RefResourceAllocations = _reference_types(runner)
    strategy = hip_strategy(runner._strategy)
    if strategy is None:  # the reference's own per-object path (runner.py:109-120)
        original = getattr(type(runner), _ORIGINAL_ATTR, None)
        if original is not None:
            return await original(runner, objects)
        recs = await asyncio.gather(*[runner._calculate_object_recommendations(o) for o in objects])
        return [RefResourceAllocations(requests={rt: r[rt].request for rt in RefResourceType},
                                       limits={rt: r[rt].limit for rt in RefResourceType}) for r in recs]

    settings = runner._strategy.settings

    async def history(obj):  # runner.py:88-102, with the reference's own loaders
        loader = runner._get_prometheus_loader(obj.cluster)
        data = await asyncio.gather(*[
            loader.gather_data(obj, rt, settings.history_timedelta, timeframe=settings.timeframe_timedelta)
            for rt in RefResourceType])
        return {HipResourceType(rt.value): d for rt, d in zip(RefResourceType, data)}

    histories = await asyncio.gather(*[history(o) for o in objects])
    batched = BatchedRunner(strategy, runner.config.cpu_min_value, runner.config.memory_min_value)
    # one fleet-wide kernel pass, off the event loop like the reference's to_thread (runner.py:106)
    results = await asyncio.to_thread(batched.recommend, list(objects), histories)
    out = []
    for r in results:
        out.append(RefResourceAllocations(
            requests={rt: r[HipResourceType(rt.value)].request for rt in RefResourceType},
            limits={rt: r[HipResourceType(rt.value)].limit for rt in RefResourceType}))
    return out


def install(runner_cls: Any = None) -> Any:
    """Route ``runner_cls._gather_objects_recommendations`` (default: the reference's
    ``robusta_krr.core.runner.Runner``) through ``gather_objects_recommendations``.
    Idempotent; returns the class."""
    if runner_cls is None:
        from robusta_krr.core.runner import Runner as runner_cls  # the reference, in its own process
    if getattr(runner_cls, _ORIGINAL_ATTR, None) is None:
        setattr(runner_cls, _ORIGINAL_ATTR, runner_cls._gather_objects_recommendations)

        async def _gather_objects_recommendations(self, objects):
            return await gather_objects_recommendations(self, objects)

        runner_cls._gather_objects_recommendations = _gather_objects_recommendations
    return runner_cls


__all__ = ["gather_objects_recommendations", "hip_strategy", "install"]
