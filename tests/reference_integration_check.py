"""Build-container check that the reference's OWN Runner reaches the HIP path once
krr_amd.integration is installed (run as a subprocess by tests/test_integration.py;
needs /root/reference, so it never runs on the GPU box).

    python tests/reference_integration_check.py --engine native|oracle

It imports the reference with the SURVEY §8(c) recipe (tests/golden/make_golden.py),
installs ``krr_amd.integration`` into ``robusta_krr.core.runner.Runner``, and runs the
reference's ``Runner._gather_objects_recommendations`` on the 100 config-1 objects with a
fake PrometheusLoader (the history the real one would return, from the config-1 arrays).

--engine native  the kernel call must raise NativeUnavailable on this GPU-less host: the
                 reference runner was routed to the C ABI, not to simple.py:42-49.
--engine oracle  the device engine is stood in for by the C oracle (test infrastructure):
                 the reference's own ResourceAllocations must equal, string for string,
                 the reference's unpatched per-object path and tests/golden/config1_reference.json;
                 a custom strategy (examples/custom_strategy.py's shape) must keep the
                 reference's per-object path.
Prints one JSON line with the findings.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before the reference import recipe installs its module stubs)

import krr_amd.integration as integration  # noqa: E402  (before the reference's pydantic alias)
from krr_amd import _native  # noqa: E402
from krr_amd.utils.prom_decimal import prom_format  # noqa: E402


def oracle_run_packed(self, fleet, params):
    from krr_amd.core.engine import RawResults
    from oracle import oracle

    cv, cn, cf = oracle.percentile(fleet.cpu.values, fleet.cpu.offsets, params.mode, params.p_num, params.p_den,
                                   params.q, fleet.cpu.gaps_are_nan)
    mv, mn, mf = oracle.seg_max(fleet.mem.values, fleet.mem.offsets, fleet.mem.gaps_are_nan)
    return RawResults(cv, cn, cf.astype(np.uint32), mv, mn, mf.astype(np.uint32))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", choices=("native", "oracle"), required=True)
    ap.add_argument("--path", choices=("cli_99_5", "default_int"), default="cli_99_5")
    args = ap.parse_args()

    import config1
    from make_golden import import_reference

    ResourceType, Config, Runner, SimpleStrategy, SimpleStrategySettings = import_reference()
    from decimal import Decimal

    from robusta_krr.core.abstract.strategies import BaseStrategy, ResourceRecommendation, StrategySettings
    from robusta_krr.core.models.allocations import ResourceAllocations
    from robusta_krr.core.models.objects import K8sObjectData

    integration.install(Runner)
    assert Runner._gather_objects_recommendations.__qualname__.startswith("install"), "not installed"

    cpu, mem = config1.inputs()
    cpu_s = {}

    class FakePrometheusLoader:  # prometheus.py:108-155's output for config 1
        async def gather_data(self, obj, resource, period, *, timeframe):
            o = int(obj.name.split("-")[1])
            x = cpu if resource == ResourceType.CPU else mem
            key = (o, resource.value)
            if key not in cpu_s:
                cpu_s[key] = {pod: [Decimal(prom_format(float(v))) for v in x[o, p]]
                              for p, pod in enumerate(config1.pod_names(o))}
            return cpu_s[key]

    none = {ResourceType.CPU: None, ResourceType.Memory: None}
    objects = [K8sObjectData(cluster=None, name=f"app-{o:03d}", container="main", pods=config1.pod_names(o),
                             namespace="default", kind="Deployment",
                             allocations=ResourceAllocations(requests=none, limits=none))
               for o in range(config1.OBJECTS)]

    def make_runner(strategy=None):
        other = {"cpu_percentile": "99", "memory_buffer_percentage": "5"} if args.path == "cli_99_5" else {}
        cfg = Config(format="json", strategy="simple", log_to_stderr=True, other_args=other)
        r = Runner.__new__(Runner)
        r.config = cfg
        if strategy is not None:
            r._strategy = strategy
        elif args.path == "cli_99_5":
            r._strategy = cfg.create_strategy()  # exactly what Runner.__init__ does (runner.py:22)
        else:
            r._strategy = SimpleStrategy(SimpleStrategySettings())
        r._prometheus_loaders = {None: FakePrometheusLoader()}
        return r

    def rows(allocs):
        return [[str(a.requests[ResourceType.CPU]), str(a.requests[ResourceType.Memory]),
                 str(a.limits[ResourceType.Memory])] for a in allocs]

    report = {"engine": args.engine, "path": args.path}
    runner = make_runner()
    hip = integration.hip_strategy(runner._strategy)
    report["hip_strategy"] = type(hip).__module__ + "." + type(hip).__name__
    report["settings_types"] = {k: type(getattr(hip.settings, k)).__name__
                                for k in ("cpu_percentile", "memory_buffer_percentage")}
    if args.engine == "native":
        try:
            asyncio.run(runner._gather_objects_recommendations(objects))
            report["raised"] = None
        except _native.NativeUnavailable as e:
            report["raised"] = "NativeUnavailable"
            report["message"] = str(e)
        print(json.dumps(report))
        return

    from krr_amd.core.engine import SimpleEngine

    SimpleEngine.run_packed = oracle_run_packed
    got = asyncio.run(runner._gather_objects_recommendations(objects))
    report["result_types"] = sorted({type(a).__module__ + "." + type(a).__name__ for a in got})
    original = getattr(Runner, integration._ORIGINAL_ATTR)
    ref = asyncio.run(original(make_runner(), objects))
    with open(os.path.join(HERE, "golden", "config1_reference.json")) as fh:
        want = [[w["rounded"]["cpu_request"], w["rounded"]["mem_request"], w["rounded"]["mem_limit"]]
                for w in json.load(fh)["results"][args.path]]
    report["equals_reference_runner"] = rows(got) == rows(ref)
    report["equals_golden"] = rows(got) == want

    # a custom strategy keeps the reference's per-object run() (examples/custom_strategy.py)
    class CustomStrategySettings(StrategySettings):
        param_1: Decimal = Decimal(99)

    class CustomStrategy(BaseStrategy[CustomStrategySettings]):
        def run(self, history_data, object_data):
            return {ResourceType.CPU: ResourceRecommendation(request=self.settings.param_1, limit=None),
                    ResourceType.Memory: ResourceRecommendation(request=Decimal(7), limit=Decimal(7))}

    custom = asyncio.run(make_runner(CustomStrategy(CustomStrategySettings()))
                         ._gather_objects_recommendations(objects[:3]))
    report["custom_strategy_rows"] = rows(custom)
    report["custom_strategy_not_routed"] = integration.hip_strategy(CustomStrategy(CustomStrategySettings())) is None
    print(json.dumps(report))


if __name__ == "__main__":
    main()
