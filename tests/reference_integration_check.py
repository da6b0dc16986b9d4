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
--loader bodies|grouped, --scan fleet  (INTEGRATION.md §1 switches) the whole
                 ``Runner._collect_result`` runs against a fake Prometheus HTTP session that
                 serves config-1 query_range bodies (plus objects with dropped pods and no
                 pods) and a fake Kubernetes loader whose objects carry current allocations
                 that hit every severity, thresholds exactly included.  The unpatched
                 reference (its own PrometheusLoader.gather_data with Decimal per sample,
                 per-object ResourceScan.calculate) is run first on the same session; with
                 the oracle engine the patched Result must equal it scan for scan (values,
                 severities, object) and in score; with the native engine the patched path
                 must raise NativeUnavailable after the native packer ran (the bodies
                 reached krr_pack_parse, not Decimal()).
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
import krr_amd.core.fleet_query  # noqa: E402,F401
import krr_amd.core.models.result  # noqa: E402,F401
import krr_amd.core.prom_native  # noqa: E402,F401
from krr_amd import _native  # noqa: E402
from krr_amd.utils.prom_decimal import prom_format  # noqa: E402


from _standin import oracle_run_packed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", choices=("native", "oracle"), required=True)
    ap.add_argument("--path", choices=("cli_99_5", "default_int"), default="cli_99_5")
    ap.add_argument("--loader", choices=integration.LOADERS, default="reference")
    ap.add_argument("--scan", choices=integration.SCANS, default="reference")
    ap.add_argument("--objects", type=int, default=100, help="config-1 objects in the collect check")
    ap.add_argument("--exact", action="store_true",
                    help="histories from tests/golden/simple_strategy_exact.json (hand-built Decimals)")
    args = ap.parse_args()
    if args.loader != "reference" or args.scan != "reference":
        return collect_check(args)

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
    exact_cases = []
    if args.exact:  # hand-built HistoryData whose runs the reference completes on this settings path
        with open(os.path.join(HERE, "golden", "simple_strategy_exact.json")) as fh:
            exact_cases = [c for c in json.load(fh)["cases"] if "rounded" in c["results"][args.path]]

    class FakePrometheusLoader:  # prometheus.py:108-155's output for config 1 (or the exact cases)
        async def gather_data(self, obj, resource, period, *, timeframe):
            o = int(obj.name.split("-")[1])
            if args.exact:
                pods = exact_cases[o]["cpu" if resource == ResourceType.CPU else "mem"]
                return {k: [Decimal(s) for s in v] for k, v in pods.items() if v}
            x = cpu if resource == ResourceType.CPU else mem
            key = (o, resource.value)
            if key not in cpu_s:
                cpu_s[key] = {pod: [Decimal(prom_format(float(v))) for v in x[o, p]]
                              for p, pod in enumerate(config1.pod_names(o))}
            return cpu_s[key]

    none = {ResourceType.CPU: None, ResourceType.Memory: None}
    n_obj = len(exact_cases) if args.exact else config1.OBJECTS
    objects = [K8sObjectData(cluster=None, name=f"app-{o:03d}", container="main",
                             pods=(list(exact_cases[o]["cpu"]) if args.exact else config1.pod_names(o)),
                             namespace="default", kind="Deployment",
                             allocations=ResourceAllocations(requests=none, limits=none))
               for o in range(n_obj)]

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
    if args.exact:
        want = [[c["results"][args.path]["rounded"][k] for k in ("cpu_request", "mem_request", "mem_limit")]
                for c in exact_cases]
        want = [["?" if v == "NaN" else v for v in w] for w in want]
        report["n_objects"] = n_obj
    else:
        with open(os.path.join(HERE, "golden", "config1_reference.json")) as fh:
            want = [[w["rounded"]["cpu_request"], w["rounded"]["mem_request"], w["rounded"]["mem_limit"]]
                    for w in json.load(fh)["results"][args.path]]
    report["equals_reference_runner"] = rows(got) == rows(ref)
    report["equals_golden"] = rows(got) == want
    if not report["equals_golden"]:
        report["first_diff"] = next([i, a, b] for i, (a, b) in enumerate(zip(rows(got), want)) if a != b)

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


# ---- the whole _collect_result against a fake Prometheus ---------------------------------------

class FakeResponse:
    def __init__(self, status_code, content):
        self.status_code, self.content = status_code, content


class FakePrometheusSession:
    """Serves /api/v1/query_range for the reference's per-pod queries (prometheus.py:123, :137)
    and the build's grouped ``sum by (pod)`` queries from per-pod float64 arrays."""

    def __init__(self, series, url, headers):
        import re

        self.series = series            # {(resource, pod): float64 array}; absent = no data
        self.url, self.headers = url, headers
        self.calls = 0
        self.params = set()
        self._strs = {}
        self._pod = re.compile(r'pod="([^"]*)"')
        self._pods = re.compile(r'pod=~"([^"]*)"')

    def _values(self, rt, pod, start, step_s):
        from krr_amd.utils.prom_decimal import prom_format

        strs = self._strs.get((rt, pod))
        if strs is None:
            strs = self._strs[(rt, pod)] = [prom_format(float(v)) for v in self.series[(rt, pod)]]
        return [[start + i * step_s + 0.25, v] for i, v in enumerate(strs)]

    def get(self, url, params=None, verify=None, headers=None):
        assert url == f"{self.url}/api/v1/query_range", url
        assert headers == self.headers and verify is True
        self.calls += 1
        q = params["query"]
        self.params.add((params["step"], params["end"] - params["start"]))
        rt = "cpu" if "container_cpu_usage_seconds_total" in q else "memory"
        step_s = int(params["step"][:-1]) * 60
        if q.startswith("sum by (pod) ("):
            pods = self._pods.search(q).group(1).split("|")
            result = [{"metric": {"pod": p}, "values": self._values(rt, p, params["start"], step_s)}
                      for p in pods if (rt, p) in self.series]
        else:
            pod = self._pod.search(q).group(1)
            result = ([{"metric": {}, "values": self._values(rt, pod, params["start"], step_s)}]
                      if (rt, pod) in self.series else [])
        body = {"status": "success", "data": {"resultType": "matrix", "result": result}}
        return FakeResponse(200, json.dumps(body).encode())


class FakePrometheusConnect:
    """The reference's CustomPrometheusConnect (prometheus.py:41-53) over the fake session;
    custom_query_range as prometheus-api-client 0.5.3 implements it [external]."""

    def __init__(self, session):
        self._session, self.url, self.headers, self.ssl_verification = session, session.url, session.headers, True

    def custom_query_range(self, query, start_time, end_time, step, params=None):
        r = self._session.get(f"{self.url}/api/v1/query_range",
                              params={"query": query, "start": round(start_time.timestamp()),
                                      "end": round(end_time.timestamp()), "step": step, **(params or {})},
                              verify=self.ssl_verification, headers=self.headers)
        if r.status_code != 200:
            raise RuntimeError(f"HTTP Status Code {r.status_code}")
        return json.loads(r.content)["data"]["result"]


def collect_check(args):
    import config1
    from make_golden import import_reference

    ResourceType, Config, Runner, SimpleStrategy, SimpleStrategySettings = import_reference()
    from decimal import Decimal

    from robusta_krr.core.integrations.prometheus import PrometheusLoader
    from robusta_krr.core.models.allocations import ResourceAllocations
    from robusta_krr.core.models.objects import K8sObjectData

    cpu, mem = config1.inputs()
    series = {}
    pods_of = {}
    n_obj = max(1, min(args.objects, config1.OBJECTS))
    for o in range(n_obj):
        pods_of[o] = config1.pod_names(o)
        for p, pod in enumerate(pods_of[o]):
            if o % 17 == 5 and p == 1:
                continue  # no series for this pod: dropped (prometheus.py:154)
            series[("cpu", pod)] = cpu[o, p]
            series[("memory", pod)] = mem[o, p]
    session = FakePrometheusSession(series, "http://prometheus.fake:9090", {"Authorization": "Bearer t"})

    with open(os.path.join(HERE, "golden", "config1_reference.json")) as fh:
        golden = json.load(fh)["results"][args.path]
    factors = [None, Decimal("0.4"), Decimal("0.5"), Decimal("0.75"), Decimal(1), Decimal("1.5"), Decimal(2),
               Decimal("2.5"), Decimal("0.3")]

    def current(o, k, rec):
        f = factors[(o + k) % len(factors)]
        return None if f is None else Decimal(rec) * f

    objects = []
    for o in range(n_obj):
        g = golden[o]["rounded"]
        req = {ResourceType.CPU: current(o, 0, g["cpu_request"]), ResourceType.Memory: current(o, 1, g["mem_request"])}
        lim = {ResourceType.CPU: current(o, 2, g["cpu_request"]), ResourceType.Memory: current(o, 3, g["mem_limit"])}
        objects.append(K8sObjectData(cluster=None, name=f"app-{o:03d}", container="main", pods=pods_of[o],
                                     namespace="default", kind="Deployment",
                                     allocations=ResourceAllocations(requests=req, limits=lim)))
    none = {ResourceType.CPU: None, ResourceType.Memory: None}
    objects.append(K8sObjectData(cluster=None, name="no-data", container="main", pods=["gone-0", "gone-1"],
                                 namespace="default", kind="Deployment",
                                 allocations=ResourceAllocations(requests=none, limits=none)))
    objects.append(K8sObjectData(cluster=None, name="no-pods", container="main", pods=[], namespace="other",
                                 kind="Job", allocations=ResourceAllocations(requests=none, limits=none)))

    class FakeKubernetesLoader:  # core/integrations/kubernetes.py's listing, already done
        async def list_clusters(self):
            return None

        async def list_scannable_objects(self, clusters):
            return objects

    def make_runner():
        other = {"cpu_percentile": "99", "memory_buffer_percentage": "5"} if args.path == "cli_99_5" else {}
        cfg = Config(format="json", strategy="simple", log_to_stderr=True, other_args=other)
        r = Runner.__new__(Runner)
        r.config = cfg
        r._strategy = cfg.create_strategy() if args.path == "cli_99_5" else SimpleStrategy(SimpleStrategySettings())
        r._k8s_loader = FakeKubernetesLoader()
        lo = PrometheusLoader.__new__(PrometheusLoader)  # its gather_data, without discovery/kube
        lo.config = cfg
        lo.prometheus = FakePrometheusConnect(session)
        r._prometheus_loaders = {None: lo}
        return r

    def digest(res):
        rows = []
        for sc in res.scans:
            per = []
            for rt in ResourceType:
                for sel in ("requests", "limits"):
                    rec = getattr(sc.recommended, sel)[rt]
                    per.append([str(rec.value), rec.severity.value, type(rec.severity).__module__])
            rows.append([sc.object.name, sc.severity.value, per])
        return {"rows": rows, "score": res.score, "types": sorted({type(x).__module__ + "." + type(x).__name__
                                                                    for x in [res] + list(res.scans)})}

    report = {"engine": args.engine, "path": args.path, "loader": args.loader, "scan": args.scan}
    integration.uninstall(Runner)
    ref = asyncio.run(make_runner()._collect_result())  # the reference, unpatched
    ref_calls = session.calls
    ref_params = sorted(session.params)
    integration.install(Runner, loader=args.loader, scan=args.scan)
    report["collect_patched"] = Runner._collect_result.__qualname__.startswith("install")
    session.calls, session.params = 0, set()
    gather_data_calls = []
    orig_gather_data = PrometheusLoader.gather_data

    async def counting_gather_data(self, *a, **k):
        gather_data_calls.append(1)
        return await orig_gather_data(self, *a, **k)

    PrometheusLoader.gather_data = counting_gather_data
    from krr_amd.core import prom_native

    packed = []
    orig_pack = prom_native.load_library

    def counting_load_library():
        packed.append(1)
        return orig_pack()

    prom_native.load_library = counting_load_library
    import krr_amd.core.fleet_query as fq
    fq.load_library = counting_load_library
    # --engine native: the real engine (it must stop at the kernel call); the oracle stand-in
    # second (--engine oracle adds it; both share the reference run above)
    try:
        asyncio.run(make_runner()._collect_result())
        report["raised"] = None
    except _native.NativeUnavailable as e:
        report["raised"] = "NativeUnavailable"
        report["message"] = str(e)
    report["raised_before_host_packer"] = not packed  # the device packer's context came first
    if args.engine == "oracle":
        from krr_amd.core.engine import SimpleEngine

        SimpleEngine.run_packed = oracle_run_packed
        # the device packer needs the GPU too: the stand-in run packs on the host
        integration.install(Runner, loader=args.loader, scan=args.scan, parser="host")
        packed.clear()
        session.calls, session.params = 0, set()
        got = asyncio.run(make_runner()._collect_result())
        a, b = digest(got), digest(ref)
        report["equals_reference_result"] = a == b
        report["n_scans"] = len(a["rows"])
        report["score"] = a["score"]
        report["types"] = a["types"]
        report["severities"] = sorted({r[1] for r in a["rows"]} | {x[1] for r in a["rows"] for x in r[2]})
        if a != b:
            report["first_diff"] = next([x, y] for x, y in zip(a["rows"], b["rows"]) if x != y) \
                if a["rows"] != b["rows"] else [a["score"], b["score"], a["types"], b["types"]]
    report["http_requests"] = {"reference": ref_calls, "patched": session.calls}
    report["same_window_and_step"] = sorted(session.params) == ref_params
    report["gather_data_calls"] = len(gather_data_calls)
    report["native_packer_used"] = bool(packed)
    print(json.dumps(report))


if __name__ == "__main__":
    main()
