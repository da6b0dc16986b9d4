"""Generate golden vectors for the SimpleStrategy hot path BY IMPORTING THE REFERENCE.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden.py        # writes tests/golden/simple_strategy.json

Import recipe: alias pydantic -> pydantic.v1, stub the
kubernetes / prometheus_api_client / cachetools imports that are not on the
arithmetic path, and mount /root/reference/robusta_krr as a bare package so the
kubeconfig loading in robusta_krr/__init__ -> main -> config is bypassed.
Nothing from the reference is copied into the repository: only inputs (as the
strings Prometheus would send) and the reference's outputs are written.

Outputs per case:
  raw       - SimpleStrategy.run() result (Decimal strings), or the exception name
  rounded   - Runner._format_result() of it (runner.py:79-86)
  sorted    - calculate_cpu_proposal over the pre-sorted samples (SORTED_LOWER rule)
  linear    - numpy.percentile(samples, float(p)) (numpy is a third-party oracle)
both for the CLI settings path (Decimal('99'), Decimal('5')) and the default
int path (SimpleStrategySettings()).
"""
from __future__ import annotations

import json
import math
import os
import sys
import types
from decimal import Decimal

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from krr_amd.utils.prom_decimal import prom_format  # noqa: E402


def import_reference():
    import pydantic.v1 as pv1

    sys.modules["pydantic"] = pv1

    class _Any:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, k):
            return _Any()

        def __call__(self, *a, **k):
            return _Any()

    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        m.__getattr__ = lambda k: _Any
        sys.modules[name] = m
        return m

    k8s = stub("kubernetes")
    kc = stub("kubernetes.client")
    stub("kubernetes.client.models")
    kcfg = stub("kubernetes.config", load_incluster_config=lambda: None, load_kube_config=lambda: None)
    stub("kubernetes.config.config_exception", ConfigException=Exception)
    stub("kubernetes.client.api_client")
    stub("kubernetes.client.models.v1_service")
    stub("kubernetes.client.models.v1_ingress")
    stub("prometheus_api_client")
    stub("cachetools", TTLCache=dict)
    k8s.client = kc
    k8s.config = kcfg
    pkg = types.ModuleType("robusta_krr")
    pkg.__path__ = [os.path.join(REF, "robusta_krr")]
    pkg.__version__ = "1.0.0"
    sys.modules["robusta_krr"] = pkg
    from robusta_krr.core.abstract.strategies import ResourceType
    from robusta_krr.core.models.config import Config
    from robusta_krr.core.runner import Runner
    from robusta_krr.strategies.simple import SimpleStrategy, SimpleStrategySettings

    return ResourceType, Config, Runner, SimpleStrategy, SimpleStrategySettings


def dstr(x):
    return None if x is None else str(x)


def main():
    ResourceType, Config, Runner, SimpleStrategy, SimpleStrategySettings = import_reference()
    rng = np.random.default_rng(20260101)

    def cli_strategy(p, b, cpu_min=5, mem_min=10):
        cfg = Config(format="json", strategy="simple", log_to_stderr=True, cpu_min_value=cpu_min,
                     memory_min_value=mem_min, other_args={"cpu_percentile": p, "memory_buffer_percentage": b})
        runner = Runner.__new__(Runner)
        runner.config = cfg
        return cfg.create_strategy(), runner

    def default_strategy():
        cfg = Config(format="json", strategy="simple", log_to_stderr=True, other_args={})
        runner = Runner.__new__(Runner)
        runner.config = cfg
        return SimpleStrategy(SimpleStrategySettings()), runner

    # ---------------- input cases: pods -> list of Prometheus value strings ----------
    def fmt(xs):
        return [prom_format(float(x)) for x in xs]

    cases = []

    def add(name, cpu_pods, mem_pods):
        cases.append({"name": name, "cpu": cpu_pods, "mem": mem_pods})

    add("empty_object", {}, {})
    add("one_sample", {"p0": ["0.25"]}, {"p0": ["123456789"]})
    add("two_samples", {"p0": ["0.5", "0.1"]}, {"p0": ["1", "2"]})
    add("three_dec_ceil_trap", {"p0": ["2.007", "0.001", "0.0049"]}, {"p0": ["20000000"]})
    add("below_min_clamp", {"p0": ["0.0001", "0.002"]}, {"p0": ["1000", "5"]})
    add("ties", {"a": ["0.3"] * 50, "b": ["0.3", "0.2"] * 25}, {"a": ["500000000"] * 10})
    add("zeros_signed", {"a": ["0", "-0", "0", "-0"]}, {"a": ["-0", "0"]})
    add("zeros_signed_2", {"a": ["-0", "0", "0"]}, {"a": ["0", "-0"]})
    add("inf_cpu", {"a": ["0.1", "+Inf", "0.2"]}, {"a": ["10000000"]})
    add("nan_cpu_index", {"a": ["0.1", "NaN", "0.2", "0.3"]}, {"a": ["10000000"]})
    add("nan_mem_raises", {"a": ["0.1"]}, {"a": ["1", "NaN", "3"]})
    add("nan_mem_single", {"a": ["0.1"]}, {"a": ["NaN"]})
    add("nan_cpu_single", {"a": ["NaN"]}, {"a": ["2"]})
    add("empty_pod_dropped_order", {"x": ["0.9", "0.8"], "y": [], "z": ["0.1"]}, {"x": ["3"], "z": ["4"]})
    add("large_memory", {"a": ["1.5"]}, {"a": ["987654321987", "987654321986.5"]})
    add("tiny_cpu", {"a": fmt([1e-9, 5e-7, 3e-12])}, {"a": ["999999"]})
    add("negative_cpu", {"a": ["-0.5", "-0.25", "0.1"]}, {"a": ["-5", "-7"]})
    for i in range(48):
        npods = int(rng.integers(1, 6))
        cpu, mem = {}, {}
        for p in range(npods):
            n = int(rng.integers(0, 160))
            kind = i % 4
            if kind == 0:
                v = rng.gamma(2.0, 0.05, n)
            elif kind == 1:
                v = np.round(rng.gamma(2.0, 0.05, n), 3)  # 3-decimal values: float-ceil traps
            elif kind == 2:
                v = rng.integers(0, 4, n) * 0.125  # heavy ties
            else:
                v = rng.lognormal(-3, 2, n)
            cpu[f"pod{p}"] = fmt(v)
            mem[f"pod{p}"] = fmt(np.floor(rng.normal(2e8, 2e7, int(rng.integers(0, 120)))))
        add(f"random_{i}", cpu, mem)

    # ---------------- run the reference ---------------------------------------------
    settings_paths = [
        ("cli_99_5", lambda: cli_strategy("99", "5")),
        ("cli_50_0.5", lambda: cli_strategy("50", "0.5")),
        ("cli_99.9_100", lambda: cli_strategy("99.9", "100")),
        ("cli_0.1_5", lambda: cli_strategy("0.1", "5")),
        ("cli_100_5_min", lambda: cli_strategy("100", "5", cpu_min=50, mem_min=300)),
        ("default_int", default_strategy),
    ]

    def to_hist(case):
        return {
            ResourceType.CPU: {k: [Decimal(s) for s in v] for k, v in case["cpu"].items() if v},
            ResourceType.Memory: {k: [Decimal(s) for s in v] for k, v in case["mem"].items() if v},
        }

    def run_cases(cases):
        out_cases = []
        for case in cases:
            results = {}
            for sp_name, make in settings_paths:
                strat, runner = make()
                hist = to_hist(case)
                entry = {}
                try:
                    raw = strat.run(hist, None)
                    entry["raw"] = {
                        "cpu_request": dstr(raw[ResourceType.CPU].request),
                        "cpu_limit": dstr(raw[ResourceType.CPU].limit),
                        "mem_request": dstr(raw[ResourceType.Memory].request),
                        "mem_limit": dstr(raw[ResourceType.Memory].limit),
                    }
                    try:
                        rr = runner._format_result(raw)
                        entry["rounded"] = {
                            "cpu_request": dstr(rr[ResourceType.CPU].request),
                            "cpu_limit": dstr(rr[ResourceType.CPU].limit),
                            "mem_request": dstr(rr[ResourceType.Memory].request),
                            "mem_limit": dstr(rr[ResourceType.Memory].limit),
                        }
                    except Exception as e:  # e.g. ceil(Infinity)
                        entry["rounded_error"] = type(e).__name__
                except Exception as e:
                    entry["error"] = type(e).__name__
                # SORTED_LOWER: the reference's own index rule over pre-sorted samples
                flat = [Decimal(s) for v in case["cpu"].values() for s in v]
                try:
                    entry["sorted"] = dstr(strat.settings.calculate_cpu_proposal({"all": sorted(flat)}))
                except Exception as e:
                    entry["sorted_error"] = type(e).__name__
                # LINEAR: numpy.percentile on the float64 samples
                f = np.array([float(s) for s in flat], dtype=np.float64)
                if f.size:
                    lin = float(np.percentile(f, float(strat.settings.cpu_percentile)))
                    entry["linear_hex"] = lin.hex() if not math.isnan(lin) else "nan"
                results[sp_name] = entry
            out_cases.append({"name": case["name"], "cpu": case["cpu"], "mem": case["mem"], "results": results})
        return out_cases

    out_cases = run_cases(cases)

    # ---------------- the index rule over (n, p) -------------------------------------
    strat, _ = cli_strategy("99", "5")
    index_table = []
    for p in ["99", "50", "0.1", "99.9", "100", "95", "33.3", "1", "12.5"]:
        s, _ = cli_strategy(p, "5")
        ns = [1, 2, 3, 10, 100, 101, 1000, 1001, 1440, 10080, 10081, 30240, 50400, 172800, 1000003]
        for n in ns:
            # calculate_cpu_proposal returns data_[k]; a range() list makes it return k itself
            k = s.settings.calculate_cpu_proposal({"r": list(range(n))})
            index_table.append({"p": p, "n": n, "k": int(k)})
    ds, _ = default_strategy()
    for n in [1, 2, 3, 100, 101, 10080, 50400, 172800]:
        index_table.append({"p": "int99", "n": n, "k": int(ds.settings.calculate_cpu_proposal({"r": list(range(n))}))})

    doc = {
        "generator": "tests/golden/make_golden.py",
        "reference": "yonahd/krr 1.0.0 @ /root/reference (imported, not copied)",
        "settings_paths": [n for n, _ in settings_paths],
        "cases": out_cases,
        "index_table": index_table,
    }
    path = os.path.join(HERE, "simple_strategy.json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(out_cases)} cases x {len(settings_paths)} settings paths, "
          f"{len(index_table)} index rows")

    # ---------------- HistoryData beyond Prometheus' strings --------------------------
    # The plugin API takes ANY HistoryData (core/abstract/strategies.py:35-36, 54-56): hand-built
    # Decimals, non-canonical forms, more digits than a float64 holds.  The reference returns
    # the sample object itself (simple.py:29, :36), so these pin representation and exact ties.
    exact = exact_cases()
    doc = {
        "generator": "tests/golden/make_golden.py",
        "reference": "yonahd/krr 1.0.0 @ /root/reference (imported, not copied)",
        "settings_paths": [n for n, _ in settings_paths],
        "cases": run_cases(exact),
        "note": "inputs are str(Decimal) of the HistoryData samples, NOT Prometheus strings",
    }
    path = os.path.join(HERE, "simple_strategy_exact.json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(exact)} cases x {len(settings_paths)} settings paths")


def exact_cases():
    """Sample strings (Decimal(s) is the HistoryData sample) outside Prometheus' canonical form."""
    rng = np.random.default_rng(20261018)
    cases = []

    def add(name, cpu_pods, mem_pods):
        cases.append({"name": name, "cpu": cpu_pods, "mem": mem_pods})

    # the round-4 probe (VERDICT.md Weak 1)
    add("probe_trailing_zeros", {"a": ["0.10", "0.20"]}, {"a": ["1.0E+7", "2.00E+7"]})
    add("probe_25_digits", {"a": ["0.0010000000000000000000001"]}, {"a": ["100000000.0000000000000001"]})
    add("probe_float_collision", {"a": ["0.1", "0.1000000000000000055511151231257827"]},
        {"a": ["20000000.00000000000000001", "20000000"]})
    add("collision_max_not_first", {"a": ["0.5", "0.50000000000000000001", "0.5"]},
        {"a": ["20000000", "19999999.99999999999999999", "20000000.000000000000000001", "20000000.00000000000000001",
               "20000000"]})
    add("equal_values_repr_ties", {"a": ["0.30", "0.3", "0.300", "0.1"] * 30},
        {"a": ["2E+7", "20000000", "2.0E+7", "1E+7"], "b": ["2.000E+7"]})
    add("sorted_ties_repr", {"a": ["0.5", "0.50", "0.500", "0.1", "0.5000", "0.9"]}, {"a": ["5", "5.0"]})
    add("exponent_forms", {"a": ["1E+2", "100", "1.00E+2", "5E-3", "0.0050"]}, {"a": ["1E+30", "1.0E+30"]})
    add("zero_forms", {"a": ["0.0", "-0.00", "0E+3", "0", "-0"]}, {"a": ["0.0", "0E+3", "-0.000"]})
    add("long_digits", {"a": ["0.123456789123456789123456789", "0.0123456789012345678901234567890123"]},
        {"a": ["123456789.123456789123456789", "123456789.1234567891234567890"]})
    add("collision_group_sorted", {"a": ["0.3", "0.29999999999999998889776975", "0.3000000000000000166533453694",
                                         "0.29999999999999998", "0.2", "0.4"] * 7},
        {"a": ["1073741824.0000000000000000001", "1073741824", "1073741824.00000000000000000001"]})
    add("nan_forms", {"a": ["0.1", "-NaN", "0.2"]}, {"a": ["7.0"]})
    for i in range(24):
        npods = int(rng.integers(1, 4))
        cpu, mem = {}, {}
        for p in range(npods):
            n = int(rng.integers(1, 120))
            x = rng.gamma(2.0, 0.05, n)
            if i % 3 == 0:
                x = np.round(x, 2)  # ties
            m = np.floor(rng.normal(2e8, 2e7, int(rng.integers(1, 90))))
            if i % 2 == 0:
                m[rng.integers(0, m.size, max(1, m.size // 3))] = m.max()  # several copies of the max
            cpu[f"pod{p}"] = [_variant(rng, float(v), i) for v in x]
            mem[f"pod{p}"] = [_variant(rng, float(v), i + 1) for v in m]
        add(f"random_exact_{i}", cpu, mem)
    return cases


def _variant(rng, x: float, i: int) -> str:
    """One sample string: canonical, a trailing-zero / exponent form of the same value, or the
    float's full binary expansion (a different Decimal with the same float64)."""
    from decimal import Decimal as D

    r = float(rng.random())
    canon = str(D(prom_format(x)))
    if r < 0.4:
        return canon
    if r < 0.6:
        return canon + ("0" * int(rng.integers(1, 4)) if "." in canon else ".0")
    if r < 0.75:
        return format(D(canon), "E")
    if i % 2 and r < 0.95:
        return str(D(x))  # exact binary value: > 17 digits, same float, distinct Decimal
    return canon


def pct_main():
    """simple_strategy_pct.json: the reference's index rule and results for cpu_percentile values
    whose Decimal product rounds, on both settings paths: the CLI's strings
    (Config.other_args) and direct construction with a Decimal or a float (pydantic-validated)."""
    import decimal

    from pct_inputs import INDEX_NS, INDEX_SCAN, PERCENTILES, RUN_NS, cpu_values, mem_values, pods_of

    ResourceType, Config, Runner, SimpleStrategy, SimpleStrategySettings = import_reference()
    assert decimal.getcontext().prec == 28

    def runner_for(cfg):
        runner = Runner.__new__(Runner)
        runner.config = cfg
        return runner

    base_cfg = Config(format="json", strategy="simple", log_to_stderr=True, other_args={})

    def make(path, p):
        if path == "cli":
            cfg = Config(format="json", strategy="simple", log_to_stderr=True,
                         other_args={"cpu_percentile": p, "memory_buffer_percentage": "5"})
            return cfg.create_strategy(), runner_for(cfg)
        value = Decimal(p) if path == "direct_decimal" else float(p)
        return SimpleStrategy(SimpleStrategySettings(cpu_percentile=value)), runner_for(base_cfg)

    paths = ["cli", "direct_decimal", "direct_float"]
    index_rows = []
    for path in paths:
        for p in PERCENTILES:
            strat, _ = make(path, p)
            st = strat.settings
            ns = sorted(set(INDEX_NS) | set(range(1, INDEX_SCAN + 1)))
            ks = [int(st.calculate_cpu_proposal({"r": list(range(n))})) for n in ns]
            index_rows.append({"path": path, "p": p, "setting": str(st.cpu_percentile),
                               "setting_type": type(st.cpu_percentile).__name__, "n": ns, "k": ks})

    inputs = {}
    for n in RUN_NS:
        c, m = cpu_values(n), mem_values(n)
        cs = [prom_format(float(x)) for x in c]
        ms = [prom_format(float(x)) for x in m]
        pods, o = [], 0
        for ln in pods_of(n):
            pods.append((o, o + ln))
            o += ln
        inputs[n] = ({f"pod{i}": [Decimal(x) for x in cs[a:b]] for i, (a, b) in enumerate(pods)},
                     {f"pod{i}": [Decimal(x) for x in ms[a:b]] for i, (a, b) in enumerate(pods)},
                     np.array([float(x) for x in cs]))
    runs = []
    for path in paths:
        for p in PERCENTILES:
            strat, runner = make(path, p)
            for n in RUN_NS:
                cpu, mem, f = inputs[n]
                raw = strat.run({ResourceType.CPU: cpu, ResourceType.Memory: mem}, None)
                rr = runner._format_result(raw)
                flat = [x for v in cpu.values() for x in v]
                srt = strat.settings.calculate_cpu_proposal({"all": sorted(flat)})
                lin = float(np.percentile(f, float(strat.settings.cpu_percentile)))
                runs.append({"path": path, "p": p, "n": n,
                             "raw": {"cpu_request": dstr(raw[ResourceType.CPU].request),
                                     "mem_request": dstr(raw[ResourceType.Memory].request)},
                             "rounded": {"cpu_request": dstr(rr[ResourceType.CPU].request),
                                         "mem_request": dstr(rr[ResourceType.Memory].request),
                                         "mem_limit": dstr(rr[ResourceType.Memory].limit)},
                             "sorted": dstr(srt), "linear_hex": lin.hex()})
    doc = {
        "generator": "tests/golden/make_golden.py pct (inputs: tests/golden/pct_inputs.py)",
        "reference": "yonahd/krr 1.0.0 @ /root/reference (imported, not copied)",
        "paths": {"cli": "Config(other_args={'cpu_percentile': p, 'memory_buffer_percentage': '5'}).create_strategy()",
                  "direct_decimal": "SimpleStrategy(SimpleStrategySettings(cpu_percentile=Decimal(p)))",
                  "direct_float": "SimpleStrategy(SimpleStrategySettings(cpu_percentile=float(p)))"},
        "index": index_rows,
        "runs": runs,
    }
    path = os.path.join(HERE, "simple_strategy_pct.json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(index_rows)} index rows, {len(runs)} runs")


if __name__ == "__main__":
    sys.path.insert(0, HERE)
    if sys.argv[1:] == ["pct"]:
        pct_main()
    else:
        main()
        pct_main()
