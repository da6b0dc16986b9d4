"""Golden outputs of the REFERENCE on BASELINE.json configs[0] (config 1), by import.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_config1_golden.py   # writes tests/golden/config1_reference.json

Same import recipe as make_golden.py.  The 6,048,000 inputs are not stored:
`config1.inputs()` regenerates them from PCG64 seed 0 and the fixture records their sha256,
so a test can prove it is looking at the same samples.  Per object the fixture holds the
reference's `SimpleStrategy.run()` result and `Runner._format_result()` of it (Decimal
strings) for the CLI settings path (`--cpu_percentile 99 --memory_buffer_percentage 5`)
and the int-default path (`SimpleStrategySettings()`), plus the reference's own wall time
for parse + run + round on this container's CPU (one core; GIL + Decimal).
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time
from decimal import Decimal

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import config1  # noqa: E402
from make_golden import dstr, import_reference  # noqa: E402

from krr_amd.utils.prom_decimal import prom_format  # noqa: E402


def main():
    ResourceType, Config, Runner, SimpleStrategy, SimpleStrategySettings = import_reference()
    cpu, mem = config1.inputs()
    t0 = time.perf_counter()
    cpu_s = [[[prom_format(float(x)) for x in cpu[o, p]] for p in range(config1.PODS)] for o in range(config1.OBJECTS)]
    mem_s = [[[prom_format(float(x)) for x in mem[o, p]] for p in range(config1.PODS)] for o in range(config1.OBJECTS)]
    t_fmt = time.perf_counter() - t0

    def cli():
        cfg = Config(format="json", strategy="simple", log_to_stderr=True,
                     other_args={"cpu_percentile": "99", "memory_buffer_percentage": "5"})
        r = Runner.__new__(Runner)
        r.config = cfg
        return cfg.create_strategy(), r

    def default():
        cfg = Config(format="json", strategy="simple", log_to_stderr=True, other_args={})
        r = Runner.__new__(Runner)
        r.config = cfg
        return SimpleStrategy(SimpleStrategySettings()), r

    out = {}
    timing = {}
    for name, make in (("cli_99_5", cli), ("default_int", default)):
        strat, runner = make()
        t0 = time.perf_counter()
        hists = []
        for o in range(config1.OBJECTS):
            pods = config1.pod_names(o)
            # prometheus.py:150-155: {pod: [Decimal(value) ...]} in object.pods order
            hists.append({ResourceType.CPU: {pods[p]: [Decimal(s) for s in cpu_s[o][p]] for p in range(config1.PODS)},
                          ResourceType.Memory: {pods[p]: [Decimal(s) for s in mem_s[o][p]]
                                                for p in range(config1.PODS)}})
        t1 = time.perf_counter()
        rows = []
        for h in hists:
            raw = strat.run(h, None)
            rr = runner._format_result(raw)
            rows.append({
                "raw": {"cpu_request": dstr(raw[ResourceType.CPU].request), "cpu_limit": dstr(raw[ResourceType.CPU].limit),
                        "mem_request": dstr(raw[ResourceType.Memory].request),
                        "mem_limit": dstr(raw[ResourceType.Memory].limit)},
                "rounded": {"cpu_request": dstr(rr[ResourceType.CPU].request),
                            "cpu_limit": dstr(rr[ResourceType.CPU].limit),
                            "mem_request": dstr(rr[ResourceType.Memory].request),
                            "mem_limit": dstr(rr[ResourceType.Memory].limit)},
            })
        t2 = time.perf_counter()
        out[name] = rows
        timing[name] = {"decimal_parse_s": t1 - t0, "run_and_round_s": t2 - t1,
                        "containers_per_s_run_and_round": config1.OBJECTS / (t2 - t1),
                        "containers_per_s_parse_run_round": config1.OBJECTS / (t2 - t0)}
    doc = {
        "generator": "tests/golden/make_config1_golden.py",
        "reference": "yonahd/krr 1.0.0 @ /root/reference (imported, not copied)",
        "workload": f"config 1: {config1.OBJECTS} containers x {config1.PODS} pods x {config1.SAMPLES} samples "
                    f"(7d@1m) per resource, PCG64 seed {config1.SEED}",
        "input_sha256": config1.sha256(cpu, mem),
        "pod_names": "app-{o:03d}-pod-{p}",
        "results": out,
        "reference_timing_build_container": {"cpu": platform.processor() or platform.machine(), "cores": 1,
                                             "format_strings_s": t_fmt, **timing},
    }
    path = os.path.join(HERE, "config1_reference.json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    print(f"wrote {path}; reference timing: {json.dumps(timing)}")


if __name__ == "__main__":
    main()
