"""Generate golden vectors for Severity / ResourceScan / Result (reference
robusta_krr/core/models/result.py:14-150) BY IMPORTING THE REFERENCE.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_result_golden.py      # writes tests/golden/result_scan.json

Same import recipe as make_golden.py.  Inputs are Kubernetes quantity strings (the
objects' current allocations, parsed by the reference's resource_units) and the
recommendation values as the runner produces them (Decimal strings, "?" or None);
outputs are the reference's per-pair severities, each scan's severity, the
exception a scan raises (if any) and Result.score for several fleet sizes.
"""
from __future__ import annotations

import json
import os
import random
from decimal import Decimal

from make_golden import import_reference

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ResourceType = import_reference()[0]
    from robusta_krr.core.models.allocations import ResourceAllocations
    from robusta_krr.core.models.objects import K8sObjectData
    from robusta_krr.core.models.result import Result, ResourceScan, Severity

    rng = random.Random(20261016)
    rts = [ResourceType.CPU, ResourceType.Memory]

    def rec_value(s):
        # the runner hands NaN for "no data"; the validator turns it into "?" (allocations.py:40-41)
        return None if s is None else (Decimal("NaN") if s == "?" else Decimal(s))

    cases = []

    def add(name, cur, rec):
        """cur: {sel: [cpu, mem]} quantity strings / None; rec: {sel: [cpu, mem]} Decimal strings / "?" / None."""
        cases.append({"name": name, "current": cur, "recommended": rec})

    # boundaries of the buckets (result.py:43-50): diff exactly at 1.0, -0.5, 0.5, -0.25 and just off them
    for r in ["0.25", "1", "3", "0.007", "123456789", "2.1E+7", "0.1"]:
        R = Decimal(r)
        for mult in ["2", "0.5", "1.5", "0.75", "1", "3", "0.1", "0"]:
            for eps in ["0", "1e-9", "-1e-9", "1e-20", "-1e-20", "1e-27", "-1e-27", "1e-29", "-1e-29"]:
                c = R * (Decimal(mult) + Decimal(eps))
                add(f"edge r={r} m={mult} e={eps}", {"requests": [str(c), None], "limits": [None, None]},
                    {"requests": [r, r], "limits": [None, "?"]})
    # random fleet with Kubernetes quantity strings
    units = ["", "m", "Ki", "Mi", "Gi", "k", "M", "G"]
    for i in range(400):
        def qty():
            u = rng.choice(units)
            mag = rng.choice([1, 10, 100, 1000, 0.5, 0.25, 2.5])
            return f"{rng.randint(1, 999) * mag:g}{u}" if rng.random() < 0.85 else None

        def recv():
            x = rng.random()
            if x < 0.05:
                return "?"
            if x < 0.08:
                return None
            return str(Decimal(rng.randint(1, 10 ** 6)) * Decimal(10) ** rng.randint(-4, 6))

        add(f"random {i}", {"requests": [qty(), qty()], "limits": [qty(), qty()]},
            {"requests": [recv(), recv()], "limits": [recv(), recv()]})
    # zero recommendations: the reference's Decimal division raises
    add("zero rec", {"requests": ["1", None], "limits": [None, None]}, {"requests": ["0", None], "limits": [None, None]})
    add("zero/zero", {"requests": ["0", None], "limits": [None, None]}, {"requests": ["0", None], "limits": [None, None]})
    add("all unset", {"requests": [None, None], "limits": [None, None]}, {"requests": [None, None], "limits": [None, None]})
    add("all unknown", {"requests": [None, "1"], "limits": ["2", None]}, {"requests": ["?", "?"], "limits": ["?", "?"]})

    objects, recs = [], []
    for k, c in enumerate(cases):
        alloc = ResourceAllocations(requests=dict(zip(rts, c["current"]["requests"])),
                                    limits=dict(zip(rts, c["current"]["limits"])))
        obj = K8sObjectData(cluster=None, name=f"obj{k}", container="app", pods=[f"p{k}"], namespace="default",
                            kind="Deployment", allocations=alloc)
        rec = ResourceAllocations(requests={rt: rec_value(v) for rt, v in zip(rts, c["recommended"]["requests"])},
                                  limits={rt: rec_value(v) for rt, v in zip(rts, c["recommended"]["limits"])})
        try:
            scan = ResourceScan.calculate(obj, rec)
            c["severity"] = scan.severity.value
            c["pairs"] = {sel: [getattr(scan.recommended, sel)[rt].severity.value for rt in rts]
                          for sel in ("requests", "limits")}
            objects.append(obj)
            recs.append(rec)
        except Exception as e:  # noqa: BLE001 - the reference's own exception is the expected output
            c["raises"] = type(e).__name__
        c["current_parsed"] = {sel: [None if v is None else str(v) for v in getattr(alloc, sel).values()]
                               for sel in ("requests", "limits")}

    scores = {}
    for n in [0, 1, 2, 7, 100, len(objects)]:
        scans = [ResourceScan.calculate(o, r) for o, r in zip(objects[:n], recs[:n])]
        scores[str(n)] = Result(scans=scans).score
    colors = {s.value: s.color for s in Severity}
    doc = {"source": "robusta_krr/core/models/result.py via import (make_result_golden.py)",
           "cases": cases, "scores": scores, "colors": colors}
    with open(os.path.join(HERE, "result_scan.json"), "w") as fh:
        json.dump(doc, fh, indent=0)
    print(f"{len(cases)} cases, {sum('raises' in c for c in cases)} raising; scores {scores}")


if __name__ == "__main__":
    main()
