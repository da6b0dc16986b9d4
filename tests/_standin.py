"""TEST INFRASTRUCTURE: the device engine stood in for by the CPU oracle (GPU-less container).

``oracle_run_packed`` replaces ``SimpleEngine.run_packed`` in CPU tests: the fused pass's
values / counts / flags from oracle/krr_oracle.c, and krr_locate's answers for HistoryData
segments outside Prometheus' canonical strings from ``oracle.locate`` with the ranks the
engine itself would pass (``krr_amd.core.engine.locate_ranks``)."""
from __future__ import annotations

import numpy as np


def k_table_for(series, params):
    """The index table the engine binds for this series (_native.bind_index_table), or None."""
    from krr_amd import _native

    rule = getattr(params, "rule", None)
    offs = np.asarray(series.offsets)
    max_n = int(np.diff(offs).max()) if offs.size > 1 else 0
    if rule is None or params.mode == _native.KRR_PCT_LINEAR or not rule.needs_table(max_n):
        return None
    return rule.table(max(max_n, 1))


def oracle_run_packed(self, fleet, params):
    from krr_amd.core.engine import RawResults, locate_ranks, needs_locate
    from oracle import oracle

    cv, cn, cf = oracle.percentile(fleet.cpu.values, fleet.cpu.offsets, params.mode, params.p_num, params.p_den,
                                   params.q, fleet.cpu.gaps_are_nan, k_table=k_table_for(fleet.cpu, params))
    mv, mn, mf = oracle.seg_max(fleet.mem.values, fleet.mem.offsets, fleet.mem.gaps_are_nan)
    raw = RawResults(cv, cn, cf.astype(np.uint32), mv, mn, mf.astype(np.uint32))
    if needs_locate(fleet, params):
        raw.locate = {}
        for name, ps, val, cnt, fl in (("cpu", fleet.cpu, cv, cn, cf), ("mem", fleet.mem, mv, mn, mf)):
            if ps.exact is None:
                continue
            rank = locate_ranks(name, ps.exact, cnt, fl, params)
            if rank is not None:
                raw.locate[name] = oracle.locate(np.asarray(ps.values), np.asarray(ps.offsets), val, rank)
    return raw
