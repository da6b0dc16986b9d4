"""Full-size GPU checks (BASELINE configs 2, 3 and 5 shapes) through size-independent
properties, computed with plain torch ops independent of the kernels:
  SORTED_LOWER:  #(x < v) <= k < #(x <= v)            (v is the k-th order statistic)
  LINEAR:        x_(r0) <= v <= x_(r1)  via  #(x < v) <= r1 and #(x <= v) >= r0 + 1
  max / count:   nan-ignoring max (bits) and #present
The oracle-level bit-exact checks live in test_gpu_kernels.py at smaller sizes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from krr_amd import _native

    c = _native.Context(0)
    yield c
    c.close()


def _run(ctx, cpu, mem, offs, maxlen, gaps, mode, pct):
    import torch

    from krr_amd.core.engine import percentile_params

    S = offs.numel() - 1
    dev = cpu.device
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    ctx.simple_run(ctx.series(cpu, offs, maxlen, gaps), ctx.series(mem, offs, maxlen, gaps),
                   percentile_params(pct, mode), out)
    torch.cuda.synchronize()
    return out


def _ranks(n, mode, pct):
    import torch

    if mode == "sorted_lower":
        k = ((n - 1) * int(pct * 1000)) // 100000
        return k, k
    vidx = (n - 1).to(torch.float64) * (pct / 100.0)
    r0 = torch.floor(vidx).to(torch.int64)
    r1 = torch.minimum(r0 + 1, n - 1)
    return r0, r1


def _check_dense(cpu2d, mem2d, out, mode, pct):
    """Rows of a [S, L] view; NaN = absent."""
    import torch

    present = ~torch.isnan(cpu2d)
    n = present.sum(1)
    assert torch.equal(out["cpu_count"], n)
    v = out["cpu_value"]
    lt = (cpu2d < v[:, None]).sum(1)
    le = (cpu2d <= v[:, None]).sum(1)
    r0, r1 = _ranks(n, mode, pct)
    assert bool((lt <= r1).all()) and bool((le >= r0 + 1).all())
    mmax = torch.where(torch.isnan(mem2d), torch.full_like(mem2d, -float("inf")), mem2d).max(1).values
    assert torch.equal(out["mem_value"].view(torch.int64), mmax.view(torch.int64))
    assert torch.equal(out["mem_count"], (~torch.isnan(mem2d)).sum(1))
    assert bool((out["cpu_flags"] == 0).all()) and bool((out["mem_flags"] == 0).all())


@pytest.mark.parametrize("mode,pct", [("linear", 99.0), ("sorted_lower", 99.0), ("linear", 50.0),
                                      ("sorted_lower", 95.0)])
def test_config2_full_size(ctx, mode, pct):
    """10,000 containers x 5 pods x 10,080 slots, NaN-gapped: the bench's workload."""
    import torch

    S, L = 10_000, 5 * 10080
    dev = torch.device("cuda:0")
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    cpu = torch.empty(S * L, dtype=torch.float64, device=dev)
    mem = torch.empty(S * L, dtype=torch.float64, device=dev)
    ctx.synth_fill(cpu, offs, 11, 0, 10080, True)
    ctx.synth_fill(mem, offs, 12, 1, 10080, True)
    out = _run(ctx, cpu, mem, offs, L, True, mode, pct)
    c2, m2 = cpu.view(S, L), mem.view(S, L)
    for a in range(0, S, 1000):
        sub = {k: v[a:a + 1000] for k, v in out.items()}
        _check_dense(c2[a:a + 1000], m2[a:a + 1000], sub, mode, pct)


@pytest.mark.parametrize("mode,pct", [("linear", 99.0), ("sorted_lower", 50.0)])
def test_config3_ragged(ctx, mode, pct):
    """Config 3's shape (1..14 days @1m, compact CSR), 20,000 containers."""
    import torch

    rng = np.random.default_rng(3)
    S = 20_000
    lens = rng.integers(1, 15, size=S) * 1440
    offs_np = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    dev = torch.device("cuda:0")
    offs = torch.from_numpy(offs_np).to(dev)
    N = int(offs_np[-1])
    cpu = torch.empty(N, dtype=torch.float64, device=dev)
    mem = torch.empty(N, dtype=torch.float64, device=dev)
    ctx.synth_fill(cpu, offs, 13, 0, 0, False)
    ctx.synth_fill(mem, offs, 14, 1, 0, False)
    out = _run(ctx, cpu, mem, offs, int(lens.max()), False, mode, pct)
    seg = torch.repeat_interleave(torch.arange(S, device=dev), torch.from_numpy(lens).to(dev))
    v = out["cpu_value"][seg]
    lt = torch.bincount(seg, weights=(cpu < v).to(torch.float64), minlength=S).to(torch.int64)
    le = torch.bincount(seg, weights=(cpu <= v).to(torch.float64), minlength=S).to(torch.int64)
    n = torch.from_numpy(lens).to(dev)
    assert torch.equal(out["cpu_count"], n)
    r0, r1 = _ranks(n, mode, pct)
    assert bool((lt <= r1).all()) and bool((le >= r0 + 1).all())
    mmax = torch.full((S,), -float("inf"), dtype=torch.float64, device=dev).scatter_reduce(0, seg, mem, "amax")
    assert torch.equal(out["mem_value"], mmax)


def test_config5_sketch_rank_error_bound(ctx):
    """1,000 series x 172,800 samples (30d@15s), sketch mode: the answer's rank error is
    bounded by the mass of its bin (+ the interpolation's half sample)."""
    import torch

    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    S, T = 1000, 172_800
    dev = torch.device("cuda:0")
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * T
    x = torch.empty(S * T, dtype=torch.float64, device=dev)
    ctx.synth_fill_window(x, offs, 77, 0, 0, False, 0, T)
    ser = ctx.series(x, offs, T, False)
    cfg = sketch.SketchConfig()
    sk = sketch.build(ctx, ser, cfg)
    res = sketch.query(ctx, sk, cfg, percentile_params(99, "sorted_lower"))
    torch.cuda.synchronize()
    x2 = x.view(S, T)
    v = res["value"]
    lt = (x2 < v[:, None]).sum(1)
    le = (x2 <= v[:, None]).sum(1)
    k = ((T - 1) * 99) // 100
    err = torch.clamp(torch.maximum(lt - k, k - (le - 1)), min=0)
    maxbin = sk["counts"].max(1).values.to(torch.int64)
    assert bool((err <= maxbin).all())
    assert float(err.max()) / T < 1e-3
