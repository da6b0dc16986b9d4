"""Multi-rank paths on the GPU box (one MI355X: ranks share it over gloo; RCCL gets a
one-rank communicator), each rank a fresh interpreter started by a parent process:

* BatchedRunner's sharded mode (shard -> one fused kernel pass per rank -> records gathered
  -> exact rounding on rank 0) against the reference's own config-1 strings;
* `bench.py --gpus 2` (self-launching two ranks, gloo rehearsal): n_gpus 2 and the gathered
  records equal the oracle and rank 0's kernel on samples regenerated from every shard;
* config 5 at 2 and 3 time-sharded ranks: sketch reduce-scatter + exact refinement equal one
  select over the regathered full series; sketch-only rank error within bound;
* the C-ABI gather (krr_gather_results over RCCL, include/krr_amd.h), with a communicator of
  its own and with PyTorch's;
* global-index synthesis: shards generated apart equal the fleet generated whole.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

from test_distributed import expected_rows, run_sharded_workers  # noqa: E402


@pytest.mark.parametrize("entry,path", [("packed", "cli_99_5"), ("loader", "default_int"), ("bodies", "cli_99_5")])
def test_sharded_runner_two_ranks_on_gpu(entry, path, tmp_path):
    assert run_sharded_workers(2, "gpu", entry, path, tmp_path, timeout=240) == expected_rows(path)


def _bench(args, timeout=240):
    env = dict(os.environ, KRR_BENCH_BACKEND="gloo")
    p = subprocess.run(["timeout", "-k", "10", str(timeout), sys.executable, os.path.join(ROOT, "bench.py"), *args],
                       capture_output=True, text=True, env=env, timeout=timeout + 30)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("cfg,extra", [("2", ["--containers", "400"]), ("3", ["--containers", "2000"]),
                                       ("4", ["--containers", "3000", "--mode", "sorted_lower"])])
def test_bench_self_launches_ranks(cfg, extra):
    r = _bench(["--gpus", "2", "--config", cfg, "--steps", "2", "--warmup", "1", "--parity-block", "64", *extra])
    assert r["n_gpus"] == 2 and r["config"]["backend"] == "gloo"
    assert r["parity_vs_oracle_on_sample"] is True and r["parity_gathered_vs_rank0_kernel"] is True, r
    assert r["parity_sample_containers"] >= 2 * 64
    assert "cpu_baseline" not in r  # rank 0 at N = 1 only


def test_bench_under_torchrun_like_the_driver():
    """The driver's N > 1 command shape: torch.distributed.run launches the ranks (WORLD_SIZE
    set by it, bench.py's own per-rank watchdog armed, not fired), rank 0 alone prints the
    one JSON line; gloo here (two ranks share the one GPU), RCCL on the driver's node."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, KRR_BENCH_BACKEND="gloo")
    env.pop("KRR_BENCH_LAUNCHED", None)
    p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--containers", "400", "--steps", "2",
                        "--warmup", "1", "--parity-block", "64", "--deadline", "200"],
                       capture_output=True, text=True, env=env, timeout=270)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["backend"] == "gloo" and "status" not in r
    assert r["parity_vs_oracle_on_sample"] is True and r["parity_gathered_vs_rank0_kernel"] is True, r
    assert len(r["per_rank_kernel_ms"]) == 2


@pytest.mark.parametrize("gather,comm", [("stream", "own"), ("stream", "torch"), ("torch", "own"),
                                        ("blocking", "own")])
def test_bench_rccl_path_one_rank(gather, comm):
    """The N > 1 step over RCCL at one rank (`--force-dist`): the C-ABI gather on the launch
    stream with the library's own communicator (default: krr_comm_unique_id on rank 0, the id
    broadcast over torch.distributed, krr_comm_init_timeout) or torch's (--comm torch), rank
    0's launch writing into the rotating receive buffers; or torch.distributed.gather from two
    alternating send buffers; the gathered records go to the host on the second stream, and
    the host copy after the timed steps equals the records of the last launch."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), KRR_BENCH_BACKEND="nccl")
    p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.join(ROOT, "bench.py"), "--force-dist",
                        "--containers", "400", "--steps", "5", "--warmup", "2", "--gather", gather,
                        "--comm", comm, "--no-cpu-baseline"], capture_output=True, text=True, env=env, timeout=270)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["n_gpus"] == 1 and r["config"]["records"] == "HBM + RCCL gather to rank 0"
    assert r["config"]["gather"].startswith("RCCL send/recv" if gather == "stream" else "torch.distributed")
    assert r["records_host_equal_device"] is True, r
    if gather == "stream":  # the communicator the C-ABI gather ran on, and that RCCL saw this rank
        assert r["rccl_comm"]["ranks"] == 1, r["rccl_comm"]
        want = "krr_comm_unique_id" if comm == "own" else "torch.distributed"
        assert r["rccl_comm"]["communicator"].startswith(want), r["rccl_comm"]


@pytest.mark.parametrize("world,mode,pct,method", [(2, "linear", "99", "window"), (3, "sorted_lower", "50", "window"),
                                                   (2, "linear", "95", "window"), (3, "linear", "99", "sketch"),
                                                   (2, "sorted_lower", "50", "sketch")])
def test_bench_config5_time_sharded_ranks(world, mode, pct, method):
    """Config 5 through `bench.py --gpus N` (gloo ranks sharing the GPU): every series is
    time-sharded over N ranks.  window (default): each rank streams its slices once and
    exports its windows, one all-to-all hands them to the owners, which merge them;
    sketch: per-slice sketches reduce-scattered, the needed bins located, the samples in
    them collected (second pass), all-to-all'd and selected.  Rank 0 checks the gathered
    answers bit for bit against one k_select/hselect pass AND the C oracle over the full
    172,800-sample series (regathered from every rank)."""
    r = _bench(["--gpus", str(world), "--config", "5", "--containers", "600", "--steps", "2", "--warmup", "1",
                "--mode", mode, "--percentile", pct, "--error-sample", "600", "--c5-method", method], timeout=300)
    assert r["n_gpus"] == world and r["config"]["parallelism"].startswith(f"time-shard{world}")
    assert r["config"]["method"] == method
    assert r["parity_vs_single_window_select"] is True and r["parity_sample_series"] == 600, r
    assert r["parity_vs_oracle_on_sample"] is True and r["parity_oracle_sample_series"] == 600, r
    assert "cpu_baseline" not in r
    if method == "window":
        assert r["roofline"]["kernel"] == "k_window_export" and r["window"]["hbm_passes_per_step"] == 1
        assert r["window"]["misses_per_step"] == 0, r["window"]


def test_bench_config5_window_refine_one_rank():
    """--c5-refine at N = 1: the time-sharded one-pass path on one rank; its answers equal the
    oracle on the CPU-baseline sample and k_select on the error sample."""
    p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.join(ROOT, "bench.py"), "--config", "5",
                        "--containers", "800", "--c5-refine", "--steps", "2", "--warmup", "1", "--error-sample", "300",
                        "--cpu-sample", "100"], capture_output=True, text=True, timeout=270)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["config"]["method"] == "window" and r["parity_vs_single_window_select"] is True, r
    assert r["parity_vs_oracle_on_sample"] is True and r["parity_oracle_sample_series"] == 500, r


def test_bench_config5_sketch_only_two_ranks():
    """Sketch-only answers merged across two time-sharded ranks: the rank error stays within
    the log-linear sketch's bin mass (2^5 bins per octave; the same bound the N = 1 sketch
    test holds) and is reported beside the value."""
    r = _bench(["--gpus", "2", "--config", "5", "--containers", "600", "--steps", "2", "--warmup", "1",
                "--sketch-only", "--sketch-kind", "loglinear", "--error-sample", "600"], timeout=300)
    e = r["sketch_error"]
    assert e["sample_series"] == 600 and 0.0 <= e["rank_error_max"] < 1e-3 and e["value_rel_error_max"] < 0.01, e


@pytest.mark.parametrize("world,pct", [(2, "99"), (3, "99"), (2, "50")])
def test_bench_config5_kll_time_sharded_ranks(world, pct):
    """KLL sketch-only over 2 and 3 time-sharded ranks: every rank builds its slices' rows,
    one all-to-all hands each series' rows to its owner, which folds them (krr_kll_merge) and
    queries.  p99 falls in the rows' exact tail: the answers gathered to rank 0 equal the
    exact path's bit for bit.  p50 falls in the body: rank error within the rows'
    data-independent bound (+ one rank for LINEAR's interpolation)."""
    r = _bench(["--gpus", str(world), "--config", "5", "--containers", "600", "--steps", "2", "--warmup", "1",
                "--sketch-only", "--sketch-kind", "kll", "--error-sample", "300", "--percentile", pct], timeout=300)
    e = r["sketch_error"]
    assert r["config"]["method"] == "kll" and e["kind"] == "kll" and e["sample_series"] == 300, e
    assert e["within_bound"] is True and e["tail_answers_equal_exact"] is True, e
    if pct == "99":
        assert e["rank_in_exact_tail_fraction"] == 1.0 and e["value_rel_error_max"] == 0.0, e
    else:
        assert e["rank_error_max"] <= e["body_rank_error_bound_max"] + 1e-4 < 0.05, e


def test_synth_global_index_shards_equal_whole_fleet():
    import torch

    from krr_amd import _native

    ctx = _native.Context(0)
    dev = torch.device("cuda:0")
    S, L = 600, 5 * 10080
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    whole = torch.empty(S * L, dtype=torch.float64, device=dev)
    ctx.synth_fill(whole, offs, 1234, 0, 10080, True)
    parts = []
    for a, b in ((0, 250), (250, 600)):
        o = torch.arange(b - a + 1, dtype=torch.int64, device=dev) * L
        x = torch.empty((b - a) * L, dtype=torch.float64, device=dev)
        ctx.synth_fill(x, o, 1234, 0, 10080, True, seg_base=a)
        parts.append(x)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts).view(torch.int64), whole.view(torch.int64))
    ctx.close()


def _records(n, seed, dev):
    import torch

    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(-2**62, 2**62, (n, 4), generator=g, dtype=torch.int64).to(dev)


def test_c_abi_gather_one_rank_rccl():
    """krr_comm_unique_id -> krr_comm_init(1 rank) -> krr_gather_results: the root's own
    records land in `out` (counts given and not given), and bad arguments are refused."""
    import torch

    from krr_amd import _native

    ctx = _native.Context(0)
    dev = torch.device("cuda:0")
    uid = ctx.comm_unique_id()
    comm = ctx.comm_init(1, uid, 0)
    try:
        rec = _records(1000, 1, dev)
        out = torch.full((1000, 4), -1, dtype=torch.int64, device=dev)
        ctx.gather_results(comm, 0, rec, counts=[1000], out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, rec)
        out2 = torch.zeros((1000, 4), dtype=torch.int64, device=dev)
        ctx.gather_results(comm, 0, rec, out=out2)
        torch.cuda.synchronize()
        assert torch.equal(out2, rec)
        with pytest.raises(_native.NativeError):
            ctx.gather_results(comm, 1, rec, out=out2)  # root out of range
        with pytest.raises(_native.NativeError):
            ctx.gather_results(comm, 0, rec, counts=[999], out=out2)  # counts[root] != n_local
    finally:
        ctx.comm_destroy(comm)
        ctx.close()


def test_c_abi_comm_init_timeout_one_rank():
    """krr_comm_init_timeout: a bounded (nonblocking) 1-rank communicator works for the
    gather like the blocking one."""
    import torch

    from krr_amd import _native

    ctx = _native.Context(0)
    dev = torch.device("cuda:0")
    comm = ctx.comm_init(1, ctx.comm_unique_id(), 0, timeout_s=60.0)
    try:
        rec = _records(500, 3, dev)
        out = torch.zeros((500, 4), dtype=torch.int64, device=dev)
        ctx.gather_results(comm, 0, rec, counts=[500], out=out)
        torch.cuda.synchronize()
        assert torch.equal(out, rec)
    finally:
        ctx.comm_destroy(comm)
        ctx.close()


_MISSING_PEER = """
import sys, time
sys.path.insert(0, {root!r})
import torch
from krr_amd import _native
ctx = _native.Context(0)
t0 = time.time()
try:
    ctx.comm_init(2, ctx.comm_unique_id(), 0, timeout_s=3.0)   # rank 1 never comes
    print("NO-TIMEOUT")
except _native.NativeError as e:
    print("TIMEOUT" if "error -5" in str(e) else "OTHER " + str(e), round(time.time() - t0, 1))
"""


def test_c_abi_comm_init_timeout_missing_peer():
    """A 2-rank init whose second rank never arrives returns KRR_E_TIMEOUT after the bound
    instead of hanging (run in a child process under its own time limit)."""
    p = subprocess.run(["timeout", "-k", "5", "90", sys.executable, "-c", _MISSING_PEER.format(root=ROOT)],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    out = p.stdout.strip().splitlines()[-1]
    assert out.startswith("TIMEOUT"), out
    assert float(out.split()[-1]) < 30


def test_c_abi_gather_with_torch_process_group_comm():
    """The communicator of a torch.distributed "nccl" group (PyTorch's own librccl.so.1) goes
    straight into krr_gather_results: the ABI binds the RCCL already in the process."""
    import torch
    import torch.distributed as dist

    from krr_amd import _native

    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    ctx = _native.Context(0)
    try:
        t = torch.ones(4, device=dev)
        dist.all_reduce(t)  # creates the communicator
        backend = dist.group.WORLD._get_backend(dev)
        comm_ptr = getattr(backend, "_comm_ptr", None)
        if comm_ptr is None:
            pytest.skip("this torch build does not expose the RCCL communicator")
        rec = _records(777, 2, dev)
        out = torch.zeros((777, 4), dtype=torch.int64, device=dev)
        ctx.gather_results(int(comm_ptr()), 0, rec, counts=[777], out=out,
                           stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert torch.equal(out, rec)
    finally:
        ctx.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,gaps", [("linear", True), ("sorted_lower", False), ("ref_index", True),
                                       ("ref_index", False)])
@pytest.mark.parametrize("units", [1, 1000, 4096, 4097, 40_000])
def test_simple_run_forward_copy(mode, gaps, units):
    """krr_simple_run_forward: the launch copies `units` x 16 B (device -> page-locked host and
    device -> device) as its first work items, and its results and records equal those of the
    plain launch (compact REF_INDEX, which is not fused, copies on the stream instead)."""
    import torch

    from decimal import Decimal

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    ctx = _native.Context(0)
    dev = torch.device("cuda:0")
    S, L = 300, 3 * 10080
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    cpu = torch.empty(S * L, dtype=torch.float64, device=dev)
    mem = torch.empty(S * L, dtype=torch.float64, device=dev)
    ctx.synth_fill(cpu, offs, 11, 0, 10080 if gaps else 0, gaps)
    ctx.synth_fill(mem, offs, 12, 1, 10080 if gaps else 0, gaps)
    cs, ms = ctx.series(cpu, offs, L, gaps), ctx.series(mem, offs, L, gaps)
    params = percentile_params(Decimal("95"), mode)

    def outs():
        return {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
                (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
                 ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}

    src = _records(units // 2 + (units % 2), 7, dev).view(-1)[: 2 * units].contiguous()
    host = torch.full((2 * units,), -1, dtype=torch.int64).pin_memory()
    ddst = torch.full((2 * units,), -1, dtype=torch.int64, device=dev)
    o0, o1, o2 = outs(), outs(), outs()
    r0 = torch.empty((S, 4), dtype=torch.int64, device=dev)
    r1 = torch.empty((S, 4), dtype=torch.int64, device=dev)
    ctx.simple_run(cs, ms, params, o0, records=r0)
    ctx.simple_run(cs, ms, params, o1, records=r1, forward=(src, host))
    ctx.simple_run(cs, ms, params, o2, forward=(src, ddst))
    torch.cuda.synchronize()
    assert torch.equal(host, src.cpu()) and torch.equal(ddst, src)
    assert torch.equal(r0, r1)
    for k in o0:
        assert torch.equal(o0[k].view(torch.int64) if o0[k].dtype == torch.float64 else o0[k],
                           o2[k].view(torch.int64) if o2[k].dtype == torch.float64 else o2[k]), k
    with pytest.raises(ValueError):
        ctx.simple_run(cs, ms, params, o1, forward=(src, host[:-2]))
    ctx.close()


@pytest.mark.parametrize("args", [["--config", "4", "--containers", "3000", "--chunk-gib", "0.05"],
                                  ["--config", "2", "--containers", "400", "--chunk-gib", "0.05", "--mode", "ref_index"],
                                  ["--config", "4", "--containers", "3000", "--chunk-gib", "0.05", "--separate"]])
def test_bench_chunked_fleet_one_rank(args):
    """A fleet cut into chunks (buffers of their own, one launch per chunk, records rows per
    chunk written into the host buffer): parity with the oracle on every container and the
    host records equal to the device results."""
    p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.join(ROOT, "bench.py"), *args,
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=270)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["launches_per_step"] > 1 and r["parity_vs_oracle_on_sample"] is True, r
    assert r["parity_sample_containers"] == r["config"]["containers"]
    if "--separate" not in args:
        assert r["records_host_equal_device"] is True


def test_bench_config5_direct_chunked():
    """Config 5 at N = 1 (exact single-window select per chunk of series): equal bits to the
    select over the regathered series."""
    p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.join(ROOT, "bench.py"), "--config", "5",
                        "--containers", "600", "--c5-chunk-gib", "0.2", "--steps", "2", "--warmup", "1",
                        "--error-sample", "600", "--no-cpu-baseline"], capture_output=True, text=True, timeout=270)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["parity_vs_single_window_select"] is True and r["parity_sample_series"] == 600, r
    assert r["launches_per_step"] > 1


def test_bench_config5_direct_oracle_parity():
    """Config 5 at N = 1 with the CPU baseline: the run's own answers on the baseline sample
    equal the oracle (parity_vs_oracle_on_sample), beside the k_select check."""
    p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.join(ROOT, "bench.py"), "--config", "5",
                        "--containers", "700", "--c5-chunk-gib", "0.3", "--steps", "2", "--warmup", "1",
                        "--error-sample", "200", "--cpu-sample", "60"], capture_output=True, text=True, timeout=270)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["parity_vs_oracle_on_sample"] is True and r["parity_oracle_sample_series"] == 300, r
    assert r["cpu_baseline"]["kind"] == "port"


def test_bench_four_ranks_chunked_shards():
    """Four gloo ranks sharing the GPU, config 4 cut into shards that are each chunked (buffers
    of their own, one launch per chunk): the gathered records equal the oracle and rank 0's
    kernel on samples from every shard."""
    r = _bench(["--gpus", "4", "--config", "4", "--containers", "2000", "--chunk-gib", "0.03", "--steps", "2",
                "--warmup", "1", "--parity-block", "64"], timeout=300)
    assert r["n_gpus"] == 4 and r["launches_per_step"] > 1
    assert r["parity_vs_oracle_on_sample"] is True and r["parity_gathered_vs_rank0_kernel"] is True, r


@pytest.mark.parametrize("world", [1, 2, 4])
def test_bench_config4_strong_scaling_leg(world):
    """The config-4 strong-scaling leg after the config-2 loop: a fixed fleet cut over N ranks
    (gloo ranks sharing the GPU; N = 1 chunked, records written into page-locked memory),
    every shard's gathered records equal to the oracle and to rank 0's kernel on sampled
    blocks, per-rank kernel times reported."""
    r = _bench(["--gpus", str(world), "--containers", "400", "--steps", "2", "--warmup", "1", "--parity-block", "64",
                "--c4-containers", "6000", "--c4-steps", "2", "--chunk-gib", "0.1", "--no-cpu-baseline",
                "--no-host-path"], timeout=300)
    assert r["n_gpus"] == world
    assert r["config4_parity_vs_oracle_on_sample"] is True, r
    assert r["config4_parity_gathered_vs_rank0_kernel"] is True, r
    assert r["config4_parity_sample_containers"] >= world * 64
    assert len(r["config4_per_rank_kernel_ms"]) == world and r["config4_containers_per_s"] > 0
    assert r["config4_kernel_ms_max"] == max(r["config4_per_rank_kernel_ms"])
    if world > 1:
        assert len(r["config4_per_rank_gather_ms"]) == world


def test_bench_sharded_host_path_two_ranks():
    """N > 1 host path (gloo rehearsal): every rank packs ITS objects' query_range bodies on its
    GPU with the hybrid parser (BatchedRunner.recommend_bodies_shard), rank 0 rounds the whole
    fleet; the per-rank e2e times are reported and sampled objects of every shard equal the
    host packer's path."""
    r = _bench(["--gpus", "2", "--containers", "400", "--steps", "2", "--warmup", "1", "--parity-block", "64",
                "--c4-containers", "0", "--no-cpu-baseline", "--host-objects", "300"], timeout=300)
    assert r["e2e_parser"] == "hybrid" and len(r["e2e_per_rank_s"]) == 2 and r["e2e_objects_per_s"] > 0, r
    assert r["e2e_sharded_equals_host_parse"] is True and r["e2e_parity_objects"] == 2 * 2 * 32


def test_bench_rccl_one_rank_config4_leg_and_sharded_host_path():
    """The N > 1 code of the config-4 leg (C-ABI gather on the launch stream, receive buffers
    forwarded to the host by the next launch) and of the sharded host path
    (recommend_bodies_shard's records gathered over RCCL) at one RCCL rank (`--force-dist`):
    every key present, parity true."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), KRR_BENCH_BACKEND="nccl")
    p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.join(ROOT, "bench.py"), "--force-dist",
                        "--containers", "400", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--c4-containers", "5000", "--c4-steps", "2", "--chunk-gib", "0.1", "--sharded-host-path",
                        "--host-objects", "200"], capture_output=True, text=True, env=env, timeout=270)
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["config4_parity_vs_oracle_on_sample"] is True and r["config4_parity_gathered_vs_rank0_kernel"] is True
    assert r["config4_definition"].find("RCCL gather") >= 0 and r["config4_gather_ms_max"] >= 0
    assert r["e2e_sharded_equals_host_parse"] is True and len(r["e2e_per_rank_s"]) == 1
