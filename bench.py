"""Throughput bench of the KRR SimpleStrategy hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--mode linear|sorted_lower|ref_index]

One "step" = one pass of the hot path over the rank's whole synthetic fleet
shard, inputs resident in HBM: the CPU-percentile kernel over every CPU series,
the max+count kernel over every memory series, and (N > 1) the RCCL gather of
the 32-B per-container result records to rank 0 on the same stream, whose copy to
host memory is done by rank 0's next launch (the last one's after the loop).

Ranks: one process per GPU.  Under torchrun (WORLD_SIZE set) the world size must
equal --gpus.  Without it, `--gpus N > 1` makes this process a launcher: it spawns
N ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT)
before anything touches the GPU, never touches the GPU itself, and exits non-zero
if any rank fails.  Backend "nccl" (RCCL over xGMI) needs N GPUs;
KRR_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share a device).

Workloads (BASELINE.json configs); every container is generated from its GLOBAL
index, so an N-rank fleet is the N=1 fleet cut into shards (config 4) or extended
by more containers (weak scaling, configs 2-3):
  2 (default) 10k containers x 5 pods x 10,080 slots (7d@1m) per rank, NaN-gapped dense layout
  3           100k containers per rank x 1 pod, windows of 1..14 days @1m (1,440-20,160 samples), compact CSR
  4           1M containers x 10,080 samples (7d@1m) split across the ranks, compact CSR
  5           sketch mode: 100k CPU series x 172,800 samples (30d@15s) TIME-sharded across the
              ranks (rank r holds the r-th time slice of every series); per-slice log-linear
              sketches merged by one reduce-scatter, rank error vs the exact path reported
Data are generated on the device by krr_synth_fill_global (counter hash; no host packing, no PCIe).

Prints ONE JSON line on rank 0 (contract in the task brief): value = containers of ALL
ranks / max-over-ranks step time; roofline = the fused kernel's algorithmic
bytes / its average launch time (HIP events on the launch stream) against 8 TB/s;
cpu_baseline = the C oracle (OpenMP, the lease's cores) on a bounded sample copied from
the device (N = 1); parity_vs_oracle_on_sample = this run's results (N > 1: the records
gathered to rank 0) against the oracle on a sample regenerated from every shard.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time
from typing import Optional
from decimal import Decimal

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "container-series/sec right-sized (7d@1m) + % of HBM BW, 1/2/4/8 MI355X"
HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SLOTS_7D = 10080


_JSON_OUT = sys.stdout


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--sketch-bits", type=int, default=5, help="config 5: log-linear bins per octave = 2^bits")
    ap.add_argument("--sketch-only", action="store_true",
                    help="config 5: stop at the sketch answer (approximate) instead of the exact refinement")
    ap.add_argument("--sketch-kind", choices=("kll", "loglinear"), default="kll",
                    help="config 5 --sketch-only: kll = KLL-style compactor sketch (rank error bounded whatever the "
                         "data, reported as sketch_error.rank_error_bound); loglinear = the log-linear histogram "
                         "(value error <= 2^-bits, rank error measured only)")
    ap.add_argument("--kll-budget", type=int, default=512, help="config 5 kll: body keys kept per row")
    ap.add_argument("--kll-tail", type=int, default=-1,
                    help="config 5 kll: exact top keys per row (-1: just enough for --percentile of the whole "
                         "30d@15s series, i.e. p99 answered exactly; none when more than 4,096 would be needed)")
    ap.add_argument("--c5-refine", action="store_true",
                    help="config 5 at N=1: run the time-sharded exact path (--c5-method) instead of the direct "
                         "single-window select (N>1 always uses it)")
    ap.add_argument("--c5-method", choices=("window", "sketch"), default="window",
                    help="config 5 time-sharded exact path: window = one HBM pass (window export + all-to-all + "
                         "merge, misses regathered); sketch = sketch build + reduce-scatter + locate + collect "
                         "(a second HBM pass) + refine")
    ap.add_argument("--error-sample", type=int, default=256, help="config 5: series checked against the exact path")
    ap.add_argument("--mode", default="linear", choices=["linear", "sorted_lower", "ref_index"])
    ap.add_argument("--percentile", default="99")
    ap.add_argument("--containers", type=int, default=0, help="override containers per rank (testing)")
    ap.add_argument("--pods", type=int, default=5, help="config 2: pods per container (segment = pods x 10,080)")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="containers in the CPU-baseline / parity sample (0: the whole rank, capped at 1.1e9 slots)")
    ap.add_argument("--numpy-seconds", type=float, default=5.0,
                    help="time budget of the single-thread numpy reference-path baseline")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the lease's cores (affinity set, capped by OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-blocks", type=int, default=4, help="N > 1 parity: sampled blocks per shard")
    ap.add_argument("--parity-block", type=int, default=128, help="N > 1 parity: containers per sampled block")
    ap.add_argument("--separate", action="store_true", help="two launches (percentile, max) instead of the fused one")
    ap.add_argument("--gather", choices=("stream", "torch", "blocking"), default="stream",
                    help="N > 1 records path: stream = RCCL send/recv through the C ABI on the launch stream "
                         "(gloo: torch); torch = torch.distributed.gather on its own stream, step k's gather "
                         "overlapping step k+1's kernel; blocking = torch gather + host copy after each kernel")
    ap.add_argument("--comm", choices=("own", "torch"), default="own",
                    help="N > 1, --gather stream: the RCCL communicator the C-ABI gather uses: own = the "
                         "library's (krr_comm_unique_id on rank 0, the id broadcast over torch.distributed, "
                         "krr_comm_init_timeout on every rank); torch = torch.distributed's own (a private "
                         "ProcessGroupNCCL accessor)")
    ap.add_argument("--records", choices=("host", "device"), default="host",
                    help="N = 1: the fused launch writes the 32-B records straight into page-locked host "
                         "memory (host) or into HBM followed by a D2H copy (device)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the N > 1 path (process group + pipelined RCCL gather) even with one rank (testing)")
    ap.add_argument("--c5-chunk-gib", type=float, default=3.0,
                    help="config 5 at N = 1 (direct): series per launch, in GiB of values, each chunk in buffers "
                         "of its own; 2-4 GiB streamed at 83-85%% of peak, 8 GiB at 82%%, 16-32 GiB at 81-82%%, "
                         "one 138-GB buffer at 77%% (profiles/r03/f, profiles/r03/g)")
    ap.add_argument("--chunk-gib", type=float, default=8.0,
                    help="fleets of more than twice this many GiB of values per resource run as chunks of "
                         "about this size, in buffers of their own, one launch per chunk")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--deadline", type=float, default=float(os.environ.get("KRR_BENCH_DEADLINE", "540")),
                    help="--gpus N > 1 launcher: seconds before every rank is stopped (SIGTERM, then SIGKILL) and "
                         "one JSON line with status 'timeout' and each rank's last phase is printed")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds torch.distributed waits in a collective / rendezvous before failing")
    ap.add_argument("--c4-containers", type=int, default=-1,
                    help="config 2 runs: containers of the config-4 strong-scaling leg after the timed loop "
                         "(-1: 1,000,000 on the default workload, off when --containers is given; 0: off)")
    ap.add_argument("--c4-steps", type=int, default=5, help="config-4 leg: timed steps")
    ap.add_argument("--c4-warmup", type=int, default=1, help="config-4 leg: warmup steps")
    ap.add_argument("--host-objects", type=int, default=2000,
                    help="host path: config-1-shaped objects per rank (3 pods x 10,080 samples x 2 resources)")
    ap.add_argument("--sharded-host-path", action="store_true",
                    help="testing: the N > 1 host path (recommend_bodies_shard) at one rank (with --force-dist)")
    ap.add_argument("--host-parser", choices=("hybrid", "device", "host"), default="hybrid",
                    help="N > 1 host path: the parser each rank uses for its shard's bodies")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-path measurements (H2D, native packer, end-to-end from JSON bodies)")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="leave the process on every CPU it may use (default: the GPU-local NUMA node's)")
    ap.add_argument("--no-right-size", action="store_true",
                    help="config-4 leg: skip right-sizing + scanning the whole fleet on rank 0 after its steps")
    args = ap.parse_args()
    if args.c4_containers < 0:
        args.c4_containers = 1_000_000 if args.containers == 0 else 0
    return args


_LAST_PHASE = ["started"]


_NUMA: Optional[dict] = None  # this rank's NUMA binding (main), reported in the host-path keys


def phase(name: str) -> None:
    """This rank's progress on stderr (the launcher keeps each rank's last phase)."""
    _LAST_PHASE[0] = name
    print(f"KRR_PHASE rank={os.environ.get('RANK', '0')} {name}", file=sys.stderr, flush=True)


def start_rank_watchdog(args, rank: int, world: int) -> None:
    """Under an external launcher (torchrun: the driver's N > 1 runs) nothing stops a rank
    that hangs in a rendezvous or a collective before the launcher's own limit, and the run
    would end with no JSON line.  After --deadline seconds this thread ends the rank:
    rank 0 first prints ONE JSON line with status "timeout" and its last phase, then every
    rank exits with 124 (os._exit: nothing the hung main thread holds is waited for)."""
    import threading

    def watch():
        time.sleep(args.deadline)
        print(f"bench.py rank {rank}: deadline of {args.deadline:.0f} s passed in phase {_LAST_PHASE[0]!r}",
              file=sys.stderr, flush=True)
        if rank == 0 and _JSON_OUT is not None:
            try:
                print(json.dumps({"metric": METRIC, "n_gpus": world, "status": "timeout", "deadline_s": args.deadline,
                                  "rank_phases": {"0": _LAST_PHASE[0]}}), file=_JSON_OUT, flush=True)
            except (OSError, ValueError):
                pass
        os._exit(124)

    threading.Thread(target=watch, daemon=True, name="krr-bench-watchdog").start()


def _splitmix(x: np.ndarray) -> np.ndarray:
    z = (x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def container_lengths(cfg: int, g0: int, g1: int, pods: int = 5) -> np.ndarray:
    """Slots per container for GLOBAL container indices [g0, g1) (same on every rank)."""
    n = max(g1 - g0, 0)
    if cfg == 2:
        return np.full(n, pods * SLOTS_7D, dtype=np.int64)
    if cfg == 3:  # window uniform over {1..14} days @1m
        with np.errstate(over="ignore"):
            h = _splitmix(np.arange(g0, g1, dtype=np.uint64) ^ np.uint64(0xC0F1_6303))
        return ((h % np.uint64(14)).astype(np.int64) + 1) * 1440
    return np.full(n, SLOTS_7D, dtype=np.int64)


def fleet_shard(cfg: int, rank: int, world: int, override: int) -> tuple[int, int, int]:
    """(g0, g1, containers_total): the global container range rank `rank` owns."""
    if cfg in (2, 3):  # weak scaling: a fixed number of containers per rank
        n = override or (10_000 if cfg == 2 else 100_000)
        return rank * n, (rank + 1) * n, n * world
    total = override * world if override else 1_000_000
    from krr_amd.core.distributed import shard_bounds  # equal lengths: contiguous equal cuts

    g0, g1 = shard_bounds(np.full(total, SLOTS_7D, dtype=np.int64), world)[rank]
    return g0, g1, total


def workload(cfg: int, rank: int, world: int, override: int, pods: int = 5):
    """Per-rank (offsets, pod_len, gaps, description, containers_total, g0)."""
    g0, g1, total = fleet_shard(cfg, rank, world, override)
    L = container_lengths(cfg, g0, g1, pods)
    offs = np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
    n = g1 - g0
    if cfg == 2:
        return offs, SLOTS_7D, True, (f"config2: {n} containers/rank x {pods} pods x 10080 slots (7d@1m), "
                                      f"NaN-gapped dense"), total, g0
    if cfg == 3:
        return offs, 0, False, f"config3: {n} containers/rank x 1 pod, 1..14 days @1m, compact CSR", total, g0
    return offs, 0, False, (f"config4: {total} containers x 10080 samples (7d@1m) over {world} ranks, "
                            f"compact CSR"), total, g0


def fleet_chunks(offs_np: np.ndarray, chunk_gib: float) -> list[tuple[int, int]]:
    """Contiguous object ranges of about chunk_gib GiB of values each (one range when the
    fleet holds at most twice that), cut by sample-balanced prefix sums."""
    from krr_amd.core.distributed import shard_bounds

    S = offs_np.size - 1
    nbytes = 8 * int(offs_np[-1])
    limit = max(chunk_gib, 1e-3) * 2**30
    if S == 0 or nbytes <= 2 * limit:
        return [(0, S)]
    n = int(np.ceil(nbytes / limit))
    return [(lo, hi) for lo, hi in shard_bounds(np.diff(offs_np), n) if hi > lo]


class _gc_timer:
    """Python garbage-collector passes (per generation) and their seconds until stop()."""

    def __init__(self):
        import gc

        self.t = {}
        self.n = {}
        self._t0 = None

        def cb(phase, info):
            if phase == "start":
                self._t0 = time.perf_counter()
            elif self._t0 is not None:
                g = info.get("generation", -1)
                self.t[g] = self.t.get(g, 0.0) + time.perf_counter() - self._t0
                self.n[g] = self.n.get(g, 0) + 1
                self._t0 = None

        self._cb = cb
        gc.callbacks.append(cb)

    def stop(self) -> dict:
        import gc

        gc.callbacks.remove(self._cb)
        return {f"gen{g}": [self.n[g], round(self.t[g], 5)] for g in sorted(self.t)}


def cgroup_cpu() -> dict:
    """The CPU controller's quota and throttling counters of this process's cgroup (v2 or v1
    files; {} where absent): a host phase that runs more busy threads than the quota allows is
    stopped for the rest of each period, which shows up as nr_throttled / throttled_usec."""
    out = {}
    for base in ("/sys/fs/cgroup", "/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
        try:
            with open(os.path.join(base, "cpu.stat")) as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    if k in ("nr_periods", "nr_throttled", "throttled_usec", "throttled_time", "usage_usec"):
                        out[k] = int(v)
        except (OSError, ValueError):
            continue
        for name in ("cpu.max", "cpu.cfs_quota_us"):
            try:
                with open(os.path.join(base, name)) as fh:
                    out[name] = fh.read().strip()
            except OSError:
                pass
        break
    return out


def cpu_lease() -> dict:
    """Host cores this process may use: the affinity set, capped by OMP_NUM_THREADS when the
    box sets it (the GPU box leases 16 CPUs per GPU but shows the whole machine's)."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = list(range(os.cpu_count() or 1))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    n = len(aff)
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return {"threads": max(n, 1), "nproc": os.cpu_count(), "affinity_cpus": len(aff),
            "omp_num_threads": omp or None}


def launch_ranks(args) -> int:
    """--gpus N > 1 without torchrun: spawn N ranks (fresh interpreters, nothing here
    touches the GPU), forward their output, return the first failing exit code.

    Every rank reports its phase on stderr (init, synth, warmup, step k, gather, report);
    the launcher keeps each rank's last one.  If the ranks are still running after
    --deadline seconds (e.g. one hangs in a rendezvous or a collective), they are all
    stopped (SIGTERM, then SIGKILL) and ONE JSON line with status "timeout" and every
    rank's last phase is printed, exit code 124."""
    import signal
    import socket
    import subprocess
    import threading

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs, phases = [], {}
    lock = threading.Lock()

    def pump(r, pipe):
        for raw in iter(pipe.readline, b""):
            line = raw.decode(errors="replace")
            if line.startswith("KRR_PHASE "):
                with lock:
                    phases[r] = line.split(" ", 2)[2].strip()
            sys.stderr.write(line)
            sys.stderr.flush()

    pumps = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   KRR_BENCH_LAUNCHED="1")
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                             stderr=subprocess.PIPE)
        procs.append(p)
        phases[r] = "started"
        t = threading.Thread(target=pump, args=(r, p.stderr), daemon=True)
        t.start()
        pumps.append(t)
    rc = 0
    alive = set(range(args.gpus))
    kill_at = None
    t_end = time.time() + args.deadline
    timed_out = False
    while alive:
        for r in sorted(alive):
            c = procs[r].poll()
            if c is None:
                continue
            alive.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench.py launcher: rank {r} exited with {c}; stopping the others", file=sys.stderr)
                for q in alive:
                    procs[q].send_signal(signal.SIGTERM)
                kill_at = time.time() + 20
        if alive and not timed_out and time.time() > t_end:
            timed_out = True
            with lock:
                last = {str(q): phases.get(q) for q in range(args.gpus)}
            print(f"bench.py launcher: deadline of {args.deadline:.0f} s passed; stopping ranks {sorted(alive)}",
                  file=sys.stderr)
            for q in alive:
                procs[q].send_signal(signal.SIGTERM)
            kill_at = time.time() + 10
            print(json.dumps({"metric": METRIC, "n_gpus": args.gpus, "status": "timeout",
                              "deadline_s": args.deadline, "ranks_running": sorted(alive), "rank_phases": last}),
                  file=_JSON_OUT, flush=True)
            rc = 124
        if kill_at is not None and time.time() > kill_at:
            for q in alive:
                procs[q].kill()
            kill_at = None
        time.sleep(0.1)
    for t in pumps:
        t.join(timeout=5)
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} "
                     f"(launch one rank per GPU: torchrun --nproc-per-node {args.gpus}, or no torchrun)")
    elif args.gpus > 1:
        sys.exit(launch_ranks(args))
    elif args.force_dist:  # a one-rank process group of its own
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # Native libraries (RCCL's version banner, gloo's peer messages) write to fd 1:
    # point fd 1 at stderr and keep the real stdout for the ONE JSON line.
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if "WORLD_SIZE" in os.environ and not os.environ.get("KRR_BENCH_LAUNCHED"):
        start_rank_watchdog(args, int(os.environ.get("RANK", "0")), int(os.environ["WORLD_SIZE"]))
    if os.environ.get("KRR_BENCH_TEST_HANG"):  # tests: a rank that never finishes (deadlines)
        phase("init")
        while True:
            time.sleep(1)
    import torch
    import torch.distributed as dist

    from krr_amd import _native
    from krr_amd.core.distributed import gather_records, record_counts
    from krr_amd.core.engine import percentile_params

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --force-dist: run the N > 1 code path (process group, pipelined gather) even at
    # one rank, so the RCCL path is exercised on a one-GPU box
    dist_on = world > 1 or args.force_dist
    ndev = torch.cuda.device_count()
    if os.environ.get("KRR_BENCH_BACKEND", "nccl") != "nccl":
        local %= max(ndev, 1)  # rehearsal: several ranks may share a GPU
    elif local >= ndev:
        sys.exit(f"bench.py rank {rank}: LOCAL_RANK {local} but only {ndev} GPU(s) visible; RCCL needs one GPU "
                 f"per rank (KRR_BENCH_BACKEND=gloo rehearses several ranks on one GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # the host side (staging, host packer, DMA sources) next to this rank's GPU: threads created
    # and pages first touched from here on stay on its NUMA node (krr_amd.utils.numa)
    global _NUMA
    if not args.no_numa_bind:
        from krr_amd.utils.numa import bind_local, gpu_numa_node

        cpus = bind_local(local)
        _NUMA = {"gpu_node": gpu_numa_node(local), "bound_cpus": len(cpus) if cpus else None}
    # RCCL ("nccl") over xGMI in production; KRR_BENCH_BACKEND=gloo rehearses the
    # N>1 path with several ranks on ONE GPU (RCCL refuses duplicate devices).
    backend = os.environ.get("KRR_BENCH_BACKEND", "nccl")
    if dist_on:
        import datetime

        phase("init")
        tmo = datetime.timedelta(seconds=args.dist_timeout)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    if args.config == 5:
        return run_config5(args, world, rank, local, dev, coll_dev)

    offs_np, pod_len, gaps, desc, containers_total, g0 = workload(args.config, rank, world, args.containers,
                                                                   args.pods)
    S = offs_np.size - 1
    N = int(offs_np[-1])
    ctx = _native.Context(local)
    seed = 1000003 * (args.config + 1)  # one fleet: containers are generated from their global index
    params = percentile_params(Decimal(args.percentile), args.mode)
    # A fleet of more than 2 chunks' values per resource lives in buffers of about
    # --chunk-gib each, one launch per chunk (config 4 at N <= 2): at 700k containers one
    # 113 GB launch streamed at 79.8% of peak and 7 launches over buffers of their own at
    # 84.3%, on a box where 125k containers in one launch ran at 83.6% (same process,
    # scripts/footprint_ab.py, profiles/r02/footprint)
    chunks = fleet_chunks(offs_np, args.chunk_gib)
    phase("synth")
    parts = []
    for lo, hi in chunks:
        o_np = (offs_np[lo:hi + 1] - offs_np[lo]).astype(np.int64)
        o = torch.from_numpy(o_np).to(dev)
        c = torch.empty(int(o_np[-1]), dtype=torch.float64, device=dev)
        m = torch.empty(int(o_np[-1]), dtype=torch.float64, device=dev)
        ctx.synth_fill(c, o, seed, 0, pod_len, gaps, seg_base=g0 + lo)
        ctx.synth_fill(m, o, seed ^ 0x5A5A, 1, pod_len, gaps, seg_base=g0 + lo)
        ml = int(np.max(np.diff(o_np))) if hi > lo else 0
        parts.append((lo, hi, c, m, ctx.series(c, o, ml, gaps), ctx.series(m, o, ml, gaps)))
    torch.cuda.synchronize()

    def host_values(end):
        """The first `end` slots of both resources on the host (parity / CPU baseline)."""
        cs_, ms_ = [], []
        for lo, hi, c, m, _, _ in parts:
            a = int(offs_np[lo])
            if a >= end:
                break
            k = min(end, int(offs_np[hi])) - a
            cs_.append(c[:k].cpu().numpy())
            ms_.append(m[:k].cpu().numpy())
        return np.concatenate(cs_), np.concatenate(ms_)
    out = {
        "cpu_value": torch.empty(S, dtype=torch.float64, device=dev),
        "cpu_count": torch.empty(S, dtype=torch.int64, device=dev),
        "cpu_flags": torch.empty(S, dtype=torch.int32, device=dev),
        "mem_value": torch.empty(S, dtype=torch.float64, device=dev),
        "mem_count": torch.empty(S, dtype=torch.int64, device=dev),
        "mem_flags": torch.empty(S, dtype=torch.int32, device=dev),
    }
    stream = torch.cuda.current_stream()
    host_rec = torch.empty((containers_total if rank == 0 else S, 4), dtype=torch.int64, pin_memory=True)
    counts = record_counts(S, coll_dev) if dist_on else None  # shard sizes are fixed: exchange once
    gather_mode = args.gather if dist_on else None
    if gather_mode == "stream" and args.separate:
        gather_mode = "torch"
    comm, comm_src = None, None
    if gather_mode == "stream" and backend == "nccl":
        comm, comm_src = make_comm(args, ctx, dev, world, rank)
    if gather_mode == "stream" and comm is None:
        gather_mode = "torch"
    # N > 1 over RCCL, "stream" (default): the gather is enqueued on the launch stream through
    # the C ABI (krr_gather_results with torch's communicator), so a step is launch -> send/recv
    # with no cross-stream dependency in the launch queue (each cost 20-30 us of idle queue,
    # profiles/r02/fdtrace).  Rank 0's launch writes its own records into the head of the
    # receive buffer (no self copy) and, as its first work items, forwards the PREVIOUS step's
    # gathered records (N x 320 KB) into page-locked host memory (krr_simple_run_forward): no
    # second stream, no separate D2H (on the launch stream 2.56 MB cost +60 us per step;
    # scripts/d2h_overlap.py).  Two receive buffers alternate; the last step's records are
    # copied after the loop, inside the timed region.
    copy_stream = torch.cuda.Stream(device=dev) if dist_on and coll_dev.type == "cuda" else None
    recv = [torch.empty((containers_total, 4), dtype=torch.int64, device=dev) for _ in range(2)] \
        if gather_mode == "stream" and rank == 0 else []
    # "torch": torch.distributed.gather on torch's RCCL stream, step k's gather waited for
    # one step later; two send buffers alternate so it sends from the buffer the launch wrote
    dev_recs = [torch.empty((S, 4), dtype=torch.int64, device=dev) for _ in range(2)]
    dev_rec = dev_recs[0]

    # N = 1, fused: the launch can write its records straight into the page-locked host
    # buffer (mapped into the device's address space) instead of HBM + a D2H copy
    zero_copy = args.records == "host" and not dist_on and not args.separate

    def run_all(records, fwd=None):
        """The fused launch over every chunk (one chunk: one launch); records rows follow
        the containers; the forward copy rides the first launch."""
        for j, (lo, hi, _, _, cs, ms) in enumerate(parts):
            ctx.simple_run(cs, ms, params, {key: v[lo:hi] for key, v in out.items()}, stream,
                           records=records[lo:hi], forward=fwd if j == 0 else None)

    nstep = [0]

    def step(events=None):
        k = nstep[0]
        nstep[0] += 1
        dev_rec = dev_recs[k % 2] if copy_stream is not None else dev_recs[0]
        if gather_mode == "stream":
            fwd = None
            if rank == 0:
                dev_rec = recv[k % 2][:S]
                if k > 0:
                    fwd = (recv[(k - 1) % 2], host_rec)
            if events is not None:
                events[0].record(stream)
            run_all(dev_rec, fwd)
            if events is not None:
                events[1].record(stream)
            if rank == 0:
                ctx.gather_results(comm, 0, dev_rec, counts=counts, out=recv[k % 2], stream=stream)
                last[0] = recv[k % 2]
            else:
                ctx.gather_results(comm, 0, dev_rec, stream=stream)
            if events is not None:
                events[2].record(stream)
            return
        if events is not None:
            events[0].record(stream)
        if zero_copy:
            run_all(host_rec)
            if events is not None:
                events[1].record(stream)
            return
        if args.separate:
            for lo, hi, _, _, cs, _ in parts:
                ctx.segmented_percentile(cs, params, out["cpu_value"][lo:hi], out["cpu_count"][lo:hi],
                                         out["cpu_flags"][lo:hi], stream)
            if events is not None:
                events[1].record(stream)
            for lo, hi, _, _, _, ms in parts:
                ctx.segmented_max(ms, out["mem_value"][lo:hi], out["mem_count"][lo:hi], out["mem_flags"][lo:hi],
                                  stream)
            if events is not None:
                events[2].record(stream)
        if args.separate:
            ctx.pack_records(out, dev_rec, stream)  # one launch: 32-B records
        else:  # ONE launch per chunk: CPU percentile + memory max for every container, records included
            run_all(dev_rec)
            if events is not None:
                events[1].record(stream)
        if not dist_on:
            host_rec.copy_(dev_rec, non_blocking=True)
            return
        # this step's gather stays in flight (torch's RCCL stream) while the next step's
        # kernel runs; it is waited for one step later (and by finish())
        pend = gather_records(dev_rec.to(coll_dev), dst=0, counts=counts, async_op=True,
                              copy_local=copy_stream is None)
        if gather_mode == "blocking":  # no overlap: the step ends with its own gather
            inflight.append(pend)
            finish()
            return
        finish()
        inflight.append(pend)

    inflight = []
    last = [None]

    def finish():
        if last[0] is not None:  # "stream": the last step's gathered records (no launch follows)
            host_rec.copy_(last[0], non_blocking=True)
            last[0] = None
        while inflight:
            pend = inflight.pop()
            if copy_stream is None:  # gloo (host tensors)
                rec = pend.wait()
                if rank == 0:
                    host_rec[: rec.shape[0]].copy_(rec, non_blocking=True)
                continue
            # the launch stream waits for the gather (done long since: it overlapped the
            # launch just enqueued) before the NEXT launch rewrites the buffer it sent
            rec = pend.wait()
            if rank == 0:
                ready = torch.cuda.Event()
                ready.record(stream)
                copy_stream.wait_event(ready)
                with torch.cuda.stream(copy_stream):
                    host_rec[: rec.shape[0]].copy_(rec, non_blocking=True)
                rec.record_stream(copy_stream)  # the receive buffer outlives the copy

    rccl_info = None
    if comm is not None:
        try:
            n_comm, r_comm = ctx.comm_info(comm)
            rccl_info = {"ranks": n_comm, "rank0_rank": r_comm, "communicator": comm_src,
                         "source": "ncclCommCount/ncclCommUserRank through krr_comm_info"}
        except _native.NativeError as e:
            rccl_info = {"error": str(e), "communicator": comm_src}
    elif dist_on and backend == "nccl":
        rccl_info = {"ranks": None, "note": "torch.distributed's communicator not exposed: torch.distributed.gather"}
    if gather_mode == "stream":
        # first use of the C-ABI gather on torch's communicator: if it fails on any rank
        # (an error return, not a hang), every rank falls back to torch.distributed.gather
        ok = True
        try:
            step()
            torch.cuda.synchronize()
        except _native.NativeError as e:
            print(f"bench.py rank {rank}: C-ABI gather failed ({e}); using torch.distributed.gather",
                  file=sys.stderr)
            ok = False
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            gather_mode = "torch"
            last[0] = None
    phase("warmup")
    for _ in range(args.warmup):
        step()
    finish()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    phase(f"timed {args.steps} steps")
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    finish()  # the last step's gather + host copy are inside the timed region
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    t1 = time.perf_counter()
    phase("report")
    dt = torch.tensor([(t1 - t0) / args.steps], dtype=torch.float64, device=coll_dev)
    if dist_on:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    step_s = float(dt.item())
    k1_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    k2_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs])) if args.separate else 0.0
    # N > 1: where each rank's step goes (kernel on the launch stream; the RCCL gather
    # enqueued after it on the same stream, "stream" mode only)
    per_rank = None
    if dist_on:
        g_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs])) if gather_mode == "stream" else float("nan")
        mine = torch.tensor([k1_ms, g_ms], dtype=torch.float64, device=coll_dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[float(x) for x in t.cpu().tolist()] for t in allr]

    # algorithmic bytes per launch: every stored slot once, offsets, outputs
    seg_bytes = 8 * N + 8 * (S + 1) + (8 + 8 + 4) * S  # one resource
    # compact REF_INDEX reads one sample per CPU segment (an index into the unsorted list),
    # not the segment: offsets + the gathered sample + outputs
    dense_ref = args.mode == "ref_index" and not gaps
    cpu_bytes = 8 * (S + 1) + 8 * S + (8 + 8 + 4) * S if dense_ref else seg_bytes
    if args.separate:
        kname = "k_select" if args.mode != "ref_index" else ("k_refindex_gaps" if gaps else "k_refindex_dense")
        kbytes, kms = cpu_bytes, k1_ms
        kernels = {kname: k1_ms, "k_max": k2_ms}
    else:
        kname = "k_simple" if not dense_ref else "k_refindex_dense+k_max"
        kbytes, kms = cpu_bytes + seg_bytes, k1_ms
        kernels = {kname: k1_ms}
    achieved = kbytes / (kms * 1e-3)
    step_bytes_all = (cpu_bytes + seg_bytes) * world
    result = {
        "metric": METRIC,
        "value": containers_total / step_s,
        "unit": "container-series/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if args.config != 4 else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device counter-hash: CPU ~ Gamma(2, 0.05) cores, memory ~ floor(N(2e8, 2e7)) bytes)",
        "config": {
            "workload": desc,
            "percentile_mode": args.mode,
            "cpu_percentile": args.percentile,
            "memory_buffer": "max x 1.05 (exact decimal, host)",
            "containers": containers_total,
            "slots_per_rank": 2 * N,
            "parallelism": f"shard{world} (contiguous container ranges, RCCL gather of 32-B records)",
        },
        "samples_per_s": 2 * N * world / step_s,
        "launches_per_step": len(parts),
        "hbm_frac_step": step_bytes_all / step_s / (HBM_PEAK * world),
        "kernels_ms": kernels,
        "roofline": {
            "kernel": kname,
            "bound": "hbm",
            "achieved": achieved / 1e9,
            "peak": HBM_PEAK / 1e9,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK,
            "traffic": None,
            "algorithmic_bytes_per_launch": kbytes,
        },
    }
    if args.mode == "ref_index" and not gaps:
        result["roofline"]["note"] = ("compact REF_INDEX: the CPU half is one gather per segment (offsets + one "
                                      "sample + outputs), the memory half streams every slot")
    result["config"]["records"] = "page-locked host memory, written by the launch" if zero_copy else \
        "HBM + D2H copy" if not dist_on else "HBM + RCCL gather to rank 0"
    if per_rank is not None:
        result["per_rank_kernel_ms"] = [r[0] for r in per_rank]
        result["kernel_ms_max"] = max(r[0] for r in per_rank)
        if gather_mode == "stream":
            result["per_rank_gather_ms"] = [r[1] for r in per_rank]
            result["gather_ms_max"] = max(r[1] for r in per_rank)
    if dist_on:
        result["config"]["gather"] = {"stream": "RCCL send/recv on the launch stream (C ABI krr_gather_results)",
                                      "torch": "torch.distributed.gather, overlapping the next launch",
                                      "blocking": "torch.distributed.gather, waited for each step"}[gather_mode]
        # what actually carried the records (after any fallback), and how many ranks RCCL saw
        result["gather_mode_requested"] = args.gather
        result["gather_mode_used"] = gather_mode
        result["rccl_comm"] = rccl_info
    if zero_copy or (dist_on and rank == 0 and not args.separate):
        # the host buffer holds exactly what the launch computed (after the last step's sync);
        # N > 1: rank 0's own shard leads the gathered records
        ctx.pack_records(out, dev_rec, stream)
        torch.cuda.synchronize()
        result["records_host_equal_device"] = bool(torch.equal(dev_rec.cpu(), host_rec[:S]))
    # PMC-measured HBM bytes per launch of the same kernel/workload (profiles/pmc_traffic.json)
    try:
        with open(args.traffic) as fh:
            tr = json.load(fh)
        key = f"config{args.config}:{args.mode}:p{args.percentile}:{result['roofline']['kernel']}"
        if key in tr and int(tr[key].get("containers_per_rank", -1)) == S:
            result["roofline"]["traffic"] = tr[key]["hbm_bytes_per_launch"]
            result["roofline"]["traffic_source"] = tr[key].get("source")
    except (OSError, ValueError):
        pass

    # parity of this very run on a sample + the CPU baseline (rank 0, N = 1 only)
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        from oracle import oracle

        m = S if args.cpu_sample <= 0 else max(1, min(args.cpu_sample, S))
        m = max(1, min(m, int(np.searchsorted(offs_np, 1_100_000_000, side="right")) - 1))
        end = int(offs_np[m])
        c_host, m_host = host_values(end)
        o_host = offs_np[: m + 1].copy()
        lease = cpu_lease()
        threads = args.cpu_threads or lease["threads"]
        t_a = time.perf_counter()
        ov, on, of = oracle.percentile(c_host, o_host, params.mode, params.p_num, params.p_den, params.q, gaps,
                                       threads)
        mv, mn, mf = oracle.seg_max(m_host, o_host, gaps, threads)
        t_b = time.perf_counter()
        gv = out["cpu_value"][:m].cpu().numpy()
        same = (gv.view(np.uint64) == ov.view(np.uint64)) | (np.isnan(gv) & np.isnan(ov))
        if args.mode == "linear":
            same |= (gv == 0) & (ov == 0)
        parity = bool(same.all() and np.array_equal(out["cpu_count"][:m].cpu().numpy(), on)
                      and np.array_equal(out["mem_value"][:m].cpu().numpy(), mv, equal_nan=True)
                      and np.array_equal(out["mem_count"][:m].cpu().numpy(), mn))
        cpu_model = ""
        try:
            with open("/proc/cpuinfo") as fh:
                cpu_model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
        except OSError:
            pass
        result["cpu_baseline"] = {
            "value": m / (t_b - t_a),
            "unit": "container-series/s",
            "cores": threads,
            "kind": "port",
            "sample": f"first {m} containers of this run ({2 * end} slots) copied D2H; oracle/krr_oracle.c "
                      f"{args.mode} + max, OpenMP {threads} threads on {cpu_model or platform.processor()}",
            "host": {"cpu_model": cpu_model or platform.processor(), **lease},
        }
        result["parity_vs_oracle_on_sample"] = parity
        result["parity_sample_containers"] = m
        # the reference's path restated in numpy (single thread): per container, the
        # pods' present samples -> np.percentile / np.max, as long as the time budget lasts
        t_c = time.perf_counter()
        done = 0
        qv = float(args.percentile)
        while done < m and time.perf_counter() - t_c < args.numpy_seconds:
            a, b = int(o_host[done]), int(o_host[done + 1])
            xc = c_host[a:b]
            xm = m_host[a:b]
            if gaps:
                xc = xc[~np.isnan(xc)]
                xm = xm[~np.isnan(xm)]
            if xc.size:
                np.percentile(xc, qv)
            if xm.size:
                xm.max()
            done += 1
        t_d = time.perf_counter()
        result["cpu_baseline_numpy"] = {
            "value": done / (t_d - t_c), "unit": "container-series/s", "cores": 1, "kind": "port",
            "sample": f"first {done} containers of this run, np.percentile(method='linear') + max per container, "
                      f"one thread, {args.numpy_seconds:.0f} s budget"}
        # the reference's own CPU path, measured in the build container only (cannot travel):
        result["reference_cpu_measured_in_build_container"] = {
            "value": 492.0, "unit": "container-series/s", "cores": 1, "measured_in_this_run": False,
            "kind": "carried_constant",
            "source": "carried constant from BASELINE.md (SimpleStrategy.run + _format_result, config 1, "
                      "measured once in the build container; the reference cannot travel to the GPU box)"}

    if rank == 0:
        phase("right-size")
        result.update(right_size(args, host_rec[:containers_total].numpy()))
    if rank == 0 and world == 1 and not args.no_host_path and not args.sharded_host_path:
        phase("host path")
        result.update(host_path(args, dev, c_host_sample=parts[0][2], objects=args.host_objects))
    if args.c4_containers > 0 and args.config == 2:
        phase("config-4 leg")
        del parts, out
        torch.cuda.empty_cache()
        leg = config4_leg(args, ctx, dev, world, rank, dist_on, backend, coll_dev,
                          comm if gather_mode == "stream" else None, params)
        if rank == 0:
            result.update(leg)
    if (world > 1 or args.sharded_host_path) and dist_on and not args.no_host_path:
        phase("host path (sharded)")
        hp = host_path_sharded(args, dev, world, rank, coll_dev, objects=args.host_objects)
        if rank == 0:
            result.update(hp)
    if world > 1:
        result["config"]["backend"] = backend
        if backend != "nccl":
            result["config"]["ranks_share_gpus"] = f"{world} ranks on {ndev} GPU(s) (gloo rehearsal)"
        if rank == 0:
            result.update(parity_gathered(args, ctx, dev, world, params, host_rec, gaps, pod_len, seed))
    if rank == 0:
        print(json.dumps(result), file=_JSON_OUT, flush=True)
    if dist_on:
        dist.barrier()
        if comm is not None and args.comm == "own":
            torch.cuda.synchronize()
            ctx.comm_destroy(comm)
        dist.destroy_process_group()
    ctx.close()


BODY_HEAD = '{"status":"success","data":{"resultType":"matrix","result":['


def body_fleet(o0: int, o1: int, pods: int = 3, distinct: int = 48):
    """Config-1-shaped query_range bodies of GLOBAL objects [o0, o1): `distinct` random pod
    series per resource (seeded: the same on every rank), pod i of object o taking pool entry
    (o * pods + i) % distinct (CPU) and (o * pods + 7 i) % distinct (memory).  Returns
    (cpu value strings, memory value strings, cpu bodies, memory bodies)."""
    rng = np.random.default_rng(0)
    ts = [repr(1.7e9 + 60.0 * i) for i in range(SLOTS_7D)]

    def values_part(xs):
        return ",".join(f'[{t},"{x!r}"]' for t, x in zip(ts, xs.tolist()))

    cpu_vals = [values_part(rng.gamma(2.0, 0.05, SLOTS_7D)) for _ in range(distinct)]
    mem_vals = [values_part(np.floor(rng.normal(2e8, 2e7, SLOTS_7D))) for _ in range(distinct)]
    cpu_pool = [(BODY_HEAD + '{"metric":{"pod":"p"},"values":[' + v + ']}]}}').encode() for v in cpu_vals]
    mem_pool = [(BODY_HEAD + '{"metric":{"pod":"p"},"values":[' + v + ']}]}}').encode() for v in mem_vals]
    cpu_b = [[cpu_pool[(o * pods + i) % distinct] for i in range(pods)] for o in range(o0, o1)]
    mem_b = [[mem_pool[(o * pods + i * 7) % distinct] for i in range(pods)] for o in range(o0, o1)]
    return cpu_vals, mem_vals, cpu_b, mem_b


def host_path(args, dev, c_host_sample, objects: int = 2000, pods: int = 3, distinct: int = 48) -> dict:
    """The host side of the path, measured after the timed region (never part of `value`):

    * h2d_GBps: page-locked chunks of this run's own CPU series copied to HBM (the PCIe leg a
      caller holding host buffers pays; krr_simple_run_host / SimpleEngine.run_packed);
    * pack_samples_per_s: the native query_range JSON -> CSR packer (include/krr_pack.h) on
      config-1-shaped bodies (objects x pods x 10,080 samples, both resources), the lease's
      threads — the reference's loader does this with json + Decimal(value)
      (robusta_krr/core/integrations/prometheus.py:150-155);
    * device_pack_samples_per_s: the device packer (krr_amd.core.device_pack: bodies staged,
      copied to HBM raw and parsed there, one wave per body) on the same bodies;
    * e2e_objects_per_s: BatchedRunner.recommend_from_bodies on the same bodies (device
      parse -> fused kernel -> exact-decimal rounding -> RunResults); e2e_objects_per_s_host_parse
      the same with the host packer;
    * e2e_grouped_objects_per_s(_host_parse): the same fleet as grouped `sum by (pod)` bodies
      (20 namespaces; krr_amd.core.fleet_query), BatchedRunner.recommend_from_grouped.
    Bodies are Prometheus-formatted (shortest-repr sample strings); `distinct` random pod
    series per resource are reused across the fleet (the packer's cost is per byte)."""
    import torch

    from krr_amd.core.prom_native import pack_query_range_bodies
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    out = {}
    # --- H2D of the run's own data, 1 GiB in 256 MiB pinned chunks
    n = min(c_host_sample.numel(), 1 << 27)
    host = torch.empty(n, dtype=torch.float64, pin_memory=True)
    host.copy_(c_host_sample[:n])
    dst = torch.empty(n, dtype=torch.float64, device=dev)
    chunk = 1 << 25
    torch.cuda.synchronize()
    reps = 4
    t0 = time.perf_counter()
    for _ in range(reps):
        for a in range(0, n, chunk):
            dst[a:a + chunk].copy_(host[a:a + chunk], non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    out["h2d_GBps"] = reps * n * 8 / (t1 - t0) / 1e9
    del host, dst
    # --- config-1-shaped query_range bodies
    L = SLOTS_7D
    t_g = time.perf_counter()
    cpu_vals, mem_vals, cpu_b, mem_b = body_fleet(0, objects, pods, distinct)
    head = BODY_HEAD
    t_g = time.perf_counter() - t_g
    json_bytes = sum(len(b) for bs in cpu_b for b in bs) + sum(len(b) for bs in mem_b for b in bs)
    threads = args.cpu_threads or cpu_lease()["threads"]
    samples = 2 * objects * pods * L
    pack_query_range_bodies(cpu_b[:4], threads=threads)  # warm-up (library load)
    best = float("inf")
    for _ in range(2):
        t0 = time.perf_counter()
        pack_query_range_bodies(cpu_b, threads=threads)
        pack_query_range_bodies(mem_b, threads=threads)
        best = min(best, time.perf_counter() - t0)
    out["pack_samples_per_s"] = samples / best
    runner = BatchedRunner(SimpleStrategy(SimpleStrategySettings(cpu_percentile=99, memory_buffer_percentage=5)))
    e2e = {}
    for parser in ("host", "device", "hybrid"):
        runner.recommend_from_bodies(cpu_b[:8], mem_b[:8], threads=threads, parser=parser)  # warm-up
        if parser == "hybrid":  # the host share settles on the rates both sides reach together
            for _ in range(5):
                runner.recommend_from_bodies(cpu_b, mem_b, threads=threads, parser=parser)
        runs_e = []
        for _ in range(3 if parser == "host" else 7):
            t0 = time.perf_counter()
            res = runner.recommend_from_bodies(cpu_b, mem_b, threads=threads, parser=parser)
            runs_e.append(time.perf_counter() - t0)
            if parser != "host":
                assert runner.last_pack_via == (parser, parser), runner.last_pack_via
        assert len(res) == objects
        e2e[parser] = (float(np.median(runs_e)), [(str(r[k].request), str(r[k].limit)) for r in res for k in r],
                       sorted(runs_e))
    # e2e_objects_per_s: the hybrid parser (host packer on a share of the bodies while the
    # link carries the rest); the device-only and host-only figures beside it
    out["e2e_objects_per_s"] = objects / e2e["hybrid"][0]
    out["e2e_objects_per_s_spread"] = [objects / e2e["hybrid"][2][-1], objects / e2e["hybrid"][2][0]]
    out["e2e_objects_per_s_device_parse"] = objects / e2e["device"][0]
    out["e2e_objects_per_s_host_parse"] = objects / e2e["host"][0]
    out["e2e_device_equals_host"] = e2e["device"][1] == e2e["host"][1]
    out["e2e_hybrid_equals_host"] = e2e["hybrid"][1] == e2e["host"][1]
    out["e2e_hybrid_split"] = runner.hybrid_last
    out["host_numa"] = _NUMA
    from krr_amd.core.device_pack import default_packer as _dp

    # the device side's last staging: JSON bytes vs bytes over PCIe (timestamps cut, krr_strip.h)
    out["e2e_device_upload"] = _dp(dev.index or 0).last_upload
    # the device packer alone: staging copy -> H2D -> parse -> CSR in HBM, both resources
    from krr_amd.core.device_pack import default_packer

    packer = default_packer(dev.index or 0)
    best_d = float("inf")
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        packer.pack(cpu_b)
        packer.pack(mem_b)
        torch.cuda.synchronize()
        best_d = min(best_d, time.perf_counter() - t0)
    out["device_pack_samples_per_s"] = samples / best_d
    # the reference's own loader (json + Decimal(value) per sample, prometheus.py:150-155),
    # measured in the build container only (it cannot travel): SURVEY.md §8(a) A1
    out["reference_loader_samples_per_s_build_container"] = 4.57e6
    # --- the same fleet through fleet-batched queries: one `sum by (pod)` body per
    # (namespace, container) group (krr_amd.core.fleet_query), 20 namespaces
    from krr_amd.core.fleet_query import FleetQueryPlan

    class _Obj:
        def __init__(self, o):
            self.namespace, self.container = f"ns{o % 20}", "main"
            self.pods = [f"pod-{o}-{i}" for i in range(pods)]

    fleet_objs = [_Obj(o) for o in range(objects)]
    plan = FleetQueryPlan.for_settings(fleet_objs, runner.strategy.settings)

    def grouped(vals, shift):
        out_b = []
        for gq in plan.groups:
            parts = [f'{{"metric":{{"pod":"{pod}"}},"values":[{vals[(i + shift) % distinct]}]}}'
                     for i, pod in enumerate(reversed(gq.pods))]
            out_b.append((head + ",".join(parts) + ']}}').encode())
        return out_b

    g_cpu, g_mem = grouped(cpu_vals, 0), grouped(mem_vals, 7)
    eg = {}
    g_state = {}
    for parser in ("host", "device", "hybrid"):
        runner.recommend_from_grouped(plan, g_cpu, g_mem, threads=threads, parser=parser)  # warm-up
        if parser == "hybrid":  # the host share settles on the rates both sides reach together
            for _ in range(4):
                runner.recommend_from_grouped(plan, g_cpu, g_mem, threads=threads, parser=parser)
        runs_g = []
        cg0 = cgroup_cpu()
        gc_t = _gc_timer()
        for _ in range(3 if parser == "host" else 7):
            t0 = time.perf_counter()
            res_g = runner.recommend_from_grouped(plan, g_cpu, g_mem, threads=threads, parser=parser)
            runs_g.append(time.perf_counter() - t0)
        assert len(res_g) == objects
        eg[parser] = (float(np.median(runs_g)), [(str(r[k].request), str(r[k].limit)) for r in res_g for k in r],
                      sorted(runs_g))
        cg1 = cgroup_cpu()
        g_state.setdefault("cgroup", {})[parser] = {k: cg1[k] - cg0.get(k, 0) for k in cg1 if isinstance(cg1[k], int)}
        g_state["cgroup"][parser]["gc"] = gc_t.stop()
        g_state["cgroup"]["quota"] = cg1.get("cpu.max") or cg1.get("cpu.cfs_quota_us")
        if parser != "host":  # the last run's staging and phases
            g_state[parser] = {"upload": dict(_dp(dev.index or 0).last_upload or {},
                                              stage_nodes=getattr(_dp(dev.index or 0), "stage_nodes", None),
                                              stage_mapping=getattr(_dp(dev.index or 0), "stage_mapping", None)),
                               "phases": dict(getattr(runner, "grouped_last", {}),
                                              **getattr(_dp(dev.index or 0), "last_grouped_phases", {}))}
    assert runner.last_pack_via == ("device", "device"), runner.last_pack_via
    # e2e_grouped_objects_per_s: the device parser (a grouped body is ~100 MB: the host packer
    # cannot split one across its threads, so the hybrid's host share only slows the staging
    # threads it borrows — measured beside it); the host-only figure too
    out["e2e_grouped_objects_per_s"] = objects / eg["device"][0]
    out["e2e_grouped_objects_per_s_spread"] = [objects / eg["device"][2][-1], objects / eg["device"][2][0]]
    out["e2e_grouped_objects_per_s_hybrid"] = objects / eg["hybrid"][0]
    out["e2e_grouped_hybrid_equals_host"] = eg["hybrid"][1] == eg["host"][1]
    out["e2e_grouped_hybrid_split"] = getattr(_dp(dev.index or 0), "last_grouped_hybrid", None)
    out["e2e_grouped_objects_per_s_host_parse"] = objects / eg["host"][0]
    out["e2e_grouped_upload"] = g_state["device"]["upload"]
    out["e2e_grouped_phases_s"] = g_state["device"]["phases"]
    out["e2e_grouped_hybrid_phases_s"] = g_state["hybrid"]["phases"]
    out["e2e_grouped_cgroup_cpu"] = g_state["cgroup"]
    from krr_amd.utils.numa import page_nodes

    from krr_amd.utils.numa import mapping_info

    b_addr = ctypes.cast(ctypes.c_char_p(g_cpu[0]), ctypes.c_void_p).value
    out["e2e_grouped_body_nodes"] = page_nodes(b_addr, len(g_cpu[0]), 16)
    out["e2e_grouped_body_mapping"] = mapping_info(b_addr, len(g_cpu[0]))
    out["e2e_grouped_device_equals_host"] = eg["device"][1] == eg["host"][1]
    out["host_path"] = {
        "h2d": f"{n * 8 >> 20} MiB of this run's CPU series, page-locked, {chunk * 8 >> 20}-MiB copies, {reps} reps",
        "bodies": f"{objects} objects x {pods} pods x {L} samples x 2 resources = {samples} samples, "
                  f"{json_bytes / 1e9:.2f} GB of query_range JSON ({distinct} distinct pod series per resource, "
                  f"generated in {t_g:.1f} s)",
        "pack_s": best, "device_pack_s": best_d, "e2e_s": e2e["hybrid"][0], "e2e_device_parse_s": e2e["device"][0],
        "e2e_runs_s": {p: [round(t, 5) for t in e2e[p][2]] for p in e2e},
        "e2e_grouped_runs_s": {p: [round(t, 5) for t in eg[p][2]] for p in eg},
        "e2e_host_parse_s": e2e["host"][0],
        "grouped": f"{len(plan.groups)} grouped bodies per resource ({sum(len(b) for b in g_cpu) / 1e9:.2f} GB of "
                   f"CPU JSON), e2e {eg['device'][0]:.3f} s device parse, {eg['host'][0]:.3f} s host parse",
        "threads": threads,
        "pack_GBps_json": json_bytes / best / 1e9, "device_pack_GBps_json": json_bytes / best_d / 1e9,
        "definition": "pack = krr_pack_parse/copy of every body on the host (CPU + memory); device_pack = "
                      "krr_amd.core.device_pack: staging copy into page-locked memory -> H2D -> krr_json_parse "
                      "(one wave per body) -> CSR in HBM; e2e = BatchedRunner.recommend_from_bodies with "
                      "parser='hybrid' (the last share of the bodies parsed by the host packer while the rest "
                      "crosses PCIe raw and is parsed on the device; e2e_device_parse: parser='device'; "
                      "e2e_host_parse: parser='host'): pack -> fused kernel -> native exact-decimal rounding -> "
                      "RunResults (the median of 7 runs, 3 for the host parser, each run's seconds in e2e_runs_s and "
                      "the slowest / fastest rate in *_spread; every object's strings compared across the parsers); "
                      "e2e_grouped: recommend_from_grouped with parser='device' (the same median rule, bodies "
                      "staged with their timestamps cut as the per-pod ones, e2e_grouped_upload; chunks parsed "
                      "(values arrays in 16-KiB parts, one wave each) and routed as they land, "
                      "e2e_grouped_phases_s), parser='hybrid' and parser='host' beside "
                      "it, every object compared"}
    return out


def config4_leg(args, ctx, dev, world, rank, dist_on, backend, coll_dev, comm, params) -> dict:
    """The config-4 strong-scaling leg, after the timed config-2 loop (which keeps `value`, so
    N = 1 and the driver's SCALE lines stay comparable): a FIXED fleet of --c4-containers x
    10,080 samples (7d@1m, compact CSR, both resources; 1 M containers = 161 GB) cut over the N
    ranks by sample-balanced contiguous ranges, each rank's shard resident in buffers of about
    --chunk-gib, one fused launch per chunk and step.  A step ends with every container's
    32-B record on rank 0's host: N = 1, written by the launch into page-locked memory; N > 1
    over RCCL, enqueued on the launch stream (krr_gather_results) into two alternating
    receive buffers, the previous step's forwarded to the host by the next launch (as in the
    main loop); gloo rehearsal, torch.distributed.gather after each step.  Reported:
    config4_containers_per_s (total containers / max-over-ranks step time), the aggregate HBM
    fraction, per-rank kernel and gather times, and the gathered records' parity with the
    oracle and rank 0's kernel on blocks sampled from EVERY shard."""
    import torch
    import torch.distributed as dist

    from krr_amd.core.distributed import gather_records, record_counts, shard_bounds

    total = args.c4_containers
    L = SLOTS_7D
    shards = shard_bounds(np.full(total, L, dtype=np.int64), world)
    g0, g1 = shards[rank]
    S = g1 - g0
    offs_np = np.arange(S + 1, dtype=np.int64) * L
    seed = 1000003 * 5  # config 4's fleet (main's seed for --config 4)
    stream = torch.cuda.current_stream()
    phase("c4 synth")
    parts = []
    for lo, hi in fleet_chunks(offs_np, args.chunk_gib):
        o = torch.from_numpy(offs_np[lo:hi + 1] - offs_np[lo]).to(dev)
        n = (hi - lo) * L
        c = torch.empty(n, dtype=torch.float64, device=dev)
        m = torch.empty(n, dtype=torch.float64, device=dev)
        ctx.synth_fill(c, o, seed, 0, 0, False, seg_base=g0 + lo)
        ctx.synth_fill(m, o, seed ^ 0x5A5A, 1, 0, False, seg_base=g0 + lo)
        parts.append((lo, hi, o, c, m, ctx.series(c, o, L, False), ctx.series(m, o, L, False)))
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    host_rec = torch.empty((total if rank == 0 else 1, 4), dtype=torch.int64, pin_memory=True)
    torch.cuda.synchronize()
    counts = [b - a for a, b in shards]
    stream_gather = dist_on and backend == "nccl" and comm is not None
    recv = [torch.empty((total, 4), dtype=torch.int64, device=dev) for _ in range(2)] \
        if stream_gather and rank == 0 else []
    dev_rec = torch.empty((S, 4), dtype=torch.int64, device=dev)
    nstep = [0]
    last = [None]

    def step(ev=None):
        k = nstep[0]
        nstep[0] += 1
        rec, fwd = dev_rec, None
        if not dist_on:
            rec = host_rec
        elif stream_gather and rank == 0:
            rec = recv[k % 2][:S]
            fwd = (recv[(k - 1) % 2], host_rec) if k > 0 else None
        if ev is not None:
            ev[0].record(stream)
        for j, (lo, hi, _, _, _, cs, ms) in enumerate(parts):
            ctx.simple_run(cs, ms, params, {key: v[lo:hi] for key, v in out.items()}, stream,
                           records=rec[lo:hi], forward=fwd if j == 0 else None)
        if ev is not None:
            ev[1].record(stream)
        if not dist_on:
            return
        if stream_gather:
            if rank == 0:
                ctx.gather_results(comm, 0, rec, counts=counts, out=recv[k % 2], stream=stream)
                last[0] = recv[k % 2]
            else:
                ctx.gather_results(comm, 0, rec, stream=stream)
        else:  # gloo rehearsal: host tensors, one blocking gather
            got = gather_records(rec.to(coll_dev), dst=0, counts=counts)
            if rank == 0:
                host_rec.copy_(got)
        if ev is not None:
            ev[2].record(stream)

    def finish():
        if last[0] is not None:
            host_rec.copy_(last[0], non_blocking=True)
            last[0] = None

    phase("c4 warmup")
    for _ in range(max(args.c4_warmup, 0)):
        step()
    finish()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    K = max(args.c4_steps, 1)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    phase(f"c4 timed {K} steps")
    t0 = time.perf_counter()
    for k in range(K):
        step(evs[k])
    finish()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    t1 = time.perf_counter()
    dt = torch.tensor([(t1 - t0) / K], dtype=torch.float64, device=coll_dev)
    k_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    g_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs])) if dist_on else 0.0
    mine = torch.tensor([k_ms, g_ms], dtype=torch.float64, device=coll_dev)
    if dist_on:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[float(x) for x in t.cpu().tolist()] for t in allr]
    else:
        per_rank = [[k_ms, g_ms]]
    step_s = float(dt.item())
    del parts, out, recv, dev_rec
    torch.cuda.empty_cache()
    res = None
    if rank == 0:
        # algorithmic bytes of one fused launch per resource, summed over ranks
        nbytes = sum(2 * (8 * (b - a) * L + 8 * (b - a + 1) + 20 * (b - a)) for a, b in shards)
        kmax = max(r[0] for r in per_rank)
        res = {
            "config4_containers_per_s": total / step_s,
            "config4_ms_per_step": step_s * 1e3,
            "config4_hbm_frac_aggregate": nbytes / step_s / (HBM_PEAK * world),
            "config4_kernel_hbm_frac_aggregate": nbytes / (kmax * 1e-3) / (HBM_PEAK * world),
            "config4_per_rank_kernel_ms": [r[0] for r in per_rank],
            "config4_kernel_ms_max": kmax,
            "config4_per_rank_gather_ms": [r[1] for r in per_rank] if dist_on else None,
            "config4_gather_ms_max": max(r[1] for r in per_rank) if dist_on else None,
            "config4_definition": (
                f"strong scaling: {total} containers x {L} samples x 2 resources (7d@1m, compact CSR, "
                f"{2 * 8 * total * L / 1e9:.0f} GB) cut over {world} rank(s), shards resident in "
                f"~{args.chunk_gib:g}-GiB buffers, one fused launch per chunk; a step ends with every record on "
                f"rank 0's host ({'page-locked memory written by the launch' if not dist_on else 'RCCL gather on the launch stream' if stream_gather else 'torch.distributed.gather'}); "
                f"{K} timed steps after {args.c4_warmup} warmup, max over ranks"),
        }
    # the gathered records against the oracle and rank 0's kernel, blocks from every shard
    if rank == 0:
        res.update({("config4_" + k): v for k, v in parity_gathered(
            args, ctx, dev, world, params, host_rec, False, 0, seed, cfg=4, shards=shards).items()})
        if not args.no_right_size:
            phase("c4 right-size")
            res.update(config4_right_size(args, host_rec.numpy(), shards))
    return res


def host_path_sharded(args, dev, world, rank, coll_dev, objects: int = 2000, pods: int = 3) -> Optional[dict]:
    """N > 1: the host path per rank (BatchedRunner.recommend_bodies_shard): every rank holds
    the query_range bodies of ITS `objects` consecutive objects of a fleet of objects x N
    (weak scaling; body_fleet, global object indices), packs them on its own GPU — each
    rank's PCIe link carries its shard's JSON, the hybrid parser splitting it with the rank's
    host cores — runs one kernel pass and sends its 32-B records to rank 0, which rounds
    every object.  e2e_objects_per_s = the fleet's objects / the max over ranks of the
    collective call's wall time (best of 3 after warm-up).  Rank 0 checks the first and last
    32 objects of every shard against the host packer + kernel on the same bodies."""
    import torch
    import torch.distributed as dist

    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    lease = cpu_lease()
    # ranks of one node share its cores unless OMP_NUM_THREADS names a per-rank lease
    threads = args.cpu_threads or (lease["threads"] if lease["omp_num_threads"] else
                                   max(1, lease["affinity_cpus"] // world))
    lo, hi = rank * objects, (rank + 1) * objects
    _, _, cpu_b, mem_b = body_fleet(lo, hi, pods)
    settings = SimpleStrategySettings(cpu_percentile=99, memory_buffer_percentage=5, device=dev.index or 0)
    runner = BatchedRunner(SimpleStrategy(settings))
    parser = args.host_parser
    per = []
    res = None
    for it in range(5):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        res = runner.recommend_bodies_shard(cpu_b, mem_b, device=dev.index or 0, parser=parser, threads=threads)
        torch.cuda.synchronize(dev)
        per.append(time.perf_counter() - t0)
    mine = torch.tensor([min(per[2:])], dtype=torch.float64, device=coll_dev)
    allr = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    per_rank = [float(t.item()) for t in allr]
    if rank != 0:
        return None
    total = objects * world
    assert res is not None and len(res) == total
    ok = True
    checked = 0
    for r in range(world):
        for a in (r * objects, (r + 1) * objects - 32):
            _, _, cb, mb = body_fleet(a, a + 32, pods)
            want = runner.recommend_from_bodies(cb, mb, threads=threads, parser="host")
            got = res[a:a + 32]
            ok &= [(str(x[k].request), str(x[k].limit)) for x in got for k in x] == \
                  [(str(x[k].request), str(x[k].limit)) for x in want for k in x]
            checked += 32
    return {"e2e_objects_per_s": total / max(per_rank),
            "e2e_per_rank_s": per_rank,
            "e2e_parser": parser,
            "e2e_sharded_equals_host_parse": bool(ok),
            "e2e_parity_objects": checked,
            "e2e_definition": (f"BatchedRunner.recommend_bodies_shard, parser={parser!r}: {objects} objects x {pods} "
                               f"pods x {SLOTS_7D} samples x 2 resources of query_range JSON per rank, packed on the "
                               f"rank's GPU with {threads} host threads, one kernel pass, records gathered to rank 0 "
                               f"and rounded there; {total} objects / max over ranks of the call (best of 3)")}


def make_comm(args, ctx, dev, world: int, rank: int):
    """The RCCL communicator of the C-ABI gather and where it came from, or (None, reason).

    --comm own (default): the library's own — rank 0 makes the id (krr_comm_unique_id), every
    rank receives it over torch.distributed (broadcast_object_list, a public API) and joins with
    krr_comm_init_timeout, which gives up after 60 s instead of hanging when a peer never
    arrives; every rank then agrees (one all_reduce) that all of them hold one, else none is used.
    --comm torch: torch.distributed's own communicator (pg_comm, a private accessor)."""
    import torch
    import torch.distributed as dist

    if args.comm == "torch":
        c = pg_comm(dev)
        return (c, "torch.distributed ProcessGroupNCCL._comm_ptr()") if c is not None else (None, "not exposed")
    uid = [None]
    err = None
    if rank == 0:
        try:
            uid[0] = ctx.comm_unique_id()
        except _native.NativeError as e:
            err = str(e)
    dist.broadcast_object_list(uid, src=0)
    comm = None
    if uid[0] is not None:
        try:
            comm = ctx.comm_init(world, uid[0], rank, timeout_s=60.0)
        except _native.NativeError as e:
            err = str(e)
    ok = torch.tensor([1 if comm else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        if comm:
            ctx.comm_destroy(comm)
        print(f"bench.py rank {rank}: own RCCL communicator unavailable ({err}); torch.distributed.gather",
              file=sys.stderr)
        return None, f"own communicator failed: {err}"
    return comm, "krr_comm_unique_id + krr_comm_init_timeout (the id broadcast over torch.distributed)"


def pg_comm(dev):
    """The ncclComm_t of torch.distributed's default "nccl" group on `dev` (as an int), or
    None when this torch build does not expose it."""
    import torch.distributed as dist

    try:
        fn = getattr(dist.group.WORLD._get_backend(dev), "_comm_ptr", None)
        return int(fn()) if fn is not None else None
    except (RuntimeError, AttributeError):
        return None


def right_size(args, records) -> dict:
    """After the timed region, on rank 0: the run's records (every rank's, gathered) -> the
    reference's Runner output, one ResourceAllocations per container (runner.py:113-120, after
    Runner._format_result's exact rounding, runner.py:49-86): native rounding +
    bulk-built models (krr_amd.core.fast_round.allocations_batch).  Checked against the
    per-object path (SimpleStrategy result -> Decimal rounding -> the pydantic-validated
    model) on a sample."""
    from krr_amd.core.distributed import raw_from_records
    from krr_amd.core.engine import RawResults
    from krr_amd.core.fast_round import allocations_batch
    from krr_amd.core.rounding import format_result
    from krr_amd.core.runner import to_allocations
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    settings = SimpleStrategySettings(cpu_percentile=str(args.percentile), memory_buffer_percentage="5")
    raw = raw_from_records(records)
    n = int(raw.cpu_value.size)
    threads = args.cpu_threads or cpu_lease()["threads"]
    k = min(500, n)
    sub = RawResults(*(np.asarray(a)[:k] for a in (raw.cpu_value, raw.cpu_count, raw.cpu_flags, raw.mem_value,
                                                   raw.mem_count, raw.mem_flags)))
    allocations_batch(sub, settings, threads=threads)  # loads the host libraries
    times = []
    for _ in range(3):
        t_a = time.perf_counter()
        got = allocations_batch(raw, settings, threads=threads)
        times.append(time.perf_counter() - t_a)
    dt = sorted(times)[1]
    want = [to_allocations(format_result(r)) for r in SimpleStrategy(settings).results_from_raw(sub)]
    same = all(g == w and g.json() == w.json() for g, w in zip(got[:k], want))
    return {"round_objects_per_s": n / dt,
            "round_ms": dt * 1e3,
            "round_objects": n,
            "round_equal_per_object_path": bool(same and len(got) == n),
            "round_definition": (f"all {n} containers' 32-B records -> native exact-decimal rounding (krr_round_simple, "
                                 f"{threads} threads) -> one ResourceAllocations per container built in bulk; median "
                                 f"of 3; checked equal (values, exponents, JSON) to the per-object reference path on "
                                 f"the first {k}")}


def kll_nchunks_np(beg: np.ndarray, end: np.ndarray) -> np.ndarray:
    """krr_kll.h kll_nchunks per segment: the 1,024-slot chunks the KLL passes stream."""
    a0 = np.minimum((beg + 1) & ~1, end)
    a1 = np.maximum(end & ~1, a0)
    units = (a1 - a0) >> 1
    full = units // 512
    return full + (((units - full * 512) > 0) | (a0 > beg) | (a1 < end)).astype(np.int64)


def fleet_objects(n: int) -> list:
    """n synthetic K8sObjectData (untimed set-up of the right-size leg): distinct objects whose
    current allocations cycle through a pool that puts the recommendations in every severity
    bucket (None, "?"-free values below, near and far above the usual recommendation)."""
    from decimal import Decimal

    from krr_amd.core.models.allocations import ResourceAllocations, ResourceType
    from krr_amd.core.models.objects import K8sObjectData

    cpu_rt, mem_rt = ResourceType.CPU, ResourceType.Memory
    # the synthetic fleet's recommendations sit near 0.35 cores and 3.0e8 B: currents from far
    # below to far above them, plus unset ones
    cpus = [None] + [Decimal(x) for x in ("0.1", "0.25", "0.35", "0.4", "0.5", "1", "2")]
    mems = [None] + [Decimal(x) for x in ("100000000", "250000000", "300000000", "350000000", "536870912",
                                          "1073741824")]
    pool = []
    for i in range(64):
        c, m = cpus[i % len(cpus)], mems[(i * 5) % len(mems)]
        pool.append(ResourceAllocations.construct(requests={cpu_rt: c, mem_rt: m},
                                                  limits={cpu_rt: None if i % 2 else cpus[(i * 3) % len(cpus)],
                                                          mem_rt: mems[(i * 7) % len(mems)]}))
    new = K8sObjectData.construct
    return [new(cluster=None, name=f"app-{i}", container="main", pods=[f"app-{i}-0"], namespace=f"ns-{i % 97}",
                kind="Deployment", allocations=pool[i % 64]) for i in range(n)]


def config4_right_size(args, records: np.ndarray, shards) -> dict:
    """After the config-4 leg, on rank 0: ALL containers' gathered 32-B records -> the
    reference's Runner output and Result (runner.py:49-131): native exact-decimal rounding,
    one ResourceAllocations per container, then Runner._collect_result's ResourceScan per
    container and the Result score (result.py:33-150), all in bulk
    (fast_round.allocations_batch, models.result.collect_result).  Timed whole and by phase.
    Checked on 64-object blocks at both ends of EVERY shard against the per-object path
    (SimpleStrategy result -> Decimal rounding -> validated ResourceAllocations ->
    ResourceScan.calculate)."""
    import gc

    from krr_amd.core.distributed import raw_from_records
    from krr_amd.core.engine import RawResults
    from krr_amd.core.fast_round import result_batch
    from krr_amd.core.models.result import ResourceScan
    from krr_amd.core.rounding import format_result
    from krr_amd.core.runner import to_allocations
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    n = int(records.shape[0])
    settings = SimpleStrategySettings(cpu_percentile=str(args.percentile), memory_buffer_percentage="5")
    threads = args.cpu_threads or cpu_lease()["threads"]
    t_obj = time.perf_counter()
    objects = fleet_objects(n)
    t_obj = time.perf_counter() - t_obj
    warm = RawResults(*(np.asarray(a)[:1000] for a in raw_from_records(records[:1000]).__dict__.values()
                        if isinstance(a, np.ndarray)))
    result_batch(objects[:1000], warm, settings, threads=threads)  # loads the libraries
    gc.collect()
    tm: dict = {}
    t0 = time.perf_counter()
    raw = raw_from_records(records)
    t1 = time.perf_counter()
    # rounding -> value columns -> ResourceScan per container + score, one native pass (the
    # ResourceAllocations the reference builds in between are read by its scan only)
    result = result_batch(objects, raw, settings, threads=threads, timings=tm)
    t3 = time.perf_counter()
    t2 = t3 - tm.get("scan_s", 0.0)
    total = t3 - t0
    # equality with the per-object path: 64-object blocks at both ends of every shard plus a
    # stride over the whole fleet (every pool entry of fleet_objects, so every severity bucket)
    idx = set(range(0, n, max(1, n // 4096)))
    for a, b in shards:
        for lo in sorted({a, max(a, b - 64)}):
            idx.update(range(lo, min(lo + 64, b)))
    idx = np.array(sorted(idx), dtype=np.int64)
    sub = RawResults(*(np.asarray(x)[idx] for x in (raw.cpu_value, raw.cpu_count, raw.cpu_flags,
                                                    raw.mem_value, raw.mem_count, raw.mem_flags)))
    want = [to_allocations(format_result(r)) for r in SimpleStrategy(settings).results_from_raw(sub)]
    same, checked, pair_sev = True, 0, {}
    for i, w in zip(idx.tolist(), want):
        ref_scan = ResourceScan.calculate(objects[i], w)
        same &= (result.scans[i] == ref_scan and result.scans[i].severity == ref_scan.severity
                 and result.scans[i].json() == ref_scan.json())
        for sel in (ref_scan.recommended.requests, ref_scan.recommended.limits):
            for r in sel.values():
                pair_sev[r.severity.value] = pair_sev.get(r.severity.value, 0) + 1
        checked += 1
    sev = {}
    for s in result.scans[:: max(1, n // 20000)]:
        sev[s.severity.value] = sev.get(s.severity.value, 0) + 1
    del result, objects
    gc.collect()
    return {
        "config4_right_size_s": total,
        "config4_right_size_objects_per_s": n / total,
        "config4_right_size_split_s": {"unpack": t1 - t0, "round": tm.get("round_s"), "decimal": tm.get("decimal_s"),
                                       "scan_and_score": t3 - t2},
        "config4_scan_objects_per_s": n / (t3 - t2),
        "config4_right_size_equal_per_object_path": bool(same),
        "config4_right_size_checked_objects": checked,
        "config4_right_size_severities_sampled": sev,
        "config4_right_size_checked_pair_severities": pair_sev,
        "config4_right_size_definition": (
            f"rank 0, all {n} containers' gathered records -> krr_round_simple ({threads} threads) -> the rounded "
            f"value columns -> Runner._collect_result's ResourceScan per container + Result score, in one native "
            f"pass (fast_round.result_batch; the ResourceAllocations the reference builds between them are only "
            f"read by its scan, so they are not materialised); one run after a warm-up on 1000; the {n} "
            f"K8sObjectData are built beforehand "
            f"({t_obj:.1f} s, untimed); checked equal to the per-object path on {checked} containers (64-object "
            f"blocks at both ends of every shard and a stride over the fleet; per (resource, selector) "
            f"severities of the checked ones in _checked_pair_severities)")}


def parity_gathered(args, ctx, dev, world, params, host_rec, gaps, pod_len, seed, cfg=None, shards=None) -> dict:
    """N > 1: check the records gathered to rank 0 against a sample regenerated from
    EVERY shard (blocks of consecutive global containers at the start, inside and at
    the end of each rank's range): the C oracle on the host, and this GPU's own
    kernel on the same containers (a shard computed elsewhere must equal it bit for bit).
    `cfg` / `shards` (default: the run's --config and fleet_shard) name another fleet
    (the config-4 leg)."""
    import torch

    from krr_amd.core.distributed import unpack_records
    from oracle import oracle

    threads = args.cpu_threads or cpu_lease()["threads"]
    gathered = unpack_records(host_rec.numpy())
    ok_oracle = ok_local = True
    checked = 0
    cfg = args.config if cfg is None else cfg
    if shards is None:
        shards = [fleet_shard(cfg, r, world, args.containers)[:2] for r in range(world)]
    for g0, g1 in shards:
        n = g1 - g0
        b = max(1, min(args.parity_block, n))
        starts = sorted({g0 + ((n - b) * j) // max(args.parity_blocks - 1, 1) for j in range(args.parity_blocks)})
        for a in starts:
            L = container_lengths(cfg, a, a + b, args.pods)
            offs_np = np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
            offs = torch.from_numpy(offs_np).to(dev)
            N = int(offs_np[-1])
            cpu = torch.empty(N, dtype=torch.float64, device=dev)
            mem = torch.empty(N, dtype=torch.float64, device=dev)
            ctx.synth_fill(cpu, offs, seed, 0, pod_len, gaps, seg_base=a)
            ctx.synth_fill(mem, offs, seed ^ 0x5A5A, 1, pod_len, gaps, seg_base=a)
            out = {k: torch.empty(b, dtype=dt, device=dev) for k, dt in
                   (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
                    ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
            maxlen = int(L.max())
            ctx.simple_run(ctx.series(cpu, offs, maxlen, gaps), ctx.series(mem, offs, maxlen, gaps), params, out)
            c_host, m_host = cpu.cpu().numpy(), mem.cpu().numpy()
            ov, on, _ = oracle.percentile(c_host, offs_np, params.mode, params.p_num, params.p_den, params.q, gaps,
                                          threads)
            mv, mn, _ = oracle.seg_max(m_host, offs_np, gaps, threads)
            gv = gathered["cpu_value"][a:a + b]
            same = (gv.view(np.uint64) == ov.view(np.uint64)) | (np.isnan(gv) & np.isnan(ov))
            if args.mode == "linear":  # the sign of a zero LINEAR result is unspecified
                same |= (gv == 0) & (ov == 0)
            ok_oracle &= bool(same.all() and np.array_equal(gathered["cpu_count"][a:a + b], on)
                              and np.array_equal(gathered["mem_value"][a:a + b], mv, equal_nan=True)
                              and np.array_equal(gathered["mem_count"][a:a + b], mn))
            lv = out["cpu_value"].cpu().numpy()
            ok_local &= bool(np.array_equal(gv.view(np.uint64), lv.view(np.uint64))
                             and np.array_equal(gathered["mem_value"][a:a + b].view(np.uint64),
                                                out["mem_value"].cpu().numpy().view(np.uint64))
                             and np.array_equal(gathered["cpu_count"][a:a + b], out["cpu_count"].cpu().numpy())
                             and np.array_equal(gathered["mem_count"][a:a + b], out["mem_count"].cpu().numpy())
                             and np.array_equal(gathered["cpu_flags"][a:a + b],
                                                out["cpu_flags"].cpu().numpy().view(np.uint32)))
            checked += b
            del cpu, mem, offs, out
    return {"parity_vs_oracle_on_sample": ok_oracle, "parity_gathered_vs_rank0_kernel": ok_local,
            "parity_sample_containers": checked,
            "parity_definition": (f"records gathered to rank 0 vs oracle/krr_oracle.c and vs rank 0's own kernel on "
                                  f"{args.parity_blocks} blocks of {args.parity_block} consecutive containers per "
                                  f"shard, regenerated on rank 0 from their global indices")}


SLOTS_30D_15S = 30 * 24 * 60 * 4  # 172,800


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            return next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        return platform.processor()


def run_config5(args, world, rank, local, dev, coll_dev):
    """Config 5: time-sharded 30d@15s series (see krr_amd/core/sketch.py).

    N = 1 (default): every series whole on the GPU: ONE exact select pass per chunk of
    series, consecutive chunks' launches alternating between two streams so one's drain
    overlaps the next one's start.
    Time-sharded (N > 1, or --c5-refine at N = 1), exact, --c5-method window (default):
    ONE HBM pass per rank (window export) -> one all-to-all of the windows to each series'
    owner (RCCL) -> merge (exact counts decide; misses regathered and selected whole) ->
    results gathered to rank 0.  --c5-method sketch: sketch build -> reduce-scatter ->
    locate -> collect (a second HBM pass) -> all-to-all -> refine.  --sketch-only stops at
    the interpolated sketch answer (value error <= 2^-m; rank error measured, not bounded).
    """
    import torch
    import torch.distributed as dist

    from krr_amd import _native
    from krr_amd.core import sketch
    from krr_amd.core.distributed import gather_records, record_counts
    from krr_amd.core.engine import percentile_params

    S = args.containers or 100_000
    T = SLOTS_30D_15S
    t0, t1 = (T * rank) // world, (T * (rank + 1)) // world
    Lr = t1 - t0
    ctx = _native.Context(local)
    seed = 1000003 * 6
    cfg = sketch.SketchConfig(mantissa_bits=args.sketch_bits)
    params = percentile_params(Decimal(args.percentile), params_mode(args))
    exact = not args.sketch_only
    direct = exact and world == 1 and not args.c5_refine
    method = "direct" if direct else (args.c5_method if exact else ("kll" if args.sketch_kind == "kll" else
                                                                     "sketch-only"))
    # auto: the tail that answers --percentile exactly, or none when no row can hold it (p50)
    ktail = args.kll_tail if args.kll_tail >= 0 else sketch.KllConfig.tail_for(T, args.percentile)
    kcfg = sketch.KllConfig(budget=args.kll_budget, tail=ktail)
    # the direct pass and the window export run per chunk of series in buffers of their own
    # (as configs 2-4, fleet_chunks); the sketch paths keep one buffer per rank
    chunked = direct or method == "window"
    chunks = fleet_chunks(np.arange(S + 1, dtype=np.int64) * Lr, args.c5_chunk_gib) if chunked else [(0, S)]
    phase("synth")
    parts = []
    for lo, hi in chunks:
        o = torch.arange(hi - lo + 1, dtype=torch.int64, device=dev) * Lr
        c = torch.empty((hi - lo) * Lr, dtype=torch.float64, device=dev)
        ctx.synth_fill_window(c, o, seed, 0, 0, False, t0, T, seg_base=lo)
        parts.append((lo, hi, c, ctx.series(c, o, Lr, False)))
    torch.cuda.synchronize()
    ser = parts[0][3]  # the whole rank when it is one chunk (the sketch paths)
    ser_parts = [(lo, hi, ser_c) for lo, hi, _, ser_c in parts]

    def first_rows(k):
        """[k, Lr] device view/copy of the first k series."""
        rows = [c.view(hi - lo, Lr)[: max(0, min(k, hi) - lo)] for lo, hi, c, _ in parts if lo < k]
        return rows[0] if len(rows) == 1 else torch.cat(rows)
    stream = torch.cuda.current_stream()
    # direct, several chunks: consecutive launches alternate between two streams (each
    # launch of ~5,900 whole series is ~3 wave lifetimes long: its drain is a large share)
    side = torch.cuda.Stream(device=dev) if direct and len(parts) > 1 else None
    dres = None
    if direct:
        dres = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
                (("value", torch.float64), ("count", torch.int64), ("flags", torch.int32))}
    if world > 1:  # owner blocks are fixed: exchange the record counts once
        blk = sketch.owner_blocks(S, world)[rank]
        counts = record_counts(blk[1] - blk[0], coll_dev)
    else:
        counts = None
    host_rec = torch.empty((S, 4), dtype=torch.int64, pin_memory=True)
    state = {"misses": 0, "steps": 0}

    def step(ev=None):
        if method == "direct":
            if ev is not None:
                ev[0].record(stream)
            if side is not None:
                fork = torch.cuda.Event()
                fork.record(stream)
                side.wait_event(fork)
            for j, (lo, hi, _, ser_c) in enumerate(parts):
                st = side if (side is not None and j % 2) else stream
                ctx.segmented_percentile(ser_c, params, dres["value"][lo:hi], dres["count"][lo:hi],
                                         dres["flags"][lo:hi], st)
            if side is not None:
                join = torch.cuda.Event()
                join.record(side)
                stream.wait_event(join)
            if ev is not None:
                ev[1].record(stream)
            rec = torch.stack([dres["value"].view(torch.int64),
                               dres["count"] | (dres["flags"].to(torch.int64) << 48),
                               torch.zeros_like(dres["count"]), torch.zeros_like(dres["count"])], dim=1)
            host_rec[: rec.shape[0]].copy_(rec, non_blocking=True)
            return
        if method == "kll":
            # events: before the body pass, between it and the tail pass, after the tail pass
            kst: dict = {}
            res = sketch.kll_time_sharded(ctx, ser_parts, kcfg, params, stream=stream,
                                          events=None if ev is None else (ev[0], ev[3], ev[1]), stats=kst)
            state["rows"], state["rows_per_series"] = res["rows"], res["rows_per_series"]
            state["kll_stats"] = kst
        elif method == "window":
            res = sketch.window_exact_time_sharded(ctx, ser_parts, params, ext_slots=T - Lr, stream=stream,
                                                   events=None if ev is None else ev[0:2])
            state["misses"] += res["misses"]
            state["key_cap"] = res["key_cap"]
            state["exchanged_bytes"] = res["exchanged_bytes"]
            state["hdr"] = res["hdr"]
        else:
            if ev is not None:
                ev[0].record(stream)
            sk = sketch.build(ctx, ser, cfg, stream)
            if ev is not None:
                ev[1].record(stream)
            merged = sketch.merge_time_sharded(sk)
            if exact:
                res = sketch.exact_time_sharded(ctx, ser, sk, merged, cfg, params, stream=stream,
                                                events=None if ev is None else ev[3:5])
                state["collected"] = res["collected"]
            else:
                res = sketch.query(ctx, merged, cfg, params, stream)
        if ev is not None:
            ev[2].record(stream)
        rec = torch.stack([res["value"].view(torch.int64), res["count"] | (res["flags"].to(torch.int64) << 48),
                           torch.zeros_like(res["count"]), torch.zeros_like(res["count"])], dim=1)
        if world > 1:
            rec = gather_records(rec.to(coll_dev), dst=0, counts=counts)
        if rank == 0:
            host_rec[: rec.shape[0]].copy_(rec, non_blocking=True)
        state["steps"] += 1

    phase("warmup")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    state["misses"] = state["steps"] = 0
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(args.steps)]
    phase(f"timed {args.steps} steps")
    t_a = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_b = time.perf_counter()
    phase("report")
    dt = torch.tensor([(t_b - t_a) / args.steps], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    step_s = float(dt.item())
    kms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    N = S * Lr
    kernels_ms = {}
    kll_sparse = None
    if method == "direct":
        kname = "k_select"
        kbytes = 8 * N + 8 * (S + 1) + 20 * S
    elif method == "kll":
        kname = "k_kll_build"
        # every slot once + offsets + the exported rows
        kbytes = 8 * N + 8 * (S + 1) + 8 * kcfg.row_words * S
        kernels_ms["exchange_merge_query_ms"] = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
        if kcfg.tail > 0 and not kcfg.one_pass_tail:  # the body pass alone; the tail pass beside it
            kms = float(np.mean([e[0].elapsed_time(e[3]) for e in evs]))
            tms = float(np.mean([e[3].elapsed_time(e[1]) for e in evs]))
            kernels_ms["k_kll_tail"] = tms
            kst = state.get("kll_stats") or {}
            if "lines_read" in kst:
                # sparse tail pass (krr_kll_tail_lines): the body also writes 4 B of line maximum per
                # 128-B line; the tail pass reads those maxima, the lines that can hold a tail key,
                # offsets, each row's header and body, and writes its tail
                seg = np.arange(S + 1, dtype=np.int64) * Lr
                nch = kll_nchunks_np(seg[:-1], seg[1:])
                nlines = int(nch.sum()) * 64
                kbytes += 4 * 64 * int(((nch + 7) & ~7).sum())  # the build streams a multiple of 8 chunks
                read = int(kst["lines_read"].sum().item())
                tbytes = 4 * nlines + 128 * read + 8 * (S + 1) + 8 * (16 + kcfg.budget) * S + 8 * kcfg.tail * S
                kll_sparse = {
                    "lines_read_frac": read / max(nlines, 1), "lines_read": read, "lines_total": nlines,
                    "definition": "fraction of the slice's 128-B lines the tail pass read (the rest cannot hold "
                                  "a key above its threshold: their maxima, recorded by the body pass, are below it)"}
            else:
                # every slot once + offsets + each row's header and body read + its tail written
                tbytes = 8 * N + 8 * (S + 1) + 8 * (16 + kcfg.budget) * S + 8 * kcfg.tail * S
    elif method == "window":
        kname = "k_window_export"
        hdr = state["hdr"]
        cw = hdr[:, 4] & 0xFFFFFFFF
        fl = hdr[:, 4] >> 32
        stored = (fl & (_native.KRR_WIN_FAIL | _native.KRR_WIN_POINT)) == 0
        keys_out = int(torch.where(stored, cw, torch.zeros_like(cw)).sum().item())
        # every slot once + offsets + a 40-B header and the exported keys per series
        kbytes = 8 * N + 8 * (S + 1) + 40 * S + 8 * keys_out
        kernels_ms["merge_exchange_ms"] = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    else:
        kname = "k_sketch_build"
        kbytes = 8 * N + 8 * (S + 1) + S * (4 * cfg.width + 8 + 8 + 4)
    kernels_ms = {kname: kms, **kernels_ms}
    if method == "sketch":
        # collect: every slot read once + locations in, collected samples out
        cms = float(np.mean([e[3].elapsed_time(e[4]) for e in evs]))
        kernels_ms["k_sketch_collect"] = cms
        cbytes = 8 * N + 8 * (S + 1) + 56 * S + 8 * S + 8 * int(state.get("collected", 0))
    kind = {"direct": (f"config5: {S} CPU series x {T} samples (30d@15s) on one GPU: exact single-window select, "
                       f"one pass (no time sharding at N=1; {len(parts)} launches alternating on 2 streams)"),
            "window": (f"config5: {S} CPU series x {T} samples (30d@15s), time-sharded over {world} ranks ({Lr} "
                       f"samples/series/rank): exact, one HBM pass (window export in {len(parts)} launches "
                       f"alternating on 2 streams -> all-to-all -> merge)"),
            "sketch": (f"config5: {S} CPU series x {T} samples (30d@15s), time-sharded over {world} ranks ({Lr} "
                       f"samples/series/rank), log-linear sketch 2^{cfg.mantissa_bits} bins/octave + exact "
                       f"refinement (collect + select in the located bins; two HBM passes)"),
            "sketch-only": (f"config5: {S} CPU series x {T} samples (30d@15s), time-sharded over {world} ranks "
                            f"({Lr} samples/series/rank), log-linear sketch 2^{cfg.mantissa_bits} bins/octave, "
                            f"approximate"),
            "kll": (f"config5: {S} CPU series x {T} samples (30d@15s), time-sharded over {world} ranks ({Lr} "
                    f"samples/series/rank), KLL sketch (row format 2: {kcfg.budget} body keys + {kcfg.tail} exact "
                    f"tail keys per row, one build launch per rank, rows folded per series)")}[method]
    par = {"direct": "single GPU, whole series",
           "window": f"time-shard{world} (all-to-all of per-slice windows to the series' owners, RCCL)",
           "sketch": f"time-shard{world} (reduce-scatter of {cfg.width}-word sketches, RCCL)",
           "sketch-only": f"time-shard{world} (reduce-scatter of {cfg.width}-word sketches, RCCL)",
           "kll": f"time-shard{world} (all-to-all of {kcfg.row_words}-word rows to the series' owners, RCCL)"}[method]
    result = {
        "metric": METRIC,
        "value": S / step_s,
        "unit": "cpu-series/s (30d@15s, exact)" if exact else "cpu-series/s (30d@15s, sketch mode)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device counter-hash: CPU ~ Gamma(2, 0.05) cores), generated per time slice",
        "config": {"workload": kind, "percentile_mode": params_mode(args), "cpu_percentile": args.percentile,
                   "series": S, "slots_per_rank": N, "parallelism": par, "method": method},
        "samples_per_s": S * T / step_s,
        "launches_per_step": len(parts),
        "kernels_ms": kernels_ms,
        "roofline": {"kernel": kname, "bound": "hbm", "achieved": kbytes / (kms * 1e-3) / 1e9,
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": kbytes / (kms * 1e-3) / HBM_PEAK,
                     "traffic": None, "algorithmic_bytes_per_launch": kbytes},
    }
    if method == "window":
        result["window"] = {"key_cap": state["key_cap"], "keys_exported_per_series": keys_out / max(S, 1),
                            "alltoall_bytes_sent_per_rank": state["exchanged_bytes"],
                            "misses_per_step": state["misses"] / max(args.steps, 1),
                            "hbm_passes_per_step": 1}
    if kll_sparse:
        result["kll_sparse_tail"] = kll_sparse
    if method == "kll":
        # what one slice of one series puts on the all-to-all (a rank sends (N-1)/N of its
        # rows), beside the exact window path's row for the same slicing (krr_window_key_cap)
        l8 = -(-T // 8)
        result["exchange_bytes_per_series_slice"] = {
            "kll_row": 8 * kcfg.row_words,
            "window_row": 8 * (_native.HDR_WORDS + _native.window_key_cap(max(Lr, 1), T - Lr, params)),
            "window_row_at_n8": 8 * (_native.HDR_WORDS + _native.window_key_cap(l8, T - l8, params)),
            "n": world}
    if "k_kll_tail" in kernels_ms:
        # the KLL build in two passes: the body (k_kll_build, above) and the exact tail
        # (k_kll_tail, candidates above a threshold read from the row's body); both HBM streams
        tms = kernels_ms["k_kll_tail"]
        result["roofline_tail"] = {"kernel": "k_kll_tail", "bound": "hbm", "achieved": tbytes / (tms * 1e-3) / 1e9,
                                   "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": tbytes / (tms * 1e-3) / HBM_PEAK,
                                   "algorithmic_bytes_per_launch": tbytes}
        result["kll_build_both_passes"] = {
            "ms": kms + tms, "series_per_s": S / ((kms + tms) * 1e-3),
            "frac_of_one_pass": kbytes / ((kms + tms) * 1e-3) / HBM_PEAK,
            "definition": "body + tail passes together, against the bytes of ONE pass over the slice"}
    if method == "sketch":
        result["roofline_collect"] = {"kernel": "k_sketch_collect", "bound": "hbm",
                                      "achieved": cbytes / (cms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                                      "frac": cbytes / (cms * 1e-3) / HBM_PEAK, "algorithmic_bytes_per_launch": cbytes}
    if world > 1:
        mine = torch.tensor([kms], dtype=torch.float64, device=coll_dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        result["per_rank_kernel_ms"] = [float(t.item()) for t in allr]
        result["kernel_ms_max"] = max(result["per_rank_kernel_ms"])
    try:
        with open(args.traffic) as fh:
            tr = json.load(fh)
        key = f"config5:{params_mode(args)}:p{args.percentile}:{kname}"
        if (key in tr and int(tr[key].get("containers_per_rank", -1)) == S
                and int(tr[key].get("slots_per_rank", N)) == N):  # the same slice size per rank
            result["roofline"]["traffic"] = tr[key]["hbm_bytes_per_launch"]
            result["roofline"]["traffic_source"] = tr[key].get("source")
        tkey = f"config5:{params_mode(args)}:p{args.percentile}:k_kll_tail"
        if ("roofline_tail" in result and tkey in tr and int(tr[tkey].get("containers_per_rank", -1)) == S
                and int(tr[tkey].get("slots_per_rank", N)) == N):
            result["roofline_tail"]["traffic"] = tr[tkey]["hbm_bytes_per_launch"]
            result["roofline_tail"]["traffic_source"] = tr[tkey].get("source")
    except (OSError, ValueError):
        pass
    # parity / rank error on a sample of series, regathered whole on rank 0
    phase("parity")
    m = max(1, min(args.error_sample, S))
    piece = first_rows(m).contiguous()
    if world > 1:
        width = (T + world - 1) // world
        pad = torch.full((m, width), float("nan"), dtype=torch.float64, device=dev)
        pad[:, :Lr] = piece
        bufs = [torch.empty_like(pad, device=coll_dev) for _ in range(world)] if rank == 0 else None
        dist.gather(pad.to(coll_dev), gather_list=bufs, dst=0)
        if rank == 0:
            full = torch.cat([b[:, : ((T * (r + 1)) // world - (T * r) // world)].to(dev)
                              for r, b in enumerate(bufs)], dim=1).contiguous()
    else:
        full = piece
    if rank == 0:
        from oracle import oracle

        rec = host_rec[:m].numpy()
        got = rec[:, 0].copy().view(np.float64)
        got_n = rec[:, 1] & ((1 << 48) - 1)  # config-5 records: value bits, count | flags << 48, 0, 0
        fo = torch.arange(m + 1, dtype=torch.int64, device=dev) * T
        fser = ctx.series(full.view(-1), fo, T, False)
        ev_ = torch.empty(m, dtype=torch.float64, device=dev)
        en_ = torch.empty(m, dtype=torch.int64, device=dev)
        ef_ = torch.empty(m, dtype=torch.int32, device=dev)
        exact_params = percentile_params(Decimal(args.percentile), params_mode(args))
        ctx.segmented_percentile(fser, exact_params, ev_, en_, ef_)
        lt = torch.empty(m, dtype=torch.int64, device=dev)
        le = torch.empty(m, dtype=torch.int64, device=dev)
        ctx.rank_of(fser, torch.from_numpy(got).to(dev), lt, le)
        torch.cuda.synchronize()
        n = en_.cpu().numpy().astype(np.float64)
        target = (n - 1) * float(args.percentile) / 100.0
        ltn, len_ = lt.cpu().numpy(), le.cpu().numpy()
        err = np.maximum(0.0, np.maximum(ltn - target, target - (len_ - 1))) / n
        exact_v = ev_.cpu().numpy()
        threads = args.cpu_threads or cpu_lease()["threads"]

        def same_bits(a, b):
            ok = (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))
            if params_mode(args) == "linear":  # zero sign of a LINEAR result is unspecified
                ok |= (a == b)
            return ok

        if exact:
            bad = ~same_bits(got, exact_v) | (got_n != en_.cpu().numpy())
            result["parity_vs_single_window_select"] = bool(not bad.any())
            if bad.any():
                i = int(np.nonzero(bad)[0][0])
                result["parity_mismatch"] = {"series": int(bad.sum()), "first": i, "got": float(got[i]),
                                             "want": float(exact_v[i]), "got_n": int(got_n[i]),
                                             "want_n": int(en_[i].item()), "got_flags": int(rec[i, 1] >> 48)}
            result["parity_sample_series"] = m
            if world > 1:  # the oracle on the regathered series, beside k_select
                full_h = full.cpu().numpy().ravel()
                ov, on, _ = oracle.percentile(full_h, (np.arange(m + 1) * T).astype(np.int64), exact_params.mode,
                                              exact_params.p_num, exact_params.p_den, exact_params.q, False, threads)
                result["parity_vs_oracle_on_sample"] = bool(same_bits(got, ov).all() and np.array_equal(got_n, on))
                result["parity_oracle_sample_series"] = m
            result["parity_definition"] = ("answers gathered on rank 0 (bits, counts) == k_select over the full "
                                           "172,800-sample series regathered from every rank"
                                           + (" and == oracle/krr_oracle.c on the same series" if world > 1 else "")
                                           + ", first sample series")
            if method == "sketch":
                result["collected_samples_per_rank"] = int(state.get("collected", 0))
        elif method == "kll":
            rel = np.abs(got - exact_v) / np.abs(exact_v)
            # the bound comes from the folded rows, which rank 0 holds for its owner block only
            mb = min(m, state["rows"].shape[0])
            rows_b = state["rows"][:mb]
            body_bound = sketch.kll_rank_bound(rows_b, 1, delta=0.01)
            # ranks of this percentile inside each row's exact tail have no error at all
            rr = np.floor(target[:mb]).astype(np.int64)
            in_tail = sketch.kll_tail_covers(rows_b, rr)
            bound = np.where(in_tail, 0.0, body_bound)
            # a LINEAR answer interpolates ranks floor(t) and floor(t) + 1: its rank interval
            # can sit up to one rank from t even when exact, so tail-covered answers are held
            # to the exact answer's bits and body answers to the bound plus that one rank
            n_b = np.maximum(n[:mb], 1.0)
            ok_b = np.where(in_tail, same_bits(got[:mb], exact_v[:mb]), err[:mb] <= body_bound + 1.0 / n_b + 1e-12)
            result["sketch_error"] = {
                "kind": "kll", "sample_series": m, "rank_error_max": float(err.max()),
                "rank_error_mean": float(err.mean()), "rank_error_bound_max": float(np.nanmax(bound)),
                "rank_error_bound_mean": float(np.nanmean(bound)), "bound_confidence": 0.99,
                "body_rank_error_bound_max": float(np.nanmax(body_bound)),
                "within_bound": bool(np.all(ok_b)), "bound_sample_series": mb,
                "tail_answers_equal_exact": bool(np.all(same_bits(got[:mb], exact_v[:mb])[in_tail])),
                "rank_in_exact_tail_fraction": float(np.mean(in_tail)),
                "value_rel_error_max": float(rel.max()), "value_rel_error_mean": float(rel.mean()),
                "budget_keys_per_row": kcfg.budget, "tail_keys_per_row": kcfg.tail,
                "row_bytes": 8 * kcfg.row_words,
                "guarantee": ("ranks r with n - r <= tail: exact (the row keeps the tail largest samples); other "
                              "ranks: |rank(answer) - r| / n <= sqrt(2 ln(4/delta) sum w^2) / n with probability "
                              ">= 1 - delta, sum w^2 fixed by the compaction schedule (presence pattern only; "
                              "krr_amd.core.sketch.kll_rank_bound)"),
                "definition": "rank error = distance of (n-1)p/100 from the sketch answer's rank interval "
                              "[#<v, #<=v - 1] over n; exact path = k_select/hselect on the gathered full series; "
                              "within_bound: answers whose rank the exact tail covers equal the exact answer bit for "
                              "bit, the others' rank error <= the body bound + 1/n (LINEAR interpolates two ranks)"}
        else:
            rel = np.abs(got - exact_v) / np.abs(exact_v)
            result["sketch_error"] = {
                "sample_series": m, "rank_error_max": float(err.max()), "rank_error_mean": float(err.mean()),
                "value_rel_error_max": float(rel.max()), "value_rel_error_mean": float(rel.mean()),
                "value_rel_bound": 2.0 ** -cfg.mantissa_bits,
                "guarantee": (f"value: |v - exact| / exact <= 2^-{cfg.mantissa_bits} when the needed ranks fall in "
                              f"binned octaves (else KRR_FLAG_SKETCH_RANGE); rank: no data-independent bound (a "
                              f"low-dispersion series can put most samples in one bin) - exact refinement is the "
                              f"default at every N"),
                "definition": "rank error = distance of (n-1)p/100 from the sketch answer's rank interval "
                              "[#<v, #<=v - 1] over n; exact path = k_select/hselect on the gathered full series"}
        if not args.no_cpu_baseline and world == 1:
            cs = max(1, min(args.cpu_sample * 5 if args.cpu_sample else 4096, S))  # ~10 s on 16 cores
            host = first_rows(cs).cpu().numpy().ravel()
            ho = (np.arange(cs + 1) * Lr).astype(np.int64)
            ta = time.perf_counter()
            ov, on, _ = oracle.percentile(host, ho, exact_params.mode, exact_params.p_num, exact_params.p_den,
                                          exact_params.q, False, threads)
            tb = time.perf_counter()
            result["cpu_baseline"] = {
                "value": cs / (tb - ta), "unit": "cpu-series/s (exact)", "cores": threads, "kind": "port",
                "sample": f"first {cs} series ({cs * Lr} samples) copied D2H; oracle/krr_oracle.c exact "
                          f"{args.mode}, OpenMP {threads} threads on {_cpu_model()}"}
            if exact:  # this run's answers on the same series against the oracle
                recs = host_rec[:cs].numpy()
                gv = recs[:, 0].copy().view(np.float64)
                result["parity_vs_oracle_on_sample"] = bool(same_bits(gv, ov).all()
                                                            and np.array_equal(recs[:, 1] & ((1 << 48) - 1), on))
                result["parity_oracle_sample_series"] = cs
        print(json.dumps(result), file=_JSON_OUT, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


def params_mode(args) -> str:
    return args.mode if args.mode != "ref_index" else "linear"


if __name__ == "__main__":
    main()
