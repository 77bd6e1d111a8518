"""bench.py -- env steps/s of the MI355X-native BlueSky-Gym step path.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; N>1 is launched with
torch.distributed.run, one rank per GPU.  Rank 0 prints ONE JSON line.

Workload (BASELINE.json metric): MergeEnv-v0, 32 aircraft per env, 4096 envs in total
split over the N GPUs (strong scaling, SURVEY C4: 4096/N envs per rank; `--weak` keeps
4096 envs per GPU instead), ACTION_FREQUENCY=10 substeps of DT=5 s,
StateBased all-pairs CPA on every step, Gymnasium NEXT_STEP autoreset inside the timed
region.  Spawns are drawn on the device (Philox); actions come from a bank of U(-1,1)
batches resident in HBM before timing starts.  With N>1 every step also all-gathers the
[E, obs+3] fp32 learner rows over RCCL (the north-star's learner hand-off, one per RL
step); the block-gather variant (one all_gather per 8 steps) is timed afterwards and
reported in the `gather_block` object.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "bluesky-gym-hallucination_amd")]

METRIC = "env steps/sec (whole node), MergeEnv-v0 4096 envs × 32 aircraft, 1/2/4/8 GPUs"
TIMING_EVERY = 10              # post-region cross-check: event pair around every 10th launch
MIN_SAMPLES = 10               #   ... until at least this many launches are sampled
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)


def survey_bytes_per_env_step(N, A=2, O=40, K=5):
    """SURVEY.md §8(d) algorithmic bytes per Merge env-step:
    2*N*10*8 (6 kinematic + 4 autopilot fp64 fields, read+write) + 4A + 4O + 6
    + ceil(N^2/8) (conflict bitmask) + ceil(N/8) (LoS bitmask) + 4K (top-K int32)."""
    return 2 * N * 10 * 8 + 4 * A + 4 * O + 6 + -(-N * N // 8) + -(-N // 8) + 4 * K


def layout_bytes_per_env_step(N, A=2, O=40, K=5, cd=True):
    """Bytes this build's layout actually moves per env-step:
    12 fp64 + 1 int32 per aircraft read+write, 56 B of env scalars read+write, fp64
    actions, fp32 obs, reward/term/trunc, int32 top-K, u64 intrusion mask, and with CD
    u64 conflict + LoS rows, fp32 tcpamax per aircraft and fp32 min separation."""
    b = 2 * N * (12 * 8 + 4) + 2 * 56 + 8 * A + 4 * O + 6 + 4 * K + 8
    if cd:
        b += N * (8 + 8 + 4) + 4
    return b


def _cpu_worker(args):
    """One host core: the batched NumPy oracle on E Merge envs x 32 aircraft (128: the
    batched form; 1: one env per process, the reference's SubprocVecEnv layout), CD on,
    NEXT_STEP autoreset, stepped for `seconds`.  Returns (env-steps, elapsed s)."""
    seconds, seed, E = args
    import numpy as np
    from oracle import batched as ob
    o = ob.MergeOracle(E, num_ac=32, seed=seed, compute_cd=True)
    o.reset()
    rng = np.random.default_rng(seed)
    o.step(rng.uniform(-1, 1, (E, 2)))
    n = 0
    t0 = time.perf_counter()
    while True:
        o.step(rng.uniform(-1, 1, (E, 2)))
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 3:
            return E * n, el


def cpu_baseline(seconds: float):
    """Time the CPU oracle on the host cores of this box on a bounded sample of the same
    workload: one process per core (the reference's SubprocVecEnv layout,
    scripts/multi_processing_example.py:51-53), each stepping the batched NumPy
    restatement (oracle/batched.py, the fastest CPU form of the path) on 128 Merge envs x
    32 aircraft with CD on for `seconds`.  Runs before anything touches the GPU (the
    workers are forked).  value = sum of the per-core rates."""
    import multiprocessing as mp
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    # the GPU box's CPU share is 16 per GPU (os.cpu_count() there is the whole machine)
    P = max(1, min(int(os.environ.get("BENCH_CPU_WORKERS", "16")), avail))
    for v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[v] = "1"
    with mp.get_context("fork").Pool(P) as pool:
        res = pool.map(_cpu_worker, [(seconds, 11 + w, 128) for w in range(P)])
        res1 = pool.map(_cpu_worker, [(seconds / 3, 11 + w, 1) for w in range(P)])
    value = sum(n / el for n, el in res)
    per = [n / el for n, el in res]
    per1 = [n / el for n, el in res1]
    model = platform.processor() or "unknown"
    cores = set()
    try:
        with open("/proc/cpuinfo") as f:
            phys = core = None
            for line in f:
                if line.startswith("model name") and model in ("unknown", platform.processor()):
                    model = line.split(":", 1)[1].strip()
                elif line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                elif not line.strip():
                    if core is not None:
                        cores.add((phys, core))
                    phys = core = None
            if core is not None:
                cores.add((phys, core))
    except OSError:
        pass
    node_cores = len(cores) or (os.cpu_count() or P)
    return {"value": value, "unit": "env_steps/s", "cores": P, "kind": "port",
            "sample": f"oracle/batched.py MergeOracle, {P} processes x 128 envs x 32 aircraft, "
                      f"CD on, {seconds:.0f} s each ({min(per):.0f}-{max(per):.0f} env-steps/s "
                      f"per core), NumPy fp64 one thread per process on '{model}' "
                      f"({avail} CPUs available to this process, {os.cpu_count()} on the host)",
            # the whole node's CPUs, beside the per-GPU share.  Not run on
            # them (a GPU box's CPU share is 16 per GPU): the measured mean per-core rate times
            # the host's physical cores -- an extrapolation, labelled as one
            "node": {"value": value / P * node_cores, "unit": "env_steps/s", "cores": node_cores,
                     "kind": "port", "measured": False,
                     "sample": f"extrapolated: the {P} processes' mean {value / P:.0f} env-steps/s "
                               f"per core x {node_cores} physical cores of '{model}' "
                               f"({os.cpu_count()} logical CPUs); the 16-core share above is "
                               f"the measured figure"},
            # one env per process, as the reference runs (SubprocVecEnv): the same oracle at E=1
            "per_env": {"value": sum(per1), "unit": "env_steps/s", "cores": P,
                        "sample": f"MergeOracle with 1 env x 32 aircraft per process, {P} processes, "
                                  f"{seconds / 3:.0f} s each ({min(per1):.0f}-{max(per1):.0f} "
                                  f"env-steps/s per core)"}}


def load_profile(E):
    """Per-launch HBM bytes and VALU counts from the committed rocprofv3 PMC passes
    (tools/profile.sh -> profiles/traffic.json); None when absent or for another size."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
        if int(t.get("envs", -1)) == E:
            return t
    except (OSError, ValueError, KeyError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--total-envs", type=int, default=4096,
                    help="strong scaling (default, SURVEY C4): envs over all GPUs")
    ap.add_argument("--weak", action="store_true", help="weak scaling: --envs-per-gpu on every GPU")
    ap.add_argument("--envs-per-gpu", type=int, default=4096)
    ap.add_argument("--num-ac", type=int, default=32)
    ap.add_argument("--steps-per-gather", type=int, default=1,
                    help="N>1: learner rows all-gathered once per block of this many steps "
                         "(one RCCL all_gather of [k, E, obs+3] fp32; the last partial block is "
                         "flushed inside the timed region); 1 (default, SURVEY §8(e), BASELINE C4) "
                         "= one all_gather per RL step")
    ap.add_argument("--transport", default="rccl", choices=("rccl", "torch"),
                    help="N>1 over RCCL: the learner-row gather as libbsg's direct RCCL calls "
                         "(default) or torch.distributed.all_gather_into_tensor")
    ap.add_argument("--require-rccl", action="store_true",
                    help="N>1 over RCCL: exit non-zero (after printing the line) unless the "
                         "learner-row gather ran on libbsg's RCCL communicator of N ranks and "
                         "the cross-rank row check passed")
    ap.add_argument("--gather-block", type=int, default=8,
                    help="N>1: also time the block-gather variant (one all_gather per this many "
                         "steps) after the headline, reported in the `gather_block` object; 0 = skip")
    ap.add_argument("--no-cd", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--skip-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the short C5 (Descent + policy) leg")
    ap.add_argument("--no-c5-learner", action="store_true",
                    help="skip C5's learner-in-the-loop leg inside the default run")
    ap.add_argument("--workload", default="merge", choices=("merge", "descent-sac"),
                    help="merge: the BASELINE metric (default); descent-sac: BASELINE configs[4], "
                         "DescentEnv-v0 with the SAC learner in the loop")
    ap.add_argument("--no-graph", action="store_true", help="descent-sac: eager, no HIP graph")
    ap.add_argument("--learner-reduce", default="auto", choices=("auto", "rccl", "torch"),
                    help="descent-sac: the learner's gradient all-reduce -- rccl: libbsg's "
                         "communicator (bsg_comm_all_reduce on the update's stream, inside the "
                         "iteration's HIP graph; at one rank a one-rank communicator), torch: "
                         "torch.distributed (eager); auto = rccl over the nccl backend (and at "
                         "one rank), torch otherwise")
    ap.add_argument("--torch-policy", action="store_true",
                    help="descent-sac: sample actions with the torch actor instead of bsg_policy_sac")
    ap.add_argument("--blas", default="cublas", choices=("default", "cublas", "cublaslt"),
                    help="descent-sac: torch.backends.cuda.preferred_blas_library for the learner's "
                         "GEMMs (cublas = rocBLAS/hipBLAS on ROCm, cublaslt = hipBLASLt)")
    args = ap.parse_args()
    if args.workload == "descent-sac":
        return bench_descent_sac(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # the step kernel's ~1.1 KB of kernel arguments from device memory (AMD's launch-latency
    # setting for MI300-class parts): -0.3..0.4 us per step at the driver's 20-step region,
    # three runs each (profiles/r06/timed_region_ab.txt).  Read by HIP at initialisation.
    os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
    # CPU baseline first, on rank 0 at N=1 only, before anything initialises the GPU
    cpu = None if (world > 1 or args.skip_cpu_baseline) else cpu_baseline(args.cpu_seconds)

    import torch
    import torch.distributed as dist
    from bluesky_gym.parallel import ShardedVectorEnv
    from bluesky_gym.vector import MergeVectorEnv

    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (test only)
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(local % torch.cuda.device_count())
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    E = args.envs_per_gpu if args.weak else args.total_envs // world
    if not args.weak and E * world != args.total_envs:
        raise SystemExit(f"--total-envs {args.total_envs} does not split over {world} GPUs")
    gather = world > 1 and not args.no_gather
    make_local = lambda **kw: MergeVectorEnv(num_ac=args.num_ac, seed=1234,  # noqa: E731
                                             compute_cd=not args.no_cd, **kw)
    transport_note = None
    if gather:
        # RCCL (backend nccl): libbsg's direct RCCL gather (parallel.RcclGather); torch's
        # all_gather_into_tensor only if that cannot start (recorded in the JSON line)
        transport = args.transport if backend == "nccl" else "torch"
        try:
            env = ShardedVectorEnv(make_local, world * E, overlap=(backend == "nccl"),
                                   steps_per_gather=args.steps_per_gather, transport=transport)
        except Exception as ex:          # noqa: BLE001 - reported, not hidden
            # RcclGather's construction is collective: it raises on every rank or on none
            # (parallel.RcclGather), so every rank falls back together
            if transport != "rccl":
                raise
            transport_note = f"native RCCL gather failed to start ({ex}); torch.distributed used"
            env = ShardedVectorEnv(make_local, world * E, overlap=True,
                                   steps_per_gather=args.steps_per_gather, transport="torch")
        batch = env.local.batch
        env.reset()
    else:
        venv = make_local(num_envs=E, env_offset=rank * E)
        batch = venv.batch
        venv.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(17 + rank)
    bank = torch.rand((16, E, 2), dtype=torch.float64, device=dev, generator=gen) * 2 - 1
    acts = [bank[k] for k in range(16)]          # views made once, outside the timed region

    def one(k):
        if gather:
            env.step(acts[k % 16])
        else:
            batch.step(acts[k % 16])

    for k in range(args.warmup):
        one(k)
    if gather:
        env.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on the launch stream (torch's current stream: core.DeviceBatch launches
    # there) bracket the K back-to-back launches; nothing is inserted between launches
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for k in range(args.steps):
        one(k)
    if gather:
        _, ready = env.flush()                 # the last partial block's rows, inside the region
        if ready is not None:
            ready.wait()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern_avg_ms = ev0.elapsed_time(ev1) / args.steps
    step_avg_ms = kern_avg_ms
    if gather:
        # with the gather the bracket above also holds the RCCL Work.wait() stream waits;
        # the kernel's own time comes from the same launches without the collective
        for k in range(args.warmup):
            batch.step(acts[k % 16])
        torch.cuda.synchronize()
        ev0.record()
        for k in range(args.steps):
            batch.step(acts[k % 16])
        ev1.record()
        torch.cuda.synchronize()
        kern_avg_ms = ev0.elapsed_time(ev1) / args.steps
    # cross-check after the timed region: an event pair around every TIMING_EVERY-th launch
    # (each pair serialises the stream, so it is kept out of the timed region), >= 10 samples
    batch.step_timing()                       # discard
    batch.set_timing(TIMING_EVERY)
    for k in range(TIMING_EVERY * MIN_SAMPLES):
        one(k)
    torch.cuda.synchronize()
    batch.set_timing(False)
    samp_ms, samples = batch.step_timing()
    samp_ms = samp_ms / max(samples, 1)
    if world > 1:
        t = torch.tensor([el, kern_avg_ms, samp_ms, step_avg_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, kern_avg_ms, samp_ms, step_avg_ms = (float(x) for x in t)
    comm = check = None
    if gather:
        comm = comm_record(env, world, dev)
        check = row_check(env, acts, world, dev)
    blk = None
    if gather and args.gather_block > 1 and args.gather_block != args.steps_per_gather:
        blk = bench_gather_block(args, make_local, world, E, acts, backend, dev)
    c5 = None
    if world == 1 and not args.no_c5:
        c5 = bench_c5_quick(args, dev)

    if rank == 0:
        total = world * E * args.steps
        value = total / el
        N = args.num_ac
        B = survey_bytes_per_env_step(N)
        achieved = B * E / (kern_avg_ms * 1e-3) / 1e9
        prof = load_profile(E) if args.num_ac == 32 and not args.no_cd else None
        valu = None
        if prof and "valu_issue_cycles_per_simd" in prof:
            # VALU issue utilisation of the same kernel: PMC instruction counts priced at
            # 4 cycles per f64 and 2 per other wave64 VALU instruction, over 1024 SIMDs
            # at the 2.4 GHz peak clock, divided by this run's kernel time
            cyc = prof["valu_issue_cycles_per_simd"]
            valu = {"valu_insts_per_launch": prof["valu_insts_per_launch"],
                    "f64_insts_per_launch": prof["valu_f64_insts_per_launch"],
                    "issue_frac": cyc / (kern_avg_ms * 1e-3 * 2.4e9)}
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env_steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: device Philox spawns (merge_env.py distributions), U(-1,1) actions",
            "config": {
                "workload": f"MergeEnv-v0 {world * E} envs x {N} aircraft ({E} per GPU), 10 substeps x DT 5 s, "
                            f"StateBased CD {'off' if args.no_cd else 'on'}, NEXT_STEP autoreset"
                            + ((", RCCL" if backend == "nccl" else f", {backend}")
                               + (" all_gather of [E, obs+3] fp32 per step" if args.steps_per_gather == 1 else
                                  f" all_gather of [{args.steps_per_gather}, E, obs+3] fp32 per {args.steps_per_gather} steps")
                               if gather else ""),
                "envs_total": world * E,
                "envs_per_gpu": E,
                "num_ac": N,
                "parallelism": f"env-shard x{world}" + ((" + RCCL all_gather (overlapped)" if backend == "nccl"
                                                          else f" + {backend} all_gather") if gather else ""),
                "backend": backend if world > 1 else None,
                "steps_per_gather": args.steps_per_gather if gather else None,
                "gather_transport": (env.transport if gather else None),
                "gather_transport_note": transport_note,
                "rccl": comm,
                "row_check": check,
                # kernel arguments in device memory (HIP_FORCE_DEV_KERNARG, set in main unless
                # the caller set it): the ~1.1 KB KParams per launch is fetched from HBM
                "hip_force_dev_kernarg": os.environ.get("HIP_FORCE_DEV_KERNARG"),
            },
            "roofline": {
                # the binding limit is fp64 VALU dependency latency; `frac`
                # is the HBM fraction the roofline contract asks for, `valu` the VALU view
                "bound": "valu-latency",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": prof["hbm_bytes_per_launch"] if prof else None,
                "traffic_source": (f"profiles/traffic.json: rocprofv3 FETCH_SIZE/WRITE_SIZE passes of "
                                   f"this workload ({prof.get('source', '')}), not this run")
                                  if prof else None,
                "kernel": "bsg::step_kernel<MERGE,32>",
                # achieved / frac / kernel_avg_ms describe ONE GPU: a rank's shard of E envs
                "scope": f"per GPU (one rank's launch over its {E} envs)",
                "kernel_avg_ms": kern_avg_ms,
                "kernel_timing": (f"HIP events on the launch stream bracketing the {args.steps} "
                                  f"back-to-back launches of the timed region (GPU time per launch, "
                                  f"incl. the dispatch gap between launches)") if not gather else
                                 (f"HIP events bracketing {args.steps} back-to-back launches of a "
                                  f"second pass WITHOUT the gather (max over ranks); the timed "
                                  f"region's bracket incl. the gather's stream waits is "
                                  f"step_avg_ms"),
                "step_avg_ms": step_avg_ms,
                "sampled_launch_ms": samp_ms,
                "sampled_launch_timing": f"cross-check after the timed region: event pair around "
                                         f"every {TIMING_EVERY}th launch, {samples} samples "
                                         f"(each pair serialises the stream)",
                "bytes_per_env_step": B,
                "layout_bytes_per_env_step": layout_bytes_per_env_step(N, cd=not args.no_cd),
                "valu": valu,
            },
        }
        if cpu is not None:
            out["cpu_baseline"] = cpu
        if c5 is not None:
            out["c5"] = c5
        if blk is not None:
            out["gather_block"] = blk
        print(json.dumps(out), flush=True)
    failed = None
    if args.require_rccl and gather:
        if env.transport != "rccl" or comm is None or any(n != world for n in comm["nranks"]):
            failed = f"--require-rccl: the gather did not run on an RCCL communicator of {world} ranks"
        elif not check["ok"]:
            failed = "--require-rccl: the cross-rank row check failed"
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if failed:
        raise SystemExit(failed)


def comm_record(env, world, dev):
    """Per rank, what libbsg's communicator says it is (bsg_comm_get_info: ncclCommCount,
    ncclCommUserRank) -- so a node run's line shows that RCCL saw every rank -- gathered to
    every rank by the process group; None unless the transport is libbsg's RCCL."""
    import torch
    import torch.distributed as dist
    if env.transport != "rccl":
        return None
    inf = env._rccl.info()
    mine = torch.tensor([inf["nranks"], inf["rank"], inf["device"], inf["gathers"]],
                        dtype=torch.int64, device=dev)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    rows = [[int(x) for x in t.cpu()] for t in allv]
    return {"nranks": [r[0] for r in rows], "rank": [r[1] for r in rows],
            "device": [r[2] for r in rows], "gathers": [r[3] for r in rows],
            "source": "bsg_comm_get_info (ncclCommCount / ncclCommUserRank) on each rank"}


def row_check(env, acts, world, dev):
    """After the timed region, one more step: every rank compares the rows the transport
    gathered with every rank's own rows of that step, which the process group delivers once
    by its own all-gather (c10d, independent of libbsg's communicator) -- bit for bit, rank by
    rank.  Returns {"ok", "bad_rows" (summed over ranks), ...} for the line."""
    import torch
    import torch.distributed as dist
    from bluesky_gym.parallel import all_gather_rows
    env.flush()
    rows, ready = env.step(acts[0])
    if rows is None:                          # k > 1: close the block (one step long)
        blk, ready = env.flush()
        n = blk.shape[0]
        rows = blk[n - 1]                     # [world, n_local, row]
        local = env.local_rows(ready)[n - 1]
    else:
        local = env.local_rows(ready)
    ready.wait()
    torch.cuda.synchronize()
    ref = torch.empty((world * env.n_local, env.row_dim), dtype=torch.float32, device=dev)
    all_gather_rows(ref, local.contiguous())
    torch.cuda.synchronize()
    got = rows.reshape(world, env.n_local, env.row_dim).view(torch.int32)
    want = ref.reshape(world, env.n_local, env.row_dim).view(torch.int32)
    bad = (got != want).any(dim=2).sum(dim=1).to(torch.int64)         # per source rank
    dist.all_reduce(bad)
    bad = [int(x) for x in bad.cpu()]
    return {"ok": sum(bad) == 0, "bad_rows": sum(bad), "bad_rows_by_source_rank": bad,
            "checked": f"{world} ranks x {world * env.n_local} rows x {env.row_dim} fp32, bitwise",
            "reference": "each rank's local rows of that step via torch.distributed all_gather "
                         "(c10d), compared with the transport's gathered rows on every rank"}


def bench_gather_block(args, make_local, world, E, acts, backend, dev):
    """N > 1: the same workload with the learner rows gathered once per block of k steps
    (one all_gather of [k, E, obs+3] per k steps: fewer, larger collectives; the learner
    sees each step's rows up to k - 1 steps late).  Not the headline: BASELINE C4 and SURVEY
    §8(e) gather every step.  Same timing rules (barrier + synchronize on both sides, max
    over ranks), own env instance."""
    import torch
    import torch.distributed as dist
    from bluesky_gym.parallel import ShardedVectorEnv
    k = args.gather_block
    transport = args.transport if backend == "nccl" else "torch"
    try:
        env = ShardedVectorEnv(make_local, world * E, overlap=(backend == "nccl"), steps_per_gather=k,
                               transport=transport)
    except Exception:                    # noqa: BLE001 - the headline line records the failure
        env = ShardedVectorEnv(make_local, world * E, overlap=True, steps_per_gather=k)
    env.reset()
    for i in range(args.warmup):
        env.step(acts[i % 16])
    env.flush()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        env.step(acts[i % 16])
    _, ready = env.flush()
    if ready is not None:
        ready.wait()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t[0])
    env.close()
    return {"steps_per_gather": k, "transport": env.transport, "value": world * E * args.steps / el,
            "ms_per_step": el * 1e3 / args.steps, "unit": "env_steps/s",
            "note": f"one all_gather of [{k}, E, obs+3] fp32 per {k} steps (the learner sees a "
                    f"step's rows up to {k - 1} steps late); not the C4 contract"}


def bench_c5_quick(args, dev):
    """BASELINE configs[4] on this GPU, in a few seconds, after the headline timing
    (its own buffers; the headline value is unaffected): DescentEnv-v0 x 4096 envs, SAME_STEP
    autoreset + final_obs as SB3 consumes it, (a) env only (U(-1,1) actions from HBM) and
    (b) env + the policy's action sample -- the reference's saved Descent SAC actor,
    stochastic, as the fused HIP kernel bsg_policy_sac on the kernel's own fp32 obs rows,
    the iteration captured as one HIP graph.  The SAC update itself (learner-bound, tools/
    sac_torch.py) is `--workload descent-sac`; DESIGN.md §12."""
    import numpy as np
    import torch
    from bluesky_gym import _native as nat, config, core
    from bluesky_gym.policy import SACPolicy
    E = 4096
    steps, warm = max(args.steps, 20), max(args.warmup, 5)
    b = core.DeviceBatch(config.descent_config(), E, autoreset=nat.AUTORESET_SAME_STEP,
                         compute_cd=False, seed=1234)
    b.reset()
    gen = torch.Generator(device=dev)
    gen.manual_seed(29)
    bank = torch.rand((16, E, 1), dtype=torch.float64, device=dev, generator=gen) * 2 - 1

    def timed(fn):
        for k in range(warm):
            fn(k)
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for k in range(steps):
            fn(k)
        ev1.record()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps, ev0.elapsed_time(ev1) / steps

    wall_env, ev_env = timed(lambda k: b.step(bank[k % 16]))
    W = dict(np.load(os.path.join(REPO, "tests", "golden", "sac_actors.npz")))
    pol = SACPolicy({k: W[f"descent/{k}"] for k in ("latent_pi.0.weight", "latent_pi.0.bias",
                     "latent_pi.2.weight", "latent_pi.2.bias", "mu.weight", "mu.bias",
                     "log_std.weight", "log_std.bias")}, dev)
    act = torch.zeros((E, 1), dtype=torch.float64, device=dev)
    eps = torch.zeros((E, 1), dtype=torch.float32, device=dev)

    def it():
        eps.normal_()
        pol(b.obs, eps, out=act)
        b.step(act)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            it()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        it()
    wall_pol, ev_pol = timed(lambda k: g.replay())
    learner = None
    if not args.no_c5_learner:
        learner = c5_learner_leg(b, W, dev, steps, warm)
    return {"workload": "DescentEnv-v0 4096 envs, 30 substeps x DT 1 s, SAME_STEP autoreset + "
                        "final_obs (BASELINE configs[4], one GPU; the learner leg as "
                        "--workload descent-sac's graph)",
            "steps": steps,
            "env_policy_learner": learner,
            "env_only": {"value": E / wall_env, "ms_per_step": wall_env * 1e3,
                         "kernel_avg_ms": ev_env, "kernel": "bsg::step_kernel<DESCENT,1>"},
            "env_policy": {"value": E / wall_pol, "ms_per_step": wall_pol * 1e3,
                           "event_ms_per_step": ev_pol,
                           "policy": "reference's saved Descent SAC actor, stochastic, fused HIP "
                                     "kernel bsg_policy_sac, HIP graph of sample + step"},
            "unit": "env_steps/s"}


def c5_learner_leg(b, W, dev, steps, warm):
    """BASELINE configs[4] end to end on this GPU, inside the default run (the
    learner-in-the-loop figure was never driver-timed): every vector step = the SAC actor's
    sample (fused kernel) -> bsg_step -> replay insert -> one SAC update (SB3 2.x SAC,
    scripts/descent_env_sac.py:25-34: batch 256, lr 1e-3, gradient_steps 1; tools/sac_torch.py),
    the iteration captured as one HIP graph; the learner's GEMMs on rocBLAS."""
    import torch
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import sac_torch
    torch.backends.cuda.preferred_blas_library("cublas")
    os.environ["DISABLE_ADDMM_CUDA_LT"] = "1"
    # FusedSAC: the update's forward / backward written out (tools/sac_fused.hip, 19 launches
    # per update instead of ~100); SAC_FUSED=0 = the autograd update
    cls = sac_torch.FusedSAC if os.environ.get("SAC_FUSED", "1") == "1" else sac_torch.SAC
    sac = cls(b.obs_dim, b.act_dim, dev, group=None, seed=0, lr=1e-3)
    sac.actor.load_sb3(W, "descent")
    rl = sac_torch.RLLoop(b, sac, learn=True, fused_policy=True)
    rl.obs.copy_(b.obs)
    for _ in range(8):                                # fill the buffer past one batch
        rl.step()
    # C5_GRAPH_ITERS RL iterations per graph replay (the timed region still runs `steps`
    # iterations: steps // iters replays)
    iters = max(1, int(os.environ.get("C5_GRAPH_ITERS", "1")))
    steps = max(iters, steps - steps % iters)
    rl.capture(iters=iters)
    for _ in range(max(1, warm // iters)):
        rl.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // iters):
        rl.replay()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    lq, la = sac.update()
    return {"value": b.E / wall, "ms_per_step": wall * 1e3, "unit": "env_steps/s",
            "critic_loss": float(lq), "actor_loss": float(la),
            "learner": "SB3 SAC restated (tools/sac_torch.py): twin critics + actor 256-256, "
                       "batch 256, one update per vector step, HIP graph",
            "update": type(sac).__name__, "products": getattr(sac, "gemm", "torch"),
            "noise": getattr(sac, "noise", "torch"), "iters_per_graph": iters, "timed_iterations": steps}


def bench_descent_sac(args):
    """BASELINE configs[4]: DescentEnv-v0 x 4096 envs (4096/N per rank) with the learner in
    the loop (scripts/descent_env_sac.py:25-34: SB3 SAC, MultiInputPolicy, lr 1e-3, batch
    256, buffer 1e6, train_freq 1, gradient_steps 1).  Three rates over the same envs:
    env only (U(-1,1) actions from HBM), env + policy (the reference's saved SAC actor,
    stochastic, forward on the kernel's fp32 obs rows), env + policy + one SAC update per
    vector step (tools/sac_torch.py; the whole iteration one HIP graph, the gradient
    all-reduce inside it over libbsg's RCCL communicator).  value = the last, whole job."""
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import sac_torch
    from bluesky_gym import _native as nat, config, core

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("BENCH_BACKEND", "nccl")   # gloo: multi-rank rehearsal on one GPU
    if world > 1:
        torch.cuda.set_device(local % torch.cuda.device_count())
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.blas != "default":
        # the learner's GEMMs are batch-256 x 256-wide: hipBLASLt's default pick for them is a
        # 256x256 macro tile, i.e. one or a few workgroups for the whole product
        torch.backends.cuda.preferred_blas_library(args.blas)
        if args.blas == "cublas":
            # nn.Linear's addmm-with-bias otherwise still goes to hipBLASLt's bias epilogue
            os.environ["DISABLE_ADDMM_CUDA_LT"] = "1"
    E = args.total_envs // world
    cfg = config.descent_config()
    b = core.DeviceBatch(cfg, E, autoreset=nat.AUTORESET_SAME_STEP, compute_cd=False,
                         seed=1234, env_offset=rank * E)
    b.reset()
    W = dict(np.load(os.path.join(REPO, "tests", "golden", "sac_actors.npz")))
    # FusedSAC (tools/sac_fused.hip) with the gradients all-reduced before each Adam launch:
    # over libbsg's RCCL communicator on the update's stream (the iteration stays one HIP
    # graph at any rank count; at one rank a one-rank communicator, so the reduce is timed)
    # or torch.distributed (eager: the gloo rehearsal); SAC_FUSED=0 = the autograd update
    cls = sac_torch.FusedSAC if os.environ.get("SAC_FUSED", "1") == "1" else sac_torch.SAC
    reduce = args.learner_reduce
    if reduce == "auto":
        reduce = "rccl" if (world == 1 or backend == "nccl") else "torch"
    comm = None
    if reduce == "rccl":
        from bluesky_gym.parallel import RcclGather
        comm = RcclGather(dev, dist.group.WORLD if world > 1 else None)
    sac = cls(b.obs_dim, b.act_dim, dev, group=dist.group.WORLD if world > 1 else None,
              seed=rank, lr=1e-3, comm=comm)
    sac.actor.load_sb3(W, "descent")
    gen = torch.Generator(device=dev)
    gen.manual_seed(17 + rank)
    bank = torch.rand((16, E, 1), dtype=torch.float64, device=dev, generator=gen) * 2 - 1

    def timed(fn, steps):
        for k in range(args.warmup):
            fn(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            fn(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t[0])
        return el

    el_env = timed(lambda k: b.step(bank[k % 16]), args.steps)
    # (torch.distributed's eager all-reduce cannot sit in the graph; libbsg's can)
    graph = not args.no_graph and (world == 1 or comm is not None)
    fused = not args.torch_policy

    def policy_loop(fused_policy):
        pol = sac_torch.RLLoop(b, sac, learn=False, fused_policy=fused_policy)
        pol.obs.copy_(b.obs)
        if graph:
            pol.capture()
        return timed((lambda k: pol.replay()) if graph else (lambda k: pol.step()), args.steps)

    el_pol = policy_loop(fused)
    el_pol_torch = policy_loop(False) if fused else el_pol
    rl = sac_torch.RLLoop(b, sac, learn=True, fused_policy=fused)
    rl.obs.copy_(b.obs)
    for _ in range(8):                                # fill the buffer past one batch
        rl.step()
    if graph:
        rl.capture()
    el_rl = timed((lambda k: rl.replay()) if graph else (lambda k: rl.step()), args.steps)
    lq, la = sac.update()                             # one more update: finite losses
    torch.cuda.synchronize()
    reduces = comm.info()["reduces"] if comm is not None else 0
    if rank == 0:
        total = world * E * args.steps
        out = {
            "metric": "env steps/sec incl. SAC learner (whole node), DescentEnv-v0 4096 envs, "
                      "1/2/4/8 GPUs (BASELINE configs[4])",
            "value": total / el_rl,
            "unit": "env_steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el_rl * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64 env / fp32 learner",
            "data": "synthetic: device Philox spawns (descent_env.py distributions); actor "
                    "initialised from the reference's saved SAC actor (weights only)",
            "config": {"workload": f"DescentEnv-v0 {world * E} envs ({E} per GPU), 30 substeps x "
                                   f"DT 1 s, SAME_STEP autoreset + final_obs, SAC batch 256 "
                                   f"buffer 1e6 train_freq 1 gradient_steps 1",
                       "envs_total": world * E, "envs_per_gpu": E,
                       "parallelism": f"env-shard x{world}" + (
                           (" + RCCL" if backend == "nccl" else f" + {backend}") +
                           " gradient all_reduce (data-parallel SAC)" if world > 1 else ""),
                       "policy": "fused HIP actor (bsg_policy_sac)" if fused else "torch actor",
                       "adam": "one launch per step (tools/sac_adam.hip)" if sac.hip_adam else
                               "torch " + os.environ.get("SAC_ADAM", "fused"),
                       "hip_graph": graph, "blas": str(torch.backends.cuda.preferred_blas_library()),
                       "update": type(sac).__name__,
                       "learner_reduce": ("rccl: bsg_comm_all_reduce (ncclAllReduce avg) of the "
                                          "critics' and the actor's gradients on the update's "
                                          f"stream, {comm.world} rank(s), {reduces} calls issued "
                                          "(a graph replay re-runs its captured ones)"
                                          if comm is not None else
                                          "torch.distributed all_reduce (eager)" if world > 1 else
                                          "none (one rank)")},
            "env_only": {"value": total / el_env, "ms_per_step": el_env * 1e3 / args.steps},
            "env_policy": {"value": total / el_pol, "ms_per_step": el_pol * 1e3 / args.steps,
                           "policy": "fused HIP actor (bsg_policy_sac)" if fused else "torch actor"},
            "env_policy_torch_actor": {"value": total / el_pol_torch,
                                       "ms_per_step": el_pol_torch * 1e3 / args.steps},
            "env_policy_learner": {"value": total / el_rl, "ms_per_step": el_rl * 1e3 / args.steps,
                                   "critic_loss": float(lq), "actor_loss": float(la)},
        }
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
