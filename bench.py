"""Benchmark: device-resident share-encode + recombine+verify, secret words/s.

One step = one pass of the hot path over one batch of words:
  K_MASK  createSecret arithmetic: verify the N-party Input Mask ODOs and mask
          every secret word (DefaultAmphoraClient.java:150-160)
  K_RV    getSecret arithmetic: recombine the N-party share ODOs and verify
          the MACs (DefaultAmphoraClient.java:206-217,476-505)
Inputs are synthetic honest N-party ODOs generated on the device (seeded),
resident in HBM before the timed region.

Default workload at EVERY world size = BASELINE config C4: 2^26 words in
total, 2 parties, the reference's test prime, one contiguous 2^26 / N-word
shard resident on each rank (strong scaling, no data-path collective), so
the N = 1, 2, 4, 8 lines are points of one curve.  The per-step verify
verdicts are combined with one RCCL all-reduce(MIN) of the per-step
first-fail vector after the last step.  `--workload c2|c3` runs the per-GPU
(weak-scaling) C2 / C3 arrays instead (builder-side lines).

Multi-GPU (one rank per GPU): `--gpus N` under torch.distributed.run, or
`--gpus N` alone, which starts torch.distributed.run itself as a child
process before anything touches the GPU.  With a process group the line
also carries `scatter_gather`: the same C4 job with the whole arrays held by
rank 0, scattered and gathered every step by one grouped RCCL send/recv
batch per direction over xGMI (SURVEY.md 8e's second curve).

Prints ONE JSON line (rank 0).  Per-kernel HIP-event timings on the launch
stream (--samples launches of each kernel, spread over the timed steps) feed
`roofline`; `cpu_baseline` times the C oracle (a multithreaded port of the
reference's BigInteger algorithm) on a bounded sample, on rank 0 at every
world size, after all GPU work and the process group are done.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "secret words/s device-resident share+recombine, 128-bit prime, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
NO_FAIL = 0x7F7F7F7F7F7F7F7F

# stdout carries exactly ONE line, the JSON result: everything else written to
# file descriptor 1 (RCCL's version banner, gloo's connection messages, HIP
# runtime notes) is sent to stderr, and emit() writes to the saved stdout.
_RESULT_FD = None


def _claim_stdout():
    global _RESULT_FD
    if _RESULT_FD is None:
        sys.stdout.flush()
        _RESULT_FD = os.dup(1)
        os.dup2(2, 1)


def emit(obj) -> None:
    data = (json.dumps(obj) + "\n").encode()
    fd = _RESULT_FD if _RESULT_FD is not None else 1
    while data:
        data = data[os.write(fd, data):]


def kbytes(kernel: str, n: int) -> int:
    """Algorithmic HBM bytes per word."""
    return {"k_rv": 80 * n + 16, "k_mask": 80 * n + 32}[kernel]


# BASELINE.json configs the device-resident bench runs: (words, parties,
# words are per GPU (weak) or the whole job split over the ranks (strong))
WORKLOADS = {"c2": (1 << 20, 2, "weak"), "c3": (1 << 24, 3, "weak"), "c4": (1 << 26, 2, "strong")}


def config_name(words: int, parties: int) -> str:
    """BASELINE.json config a device-resident run corresponds to (per GPU)."""
    return {(1 << 20, 2): "C2", (1 << 24, 3): "C3", (1 << 26, 2): "C4 size"}.get(
        (words, parties), "custom")


def available_cpus():
    """CPUs this process may use: its affinity mask, capped by a cgroup-v2
    CPU quota when one is set (a GPU box leases a share of a large host)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(a) -> int:
    """`bench.py --gpus N` with no launcher: run N ranks under
    torch.distributed.run as a CHILD process (nothing here has touched the
    GPU, and nothing is exec'd), pass its one JSON line through, return its
    exit code."""
    import subprocess
    argv = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            "--nproc-per-node", str(a.gpus), "--master-addr", "127.0.0.1",
            "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(argv, env=env)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # device mode: a C2 step is ~70 us, so 1000 timed steps after 100 warm-up
    # steps take ~80 ms; host and scatter modes move GBs per step: 5 after 1
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", choices=["auto", "c2", "c3", "c4"], default="auto",
                    help="device mode: BASELINE config; auto = C4 (2^26 words in total, 2 parties, "
                         "split over the ranks) at every world size; c2 / c3 are per-GPU "
                         "(weak-scaling) builder-side lines")
    ap.add_argument("--words", type=int, default=None,
                    help="words per GPU (custom device workload; host mode: words per rank)")
    ap.add_argument("--parties", type=int, default=None)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher rehearsal without a GPU: rendezvous, shard ranges, the "
                         "verdict and timing reductions over the process group; no kernels")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--samples", type=int, default=32,
                    help="event-stamped launches per kernel, spread evenly over the timed "
                         "steps, at most one per step (each costs ~3-4 us of dispatch, "
                         "tools/step_overhead.py)")
    ap.add_argument("--event-mode", choices=["launch", "record"], default="launch",
                    help="launch: events stamped by the kernel dispatch (hipExtLaunchKernel); "
                         "record: hipEventRecord on the stream right before and after the call")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--mode", choices=["device", "host"], default="device",
                    help="host: inputs/outputs in host memory (PCIe-inclusive rate, C5)")
    ap.add_argument("--pin", action="store_true", help="host mode: page-lock the inputs first")
    ap.add_argument("--batch-words", type=int, default=4 << 20)
    ap.add_argument("--host-devices", default="",
                    help="host mode: comma list of device ordinals for one amph_ctx_create_multi "
                         "context (each GPU streams its own shard over its own PCIe link)")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) on the GPU node; gloo to "
                    "rehearse several ranks on one GPU")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank uses cuda:0 (only with --backend gloo)")
    ap.add_argument("--dist", action="store_true",
                    help="create the process group even at world size 1 (runs the RCCL "
                         "verdict reduction / scatter-gather path on one GPU)")
    ap.add_argument("--no-scatter-gather", action="store_true",
                    help="skip the root-held (RCCL scatter/gather-inclusive) C4 measurement that "
                         "follows the device-resident one when a process group exists")
    ap.add_argument("--pad-words", type=int, default=0,
                    help="device mode: allocate each party's five ODO fields as rows of a slab "
                         "W + PAD words long (PAD = 0: rows exactly 2^k words apart)")
    ap.add_argument("--sg-steps", type=int, default=3)
    ap.add_argument("--sg-warmup", type=int, default=1)
    ap.add_argument("--sg-timeout", type=float, default=60.0,
                    help="seconds any one point-to-point batch or collective of the scatter/gather "
                         "phase may take before the phase is abandoned (its sub-object then says "
                         "`skipped`, the communicator is aborted and the line still prints)")
    ap.add_argument("--pg-timeout", type=float, default=180.0,
                    help="process-group timeout (seconds) for every other collective")
    ap.add_argument("--inject-sg-fault", choices=["", "error", "hang", "host-hang"], default="",
                    help=argparse.SUPPRESS)  # tests: rank 1 raises / never posts its gather sends /
    # (--dry-run) never joins the host phase's size agreement
    ap.add_argument("--no-host-phase", action="store_true",
                    help="device mode: skip the PCIe-inclusive host_memory sub-object")
    ap.add_argument("--host-words", type=int, default=32 << 20,
                    help="host_memory phase: words per rank (C5's per-GPU share, 2^28 / 8)")
    ap.add_argument("--host-parties", type=int, default=3)
    ap.add_argument("--host-steps", type=int, default=3)
    ap.add_argument("--host-warmup", type=int, default=1)
    ap.add_argument("--host-timeout", type=float, default=120.0,
                    help="seconds any one collective of the host_memory phase may wait for a peer "
                         "before the phase is abandoned (the line still prints)")
    a = ap.parse_args()
    if a.workload == "auto":
        a.workload = "c4"
    wl_words, wl_parties, a.scaling = WORKLOADS[a.workload]
    if a.words is None:
        a.words = (1 << 20) if a.mode == "host" else wl_words
    else:
        a.workload, a.scaling = "custom", "weak"
    if a.parties is None:
        a.parties = 2 if (a.mode == "host" or a.workload == "custom") else wl_parties
    elif a.parties != wl_parties and a.workload != "custom":
        a.workload, a.scaling = "custom", "weak"
    bulk = a.mode == "host"
    if a.steps is None:
        a.steps = 5 if bulk else 1000
    if a.warmup is None:
        a.warmup = 1 if bulk else 100
    return a


def scatter_gather_phase(a, A, torch, dist, ctx, rank, world, value_resident):
    """BASELINE C4 with the arrays held by ONE GPU, after the
    device-resident measurement: rank 0 holds the 10N+1 whole W-word input
    arrays (N-party mask ODOs, N-party share ODOs, secrets) and every step
    scatters them in contiguous shards, runs K_MASK + K_RV on each shard and
    gathers the masked words and canonical secrets straight into rank 0's
    output array.  Each direction is ONE grouped point-to-point batch
    (`RootScatterGather`: RCCL ncclGroupStart / ncclSend x peers x arrays /
    ncclRecv / ncclGroupEnd over xGMI); nothing is allocated per step.
    Returns the `scatter_gather` sub-object of rank 0's line.

    Every point-to-point batch and collective after the set-up is bounded by
    --sg-timeout: a peer that never posts its half (the first RCCL P2P
    between distinct GPUs is the one path no one-GPU rehearsal executes)
    becomes `{"skipped": ..., "aborted": true}` on the ranks that saw it,
    and main() then aborts the communicator instead of tearing it down, so
    the device-resident and host-memory numbers still print."""
    from amphora_amd.shard import RootScatterGather
    lib = A._lib
    W, n = a.words, a.parties
    sg = full_in = full_out = splain = None
    err = None
    try:  # every allocation first; the ranks agree before any point-to-point op is posted
        sg = RootScatterGather(W, 10 * n + 1, 2, device="cuda")
        if rank == 0:
            full_in = torch.empty((10 * n + 1, W, 16), dtype=torch.uint8, device="cuda")
            ctx.synth_odos(seed=21, n=n, words=W, buf=full_in[:5 * n].view(5, n, W, 16))
            _, _, splain = ctx.synth_odos(seed=22, n=n, words=W, with_plain=True,
                                          buf=full_in[5 * n:10 * n].view(5, n, W, 16))
            ctx.synth_words(seed=23, count=W, out=full_in[10 * n])
            full_out = torch.empty((2, W, 16), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
    except (RuntimeError, MemoryError) as e:  # (torch.OutOfMemoryError is a RuntimeError)
        err = "%s: %s" % (type(e).__name__, str(e).splitlines()[0][:200] if str(e) else "")
    failed = torch.tensor([1 if err else 0], dtype=torch.int32,
                          device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(failed, op=dist.ReduceOp.MAX)
    if failed.item():
        # a rank could not set up: skip the phase on every rank (no send or
        # receive was posted, so nothing is left waiting); the device-resident
        # line stands
        del full_in, full_out, splain
        torch.cuda.empty_cache()
        return {"skipped": "setup failed on %s: %s" % ("rank 0" if err and rank == 0 else "a rank",
                                                      err or "see that rank's stderr")}
    count = sg.count
    T = getattr(a, "sg_timeout", 60.0)
    inject = getattr(a, "inject_sg_fault", "")
    try:
        return _scatter_gather_timed(a, torch, dist, ctx, lib, rank, world, value_resident, sg, full_in,
                                     full_out, splain, count, T, inject)
    except Exception as e:  # a P2P batch or collective that timed out or failed (RCCL / gloo error)
        return {"skipped": "scatter/gather aborted on rank %d: %s: %s" % (
                    rank, type(e).__name__, (str(e).splitlines() or [""])[0][:300]),
                "aborted": True, "timeout_s": T}


def maybe_inject(inject, rank, world):
    """Test hook (--inject-sg-fault): rank 1 raises ("error") or silently
    skips posting its half of the gather ("hang"), as a stuck RCCL peer
    would.  Returns True when the caller must skip its gather."""
    if inject not in ("error", "hang") or world < 2 or rank != 1:
        return False
    if inject == "error":
        raise RuntimeError("injected scatter/gather fault on rank 1")
    return True


def guarded_all_reduce(dist, t, op, timeout_s):
    """all_reduce that gives up after `timeout_s` (raises) instead of blocking
    for ever when a peer has left the phase."""
    import datetime
    w = dist.all_reduce(t, op=op, async_op=True)
    if not w.wait(timeout=datetime.timedelta(seconds=timeout_s)):
        raise TimeoutError("all_reduce not complete after %.0f s" % timeout_s)
    return t


def _scatter_gather_timed(a, torch, dist, ctx, lib, rank, world, value_resident, sg, full_in, full_out,
                          splain, count, T, inject):
    import ctypes as C
    n, W = a.parties, a.words
    ff = torch.full((2,), NO_FAIL, dtype=torch.int64, device="cuda")
    ffp = [C.cast(C.c_void_p(ff.data_ptr() + 8 * i), C.POINTER(C.c_int64)) for i in range(2)]
    flags = lib.AMPH_F_DEVICE | lib.AMPH_F_ACCUMULATE
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    structs = {}
    sync_dev = "cuda" if dist.get_backend() == "nccl" else "cpu"

    def barrier():
        torch.cuda.synchronize()
        guarded_all_reduce(dist, torch.zeros(1, dtype=torch.int32, device=sync_dev), dist.ReduceOp.MAX, T)

    def step():
        local = sg.scatter(full_in, timeout=T)
        out = sg.out_view(full_out)
        if count:
            if not structs:  # the shard views never move: build the ODO structs once
                structs["m"] = ctx._odo_structs([tuple(local[k * n + j] for k in range(5)) for j in range(n)])
                structs["s"] = ctx._odo_structs([tuple(local[5 * n + k * n + j] for k in range(5))
                                                 for j in range(n)])
            assert lib.lib.amph_mask_input(ctx._h, structs["m"][0], n, local[10 * n].data_ptr(), count,
                                           out[0].data_ptr(), ffp[0], flags, stream) == 0
            assert lib.lib.amph_recombine_verify(ctx._h, structs["s"][0], n, out[1].data_ptr(), ffp[1],
                                                 flags, stream) == 0
        if not maybe_inject(inject, rank, world):
            sg.gather(full_out, timeout=T)

    for _ in range(a.sg_warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.sg_steps):
        step()
    barrier()
    el = time.perf_counter() - t0
    g = torch.where(ff == NO_FAIL, ff, ff + sg.start)
    guarded_all_reduce(dist, g, dist.ReduceOp.MIN, T)
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    guarded_all_reduce(dist, t, dist.ReduceOp.MAX, T)
    el = t.item()
    checks = {"honest_verdicts": bool((g == NO_FAIL).all().item())}
    res = None
    if rank == 0:
        # the gathered secrets are the generated ones; the gathered masked
        # words equal one K_MASK launch over the root's whole arrays
        checks["secrets_match"] = bool(torch.equal(full_out[1], splain))
        mo = [tuple(full_in[k * n + j] for k in range(5)) for j in range(n)]
        ref = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
        marr, _ = ctx._odo_structs(mo)
        ff1 = torch.full((1,), NO_FAIL, dtype=torch.int64, device="cuda")
        assert lib.lib.amph_mask_input(ctx._h, marr, n, full_in[10 * n].data_ptr(), W, ref.data_ptr(),
                                       C.cast(C.c_void_p(ff1.data_ptr()), C.POINTER(C.c_int64)),
                                       flags, stream) == 0
        checks["masked_match_one_gpu"] = bool(torch.equal(full_out[0], ref))
        moved = sg.moved_bytes()
        ms = el * 1e3 / a.sg_steps
        value = W * a.sg_steps / el
        res = {"words_per_s": value, "ms_per_step": ms, "steps": a.sg_steps, "warmup": a.sg_warmup,
               "vs_device_resident": round(value / value_resident, 4) if value_resident else None,
               "root_bytes_per_step": moved, "root_link_GBps": round(moved / (ms * 1e-3) / 1e9, 1),
               "collective": "RootScatterGather: one batch_isend_irecv group per direction "
                             "(%s), %d sends per peer each way" % (
                                 "RCCL ncclSend/ncclRecv over xGMI" if dist.get_backend() == "nccl"
                                 else dist.get_backend() + " rehearsal, staged through host memory",
                                 10 * n + 1),
               "timeout_s": T, "verified": all(checks.values()), "verify_checks": checks}
    return res


def _read_int(path):
    try:
        with open(path) as fh:
            s = fh.read().strip()
        return None if s in ("", "max") else int(s)
    except (OSError, ValueError):
        return None


def _cgroup_paths(proc_cgroup):
    """This process's cgroup path for the v2 hierarchy ("0::/path") and for
    the v1 memory controller ("N:...memory...:/path"), from /proc/self/cgroup."""
    v2 = v1 = None
    try:
        with open(proc_cgroup) as fh:
            for ln in fh:
                parts = ln.rstrip("\n").split(":", 2)
                if len(parts) != 3:
                    continue
                if parts[0] == "0" and parts[1] == "":
                    v2 = parts[2] or "/"
                elif "memory" in parts[1].split(","):
                    v1 = parts[2] or "/"
    except OSError:
        pass
    return v2, v1


def _cgroup_headroom(base, rel, limit_f, usage_f, stat_keys):
    """Walk from this process's cgroup up to the hierarchy's root: every
    ancestor's limit binds, so the headroom is the smallest (limit - usage
    + reclaimable inactive file pages) along the way.  Returns (limit, used,
    directory) of the binding level, or None when no level sets a limit."""
    best = None
    d = os.path.normpath(base + "/" + (rel or "/").lstrip("/"))
    base = os.path.normpath(base)
    while True:
        lim = _read_int(os.path.join(d, limit_f))
        if lim is not None and lim < 1 << 60:  # (v1 "unlimited" is a huge number)
            used = _read_int(os.path.join(d, usage_f)) or 0
            try:
                with open(os.path.join(d, "memory.stat")) as fh:
                    for ln in fh:
                        k, _, v = ln.partition(" ")
                        if k in stat_keys:
                            used = max(0, used - int(v))
                            break
            except (OSError, ValueError):
                pass
            if best is None or lim - used < best[0] - best[1]:
                best = (lim, used, d)
        if d == base or len(d) <= len(base):
            break
        d = os.path.dirname(d)
    return best


def memory_limits():
    """Host memory this process may still use, from the two sources that can
    end it: its memory cgroup -- the process's own cgroup and every ancestor
    (v2 `memory.max` / `memory.current`, or v1 `memory.limit_in_bytes` /
    `memory.usage_in_bytes`; usage minus reclaimable inactive file pages) --
    and the host's `MemAvailable`.  AMPH_BENCH_MEM_LIMIT_BYTES /
    AMPH_BENCH_MEM_AVAILABLE_BYTES replace the probed values (tests inject a
    small limit; a harness may pin one); AMPH_BENCH_CGROUP_ROOT /
    AMPH_BENCH_PROC_CGROUP point the probe at another tree (tests).  Returns a
    dict of what was found; `headroom_bytes` is the smaller of the two
    headrooms (None: nothing known)."""
    root = os.environ.get("AMPH_BENCH_CGROUP_ROOT", "/sys/fs/cgroup")
    v2, v1 = _cgroup_paths(os.environ.get("AMPH_BENCH_PROC_CGROUP", "/proc/self/cgroup"))
    found = None
    if os.path.exists(os.path.join(root, "cgroup.controllers")) or v2 is not None:
        found = _cgroup_headroom(root, v2 or "/", "memory.max", "memory.current", ("inactive_file",))
    if found is None:
        found = _cgroup_headroom(os.path.join(root, "memory"), v1 or "/", "memory.limit_in_bytes",
                                 "memory.usage_in_bytes", ("total_inactive_file", "inactive_file"))
    cg_limit, cg_used, cg_dir = found if found else (None, None, None)
    avail = None
    try:
        with open("/proc/meminfo") as fh:
            for ln in fh:
                if ln.startswith("MemAvailable:"):
                    avail = int(ln.split()[1]) * 1024
                    break
    except (OSError, ValueError, IndexError):
        pass
    src = {"limit": "cgroup %s" % cg_dir if cg_limit is not None else None, "available": "/proc/meminfo"}
    if os.environ.get("AMPH_BENCH_MEM_LIMIT_BYTES"):
        cg_limit, cg_used, src["limit"] = int(os.environ["AMPH_BENCH_MEM_LIMIT_BYTES"]), 0, "env"
    if os.environ.get("AMPH_BENCH_MEM_AVAILABLE_BYTES"):
        avail, src["available"] = int(os.environ["AMPH_BENCH_MEM_AVAILABLE_BYTES"]), "env"
    heads = [h for h in ((cg_limit - cg_used) if cg_limit is not None else None, avail) if h is not None]
    return {"mem_limit_bytes": cg_limit, "mem_limit_used_bytes": cg_used, "mem_available_bytes": avail,
            "headroom_bytes": min(heads) if heads else None, "source": src}


HOST_FIXED_BYTES = 256 << 20  # per rank beyond the arrays: small-call arena, numpy/torch temporaries


def host_bytes_per_word(n):
    """Host footprint of host_memory_phase per word and rank: one n-party ODO
    set (5 fields) + secrets, plain secrets, masked words and canonical
    secrets, all page-locked; with page-locked caller arrays the pipeline
    stages nothing on the host."""
    return 80 * n + 64


def plan_host_words(a, dist, distributed, sync_dev, timeout_s):
    """How many words each rank streams in host_memory_phase, decided BEFORE
    anything is allocated: the ranks on this node share its memory, so each
    may use at most half of the smaller headroom (cgroup limit, MemAvailable)
    divided by the node's rank count; the size is whole --batch-words
    batches, at most --host-words, and the ranks agree on the smallest (one
    all-reduce(MIN)).  Returns (words, record): words 0 means "skip the
    phase", with the reason in record["skipped"].  A SIGKILL from the OOM
    killer cannot be caught, so this is the only guard that keeps the line."""
    import torch
    lim = memory_limits()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    per_word = host_bytes_per_word(a.host_parties)
    want = max(0, a.host_words)
    unit = max(1, min(a.batch_words, want))  # whole batches (or the whole request when smaller)
    if lim["headroom_bytes"] is None:
        words = want
        budget = None
    else:
        budget = lim["headroom_bytes"] // 2 // max(1, local_world)
        fit = max(0, budget - HOST_FIXED_BYTES) // per_word
        words = min(want, fit // unit * unit)
    if distributed:
        t = torch.tensor([words], dtype=torch.int64, device=sync_dev)
        guarded_all_reduce(dist, t, dist.ReduceOp.MIN, timeout_s)
        words = int(t.item())
    rec = dict(lim, local_world_size=local_world, budget_bytes_per_rank=budget, host_bytes_per_word=per_word,
               fixed_bytes_per_rank=HOST_FIXED_BYTES, host_words_requested=want, host_words_chosen=words,
               rule="per rank: min(cgroup headroom, MemAvailable) / 2 / ranks on the node, whole "
                    "batches, min over ranks")
    if words < unit:
        rec["skipped"] = ("host memory: %s B of headroom gives %s B per rank, under one %d-word batch "
                          "(%d B at %d B/word + %d B fixed)"
                          % (lim["headroom_bytes"], budget, unit, unit * per_word, per_word,
                             HOST_FIXED_BYTES))
        return 0, rec
    return words, rec


def host_memory_phase(a, torch, dist, ctx, rank, world, distributed):
    """PCIe-inclusive rate inside the default line (the
    reference path starts and ends in host memory, DefaultAmphoraClient.java:
    150-170,206-217): on every rank, C5's per-GPU share (--host-words,
    2^28 / 8 = 32 Mi words, --host-parties 3) in page-locked host arrays,
    streamed through this rank's GPU in --batch-words batches by the two
    host-pointer calls a client makes (amph_mask_input, then
    amph_recombine_verify; 3-slot HtoD / kernel / DtoH pipeline), outputs
    written back to caller-owned page-locked arrays.  One n-party ODO set
    serves as both the mask and the share ODOs (the bytes moved are the
    same as with two sets; host RAM per rank stays ~9.5 GiB).

    --host-warmup untimed and --host-steps timed steps, bracketed by a
    barrier + synchronize, max over ranks; words/s sums every rank's words.
    A pinned-copy probe of the same link (1 GiB HtoD, 512 MiB DtoH, same
    arrays) gives the fraction of what the link delivers.  verified: both
    calls report no MAC failure at every step, every canonical secret equals
    the generated one, and a 4096-word sample of the masked words equals
    toGfp((s - y) mod p) recomputed with Python integers
    (SecretShareUtil.java:65-68).  Returns rank 0's `host_memory`
    sub-object (None elsewhere)."""
    import numpy as np
    from amphora_amd.spdz import TEST_PRIME
    n = a.host_parties
    sync_dev = "cuda" if distributed and dist.get_backend() == "nccl" else "cpu"
    T = a.host_timeout
    try:
        W, plan = plan_host_words(a, dist, distributed, sync_dev, T)
    except Exception as e:  # noqa: BLE001 (a rank left before the plan: abandon, keep the line)
        return _host_abort(rank, "size agreement", e, T)
    if not W:
        return dict(plan) if rank == 0 else None
    arrays, err = [], None
    try:  # allocate + page-lock first; the ranks agree before anything is timed
        odos_h = np.empty((5, n, W, 16), np.uint8)
        sec_h, plain_h, masked_h, ys_h = (np.empty((W, 16), np.uint8) for _ in range(4))
        for arr in (odos_h, sec_h, plain_h, masked_h, ys_h):
            ctx.host_register(arr)
            arrays.append(arr)
        _, buf, plain = ctx.synth_odos(seed=4000 + rank, n=n, words=W, with_plain=True)
        torch.from_numpy(odos_h).copy_(buf)
        torch.from_numpy(plain_h).copy_(plain)
        del buf, plain
        torch.from_numpy(sec_h).copy_(ctx.synth_words(seed=5000 + rank, count=W))
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    except Exception as e:  # noqa: BLE001 (page-lock / OOM / HIP error: report, do not lose the line)
        err = "%s: %s" % (type(e).__name__, (str(e).splitlines() or [""])[0][:200])
    try:
        if distributed:
            f = torch.tensor([1 if err else 0], dtype=torch.int32, device=sync_dev)
            guarded_all_reduce(dist, f, dist.ReduceOp.MAX, T)
            if f.item() and not err:
                err = "set-up failed on another rank"
        if err:
            return dict(plan, skipped="rank %d: %s" % (rank, err)) if rank == 0 else None
        return _host_timed(a, torch, dist, ctx, rank, world, distributed, sync_dev, T, W, n, plan,
                           odos_h, sec_h, plain_h, masked_h, ys_h, TEST_PRIME)
    except Exception as e:  # noqa: BLE001 (a collective timed out / a rank failed mid-phase)
        return _host_abort(rank, "timed section", e, T)
    finally:
        for arr in arrays:
            ctx.host_unregister(arr)


def _host_abort(rank, where, e, T):
    """host_memory_phase gave up after a collective timed out or a call
    failed: the sub-object says so, and `aborted` makes main() skip the
    scatter/gather phase and abort the communicator (its state is unknown)
    while still printing the line.  Every rank returns it (main() reads
    `aborted` on each)."""
    return {"skipped": "host phase aborted on rank %d (%s): %s: %s" % (
                rank, where, type(e).__name__, (str(e).splitlines() or [""])[0][:300]),
            "aborted": True, "timeout_s": T}


def _host_timed(a, torch, dist, ctx, rank, world, distributed, sync_dev, T, W, n, plan,
                odos_h, sec_h, plain_h, masked_h, ys_h, prime):
    import numpy as np

    def barrier():
        torch.cuda.synchronize()
        if distributed:
            guarded_all_reduce(dist, torch.zeros(1, dtype=torch.int32, device=sync_dev), dist.ReduceOp.MAX, T)

    ctx.set_batch_words(a.batch_words)
    odos = [tuple(odos_h[k, j] for k in range(5)) for j in range(n)]
    # the link itself, same arrays: pinned HtoD / DtoH copies on one stream
    src = torch.from_numpy(odos_h.reshape(-1)[:min(1 << 30, odos_h.nbytes)])
    dst = torch.from_numpy(masked_h.reshape(-1)[:min(1 << 29, masked_h.nbytes)])
    probe_dev = torch.empty(src.numel(), dtype=torch.uint8, device="cuda")

    def copy_rate(fn, nbytes, reps=3):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return reps * nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9

    htod_link = copy_rate(lambda: probe_dev.copy_(src, non_blocking=True), src.numel())
    dtoh_link = copy_rate(lambda: dst.copy_(probe_dev[:dst.numel()], non_blocking=True), dst.numel())
    del probe_dev
    torch.cuda.empty_cache()
    ok = True
    for _ in range(a.host_warmup):
        ctx.mask_input(odos, sec_h, out=masked_h)
        ctx.recombine_verify(odos, out=ys_h)
    masked_h.fill(0)
    ys_h.fill(0)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.host_steps):
        _, f1 = ctx.mask_input(odos, sec_h, out=masked_h)
        _, f2 = ctx.recombine_verify(odos, out=ys_h)
        ok &= f1 == -1 and f2 == -1
    barrier()
    el = time.perf_counter() - t0
    checks = {"honest_verdicts": bool(ok), "secrets_match": bool(np.array_equal(ys_h, plain_h))}
    idx = np.unique(np.random.default_rng(17).integers(0, W, 4096))
    R = (1 << 128) % prime
    good = True
    for i in idx:
        s_i = int.from_bytes(sec_h[i].tobytes(), "little")
        y_i = int.from_bytes(plain_h[i].tobytes(), "little")
        good &= (((s_i - y_i) % prime) * R % prime).to_bytes(16, "little") == masked_h[i].tobytes()
    checks["masked_sample_match"] = bool(good)
    ok = all(checks.values())
    vals = [el, 0.0 if ok else 1.0, htod_link, dtoh_link]
    if distributed:
        t = torch.tensor(vals[:2], dtype=torch.float64, device=sync_dev)
        guarded_all_reduce(dist, t, dist.ReduceOp.MAX, T)
        lk = torch.tensor(vals[2:], dtype=torch.float64, device=sync_dev)
        guarded_all_reduce(dist, lk, dist.ReduceOp.MIN, T)
        vals = t.tolist() + lk.tolist()
    el, bad, htod_link, dtoh_link = vals
    if rank != 0:
        return None
    htod_b, dtoh_b = 160 * n + 16, 32  # per word and step: 2 ODO sets + secrets in, 2 outputs out
    ms = el * 1e3 / a.host_steps
    htod = htod_b * W * a.host_steps / el / 1e9  # per rank, the slowest rank's time
    return {"words_per_s": W * world * a.host_steps / el, "ms_per_step": ms,
            "steps": a.host_steps, "warmup": a.host_warmup,
            "words_per_rank": W, "parties": n, "batch_words": a.batch_words,
            "host_bytes_per_step": (htod_b + dtoh_b) * W * world,
            "host_GBps": (htod_b + dtoh_b) * W * world * a.host_steps / el / 1e9,
            "htod_GBps_per_rank": round(htod, 2),
            "link_probe_GBps": {"htod": round(htod_link, 2), "dtoh": round(dtoh_link, 2),
                                "bytes": [int(src.numel()), int(dst.numel())],
                                "note": "pinned copies of the same arrays (HtoD, DtoH bytes), min over ranks"},
            "frac_of_link": round(htod / htod_link, 4),
            "memory": "page-locked caller arrays (amph_host_register), outputs reused across calls",
            "memory_plan": plan,
            "workload": "C5 per-GPU share: amph_mask_input + amph_recombine_verify from host "
                        "memory, %d words x %d parties per rank" % (W, n),
            "verified": bad == 0.0, "verify_checks": checks}


def host_mode(a, A, torch, ctx, dist=None, rank=0, world=1):
    """End-to-end host-memory rate: ODOs and secrets live in
    (pageable or page-locked) host memory; each step streams them through the
    GPU in --batch-words batches (3-slot HtoD/compute/DtoH pipeline) and
    writes the masked words and canonical secrets back to host memory.  Under
    torchrun every rank streams its own W-word shard from its own host memory
    over its own PCIe link (weak scaling, C5 on 8 GPUs = 32 Mi words per
    rank); the timed region is bracketed by barriers, the time is the max
    over ranks and `value` counts every rank's words.  Not the headline
    metric; recorded in DESIGN.md."""
    import numpy as np
    W, n = a.words, a.parties
    coll = dist is not None and dist.is_initialized()
    gen = ctx
    if a.host_devices:  # one context over several devices: per-GPU shards from host memory
        ctx = A.Context(ctx.prime, ctx.r, ctx.r_inv, devices=[int(d) for d in a.host_devices.split(",")])
    ctx.set_batch_words(a.batch_words)
    _, mb, _ = gen.synth_odos(seed=11, n=n, words=W)
    mask_h = mb.cpu().numpy()
    del mb
    _, sb, splain = gen.synth_odos(seed=12, n=n, words=W, with_plain=True)
    share_h = sb.cpu().numpy()
    plain_h = splain.cpu().numpy()
    del sb, splain
    sec_h = gen.synth_words(seed=13, count=W).cpu().numpy()
    torch.cuda.empty_cache()
    mask_odos = [tuple(mask_h[k, j] for k in range(5)) for j in range(n)]
    share_odos = [tuple(share_h[k, j] for k in range(5)) for j in range(n)]
    # output buffers the caller keeps across calls (a client reuses them; a
    # fresh 16 B/word array per call would time numpy's page faults and frees)
    masked_h = np.empty((W, 16), np.uint8)
    ys_h = np.empty((W, 16), np.uint8)
    masked_h.fill(0)
    ys_h.fill(0)
    if a.pin:
        for arr in (mask_h, share_h, sec_h, masked_h, ys_h):
            ctx.host_register(arr)
    for _ in range(a.warmup):
        ctx.mask_input(mask_odos, sec_h, out=masked_h)
        ctx.recombine_verify(share_odos, out=ys_h)
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    t0 = time.perf_counter()
    ok = True
    for _ in range(a.steps):
        _, f1 = ctx.mask_input(mask_odos, sec_h, out=masked_h)
        _, f2 = ctx.recombine_verify(share_odos, out=ys_h)
        ok &= f1 == -1 and f2 == -1
    torch.cuda.synchronize()
    if coll:
        dist.barrier()
    el = time.perf_counter() - t0
    ok &= bool(np.array_equal(ys_h, plain_h))  # outputs, not only the verdicts
    if coll:
        t = torch.tensor([el, 0.0 if ok else 1.0], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, ok = t[0].item(), t[1].item() == 0.0
    hbytes = (kbytes("k_mask", n) + kbytes("k_rv", n)) * W  # per rank
    gpus = ctx.device_count * world
    if rank == 0:
        line = {"metric": "secret words/s host-memory share+recombine (PCIe-inclusive)",
                "value": W * world * a.steps / el, "unit": "words/s", "n_gpus": gpus,
                "steps": a.steps, "warmup": a.warmup, "ms_per_step": el * 1e3 / a.steps,
                "higher_is_better": True, "scaling": "weak", "verified": ok,
                "pinned_inputs": a.pin, "batch_words": a.batch_words,
                "host_bytes_per_step": hbytes * world, "host_GBps": hbytes * world * a.steps / el / 1e9,
                "config": {"workload": "K_MASK + K_RV from host memory", "words_per_rank": W,
                           "parties": n, "parallelism": "dp%d" % gpus}}
        emit(line)
    if a.pin:
        for arr in (mask_h, share_h, sec_h, masked_h, ys_h):
            ctx.host_unregister(arr)


def cpu_baseline(n: int, budget_s: float):
    """Time the C oracle (oracle/amphora_oracle.c: schoolbook multiply + Knuth
    division per fromGfp/toGfp, like BigInteger) on a bounded sample of the
    same workload: K_MASK + K_RV arithmetic over W_s words, N parties, on
    every CPU the lease grants (affinity mask capped by the cgroup quota),
    plus a short 1-thread pass for the per-core rate."""
    from oracle import coracle
    threads, affinity, quota = available_cpus()
    F = coracle.test_field(threads=threads)
    Ws = max(1 << 16, min(1 << 20, 8192 * threads))  # ~ms of work per call at any thread count
    mask_odos, _ = F.synth_odos(seed=3, n=n, W=Ws)
    share_odos, _ = F.synth_odos(seed=4, n=n, W=Ws)
    secrets = F.synth_words(seed=5, count=Ws, mont=False)

    def timed(budget, words):
        sec = secrets[:words]
        mo = [tuple(f[:words] for f in o) for o in mask_odos]
        so = [tuple(f[:words] for f in o) for o in share_odos]
        F.mask_input(sec, mo)  # warm-up
        done, t0 = 0, time.perf_counter()
        while True:
            _, f1 = F.mask_input(sec, mo)
            _, f2 = F.recombine_verify(so)
            assert f1 == -1 and f2 == -1
            done += words
            el = time.perf_counter() - t0
            if el >= budget:
                return done, el

    done, el = timed(budget_s, Ws)
    F.threads = 1
    done1, el1 = timed(max(1.0, budget_s / 5), 4096)
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": done / el, "unit": "words/s", "cores": threads, "kind": "port",
            "label": "C port of the BigInteger path (no JVM available)",
            "value_1_thread": done1 / el1,
            "cpu_model": model, "host_cpus": os.cpu_count(), "affinity_cpus": affinity,
            "cgroup_quota_cpus": quota,
            "sample": "%d words x %d reps (%.1f s): C oracle restating the Java BigInteger "
                      "path (maskInput+verify on %d-party mask ODOs, recombine+verify on "
                      "share ODOs), OpenMP %d threads; 1 thread: 4096 words x %d reps (%.1f s)"
                      % (Ws, done // Ws, el, n, threads, done1 // 4096, el1)}


def stream_probe_ms(lib, C, ctx, mask_arr, n, secrets, W, stream, samples, before):
    """Average duration (ms) of amph_stream_probe over `samples` launches
    stamped by their own dispatch.  Each follows a K_RV launch (`before`),
    as every K_MASK does in the timed steps, so the probe meets the same
    cache state: launched back to back on its own inputs it reads part of
    them from the 256 MB Infinity Cache at C2 and looks faster than HBM."""
    import torch
    out = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
    evs = [(lib.TimingEvent(), lib.TimingEvent()) for _ in range(samples)]
    res = []
    for back_to_back in (False, True):
        for e0, e1 in evs:
            if back_to_back:
                assert lib.lib.amph_stream_probe(ctx._h, mask_arr, n, secrets.data_ptr(), W,
                                                 out.data_ptr(), stream) == 0
            else:
                before()
            lib.lib.amph_time_next_launch(e0.handle, e1.handle)
            assert lib.lib.amph_stream_probe(ctx._h, mask_arr, n, secrets.data_ptr(), W, out.data_ptr(),
                                             stream) == 0
        torch.cuda.synchronize()
        res.append(sum(e0.elapsed_ms(e1) for e0, e1 in evs) / samples)
    return res  # [after K_RV (the timed steps' order), right after itself]


def pattern_probe(probe_ms, n, W, kern):
    """K_MASK's bandwidth against its own access pattern's, same run."""
    bpw = kbytes("k_mask", n)
    after, b2b = probe_ms
    gbs = bpw * W / (after * 1e-3) / 1e9
    return {"kernel": "k_stream_probe (K_MASK's loads/stores, XOR instead of field arithmetic)",
            "ms": round(after, 5), "GBps": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4),
            "k_mask_frac_of_probe": round(after / kern["k_mask"], 4),
            "ms_back_to_back": round(b2b, 5),
            "timing": "each probe launch follows a K_RV launch, as K_MASK does in the timed steps; "
                      "ms_back_to_back: each follows another probe launch over the same inputs"}


def check_outputs(ctx, lib, torch, C, stream, flags, n, W, secrets, masked, ys, mplain, splain,
                  share_arr, share_odos, prime, sample=4096):
    """Output checks of the last timed step, independent of the kernels:

    * K_RV's canonical secrets equal the secrets the share ODOs were generated
      from (every word, on the device);
    * K_MASK's masked words equal toGfp((s - m) mod p) for a sample of words,
      recomputed here with Python integers from the plain secrets s and the
      plain input masks m (SecretShareUtil.maskInput, SecretShareUtil.java:65-68);
    * a MAC fault injected into one share word (party 1's w at W // 3) is
      reported at exactly that index, and the word is restored afterwards."""
    torch.cuda.synchronize()
    out = {"secrets_match": bool(torch.equal(ys, splain))}
    idx = torch.unique(torch.randint(0, W, (min(sample, W),), generator=torch.Generator().manual_seed(7)))
    s_h = secrets[idx.cuda()].cpu().numpy()
    m_h = mplain[idx.cuda()].cpu().numpy()
    got = masked[idx.cuda()].cpu().numpy()
    R = (1 << 128) % prime
    good = True
    for k in range(len(idx)):
        s_i = int.from_bytes(s_h[k].tobytes(), "little")
        m_i = int.from_bytes(m_h[k].tobytes(), "little")
        exp = (((s_i - m_i) % prime) * R % prime).to_bytes(16, "little")
        good &= exp == got[k].tobytes()
    out["masked_sample_match"] = bool(good)
    fi = W // 3
    wf = share_odos[1 if n > 1 else 0][3]
    wf[fi, 0] ^= 1
    ff = torch.full((1,), NO_FAIL, dtype=torch.int64, device="cuda")
    tmp = torch.empty_like(ys)
    st = lib.lib.amph_recombine_verify(ctx._h, share_arr, n, tmp.data_ptr(),
                                       C.cast(C.c_void_p(ff.data_ptr()), C.POINTER(C.c_int64)),
                                       flags, stream)
    wf[fi, 0] ^= 1
    out["fault_detected"] = st == 0 and int(ff.item()) == fi
    return out


def dry_run(a, world, rank):
    """--dry-run: the multi-rank plumbing of the device bench with no GPU --
    rendezvous, this rank's shard of the workload, the batched verdict
    all-reduce(MIN) with local indices made global, the max-over-ranks time,
    one line from rank 0.  `value` is null: nothing is measured."""
    import torch
    import torch.distributed as dist
    from amphora_amd.shard import shard_range
    if world > 1 or a.dist:
        dist.init_process_group("gloo", timeout=pg_timeout(a))
    total = a.words if a.scaling == "strong" else a.words * world
    start, count = shard_range(total, rank, world) if a.scaling == "strong" else (rank * a.words, a.words)
    steps = a.warmup + a.steps
    verdicts = torch.full((steps, 2), NO_FAIL, dtype=torch.int64)
    if rank == world - 1:  # a fault in the last rank's shard, local index count // 3
        verdicts[-1, 1] = count // 3
    t0 = time.perf_counter()
    verdicts = torch.where(verdicts == NO_FAIL, verdicts, verdicts + start)
    if dist.is_initialized():
        dist.all_reduce(verdicts, op=dist.ReduceOp.MIN)
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ranks = [rank_record(torch, rank, local, el.item(), 0.0, 0.0, count)]
    if dist.is_initialized():
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        sizes = torch.tensor([count], dtype=torch.int64)
        dist.all_reduce(sizes)
        covered = int(sizes.item())
        ranks = [None] * world
        dist.all_gather_object(ranks, rank_record(torch, rank, local, el.item(), 0.0, 0.0, count))
    else:
        covered = count
    sg_ok, sg_res = None, None
    if dist.is_initialized() and a.scaling == "strong":
        # the root-held exchange of scatter_gather_phase on a small array:
        # one grouped scatter of 10N+1 arrays, a copy standing in for the
        # kernels, one grouped gather into the root's preallocated output,
        # bounded by --sg-timeout exactly as on the GPU
        from amphora_amd.shard import RootScatterGather
        n, Ws = a.parties, 4099
        sg = RootScatterGather(Ws, 10 * a.parties + 1, 2)
        full_in = torch.randint(0, 256, (10 * n + 1, Ws, 16), dtype=torch.uint8,
                                generator=torch.Generator().manual_seed(5)) if rank == 0 else None
        full_out = torch.zeros((2, Ws, 16), dtype=torch.uint8) if rank == 0 else None
        try:
            local = sg.scatter(full_in, timeout=a.sg_timeout)
            out = sg.out_view(full_out)
            out[0].copy_(local[0])
            out[1].copy_(local[10 * n])
            if not maybe_inject(a.inject_sg_fault, rank, world):
                sg.gather(full_out, timeout=a.sg_timeout)
            guarded_all_reduce(dist, torch.zeros(1, dtype=torch.int32), dist.ReduceOp.MAX, a.sg_timeout)
            if rank == 0:
                sg_ok = bool(torch.equal(full_out[0], full_in[0]) and torch.equal(full_out[1], full_in[10 * n]))
        except Exception as e:  # noqa: BLE001 (same guard as scatter_gather_phase)
            sg_res = {"skipped": "scatter/gather aborted on rank %d: %s: %s" % (
                          rank, type(e).__name__, (str(e).splitlines() or [""])[0][:300]),
                      "aborted": True, "timeout_s": a.sg_timeout}
    # host_memory_phase's size decision (the probe, the per-node split, the
    # agreement over ranks), with nothing allocated
    hm_plan = None
    if not a.no_host_phase and not sg_res:
        try:
            if a.inject_sg_fault == "host-hang" and world > 1 and rank == 1:
                # a rank stuck before the agreement (as one the OOM killer is
                # about to take): it never joins; the others give up after
                # --host-timeout and the line still prints
                time.sleep(a.host_timeout + 2)
                raise TimeoutError("injected: rank 1 never joined the host phase")
            w, hm_plan = plan_host_words(a, dist, dist.is_initialized(), "cpu", a.host_timeout)
        except Exception as e:  # noqa: BLE001
            hm_plan = _host_abort(rank, "size agreement", e, a.host_timeout)
    aborted = bool(sg_res and sg_res.get("aborted")) or bool(hm_plan and hm_plan.get("aborted"))
    if rank == 0:
        emit({"metric": METRIC, "value": None, "unit": "words/s", "n_gpus": world, "dry_run": True,
              "host_memory_plan": hm_plan,
              "partial": [k for k, v in (("host_memory", hm_plan), ("scatter_gather", sg_res))
                          if v and v.get("aborted")] or None,
              "scatter_gather_round_trip": sg_ok, "scatter_gather": sg_res,
              "per_rank": ranks, "ranks_summary": ranks_summary(ranks, world),
              "world_size": world, "backend": dist.get_backend() if dist.is_initialized() else None,
              "scaling": a.scaling, "steps": a.steps, "warmup": a.warmup,
              "words_covered": covered, "fault_reported_at": int(verdicts[-1, 1].item()),
              "fault_expected_at": shard_range(total, world - 1, world)[0] + count // 3
              if a.scaling == "strong" else (world - 1) * a.words + count // 3,
              "config": workload_config(a, world)})
    finish_pg(dist, aborted)
    return aborted


def pg_timeout(a):
    import datetime
    return datetime.timedelta(seconds=a.pg_timeout)


def finish_pg(dist, aborted):
    """Normal end: barrier + destroy.  After an abandoned scatter/gather the
    communicator may hold operations a peer never matched: abort it (RCCL:
    ncclCommAbort, which also ends the stuck kernels) and skip the barrier
    and destroy, which would block or raise."""
    if not dist.is_initialized():
        return
    if not aborted:
        dist.barrier()
        dist.destroy_process_group()  # every collective is done: the other ranks may exit
        return
    try:
        from torch.distributed.distributed_c10d import _abort_process_group
        _abort_process_group()
    except Exception as e:  # noqa: BLE001 (gloo has no abort; the process ends right after)
        print("bench.py: process-group abort: %s: %s" % (type(e).__name__, e), file=sys.stderr)


def exit_after_abort(code):
    """After an aborted communicator, end the process without running the
    process group's destructors (they may wait on the abandoned operations).
    This is a plain exit of this process, nothing is exec'd."""
    sys.stderr.flush()
    os._exit(code)


def _dpm_current(path):
    """Current level of a pp_dpm_* file ("1: 2400Mhz *") in MHz, or None."""
    try:
        with open(path) as fh:
            for ln in fh:
                if ln.rstrip().endswith("*"):
                    v = ln.split(":", 1)[1].strip().rstrip("*").strip().lower()
                    return float(v.replace("mhz", "").strip())
    except (OSError, ValueError, IndexError):
        pass
    return None


def box_state(bus):
    """One reading of the GPU's clocks, power and temperatures from sysfs
    (no driver calls; safe beside running kernels): pp_dpm_{sclk,mclk,fclk}
    current levels, and the hwmon freq*/power*/temp* inputs by label.  Units:
    MHz, W, degrees C.  {} when the device has no such files."""
    import glob
    out = {}
    if not bus:
        return out
    dev = "/sys/bus/pci/devices/%s" % bus
    for k in ("sclk", "mclk", "fclk", "socclk"):
        v = _dpm_current("%s/pp_dpm_%s" % (dev, k))
        if v is not None:
            out["dpm_%s_mhz" % k] = v
    for hw in sorted(glob.glob(dev + "/hwmon/hwmon*")):
        for f in sorted(glob.glob(hw + "/*_input")) + sorted(glob.glob(hw + "/power*_cap")) + \
                sorted(glob.glob(hw + "/power*_average")):
            name = os.path.basename(f)
            kind = name.split("_", 1)[0]
            base = kind.rstrip("0123456789")
            if base not in ("freq", "power", "temp"):
                continue
            try:
                raw = int(open(f).read().strip())
            except (OSError, ValueError):
                continue
            label = kind
            try:
                label = open("%s/%s_label" % (hw, kind)).read().strip().replace(" ", "_") or kind
            except OSError:
                pass
            suffix = name[len(kind) + 1:]
            if base == "freq":
                out["%s_mhz" % label] = raw / 1e6
            elif base == "power":
                out["%s_%s_w" % (label, suffix)] = raw / 1e6
            else:
                out["%s_c" % label] = raw / 1e3
    return out


class BoxSampler:
    """Samples box_state() every `period` seconds on a thread while the timed
    region runs (the reads are sysfs files: the launch loop is not
    perturbed).  record() gives the readings before and after and, per
    field, the min / mean / max over the samples taken in between."""

    def __init__(self, bus, period=0.05):
        import threading
        self.bus, self.period = bus, period
        self.samples = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self.before = self.after = None

    def _run(self):
        while not self._stop.wait(self.period):
            self.samples.append(box_state(self.bus))

    def start(self):
        self.before = box_state(self.bus)
        if self.before:
            self._t.start()
        return self

    def stop(self):
        self._stop.set()
        if self._t.is_alive():
            self._t.join()
        self.after = box_state(self.bus)
        return self

    def record(self):
        if not self.before:
            return {"available": False, "note": "no pp_dpm_* / hwmon files for %s" % self.bus}
        during = {}
        for k in sorted({k for s in self.samples for k in s}):
            v = [s[k] for s in self.samples if k in s]
            during[k] = {"min": min(v), "mean": round(sum(v) / len(v), 3), "max": max(v)}
        return {"available": True, "before": self.before, "after": self.after, "during": during,
                "samples": len(self.samples), "period_s": self.period,
                "source": "/sys/bus/pci/devices/%s (pp_dpm_*, hwmon)" % self.bus}


def gpu_identity(torch, local):
    """(PCI address, UUID) of the GPU this rank drives; (None, None) without one."""
    if not torch.cuda.is_available():  # (--dry-run on a host without a GPU: no identity)
        return None, None
    p = torch.cuda.get_device_properties(local)
    return ("%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id),
            str(getattr(p, "uuid", "")))


def board_identity(bus):
    """What tells two boards apart when their PCI addresses agree (every
    1-GPU lease shows the same address): the host name and the board's own
    sysfs identity (unique_id / serial_number / vbios_version, when readable)."""
    import socket
    out = {"host": socket.gethostname()}
    for k in ("unique_id", "serial_number", "vbios_version", "product_name"):
        try:
            v = open("/sys/bus/pci/devices/%s/%s" % (bus, k)).read().strip()
            if v:
                out[k] = v
        except (OSError, TypeError):
            pass
    return out


def rank_record(torch, rank, local, wall_s, k_mask_ms, k_rv_ms, words):
    """This rank's identity (PCI address and UUID of the GPU it drove, the
    host and the board's sysfs identity) and its own device-resident timings."""
    bus, uuid = gpu_identity(torch, local)
    return {"rank": rank, "board": board_identity(bus), "local_rank": local, "pci_bus_id": bus, "uuid": uuid, "words": words,
            "wall_s": wall_s, "k_mask_ms": round(k_mask_ms, 5), "k_rv_ms": round(k_rv_ms, 5)}


def ranks_summary(ranks, pg_world):
    """min / max over ranks of the kernel times, and whether every rank
    drove its own GPU."""
    out = {"pg_world_size": pg_world,
           "distinct_gpus": len({r["pci_bus_id"] for r in ranks if r["pci_bus_id"] is not None})}
    for k in ("k_mask_ms", "k_rv_ms", "wall_s"):
        v = [r[k] for r in ranks]
        out[k] = {"min": min(v), "max": max(v)}
    return out


def workload_config(a, world):
    W, n = a.words, a.parties
    if a.scaling == "strong":
        name = "C4" if (W, n) == WORKLOADS["c4"][:2] else "custom"
        return {"workload": "%s: K_MASK (share-encode) + K_RV (recombine+verify), %d words in total "
                            "split into %d contiguous device-resident shards, %d parties, "
                            "p = 2^127 < p < 2^128 test prime" % (name, W, world, n),
                "words_total": W, "words_per_gpu": -(-W // world), "parties": n,
                "parallelism": "dp%d" % world}
    return {"workload": "%s: K_MASK (share-encode) + K_RV (recombine+verify), "
                        "%d words per GPU, %d parties, p = 2^127 < p < 2^128 test prime"
                        % (config_name(W, n), W, n),
            "words_total": W * world, "words_per_gpu": W, "parties": n, "parallelism": "dp%d" % world}


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a))  # before anything initialises the GPU
    _claim_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if a.dry_run:
        if dry_run(a, world, rank):
            exit_after_abort(0)
        return
    import torch
    import torch.distributed as dist
    import amphora_amd as A
    from amphora_amd.spdz import TEST_PRIME, TEST_R, TEST_RINV

    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    distributed = world > 1 or a.dist
    if a.gpus != world and rank == 0:
        print("bench.py: --gpus %d but WORLD_SIZE=%d (measuring %d)" % (a.gpus, world, world),
              file=sys.stderr)
    if distributed:
        # an explicit timeout on every collective, and RCCL errors / timeouts
        # cleaned up (communicator aborted) without tearing the process down,
        # so a stuck phase cannot take the finished numbers with it
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout(a))
        else:
            dist.init_process_group(a.backend, timeout=pg_timeout(a))

    # the library measured is this tree's build (compiled-in id = digest of the
    # sources that travelled with it); refuse to measure anything else
    build = {"id": A._lib.build_id(), "tree": A._lib.tree_build_id()}
    build["match"] = build["id"] == build["tree"]
    if not build["match"]:
        sys.exit("bench.py: libamphora_hip.so build id %s != tree digest %s: rebuild first"
                 % (build["id"], build["tree"]))
    print("bench.py: libamphora_hip.so build id %s (= tree digest)" % build["id"], file=sys.stderr)
    ctx = A.Context(TEST_PRIME, TEST_R, TEST_RINV, device=local)
    if a.mode == "host":
        host_mode(a, A, torch, ctx, dist, rank, world)
        if distributed:
            dist.destroy_process_group()
        return
    from amphora_amd.shard import shard_range
    n = a.parties
    if a.scaling == "strong":  # C4: this rank's contiguous shard of the whole job
        start, W = shard_range(a.words, rank, world)
        total_words = a.words
    else:  # C2 / C3 / custom: W words on every rank
        start, W = rank * a.words, a.words
        total_words = a.words * world
    slab = (lambda: torch.empty((5, n, W + a.pad_words, 16), dtype=torch.uint8, device="cuda")) \
        if a.pad_words else (lambda: None)
    mask_odos, mbuf, mplain = ctx.synth_odos(seed=1000 + rank, n=n, words=W, with_plain=True, buf=slab())
    share_odos, sbuf, splain = ctx.synth_odos(seed=2000 + rank, n=n, words=W, with_plain=True, buf=slab())
    secrets = ctx.synth_words(seed=3000 + rank, count=W)
    torch.cuda.synchronize()

    # One first-fail word per launch per step: verdicts[s] = (K_MASK, K_RV) of
    # step s, set to the sentinel once up front; the kernels min-combine into
    # them (AMPH_F_ACCUMULATE), so a step costs exactly its two launches.  The
    # shards need no collective on the data path: the per-step GLOBAL verdicts
    # are one RCCL all_reduce(MIN) of this vector after the last step, inside
    # the timed region (batched verdict exchange -- a per-step 8-byte
    # all-reduce cost 32 us of a 105 us step even at world size 1).
    total = a.warmup + a.steps
    verdicts = torch.full((total, 2), NO_FAIL, dtype=torch.int64, device="cuda")
    flags = A._lib.AMPH_F_DEVICE | A._lib.AMPH_F_ACCUMULATE
    lib = A._lib
    mask_arr, mviews = ctx._odo_structs(mask_odos)
    share_arr, sviews = ctx._odo_structs(share_odos)
    masked = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
    ys = torch.empty((W, 16), dtype=torch.uint8, device="cuda")
    import ctypes as C
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    vptr = [(C.cast(C.c_void_p(verdicts[s].data_ptr()), C.POINTER(C.c_int64)),
             C.cast(C.c_void_p(verdicts[s].data_ptr() + 8), C.POINTER(C.c_int64)))
            for s in range(total)]
    step_no = [0]

    def step(ev_mask=None, ev_rv=None):
        # kernel timing: hipExtLaunchKernel stamps the events at each kernel's
        # own dispatch start/end (amph_time_next_launch), on the launch stream
        ff0, ff1 = vptr[step_no[0]]
        rec = a.event_mode == "record"
        if ev_mask is not None:
            if rec:
                lib.lib.amph_timing_event_record(ev_mask[0].handle, stream)
            else:
                lib.lib.amph_time_next_launch(ev_mask[0].handle, ev_mask[1].handle)
        st = lib.lib.amph_mask_input(ctx._h, mask_arr, n, secrets.data_ptr(), W, masked.data_ptr(),
                                     ff0, flags, stream)
        assert st == 0
        if ev_mask is not None and rec:
            lib.lib.amph_timing_event_record(ev_mask[1].handle, stream)
        if ev_rv is not None:
            if rec:
                lib.lib.amph_timing_event_record(ev_rv[0].handle, stream)
            else:
                lib.lib.amph_time_next_launch(ev_rv[0].handle, ev_rv[1].handle)
        st = lib.lib.amph_recombine_verify(ctx._h, share_arr, n, ys.data_ptr(), ff1, flags, stream)
        assert st == 0
        if ev_rv is not None and rec:
            lib.lib.amph_timing_event_record(ev_rv[1].handle, stream)
        step_no[0] += 1

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # Sampled kernel timing: `samples` launches of each kernel get timing-only
    # events (no system-scope fence on record), K_MASK and K_RV stamped in
    # different steps spread evenly over the timed region.  A stamped launch
    # still costs ~3-4 us of dispatch; over the default 1000 steps that is
    # ~0.06 us per step.
    ns = max(1, min(a.samples, a.steps // 2 if a.steps >= 2 else 1))
    mask_at = {int((j + 0.25) * a.steps / ns): j for j in range(ns)}
    rv_at = {int((j + 0.75) * a.steps / ns): j for j in range(ns)}
    ev_mask = [(lib.TimingEvent(), lib.TimingEvent()) for _ in range(ns)]
    ev_rv = [(lib.TimingEvent(), lib.TimingEvent()) for _ in range(ns)]
    sampler = BoxSampler(gpu_identity(torch, local)[0])
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    sampler.start()
    t0 = time.perf_counter()
    for s in range(a.steps):
        jm, jr = mask_at.get(s), rv_at.get(s)
        step(ev_mask[jm] if jm is not None else None, ev_rv[jr] if jr is not None else None)
    if distributed:
        if start:  # local first-fail indices -> global word indices
            verdicts = torch.where(verdicts == NO_FAIL, verdicts, verdicts + start)
        dist.all_reduce(verdicts, op=dist.ReduceOp.MIN)  # per-step global verdicts
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    el = time.perf_counter() - t0
    sampler.stop()
    d_mask = sorted(e0.elapsed_ms(e1) for e0, e1 in ev_mask)
    d_rv = sorted(e0.elapsed_ms(e1) for e0, e1 in ev_rv)
    t_mask = sum(d_mask) / ns  # ms per launch (mean: the roofline's figure)
    t_rv = sum(d_rv) / ns
    med = {"k_mask": d_mask[ns // 2], "k_rv": d_rv[ns // 2]}  # (median of >= 10)
    # which physical GPU this rank drove, and its own timings: every rank's
    # record reaches rank 0 (the reported times stay the max over ranks)
    mine = rank_record(torch, rank, local, el, t_mask, t_rv, W)
    # the box's clocks / power / temperatures around and during the timed
    # region: a slower kernel on an unchanged build is then silicon or power,
    # not code, when the clocks say so
    mine["box"] = sampler.record()
    ranks = [mine]
    if distributed:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        el = max(r["wall_s"] for r in ranks)
        t_mask = max(r["k_mask_ms"] for r in ranks)
        t_rv = max(r["k_rv_ms"] for r in ranks)
    ok = bool((verdicts == NO_FAIL).all().item())
    # After the timed region: the same access pattern as K_MASK with no
    # arithmetic (amph_stream_probe), stamped the same way -- what this
    # pattern achieves at this size on this GPU, beside the 8 TB/s spec peak.
    scratch_ff = torch.full((1,), NO_FAIL, dtype=torch.int64, device="cuda")
    ys2 = torch.empty_like(ys)

    def k_rv_launch():  # the launch that precedes every K_MASK in the timed steps
        assert lib.lib.amph_recombine_verify(
            ctx._h, share_arr, n, ys2.data_ptr(),
            C.cast(C.c_void_p(scratch_ff.data_ptr()), C.POINTER(C.c_int64)), flags, stream) == 0

    probe_ms = stream_probe_ms(lib, C, ctx, mask_arr, n, secrets, W, stream, ns, k_rv_launch)
    # After the timed region: the outputs themselves are checked, not only the
    # absence of a MAC failure (a kernel that flags nothing and writes wrong
    # words must not report verified).
    checks = check_outputs(ctx, lib, torch, C, stream, flags, n, W, secrets, masked, ys, mplain, splain,
                           share_arr, share_odos, TEST_PRIME)
    checks["honest_verdicts"] = ok
    if distributed:
        cv = torch.tensor([int(all(checks.values()))], dtype=torch.int64, device="cuda")
        dist.all_reduce(cv, op=dist.ReduceOp.MIN)
        checks["all_ranks"] = bool(cv.item())
    ok = all(checks.values())

    if rank == 0:
        ms = el * 1000.0 / a.steps
        value = total_words * a.steps / el
        kern = {"k_mask": t_mask, "k_rv": t_rv}
        dom = max(kern, key=kern.get)
        bpw = kbytes(dom, n)
        achieved = bpw * W / (kern[dom] * 1e-3) / 1e9
        traffic = None
        if os.path.exists(a.traffic_json):
            try:
                tj = json.load(open(a.traffic_json))
                key = "%s_n%d_w%d" % (dom, n, W)
                traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
            except (ValueError, OSError):
                traffic = None
        line = {
            "metric": METRIC, "value": value, "unit": "words/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True,
            "scaling": a.scaling, "vs_baseline": None, "dtype": "u128 mod-p (4x u32 limbs)",
            "data": "synthetic: device-generated honest %d-party ODOs + secrets (seeded)" % n,
            "config": workload_config(a, world),
            "layout": {"pad_words": a.pad_words, "field_stride_bytes": 16 * (W + a.pad_words),
                       "note": "each party's 5 ODO fields are rows of one slab (device-generated)"},
            "world_size": world,
            "backend": dist.get_backend() if distributed else None,
            "build": build,
            "verified": ok,
            "verify_checks": checks,
            "kernels_ms": {k: round(v, 5) for k, v in kern.items()},
            "kernels_ms_median": {k: round(v, 5) for k, v in med.items()},
            "kernel_timing": ("HIP events (hipEventDisableSystemFence) %s on the launch stream: "
                              "%d launches of each kernel spread over the %d timed steps"
                              % ("stamped by the kernel dispatch (hipExtLaunchKernel)"
                                 if a.event_mode == "launch" else
                                 "recorded right before and after the call (hipEventRecord)",
                                 ns, a.steps)),
            "kernels_gbs": {k: round(kbytes(k, n) * W / (v * 1e-3) / 1e9, 1) for k, v in kern.items()},
            # share-encode and recombine+verify rates separately
            # (per GPU, from the kernel timings); `value` is the round trip
            "kernels_words_per_s": {k: round(W / (v * 1e-3)) for k, v in kern.items()},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "bytes_per_word": bpw, "traffic": traffic},
            "pattern_probe": pattern_probe(probe_ms, n, W, kern),
            "per_rank": ranks,
            "ranks_summary": ranks_summary(ranks, dist.get_world_size() if distributed else 1),
            "host_memory": None,
            "scatter_gather": None,
            "cpu_baseline": None,
        }
    # The root-held C4 rate (RCCL scatter/gather over xGMI) in the same run,
    # once the device-resident arrays are gone.
    resident = total_words * a.steps / el
    del mask_odos, mbuf, mplain, share_odos, sbuf, splain, secrets, masked, ys, ys2
    del mviews, sviews, mask_arr, share_arr
    torch.cuda.empty_cache()
    # The PCIe-inclusive rate (C5's per-GPU share from page-locked host
    # memory), before the scatter/gather phase: nothing it measures depends
    # on a point-to-point exchange.
    hm = None
    if not a.no_host_phase:
        hm = host_memory_phase(a, torch, dist, ctx, rank, world, distributed)
        if rank == 0 and hm and "verified" in hm:
            ok = ok and hm["verified"]
    host_aborted = bool(hm and hm.get("aborted"))
    sg = None
    if distributed and a.scaling == "strong" and not a.no_scatter_gather and not host_aborted:
        sg = scatter_gather_phase(a, A, torch, dist, ctx, rank, world, resident)
        if rank == 0 and sg and "verified" in sg:
            ok = ok and sg["verified"]
    aborted = host_aborted or bool(sg and sg.get("aborted"))
    if distributed:
        if not aborted:  # a rank that saw a phase abort tells the others (ranks that finished it
            # wait here at most --sg-timeout, then abort too)
            flag = torch.zeros(1, dtype=torch.int32, device="cuda" if dist.get_backend() == "nccl" else "cpu")
            try:
                guarded_all_reduce(dist, flag, dist.ReduceOp.MAX, a.sg_timeout)
            except Exception:  # noqa: BLE001
                aborted = True
        finish_pg(dist, aborted)
    if rank == 0:
        line["verified"] = ok
        line["host_memory"] = hm if not a.no_host_phase else {"skipped": "--no-host-phase"}
        if aborted and sg is not None and "aborted" not in sg:
            sg = dict(sg, aborted_after=True)
        if sg is not None:
            line["scatter_gather"] = sg
        elif host_aborted and a.scaling == "strong" and not a.no_scatter_gather and distributed:
            line["scatter_gather"] = {"skipped": "not run: the host_memory phase aborted the process group"}
        elif a.scaling == "strong" and not a.no_scatter_gather:
            line["scatter_gather"] = {"skipped": "world size 1: the root's arrays are the only shard, "
                                                 "nothing crosses a link (device-resident value = "
                                                 "this point)"}
        # phases that were abandoned: `value` and `verified` stand for the
        # device-resident measurement; these sub-objects carry no number
        partial = [k for k in ("host_memory", "scatter_gather")
                   if isinstance(line.get(k), dict) and (line[k].get("aborted") or line[k].get("aborted_after"))]
        if aborted and not partial:
            partial = ["process group aborted after the phases"]
        line["partial"] = partial or None
        # the CPU baseline on rank 0 at EVERY world size, after the GPU work
        if not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(n, a.cpu_seconds)
        emit(line)
    if aborted:
        exit_after_abort(0 if ok else 1)
    if not ok:
        bad = (verdicts != NO_FAIL).any(dim=1).nonzero().flatten().tolist()
        sys.exit("verification failed: checks %r, MAC failures at steps %r" % (checks, bad[:10]))


if __name__ == "__main__":
    main()
