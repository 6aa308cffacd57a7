"""Multi-process (world_size 2, gloo on CPU) tests of the data-parallel path:
contiguous word shards, root scatter / gather of word arrays (RCCL over xGMI
on the GPU node, gloo here), and the min-combine of the verify verdict.
The per-shard arithmetic here is the C oracle (CPU); on the GPU node it is
the HIP kernels (bench.py)."""
import os
import socket

import numpy as np
import pytest

from amphora_amd.shard import (NO_FAILURE, combine_first_fail, gather_words, global_first_fail,
                               scatter_words, shard_range)


def test_shard_range_covers_exactly():
    for W in (0, 1, 7, 8, 1000, 1 << 20, 10007):
        for world in (1, 2, 3, 8):
            spans = [shard_range(W, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == W
            pos = 0
            for s, c in spans:
                if c:
                    assert s == pos
                pos += c


def test_global_first_fail():
    assert global_first_fail(-1, 100) == NO_FAILURE
    assert global_first_fail(NO_FAILURE, 100) == NO_FAILURE
    assert global_first_fail(5, 100) == 105


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, fault, result_dir):
    import torch
    import torch.distributed as dist
    from oracle import coracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F = coracle.test_field(threads=1)
    n = 2
    like = torch.empty((0, 16), dtype=torch.uint8)
    fields = []
    if rank == 0:
        odos, buf = F.synth_odos(seed=77, n=n, W=W, fault_index=fault)
        full = [torch.from_numpy(np.ascontiguousarray(buf[k, j])) for k in range(5) for j in range(n)]
    for idx in range(5 * n):
        fields.append(scatter_words(full[idx] if rank == 0 else None, W, 16, like=like))
    start, count = shard_range(W, rank, world)
    local = [tuple(fields[k * n + j].numpy() for k in range(5)) for j in range(n)]
    y, ff = F.recombine_verify(local) if count else (np.zeros((0, 16), np.uint8), -1)
    g = combine_first_fail(ff, start)
    yfull = gather_words(torch.from_numpy(y), W, 16)
    if rank == 0:
        ref_y, ref_ff = F.recombine_verify(odos)
        ok = g == ref_ff and np.array_equal(yfull.numpy(), ref_y)
        with open(os.path.join(result_dir, "ok"), "w") as f:
            f.write("%d %d %d" % (int(ok), g, ref_ff))
    dist.destroy_process_group()


@pytest.mark.parametrize("W,fault", [(10007, 7777), (10007, 3), (5, -1)])
def test_scatter_verify_gather_two_ranks(tmp_path, W, fault):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(2, _free_port(), W, fault, str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    ok, g, ref = open(tmp_path / "ok").read().split()
    assert ok == "1", (g, ref)
    assert int(g) == fault


@pytest.mark.parametrize("gpus,extra,scaling,words", [(2, [], "strong", 1 << 26),
                                                       (1, [], "strong", 1 << 26),
                                                       (2, ["--workload", "c2"], "weak", 2 << 20)])
def test_bench_spawns_ranks_itself(gpus, extra, scaling, words):
    """`bench.py --gpus 2` with no launcher starts torch.distributed.run as a
    child process (nothing touches a GPU first) and prints ONE JSON line from
    rank 0: n_gpus 2, the C4 workload (2^26 words split into two shards) by
    default, and the verdict all-reduce turns rank 1's local fault index into
    the global one; the grouped root scatter/gather round-trips its arrays.
    The driver's N = 1 default (`bench.py` alone) is the same C4 workload, so
    BENCH and SCALE measure one curve.  --dry-run: the plumbing without
    kernels."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    argv = [sys.executable, os.path.join(root, "bench.py"), "--dry-run"]
    if gpus > 1:
        argv += ["--gpus", str(gpus), "--backend", "gloo", "--same-device"]
    r = subprocess.run(argv + extra, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == gpus and line["world_size"] == gpus
    assert line["backend"] == ("gloo" if gpus > 1 else None)
    assert line["scaling"] == scaling and line["words_covered"] == words
    assert line["fault_reported_at"] == line["fault_expected_at"]
    assert line["config"]["workload"].startswith("C4" if scaling == "strong" else "C2")
    assert line["config"]["words_total"] == words
    assert line["scatter_gather_round_trip"] is (True if gpus > 1 and scaling == "strong" else None)
    # per-rank identity and timings reach rank 0 (SCALE lines are self-identifying)
    assert [r["rank"] for r in line["per_rank"]] == list(range(gpus))
    for r in line["per_rank"]:
        assert {"rank", "local_rank", "pci_bus_id", "uuid", "words", "wall_s", "k_mask_ms", "k_rv_ms"} <= set(r)
    assert sum(r["words"] for r in line["per_rank"]) == words
    summ = line["ranks_summary"]
    assert summ["pg_world_size"] == gpus
    for k in ("k_mask_ms", "k_rv_ms", "wall_s"):
        assert summ[k]["min"] <= summ[k]["max"]


@pytest.mark.parametrize("fault", ["error", "hang"])
def test_bench_line_survives_a_failed_scatter_gather(fault):
    """A point-to-point exchange that fails (rank 1 raises) or never completes
    (rank 1 never posts its gather sends, as a stuck RCCL peer would) is
    bounded by --sg-timeout: every rank abandons the phase, the communicator
    is aborted instead of torn down, and rank 0 still prints its ONE line,
    with the rest of the line intact and `scatter_gather.skipped` set."""
    import json
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    argv = [sys.executable, os.path.join(root, "bench.py"), "--dry-run", "--gpus", "2", "--backend", "gloo",
            "--same-device", "--inject-sg-fault", fault, "--sg-timeout", "5"]
    t0 = time.time()
    r = subprocess.run(argv, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    assert time.time() - t0 < 120
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    sg = line["scatter_gather"]
    assert sg["aborted"] is True and sg["skipped"].startswith("scatter/gather aborted on rank 0")
    assert line["scatter_gather_round_trip"] is None
    assert line["fault_reported_at"] == line["fault_expected_at"]
    assert len(line["per_rank"]) == 2 and line["words_covered"] == 1 << 26


def _sg_worker(rank, world, port, W, fault, result_dir):
    """Root holds the 10N+1 C4 input arrays ([mask ODO fields x parties,
    share ODO fields x parties, secrets]); one grouped scatter, per-shard
    K_MASK + K_RV arithmetic (the C oracle on CPU here, the HIP kernels in
    bench.py), one grouped gather of (masked, secrets) into the root's
    preallocated output -- twice, to show nothing is reallocated."""
    import torch
    import torch.distributed as dist
    from oracle import coracle
    from amphora_amd.shard import RootScatterGather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F = coracle.test_field(threads=1)
    n = 2
    sg = RootScatterGather(W, 10 * n + 1, 2)
    full_in = full_out = None
    if rank == 0:
        _, mbuf = F.synth_odos(seed=31, n=n, W=W)
        _, sbuf = F.synth_odos(seed=32, n=n, W=W, fault_index=fault)
        sec = F.synth_words(seed=33, count=W, mont=False)
        full_in = torch.empty((10 * n + 1, W, 16), dtype=torch.uint8)
        for k in range(5):
            for j in range(n):
                full_in[k * n + j] = torch.from_numpy(np.ascontiguousarray(mbuf[k, j]))
                full_in[5 * n + k * n + j] = torch.from_numpy(np.ascontiguousarray(sbuf[k, j]))
        full_in[10 * n] = torch.from_numpy(sec)
        full_out = torch.zeros((2, W, 16), dtype=torch.uint8)
    ptrs = set()
    for _ in range(2):
        local = sg.scatter(full_in)
        out = sg.out_view(full_out)
        ptrs.add((local.data_ptr(), out.data_ptr()))
        ff = [-1, -1]
        if sg.count:
            lnp = local.numpy()
            mo = [tuple(lnp[k * n + j] for k in range(5)) for j in range(n)]
            so = [tuple(lnp[5 * n + k * n + j] for k in range(5)) for j in range(n)]
            m, ff[0] = F.mask_input(np.ascontiguousarray(lnp[10 * n]), mo)
            y, ff[1] = F.recombine_verify(so)
            out[0].copy_(torch.from_numpy(m))
            out[1].copy_(torch.from_numpy(y))
        g = [combine_first_fail(f, sg.start) for f in ff]
        sg.gather(full_out)
    if rank == 0:
        fn = full_in.numpy()
        mo = [tuple(np.ascontiguousarray(fn[k * n + j]) for k in range(5)) for j in range(n)]
        so = [tuple(np.ascontiguousarray(fn[5 * n + k * n + j]) for k in range(5)) for j in range(n)]
        ref_m, ref_mf = F.mask_input(np.ascontiguousarray(fn[10 * n]), mo)
        ref_y, ref_yf = F.recombine_verify(so)
        ok = (np.array_equal(full_out[0].numpy(), ref_m) and np.array_equal(full_out[1].numpy(), ref_y)
              and g == [ref_mf, ref_yf] and len(ptrs) == 1)
        with open(os.path.join(result_dir, "ok"), "w") as f:
            f.write("%d %d %d" % (int(ok), g[1], sg.moved_bytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("W,fault", [(10007, 9001), (4096, -1), (1, -1)])
def test_root_scatter_gather_grouped_two_ranks(tmp_path, W, fault):
    """bench.py's root-held C4 exchange (RootScatterGather): gathered masked
    words and canonical secrets bit-exact with the oracle over the whole
    array, the verdict min-combined to the global index, no per-step
    buffers, and exactly rank 1's shard crossing the link each way."""
    import torch.multiprocessing as mp
    mp.start_processes(_sg_worker, args=(2, _free_port(), W, fault, str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    ok, g, moved = open(tmp_path / "ok").read().split()
    assert ok == "1"
    assert int(g) == fault
    assert int(moved) == (W - (W + 1) // 2) * 23 * 16  # rank 1's shard, 21 arrays out + 2 back


def _sg_skip_worker(rank, world, port, result_dir):
    import json
    import sys
    import types
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import amphora_amd as A
    a = types.SimpleNamespace(words=1 << 10, parties=2, sg_steps=1, sg_warmup=0)
    # no GPU here: every rank's device allocation fails, and the phase must
    # return "skipped" on every rank without posting a send or a receive
    res = bench.scatter_gather_phase(a, A, torch, dist, None, rank, world, 1.0)
    dist.barrier()  # every rank got here: nothing is left waiting in a point-to-point op
    with open(os.path.join(result_dir, "r%d" % rank), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def test_scatter_gather_phase_skips_together_when_setup_fails(tmp_path):
    """bench.py's root-held scatter/gather phase allocates everything first and
    the ranks agree (an all-reduce of a failure flag) before any grouped
    send/recv is posted: when a rank cannot set up, every rank skips the phase
    and the device-resident line still prints, instead of one rank waiting
    forever in a receive the root never posts."""
    import json
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.is_available():
        pytest.skip("needs a host without a GPU (the allocation failure is the trigger)")
    mp.start_processes(_sg_skip_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r0 = json.load(open(tmp_path / "r0"))
    r1 = json.load(open(tmp_path / "r1"))
    assert set(r0) == {"skipped"} and r0["skipped"].startswith("setup failed on rank 0: ")
    assert set(r1) == {"skipped"}


def _dry_line(extra, env_extra, gpus=2):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    argv = [sys.executable, os.path.join(root, "bench.py"), "--dry-run"]
    if gpus > 1:
        argv += ["--gpus", str(gpus), "--backend", "gloo", "--same-device"]
    r = subprocess.run(argv + extra, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_host_phase_sizes_itself_to_the_memory_limit():
    """host_memory_phase decides its per-rank size before allocating (VERDICT
    r5 item 1): half the smaller headroom (cgroup limit, MemAvailable),
    split over the node's ranks, in whole batches, agreed over ranks.  An
    injected limit that fits two 4 Mi-word batches per rank (3 parties, 2
    ranks) shrinks the 32 Mi-word request to 8 Mi; the line still prints."""
    per_word, fixed, batch = 80 * 3 + 64, 256 << 20, 4 << 20
    limit = 2 * 2 * (2 * batch * per_word + fixed) + batch * per_word  # < 3 batches per rank
    line = _dry_line([], {"AMPH_BENCH_MEM_LIMIT_BYTES": str(limit)})
    plan = line["host_memory_plan"]
    assert plan["source"]["limit"] == "env" and plan["mem_limit_bytes"] == limit
    assert plan["local_world_size"] == 2 and plan["host_bytes_per_word"] == per_word
    assert plan["host_words_requested"] == 32 << 20 and plan["host_words_chosen"] == 2 * batch
    assert "skipped" not in plan and plan["mem_available_bytes"] > 0
    assert line["fault_reported_at"] == line["fault_expected_at"]


def test_host_phase_skips_when_one_batch_does_not_fit():
    """With less headroom than one batch per rank the phase is skipped with
    the reason and the limits recorded; the rest of the line stands."""
    line = _dry_line([], {"AMPH_BENCH_MEM_LIMIT_BYTES": str(1 << 30)})
    plan = line["host_memory_plan"]
    assert plan["host_words_chosen"] == 0 and plan["skipped"].startswith("host memory: ")
    assert plan["budget_bytes_per_rank"] == (1 << 30) // 4
    assert line["scatter_gather_round_trip"] is True and len(line["per_rank"]) == 2
    # MemAvailable is the other source: the smaller headroom wins
    line = _dry_line([], {"AMPH_BENCH_MEM_AVAILABLE_BYTES": str(3 << 30)}, gpus=1)
    plan = line["host_memory_plan"]
    assert plan["source"]["available"] == "env" and plan["host_words_chosen"] == 4 << 20


def test_line_survives_a_rank_lost_before_the_host_phase():
    """A rank that never joins the host phase's size agreement (stuck, or
    about to be OOM-killed) costs the others --host-timeout, not the line:
    rank 0 prints it with host_memory aborted and `partial` naming it."""
    import time
    t0 = time.time()
    line = _dry_line(["--inject-sg-fault", "host-hang", "--host-timeout", "5", "--no-scatter-gather"], {})
    assert time.time() - t0 < 120
    plan = line["host_memory_plan"]
    assert plan["aborted"] is True and plan["skipped"].startswith("host phase aborted on rank 0")
    assert line["partial"] == ["host_memory"]
    assert line["fault_reported_at"] == line["fault_expected_at"] and len(line["per_rank"]) == 2
