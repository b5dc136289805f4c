#!/usr/bin/env python3
"""Benchmark of the MI355X alignment engine — BASELINE.json metric:
"GCUPS (DP cell updates/s) + achieved HBM GB/s, 32k x 32k DNA NW, 1/2/4/8 GPU".

Default workload (--workload headline): one step = the DP fill of a 32768 x 32768 DNA global
(Needleman-Wunsch) alignment, blast scores (+5/-4), gap 5, i.i.d. uniform synthetic sequences
(splitmix64 seeds 6/7), inputs resident in HBM, direction matrix written to HBM — the reference's
throughput convention (tests/benchmarks.cu:102-187: fill + direction matrix, no traceback; our
traceback is timed separately and reported as e2e). With --gpus N every rank aligns its own pair
(a single pair does not shard: replicas, weak scaling); value = all ranks' cells / max-over-ranks time.

--workload batch: BASELINE.json config 5 — 4096 independent 2048 x 2048 DNA global pairs sharded
pair i -> rank i mod N, one fill + traceback per step per rank, scores gathered to rank 0 over
RCCL (torch.distributed 'nccl'); strong scaling.

Prints ONE JSON line on rank 0. `--gpus N` (N > 1) launched without WORLD_SIZE starts its N ranks
itself (torch.distributed.run, one process per GPU, before this process touches a GPU); launched by
torch.distributed.run, WORLD_SIZE must equal N. `--dry-run` exercises the rank plumbing only (gloo,
no GPU work, value null): the CPU test of the launcher.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sequence-alignment-gpu_amd", "python"))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)

# BASELINE.json's metric for the headline; the other workloads are its configs 2-5, labelled as such
METRICS = {
    "headline": "GCUPS (DP cell updates/s) + achieved HBM GB/s, 32k x 32k DNA NW",
    "local": "GCUPS (DP cell updates/s) + achieved HBM GB/s, 32k x 32k DNA SW (config 3)",
    "batch": "GCUPS (DP cell updates/s), 4096 x 2048^2 DNA NW batch, fill + traceback (config 5)",
    "dna8k": "GCUPS (DP cell updates/s), 8k x 8k DNA NW (config 2)",
    "protein4k": "GCUPS (DP cell updates/s), 4k x 4k protein NW, BLOSUM50 (config 4)",
}
_DNA = "synthetic (splitmix64 i.i.d. DNA, blast +5/-4, gap 5)"
DATA = {"headline": _DNA, "local": _DNA, "batch": _DNA, "dna8k": _DNA,
        "protein4k": "synthetic (splitmix64 i.i.d. protein, letters 0..19 of the 23-letter alphabet, BLOSUM50, gap 5)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["headline", "local", "batch", "dna8k", "protein4k"], default="headline")
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--pattern-len", type=int, default=0, help="headline/local: rows (default: --size)")
    ap.add_argument("--rows-per-lane", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=0, help="rows of the CPU baseline sample (default: full)")
    ap.add_argument("--batch-pipeline", type=int, default=1,
                    help="batch: overlap step k's traceback and result gather with step k+1's fill (two plan copies)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="batch, one GPU: run rank 0's shard of an N-rank deal (pairs i = 0 mod N) with the step "
                         "structure of an N-rank run (the strong-scaling curve, modelled per rank on one GPU)")
    ap.add_argument("--batch-chunks", type=int, default=1,
                    help="batch: plans per rank; chunk k's traceback overlaps chunk k+1's fill")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only (gloo, no GPU): launch / barrier / max-over-ranks / rank-0 line")
    ap.add_argument("--native", action="store_true",
                    help="batch: one process drives the C++ sa_align_batch over --gpus devices (host inputs, "
                         "per-device threads and plans, results gathered over RCCL); no torch.distributed")
    return ap.parse_args()


def _matrix_file(S: np.ndarray) -> str:
    """The score matrix as the reference's whitespace-separated text file (utilities.cpp:117-148)."""
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for row in np.asarray(S, dtype=np.int64):
            f.write(" ".join(str(int(v)) for v in row) + "\n")
        return f.name


def cpu_baseline(mode: str, n: int, rows: int, seeds=(6, 7), S=None, letters: int = 4,
                 label: str = "DNA blast") -> dict:
    """Single-core CPU fill on a bounded sample of the same workload, on this host. Prefers the
    reference's own CPU code (oracle/_ref/ref_align, built from /root/reference), else the oracle port."""
    from sa_amd import synthetic
    S = synthetic.blast_matrix() if S is None else np.asarray(S, dtype=np.int32)
    A = S.shape[0]
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_align")
    cells = rows * n
    if os.path.exists(ref):
        mat = _matrix_file(S)
        try:
            out = subprocess.run([ref, "fillbench", mode, str(rows + 1), str(n + 1), str(seeds[0]), str(seeds[1]),
                                  str(A), "5", mat, "1", str(letters)], capture_output=True, text=True, check=True,
                                 timeout=600)
            us = json.loads(out.stdout.strip().splitlines()[-1])["us"]
        finally:
            os.unlink(mat)
        kind = "reference"
    else:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        t = synthetic.random_sequence(seeds[0], n, letters)
        p = synthetic.random_sequence(seeds[1], rows, letters)
        M = np.empty((rows + 1) * (n + 1), np.uint8)
        t0 = time.perf_counter()
        oracle.fill_only(0 if mode == "global" else 1, t, p, S, 5, M)
        us = (time.perf_counter() - t0) * 1e6
        kind = "port"
    return {"value": round(cells / us / 1e3, 4), "unit": "GCUPS", "cores": 1, "kind": kind,
            "sample": f"{mode} fill {rows}x{n} {label} gap 5 (same synthetic stream), 1 thread, "
                      f"{us / 1e6:.2f} s"}


def cpu_baseline_cores(mode: str, n: int, rows: int, procs: int, seed0: int = 1000) -> dict | None:
    """All-cores CPU baseline for the batch: `procs` concurrent single-threaded fills of the
    reference's own CPU code (independent pairs, as the batch is), aggregate GCUPS. None when the
    reference build is absent."""
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_align")
    if not os.path.exists(ref):
        return None
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        f.write("5 -4 -4 -4\n-4 5 -4 -4\n-4 -4 5 -4\n-4 -4 -4 5\n")
        mat = f.name
    try:
        t0 = time.perf_counter()
        ps = [subprocess.Popen([ref, "fillbench", mode, str(rows + 1), str(n + 1), str(seed0 + 2 * k),
                                str(seed0 + 2 * k + 1), "4", "5", mat, "1"], stdout=subprocess.PIPE, text=True)
              for k in range(procs)]
        outs = [q.communicate(timeout=600)[0] for q in ps]
        wall = time.perf_counter() - t0
        if any(q.returncode != 0 for q in ps):
            return None
        us = [json.loads(o.strip().splitlines()[-1])["us"] for o in outs]
    finally:
        os.unlink(mat)
    cells = procs * rows * n
    return {"value": round(cells / max(us) / 1e3, 4), "unit": "GCUPS", "cores": procs, "kind": "reference",
            "sample": f"{procs} concurrent single-threaded {mode} fills of {rows}x{n} DNA blast gap 5 (distinct "
                      f"pairs of the batch's synthetic stream), slowest {max(us) / 1e6:.2f} s, wall {wall:.2f} s"}


def load_traffic(workload: str):
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(p):
        d = json.load(open(p))
        return d.get(workload)
    return None


class Chunked:
    """A rank's plans (one per chunk of its pairs). Fills run back to back on torch's current stream;
    with more than one chunk, chunk k's traceback runs on a second stream as soon as its fill is done,
    overlapping the next chunk's fill (the fill is HBM-bound, the traceback latency-bound)."""

    def __init__(self, jobs, torch, local):
        self.jobs, self.torch = jobs, torch
        self.s_fill = torch.cuda.current_stream(local)
        self.s_tb = torch.cuda.Stream(local) if len(jobs) > 1 else self.s_fill
        self.plan = jobs[0].plan

    def info(self) -> dict:
        infos = [j.plan.info() for j in self.jobs]
        return {"num_strips": sum(i["num_strips"] for i in infos), "rows_per_lane": infos[0]["rows_per_lane"],
                "device_bytes": sum(i["device_bytes"] for i in infos), "mask_bytes": sum(i["mask_bytes"] for i in infos)}

    def fill(self, ev=None) -> None:
        if ev is not None:
            ev[0].record(self.s_fill)
        for j in self.jobs:
            j.plan.fill(j.d_text.data_ptr(), j.d_pattern.data_ptr(), self.s_fill.cuda_stream)
        if ev is not None:
            ev[1].record(self.s_fill)

    def fill_and_traceback(self, ev=None) -> None:
        two = self.s_tb is not self.s_fill
        if ev is not None:
            ev[0].record(self.s_fill)
        for k, j in enumerate(self.jobs):
            j.plan.fill(j.d_text.data_ptr(), j.d_pattern.data_ptr(), self.s_fill.cuda_stream)
            if ev is not None and k == len(self.jobs) - 1:
                ev[1].record(self.s_fill)
            if two:
                self.s_tb.wait_stream(self.s_fill)
            j.plan.traceback(self.s_tb.cuda_stream)
        if two:
            self.s_fill.wait_stream(self.s_tb)

    def copy_results(self, buf, stream=None) -> None:
        """Every plan's sa_result array, device to device, into the rows of buf (a (k, 4) int64 tensor),
        on `stream` (default: the fill stream)."""
        row = 0
        st = (stream or self.s_fill).cuda_stream
        for j in self.jobs:
            j.plan.copy_results(buf.data_ptr() + 32 * row, st)
            row += j.plan.num_pairs

    def results(self) -> np.ndarray:
        """Every pair's sa_result (numpy structured array; one copy per plan, no per-pair objects).
        Raises if the fill aborted or any pair's status is not SA_OK."""
        res = np.concatenate([j.plan.results_array(self.s_fill.cuda_stream) for j in self.jobs])
        if len(res) and res["status"].any():
            bad = int(np.flatnonzero(res["status"])[0])
            raise RuntimeError(f"pair {bad} has status {int(res['status'][bad])}")
        return res


class Pipelined:
    """--workload batch, one rank: two copies of the rank's plans (the same pairs, each with its own
    direction planes) so that batch steps overlap two deep. Step k fills copy k % 2 on the fill stream
    once that copy's previous traceback (step k - 2) has read its planes; step k - 1's results come to
    the host while step k's fill runs; then step k's traceback goes on the traceback stream behind its
    fill. Every step still fills, traces back and returns all of its pairs (the VALU-bound fill and
    the gather-bound traceback share the CUs)."""

    def __init__(self, a: Chunked, b: Chunked, torch, local, gather=None):
        self.sets, self.torch = [a, b], torch
        self.s_fill = torch.cuda.current_stream(local)
        self.s_tb = torch.cuda.Stream(local)
        if os.environ.get("SA_BENCH_FILL_PRIO", "0") != "0":
            # experiment: the fill stream (encode + fill) at high priority, the traceback at normal
            self.s_fill = torch.cuda.Stream(local, priority=-1)
        self.fill_done = [torch.cuda.Event(), torch.cuda.Event()]
        self.tb_done = [torch.cuda.Event(), torch.cuda.Event()]
        self.k, self.pending = 0, None
        # N ranks: gather(chunked) moves the pending step's results to rank 0 (copy_results + RCCL
        # gather), issued on the traceback stream so it overlaps the next step's fill as well
        self.gather = gather

    def step(self, ev=None) -> None:
        i = self.k % 2
        jobs = self.sets[i].jobs
        if self.k >= 2:
            self.s_fill.wait_event(self.tb_done[i])
        if ev is not None:
            ev[0].record(self.s_fill)
        for j in jobs:
            j.plan.fill(j.d_text.data_ptr(), j.d_pattern.data_ptr(), self.s_fill.cuda_stream)
        if ev is not None:
            ev[1].record(self.s_fill)
        self.fill_done[i].record(self.s_fill)
        self.drain()
        self.s_tb.wait_event(self.fill_done[i])
        for j in jobs:
            j.plan.traceback(self.s_tb.cuda_stream)
        self.tb_done[i].record(self.s_tb)
        self.pending = i
        self.k += 1

    def drain(self) -> None:
        """The pending step's results to the host (waits for its traceback only)."""
        if self.pending is None:
            return
        if self.gather is not None:
            with self.torch.cuda.stream(self.s_tb):
                self.gather(self.sets[self.pending])
            self.pending = None
            return
        res = np.concatenate([j.plan.results_array(self.s_tb.cuda_stream) for j in self.sets[self.pending].jobs])
        if len(res) and res["status"].any():
            bad = int(np.flatnonzero(res["status"])[0])
            raise RuntimeError(f"pair {bad} has status {int(res['status'][bad])}")
        self.pending = None


def main_native(args) -> None:
    """--workload batch --native: each step is one sa_align_batch call (C ABI) aligning all 4096 pairs
    from host memory over devices 0..N-1 of this process: per device a thread that uploads its shard,
    builds a plan, fills and traces back; the results come back through the RCCL gather to device 0
    (sa_batch.hip). Plan setup and the PCIe copies are inside the step, so this is the C++ API's
    end-to-end rate, not the resident-input rate of the default batch line."""
    from sa_amd import engine, synthetic
    npairs, L = 4096, 2048
    S = synthetic.blast_matrix()
    texts = [synthetic.random_sequence(1000 + 2 * i, L, 4) for i in range(npairs)]
    pats = [synthetic.random_sequence(1001 + 2 * i, L, 4) for i in range(npairs)]
    for _ in range(args.warmup):
        engine.align_batch(0, texts, pats, S, 5, num_gpus=args.gpus, strings=False)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = engine.align_batch(0, texts, pats, S, 5, num_gpus=args.gpus, strings=False)
    elapsed = time.perf_counter() - t0
    stats = engine.batch_last_stats()
    cells = npairs * L * L
    print(json.dumps({
        "metric": "GCUPS (DP cell updates/s), 4096 x 2048^2 DNA NW batch, C++ sa_align_batch end to end (config 5)",
        "value": round(cells * args.steps / elapsed / 1e9, 3), "unit": "GCUPS", "n_gpus": args.gpus,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32", "data": DATA["batch"],
        "config": {"workload": f"dna_global_batch_{npairs}x{L}x{L}_native", "pairs_total": npairs, "text_len": L,
                   "pattern_len": L, "score": "blast +5/-4", "gap": 5, "parallelism": f"pairs_sharded{args.gpus}",
                   "path": "sa_align_batch (host inputs, plan per call, RCCL gather of results)"},
        "batch_stats_last_step": stats,
        "sample_result": {"pair0_score": res[0]["score"]},
    }), flush=True)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> None:
    """One rank process per GPU through torch.distributed.run (127.0.0.1 rendezvous), started from
    this process before it has made any GPU call; exits with the launcher's status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    raise SystemExit(subprocess.call(cmd, env=env))


def main_dry_run(args) -> None:
    """--dry-run: the multi-rank plumbing of main() without the engine (gloo on the CPU)."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    for _ in range(args.warmup):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank == 0:
        print(json.dumps({"metric": METRICS[args.workload], "value": None, "unit": "GCUPS", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
                          "dry_run": True, "ranks_seen": world}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus > 1 and not args.native:
        launch_ranks(args.gpus)
    if ws is not None and int(ws) != args.gpus and not args.native:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop WORLD_SIZE")
    if args.dry_run:
        main_dry_run(args)
        return
    if args.native:
        if args.workload != "batch" or int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise SystemExit("--native: --workload batch in one process (it drives --gpus devices itself)")
        main_native(args)
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SA_BENCH_ONE_DEVICE=1 (tests on a one-GPU box): every rank on device 0 and the gloo backend (RCCL
    # needs a device per rank), so the N-rank step, its pipelining and its result gather run for real
    one_device = world > 1 and os.environ.get("SA_BENCH_ONE_DEVICE") == "1"
    if one_device:
        local = 0
    if world > 1:
        if one_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    from sa_amd import distributed, synthetic
    from sa_amd.batch import DeviceBatch

    S = synthetic.blast_matrix()
    gap = 5
    npairs = 1
    if args.workload in ("dna8k", "protein4k"):
        # BASELINE.json configs 2 and 4: DNA global 8192^2 (seeds 3/4) and protein global 4096^2 with
        # BLOSUM50 (letters uniform over the 20 standard residues), one pair per GPU (replicas)
        n = m = 8192 if args.workload == "dna8k" else 4096
        A = 4 if args.workload == "dna8k" else 20
        if A == 20:
            mats = json.load(open(os.path.join(ROOT, "tests", "golden", "matrices.json")))
            S = np.array(mats["blosum50"], dtype=np.int32).reshape(23, 23)
        t = synthetic.random_sequence(3 + 1000 * rank, n, A)
        p = synthetic.random_sequence(4 + 1000 * rank, m, A)
        job = DeviceBatch(0, S, gap, [t], [p], device=local, rows_per_lane=args.rows_per_lane,
                          alphabet=None if A == 4 else b"ARNDCQEGHILKMFPSTWYVBZX-")
        cells_rank = n * m
        pairs_rank = 1
        workload = {"workload": f"{'dna' if A == 4 else 'protein'}_global_{n}x{m}", "pairs_per_gpu": 1,
                    "text_len": n, "pattern_len": m, "score": "blast +5/-4" if A == 4 else "blosum50",
                    "gap": gap, "parallelism": f"replicas{world}"}
    elif args.workload in ("headline", "local"):
        n = m = args.size
        m = args.pattern_len or n
        mode = 0 if args.workload == "headline" else 1
        t = synthetic.random_sequence(6 + 1000 * rank, n, 4)
        p = synthetic.random_sequence(7 + 1000 * rank, m, 4)
        job = DeviceBatch(mode, S, gap, [t], [p], device=local, rows_per_lane=args.rows_per_lane)
        cells_rank = n * m
        pairs_rank = 1
        workload = {"workload": ("dna_global" if mode == 0 else "dna_local") + f"_{n}x{m}", "pairs_per_gpu": 1,
                    "text_len": n, "pattern_len": m, "score": "blast +5/-4", "gap": gap,
                    "parallelism": f"replicas{world}"}
    else:
        npairs, L = 4096, 2048
        if args.shard_of > 1 and world > 1:
            raise SystemExit("--shard-of models one rank of an N-rank run on one GPU: run it with --gpus 1")
        # --shard-of N: rank 0's shard of an N-rank deal, on this one GPU (the per-rank step of the
        # strong-scaling curve; the RCCL gather of an N-rank run is not in it)
        deal = args.shard_of if args.shard_of > 1 else world
        mine = distributed.shard(npairs, deal, rank)
        texts = [synthetic.random_sequence(1000 + 2 * i, L, 4) for i in mine]
        pats = [synthetic.random_sequence(1001 + 2 * i, L, 4) for i in mine]
        # even chunk sizes (the pair-packed fill takes pairs two at a time)
        nch = max(1, min(args.batch_chunks, len(mine) // 2))
        cuts = [len(mine) * c // nch // 2 * 2 for c in range(nch)] + [len(mine)]
        chunks = [DeviceBatch(0, S, gap, texts[a:b], pats[a:b], device=local, rows_per_lane=args.rows_per_lane)
                  for a, b in zip(cuts, cuts[1:]) if b > a]
        job = Chunked(chunks, torch, local)
        # the rank's sa_result rows go device to device into this buffer and on to rank 0 (RCCL gather)
        gbuf = torch.full(((npairs + world - 1) // world, 4), -1, dtype=torch.int64, device=torch.device("cuda", local))

        def gather_pending(ch: Chunked) -> None:
            ch.copy_results(gbuf, torch.cuda.current_stream(local))
            distributed.gather_device(gbuf, npairs, world, rank)

        pipe = None
        if args.batch_pipeline and len(chunks) == 1:
            # the same two-deep step at every world size: N ranks gather the pending step's results
            # to rank 0 on the traceback stream, one rank brings them to its host
            twin = Chunked([DeviceBatch(0, S, gap, texts, pats, device=local, rows_per_lane=args.rows_per_lane)], torch, local)
            pipe = Pipelined(job, twin, torch, local, gather=gather_pending if world > 1 else None)
        cells_rank = len(mine) * L * L
        pairs_rank = len(mine)
        workload = {"workload": f"dna_global_batch_{npairs}x{L}x{L}", "pairs_total": npairs, "text_len": L,
                    "pattern_len": L, "score": "blast +5/-4", "gap": gap, "parallelism": f"pairs_sharded{world}",
                    "chunks_per_gpu": len(chunks),
                    "step_overlap": ("two-deep: step k's traceback and results overlap step k+1's fill "
                                     "(two plan copies)") if pipe is not None else "none"}
        if args.shard_of > 1:
            workload.update(workload=f"dna_global_batch_{npairs}x{L}x{L}_shard_of_{deal}", pairs_total=npairs,
                            parallelism=f"rank0_of_pairs_sharded{deal} (modelled on one GPU)")
    if not isinstance(job, Chunked):
        job = Chunked([job], torch, local)
    info = job.info()
    stream = torch.cuda.current_stream(local)

    dev = torch.device("cuda", local)

    def step(ev=None):
        # the fill launches (the dominant kernel) are bracketed by HIP events on the stream the engine
        # launches them on (torch's current stream); the rest of a batch step is timed only by the
        # wall clock
        if args.workload == "batch" and pipe is not None:
            pipe.step(ev)
        elif args.workload == "batch":
            # whole batch job per step: fill + traceback of this rank's pairs (chunk k's traceback on
            # a second stream, overlapping chunk k+1's fill), results to host, and the path's exchange
            # step — every rank's results gathered to rank 0 over RCCL (xGMI)
            job.fill_and_traceback(ev)
            if world > 1:
                # results device to device into the gather buffer, gathered to rank 0 over RCCL and
                # brought to rank 0's host there (no D2H -> H2D hop before the collective)
                job.copy_results(gbuf)
                distributed.gather_device(gbuf, npairs, world, rank)
            else:
                job.results()
        else:
            job.fill(ev)

    if args.workload != "batch":
        pipe = None
    for _ in range(args.warmup):
        step()
    if pipe is not None:
        pipe.drain()
    torch.cuda.synchronize(local)
    # a batch step builds 4096 result dicts on the host; the cyclic collector's periodic full passes
    # over the interpreter's objects (measured: one 38 ms pause every ~8 steps) are host noise, not
    # part of the job, so it is paused during the timed steps (the dicts are freed by refcount)
    gc.collect()
    gc.disable()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    if pipe is not None:
        pipe.drain()  # (the last step's traceback and results, inside the timed region)
    torch.cuda.synchronize(local)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gc.enable()
    launch_ms = [a.elapsed_time(b) for a, b in evs]
    res = job.results()  # checks the abort flag of the last fill

    # traceback / end-to-end, outside the timed region (headline: reported only); one untimed pass
    # first, so the traceback kernels' first launch in the process (code object load) is not timed
    if args.workload != "batch":
        job.fill_and_traceback()
    torch.cuda.synchronize(local)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    job.fill_and_traceback((e0, e1))
    e2.record(stream)
    res = job.results()
    # traceback: what runs after the last fill ends (with one chunk, the whole traceback)
    fill_ms_e2e, tb_ms = e0.elapsed_time(e1), e1.elapsed_time(e2)

    tmax = elapsed
    scores = [int(x) for x in res["score"]]
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if one_device else "cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tmax = float(tt.item())
        if args.workload == "batch":
            job.copy_results(gbuf)
            allres = distributed.gather_device(gbuf, npairs, world, rank)
            if rank == 0:
                scores = allres[:, 0].tolist()
    cells_total = cells_rank * world
    value = cells_total * args.steps / tmax / 1e9
    if rank == 0:
        avg_ms = float(np.mean(launch_ms))
        bytes_per_launch = float(cells_rank)  # algorithmic: 1 DIRECTION byte per cell
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        tr = load_traffic(workload["workload"])
        traffic = tr["bytes_per_launch"] if tr else None
        out = {
            "metric": METRICS[args.workload],
            "value": round(value, 3),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.workload != "batch" else "strong",
            "vs_baseline": None,
            # the pair-packed batch fill computes the int32 recurrence in u16 halves under a range guard
            # (bit-exact on every pair: DESIGN.md §3.1b); every other fill computes in int32
            "dtype": "u16x2 (int32 semantics)" if args.workload == "batch" and not os.environ.get("SA_NO_PAIR16")
            else "int32",
            "data": DATA[args.workload],
            "config": dict(workload, rows_per_lane=info["rows_per_lane"], strips_per_gpu=info["num_strips"]),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "traffic_note": (tr["source"] + "; physical HBM bytes per fill launch (direction bit-planes "
                                          "are 2 bits/cell, so traffic < algorithmic 1 B/cell)") if tr else None,
                         # what actually limits the kernel: HBM is the roofline the
                         # contract asks for, not the binding one
                         "limiter": ("VALU issue (pair-packed fill, ~82% of issue slots)" if args.workload == "batch"
                                     else "anti-diagonal dependency chain + strip hand-off latency, not HBM")},
            "fill_ms_per_launch": {"mean": round(avg_ms, 4), "min": round(min(launch_ms), 4),
                                   "median": round(float(np.median(launch_ms)), 4)},
            "gcups_best_launch": round(cells_rank / (min(launch_ms) * 1e-3) / 1e9 * world, 3),
            "gcups_reference_convention": round(pairs_rank * (workload["text_len"] + 1) * (workload["pattern_len"] + 1)
                                                / (min(launch_ms) * 1e-3) / 1e9 * world, 3),
            "e2e_ms": {"fill": round(fill_ms_e2e, 4), "traceback": round(tb_ms, 4)},
            # fill + traceback (strings included) of the same cells
            "gcups_fill_plus_traceback": round(cells_total / ((fill_ms_e2e + tb_ms) * 1e-3) / 1e9, 3)
            if fill_ms_e2e + tb_ms > 0 else None,
            "direction_bytes_physical_per_launch": info["mask_bytes"],
            "sample_result": {"pair0_score": scores[0] if scores else None, "pairs_per_gpu": pairs_rank},
        }
        if args.workload == "batch" and args.shard_of > 1:
            # one rank's step of an N-rank run, measured alone on one GPU: N ranks would finish the
            # 4096 pairs in about this step time (plus the 16-128 KiB RCCL gather, not measured here)
            out["shard_model"] = {"shard_of": args.shard_of, "pairs_this_rank": pairs_rank,
                                  "modelled_n_gpu_gcups": round(value * args.shard_of, 3),
                                  "note": "modelled, not measured on N GPUs: rank 0's shard on one GPU"}
        if world == 1 and not args.no_cpu_baseline:
            if args.workload == "batch":
                # the batch is independent pairs: the CPU baseline is every core of this GPU's host
                # share (OMP_NUM_THREADS, 16 on the GPU box) running the reference's fill at once, 64
                # pairs' worth of rows each; the single-core number is kept beside it
                procs = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
                single = cpu_baseline("global", 2048, args.cpu_rows or 2048 * 512, seeds=(1000, 1001))
                multi = cpu_baseline_cores("global", 2048, args.cpu_rows or 2048 * 64, procs)
                out["cpu_baseline"] = multi or single
                out["cpu_baseline_single_core"] = single
            elif args.workload == "dna8k":
                out["cpu_baseline"] = cpu_baseline("global", 8192, args.cpu_rows or 8192, seeds=(3, 4))
            elif args.workload == "protein4k":
                out["cpu_baseline"] = cpu_baseline("global", 4096, args.cpu_rows or 4096, seeds=(3, 4), S=S,
                                                   letters=20, label="protein BLOSUM50 (letters 0..19 of 23)")
            else:
                out["cpu_baseline"] = cpu_baseline("global" if args.workload == "headline" else "local",
                                                   args.size, args.cpu_rows or args.size)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
