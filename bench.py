#!/usr/bin/env python3
"""Headline benchmark: k=19 k-mer counting of the E. coli-sized pair at ART 30x (BASELINE.json
configs[1], "C2") on MI355X, plus the categorization SDK lookup of Nanosim-H-like 75x long
reads against the C2 export at [10,25] (configs[2], "C3"), with the CPU oracle timed beside it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--no-lookup]

A step is one pass of the counting hot path over the resident reads: bin + per-file count +
merge (hga_count_run), the specificity histogram (hga_count_spec_hist) and the sorted export
selection at [10,25] (hga_count_select_device) — everything jf_occurrences does on the device.
Inputs are resident in HBM before the timed region.  N > 1 (torchrun, one rank per GPU, RCCL):
every rank holds its own C2-sized shard of reads (weak scaling) and a step is the distributed
count of DESIGN.md §6 — local count, owner partition, all-to-all of the rows over xGMI, owner
merge + `--bc` drop, histogram reduction, per-owner export selection (hga_count_exchange in the
C ABI over the library's RCCL communicator, set up by hga_dist.OwnerExchange);
barrier + max-over-ranks timing.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "hybrid-genome-assembler_amd")]
import hga  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
K = 19
LA, LB = 4_641_652, 5_065_741  # MG1655, UTI89 lengths
DIV = 0.021
READ_LEN = 150
COVERAGE = 30
LOWER, UPPER = 10, 25
THRESHOLDS = [70.0, 85.0, 90.0, 95.0, 99.0, 100.0, 100.01]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_c2(rank):
    """Rank r's shard: its own MG1655/UTI89-sized pair at 30x (rank 0 = the N=1 workload), so the
    global genome grows with N at constant coverage (weak scaling, like SURVEY.md's C4)."""
    ga = hga.gen_genome(LA, 1 + 1000 * rank)
    gb = hga.gen_haplotype(ga, DIV, LB - LA, 2 + 1000 * rank)
    na, nb = COVERAGE * LA // READ_LEN, COVERAGE * LB // READ_LEN
    ra = hga.gen_art(ga, na, READ_LEN, 1000 + 2 * rank)
    rb = hga.gen_art(gb, nb, READ_LEN, 1001 + 2 * rank)
    return ga, gb, ra, rb


def make_c3(ga, gb, rank):
    na, nb = round(LA / 7777 * 75), round(LB / 7777 * 75)
    ra = hga.gen_nanosim(ga, na, 3000 + 2 * rank)
    rb = hga.gen_nanosim(gb, nb, 3001 + 2 * rank)
    bases = ra.bases + rb.bases
    offsets = np.concatenate([ra.offsets, rb.offsets[1:] + ra.offsets[-1]]).astype(np.uint64)
    return bases, offsets


PMC_KERNEL = {"kc_count": "kc_count_s"}   # profiler label -> device kernel of the default build


def pmc_traffic(kernel):
    """HBM bytes per launch measured by a separate rocprofv3 --pmc pass (profiles/), if any."""
    p = os.path.join(ROOT, "profiles", f"pmc_{PMC_KERNEL.get(kernel, kernel)}.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def spawn_ranks(n):
    """`--gpus N` (N > 1) started without torchrun: run N rank processes of this same command
    (torch.distributed.run, one node, 127.0.0.1) as a child and return its exit code.  Called before
    anything touches the GPU; the parent only waits."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    log(f"bench: --gpus {n} without WORLD_SIZE: starting {n} ranks (torch.distributed.run)")
    return subprocess.call(cmd, env=dict(os.environ, HGA_BENCH_SPAWNED="1"))


class Dist:
    def __init__(self, n):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if n != self.world:   # the ranks that exist must be the ranks asked for
            log(f"error: --gpus {n} but WORLD_SIZE={self.world} ranks")
            sys.exit(2)
        # HGA_BENCH_BACKEND=gloo rehearses the N>1 path on a box with fewer GPUs than ranks (the
        # library's host transport); nccl = RCCL, one rank per GPU
        backend = os.environ.get("HGA_BENCH_BACKEND", "nccl")
        self.backend = backend
        # HGA_BENCH_FORCE_DIST=1 (under torchrun): the N>1 code path at one rank — the library's
        # RCCL communicator, the exchange and the global queries — on a one-GPU box
        if self.world > 1 or os.environ.get("HGA_BENCH_FORCE_DIST") == "1":
            import torch
            import torch.distributed as dist
            dry = os.environ.get("HGA_BENCH_DRYRUN") == "1"   # launcher test: no GPU call at all
            if backend == "nccl" and not dry:
                nd = torch.cuda.device_count()   # does not initialise the GPU
                if nd < self.world:
                    log(f"error: {self.world} RCCL ranks need {self.world} GPUs, {nd} visible "
                        "(HGA_BENCH_BACKEND=gloo shares GPUs)")
                    sys.exit(2)
            elif not dry:
                self.local %= max(1, torch.cuda.device_count())
            if not dry:
                torch.cuda.set_device(self.local)
            # the communication libraries may print to fd 1; stdout must carry only the JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                if backend == "nccl":
                    dist.init_process_group("nccl", device_id=torch.device(f"cuda:{self.local}"))
                else:
                    dist.init_process_group(backend)
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.comm_dev = f"cuda:{self.local}" if backend == "nccl" else "cpu"
            self.torch, self.dist = torch, dist
            self.pg = True

    def barrier(self):
        if self.pg:
            self.torch.cuda.synchronize()
            self.dist.barrier()

    def max(self, v):
        if not self.pg:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.comm_dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if not self.pg:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.comm_dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.pg:
            self.dist.destroy_process_group()


def count_step(ctx):
    ctx.count_run(2)
    ctx.spec_hist(THRESHOLDS)
    return ctx.select_device(LOWER, UPPER)


def dist_count_step(ex):
    ex.count(2)
    ex.spec_hist(THRESHOLDS)
    return ex.select_counts(LOWER, UPPER)


KERNEL_BYTES = {
    # algorithmic bytes per step, from the per-unit figures in DESIGN.md §4
    "kc_bin1": lambda s: 1.0 * s["bytes"] + 4 * s["instances"],   # ASCII bases read (packed in LDS), 4 B/instance written
    "kc_rebin": lambda s: 8 * s["instances"],                          # 4 B/instance read + 4 B written
    "kc_count": lambda s: 4 * s["instances"] + (8 + 4 * s["files"]) * s["rows"],   # read binned, write rows
}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(ra, rb, threads, parse_s=None):
    """The oracle (C++ restatement of the count stage) timed on this box's host cores
    (BASELINE.md §3): per-file exact counts + --bc drop + merge + specificity + select.
      value          the whole C2 workload, `threads` threads (the box's CPU share), no parsing;
      with_parsing   the same plus the FASTQ parse of the C2 pair at the same thread count (ingest leg);
      one_core       1/16 of each file, 1 thread;
      reference_like 1/64 of file A, 1 thread, the reference's map-based KmerIterator loop
                     (KmerIterator.cpp:7-19,54-63) into a std::unordered_map."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    streams = [ra.seq, rb.seq]
    inst = sum(oracle.count_instances(s, K) for s in streams)

    def stage(ss, th):
        t0 = time.perf_counter()
        keys, counts = oracle.count_files_mt(ss, K, 2, th)
        oracle.specificity(counts, THRESHOLDS)
        oracle.select(keys, counts, LOWER, UPPER)
        return time.perf_counter() - t0

    dt = stage(streams, threads)
    # every host core this process may run on (BASELINE.md §3 "all host cores"; nproc counts the whole
    # host, the affinity mask what the box gives this process)
    n_all = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    dt_all = stage(streams, n_all) if n_all != threads else dt
    sub16 = [s[: s.find(b"\n", len(s) // 16)] for s in streams]
    inst16 = sum(oracle.count_instances(s, K) for s in sub16)
    dt1 = stage(sub16, 1)
    sub64 = ra.seq[: ra.seq.find(b"\n", len(ra.seq) // 64)]
    inst64 = oracle.count_instances(sub64, K)
    t0 = time.perf_counter()
    oracle.count_reference_like(sub64, K, 2)
    dtr = time.perf_counter() - t0
    out = {"value": inst / dt, "unit": "k-mers/s", "cores": threads, "kind": "port",
           "sample": f"the whole C2 workload ({inst} 19-mer windows, 2 files), resident in host memory: oracle "
                     f"count stage (range-partitioned exact counts, sort + run-length, --bc drop, merge; "
                     f"{threads} threads) + specificity + select[10,25]",
           "seconds": round(dt, 3), "nproc": os.cpu_count(), "cpu_model": cpu_model(),
           "threads_note": "threads = the GPU box's CPU share for one GPU (16); all_cores = every CPU in this "
                           "process's affinity mask (nproc counts the whole host)",
           "all_cores": {"value": round(inst / dt_all, 1), "unit": "k-mers/s", "cores": n_all,
                         "sample": "the whole C2 workload, same stage", "seconds": round(dt_all, 3)},
           "one_core": {"value": round(inst16 / dt1, 1), "unit": "k-mers/s", "cores": 1,
                        "sample": f"first 1/16 of each C2 file ({inst16} windows), same stage", "seconds": round(dt1, 3)},
           "reference_like": {"value": round(inst64 / dtr, 1), "unit": "k-mers/s", "cores": 1,
                              "sample": f"first 1/64 of the MG1655-sized file ({inst64} windows): per read the "
                                        "reference's KmerIterator loop with its unordered_map<char,Kmer> base maps, "
                                        "counted in a std::unordered_map, --bc drop, sorted dump",
                              "seconds": round(dtr, 3)}}
    if parse_s:
        out["with_parsing"] = {"value": round(inst / (dt + parse_s), 1), "unit": "k-mers/s", "cores": threads,
                               "parse_seconds": round(parse_s, 3),
                               "sample": "FASTQ parse of the C2 pair (host reader, same threads) + the count stage"}
    return out


def cpu_lookup_baseline(bases, offsets, sdk, threads):
    """construct_indices (ReadClusteringEngine.cpp:234-299) restated (oracle, all 9 outputs) on a
    bounded sample of the C3 reads: `threads` threads and 1 thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    out = {"unit": "reads/s", "kind": "port", "nproc": os.cpu_count(), "cpu_model": cpu_model()}
    for label, n_r, th in (("all", 24000, threads), ("one_core", 2000, 1)):
        n = min(len(offsets) - 1, n_r)
        sub_off = offsets[: n + 1]
        sub = bases[: int(sub_off[-1])]
        w = int(sum(max(int(l) - K + 1, 0) for l in np.diff(sub_off)))
        t0 = time.perf_counter()
        oracle.construct_indices(sub, sub_off, K, sdk, 1, threads=th)
        dt = time.perf_counter() - t0
        rec = {"value": round(n / dt, 1), "windows_per_s": round(w / dt, 1), "cores": th,
               "sample": f"first {n} C3 reads ({w} windows), oracle construct_indices (9 CSR outputs), {th} threads",
               "seconds": round(dt, 3)}
        if label == "all":
            out.update(rec)
        else:
            out["one_core"] = rec
    return out


def connections_leg(ctx2, D, reps, args):
    """get_all_connections(1) (ReadClusteringEngine.cpp:335-339, the default first clustering
    stage, :754) on the C3 indices left on the device by the lookup."""
    ctx2.connections_run(min_score=1)
    ctx2.profile(True)
    ctx2.profile_reset()
    for _ in range(reps):
        ctx2.connections_run(min_score=1)
    kern = {}
    for name in ("cn_wave", "cn_local", "cn_global", "cn_sort", "radix_upsweep", "radix_downsweep", "scan"):
        ms, n = ctx2.profile_get(name)
        if n:
            kern[name] = round(ms / reps, 4)
    ctx2.profile(False)
    D.barrier()
    ctx2.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        n_conn = ctx2.connections_run(min_score=1)
    ctx2.sync()
    D.barrier()
    dt = D.max((time.perf_counter() - t0) / reps)
    idx = ctx2.lookup_fetch()
    lens = np.diff(idx["kci_ptr"]).astype(np.float64)
    pairs_walked = float((lens * lens).sum())    # (id, candidate) pairs over all pivots
    H = float(len(idx["sorted_kid"]))
    # per pivot hit: KmerID 4 B + kci_ptr pair 16 B; per walked pair: candidate 4 B; per kept pair 12 B
    cn_bytes = 20 * H + 4 * pairs_walked + 12 * n_conn
    cn_ms = kern.get("cn_wave", 0) + kern.get("cn_local", 0) + kern.get("cn_global", 0)
    out = {"call": "get_all_connections(min_score=1) on the C3 indices", "ms": round(dt * 1e3, 3),
           "connections": int(n_conn), "pairs_walked": int(pairs_walked),
           "pivots_per_s": round(D.sum(float(len(idx["hit_ptr"]) - 1)) / dt, 1), "kernels_ms": kern,
           "roofline": {"bound": "hbm", "kernel": "cn_wave+cn_local+cn_global", "model": "20 B per hit + 4 B per walked "
                        "(id, candidate) pair + 12 B per kept pair",
                        "achieved": round(cn_bytes / (cn_ms * 1e-3) / 1e9, 1) if cn_ms else None,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s"}}
    if not args.no_cpu and D.rank == 0 and D.world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        n_p = 2000
        piv = np.arange(1, n_p + 1, dtype=np.uint32)
        t0 = time.perf_counter()
        oracle.connections(idx, pivots=piv, min_score=1)
        dtc = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n_p / dtc, 1), "unit": "pivots/s", "cores": 1, "kind": "port",
                               "sample": f"first {n_p} C3 reads as pivots, oracle get_connections "
                                         "(unordered_map per pivot, 1 thread, like the reference's default -t 1)",
                               "seconds": round(dtc, 3)}
    return out


def hll_leg(ctx2, D, n_bases, bases, offsets, args):
    """HyperLogLog k sweep of jf_occurrences' automatic k selection (KmerAnalysis.cpp:26-56):
    registers for k = 11, 13, ..., 31 over the C3 reads already resident on the device."""
    ks = list(range(11, 33, 2))
    for kk in ks[:2]:
        ctx2.hll_registers(kk)
    ctx2.profile(True)
    ctx2.profile_reset()
    for kk in ks:
        ctx2.hll_registers(kk)
    scan_ms, _ = ctx2.profile_get("hll_scan")
    ctx2.profile(False)
    D.barrier()
    t0 = time.perf_counter()
    for kk in ks:
        ctx2.hll_registers(kk)
    D.barrier()
    dt = D.max(time.perf_counter() - t0)
    per_k = scan_ms / len(ks)
    win = sum(max(int(l) - 19 + 1, 0) for l in np.diff(offsets))   # windows at k = 19
    out = {"call": "hga_hll_registers(k, b=10) for k = 11..31 step 2 on the C3 reads",
           "ms_per_k": round(dt * 1e3 / len(ks), 3), "windows_per_s": round(D.sum(win) / (dt / len(ks)), 1),
           "kernel_ms_per_k": {"hll_scan": round(per_k, 4)},
           "roofline": {"bound": "hbm", "kernel": "hll_scan", "model": "0.5 B per base (packed codes + valid + "
                        "read-start bits)", "achieved": round(0.5 * n_bases / (per_k * 1e-3) / 1e9, 1) if per_k
                        else None, "peak": HBM_PEAK_GBS, "unit": "GB/s"}}
    if not args.no_cpu and D.rank == 0 and D.world == 1:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        n = min(len(offsets) - 1, 8000)
        sub_off = offsets[: n + 1]
        sub = bases[: int(sub_off[-1])]
        w = sum(max(int(l) - 19 + 1, 0) for l in np.diff(sub_off))
        t0 = time.perf_counter()
        oracle.hll_registers(sub, sub_off, 19)
        dtc = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(w / dtc, 1), "unit": "windows/s", "cores": 1, "kind": "port",
                               "sample": f"first {n} C3 reads at k=19, oracle HyperLogLog add (1 thread)",
                               "seconds": round(dtc, 3)}
    return out


def write_kmer_text(path, codes, k):
    """The export file format of jf_occurrences (one k-mer string a line, JellyfishOccurrenceReader.cpp:
    110-135): 2-bit codes, first base in the top bits, A0 C1 G2 T3."""
    codes = np.asarray(codes, dtype=np.uint64)
    shifts = (2 * np.arange(k - 1, -1, -1)).astype(np.uint64)
    txt = np.empty((len(codes), k + 1), dtype=np.uint8)
    txt[:, :k] = np.frombuffer(b"ACGT", dtype=np.uint8)[((codes[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.intp)]
    txt[:, k] = ord("\n")
    txt.tofile(path)


def parse_print_blocks(stdout):
    """print_components' blocks of a `categorization -d` run (ReadClusteringEngine.cpp:189-198):
    per block [(component id, per-category read counts)]."""
    blocks, cur = [], None
    for ln in stdout.splitlines():
        if ln.startswith("### Printing"):
            cur = []
        elif ln == "### ###":
            blocks.append(cur)
            cur = None
        elif cur is not None and ln.startswith("#") and " : " in ln:
            head = ln.split(" [", 1)[0]
            cid, counts = head.split(" : ")
            cur.append((int(cid[1:]), [int(v) for v in counts.split("/")]))
    return blocks


def categorization_pipeline_leg(paths, sdk, threads, d, label="C3"):
    """Verdict r04 item 7: the drop-in `categorization` CLI end to end on long reads (Nanosim-like FASTA,
    both haplotypes, -d) against a [10,25] export as a k-mer text file: its own per-stage "took" lines
    (src/common/Utils.h:17-35 timeMeasure: index construction and the first connection pass on the GPU,
    union-find, merging, tails, spectral clustering, enrichment on the host), its HGA_TIMING=1 phases
    (host work around the stages), and print_components' blocks under -d (ReadClusteringEngine.cpp:
    189-198): scaffold components, final components with their per-haplotype read counts and the purity
    (reads of each final component's majority haplotype / reads in final components) — next to the
    reference's published ENP75 run on an i5-8250U (writing/Evaluation.txt:75-82) as context only."""
    import re
    import subprocess
    cli = os.path.join(ROOT, "hybrid-genome-assembler_amd", "bin", "categorization")
    if not os.path.exists(cli):
        return None
    kpath = os.path.join(d, f"{K}-mers_{LOWER}_{UPPER}_100%.txt")
    write_kmer_text(kpath, sdk, K)
    t0 = time.perf_counter()
    r = subprocess.run([cli, *paths, "-k", kpath, "-d", "-o", os.path.join(d, "clusters"), "-t", str(threads)],
                       capture_output=True, text=True, cwd=d, timeout=900, env=dict(os.environ, HGA_TIMING="1"))
    wall = time.perf_counter() - t0
    stages = {}
    for line in r.stdout.splitlines():
        m = re.match(r"(.+) took (\d+)ms$", line.strip())
        if m:
            stages[m.group(1)] = stages.get(m.group(1), 0) + int(m.group(2))
    phases = {}
    for line in r.stderr.splitlines():   # "hga-timing <phase> <ms>" (HGA_TIMING=1)
        f = line.split()
        if len(f) == 3 and f[0] == "hga-timing":
            phases[f[1]] = float(f[2])
    exported = re.search(r"Exported (\d+) components", r.stdout)
    blocks = parse_print_blocks(r.stdout)
    final = blocks[-1] if blocks else []
    tot = sum(sum(c) for _, c in final)
    return {"argv": f"categorization {' '.join(os.path.basename(p) for p in paths)} -k {os.path.basename(kpath)} "
                    f"-d -t {threads}",
            "workload": label, "rc": r.returncode, "wall_s": round(wall, 3), "stages_ms": stages,
            "phases_ms": phases,
            "components": int(exported.group(1)) if exported else None,
            "scaffold_components": len(blocks[0]) if blocks else None,
            "final_components_reads_per_haplotype": [[cid, c] for cid, c in final],
            "purity": round(sum(max(c) for _, c in final) / tot, 4) if tot else None,
            "stderr_tail": r.stderr[-300:] if r.returncode else None,
            "published_reference_ENP75_ms": {"Index construction": 49225, "All connections": 4353,
                                             "Merging into scaffold c.": 8751, "Tail connections": 7281,
                                             "Spectral clustering": 183, "Merging scaffold c.": 1914,
                                             "Enrichment connections": 116, "Merging into core c.": 2634,
                                             "note": "writing/Evaluation.txt:75-82, Intel Core i5-8250U, the "
                                                     "reference's real ENP75 reads: context, not the same input"}}


def mosaic_haplotype(ga, seed, gap=40_000, period=600_000):
    """Haplotype B for the tails workload: the C2 derivation of A (d = DIV substitutions, no inserted
    blocks, so coordinates align) made identical to A over `gap`-base stretches every `period` bases.
    Those stretches hold no SDK, so each haplotype's long-read chain breaks into pieces and the union-find
    yields more than two scaffold components — the case where run_clustering computes tail connections,
    spectral clustering and the scaffold-component merge (ReadClusteringEngine.cpp:768-777), which the
    plain C3 pair (one unbroken chain per haplotype) never reaches."""
    gb = bytearray(hga.gen_haplotype(ga, DIV, 0, seed))
    for s0 in range(period // 2, len(ga), period):
        gb[s0:s0 + gap] = ga[s0:s0 + gap]
    return bytes(gb)


def tails_pipeline_leg(ga, dev, threads):
    """the categorization CLI on a C3-sized workload that reaches the tails and spectral
    stages (mosaic_haplotype): its SDKs counted on the GPU from ART-like 30x short reads of the pair and
    exported at [10, 25] as jf_occurrences does, long reads Nanosim-like at 75x (C3's generators)."""
    import shutil
    import tempfile
    gbm = mosaic_haplotype(ga, 77)
    ra = hga.gen_art(ga, COVERAGE * LA // READ_LEN, READ_LEN, 5000)
    rb = hga.gen_art(gbm, COVERAGE * len(gbm) // READ_LEN, READ_LEN, 5001)
    with hga.Ctx(dev) as c:
        c.count_begin(K, 2)
        c.count_add(0, ra.seq)
        c.count_add(1, rb.seq)
        c.count_run(2)
        sdk, _, _ = c.select(LOWER, UPPER)
    del ra, rb
    d = tempfile.mkdtemp(prefix="hga_tails_")
    try:
        n = round(LA / 7777 * 75)
        paths = [os.path.join(d, "hapA_nanosim.fasta"), os.path.join(d, "hapB_mosaic_nanosim.fasta")]
        hga.write_nanosim_fasta(ga, "A", n, 5002, paths[0])
        hga.write_nanosim_fasta(gbm, "B", n, 5003, paths[1])
        out = categorization_pipeline_leg(paths, sdk, threads, d,
                                          label="C3-sized tails workload: haplotype B = A with d=0.021 except 40 kb "
                                                "identical stretches every 600 kb; SDKs: GPU count of ART-like 30x "
                                                "short reads, [10,25]; long reads Nanosim-like 75x")
        if out is not None:
            out["sdk"] = int(len(sdk))
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def lookup_parse_leg(ga, gb, n_reads, lookup_s, bases, offsets, threads, sdk=None):
    """BASELINE.md §3 "reads/s categorized with parsing": the C3 long reads written as Nanosim-like
    FASTA (same generators and seeds as make_c3), read back by categorization's reader
    (load_records: SequenceRecordIterator, multi-threaded) and the lookup time added.  With `sdk`, the
    whole categorization CLI is then run on the same files (categorization_pipeline_leg)."""
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="hga_c3_")
    try:
        na, nb = round(LA / 7777 * 75), round(LB / 7777 * 75)
        paths = [os.path.join(d, "mg1655_nanosim.fasta"), os.path.join(d, "uti89_nanosim.fasta")]
        hga.write_nanosim_fasta(ga, "A", na, 3000, paths[0])
        hga.write_nanosim_fasta(gb, "B", nb, 3001, paths[1])
        size = sum(os.path.getsize(p) for p in paths)
        hga.set_host_threads(threads)
        hga.load_records(paths, True)   # page cache warm
        t0 = time.perf_counter()
        rec = hga.load_records(paths, True)
        parse_s = time.perf_counter() - t0
        hga.set_host_threads(0)
        same = rec["bases"] == bases and np.array_equal(rec["offsets"], offsets)
        del rec
        out = {"files": "C3 reads as Nanosim-like FASTA", "bytes": size, "reader_threads": threads,
               "parse_s": round(parse_s, 4), "same_reads_as_resident": bool(same),
               "reads_per_s": round(n_reads / (parse_s + lookup_s), 1),
               "note": "host FASTA parse (through the ctypes mirror) + one hga_lookup_run; upload not included"}
        if sdk is not None:
            out["pipeline"] = categorization_pipeline_leg(paths, sdk, threads, d)
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def ingest_leg(ga, gb, threads):
    """Host ingest of the CLIs: the C2 pair written as ART-like FASTQ, then
    jf_stream (jf_occurrences' per-file read) and load_records (categorization / auto-k) with the
    multi-threaded readers, the sequential restatement timed beside them."""
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="hga_ingest_")
    try:
        paths = [os.path.join(d, "mg1655.fq"), os.path.join(d, "uti89.fq")]
        for g, pth, seed, name in ((ga, paths[0], 1000, "A"), (gb, paths[1], 1001, "B")):
            hga.write_art_fastq(g, name, COVERAGE * len(g) // READ_LEN, READ_LEN, seed, pth)
        size = sum(os.path.getsize(p) for p in paths)
        out = {"files": "C2 pair as ART-like FASTQ", "bytes": size}
        for label, t in (("parallel", threads), ("sequential", 1)):
            hga.set_host_threads(t)
            for _ in range(2 if t > 1 else 1):   # warm page cache / first run
                t0 = time.perf_counter()
                n = sum(len(hga.jf_stream(p)) for p in paths)
                dt_jf = time.perf_counter() - t0
            t0 = time.perf_counter()
            rec = hga.load_records(paths, True)
            dt_lr = time.perf_counter() - t0
            out[label] = {"threads": t, "jf_stream_s": round(dt_jf, 3), "jf_stream_GBps": round(size / dt_jf / 1e9, 3),
                          "load_records_s": round(dt_lr, 3), "load_records_GBps": round(size / dt_lr / 1e9, 3),
                          "bases": int(n), "records": int(len(rec["offsets"]) - 1)}
        hga.set_host_threads(0)
        out["note"] = "wall time through the ctypes mirror (includes the copy into Python bytes)"
        # the drop-in CLI end to end on the same files (src/jellyfish_occurrences.cpp's argv and
        # stdin; no dump caches yet, so it counts on the GPU and writes them, as run_jellyfish.sh would)
        cli = os.path.join(ROOT, "hybrid-genome-assembler_amd", "bin", "jf_occurrences")
        if os.path.exists(cli):
            import subprocess
            env = dict(os.environ, HGA_PLOT_CMD="cat > /dev/null", HGA_TIMING="1")
            t0 = time.perf_counter()
            r = subprocess.run([cli, *paths, "-k", str(K)], input=f"{LOWER} {UPPER} 1\n", text=True,
                               capture_output=True, cwd=d, env=env, timeout=300)
            dt = time.perf_counter() - t0
            exp = os.path.join(d, f"{K}-mers_{LOWER}_{UPPER}_100%.txt")
            phases = {}
            for line in r.stderr.splitlines():   # "hga-timing <phase> <ms>" (HGA_TIMING=1)
                f = line.split()
                if len(f) == 3 and f[0] == "hga-timing":
                    phases[f[1]] = float(f[2])
            out["cli_jf_occurrences"] = {
                "argv": f"jf_occurrences mg1655.fq uti89.fq -k {K}  (stdin: {LOWER} {UPPER} 1)",
                "rc": r.returncode, "wall_s": round(dt, 3), "phases_ms": phases,
                "dump_bytes": sum(os.path.getsize(p + f"_{K}-mers_sorted") for p in paths
                                  if os.path.exists(p + f"_{K}-mers_sorted")),
                "exported_lines": sum(1 for _ in open(exp)) if r.returncode == 0 and os.path.exists(exp) else None,
                "note": "one process: HIP init (on a thread, overlapped with the FASTQ ingest), ingest, upload, "
                        "count, the two per-file sorted dump caches written as text (on a thread, overlapped "
                        "with the histogram, plot and export), histogram wire string, export file; phases_ms "
                        "from the CLI's HGA_TIMING=1 lines (main-thread wall time between marks)"}
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


# launch labels of the owner exchange (exchange.hip / comm.hip): the hash-bucket path (count-kernel
# emission, gather, owner merge), its generic sender fallback, the wide-row path, the export re-partition
XCH_KERNELS = ("kx_xb_pack", "kx_xb_gather", "kx_xb_hist", "kx_xb_scatter", "kx_xb_owner_tot", "kx_xb_units",
               "kx_xb_merge", "kc_xb_dense", "kx_mb_compact", "kx_partition", "kx_merge", "kx_piece_hist",
               "kx_pack_scatter", "kx_mb_hist", "kx_mb_scatter", "kx_mb_merge")

C4_GENOME, C4_COV = 500_000_000, 30.0 / 8


def make_c4_shard(rank=0):
    """SURVEY.md C4 at one rank of eight: ART-like 150 bp reads of a 2 x 500 Mbp diploid (d = 0.005)
    at 30x / 8 = 3.75x, 2 files (3.77 Gbases, 3.3 G 19-mer instances).  Rank r draws its own reads
    of the same diploid (seeds 43/44 at rank 0, the N = 1 bench leg and tests/test_scale_gpu.py)."""
    t_gen = time.perf_counter()
    g4a = hga.gen_genome(C4_GENOME, 41)
    g4b = hga.gen_haplotype(g4a, 0.005, 0, 42)
    n4 = int(C4_COV * C4_GENOME / READ_LEN)
    r4a = hga.gen_art(g4a, n4, READ_LEN, 43 + 2 * rank)
    r4b = hga.gen_art(g4b, n4, READ_LEN, 44 + 2 * rank)
    del g4a, g4b
    log(f"[rank {rank}] C4 rank shard generated in {time.perf_counter() - t_gen:.1f}s: {2 * n4} reads")
    return r4a, r4b


def scale_leg(D, reps=2):
    """BASELINE configs[3] ("C4": k=19 count of a 1 Gbp diploid at ART 30x over 8 GPUs) on this run's
    ranks: every rank counts its own C4/8 shard (make_c4_shard(rank): 3.77 Gbases, 3.3 G instances,
    counted in one pass with the third split level); at N > 1 the shards are then
    merged by the owner exchange over the library's communicator (hga_count_exchange), so N = 8 is
    configs[3] itself.  The step is the headline's (count + histogram + export selection); time = max
    over ranks."""
    r4a, r4b = make_c4_shard(D.rank)
    c4 = hga.Ctx(D.local)
    try:
        c4.count_begin(K, 2)
        c4.count_add(0, r4a.seq)
        c4.count_add(1, r4b.seq)
        bases = len(r4a.seq) + len(r4b.seq)
        del r4a, r4b
        ex4 = None
        if D.pg:
            import hga_dist
            ex4 = hga_dist.OwnerExchange(c4)
        step = (lambda: dist_count_step(ex4)) if ex4 else (lambda: count_step(c4))
        c4_local_inst = 0
        if ex4:   # this rank's own instances (the local count), for the conservation invariant
            c4.count_run(1)
            c4_local_inst = c4.count_stats().instances
        step()   # warm-up (allocations)
        c4.profile(True)
        c4.profile_reset()
        step()
        names = ("kc_init", "kc_bin1", "kc_layout", "kc_rebin", "kc_split3", "kc_count", "kc_spec_hist", "kc_select",
                 *XCH_KERNELS, "radix_upsweep", "radix_downsweep", "radix_segsort", "scan")
        ker = {nm: round(c4.profile_get(nm)[0], 3) for nm in names if c4.profile_get(nm)[1]}
        c4.profile(False)
        D.barrier()
        c4.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            n_sel, n_disc = step()
        c4.sync()
        D.barrier()
        ms = D.max((time.perf_counter() - t0) / reps * 1e3)
        st = c4.count_stats()   # global after the exchange
        export = None
        if ex4:   # the full export of the last step in code order, to one writer (rank 0)
            import resource
            c4.comm_set_root(0)   # hga_comm_set_root: one copy crosses the ranks, not N
            D.barrier()
            rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
            t1 = time.perf_counter()
            keys, flags = ex4.select(LOWER, UPPER)
            D.barrier()
            exp_ms = D.max((time.perf_counter() - t1) * 1e3)
            rss1 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
            k64 = keys.astype(np.uint64)
            off_root = D.max(float(len(keys)) if D.rank != 0 else 0.0)
            # size-independent invariants of the exchanged C4 result (its rows are not checked against
            # the oracle at this size: parity unpinned here, the C2 shards carry the N > 1 parity check)
            inv = {"export_ascending": bool(len(k64) < 2 or bool(np.all(k64[1:] > k64[:-1]))),
                   "export_count_matches_select": int(len(keys)) == int(n_sel),
                   "discriminative_matches_flags": int(flags.sum()) == int(n_disc),
                   "global_instances_equal_sum_of_ranks": int(st.instances) == int(D.sum(float(c4_local_inst))),
                   "other_ranks_receive_nothing": off_root == 0.0}
            export = {"ms": round(exp_ms, 2), "keys": int(len(keys)), "bytes_on_root": int(len(keys)) * 9,
                      "max_keys_on_other_ranks": int(off_root),
                      "max_rss_growth_mb": round(D.max((rss1 - rss0) / 1024.0), 1),
                      "note": "hga_comm_set_root(0) + hga_count_select_ex after the exchange: the owners' sorted "
                              "selections re-partitioned by code range (one all-to-all), the ranges gathered to "
                              "rank 0 only, in rank order (one writer, JellyfishOccurrenceReader.cpp:110-135)",
                      "invariants": inv, "parity": "unpinned at C4 size (invariants only)"}
            c4.comm_set_root(-1)
        return {"workload": f"C4 (configs[3]): {D.world} of the 8 rank shards of ART-like 30x reads of a 2 x 500 Mbp "
                            "diploid (d=0.005), k=19, 2 files per shard; step = count_run + "
                            + ("hga_count_exchange (owner all-to-all) + " if ex4 else "")
                            + "spec_hist + select[10,25]",
                "ranks": D.world, "fraction_of_c4": D.world / 8, "bases_per_rank": int(bases),
                "instances": int(st.instances), "distinct_rows": int(st.distinct_rows),
                "buckets": int(st.buckets), "max_split": int(st.max_split), "selected": int(n_sel),
                "discriminative": int(n_disc), "ms_per_step": round(ms, 2),
                "k_mers_per_s": round(st.instances / (ms * 1e-3), 1), "kernels_ms_rank0": ker,
                **({"export": export} if export else {})}
    finally:
        c4.close()


def dist_parity(ctx, D, threads):
    """N > 1: the exchanged (global) count of the timed step against the oracle over every rank's C2
    shard — all merged rows, the histogram and the export counts — so each multi-GPU run records
    the parity of its own transport (RCCL over xGMI by default).  Rank 0 checks; all ranks take part
    in the collective reads."""
    keys, counts = ctx.rows()
    hist = ctx.spec_hist(THRESHOLDS)
    n_sel, n_disc = ctx.select_device(LOWER, UPPER)
    out = None
    if D.rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        t0 = time.perf_counter()
        shards = [make_c2(r)[2:] for r in range(D.world)]
        streams = [b"\n".join(sh[f].seq for sh in shards) for f in range(2)]
        del shards
        ok, oc = oracle.count_files_mt(streams, K, 2, threads)
        sel, nd = oracle.select(ok, oc, LOWER, UPPER)
        eq = {"rows": bool(np.array_equal(keys, ok) and np.array_equal(counts, oc)),
              "histogram": bool(np.array_equal(hist, oracle.specificity(oc, THRESHOLDS))),
              "export_counts": bool(n_sel == len(sel) and n_disc == nd)}
        out = {"checked": "global rows, histogram and export counts of the exchanged C2 shards vs the oracle "
                          f"over all {D.world} ranks' reads ({threads} threads)",
               "transport": "RCCL (hga_comm_init)" if D.backend == "nccl" else "host transport hook (gloo)",
               "rows": int(len(ok)), "equal": all(eq.values()), "parts": eq,
               "seconds": round(time.perf_counter() - t0, 1)}
        if not out["equal"]:
            log(f"error: N>1 parity check failed: {eq}")
    D.barrier()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-lookup", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the host FASTQ ingest leg")
    ap.add_argument("--no-scale", action="store_true", help="skip the C4 leg (one C4/8 shard per rank)")
    ap.add_argument("--no-check", action="store_true", help="N > 1: skip the oracle check of the exchanged count")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("HGA_CPU_THREADS", "16")))
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    D = Dist(args.gpus)
    if os.environ.get("HGA_BENCH_DRYRUN") == "1":   # launcher test (tests/test_bench_launch.py)
        if D.rank == 0:
            print(json.dumps({"dryrun": True, "n_gpus": D.world, "backend": D.backend}), flush=True)
        D.close()
        return
    dev = D.local
    t_gen = time.perf_counter()
    ga, gb, ra, rb = make_c2(D.rank)
    log(f"[rank {D.rank}] C2 generated in {time.perf_counter() - t_gen:.1f}s: {ra.n + rb.n} reads")

    ctx = hga.Ctx(dev)
    ctx.count_begin(K, 2)
    ctx.count_add(0, ra.seq)
    ctx.count_add(1, rb.seq)
    ex = None
    if D.pg:
        import hga_dist
        ex = hga_dist.OwnerExchange(ctx)   # the library's RCCL communicator (hga_comm_init)
    step = (lambda: dist_count_step(ex)) if ex else (lambda: count_step(ctx))
    for _ in range(args.warmup):
        step()
    if ex:   # this rank's own count (what its counting kernels process in a step: min 1, no exchange)
        ctx.count_run(1)
    st = ctx.count_stats()
    stats = {"bytes": st.bytes, "instances": st.instances, "rows": st.distinct_rows, "files": 2}
    # 1) untimed profiled pass: per-kernel breakdown (events around every launch)
    names = ("kc_init", "kc_bin1", "kc_layout", "kc_rebin", "kc_count", "kc_spec_hist", "kc_select",
             *XCH_KERNELS, "radix_upsweep", "radix_downsweep", "bx_colscan", "bx_scatter", "radix_segsort", "scan")
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(args.steps):
        step()
    kernels = {}
    for name in names:
        ms, n = ctx.profile_get(name)
        if n:
            kernels[name] = {"ms_total": ms, "launches": n, "ms_per_step": ms / args.steps}
    dom = max(("kc_bin1", "kc_rebin", "kc_count"), key=lambda k: kernels.get(k, {}).get("ms_total", 0))
    # 2) timed pass: HIP events only around the dominant kernel (no event overhead elsewhere)
    ctx.profile_select([dom])
    ctx.profile_reset()
    D.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_sel, n_disc = step()
    ctx.sync()
    D.barrier()
    dt = time.perf_counter() - t0
    dt_max = D.max(dt)
    ms_step = dt_max / args.steps * 1e3
    inst_total = D.sum(float(st.instances))
    value = inst_total / (dt_max / args.steps)
    dom_ms, dom_n = ctx.profile_get(dom)
    ctx.profile_select([])
    ctx.profile(False)
    per_step_launches = dom_n / args.steps
    avg_launch_ms = dom_ms / dom_n
    bytes_step = KERNEL_BYTES[dom](stats)
    bytes_launch = bytes_step / per_step_launches
    achieved = bytes_launch / (avg_launch_ms * 1e-3) / 1e9
    traffic = pmc_traffic(dom)
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": int(bytes_launch), "avg_launch_ms": round(avg_launch_ms, 4)}
    # SURVEY.md §8(d) whole-counting model: 16.25 B per k-mer instance over the step time
    pipe_gbs = 16.25 * st.instances / (ms_step * 1e-3) / 1e9
    result = {
        "metric": "k-mers/s counted + reads/s categorized, k=19 E.coli 30×; %HBM roofline",
        "value": round(value, 1), "unit": "k-mers/s", "n_gpus": D.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": "C2: k=19 count of an E. coli-sized pair (4.64 + 5.07 Mb, d=0.021), ART-like 30x "
                               "150 bp, 2 files; per step: count_run + spec_hist + select[10,25]",
                   "k": K, "reads": ra.n + rb.n, "bases": st.bytes, "instances_per_gpu": st.instances,
                   "distinct_rows": st.distinct_rows, "selected": n_sel, "discriminative": n_disc,
                   "buckets": st.buckets, "max_split": st.max_split, "parallelism": f"dp{D.world}",
                   "exchange": (f"hga_count_exchange: owner all-to-all-v over "
                                f"{'RCCL (hga_comm_init)' if os.environ.get('HGA_BENCH_BACKEND', 'nccl') == 'nccl' else 'the host transport hook (gloo)'} "
                                f"of {'packed u64 row pieces' if ctx.count_pack_bits() else '(key, counts[F]) rows'}")
                   if ex else None},
        "roofline": roofline,
        "pipeline_roofline": {"model": "16.25 B per k-mer instance (SURVEY.md §8(d))",
                              "achieved": round(pipe_gbs, 1), "frac": round(pipe_gbs / HBM_PEAK_GBS, 4)},
        "kernels_ms_per_step": {k: round(v["ms_per_step"], 4) for k, v in kernels.items()},
    }
    if ex:   # the full export of the last timed step in code order, to one writer
        ctx.comm_set_root(0)
        D.barrier()
        t1 = time.perf_counter()
        ek, ef = ex.select(LOWER, UPPER)
        D.barrier()
        off_root = D.max(float(len(ek)) if D.rank != 0 else 0.0)
        result["export"] = {"ms": round(D.max((time.perf_counter() - t1) * 1e3), 3), "keys": int(len(ek)),
                            "discriminative": int(ef.sum()), "max_keys_on_other_ranks": int(off_root),
                            "note": "hga_comm_set_root(0) + select + fetch after the exchange: owners' sorted "
                                    "selections re-partitioned by code range (one all-to-all of the export), "
                                    "ranges gathered to rank 0 in rank order"}
        ctx.comm_set_root(-1)
        del ek, ef
    if ex and not args.no_check:   # the state of the last timed step: the exchanged global count
        result["parity"] = dist_parity(ctx, D, min(16 * D.world, os.cpu_count() or 16))

    if not args.no_lookup:
        t_gen = time.perf_counter()
        bases, offsets = make_c3(ga, gb, D.rank)
        log(f"[rank {D.rank}] C3 generated in {time.perf_counter() - t_gen:.1f}s: {len(offsets) - 1} reads")
        ctx2 = hga.Ctx(dev)
        if ex:
            ex.count(2)
            sdk, _ = ex.select(LOWER, UPPER)   # the whole export on every rank
        else:
            ctx.count_run(2)
            sdk, _, _ = ctx.select(LOWER, UPPER)
        ctx2.lookup_load(K, sdk)
        ctx2.lookup_set_reads(bases, offsets, 1)
        ctx2.lookup_run()
        reps = max(1, min(args.steps, 3))
        ctx2.profile(True)                     # untimed profiled pass: per-kernel breakdown
        ctx2.profile_reset()
        for _ in range(reps):
            ctx2.lookup_run()
        lk = {}
        for name in ("lk_pack", "lk_count", "lk_emit", "lk_post", "lk_sort", "lk_kci", "radix_upsweep",
                     "radix_downsweep", "scan"):
            ms, n = ctx2.profile_get(name)
            if n:
                lk[name] = round(ms / reps, 4)
        ctx2.profile(False)
        D.barrier()                            # timed pass, no events
        ctx2.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx2.lookup_run()
        ctx2.sync()
        D.barrier()
        dtl = D.max((time.perf_counter() - t0) / reps)
        s = ctx2.lookup_sizes()
        lk_ms = lk.get("lk_count", 0) + lk.get("lk_emit", 0)
        # 0.25 B packed input + 12 B slot read per window, 12 B out per hit (once)
        lk_bytes = s.windows * 12.25 + 12 * s.hits
        result["categorize"] = {
            "workload": "C3: Nanosim-H-like 75x long reads of the C2 pair vs the C2 [10,25] export (k=19)",
            "reads": int(s.n_reads), "bases": int(len(bases)), "windows": int(s.windows), "hits": int(s.hits),
            "sdk": int(s.n_sdk), "ms": round(dtl * 1e3, 3), "reads_per_s": round(D.sum(s.n_reads) / dtl, 1),
            "windows_per_s": round(D.sum(s.windows) / dtl, 1), "kernels_ms": lk,
            "lookup_roofline": {"model": "12.25 B per window + 12 B per hit (SURVEY.md §8(d)), counted once",
                                "kernel": "lk_scan<0> + lk_scan<1> (lk_count + lk_emit)", "peak": HBM_PEAK_GBS,
                                "unit": "GB/s",
                                "achieved": round(lk_bytes / (lk_ms * 1e-3) / 1e9, 1) if lk_ms else None,
                                "frac": round(lk_bytes / (lk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if lk_ms else None,
                                "whole_lookup_achieved": round(lk_bytes / dtl / 1e9, 1),
                                "whole_lookup_frac": round(lk_bytes / dtl / 1e9 / HBM_PEAK_GBS, 4)},
        }
        result["categorize"]["ms_note"] = ("ms = hga_lookup_run: the per-base encode of the resident ASCII reads "
                                           "(lk_pack) + lookup + CSR outputs; the upload is hga_lookup_set_reads")
        if D.world == 1 and not args.no_ingest:
            wp = lookup_parse_leg(ga, gb, s.n_reads, dtl, bases, offsets, args.cpu_threads, sdk)
            if wp.get("pipeline") is not None:
                result["categorize"]["pipeline"] = wp.pop("pipeline")
            result["categorize"]["with_parsing"] = wp
        if D.world == 1 and not args.no_ingest:
            result["categorize"]["pipeline_tails"] = tails_pipeline_leg(ga, dev, args.cpu_threads)
        result["categorize"]["connections"] = connections_leg(ctx2, D, reps, args)
        result["categorize"]["hll_auto_k"] = hll_leg(ctx2, D, len(bases), bases, offsets, args)
        ctx2.close()
        if not args.no_cpu and D.rank == 0 and D.world == 1:
            result["categorize"]["cpu_baseline"] = cpu_lookup_baseline(bases, offsets, sdk, args.cpu_threads)

    if not args.no_ingest and D.rank == 0 and D.world == 1:
        result["ingest"] = ingest_leg(ga, gb, args.cpu_threads)
    if not args.no_cpu and D.rank == 0 and D.world == 1:   # CPU baselines: rank 0 at N = 1 only
        parse_s = result.get("ingest", {}).get("parallel", {}).get("jf_stream_s")
        result["cpu_baseline"] = cpu_baseline(ra, rb, args.cpu_threads, parse_s)
    ctx.close()
    del ra, rb
    if not args.no_scale:
        result["scale_c4"] = scale_leg(D)
    D.close()
    if D.rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
