#!/usr/bin/env python3
"""Headline benchmark: SSSP source-paths/s + attached-pair matrix build time
(BASELINE.json "metric"), on BASELINE.json configs[1] -- the synthetic 10k-vertex
geometric complete-ish graph with 1k attached hosts per MI355X.

A step = one pass of the hot path over one batch of input: every source this rank owns
(1000 unique attached vertices) -> shortest-latency routes to all V vertices, composed
into the attached-pair latency / reliability / hop rows on the device; with N > 1 ranks
the rows are exchanged by an RCCL all-gather so every rank holds the full matrix
(SURVEY.md 8e).  Weak scaling: per-GPU work is fixed (1000 sources), the attached set
is 1000*N vertices.

python bench.py --gpus N --steps K --warmup W        (N>1 via torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
F64_VALU_OPS = 78.6e12 / 2  # f64 vector FMA/s (78.6 TFLOP/s counts an FMA as 2)
METRIC = "SSSP source-paths/sec + attached-pair matrix build time; % HBM peak, 1/2/4/8 GPU"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_workload(config, world, scale):
    from shadow_amd import synth
    if config == "C2":
        g = synth.geometric_complete_ish(V=int(10_000 * scale), A=int(1_000 * scale) * world)
        per = int(1_000 * scale)
        desc = f"C2 synthetic geometric complete-ish graph, V={g.n}, {per} attached sources per GPU"
    elif config == "C4":
        g = synth.barabasi_albert(V=int(100_000 * scale), A=int(10_000 * scale))
        per = (len(g.attached) + world - 1) // world
        desc = f"C4 synthetic Barabasi-Albert m=3, V={g.n}, A={len(g.attached)} sharded over GPUs"
    elif config == "C3":
        g = synth.knn_geographic(V=int(7_000 * scale))
        per = (len(g.attached) + world - 1) // world
        desc = f"C3 Tor stand-in geographic 16-NN, V={g.n}, A={len(g.attached)} sharded over GPUs"
    elif config == "C5":
        g = synth.chung_lu(V=int(1_000_000 * scale), A=int(50_000 * scale))
        per = (len(g.attached) + world - 1) // world
        desc = f"C5 synthetic Chung-Lu sparse AS graph, V={g.n}, A={len(g.attached)} sharded over GPUs"
    else:
        raise SystemExit(f"unknown config {config}")
    return g, per, desc


def algorithmic_bytes_per_source(V, n_arcs, A):
    """SURVEY.md 8d's per-source figure: B_src = 4(V+1) + 12*E_arc + 12*V + 20*A (kept for
    reference; it prices a private CSR sweep per source, which the batched kernels never do)"""
    return 4 * (V + 1) + 12 * n_arcs + 12 * V + 20 * A


STATE_BYTES = 36  # per changed (vertex, source): D f64 + D32 f32 + BDU f64 + P i32 + H u32 + R f64


def dense_sweep_compulsory(Vp, st):
    """Compulsory HBM bytes of the f32 dense full sweep (k_relax_dense_f), per launch, for
    the batched formulation: the W32 table once per launch (every batch of
    the launch filters against it), and per batch its D32 rows (4 B), the f64 distances the
    thresholds start from (8 B), the per-chunk D32 minima and the change masks; plus the
    state of every (vertex, source) pair the sweep changed.  Averaged over the launches."""
    L = max(1, st["full_sweeps"])
    nchunks = -(-Vp // 32)
    per_batch = Vp * 64 * (4 + 8) + nchunks * 64 * 4 + Vp * 8
    total = L * Vp * Vp * 4 + st["full_batches"] * per_batch + st["full_changes"] * STATE_BYTES
    return total / L


def sparse_step_compulsory(V, n_arcs, sources, state_bytes=24):
    """Compulsory HBM bytes of one matrix build on a sparse graph, batched Dijkstra-
    equivalent: per 64-source batch every in-arc's tail distances once (64 x 8 B), the CSR
    once (row pointer 8 B, tail 4 B + latency 8 B per arc) and every (vertex, source) state
    written once -- 12 B for the lean rounds (distance + predecessor arc), 24 B for the
    tree-fold rounds (distance + the {R, H, P} record).  V and n_arcs are the graph the rounds
    run on (C5: the pendant-pruned view).  (r06: up to r05 every state was priced at the dense
    sweep's 36 B and C5 at its full graph, which overstated the compulsory bytes, so the
    fraction, by ~28 % on C4.)"""
    nb = -(-sources // 64)
    return nb * (n_arcs * 64 * 8 + (V + 1) * 8 + n_arcs * 12 + V * 64 * state_bytes)


VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions/s: 1024 SIMD-32s, one wave64 instruction per 2 cycles at 2.4 GHz (MI355X_MICROARCH.md)


def load_counters(key):
    """this round's rocprofv3 counter summary for the same bench command (scripts/gpu_roofline.sh
    -> profiles/roofline_counters.json): HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE,
    separate passes) and wave64 VALU instructions per launch (SQ_INSTS_VALU scaled by the
    known wave count over SQ_WAVES) of the dominant kernel"""
    p = os.path.join(ROOT, "profiles", "roofline_counters.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(key)
    except Exception:
        return None


def cpu_baseline(g, n_sources, budget_s=20.0, all_cores=16):
    """The oracle (heap-exact C restatement of the reference path, 1 thread: the reference
    serialises every Dijkstra under graphLock, topology.c:1747-1781) on a bounded sample."""
    from oracle import oracle as O
    og = O.OracleGraph(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss, directed=g.directed)
    flags = og.flags(prefer_direct=g.prefer_direct)
    done = 0
    t0 = time.perf_counter()
    while done < n_sources and time.perf_counter() - t0 < budget_s:
        og.pair_rows(flags, g.attached, done, done + 1, nthreads=1)
        done += 1
    dt = time.perf_counter() - t0
    out = {"value": done / dt, "unit": "source-paths/s", "cores": 1, "kind": "port",
           "sample": f"{done} sources x {len(g.attached)} attached targets of the same graph "
                     f"({dt:.1f} s, oracle/topo_oracle.c, 1 thread)"}
    # the same oracle over all of this process's CPU share (BASELINE.md's second CPU figure;
    # the reference itself cannot do this: its Dijkstra runs under graphLock)
    nt = max(1, min(all_cores, 64))
    done2, t0 = 0, time.perf_counter()
    while done2 < 4 * nt and time.perf_counter() - t0 < budget_s / 2:
        r0 = (done + done2) % len(g.attached)
        r1 = min(r0 + nt, len(g.attached))
        og.pair_rows(flags, g.attached, r0, r1, nthreads=nt)
        done2 += r1 - r0
    dt2 = time.perf_counter() - t0
    og.close()
    out["all_cores"] = {"value": done2 / dt2, "cores": nt,
                        "sample": f"{done2} sources, {nt} threads ({dt2:.1f} s)"}
    return out


def roofline_of(st, g, config, scale, world, rows, steps, dense_variant=0, step_ms=None):
    """Roofline of the dominant kernel, timed with HIP events on the engine's stream around
    every launch: the f32 dense full sweep (k_relax_dense_f) on complete-ish graphs, the CSR
    relax rounds (k_relax, with the k_relax_wl worklist rounds) otherwise.  achieved = that
    kernel's compulsory bytes per launch / its average launch time; traffic =
    this round's rocprofv3 FETCH/WRITE passes over the same launch shape (or None)."""
    if st["dense"]:
        kname = "k_relax_dense" if dense_variant == 1 else "k_relax_dense_f"
        launches, kms = max(1, st["full_sweeps"]), st["full_ms"]
        Vp = -(-g.n // 64) * 64
        bytes_per_launch = dense_sweep_compulsory(Vp, st)
        batches_per_launch = st["full_batches"] / launches
    else:
        # every relax round of the step (grid and worklist launches alike): achieved = the
        # step's compulsory bytes / the relax kernels' time in the step
        kname = "k_push+k_pred_pass+k_fold" if st.get("push_rounds") else "k_relax"
        launches, kms = max(1, st["relax_launches"]), st["relax_ms"]
        bytes_per_launch = sparse_step_compulsory(st.get("relax_vertices") or g.n, st.get("relax_arcs") or st["n_arcs"],
                                                  rows, 12 if st.get("lean_groups") else 24) * steps / launches
        batches_per_launch = st["relax_batches"] / launches
    avg_launch_s = kms / launches / 1e3
    achieved = bytes_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else None
    ckey = f"{config}@{scale}@{world}"
    cnt = load_counters(ckey)
    if cnt and (cnt.get("kernel") != kname or abs(cnt.get("batches_per_launch", -1) - batches_per_launch) > 0.5):
        log(f"counter record {ckey} is for another launch shape ({cnt.get('kernel')}, "
            f"{cnt.get('batches_per_launch')} batches); not used")
        cnt = None
    traffic = cnt["hbm_bytes_per_launch"] if cnt else None
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                "kernel": kname, "avg_launch_ms": avg_launch_s * 1e3,
                "launches_per_step": launches / steps, "batches_per_launch": batches_per_launch,
                "compulsory_bytes_per_launch": bytes_per_launch,
                "traffic_over_compulsory": (traffic / bytes_per_launch) if traffic else None,
                # FETCH_SIZE / WRITE_SIZE count the L2's memory-side (fabric) requests, Infinity-
                # Cache hits included (MI355X_MICROARCH.md, HBM / rocprofv3): traffic / time is the
                # L2-to-fabric rate, not HBM bandwidth, and can exceed what HBM itself sustains
                "fabric_gbs": (traffic / avg_launch_s / 1e9) if (traffic and avg_launch_s > 0) else None,
                "traffic_note": ("FETCH_SIZE x2 + WRITE_SIZE per launch: L2-to-fabric bytes, Infinity-Cache hits "
                                 "included" if traffic else None),
                "counters": (cnt.get("source") if cnt else None)}
    if cnt and cnt.get("valu_insts_per_launch") and avg_launch_s > 0:
        ach = cnt["valu_insts_per_launch"] / avg_launch_s
        roofline["valu"] = {"unit": "wave64 VALU instructions/s", "achieved": ach, "peak": VALU_PEAK,
                            "frac": ach / VALU_PEAK, "insts_per_launch": cnt["valu_insts_per_launch"],
                            "note": "SQ_INSTS_VALU of the same bench command (profiles/), scaled by known "
                                    "waves / SQ_WAVES; peak = one wave64 VALU issue per 2 cycles per SIMD-32 at 2.4 GHz"}
    # the step-level fraction: the step's compulsory bytes (every launch of the dominant kernel)
    # over the whole step, not only the kernel's own time
    if step_ms:
        roofline["frac_step"] = bytes_per_launch * launches / steps / (step_ms / 1e3) / 1e9 / HBM_PEAK_GBS
    if st["dense"] and "valu" in roofline:
        # the dense sweep is bound by VALU issue and the latency of its barrier-coupled chunk
        # loop, not by HBM (DESIGN.md 9, r05 verdict): the headline fraction is the VALU one;
        # the HBM compulsory-byte fraction and the measured traffic stay beside it
        hbm = {k: roofline[k] for k in ("achieved", "peak", "unit", "frac", "frac_step", "traffic",
                                         "compulsory_bytes_per_launch", "traffic_over_compulsory", "fabric_gbs",
                                         "traffic_note") if k in roofline}
        v = roofline["valu"]
        roofline.update(bound="valu/latency", achieved=v["achieved"], peak=v["peak"], unit=v["unit"],
                        frac=v["frac"], hbm=hbm,
                        bound_note="VALU issue fraction of the chunk loop + exact pass (SQ_INSTS_VALU, profiles/); "
                                   "the kernel is latency-bound on its barrier-coupled chunk loop, neither VALU "
                                   "nor HBM saturated; roofline.hbm holds the compulsory-byte HBM fraction")
    if not st["dense"] and st["wl_launches"]:
        roofline["worklist_kernel"] = {"kernel": "k_relax_wl", "avg_launch_ms": st["wl_ms"] / st["wl_launches"],
                                       "launches_per_step": st["wl_launches"] / steps}
    if st["dense"] and st["delta_sweeps"]:
        roofline["delta_kernel"] = {"kernel": "k_relax_dense_delta" if dense_variant == 1 else "k_relax_dense_delta_s",
                                    "avg_launch_ms": st["delta_ms"] / st["delta_sweeps"],
                                    "launches_per_step": st["delta_sweeps"] / steps}
    return roofline


def host_build_ms(eng, r0, r1, A, steps, timed):
    """SURVEY.md 8(d)'s matrix build time: rows [r0, r1) of the A x A latency / reliability /
    hops matrix (and the pair kinds) delivered into page-locked host memory -- the shim's
    buffers -- PCIe included, timed like the device steps (`timed`: barrier + synchronize on
    both sides, max over ranks, exactly `steps` builds).  Every rank delivers its own row
    block into the one host's memory, so at N ranks the node's host holds the whole matrix."""
    from shadow_amd import engine as E
    rows = r1 - r0
    outs = [E.pinned_empty((rows, A), np.float64), E.pinned_empty((rows, A), np.float64),
            E.pinned_empty((rows, A), np.uint32), E.pinned_empty((rows, A), np.uint8)]
    eng.compute_rows_into(r0, r1, *outs)  # first touch of the buffers, untimed
    el = timed(lambda: eng.compute_rows_into(r0, r1, *outs), steps)
    del outs
    return el / steps * 1e3


def fresh_build_ms(eng, sets, r0, r1, steps, timed, device):
    """The matrix build a Shadow run pays once per attach epoch (topology.c:2371-2430 attaches,
    the first query computes, :2030): before every timed build the engine gets a NEW attached
    set of the same size (two seeded sets, alternating), so everything that depends on the set
    -- the self rule, the source locality order, the pendant-peeled relaxation view (sparse
    graphs), the upload of the list -- is rebuilt inside the timed region; then rows [r0, r1)
    land in HBM.  Timed like the device steps (barrier + synchronize, max over ranks)."""
    import torch
    A = len(sets[0])
    rows = r1 - r0
    lat = torch.empty((max(rows, 1), A), dtype=torch.float64, device=device)
    rel = torch.empty_like(lat)
    hops = torch.empty((max(rows, 1), A), dtype=torch.int32, device=device)
    k = [0]

    def one():
        k[0] ^= 1
        eng.set_attached(sets[k[0]])
        if rows > 0:
            eng.compute_rows_device(r0, r1, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(),
                                    stream=torch.cuda.current_stream(device).cuda_stream)
    one()
    one()  # both sets seen once (pool sizes, staging), untimed
    eng.reset_stats()
    el = timed(one, steps)
    prep = eng.stats()["attach_prep_ms"] / steps
    eng.set_attached(sets[0])
    del lat, rel, hops
    return el / steps * 1e3, prep


def rank_values(dist, world, x):
    """[x of rank 0, x of rank 1, ...] (a float per rank; [x] at one rank)"""
    if dist is None or world == 1:
        return [x]
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if dist.get_backend() == "gloo":
        dev = torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    out = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def sharded_report(dist, world, run, steps, relax_ms_per_step, rows):
    """What an N-rank step is made of: each rank's relax time and row count (all-gathered),
    the exchange alone (pack + all-gather + unpack, timed like the steps) and its bytes.  At
    N > 1 the step time (matrix_build_ms) includes the exchange: RowExchange.step computes and
    all-gathers."""
    out = {"per_rank_relax_ms": rank_values(dist, world, relax_ms_per_step),
           "per_rank_rows": [int(v) for v in rank_values(dist, world, rows)],
           "step_includes_exchange": world > 1}
    if world > 1:
        out["exchange_ms"] = run["allgather_s"] / steps * 1e3
        out["allgather_bytes"] = run["allgather_bytes"]
    else:
        out["exchange_ms"] = 0.0
        out["allgather_bytes"] = 0
    return out


def run_sharded(dist, world, rank, device, A, compute, steps, warmup, chunks=1, on_timed_start=None,
                on_timed_end=None, on_first_step=None, codec=None, hops16=None):
    """One sharded attached-pair matrix build per step: this rank's contiguous
    row block computed by `compute(a, z, lat, rel, hops)` into packed row chunks, each chunk
    all-gathered (shard.RowExchange).  `warmup` untimed steps, then exactly `steps` bracketed
    by a barrier and a device synchronisation on both sides, max over ranks; at N > 1 the
    all-gather alone is timed the same way afterwards.  `device` may be a CPU device (the gloo
    tests drive this with the oracle as the compute stand-in)."""
    import torch
    from shadow_amd import shard
    cuda = device.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize(device)

    def timed(fn, n):
        sync()
        if dist is not None:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        sync()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([el], dtype=torch.float64, device=device)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el

    ex = shard.RowExchange(dist, A, world, rank, device, chunks, codec=codec, hops16=hops16)
    for i in range(max(1, warmup)):
        ex.step(compute)
        if i == 0 and on_first_step:
            sync()
            on_first_step()
    if on_timed_start:
        on_timed_start()
    sent0 = ex.exchanged_bytes
    elapsed = timed(lambda: ex.step(compute), steps)
    if on_timed_end:
        on_timed_end()
    out = {"exchange": ex, "elapsed_s": elapsed, "timed": timed}
    if world > 1:
        if ex.codec is not None:
            # the packed exchange alone: pack, size agreement, payload all-gather, unpack
            def gather_only():
                for c, (c0, n) in enumerate(ex.bounds):
                    ex._exchange_packed(c, c0, n, ex.r0 + c0, min(ex.r1, ex.r0 + c0 + n))
            out["allgather_bytes"] = (ex.exchanged_bytes - sent0) // max(1, steps) * world
        else:
            def gather_only():
                works = [dist.all_gather_into_tensor(ex.gathered[c], ex.packs[c], async_op=True)
                         for c in range(len(ex.bounds))]
                for w in works:
                    w.wait()
            out["allgather_bytes"] = sum(p.numel() for p in ex.packs) * world
        out["allgather_s"] = timed(gather_only, steps)
    return out


def rehearsal_check(eng, ex, A, device):
    """SHADOWTOPO_BENCH_ONE_GPU rehearsals (every rank on one device): the matrix the exchange
    assembled on this rank against the whole A x A matrix computed by this rank's engine alone,
    bit for bit (None outside a rehearsal)"""
    if os.environ.get("SHADOWTOPO_BENCH_ONE_GPU") != "1" or ex.world == 1:
        return None
    import torch
    got = ex.full()
    lat = torch.empty((A, A), dtype=torch.float64, device=device)
    rel = torch.empty_like(lat)
    hops = torch.empty((A, A), dtype=torch.int32, device=device)
    eng.compute_rows_device(0, A, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(),
                            stream=torch.cuda.current_stream(device).cuda_stream)
    torch.cuda.synchronize(device)
    same = [bool(torch.equal(x.view(torch.int64) if x.dtype == torch.float64 else x,
                             y.view(torch.int64) if y.dtype == torch.float64 else y))
            for x, y in zip(got, (lat, rel, hops))]
    del lat, rel, hops
    every = rank_values(ex.dist, ex.world, float(all(same)))
    return {"rank": ex.rank, "pairs": A * A, "lat_equal": same[0], "rel_equal": same[1], "hops_equal": same[2],
            "ranks_equal": [bool(v) for v in every]}


def north_star_c4(device, dist=None, world=1, rank=0, steps=5, warmup=1, chunks=1, project=True, hops16=True):
    """The north-star workload (BASELINE.json configs[3], SURVEY.md 8d C4: a 10^5-vertex
    Barabasi-Albert graph, 10^4 attached hosts) on every rank, timed like the headline
    (inputs resident, rows into HBM, barrier + synchronize around exactly `steps` matrix
    builds, max over ranks), so the driver's own run carries it beside the configs[1] line
    at every GPU count: the A sources are sharded over the ranks in contiguous row blocks
    (shard.shard_rows) and one RCCL all-gather per row chunk gives every rank the whole
    10^4 x 10^4 latency / reliability / hop matrix (shard.RowExchange).

    At one GPU it also times rank 0's and the last rank's row share of an N-GPU run
    (N = 2, 4, 8) on this GPU: the per-GPU half of the N-GPU figure (the all-gather over
    xGMI is the other half, measured only by an N-GPU run)."""
    import torch
    from shadow_amd import engine as E
    from shadow_amd import shard
    g, _per, desc = build_workload("C4", world, 1.0)
    A = len(g.attached)
    eng = E.Engine.from_synth(g, device=device.index or 0)
    try:
        eng.set_attached(g.attached)
        eng.set_option(E.OPT_TIMING, 1)

        def compute(a, z, lat, rel, hops):
            stream = torch.cuda.current_stream(device).cuda_stream
            eng.compute_rows_device(a, z, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=stream)

        eng_stats = {}

        def reset():
            eng.reset_stats()

        def collect():
            eng_stats.update(eng.stats())

        # sparse rows: hop counts exchanged as 16-bit halves (shard.EngineHopCodec, 18 B per pair)
        hc = shard.EngineHopCodec(eng, stream_of=lambda: torch.cuda.current_stream(device).cuda_stream) \
            if world > 1 and hops16 else None
        run = run_sharded(dist, world, rank, device, A, compute, steps, warmup, chunks,
                          on_timed_start=reset, on_timed_end=collect, hops16=hc)
        ex, elapsed, st = run["exchange"], run["elapsed_s"], eng_stats
        timed = run["timed"]
        check = rehearsal_check(eng, ex, A, device)
        rec = {"workload": desc, "n_gpus": world, "n_vertices": g.n, "n_arcs": st["n_arcs"], "attached": A,
               "steps": steps, "warmup": warmup, "matrix_build_ms": elapsed / steps * 1e3,
               "value": A * steps / elapsed, "unit": "source-paths/s",
               "parallelism": f"{A} sources sharded x{world} (rows [{ex.r0},{ex.r1}) on rank {rank})"
                              + (f" + RCCL all-gather ({len(ex.bounds)} chunks)" if world > 1 else ""),
               "rounds_per_step": st["rounds"] / steps, "lean_rounds": st["lean_groups"] > 0,
               "roofline": roofline_of(st, g, "C4", 1.0, world, ex.rows, steps)}
        rec["compose_kernel_ms"] = st["compose_kernel_ms"] / steps
        rec["sharding"] = sharded_report(dist, world, run, steps, st["relax_ms"] / steps, ex.rows)
        rec["matrix_build_host_ms"] = host_build_ms(eng, ex.r0, ex.r1, A, steps, timed)
        rec["matrix_build_host_note"] = ("rows of this rank's block delivered into page-locked host memory "
                                         "(lat, rel, hops, kind), PCIe included, max over ranks")
        # a fresh attached set before every build (a second seeded set of the same size)
        other = np.sort(np.random.default_rng(16).choice(g.n, size=A, replace=False)).astype(np.int32)
        rec["matrix_build_fresh_ms"], rec["fresh_attach_prep_ms"] = fresh_build_ms(eng, [g.attached, other], ex.r0,
                                                                                   ex.r1, steps, timed, device)
        if world > 1:
            rec["allgather_ms"] = run["allgather_s"] / steps * 1e3
            rec["allgather_bytes_per_rank"] = run["allgather_bytes"]
            rec["exchange_mode"] = "hops16" if hc is not None else "raw"
            rec["hop_overflow_steps"] = ex.overflowed
            rec["allgather_GBps_per_rank"] = run["allgather_bytes"] * (world - 1) / world / (run["allgather_s"] / steps) / 1e9
        target = {"matrix_build_ms_under": 1000.0, "hbm_frac_at_least": 0.5, "on_gpus": 8,
                  "time_met": rec["matrix_build_ms"] < 1000.0,
                  "frac_compulsory": rec["roofline"]["frac"], "frac_met": rec["roofline"]["frac"] >= 0.5}
        rec["target"] = target
        if check is not None:
            rec["rehearsal_check"] = check
        if project and world == 1:
            proj = {}
            lat = torch.empty((A, A), dtype=torch.float64, device=device)
            rel = torch.empty((A, A), dtype=torch.float64, device=device)
            hops = torch.empty((A, A), dtype=torch.int32, device=device)
            for W in (2, 4, 8):
                shares = []
                for r in sorted({0, W - 1}):
                    a, z, _ = shard.shard_rows(A, W, r)
                    compute(a, z, lat, rel, hops)
                    eng.reset_stats()
                    el = timed(lambda: compute(a, z, lat, rel, hops), steps)
                    sst = eng.stats()
                    rf = roofline_of(sst, g, "C4", 1.0, W, z - a, steps)
                    shares.append({"rank": r, "rows": z - a, "ms": el / steps * 1e3,
                                   "host_ms": host_build_ms(eng, a, z, A, steps, timed),
                                   "relax_ms": sst["relax_ms"] / steps, "roofline_frac": rf["frac"],
                                   "rounds": sst["rounds"] / steps})
                slow = max(shares, key=lambda x: x["ms"])
                proj[str(W)] = {"per_gpu_ms": slow["ms"], "per_gpu_host_ms": max(x["host_ms"] for x in shares),
                                "ranks_timed": shares,
                                "allgather_bytes_per_gpu": 20 * A * A * (W - 1) // W,
                                "allgather_bytes_per_gpu_hops16": (shard.packed_bytes(-(-A // W), A, 2) * (W - 1)
                                                                   if hops16 else None),
                                "note": "one rank's row share computed on this GPU; the all-gather over xGMI "
                                        "is not included (measured only by an N-GPU run)"}
            rec["projection"] = proj
            del lat, rel, hops
    finally:
        eng.close()
    rec["vertex_loss_variant"] = c4_vertex_loss(g, device, dist, world, rank, steps, rec)
    return rec


def c4_vertex_loss(g, device, dist, world, rank, steps, base):
    """C4L: the north-star graph with vertex loss on 30 % of the vertices (U[0, 0.02],
    synth.with_vertex_loss): the pairs whose target carries loss take the reference's full
    path fold (topology.c:1429-1462) -- compose's bounded path walk -- so its compose time is
    reported beside the no-loss one.  This rank's rows into HBM, timed like the steps."""
    import torch
    from shadow_amd import engine as E
    from shadow_amd import shard
    gl = synth_vertex_loss(g)
    A = len(gl.attached)
    r0, r1, _ = shard.shard_rows(A, world, rank)
    eng = E.Engine.from_synth(gl, device=device.index or 0)
    try:
        eng.set_attached(gl.attached)
        eng.set_option(E.OPT_TIMING, 1)
        lat = torch.empty((max(1, r1 - r0), A), dtype=torch.float64, device=device)
        rel = torch.empty_like(lat)
        hops = torch.empty((max(1, r1 - r0), A), dtype=torch.int32, device=device)

        def one():
            if r1 > r0:
                eng.compute_rows_device(r0, r1, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(),
                                        stream=torch.cuda.current_stream(device).cuda_stream)
        one()
        eng.reset_stats()
        el = timed_steps(dist, device, one, steps)
        st = eng.stats()
        walked = float(np.mean(~np.isnan(gl.vertex_packetloss[gl.attached])))
        out = {"workload": "C4 with vertex packetloss on 30 % of the vertices (U[0, 0.02], seed 9)",
               "targets_with_vertex_loss": walked, "matrix_build_ms": el / steps * 1e3,
               "compose_kernel_ms": st["compose_kernel_ms"] / steps,
               "compose_kernel_ms_no_loss": base.get("compose_kernel_ms"),
               "relax_ms": st["relax_ms"] / steps}
        if out["compose_kernel_ms_no_loss"]:
            out["compose_ratio"] = out["compose_kernel_ms"] / out["compose_kernel_ms_no_loss"]
        del lat, rel, hops
        return out
    finally:
        eng.close()


def synth_vertex_loss(g):
    from shadow_amd import synth
    return synth.with_vertex_loss(g)


def timed_steps(dist, device, fn, n):
    """barrier + synchronize on both sides of exactly n calls, max over ranks (seconds)"""
    import torch
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    return el


def shim_host_matrix(ndev, config="C4", hosts=10_000):
    """The drop-in's own multi-GPU path, as Shadow runs it (one process): topology_new on the
    config's GraphML, `hosts` host attaches (no hints: the reference's random vertex pick,
    topology.c:2327-2333), then topology_hip_prepare with one engine per device
    (topology_hip_set_devices: device k computes a contiguous block of source rows on its
    own host thread straight into the shim's page-locked lat / rel / kind matrix,
    topology_hip.c compute_rows_sharded).  The prepare time is the whole one-shot build a
    Shadow run pays: engines (graph upload + device build), locality keys, rounds, compose
    and the PCIe copies into host memory."""
    import tempfile
    from shadow_amd import synth
    from shadow_amd import topology as T
    g, _per, desc = build_workload(config, 1, 1.0)
    T.set_log_level(1)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "topology.graphml.xml")
        with open(path, "w") as f:
            f.write(synth.to_graphml(g))
        t0 = time.perf_counter()
        top = T.Topology.new(path)
        ingest_s = time.perf_counter() - t0
    if top is None:
        return {"error": "topology_new failed"}
    try:
        rnd = T.Random(12345)
        addrs = [T.Address(f"11.{k >> 16 & 255}.{k >> 8 & 255}.{(k & 255) or 1}" if k & 255 else
                           f"12.{k >> 16 & 255}.{k >> 8 & 255}.1") for k in range(hosts)]
        t0 = time.perf_counter()
        for a in addrs:
            top.attach(a, rnd)
        attach_s = time.perf_counter() - t0
        top.set_devices(list(range(ndev)))
        t0 = time.perf_counter()
        rc = top.prepare()
        prep = time.perf_counter() - t0
        inf = top.info()
        A = inf["computed_for"]
        return {"workload": desc + f" (GraphML through topology_new, {hosts} hosts attached with no hints)",
                "devices": ndev, "attached": inf["n_attached"], "rc": rc,
                "ingest_s": ingest_s, "attach_s": attach_s, "prepare_ms": prep * 1e3,
                "compute_ms": inf["compute_seconds"] * 1e3,
                "host_matrix_bytes": A * A * 17, "host_matrix_GBps": A * A * 17 / prep / 1e9 if prep > 0 else None,
                "note": "host-side (page-locked) matrix build time of the drop-in, PCIe included; "
                        "cold: engine creation on every device included"}
    finally:
        top.free()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--vertex-loss", action="store_true",
                    help="vertex packetloss on 30 %% of the vertices (synth.with_vertex_loss: C4L for --config C4)")
    ap.add_argument("--no-fresh", action="store_true", help="skip the fresh-attached-set builds (rocprof counter passes "
                                                               "read the last dispatches, which must be the timed steps)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-rate", action="store_true", help="skip the host-buffer (PCIe-inclusive) timing")
    ap.add_argument("--cpu-sources", type=int, default=12)
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the C4 north-star record (sharded over the ranks) the default C2 run adds to its line")
    ap.add_argument("--no-shim", action="store_true",
                    help="skip the drop-in's in-process multi-GPU host-matrix build (C4 through topology_new)")
    ap.add_argument("--profile-counts", action="store_true", help="count relax visits/changes (slower)")
    ap.add_argument("--batches", type=int, default=0, help="source batches in flight (0 = auto)")
    ap.add_argument("--dense-variant", type=int, default=0, help="0 = f32-filtered kernels (default), 1 = f64 kernels")
    ap.add_argument("--chunks", type=int, default=0, help="row chunks per step (0 = 2 at N>=8, else 1): "
                    "chunk c's all-gather overlaps chunk c+1's computation")
    ap.add_argument("--sweep-glds", type=int, default=-1, help="pruned dense sweep: chunk loop staged by LDS-DMA (1) "
                    "or through registers (0); -1 = engine default")
    ap.add_argument("--dense-w16", type=int, default=-1, help="pruned dense sweep: 16-bit filter weights (1), f32 (0); -1 = engine default")
    ap.add_argument("--dense-spec", type=int, default=-1, help="dense: leading rounds with no host read-back (0..4); -1 = engine default")
    ap.add_argument("--sweep-parts", type=int, default=0, help="pruned dense sweep: batches in 1 .. 4 parts on their own streams (0 = engine default)")
    ap.add_argument("--chain-parts", type=int, default=-1, help="read-back-free delta rounds on each sweep part's stream (1) or after the join (0); -1 = engine default")
    ap.add_argument("--exchange", choices=["packed", "raw"], default="packed",
                    help="N > 1: exchange rows packed (dense graphs: EngineRowCodec; sparse graphs: 16-bit hop "
                         "counts, EngineHopCodec; the default) or raw")
    ap.add_argument("--dense-tb", type=int, default=0, help="batches per wave in the f32 dense sweep (0 = engine default)")
    ap.add_argument("--source-order", type=int, default=1, help="1 = locality-ordered source batches (default), 0 = attach order")
    ap.add_argument("--device-rounds", type=int, default=-1, help="CSR worklist rounds driven from the device: 0 never, "
                    "1 when batches x vertices <= 1 Mi, 2 always; -1 = engine default")
    ap.add_argument("--csr-variant", type=int, default=1, help="sparse rounds: 1 = pull (default), 2 = push (u64 atomicMin)")
    ap.add_argument("--worklist", type=int, default=1, help="CSR rounds over compacted frontier worklists when under half the pairs are active (1, default), "
                         "always (2), or the full grid (0)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one rank per GPU: start them ourselves (a child launcher, before this process
        # touches the GPU) and report its exit status
        import socket
        import subprocess
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        log("launching: " + " ".join(cmd))
        raise SystemExit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: refusing to run a different rank count")
    # rehearsal of the N-rank path on a one-GPU box: every rank on device 0, gloo instead of
    # RCCL (RCCL refuses two ranks on one device).  The numbers mean nothing; the code path
    # (launcher, sharding, codecs, exchange, barriers, the report) is the one N GPUs run.
    one_gpu = world > 1 and os.environ.get("SHADOWTOPO_BENCH_ONE_GPU") == "1"
    if one_gpu:
        local = 0

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local}")

    from shadow_amd import engine as E
    from shadow_amd import shard
    # the device preparation (HIP queue initialisation, staging buffers, code objects) runs in
    # the background while the workload is generated, as the shim's topology_new overlaps it
    # with the GraphML parse; its own duration is reported in cold_start_parts_ms["prepare"]
    E.prepare(local)
    t = time.perf_counter()
    g, _per, desc = build_workload(args.config, world, args.scale)
    if args.vertex_loss:
        g = synth_vertex_loss(g)
        desc += ", vertex packetloss on 30 % of the vertices"
    A = len(g.attached)
    r0, r1, per = shard.shard_rows(A, world, rank)
    log(f"[rank {rank}] workload {desc}: E={g.m} built in {time.perf_counter() - t:.1f}s; rows [{r0},{r1})")
    t_cold = t = time.perf_counter()
    eng = E.Engine.from_synth(g, device=local)
    create_ms = (time.perf_counter() - t_cold) * 1e3
    eng.set_attached(g.attached)
    eng.set_option(E.OPT_TIMING, 1)
    if args.profile_counts:
        eng.set_option(E.OPT_PROFILE, 1)
    if args.batches:
        eng.set_option(E.OPT_BATCHES_IN_FLIGHT, args.batches)
    eng.set_option(E.OPT_DENSE_VARIANT, args.dense_variant)
    if args.dense_tb:
        eng.set_option(E.OPT_DENSE_BATCHES_PER_WAVE, args.dense_tb)
    if args.dense_w16 >= 0:
        eng.set_option(E.OPT_DENSE_W16, args.dense_w16)
    if args.sweep_glds >= 0:
        eng.set_option(E.OPT_SWEEP_GLDS, args.sweep_glds)
    if args.dense_spec >= 0:
        eng.set_option(E.OPT_DENSE_SPEC, args.dense_spec)
    if args.sweep_parts:
        eng.set_option(E.OPT_SWEEP_PARTS, args.sweep_parts)
    if args.chain_parts >= 0:
        eng.set_option(E.OPT_CHAIN_PARTS, args.chain_parts)
    eng.set_option(E.OPT_SOURCE_ORDER, args.source_order)
    eng.set_option(E.OPT_WORKLIST, args.worklist)
    if args.device_rounds >= 0:
        eng.set_option(E.OPT_DEVICE_ROUNDS, args.device_rounds)
    if not eng.complete and args.csr_variant != 1:
        eng.set_option(E.OPT_CSR_VARIANT, args.csr_variant)
    log(f"[rank {rank}] engine (graph resident in HBM) in {time.perf_counter() - t:.1f}s, "
        f"complete={eng.complete}")
    rows = r1 - r0
    # The rank's `per` rows (the last rank's tail is padding, so every rank contributes the
    # same bytes) are computed in `chunks` row chunks; each chunk's lat/rel/hops rows live in
    # ONE packed byte buffer [lat f64 | rel f64 | hops i32], so one RCCL all-gather per chunk
    # moves all three, and chunk c's all-gather (RCCL's own stream, xGMI) overlaps the
    # computation of chunk c+1 on the engine's stream (shard.RowExchange; the same code path
    # runs in tests/test_shard_gloo.py with world size 2 on gloo).
    # (measured at N=1: 2 chunks cost +0.9 ms of per-chunk overhead, so overlap pays only
    # where the exchange is long: 8 ranks move ~1.1 GB into every GPU per step)
    # dense graphs exchange packed rows (shard.EngineRowCodec: a bit per pair every rank
    # rebuilds from its own graph replica, the rest in full; C2 at 8 ranks ~11 MB per rank
    # instead of 160 MB), which is small enough that one chunk suffices
    dense = bool(eng.stats()["dense"])
    codec = (shard.EngineRowCodec(eng, stream_of=lambda: torch.cuda.current_stream(dev).cuda_stream)
             if world > 1 and dense and args.exchange == "packed" else None)
    # sparse graphs: no pair is rebuilt from the replica; the hop counts travel as 16-bit
    # halves (shard.EngineHopCodec: 18 B per pair instead of 20, the high halves only if a
    # count reaches 2^16)
    hops16 = (shard.EngineHopCodec(eng, stream_of=lambda: torch.cuda.current_stream(dev).cuda_stream)
              if world > 1 and not dense and args.exchange == "packed" else None)
    chunks = args.chunks or (2 if world >= 8 and codec is None else 1)

    def compute(a, z, lat, rel, hops):
        stream = torch.cuda.current_stream(dev).cuda_stream
        eng.compute_rows_device(a, z, lat.data_ptr(), rel.data_ptr(), hops.data_ptr(), stream=stream)

    cold = {}
    st = {}
    run = run_sharded(dist, world, rank, dev, A, compute, args.steps, args.warmup, chunks,
                      on_timed_start=eng.reset_stats, on_timed_end=lambda: st.update(eng.stats()),
                      # engine creation -> first finished matrix rows on the device
                      on_first_step=lambda: cold.update(ms=(time.perf_counter() - t_cold) * 1e3), codec=codec,
                      hops16=hops16)
    cold_start_ms = cold["ms"]
    elapsed = run["elapsed_s"]
    check = rehearsal_check(eng, run["exchange"], A, dev)
    total_sources = A if world > 1 else rows  # every rank's rows per step
    value = total_sources * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # roofline of the dominant kernel, timed with HIP events on the engine's stream around
    # every launch
    roofline = roofline_of(st, g, args.config, args.scale, world, rows, args.steps, args.dense_variant,
                           step_ms=ms_per_step)

    # SURVEY.md 8(d)'s matrix build time "delivered to host": the same steps with the rows
    # landing in page-locked host memory (PCIe included), beside the device-resident figure
    build_host_ms = None
    if not args.no_host_rate:  # the same condition on every rank: the timing takes barriers
        build_host_ms = host_build_ms(eng, r0, r1, A, args.steps, run["timed"])

    # the build a Shadow run pays once per attach epoch: a new attached set (same size, seed
    # 13) before every timed build, so the set-dependent work is inside the timed region
    fresh_ms = fresh_prep_ms = None
    if not args.no_fresh:
        other = np.sort(np.random.default_rng(13).choice(g.n, size=A, replace=False)).astype(np.int32)
        fresh_ms, fresh_prep_ms = fresh_build_ms(eng, [g.attached, other], r0, r1, args.steps, run["timed"], dev)
    sharding = sharded_report(dist, world, run, args.steps, st["relax_ms"] / args.steps, rows)

    # the drop-in boundary hands host buffers over (topology_hip.c: MEM_HOST); its
    # PCIe-inclusive rate, measured once outside the timed region (never `value`)
    # The shim's layout: latency, reliability and kind in page-locked host memory (no hop
    # counts: the topology API never returns them); the copy of a batch group overlaps the
    # next group's computation.  Also the same rows into ordinary pageable numpy arrays.
    host_ms = host_pageable_ms = None
    if rank == 0 and world == 1 and rows > 0 and not args.no_host_rate:
        outs = [E.pinned_empty((rows, A), np.float64), E.pinned_empty((rows, A), np.float64), None,
                E.pinned_empty((rows, A), np.uint8)]
        eng.compute_rows_into(r0, r1, *outs)  # first touch of the buffers
        h0 = time.perf_counter()
        eng.compute_rows_into(r0, r1, *outs)
        host_ms = (time.perf_counter() - h0) * 1e3
        del outs
        outs = [np.empty((rows, A), np.float64), np.empty((rows, A), np.float64), None, np.empty((rows, A), np.uint8)]
        h0 = time.perf_counter()
        eng.compute_rows_into(r0, r1, *outs)
        host_pageable_ms = (time.perf_counter() - h0) * 1e3
        del outs

    # the row exchange: at N > 1 what the timed steps moved; at N = 1 (dense) a probe packing
    # this rank's rows once, after the timing, for the packed-to-raw ratio the N-rank runs see
    exchange = {"mode": "packed" if codec is not None else ("hops16" if hops16 is not None else
                                                            ("raw" if world > 1 else None))}
    if world > 1:
        exchange.update(gathered_bytes_per_step=run["allgather_bytes"],
                        raw_bytes_per_step=sum(p.numel() for p in run["exchange"].packs) * world,
                        exchange_ms=run["allgather_s"] / args.steps * 1e3)
    elif dense and rows > 0 and args.exchange == "packed":
        ex = run["exchange"]
        lat_v, rel_v, hops_v = ex.views[0]
        n0 = min(rows, ex.bounds[0][1])
        probe = shard.EngineRowCodec(eng, stream_of=lambda: torch.cuda.current_stream(dev).cuda_stream)
        buf = torch.empty(probe.capacity(n0, A), dtype=torch.uint8, device=dev)
        nbytes = probe.pack(r0, r0 + n0, lat_v[:n0], rel_v[:n0], hops_v[:n0], buf)
        exchange.update(probe_rows=n0, probe_raw_bytes=n0 * A * 20, probe_packed_bytes=nbytes,
                        probe_ratio=n0 * A * 20 / max(1, nbytes))
    # the north-star record (C4 sharded over every rank + all-gather) at every GPU count: all
    # ranks take part (barriers, all-gather), rank 0 reports
    north = None
    if args.config == "C2" and args.scale == 1.0 and not args.no_north_star:
        eng.close()
        eng = None
        try:
            # C4 is sparse: no row codec, so its own chunking (2 overlapped chunks at N >= 8, where
            # every GPU takes in ~1.6 GB), not the headline's (1 chunk beside C2's packed rows)
            north = north_star_c4(dev, dist, world, rank, chunks=args.chunks or (2 if world >= 8 else 1),
                                  hops16=args.exchange == "packed")
        except Exception as e:  # report, never fake
            north = {"error": f"{type(e).__name__}: {e}"}

    # the drop-in's in-process multi-GPU path (one engine per device, rows straight into the
    # shim's page-locked host matrix): rank 0 drives every GPU of the node while the other
    # ranks wait at the barrier
    shim = None
    if args.config == "C2" and args.scale == 1.0 and not args.no_north_star and not args.no_shim:
        if rank == 0:
            try:
                shim = shim_host_matrix(world)
            except Exception as e:  # report, never fake
                shim = {"error": f"{type(e).__name__}: {e}"}
        if world > 1:
            dist.barrier()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            share = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
            cpu = cpu_baseline(g, args.cpu_sources, all_cores=share)
        except Exception as e:  # report, never fake
            cpu = {"value": None, "error": str(e)}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "source-paths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak" if args.config == "C2" else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md 8d generator, fixed seeds)",
            "config": {"workload": desc, "n_vertices": g.n, "n_edges": g.m, "n_arcs": st["n_arcs"],
                       "attached": A, "sources_per_gpu": rows, "matrix_build_ms": ms_per_step,
                       # a source-path is one source's row over all A attached targets, by shortest
                       # paths over the relaxation graph: the pendant-pruned view where one exists
                       # (C5; a peeled pendant vertex lies on no attached pair's path)
                       "relaxation_vertices": g.n - st.get("pruned_vertices", 0),
                       "unit_note": ("source-paths over the pendant-pruned view (%d of %d vertices)"
                                     % (g.n - st["pruned_vertices"], g.n)) if st.get("pruned_vertices") else
                                    "source-paths over every vertex",
                       "matrix_build_host_ms": build_host_ms, "matrix_build_fresh_ms": fresh_ms,
                       "fresh_attach_prep_ms": fresh_prep_ms,
                       "matrix_build_note": "matrix_build_ms: rows left in HBM (the timed steps above: every "
                                            "kernel that writes the matrix, the self rule included); "
                                            "matrix_build_host_ms: the same builds delivered into page-locked "
                                            "host memory (lat, rel, hops, kind; PCIe included), timed the same way; "
                                            "matrix_build_fresh_ms: a new attached set of the same size before "
                                            "every build (self rule, source order, relaxation view and the list's "
                                            "upload rebuilt inside the timed region)",
                       "parallelism": f"sources sharded x{world}" + (
                           "" if world == 1 else (" + packed-row RCCL all-gather (EngineRowCodec)" if codec is not None
                                                  else f" + RCCL all-gather ({chunks} chunks, overlapped)"))},
            "exchange": exchange,
            "sharding": sharding,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "north_star": north,
            "shim_host_matrix": shim,
            "engine": {"rounds_per_step": st["rounds"] / args.steps, "replayed_sources": st["replayed_sources"],
                       "relax_ms_per_step": st["relax_ms"] / args.steps,
                       "compose_ms_per_step": st["compose_ms"] / args.steps,
                       "compose_kernel_ms_per_step": st["compose_kernel_ms"] / args.steps,
                       "self_paths_per_step": st["self_paths"] / args.steps, "dense": st["dense"],
                       "lean_rounds": st["lean_groups"] > 0, "walk_targets": st["walk_targets"],
                       "engine_wall_ms_per_step": st["wall_ms"] / args.steps,
                       "pool_allocs_in_timed_steps": st["pool_allocs"],
                       "pool_alloc_ms_per_step": st["pool_alloc_ms"] / args.steps,
                       "visits_per_step": st["visits"] / args.steps, "changes_per_step": st["changes"] / args.steps,
                       "full_sweeps_per_step": st["full_sweeps"] / args.steps,
                       "delta_sweeps_per_step": st["delta_sweeps"] / args.steps,
                       "host_syncs_per_step": st["host_syncs"] / args.steps,
                       "groups_per_step": st["groups"] / args.steps,
                       "push_phases_ms_per_step": ({"push": st["push_ms"] / args.steps, "pred": st["pred_ms"] / args.steps,
                                                    "fold": st["fold_ms"] / args.steps,
                                                    "push_rounds": st["push_rounds"] / args.steps,
                                                    "fold_rounds": st["fold_rounds"] / args.steps}
                                                   if st["push_rounds"] else None),
                       "host_buffers_ms": host_ms, "host_buffers_pageable_ms": host_pageable_ms,
                       "cold_start_ms": cold_start_ms,
                       # where the cold start goes: shadowtopo_create (edge validation, upload,
                       # device build), the dense locality order, the rest of the first step;
                       # "prepare" ran before it, overlapped with the workload generation
                       "cold_start_parts_ms": {"prepare": st["prepare_ms"],
                                               "prepare_wait": st["create_prepare_wait_ms"],
                                               "create": create_ms, "validate": st["create_validate_ms"],
                                               "upload": st["create_upload_ms"],
                                               "upload_alloc": st["create_alloc_ms"], "build": st["create_build_ms"],
                                               "order": st["order_ms"],
                                               "first_step": cold_start_ms - create_ms},
                       "host_buffers_source_paths_per_s": (rows / host_ms * 1e3) if host_ms else None},
        }
        if one_gpu:
            out["rehearsal"] = f"{world} ranks on one GPU over gloo (SHADOWTOPO_BENCH_ONE_GPU): not a measurement"
            out["rehearsal_check"] = check
        print(json.dumps(out), flush=True)
    if eng is not None:
        eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
