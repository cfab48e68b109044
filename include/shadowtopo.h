/*
 * shadowtopo.h -- C ABI of libshadowtopo_hip, the MI355X (gfx950) engine behind
 * Shadow's topology path computation.
 *
 * It replaces, below the unchanged topology.h API (topology_hip.h in this repo), the
 * reference's igraph-based per-source lazy path computation:
 *   - igraph_get_shortest_paths_dijkstra call      /root/reference/src/main/routing/topology.c:1754-1775
 *   - _topology_computeSourcePaths                  topology.c:1655-1875
 *   - _topology_computePathProperties               topology.c:1407-1523
 *   - _topology_computeShortestPathToSelf           topology.c:1545-1653
 *   - _topology_lookupDirectPath                    topology.c:1877-1927
 *   - the dispatch of _topology_getPathEntry        topology.c:2019-2031
 *   - the two-level path cache                      topology.c:42-47, 1284-1386
 * with one eager, batched, many-source computation of the attached-pair matrix
 * (A x A latency / reliability / hop count) on the GPU.
 *
 * Plain C: int status codes, no exceptions, caller-owned buffers, no torch types.
 * Not thread-safe per engine: callers serialise calls on one engine (the topology shim
 * does so with a mutex / pthread_once).
 */
#ifndef SHADOWTOPO_H
#define SHADOWTOPO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct shadowtopo_engine shadowtopo_engine;

/* status codes */
#define SHADOWTOPO_OK 0
#define SHADOWTOPO_EINVAL (-1)   /* bad argument / malformed graph */
#define SHADOWTOPO_ENOMEM (-2)   /* host or device allocation failed */
#define SHADOWTOPO_EDEVICE (-3)  /* HIP runtime error, or no GPU */
#define SHADOWTOPO_ESTATE (-4)   /* call out of order (e.g. compute before set_attached) */
#define SHADOWTOPO_EINTERNAL (-5) /* iteration guard tripped, or a path walk left the predecessor tree */

/* graph flags (topology.c:751-790: isDirected, isComplete, prefersDirectPaths) */
#define SHADOWTOPO_F_DIRECTED 0x1u
#define SHADOWTOPO_F_COMPLETE 0x2u
#define SHADOWTOPO_F_PREFER_DIRECT 0x4u
/* alternative self-pair rule: the [s] path igraph >= 0.7 returns for the
 * source itself, i.e. the source's self-loop edge (topology.c:1456-1499); default is the
 * version-independent _topology_computeShortestPathToSelf rule (topology.c:1545-1653). */
#define SHADOWTOPO_F_SELF_DIJKSTRA_LOOP 0x8u
/* let the engine decide F_COMPLETE with the reference's rule (_topology_isComplete,
 * topology.c:450-552) instead of trusting the caller's F_COMPLETE bit */
#define SHADOWTOPO_F_AUTO_COMPLETE 0x10u
/* relaxation layout: default picks the dense-tile form when arcs >= V^2/4 (and the
 * V x V tables fit), the CSR form otherwise; these force one (testing / tuning) */
#define SHADOWTOPO_F_FORCE_DENSE 0x20u
#define SHADOWTOPO_F_FORCE_CSR 0x40u

/* where compute_rows' output buffers live */
#define SHADOWTOPO_MEM_HOST 0
#define SHADOWTOPO_MEM_DEVICE 1
/* host, latency and reliability interleaved: `lat` holds rows x count {lat, rel} pairs
 * (16 bytes per pair, one cache line serves a packet's getLatency and getReliability),
 * `rel` must be NULL */
#define SHADOWTOPO_MEM_HOST_LR 2

/* per-pair kind codes (optional output) */
#define SHADOWTOPO_KIND_NONE 0     /* unroutable: lat = rel = -1 (topology.c:2073, 2085) */
#define SHADOWTOPO_KIND_DIRECT 1   /* _topology_lookupDirectPath, isDirect = TRUE */
#define SHADOWTOPO_KIND_SELF 2     /* _topology_computeShortestPathToSelf */
#define SHADOWTOPO_KIND_DIJKSTRA 3 /* shortest path */

/* options for shadowtopo_set_option */
#define SHADOWTOPO_OPT_BATCHES_IN_FLIGHT 1 /* source batches (64 sources each) relaxed together */
#define SHADOWTOPO_OPT_TIMING 2            /* 1 = record HIP events around every relax launch */
#define SHADOWTOPO_OPT_MAX_ROUNDS 3        /* iteration guard (default 4*V+64) */
#define SHADOWTOPO_OPT_FORCE_REPLAY 4      /* 1 = run the heap-exact kernel for every source (testing) */
#define SHADOWTOPO_OPT_PROFILE 5           /* 1 = count visits and changes per round (see shadowtopo_stats) */
#define SHADOWTOPO_OPT_DENSE_VARIANT 6     /* dense relax kernels: SHADOWTOPO_DENSE_F32 (default) or _F64 */
/* dense relaxation kernels (both exact; F32 pre-filters every candidate in f32 against a
 * conservative threshold and re-evaluates the survivors in f64, F64 evaluates everything in f64) */
#define SHADOWTOPO_DENSE_F32 0
#define SHADOWTOPO_DENSE_F64 1
#define SHADOWTOPO_OPT_DELTA_PERMILLE 7    /* dense: a batch whose last round changed <= this many per mille of its
                                              (vertex, source) pairs gets a change-mask delta round instead of a full
                                              sweep (default 125; 0 = always full sweeps) */
#define SHADOWTOPO_OPT_CSR_VARIANT 8       /* sparse relax kernels: SHADOWTOPO_CSR_FULL (pull, default) or _PUSH */
#define SHADOWTOPO_OPT_DENSE_BATCHES_PER_WAVE 9 /* f32 dense full sweep: batches one wave filters at once (1 = default, 2, 4) */
#define SHADOWTOPO_OPT_SOURCE_ORDER 10     /* CSR rounds: 1 (default) = sources batched in locality order (Hilbert
                                              order of the top two principal axes of the distances to eight
                                              attached landmarks), 0 = attach order.
                                              Results are identical; only which sources share a wave changes. */
#define SHADOWTOPO_OPT_DENSE_SEED 11       /* dense round 0: 1 (default) = one fused pass writing every (vertex,
                                              source) state once (k_seed_dense_t), 0 = init, source seed and arc seed
                                              kernels in turn. Results are identical. */
#define SHADOWTOPO_OPT_DENSE_PRUNE 12      /* f32 dense full sweep: 1 (default) = rows and destinations in a vertex
                                              locality order (the same landmark embedding over all vertices, built on
                                              the first computation), sources batched in locality order, and a wave
                                              skips a 32-row chunk when no lane can pass any of its rows (bound: min
                                              D32 of the chunk vs max over its columns of threshold - the
                                              column's min W32 over the chunk);
                                              0 = every chunk filtered, original order. Results are identical. */

#define SHADOWTOPO_OPT_WORKLIST 14         /* CSR FULL rounds: 1 (default) = over compacted frontier worklists (one
                                              wave per active (vertex, batch) pair) when under half the pairs are
                                              active, the grid otherwise; 2 = worklists always; 0 = one wave per pair
                                              of the grid */
#define SHADOWTOPO_OPT_GRID_X 15           /* testing: largest x dimension (blocks, a multiple of 8) of the sparse
                                              relax grids before they go 2-D (default 2^23: 2^31 work-items per
                                              launch, under the dispatch packet's 32-bit count) */
#define SHADOWTOPO_OPT_PRUNE_PENDANT 16   /* CSR rows of an undirected graph: 1 (default) = relax without the
                                              pendant trees that hold no attached vertex (peeled non-attached
                                              vertices with one neighbour; they lie on no attached-pair path);
                                              0 = every vertex. Results are identical. */
#define SHADOWTOPO_OPT_DEVICE_ROUNDS 17   /* CSR FULL worklist rounds: 1 (default) = driven from the device (item
                                              counts read back once per 8 rounds) when batches x vertices <= 1 Mi,
                                              2 = always, 0 = never (one host read-back per round). Results are
                                              identical. */
/* (18: retired -- batched delta-stepping rounds, measured slower and removed in r04) */
#define SHADOWTOPO_OPT_DELTA_LIVE 19      /* dense delta rounds over live-chunk lists (only the chunks holding a
                                            changed row): 2 (default) = when the previous round changed at most
                                            1/64 of the delta batches' pairs, 1 = always, 0 = never. Results are
                                            identical. */
#define SHADOWTOPO_OPT_DENSE_W16 20       /* pruned dense sweep: 1 = the chunk loop filters with 16-bit weights (fp16,
                                            rounded down; half the LDS slab and the table), 0 (default) = f32.
                                            Results are identical. */
#define SHADOWTOPO_OPT_SWEEP_PARTS 22     /* pruned dense sweep: the batches in 1 .. 4 parts (default 2), each part's chunk
                                            loop and exact pass on a stream of its own, so one part's exact pass overlaps
                                            another's chunk-loop tail. Results are identical. */
#define SHADOWTOPO_OPT_CHAIN_PARTS 23     /* with a sweep in parts and read-back-free rounds (OPT_DENSE_SPEC > 0): 1
                                            (default) enqueues those delta rounds on each part's stream behind its share of the
                                            sweep, the parts joining once before the read-back; 0 joins after the sweep.
                                            Results are identical. */
#define SHADOWTOPO_OPT_DENSE_SPEC 21      /* dense rounds: how many leading rounds (0..4, default 2) are enqueued with no
                                            host read-back of their change counts; a round decided without them runs
                                            the delta kernel over every batch that changed. Results are identical. */
#define SHADOWTOPO_OPT_HEAVY_FIRST 27       /* pruned dense sweep in parts: 1 (default) = each part's chunk-loop blocks
                                              in decreasing order of the chunks they staged in the previous sweep of
                                              the same shape (per XCD), 0 = grid order. Results are identical. */
#define SHADOWTOPO_OPT_WALK_TPW 28          /* path walks (vertex loss, multigraphs): k_walk takes 1 target per wave with one
                                              walk per lane (1, default) or 2 targets per wave, two walks per lane in
                                              lockstep (2). Results are identical. */
#define SHADOWTOPO_OPT_CSR_LEAN 30          /* sparse (CSR pull) rounds: 1 = lean -- the rounds keep d and the predecessor arc
                                              with a local-tie bit (12 B per (vertex, source) instead of 24), only a
                                              distance change activates the out-neighbours, and a walk of every pair's
                                              tree path after the rounds yields hops, reliability and the taint;
                                              0 = the tree fold inside the rounds; 2 (default) = lean when the relaxation
                                              graph has at least 32 arcs per attached vertex. Results are identical. */
#define SHADOWTOPO_OPT_CSR_INCREMENTAL 31   /* lean sparse rounds: n > 0 = a visit of a vertex with more than n in-arcs
                                              re-reads only the in-arcs whose tail's distance changed in the last two
                                              rounds (a per-(vertex, batch) change stamp), starting from the stored
                                              state (default 32); 0 = every in-arc. Results are identical. */
#define SHADOWTOPO_OPT_SPEC_COMPOSE 33      /* dense rounds: 1 (default) = the pair compose is enqueued behind each delta
                                              round, before its read-back, and kept when that round changed nothing
                                              (one host round trip fewer per computation); 0 = after convergence.
                                              Results are identical. */
#define SHADOWTOPO_OPT_SPIN_US 35           /* host waits on the device (between rounds, for the compose) poll for up to this
                                              many microseconds before a blocking wait (default 20000) */
#define SHADOWTOPO_OPT_HOST_GROUPS 36       /* rows into page-locked host memory: computed in this many batch groups, each
                                              group's copy behind the next group's rounds; 0 (default) = automatic (one
                                              group unless the rows outweigh the rounds). Results are identical. */
#define SHADOWTOPO_OPT_SWEEP_STATS 37       /* diagnostics: 1 = after each pruned two-part sweep, the chunks its blocks staged
                                              are summed into stats.sweep_chunks (one host synchronisation per sweep;
                                              0 = off, the default) */
#define SHADOWTOPO_OPT_SWEEP_WINDOWS 38     /* pruned dense sweep: the chunk windows whose skip masks are evaluated at once:
                                              bits 0-7 = the neighbour window after the tile's own chunk (default 8,
                                              0 = none), bits 8-15 = the far windows' size (default 0 = 64).
                                              Results are identical. */
#define SHADOWTOPO_OPT_SWEEP_GLDS 39        /* pruned dense sweep: the chunk loop stages its D32 rows and W32 slab by LDS-DMA
                                              (global_load_lds, 1) or through registers (0, the default). Results are identical. */
#define SHADOWTOPO_OPT_SWEEP_REFILTER 40    /* pruned dense sweep: the exact f64 pass first re-tests the rows the chunk loop
                                              logged against its FINAL f32 thresholds and drops those no lane passes
                                              (1) or evaluates every logged row (0, the default). Results are identical. */
#define SHADOWTOPO_OPT_SWEEP_WAVES 41       /* pruned dense sweep: the chunk loop's blocks are 4 waves x 8 destinations
                                              (4, the default) or 8 waves x 8 (8: one staged chunk serves 64 columns).
                                              Results are identical. */
#define SHADOWTOPO_OPT_SEED_SKIP 42         /* dense round 0: the exact pass leaves a pair whose seed candidate (the source's
                                              own arc) won untainted unread and unwritten -- the stored state is the seed's
                                              (1, the default) -- or re-reads and compares it (0). Results are identical. */
#define SHADOWTOPO_OPT_DELTA_W16 43         /* pruned dense delta rounds: the filter's W slabs in fp16 (W rounded toward -inf:
                                              half the slab bytes, a looser but still conservative filter; 1, the
                                              default) or f32 (0). Results are identical. */
#define SHADOWTOPO_OPT_PART0_PERMILLE 29   /* pruned dense sweep in two parts: per mille of the batches part 0 (launched first)
                                              takes (default 562). Results are identical. */
/* testing: the failure paths a convergence bug would take, reported as SHADOWTOPO_EINTERNAL
 * instead of faulting the device */
#define SHADOWTOPO_OPT_TEST_UNCONVERGED 24  /* 1 = when the iteration guard (OPT_MAX_ROUNDS) trips, compose the state
                                              the rounds stopped at (bounded path walks), then fail */
#define SHADOWTOPO_OPT_TEST_SCRAMBLE_TREE 25 /* 1 / 2 = overwrite every reached pair's predecessor arc before compose
                                               (1: past the arc range, 2: the vertex's first in-arc) */
#define SHADOWTOPO_OPT_TEST_POOL_ENOMEM 26  /* 1 = the next batch-pool allocation fails after its first buffer, as if
                                              another engine had taken the HBM (exercises the re-sized retry) */
#define SHADOWTOPO_OPT_HBM_SHARE 13         /* per mille of the batch-slot HBM budget (55 % of free HBM, at least 24 GB) this
                                              engine may take (default 1000); engines sharing one device split it */

/* sparse (CSR) relaxation rounds: every active vertex's minimum is recomputed over all its
 * in-arcs' 512-byte distance rows (k_relax; rounds with few active pairs run over frontier
 * worklists, k_relax_wl / k_relax_wlp).  Changed-tail variants (masked, stamped-key, delta)
 * read fewer rows but issued more instructions and were slower on every config;
 * they were removed in r03. */
#define SHADOWTOPO_CSR_FULL 1
/* push rounds (undirected graphs): distances pushed from changed (vertex, source) pairs along
 * their out-arcs with a 64-bit atomicMin on the f64 bit pattern, then one exact pull pass for
 * the predecessors and level rounds for hops / reliability */
#define SHADOWTOPO_CSR_PUSH 2

typedef struct shadowtopo_stats {
    int64_t n_vertices;
    int64_t n_edges;
    int64_t n_arcs;          /* non-loop arcs of the relaxation in-CSR after merging parallel edges */
    int64_t n_attached;
    int64_t sources;         /* source rows computed since the last reset */
    int64_t batches;
    int64_t rounds;          /* relaxation rounds (summed over batch groups) */
    int64_t relax_launches;
    int64_t replayed_sources;/* sources resolved by the heap-exact kernel (tie-tainted) */
    int64_t tainted_pairs;
    double relax_ms;         /* HIP-event time of relax launches (OPT_TIMING=1) */
    double compose_ms;
    double replay_ms;
    double wall_ms;          /* host wall time inside compute calls */
    int32_t device;
    int32_t multigraph;
    int32_t dense;           /* 1 = dense-tile relaxation in use */
    int32_t reserved;
    int64_t visits;          /* OPT_PROFILE, CSR: active (vertex, batch) waves processed */
    int64_t changes;         /* OPT_PROFILE: CSR: (vertex, batch) waves that changed;
                                dense: (vertex, source) pairs that changed */
    int64_t full_sweeps;     /* dense: full-sweep relax launches */
    int64_t delta_sweeps;    /* dense: change-mask (delta) relax launches */
    double full_ms;          /* OPT_TIMING: HIP-event time of the dense full sweeps (k_relax_dense) */
    double delta_ms;         /* OPT_TIMING: HIP-event time of the delta rounds (k_relax_dense_delta) */
    /* launch shapes, for the per-launch rooflines (bench.py) */
    int64_t full_batches;    /* dense: batches swept by full-sweep launches (summed over launches) */
    int64_t full_changes;    /* dense: (vertex, source) pairs those full sweeps changed */
    int64_t relax_batches;   /* sparse: batches in flight, summed over relax launches */
    int64_t wl_launches;     /* sparse: relax launches over frontier worklists (k_relax_wl), included above */
    double wl_ms;            /* OPT_TIMING: their HIP-event time, included in relax_ms */
    int64_t sparse_deltas;   /* dense: delta launches that walked live-chunk lists only */
    double self_ms;          /* host wall time of the self-path rule (k_self), once per attached set
                                (the reference's selfPathTotalTime, topology.c:1608-1617) */
    int64_t self_paths;      /* attached vertices the self-path rule ran for */
    int64_t pruned_deltas;   /* dense: delta launches in the locality order with chunk bounds (OPT_DENSE_PRUNE) */
    int64_t pruned_vertices; /* CSR: vertices the relaxation view leaves out (OPT_PRUNE_PENDANT) */
    int64_t pool_allocs;     /* batch-pool (re)allocations (a computation needing more slots than held) */
    double pool_alloc_ms;    /* host wall time of those allocations */
    /* cold start (kept across shadowtopo_reset_stats): host wall time of shadowtopo_create's
       edge validation, edge-list upload and device table build (dense tables included), and
       of the dense locality order built on the first computation */
    double create_validate_ms;
    double create_upload_ms;
    double create_build_ms;
    double order_ms;
    double create_alloc_ms;  /* of create_upload_ms: the device allocation of the edge buffers */
    int64_t groups;          /* batch groups computed (a computation's rows in groups of batches in flight) */
    double prepare_ms;       /* cold start: the device preparation's own wall time (shadowtopo_prepare:
                                HIP runtime and queue initialisation, staging buffers, code objects) */
    double create_prepare_wait_ms; /* of create_validate_ms: the part shadowtopo_create waited for it */
    int64_t group_batches;   /* batches in flight per group of the last computation (its largest group) */
    int64_t host_syncs;      /* host waits on the device inside the relaxation rounds (a round's counts
                                read back before the next launch; device-driven rounds: once per block) */
    double push_ms;          /* OPT_TIMING, CSR_PUSH: distance push rounds, predecessor pass, fold rounds */
    double pred_ms;
    double fold_ms;
    int64_t push_rounds;
    int64_t fold_rounds;
    int64_t packed_pairs;    /* row exchange codec: pairs packed, and of them sent explicitly */
    int64_t packed_explicit;
    double compose_kernel_ms; /* OPT_TIMING: HIP-event time of the pair compose (k_compose + k_walk) */
    int64_t walk_targets;    /* attached targets whose pairs take the full path fold (vertex loss, multigraphs) */
    double attach_prep_ms;   /* host wall time in compute calls of the work a new attached set needs first: the
                                relaxation view, the walk list and arc table, the pools, the source order */
    int64_t lean_groups;     /* batch groups computed with lean sparse rounds (OPT_CSR_LEAN) */
    int64_t spec_composes;   /* dense: composes enqueued behind the round that found convergence (OPT_SPEC_COMPOSE) */
    int64_t spec_composes_lost; /* dense: such composes redone because that round still changed pairs */
    int64_t sweep_chunks;       /* OPT_SWEEP_STATS: 32-row chunks the pruned sweeps' blocks staged */
    int64_t sweep_chunk_slots;  /* OPT_SWEEP_STATS: blocks x chunks of those sweeps (the unpruned count) */
    int64_t sweep_hit_rows;     /* OPT_SWEEP_STATS: rows the chunk loops logged for the exact f64 passes */
    int64_t relax_vertices;     /* vertices of the graph the rounds run on (the pendant-pruned view, if any) */
    int64_t relax_arcs;         /* its arcs */
} shadowtopo_stats;

/* Number of visible HIP devices (0 if none). */
int shadowtopo_device_count(void);

/*
 * Start preparing HIP device `device` on a background thread and return at once: the HIP
 * runtime's device and queue initialisation (~85 ms on MI355X, once per process), the
 * page-locked staging buffers of the edge upload, the engine's first stream and the loading
 * of this library's code objects.  shadowtopo_create starts it itself if nobody did and waits
 * for it after validating the edge list; a caller that knows a graph is coming (the shim,
 * before it parses the GraphML file) calls it first so the work overlaps the parse.
 * Idempotent per device.  Returns SHADOWTOPO_OK, or SHADOWTOPO_EINVAL for a bad ordinal.
 */
int shadowtopo_prepare(int32_t device);

/* Message for the last failing call on this thread. */
const char* shadowtopo_last_error(void);

/*
 * Build the device-resident graph from the GraphML edge list, in the reference's edge
 * order (edge index = <edge> element order, igraph_read_graph_graphml at topology.c:386).
 *   edge_source/edge_target : vertex indices in [0, n_vertices)
 *   edge_latency            : ms, > 0 (validated as topology.c:1066-1082 does)
 *   edge_packetloss         : in [0,1]
 *   vertex_packetloss       : nullable; NaN = attribute absent on that vertex
 *                             (topology.c:330-347, 1441-1462)
 *   flags                   : SHADOWTOPO_F_*
 *   device                  : HIP device ordinal
 */
int shadowtopo_create(int32_t n_vertices, int64_t n_edges, const int32_t* edge_source, const int32_t* edge_target,
                      const double* edge_latency, const double* edge_packetloss, const double* vertex_packetloss,
                      uint32_t flags, int32_t device, shadowtopo_engine** out);

void shadowtopo_destroy(shadowtopo_engine* eng);

/* The unique attached vertices (sources and targets), topology.c:1525-1543.  Row/column
 * i of every matrix refers to attached[i]. */
int shadowtopo_set_attached(shadowtopo_engine* eng, const int32_t* attached, int32_t count);

int shadowtopo_set_option(shadowtopo_engine* eng, int32_t key, int64_t value);

/*
 * Attached-pair rows [row_begin, row_end) x count: lat (ms), rel, hops, kind.
 * Buffers are row-major with leading dimension `count`; hops and kind may be NULL.
 * mem = SHADOWTOPO_MEM_DEVICE: device pointers on the engine's device, written on
 * `stream` (a hipStream_t, NULL = the engine's own stream); the call returns after the
 * stream work is complete.  mem = SHADOWTOPO_MEM_HOST: host pointers; when they are all
 * page-locked (shadowtopo_host_alloc) the rows are copied at full PCIe rate and a batch
 * group's copy overlaps the next group's computation.
 */
int shadowtopo_compute_rows(shadowtopo_engine* eng, int32_t row_begin, int32_t row_end, double* lat, double* rel,
                            uint32_t* hops, uint8_t* kind, int32_t mem, void* stream);

/* Page-locked host memory that compute_rows copies into directly (from any device of the
 * process); free with shadowtopo_host_free.  NULL-safe free. */
int shadowtopo_host_alloc(size_t bytes, void** out);
void shadowtopo_host_free(void* p);

/*
 * Parity tooling: full single-source results for arbitrary source vertices (row-major
 * [n_sources][n_vertices], host buffers, any may be NULL): distance (f64, +inf if
 * unreached), predecessor vertex (-1 for the source / unreached), hop count, and a
 * tie flag (1 if the vertex's shortest-path tree path crosses a heap-order tie).
 */
int shadowtopo_sssp(shadowtopo_engine* eng, const int32_t* sources, int32_t n_sources, double* dist, int32_t* pred,
                    uint32_t* hops, uint8_t* tie);

/* The version-independent self-path rule (_topology_computeShortestPathToSelf,
 * topology.c:1545-1653) for every attached vertex, host buffers of `count` entries (kind
 * SHADOWTOPO_KIND_SELF, or _NONE without an incident edge), whatever the engine's
 * F_SELF_DIJKSTRA_LOOP flag: under that flag the shim needs both values, because the
 * reference caches a self pair from whichever of the two rules runs first. */
int shadowtopo_self_rule_paths(shadowtopo_engine* eng, double* lat, double* rel, uint8_t* kind);

/* Row exchange codec (multi-GPU, shard.RowExchange; dense engines): the device rows
   [row_begin, row_end) x A of lat (f64), rel (f64) and hops (u32), row-major, are packed
   into `out` (device memory, at least shadowtopo_packed_capacity bytes): a bit per pair
   that equals the value every engine rebuilds from its own graph replica (the single arc
   from the source: latency 0 + w, one hop, reliability vfac(s) * the arc's factor, compared
   bit for bit), the other pairs in full. *out_bytes = the payload's size (the call waits
   for the stream).  shadowtopo_unpack_rows rebuilds the rows, bit-identical, on any engine
   created from the same graph and attached set.  Not part of the reference's interface:
   the exchange step SURVEY.md 8(e) adds, with 1/15 of C2's bytes at 8 ranks. */
/* Sparse row exchange (shard.RowExchange, any engine): hop counts (u32, device, n entries)
   narrowed to their low 16 bits `lo` (and the high 16 bits into `hi` when not NULL) for the
   all-gather, 18 instead of 20 bytes per pair; any count >= 2^16 ORs 1 into the device word
   *overflow (the exchange then moves `hi` too).  shadowtopo_hops_widen rebuilds the u32 counts
   (hi NULL: high halves zero).  Both are enqueued on `stream` (NULL: the engine's) without a
   wait.  Not part of the reference's interface. */
int shadowtopo_hops_narrow(shadowtopo_engine* eng, const uint32_t* hops, int64_t n, uint16_t* lo, uint16_t* hi,
                           uint32_t* overflow, void* stream);
int shadowtopo_hops_widen(shadowtopo_engine* eng, const uint16_t* lo, const uint16_t* hi, int64_t n, uint32_t* hops,
                          void* stream);
size_t shadowtopo_packed_capacity(int32_t rows, int32_t A);
int shadowtopo_pack_rows(shadowtopo_engine* eng, int32_t row_begin, int32_t row_end, const double* lat,
                         const double* rel, const uint32_t* hops, void* out, size_t cap, size_t* out_bytes,
                         void* stream);
int shadowtopo_unpack_rows(shadowtopo_engine* eng, int32_t row_begin, int32_t row_end, const void* in, double* lat,
                           double* rel, uint32_t* hops, void* stream);

int shadowtopo_get_stats(const shadowtopo_engine* eng, shadowtopo_stats* out);
void shadowtopo_reset_stats(shadowtopo_engine* eng);

/* effective completeness (caller's F_COMPLETE, or the reference rule under F_AUTO_COMPLETE) */
int shadowtopo_is_complete(const shadowtopo_engine* eng);

/* igraph_get_eid(directed = graph's, error = FALSE) as _topology_getEdgeHelper uses it
 * (topology.c:401-444): lowest edge id joining (from, to), or -1. */
int64_t shadowtopo_get_eid(const shadowtopo_engine* eng, int32_t from, int32_t to);

#ifdef __cplusplus
}
#endif

#endif /* SHADOWTOPO_H */
