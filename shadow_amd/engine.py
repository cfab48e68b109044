"""ctypes binding of libshadowtopo_hip (include/shadowtopo.h).

This is the Python-side mirror a maintainer would use to drive the engine (the C host
shim, topology_hip.c, is the drop-in for Shadow itself).  There is no CPU fallback:
if the HIP library is missing or no GPU is visible every call raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SHADOWTOPO_EXP_LIB: an experiment build of the same sources (_exp/build_variant.sh, e.g. the
# phase-stamp diagnostic) for A/B runs; the product, the tests and the bench load _build/
LIB_PATH = os.environ.get("SHADOWTOPO_EXP_LIB") or os.path.join(HERE, "_build", "libshadowtopo_hip.so")

F_DIRECTED = 0x1
F_COMPLETE = 0x2
F_PREFER_DIRECT = 0x4
F_SELF_DIJKSTRA_LOOP = 0x8
F_AUTO_COMPLETE = 0x10
F_FORCE_DENSE = 0x20
F_FORCE_CSR = 0x40

MEM_HOST = 0
MEM_DEVICE = 1
MEM_HOST_LR = 2  # host rows of interleaved {lat, rel} pairs (the shim's layout)

KIND_NONE, KIND_DIRECT, KIND_SELF, KIND_DIJKSTRA = 0, 1, 2, 3

OPT_BATCHES_IN_FLIGHT = 1
OPT_TIMING = 2
OPT_MAX_ROUNDS = 3
OPT_FORCE_REPLAY = 4
OPT_PROFILE = 5
OPT_DENSE_VARIANT = 6
DENSE_F32 = 0  # f32-filtered full sweep + lane-per-pair delta rounds (default)
DENSE_F64 = 1  # f64 row-stream kernels (cross-check)
OPT_DELTA_PERMILLE = 7
OPT_CSR_VARIANT = 8
OPT_DENSE_BATCHES_PER_WAVE = 9
OPT_SOURCE_ORDER = 10
OPT_DENSE_SEED = 11
OPT_DENSE_PRUNE = 12
OPT_HBM_SHARE = 13
OPT_WORKLIST = 14
OPT_GRID_X = 15
OPT_PRUNE_PENDANT = 16
OPT_DEVICE_ROUNDS = 17
OPT_DENSE_W16 = 20  # pruned dense sweep: 16-bit filter weights in the chunk loop (1) or f32 (0, default)
OPT_CHAIN_PARTS = 23  # the read-back-free delta rounds on each sweep part's stream (1, default) or after the join (0)
OPT_SWEEP_PARTS = 22  # pruned dense sweep: batches in 1 .. 4 parts (default 2) on their own streams
OPT_DENSE_SPEC = 21  # dense: leading rounds enqueued without a host read-back (0..4, default 2)
OPT_DELTA_LIVE = 19  # dense delta rounds over live-chunk lists: 2 when sparse (default), 1 always, 0 never
OPT_WALK_TPW = 28  # path walks: 1 target per wave, one walk per lane (1, default) or 2 targets, two walks per lane (2)
OPT_CSR_LEAN = 30  # sparse rounds: lean D + predecessor state and a walk per pair (1), tree fold (0), auto (2, default)
OPT_CSR_INCREMENTAL = 31  # lean rounds: visits of vertices with more than n in-arcs re-read only fresh tails (default 32, 0 = off)
OPT_SPEC_COMPOSE = 33  # dense: compose enqueued behind each delta round, kept at convergence (1, default)
OPT_SPIN_US = 35  # host waits poll this many microseconds before blocking (default 20000)
OPT_HOST_GROUPS = 36  # page-locked host rows: batch groups (0 = automatic)
OPT_SWEEP_WINDOWS = 38  # pruned dense sweep: neighbour window (bits 0-7, default 8) | far window size << 8 (0 = 64)
OPT_SWEEP_GLDS = 39  # pruned dense sweep chunk loop: LDS-DMA staging (1) or register staging (0, default)
OPT_SWEEP_REFILTER = 40  # pruned dense sweep: exact pass re-tests logged rows against the final f32 thresholds (1) or not (0, default)
OPT_SWEEP_WAVES = 41  # pruned dense sweep chunk loop: 4 (default) or 8 waves per block
OPT_DELTA_W16 = 43  # pruned dense delta rounds: fp16 slabs in the filter (1, default) or f32 (0)
OPT_SEED_SKIP = 42  # dense round 0: untainted seed winners left unread by the exact pass (1, default) or compared (0)
OPT_SWEEP_STATS = 37  # diagnostics: chunks staged by the pruned sweeps into stats sweep_chunks / sweep_chunk_slots
OPT_PART0_PERMILLE = 29  # two sweep parts: part 0's share of the batches, per mille (default 562)
OPT_HEAVY_FIRST = 27  # pruned sweep parts: heavy-first block order from the previous sweep (1, default) or grid order
# testing: the failure paths a convergence bug or a full device would take (SHADOWTOPO_EINTERNAL /
# the re-sized pool retry instead of a fault)
OPT_TEST_UNCONVERGED = 24  # compose the state the iteration guard stopped at, then fail
OPT_TEST_SCRAMBLE_TREE = 25  # 1 / 2: predecessors overwritten before compose (out of range / not a tree)
OPT_TEST_POOL_ENOMEM = 26  # the next batch-pool allocation fails midway (ENOMEM retry)
CSR_FULL = 1  # pull: recompute every active vertex over all in-arcs (k_relax / k_relax_wl, default)
CSR_PUSH = 2  # push: distance pushes with a u64 atomicMin, then a predecessor pass and fold rounds (undirected)

# every symbol include/shadowtopo.h declares
ENGINE_SYMBOLS = (
    "shadowtopo_device_count", "shadowtopo_prepare", "shadowtopo_last_error", "shadowtopo_create", "shadowtopo_destroy",
    "shadowtopo_set_attached", "shadowtopo_set_option", "shadowtopo_compute_rows", "shadowtopo_sssp",
    "shadowtopo_get_stats", "shadowtopo_reset_stats", "shadowtopo_is_complete", "shadowtopo_get_eid",
    "shadowtopo_host_alloc", "shadowtopo_host_free", "shadowtopo_self_rule_paths",
    "shadowtopo_packed_capacity", "shadowtopo_pack_rows", "shadowtopo_unpack_rows",
    "shadowtopo_hops_narrow", "shadowtopo_hops_widen",
)


class ShadowTopoError(RuntimeError):
    pass


class Stats(ctypes.Structure):
    _fields_ = [
        ("n_vertices", ctypes.c_int64), ("n_edges", ctypes.c_int64), ("n_arcs", ctypes.c_int64),
        ("n_attached", ctypes.c_int64), ("sources", ctypes.c_int64), ("batches", ctypes.c_int64),
        ("rounds", ctypes.c_int64), ("relax_launches", ctypes.c_int64), ("replayed_sources", ctypes.c_int64),
        ("tainted_pairs", ctypes.c_int64), ("relax_ms", ctypes.c_double), ("compose_ms", ctypes.c_double),
        ("replay_ms", ctypes.c_double), ("wall_ms", ctypes.c_double), ("device", ctypes.c_int32),
        ("multigraph", ctypes.c_int32), ("dense", ctypes.c_int32), ("reserved", ctypes.c_int32),
        ("visits", ctypes.c_int64), ("changes", ctypes.c_int64),
        ("full_sweeps", ctypes.c_int64), ("delta_sweeps", ctypes.c_int64),
        ("full_ms", ctypes.c_double), ("delta_ms", ctypes.c_double),
        ("full_batches", ctypes.c_int64), ("full_changes", ctypes.c_int64), ("relax_batches", ctypes.c_int64),
        ("wl_launches", ctypes.c_int64), ("wl_ms", ctypes.c_double), ("sparse_deltas", ctypes.c_int64),
        ("self_ms", ctypes.c_double), ("self_paths", ctypes.c_int64), ("pruned_deltas", ctypes.c_int64),
        ("pruned_vertices", ctypes.c_int64), ("pool_allocs", ctypes.c_int64), ("pool_alloc_ms", ctypes.c_double),
        ("create_validate_ms", ctypes.c_double), ("create_upload_ms", ctypes.c_double),
        ("create_build_ms", ctypes.c_double), ("order_ms", ctypes.c_double),
        ("create_alloc_ms", ctypes.c_double), ("groups", ctypes.c_int64),
        ("prepare_ms", ctypes.c_double), ("create_prepare_wait_ms", ctypes.c_double),
        ("group_batches", ctypes.c_int64), ("host_syncs", ctypes.c_int64),
        ("push_ms", ctypes.c_double), ("pred_ms", ctypes.c_double), ("fold_ms", ctypes.c_double),
        ("push_rounds", ctypes.c_int64), ("fold_rounds", ctypes.c_int64),
        ("packed_pairs", ctypes.c_int64), ("packed_explicit", ctypes.c_int64),
        ("compose_kernel_ms", ctypes.c_double), ("walk_targets", ctypes.c_int64),
        ("attach_prep_ms", ctypes.c_double), ("lean_groups", ctypes.c_int64),
        ("spec_composes", ctypes.c_int64), ("spec_composes_lost", ctypes.c_int64),
        ("sweep_chunks", ctypes.c_int64), ("sweep_chunk_slots", ctypes.c_int64), ("sweep_hit_rows", ctypes.c_int64),
        ("relax_vertices", ctypes.c_int64), ("relax_arcs", ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def lib():
    """Load the in-tree HIP library (built by __graft_entry__.build()); raise if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ShadowTopoError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        vp = ctypes.c_void_p
        L.shadowtopo_device_count.restype = ctypes.c_int
        L.shadowtopo_prepare.restype = ctypes.c_int
        L.shadowtopo_prepare.argtypes = [ctypes.c_int32]
        L.shadowtopo_last_error.restype = ctypes.c_char_p
        L.shadowtopo_create.restype = ctypes.c_int
        L.shadowtopo_create.argtypes = [ctypes.c_int32, ctypes.c_int64, vp, vp, vp, vp, vp, ctypes.c_uint32,
                                        ctypes.c_int32, ctypes.POINTER(vp)]
        L.shadowtopo_destroy.argtypes = [vp]
        L.shadowtopo_set_attached.argtypes = [vp, vp, ctypes.c_int32]
        L.shadowtopo_set_option.argtypes = [vp, ctypes.c_int32, ctypes.c_int64]
        L.shadowtopo_compute_rows.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, ctypes.c_int32, vp]
        L.shadowtopo_sssp.argtypes = [vp, vp, ctypes.c_int32, vp, vp, vp, vp]
        L.shadowtopo_get_stats.argtypes = [vp, ctypes.POINTER(Stats)]
        L.shadowtopo_self_rule_paths.argtypes = [vp, vp, vp, vp]
        L.shadowtopo_packed_capacity.restype = ctypes.c_size_t
        L.shadowtopo_packed_capacity.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.shadowtopo_pack_rows.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t), vp]
        L.shadowtopo_unpack_rows.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp]
        L.shadowtopo_hops_narrow.argtypes = [vp, vp, ctypes.c_int64, vp, vp, vp, vp]
        L.shadowtopo_hops_widen.argtypes = [vp, vp, vp, ctypes.c_int64, vp, vp]
        L.shadowtopo_reset_stats.argtypes = [vp]
        L.shadowtopo_is_complete.argtypes = [vp]
        L.shadowtopo_get_eid.restype = ctypes.c_int64
        L.shadowtopo_get_eid.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.shadowtopo_host_alloc.restype = ctypes.c_int
        L.shadowtopo_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(vp)]
        L.shadowtopo_host_free.argtypes = [vp]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        msg = lib().shadowtopo_last_error()
        raise ShadowTopoError(f"shadowtopo error {rc}: {msg.decode() if msg else ''}")


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class _Pinned:
    """page-locked host allocation (shadowtopo_host_alloc), freed with the last array view"""

    def __init__(self, nbytes):
        self.p = ctypes.c_void_p()
        _check(lib().shadowtopo_host_alloc(max(1, int(nbytes)), ctypes.byref(self.p)))
        self.nbytes = int(nbytes)

    def __del__(self):
        if self.p:
            lib().shadowtopo_host_free(self.p)
            self.p = None


def pinned_empty(shape, dtype):
    """numpy array in page-locked host memory (what the topology shim allocates its matrix
    in): compute_rows copies into it at full PCIe rate"""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    buf = _Pinned(n)
    raw = (ctypes.c_uint8 * max(1, n)).from_address(buf.p.value)
    raw._owner = buf  # the allocation lives as long as any view of it
    return np.frombuffer(raw, dtype=dtype, count=int(np.prod(shape))).reshape(shape)


def device_count():
    return int(lib().shadowtopo_device_count())


def prepare(device=0):
    """Start the device preparation on a background thread (shadowtopo_prepare)."""
    rc = lib().shadowtopo_prepare(int(device))
    if rc != 0:
        raise ShadowTopoError(f"shadowtopo_prepare: {lib().shadowtopo_last_error().decode()}")


class Engine:
    """Device-resident topology graph + attached-pair computation."""

    def __init__(self, n, src, dst, latency, packetloss, vertex_packetloss=None, directed=False,
                 prefer_direct=False, complete=None, self_dijkstra_loop=False, device=0, layout="auto"):
        L = lib()
        self._keep = []
        src = np.ascontiguousarray(src, np.int32)
        dst = np.ascontiguousarray(dst, np.int32)
        lat = np.ascontiguousarray(latency, np.float64)
        loss = np.ascontiguousarray(packetloss, np.float64)
        vl = None if vertex_packetloss is None else np.ascontiguousarray(vertex_packetloss, np.float64)
        flags = 0
        if directed:
            flags |= F_DIRECTED
        if prefer_direct:
            flags |= F_PREFER_DIRECT
        if self_dijkstra_loop:
            flags |= F_SELF_DIJKSTRA_LOOP
        if layout == "dense":
            flags |= F_FORCE_DENSE
        elif layout == "csr":
            flags |= F_FORCE_CSR
        if complete is None:
            flags |= F_AUTO_COMPLETE
        elif complete:
            flags |= F_COMPLETE
        h = ctypes.c_void_p()
        _check(L.shadowtopo_create(int(n), len(src), _ptr(src), _ptr(dst), _ptr(lat), _ptr(loss), _ptr(vl), flags,
                                   int(device), ctypes.byref(h)))
        self._h = h
        self.n = int(n)
        self.device = int(device)
        self.A = 0

    @classmethod
    def from_synth(cls, g, device=0, **kw):
        return cls(g.n, g.src, g.dst, g.latency, g.packetloss, g.vertex_packetloss, directed=g.directed,
                   prefer_direct=g.prefer_direct, device=device, **kw)

    def close(self):
        if getattr(self, "_h", None):
            lib().shadowtopo_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def complete(self):
        return bool(lib().shadowtopo_is_complete(self._h))

    def get_eid(self, a, b):
        return int(lib().shadowtopo_get_eid(self._h, int(a), int(b)))

    def set_attached(self, attached):
        att = np.ascontiguousarray(attached, np.int32)
        _check(lib().shadowtopo_set_attached(self._h, _ptr(att), len(att)))
        self.A = len(att)
        self.attached = att

    def set_option(self, key, value):
        _check(lib().shadowtopo_set_option(self._h, int(key), int(value)))

    def compute_rows(self, row_begin=0, row_end=None, want_kind=True, want_hops=True, pinned=False):
        """host numpy outputs: lat, rel, hops, kind for rows [row_begin, row_end); pinned=True
        puts them in page-locked memory (the shim's layout and copy path); hops / kind are
        None when not wanted"""
        if row_end is None:
            row_end = self.A
        R = row_end - row_begin
        mk = pinned_empty if pinned else np.empty
        lat = mk((R, self.A), np.float64)
        rel = mk((R, self.A), np.float64)
        hops = mk((R, self.A), np.uint32) if want_hops else None
        kind = mk((R, self.A), np.uint8) if want_kind else None
        self.compute_rows_into(row_begin, row_end, lat, rel, hops, kind)
        return lat, rel, hops, kind

    def compute_rows_into(self, row_begin, row_end, lat, rel, hops=None, kind=None):
        """rows [row_begin, row_end) into caller-owned host arrays ([rows, A], C order)"""
        for a, dt in ((lat, np.float64), (rel, np.float64), (hops, np.uint32), (kind, np.uint8)):
            if a is not None and (a.dtype != dt or not a.flags.c_contiguous or a.size < (row_end - row_begin) * self.A):
                raise ValueError("output arrays must be C-contiguous [rows, A] of the right dtype")
        _check(lib().shadowtopo_compute_rows(self._h, int(row_begin), int(row_end), _ptr(lat), _ptr(rel), _ptr(hops),
                                             _ptr(kind), MEM_HOST, None))

    def compute_rows_lr(self, row_begin=0, row_end=None, pinned=True):
        """host rows of interleaved {lat, rel} pairs ([rows, A, 2] float64, MEM_HOST_LR: the
        topology shim's matrix layout) and the pair kinds"""
        if row_end is None:
            row_end = self.A
        R = row_end - row_begin
        mk = pinned_empty if pinned else np.empty
        lr = mk((R, self.A, 2), np.float64)
        kind = mk((R, self.A), np.uint8)
        _check(lib().shadowtopo_compute_rows(self._h, int(row_begin), int(row_end), _ptr(lr), None, None, _ptr(kind),
                                             MEM_HOST_LR, None))
        return lr, kind

    def compute_rows_device(self, row_begin, row_end, lat_ptr, rel_ptr, hops_ptr, kind_ptr=None, stream=None):
        """device outputs (raw pointers, e.g. torch tensors' data_ptr()) on `stream`"""
        vp = ctypes.c_void_p
        _check(lib().shadowtopo_compute_rows(self._h, int(row_begin), int(row_end), vp(lat_ptr), vp(rel_ptr),
                                             vp(hops_ptr), vp(kind_ptr) if kind_ptr else None, MEM_DEVICE,
                                             vp(stream) if stream else None))

    @staticmethod
    def packed_capacity(rows, A):
        """bytes a packed row block of `rows` x A pairs may need (shadowtopo_pack_rows)"""
        return int(lib().shadowtopo_packed_capacity(int(rows), int(A)))

    def pack_rows(self, row_begin, row_end, lat_ptr, rel_ptr, hops_ptr, out_ptr, cap, stream=None):
        """pack device rows [row_begin, row_end) into the device buffer out_ptr; returns the
        payload's bytes (waits for the stream)"""
        vp = ctypes.c_void_p
        n = ctypes.c_size_t(0)
        _check(lib().shadowtopo_pack_rows(self._h, int(row_begin), int(row_end), vp(lat_ptr), vp(rel_ptr), vp(hops_ptr),
                                          vp(out_ptr), int(cap), ctypes.byref(n), vp(stream) if stream else None))
        return int(n.value)

    def unpack_rows(self, row_begin, row_end, in_ptr, lat_ptr, rel_ptr, hops_ptr, stream=None):
        vp = ctypes.c_void_p
        _check(lib().shadowtopo_unpack_rows(self._h, int(row_begin), int(row_end), vp(in_ptr), vp(lat_ptr),
                                            vp(rel_ptr), vp(hops_ptr), vp(stream) if stream else None))

    def hops_narrow(self, hops_ptr, n, lo_ptr, hi_ptr, overflow_ptr, stream=None):
        """device hop counts -> low / high 16-bit halves, OR 1 into *overflow_ptr if any count
        is >= 2^16 (the sparse row exchange; enqueued, no wait)"""
        vp = ctypes.c_void_p
        _check(lib().shadowtopo_hops_narrow(self._h, vp(hops_ptr), int(n), vp(lo_ptr), vp(hi_ptr) if hi_ptr else None,
                                            vp(overflow_ptr), vp(stream) if stream else None))

    def hops_widen(self, lo_ptr, hi_ptr, n, hops_ptr, stream=None):
        vp = ctypes.c_void_p
        _check(lib().shadowtopo_hops_widen(self._h, vp(lo_ptr), vp(hi_ptr) if hi_ptr else None, int(n), vp(hops_ptr),
                                           vp(stream) if stream else None))

    def sssp(self, sources):
        s = np.ascontiguousarray(sources, np.int32)
        k = len(s)
        dist = np.empty((k, self.n), np.float64)
        pred = np.empty((k, self.n), np.int32)
        hops = np.empty((k, self.n), np.uint32)
        tie = np.empty((k, self.n), np.uint8)
        _check(lib().shadowtopo_sssp(self._h, _ptr(s), k, _ptr(dist), _ptr(pred), _ptr(hops), _ptr(tie)))
        return dist, pred, hops, tie

    def self_rule_paths(self):
        """the version-independent self-path rule for every attached vertex (lat, rel, kind)"""
        lat = np.empty(self.A, np.float64)
        rel = np.empty(self.A, np.float64)
        kind = np.empty(self.A, np.uint8)
        _check(lib().shadowtopo_self_rule_paths(self._h, _ptr(lat), _ptr(rel), _ptr(kind)))
        return lat, rel, kind

    def stats(self):
        st = Stats()
        _check(lib().shadowtopo_get_stats(self._h, ctypes.byref(st)))
        return st.as_dict()

    def reset_stats(self):
        lib().shadowtopo_reset_stats(self._h)
