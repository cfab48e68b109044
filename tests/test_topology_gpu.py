"""GPU: the drop-in topology API (topology_hip.h) end to end -- GraphML -> validation ->
attach -> per-packet getters -- against the oracle and the reference's own fixtures."""
import json
import lzma
import os

import numpy as np
import pytest

from oracle.path_cache_ref import RefPathCache, adjacency_of, entry_value
from paritylib import oracle_matrix
from shadow_amd import synth
from shadow_amd import topology as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def quiet():
    T.set_log_level(1)


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def with_vertex_ips(g):
    ips = [f"10.{(v >> 16) & 255}.{(v >> 8) & 255}.{(v & 255)}" if (v & 255) else f"10.{200 + ((v >> 16) & 7)}.{(v >> 8) & 255}.1"
           for v in range(g.n)]
    return {"ip": ("d1", "string", ips)}, ips


def attach_all(top, ips, vertices, base=0):
    """one host per vertex, pinned by an exact IP hint; host IPs in 11.x"""
    r = T.Random(7)
    hosts = []
    for k, v in enumerate(vertices, start=base):
        a = T.Address(f"11.{(k >> 16) & 255}.{(k >> 8) & 255}.{k & 255}")
        top.attach(a, r, ipHint=ips[v])
        assert top.vertex_of_ip(a.ip) == v
        hosts.append(a)
    return hosts


def ref_cache(g, lat_o, kind_o, complete=False):
    # directed graphs as the reference: (s, t) is refused once (t, s) is cached, and the query
    # (s, t) is then answered with the (t, s) Path (topology.c:1311-1317, :2033-2038)
    model = RefPathCache(lat_o, kind_o, directed=g.directed, complete=complete, prefer_direct=bool(g.prefer_direct),
                         adjacent=adjacency_of(g))
    model.calls0 = T.min_time_jump_calls()  # the stand-in's upcall count before the first query
    return model


def check_cache_state(top, model):
    """what the reference's path cache would hold after the same queries: the count of
    cached Paths, Dijkstra and self-path runs, and the minimum handed to the simulator"""
    inf = top.info()
    assert inf["cached_paths"] == len(model.cache)
    assert inf["dijkstra_runs"] == model.dijkstra_runs
    assert inf["self_path_count"] == model.self_paths
    assert inf["min_path_latency"] == model.min_latency
    if model.upcalls:
        assert T.last_min_time_jump() == model.upcalls[-1]
    # one upcall per store that lowered the minimum, as _topology_storePathInCache makes them
    # (topology.c:1374-1385), not one per miss
    assert T.min_time_jump_calls() - model.calls0 == len(model.upcalls), (T.min_time_jump_calls() - model.calls0,
                                                                             model.upcalls)


def check_against_oracle(tmp_path, g, n_hosts=None):
    """every ordered pair, queried row by row: each getter returns the entry of the Path the
    reference has cached for the pair (its own row's value, or the reverse direction's
    when the other host's Dijkstra ran first: topology.c:1983-1990)"""
    va, ips = with_vertex_ips(g)
    text = synth.to_graphml(g, extra_vattr=va, prefer_direct=("true" if g.prefer_direct else None))
    top = T.Topology.new(write(tmp_path, "g.xml", text))
    assert top is not None
    hosts = attach_all(top, ips, g.attached)
    lat_o, rel_o, hops_o, kind_o, _ = oracle_matrix(g)
    model = ref_cache(g, lat_o, kind_o)
    reversed_seen = 0
    for i, a in enumerate(hosts):
        for j, b in enumerate(hosts):
            # one model lookup per getter call: a directed pair whose reverse holds the cache
            # misses (and reruns a Dijkstra) on every call, as in the reference
            path = model.get_path_entry(i, j)
            if path is None:  # unroutable (a directed graph's unreachable pair)
                assert g.directed and top.getLatency(a, b) == -1.0, (i, j)
                assert model.get_path_entry(i, j) is None and not top.isRoutable(a, b), (i, j)
                continue
            si, sj = path
            reversed_seen += (si, sj) != (i, j)
            lat = top.getLatency(a, b)
            assert lat == lat_o[si, sj], (i, j, lat, lat_o[si, sj])
            assert model.get_path_entry(i, j) == path and top.getReliability(a, b) == rel_o[si, sj]
            assert model.get_path_entry(i, j) == path and top.isRoutable(a, b)
    inf = top.info()
    assert inf["computed_for"] == len(hosts)
    check_cache_state(top, model)
    # the lower triangle came from the upper one's Paths -- in a directed graph too, through
    # the post-computation fallback (topology.c:2033-2038)
    assert reversed_seen > 0
    return top, hosts, model


def test_sparse_graph_all_pairs(tmp_path):
    g = synth.random_sparse(V=180, avg_deg=4, seed=41, A=60)
    top, _, _ = check_against_oracle(tmp_path, g)
    top.free()


def test_directed_graph_all_pairs(tmp_path):
    """directed: once (t, s) is cached the reference refuses (s, t) (topology.c:1311-1317), so
    the query (s, t) misses every time, reruns s's Dijkstra and gets the (t, s) Path; the
    drop-in's getters, cached set and Dijkstra count follow it"""
    g = synth.random_sparse(V=150, avg_deg=4, seed=47, A=40, directed=True)
    top, hosts, model = check_against_oracle(tmp_path, g)
    i, j = next((i, j) for (j, i) in sorted(model.cache) if i != j and (i, j) not in model.cache)
    a, b = hosts[i], hosts[j]
    runs = top.info()["dijkstra_runs"]
    assert top.getLatency(a, b) == top.getLatency(b, a)  # (j, i) holds the pair
    assert top.info()["dijkstra_runs"] == runs + 1  # (i, j) missed and reran i's Dijkstra
    top.incrementPathPacketCounter(a, b)  # counted on the (j, i) Path
    va, vb = top.vertex_of_ip(a.ip), top.vertex_of_ip(b.ip)
    assert top.packet_count(vb, va) == 1 and top.packet_count(va, vb) == 0
    top.free()


def test_prefer_direct_graph(tmp_path):
    g = synth.random_sparse(V=120, avg_deg=6, seed=42, A=50)
    g.prefer_direct = True
    top, _, _ = check_against_oracle(tmp_path, g)
    assert top.info()["prefers_direct_paths"] == 1
    top.free()


def test_vertex_loss_graph(tmp_path):
    rng = np.random.default_rng(1)
    g = synth.random_sparse(V=120, avg_deg=4, seed=43, A=40, vloss=rng.uniform(0, 0.05, 120))
    top, _, _ = check_against_oracle(tmp_path, g)
    top.free()


def test_packet_counters_one_per_unordered_pair(tmp_path):
    g = synth.random_sparse(V=60, avg_deg=4, seed=44, A=10)
    top, hosts, _ = check_against_oracle(tmp_path, g)
    a, b, c = hosts[0], hosts[1], hosts[2]
    for _ in range(3):
        top.incrementPathPacketCounter(a, b)
    top.incrementPathPacketCounter(b, a)
    top.incrementPathPacketCounter(c, c)
    va, vb, vc = (top.vertex_of_ip(h.ip) for h in (a, b, c))
    assert top.packet_count(va, vb) == 4 == top.packet_count(vb, va)
    assert top.packet_count(vc, vc) == 1
    assert top.packet_count(va, vc) == 0
    top.free()


def test_shipped_topology_complete_direct_rule(tmp_path):
    text = lzma.open(os.path.join(GOLD, "c1_topology.graphml.xml.xz"), "rt").read()
    top = T.Topology.new(write(tmp_path, "c1.xml", text))
    gold = np.load(os.path.join(GOLD, "c1_direct.npz"))
    r = T.Random(99)
    hosts = [T.Address(f"11.0.{k // 200}.{k % 200 + 1}") for k in range(400)]
    for h in hosts:
        top.attach(h, r, countrycodeHint=None)
    verts = [top.vertex_of_ip(h.ip) for h in hosts]
    for i in range(0, 400, 7):
        for j in range(0, 400, 5):
            a, b = hosts[i], hosts[j]
            assert top.getLatency(a, b) == gold["lat"][verts[i], verts[j]]
            assert top.getReliability(a, b) == gold["rel"][verts[i], verts[j]]
    assert top.info()["is_complete"] == 1
    top.free()


def test_reference_test_topologies(tmp_path):
    """the 1-vertex graphs of resource/examples/shadow.config.xml and src/test/**: two
    hosts on the one vertex (the tgen client/server example)"""
    for k, case in enumerate(json.load(open(os.path.join(GOLD, "ref_test_graphs.json")))):
        top = T.Topology.new(write(tmp_path, f"t{k}.xml", case["graphml"]))
        assert top is not None
        r = T.Random(1)
        server, client = T.Address("11.0.0.1", "server"), T.Address("11.0.0.2", "client")
        top.attach(server, r)
        top.attach(client, r)
        assert top.getLatency(client, server) == case["self_latency"] == 50.0
        assert top.getReliability(client, server) == case["self_reliability"]
        assert top.getLatency(server, server) == 50.0
        top.free()


def _subset(g, k):
    import copy
    h = copy.copy(g)
    h.attached = g.attached[:k]
    return h


@pytest.mark.parametrize("directed", [False, True])
def test_late_attach_keeps_counters_and_values(tmp_path, directed):
    """hosts attached after the first query: an undirected graph computes the new rows (old
    rows get their own entries for the new targets only once an old host's Dijkstra would
    run again), a directed graph recomputes every row; every getter returns the entry of
    the Path the reference has cached at that point, and packet counters survive both late
    attaches"""
    g = synth.random_sparse(V=90, avg_deg=4, seed=45, A=30, directed=directed)
    g26 = _subset(g, 26)
    lat_o, rel_o, _, kind_o, _ = oracle_matrix(g26)
    model = ref_cache(g26, lat_o, kind_o)
    va, ips = with_vertex_ips(g)
    top = T.Topology.new(write(tmp_path, "l.xml", synth.to_graphml(g, extra_vattr=va)))
    hosts = attach_all(top, ips, g.attached[:10])
    vx = [top.vertex_of_ip(h.ip) for h in hosts]

    # every drop-in query is mirrored by one model lookup: in a directed graph a pair whose
    # reverse holds the cache misses (and reruns a Dijkstra) on every call
    def q(i, j, a, b):
        path = model.get_path_entry(i, j)
        got = top.getLatency(a, b)
        if path is None:  # unroutable (directed graphs)
            assert got == -1.0 and model.get_path_entry(i, j) is None and top.getReliability(a, b) == -1.0, (i, j)
            return got
        si, sj = path
        assert got == lat_o[si, sj], (i, j, si, sj)
        assert model.get_path_entry(i, j) == path and top.getReliability(a, b) == rel_o[si, sj], (i, j)
        return got

    def inc(i, j, a, b):
        model.get_path_entry(i, j)
        top.incrementPathPacketCounter(a, b)

    model.A = 10
    l01 = q(0, 1, hosts[0], hosts[1])
    for _ in range(3):
        inc(0, 1, hosts[0], hosts[1])
    inc(2, 5, hosts[2], hosts[5])
    q(2, 5, hosts[2], hosts[5])
    assert top.info()["computed_for"] == 10
    more = attach_all(top, ips, g.attached[10:20], base=100)
    model.A = 20
    q(0, 11, hosts[0], more[1])  # host 0's Dijkstra again: its own row for the new targets
    assert top.info()["computed_for"] == 20
    assert q(0, 1, hosts[0], hosts[1]) == l01
    q(13, 4, more[3], hosts[4])  # new source, old target
    q(4, 13, hosts[4], more[3])
    inc(0, 1, hosts[0], hosts[1])
    inc(10, 3, more[0], hosts[3])
    assert top.packet_count(vx[0], vx[1]) == 4
    assert top.packet_count(vx[2], vx[5]) == 1
    even_more = attach_all(top, ips, g.attached[20:26], base=200)
    model.A = 26
    inc(20, 0, even_more[0], hosts[0])
    assert top.info()["computed_for"] == 26
    assert top.packet_count(vx[0], vx[1]) == 4
    assert top.packet_count(top.vertex_of_ip(more[0].ip), vx[3]) == 1
    assert top.packet_count(top.vertex_of_ip(even_more[0].ip), vx[0]) == 1
    all_hosts = hosts + more + even_more
    for i, a in enumerate(all_hosts):
        for j, b in enumerate(all_hosts):
            q(i, j, a, b)
    check_cache_state(top, model)
    top.free()


def test_two_late_attaches_old_rows_get_own_entries(tmp_path):
    """two late attaches with no old-source miss between them.  The second
    late-attach matrix copies the first one's old rows, reverse copies included; the first
    Dijkstra of an old source afterwards must cache its OWN entries for the middle block of
    targets (attached by the first late attach) too, not the reverse copies."""
    g = synth.random_sparse(V=90, avg_deg=4, seed=45, A=30)
    g26 = _subset(g, 26)
    lat_o, rel_o, _, kind_o, _ = oracle_matrix(g26)
    # an old source i and a middle target t whose two directions differ in the last bits
    pairs = [(i, t) for i in range(10) for t in range(10, 20)
             if kind_o[i, t] == 3 and (lat_o[i, t] != lat_o[t, i] or rel_o[i, t] != rel_o[t, i])]
    assert pairs, "fixture graph has no asymmetric old/middle pair"
    i0, t0 = pairs[0]
    model = ref_cache(g26, lat_o, kind_o)
    va, ips = with_vertex_ips(g)
    top = T.Topology.new(write(tmp_path, "l2.xml", synth.to_graphml(g, extra_vattr=va)))
    hosts = attach_all(top, ips, g.attached[:10])

    def q(i, j):
        a, b = all_hosts[i], all_hosts[j]
        si, sj = model.get_path_entry(i, j)
        assert top.getLatency(a, b) == lat_o[si, sj], (i, j, si, sj)
        model.get_path_entry(i, j)
        assert top.getReliability(a, b) == rel_o[si, sj], (i, j, si, sj)

    all_hosts = list(hosts)
    model.A = 10
    j0 = next(j for j in range(10) if j != i0)
    q(j0, j0 ^ 1 if (j0 ^ 1) != i0 else (j0 + 2) % 10)  # a Dijkstra of another old source
    all_hosts += attach_all(top, ips, g.attached[10:20], base=100)
    model.A = 20
    s2 = next(s for s in range(10, 20) if s != t0)
    q(s2, j0)  # a new source: the first late-attach matrix, never filled
    all_hosts += attach_all(top, ips, g.attached[20:26], base=200)
    model.A = 26
    q(20, j0)  # the second late-attach matrix, copied from the unfilled one
    assert top.info()["computed_for"] == 26
    q(i0, t0)  # i0's Dijkstra: its own (i0, t0) entry
    q(t0, i0)  # answered with the cached (i0, t0) Path
    for i in range(26):
        for j in range(26):
            q(i, j)
    check_cache_state(top, model)
    top.free()


def test_cache_emulation_upcalls_and_teardown_log(tmp_path, capfd):
    """the drop-in's cache follows the reference's query order: the minimum handed to
    worker_updateMinTimeJump after each query, the Dijkstra / self-path run counts, and the
    teardown log listing every cached Path with its packet count (topology.c:1929-1967)"""
    g = synth.random_sparse(V=80, avg_deg=4, seed=48, A=12)
    va, ips = with_vertex_ips(g)
    top = T.Topology.new(write(tmp_path, "u.xml", synth.to_graphml(g, extra_vattr=va)))
    hosts = attach_all(top, ips, g.attached)
    lat_o, _, _, kind_o, _ = oracle_matrix(g)
    model = ref_cache(g, lat_o, kind_o)
    rng = np.random.default_rng(3)
    for _ in range(40):
        i, j = (int(x) for x in rng.integers(0, len(hosts), 2))
        si, sj = model.get_path_entry(i, j)
        assert top.getLatency(hosts[i], hosts[j]) == lat_o[si, sj]
        top.incrementPathPacketCounter(hosts[i], hosts[j])
        check_cache_state(top, model)
    assert 0 < model.dijkstra_runs < len(hosts)
    T.set_log_level(4)
    capfd.readouterr()
    top.free()
    T.set_log_level(1)
    err = capfd.readouterr()
    text = err.out + err.err
    found = [ln for ln in text.splitlines() if "Found path" in ln]
    assert len(found) == len(model.cache)
    assert sum(int(ln.split("PacketCount=")[1].split()[0]) for ln in found) == 40
    assert "shortest paths with dijkstra" in text


def test_c_harness_lookups_under_threads(tmp_path):
    """the C caller (tests/c/topo_harness.c): attach, one-shot compute, then 8 worker
    threads doing the per-packet call sequence of worker.c:267-279 lock-free"""
    from test_topology_shim import build_harness, run_harness
    g = synth.random_sparse(V=400, avg_deg=4, seed=47, A=None)
    va, _ = with_vertex_ips(g)
    path = write(tmp_path, "h.xml", synth.to_graphml(g, extra_vattr=va))
    res = run_harness(build_harness(tmp_path), path, 300, 8, 20000, 0)
    assert res["compute_failed"] == 0 and res["routable"] > 0
    assert res["ns_per_call_per_thread"] > 0


def test_self_pairs_follow_query_order_under_the_s_path_rule(tmp_path):
    """The [s]-path igraph (topology_hip_set_self_rule(1)): a self pair is
    cached by whichever of the two rules runs first -- a query (s, s) caches the self-path
    rule's value (topology.c:1545-1653), s's Dijkstra run caches its self-loop path
    (:1456-1499); a source without a self-loop fails its Dijkstra run after storing the
    rest, so the first query from it fails and the next one hits.  Driven in both orders
    against the cache model (oracle/path_cache_ref.py), values, counts and upcalls included."""
    g = synth.random_sparse(V=120, avg_deg=4, seed=52, A=30)
    noloop = [int(g.attached[3]), int(g.attached[7])]  # two attached vertices lose their self-loop
    keep = ~((g.src == g.dst) & np.isin(g.src, noloop))
    g.src, g.dst, g.latency, g.packetloss = g.src[keep], g.dst[keep], g.latency[keep], g.packetloss[keep]
    lat_o, rel_o, _, kind_o, og = oracle_matrix(g, self_loop_rule=True)
    sp = [og.self_path(int(v)) for v in g.attached]
    model = ref_cache(g, lat_o, kind_o)
    model.self_loop_rule = True
    model.self_lat = np.array([x[0] if x else -1.0 for x in sp])
    model.self_rel = np.array([x[1] if x else -1.0 for x in sp])
    model.self_kind = np.array([2 if x else 0 for x in sp])
    assert kind_o[3, 3] == 0 and kind_o[0, 0] == 3 and model.self_lat[0] != lat_o[0, 0]
    va, ips = with_vertex_ips(g)
    top = T.Topology.new(write(tmp_path, "s.xml", synth.to_graphml(g, extra_vattr=va)))
    top.set_self_rule(True)
    hosts = attach_all(top, ips, g.attached)

    def q(i, j):
        a, b = hosts[i], hosts[j]
        path = model.get_path_entry(i, j)
        got = top.getLatency(a, b)
        path2 = model.get_path_entry(i, j)
        gotr = top.getReliability(a, b)
        if path is None:
            assert got == -1.0, (i, j)
        else:
            assert got == entry_value(model, path, lat_o, rel_o)[0], (i, j, path)
        if path2 is None:
            assert gotr == -1.0, (i, j)
        else:
            assert gotr == entry_value(model, path2, lat_o, rel_o)[1], (i, j, path2)
        return path

    assert q(0, 0) == (0, 0) and 0 in model.self_claimed  # the self rule first
    q(0, 5)  # 0's Dijkstra: (0, 0) stays the self rule's
    assert top.getLatency(hosts[0], hosts[0]) == model.self_lat[0]
    model.get_path_entry(0, 0)
    q(1, 5)  # 1's Dijkstra first: (1, 1) is its self-loop path
    assert q(1, 1) == (1, 1) and 1 not in model.self_claimed
    assert q(3, 4) is None  # no self-loop: the run fails, after storing (3, t)
    assert q(3, 4) == (3, 4)  # a hit
    for i in range(len(hosts)):
        for j in range(len(hosts)):
            q(i, j)
    check_cache_state(top, model)
    top.free()


@pytest.mark.parametrize("tsan", [False, True])
def test_lock_free_cache_under_racing_workers(tmp_path, tsan):
    """the path cache is lock-free (a CAS claim per Path, a CAS per source store
    loop, in-place fills of old rows after a late attach).  8 C worker threads
    (tests/c/topo_race.c) query and count packets over overlapping pairs of 32 hosts, then of
    48 after a late attach that the workers themselves resolve.  Every returned value must be
    the oracle's entry of the direction the pair is cached in, no unordered pair may be cached
    in both directions, cached_paths must equal the cached cells, and no increment is lost.
    tsan: the shim's C sources compiled into the harness with ThreadSanitizer (host code
    only; the engine library stays uninstrumented and its shim copy is interposed), which
    must report no data race."""
    import platform
    import subprocess
    from test_topology_shim import INCLUDE
    from shadow_amd import engine as E
    g = synth.random_sparse(V=160, avg_deg=4, seed=51, A=48)
    assert len(set(g.attached)) == 48
    va, ips = with_vertex_ips(g)
    path = write(tmp_path, "r.xml", synth.to_graphml(g, extra_vattr=va))
    hints = write(tmp_path, "hints.txt", "\n".join(ips[v] for v in g.attached) + "\n")
    src = os.path.join(os.path.dirname(__file__), "c", "topo_race.c")
    lib_dir = os.path.dirname(E.LIB_PATH)
    exe = str(tmp_path / "topo_race")
    cmd = ["gcc", "-O2", "-std=gnu11", "-pthread", "-I", INCLUDE, src]
    env = dict(os.environ)
    if tsan:
        csrc = os.path.join(os.path.dirname(os.path.dirname(__file__)), "shadow_amd", "csrc")
        # (non-PIE: a PIE image loaded high by the box's kernel ASLR is outside TSan's expected layout)
        cmd = ["gcc", "-O1", "-g", "-fsanitize=thread", "-fno-pie", "-no-pie", "-std=gnu11", "-pthread", "-ffp-contract=off", "-I", INCLUDE,
               "-I", csrc, src] + [os.path.join(csrc, f) for f in ("topology_hip.c", "graphml.c", "shadow_hooks.c")]
        # the ROCm runtime and the engine are not instrumented: TSan cannot see their own
        # synchronisation, so what they allocate and free on their threads is not checked
        supp = write(tmp_path, "tsan.supp", "".join(f"called_from_lib:{lib}\nrace:{lib}\n" for lib in
                                                    ("libhsa-runtime64.so", "libamdhip64.so", "libshadowtopo_hip.so")))
        env["TSAN_OPTIONS"] = f"halt_on_error=1 exitcode=66 suppressions={supp}"
    subprocess.run(cmd + ["-o", exe, "-L", lib_dir, "-lshadowtopo_hip", f"-Wl,-rpath,{lib_dir}", "-lm"], check=True)
    out = str(tmp_path / "recs.bin")
    # (TSan: without address-space randomisation -- the box's kernel places mappings where this
    # TSan does not expect them)
    pre = ["setarch", platform.machine(), "-R"] if tsan else []
    res = subprocess.run(pre + [exe, path, hints, "32", "16", "8", "1000" if tsan else "3000", out],
                         capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0 and "ThreadSanitizer" not in res.stderr, res.stderr[-4000:]
    lines = res.stdout.strip().splitlines()
    head = json.loads(lines[0])
    assert head["compute_failed"] == 0
    cells = {}
    total = 0
    for ln in lines[1:]:
        _, a, b, cell, cnt = ln.split()
        a, b, cell, cnt = int(a), int(b), int(cell), int(cnt)
        assert cell in (0, 1, 2) or (a == b and cell == 1), (a, b, cell)
        if cell:
            cells[(a, b)] = (a, b) if (cell == 1) else (b, a)
        total += cnt
    assert head["cached_paths"] == len(cells)
    assert total == head["increments"]
    rec = np.fromfile(out, dtype=[("phase", "<i4"), ("i", "<i4"), ("j", "<i4"), ("pad", "<i4"),
                                  ("lat", "<f8"), ("rel", "<f8")])
    assert len(rec) == 2 * 8 * (1000 if tsan else 3000)
    lat_o, rel_o, _, kind_o, _ = oracle_matrix(g)
    for r in rec:
        i, j = int(r["i"]), int(r["j"])
        si, sj = cells[(min(i, j), max(i, j))]  # every answered pair is cached, one direction for good
        assert r["lat"] == lat_o[si, sj] and r["rel"] == rel_o[si, sj], (int(r["phase"]), i, j, si, sj)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_rows_sharded_over_engines(tmp_path, devices):
    """in-process multi-GPU: one engine per listed device, each computing a
    contiguous block of source rows on its own thread into the host matrix; the same device
    listed several times exercises the sharding on a one-GPU box"""
    g = synth.random_sparse(V=200, avg_deg=4, seed=46, A=70)
    va, ips = with_vertex_ips(g)
    top = T.Topology.new(write(tmp_path, "m.xml", synth.to_graphml(g, extra_vattr=va)))
    assert top.set_devices(devices) == 0
    hosts = attach_all(top, ips, g.attached)
    lat_o, rel_o, _, kind_o, _ = oracle_matrix(g)
    model = ref_cache(g, lat_o, kind_o)
    for i in range(0, len(hosts), 3):
        for j in range(len(hosts)):
            si, sj = model.get_path_entry(i, j)
            assert top.getLatency(hosts[i], hosts[j]) == lat_o[si, sj]
            assert top.getReliability(hosts[i], hosts[j]) == rel_o[si, sj]
    assert top.info()["n_devices"] == len(devices)
    top.free()
