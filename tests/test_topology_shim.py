"""CPU tests of the C host shim (libshadowtopo_hip.so, topology_hip.h): the library loads
and exports every declared symbol, GraphML ingest matches the independent reader,
validation accepts/rejects like topology.c, attachment matches the restated reference
algorithm.  No GPU: path queries must fail loudly (-1), never fall back to the CPU."""
import lzma
import os
import re

import numpy as np
import pytest

from oracle import attach_ref
from oracle.graphml_ref import read_graphml
from shadow_amd import engine as E
from shadow_amd import synth
from shadow_amd import topology as T

GOLD = os.path.join(os.path.dirname(__file__), "golden")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include")


@pytest.fixture(scope="module", autouse=True)
def quiet():
    T.set_log_level(1)


def declared_functions():
    names = set()
    for h in os.listdir(INCLUDE):
        txt = open(os.path.join(INCLUDE, h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\([^;{]*\)\s*;", txt, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    L = E.lib()
    names = declared_functions()
    assert set(E.ENGINE_SYMBOLS) <= names
    assert set(T.TOPOLOGY_SYMBOLS) <= names
    assert set(T.EXT_SYMBOLS) <= names
    for n in sorted(names):
        assert hasattr(L, n), f"libshadowtopo_hip.so does not export {n}"


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_shipped_topology_loads(tmp_path):
    text = lzma.open(os.path.join(GOLD, "c1_topology.graphml.xml.xz"), "rt").read()
    top = T.Topology.new(write(tmp_path, "c1.graphml.xml", text))
    assert top is not None
    inf = top.info()
    assert (inf["n_vertices"], inf["n_edges"]) == (183, 16836)
    assert inf["is_complete"] == 1 and inf["is_connected"] == 1 and inf["cluster_count"] == 1
    assert inf["is_directed"] == 0 and inf["prefers_direct_paths"] == 0
    ref = read_graphml(text)
    src, dst, lat, loss, vl = top.edges()
    assert np.array_equal(src, ref.src) and np.array_equal(dst, ref.dst)
    assert np.array_equal(lat, ref.enum("latency")) and np.array_equal(loss, ref.enum("packetloss"))
    assert np.array_equal(vl, ref.vnum("packetloss"))
    assert top.vertex_of_id(ref.ids[17]) == 17
    top.free()


@pytest.mark.parametrize("gen", ["sparse", "directed", "vloss", "geo"])
def test_graphml_ingest_matches_reference_reader(tmp_path, gen):
    if gen == "sparse":
        g = synth.random_sparse(V=300, seed=1)
    elif gen == "directed":
        g = synth.random_sparse(V=200, seed=2, directed=True)
    elif gen == "vloss":
        vl = np.where(np.arange(150) % 3 == 0, np.nan, np.linspace(0, 0.2, 150))
        g = synth.random_sparse(V=150, seed=3, vloss=vl)
    else:
        g = synth.geometric_complete_ish(V=120, A=10)
    text = synth.to_graphml(g)
    top = T.Topology.new(write(tmp_path, "g.xml", text))
    assert top is not None
    ref = read_graphml(text)
    src, dst, lat, loss, vl = top.edges()
    assert np.array_equal(src, ref.src) and np.array_equal(dst, ref.dst)
    assert np.array_equal(lat, ref.enum("latency")) and np.array_equal(lat, g.latency)
    assert np.array_equal(loss, g.packetloss)
    assert np.array_equal(vl.view(np.uint64), ref.vnum("packetloss").view(np.uint64))
    assert top.info()["is_directed"] == int(g.directed)
    top.free()


def test_graphml_numbers_convert_as_strtod(tmp_path):
    """numparse.cpp (std::from_chars, strtod fallback) gives libc strtod's value for every
    spelling a topology file may hold: signs, hex floats, 17+ significant digits, bare
    exponents, leading blanks"""
    import ctypes
    libc = ctypes.CDLL(None)
    libc.strtod.restype = ctypes.c_double
    libc.strtod.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    spellings = ["+5", "0x1p3", "0X1.8p1", "1e2", ".5", "5.", " 7", "1e", "2.5e-3", "12345678901234567890",
                 "0.12345678901234567890123", "1.7976931348623157e308", "4.9406564584124654e-300", "3E+2",
                 "1.2451401810445306", "0.1"]
    g = synth.random_sparse(V=60, avg_deg=3, seed=9)
    text = synth.to_graphml(g)
    key = re.search(r'<key attr.name="latency"[^>]*id="(\w+)"', text)
    key = key.group(1) if key else re.search(r'id="(\w+)"[^>]*attr.name="latency"', text).group(1)
    it = iter(spellings)
    text = re.sub(r'(<data key="%s">)[^<]*(</data>)' % key,
                  lambda m: m.group(1) + next(it) + m.group(2), text, count=len(spellings))
    top = T.Topology.new(write(tmp_path, "n.xml", text))
    assert top is not None
    _, _, lat, _, _ = top.edges()
    want = np.array([libc.strtod(x.encode(), None) for x in spellings])
    assert np.array_equal(lat[:len(spellings)].view(np.uint64), want.view(np.uint64)), (lat[:len(spellings)], want)
    top.free()


def test_example_config_graph_and_quirks(tmp_path):
    # CDATA, entities, comments, node declared after use, for="all" key with default
    text = """<?xml version="1.0"?>
<!-- comment <node id="x"/> -->
<graphml xmlns="http://graphml.graphdrawing.org/xmlns">
 <key attr.name="latency" attr.type="double" for="edge" id="l"><default>7.5</default></key>
 <key attr.name="packetloss" attr.type="double" for="all" id="p"/>
 <key attr.name="bandwidthdown" attr.type="int" for="node" id="bd"/>
 <key attr.name="bandwidthup" attr.type="int" for="node" id="bu"/>
 <key attr.name="type" attr.type="string" for="node" id="t"/>
 <graph edgedefault="undirected">
  <edge source="b&amp;c" target="a"><data key="p">0.5</data></edge>
  <node id="a"><data key="bd">10</data><data key="bu">20</data><data key="t"><![CDATA[re<lay]]></data>
   <data key="p">0.25</data></node>
  <node id="b&amp;c"><data key="bd">1</data><data key="bu">2</data></node>
  <edge source="a" target="a"><data key="l">3.0</data><data key="p">0.0</data></edge>
  <edge source="b&amp;c" target="b&amp;c"><data key="p">0.1</data></edge>
 </graph>
</graphml>"""
    ref = read_graphml(text)
    assert ref.ids == ["b&c", "a"]
    top = T.Topology.new(write(tmp_path, "q.xml", text))
    assert top is not None
    src, dst, lat, loss, vl = top.edges()
    assert list(src) == [0, 1, 0] and list(dst) == [1, 1, 0]
    assert list(lat) == [7.5, 3.0, 7.5]
    assert list(loss) == [0.5, 0.0, 0.1]
    assert np.isnan(vl[0]) and vl[1] == 0.25
    assert top.vertex_of_id("b&c") == 0
    inf = top.info()
    assert inf["is_complete"] == 1  # 2 vertices: each has one non-loop + loop twice - 1 = 2
    top.free()


BASE = """<graphml xmlns="http://graphml.graphdrawing.org/xmlns">
 <key attr.name="latency" attr.type="{lt}" for="edge" id="l"/>
 <key attr.name="packetloss" attr.type="double" for="edge" id="p"/>
 <key attr.name="bandwidthdown" attr.type="int" for="node" id="bd"/>
 <key attr.name="bandwidthup" attr.type="int" for="node" id="bu"/>
 <key attr.name="packetloss" attr.type="double" for="node" id="vp"/>
 {gkey}
 <graph edgedefault="{ed}">{gdata}
  <node id="a"><data key="bd">10</data><data key="bu">{bu}</data><data key="vp">{vp}</data></node>
  <node id="b"><data key="bd">10</data><data key="bu">10</data></node>
  <node id="c"><data key="bd">10</data><data key="bu">10</data></node>
  <edge source="a" target="b"><data key="l">{lat}</data><data key="p">{loss}</data></edge>
  <edge source="b" target="c"><data key="l">5</data><data key="p">0.0</data></edge>
  {extra}
 </graph>
</graphml>"""


def mk(**kw):
    d = dict(lt="double", ed="undirected", bu="10", vp="0.0", lat="3.0", loss="0.1", extra="", gkey="", gdata="")
    d.update(kw)
    return BASE.format(**d)


@pytest.mark.parametrize("kw,ok", [
    ({}, True),
    ({"lat": "0"}, False),              # latency must be > 0 (topology.c:1070)
    ({"lat": "-2"}, False),
    ({"loss": "1.5"}, False),           # packetloss in [0,1] (topology.c:1090)
    ({"bu": "0"}, False),               # bandwidthup > 0 (topology.c:866-874)
    ({"vp": "2"}, False),               # vertex packetloss in [0,1] (topology.c:957-969)
    ({"lt": "string"}, False),          # latency must be NUMERIC (topology.c:680-681)
    ({"extra": '<node id="d"><data key="bd">1</data><data key="bu">1</data></node>'}, False),  # disconnected
    ({"ed": "directed"}, False),        # a->b->c not strongly connected
    ({"ed": "directed", "extra": '<edge source="c" target="a"><data key="l">1</data><data key="p">0</data></edge>'},
     True),
])
def test_validation(tmp_path, kw, ok):
    top = T.Topology.new(write(tmp_path, "v.xml", mk(**kw)))
    assert (top is not None) == ok
    if top:
        top.free()


@pytest.mark.parametrize("val,want", [("true", 1), ("Yes", 1), ("1", 1), ("false", 0), ("no", 0)])
def test_preferdirectpaths(tmp_path, val, want):
    top = T.Topology.new(write(tmp_path, "pd.xml", mk(
        gkey='<key attr.name="preferdirectpaths" attr.type="string" for="graph" id="g"/>',
        gdata=f'<data key="g">{val}</data>')))
    assert top is not None and top.info()["prefers_direct_paths"] == want
    top.free()


def test_preferdirectpaths_boolean_type_rejected(tmp_path):
    top = T.Topology.new(write(tmp_path, "pdb.xml", mk(
        gkey='<key attr.name="preferdirectpaths" attr.type="boolean" for="graph" id="g"/>',
        gdata='<data key="g">true</data>')))
    assert top is None  # the reference requires a STRING (topology.c:601-603)


def attach_graph(n=40, seed=3, with_ip=True, dup_ips=False):
    rng = np.random.default_rng(seed)
    g = synth.random_sparse(V=n, seed=seed)
    countries = ["US", "DE", "FR", "BR"]
    types = ["relay", "client", "server"]
    cities = ["a", "b", "c", "d", "e", "f"]
    pool = [f"10.{rng.integers(0, 4)}.{rng.integers(0, 255)}.{rng.integers(1, 255)}" for _ in range(8)]
    ips = [(pool[rng.integers(0, 8)] if dup_ips else f"10.{rng.integers(0, 4)}.{rng.integers(0, 255)}.{rng.integers(1, 255)}")
           if rng.random() < 0.6 else ("0.0.0.0" if rng.random() < 0.5 else None) for _ in range(n)]
    va = {
        "countrycode": ("d2", "string", [countries[rng.integers(0, 4)] for _ in range(n)]),
        "citycode": ("d5", "string", [cities[rng.integers(0, 6)] if rng.random() < 0.5 else None for _ in range(n)]),
        "type": ("d6", "string", [types[rng.integers(0, 3)] for _ in range(n)]),
        "geocode": ("d8", "string", [countries[rng.integers(0, 4)] if rng.random() < 0.3 else None for _ in range(n)]),
    }
    if with_ip:
        va["ip"] = ("d1", "string", ips)
    vattr = {k: [(x or "") for x in v[2]] for k, v in va.items()}
    return g, synth.to_graphml(g, extra_vattr=va), vattr


def random_hints(rng, vattr, k):
    ip = [None, "10.1.2.3", "10.0.0.1", "192.168.1.1", "0.0.0.0", "127.0.0.1", "garbage", "255.255.255.255",
          "0.0.0.1"][rng.integers(0, 9)]
    if rng.random() < 0.2 and "ip" in vattr:
        cand = [x for x in vattr["ip"] if x and x != "0.0.0.0"]
        if cand:
            ip = cand[rng.integers(0, len(cand))]
    if k % 5 == 0:  # IP hint alone: the longest-prefix rule over the whole vertex set
        return dict(ipHint=ip)
    return dict(ipHint=ip,
                citycodeHint=[None, "a", "B", "zz", ""][rng.integers(0, 5)],
                countrycodeHint=[None, "us", "DE", "XX"][rng.integers(0, 4)],
                geocodeHint=[None, "FR", "br"][rng.integers(0, 3)],
                typeHint=[None, "relay", "CLIENT", "nope"][rng.integers(0, 4)])


@pytest.mark.parametrize("n,seed,with_ip,dup_ips", [(40, 3, True, False), (300, 8, True, False),
                                                   (120, 9, True, True), (60, 10, False, False)])
def test_attach_matches_reference_algorithm(tmp_path, n, seed, with_ip, dup_ips):
    """the indexed attach (hint indexes + LPM trie) picks the vertex the reference's O(V)
    scan picks, with the same random stream, for every hint combination"""
    g, text, vattr = attach_graph(n=n, seed=seed, with_ip=with_ip, dup_ips=dup_ips)
    top = T.Topology.new(write(tmp_path, "att.xml", text))
    assert top is not None
    ref_rng = attach_ref.RandR(12345 + seed)
    rnd = T.Random(12345 + seed)
    rng = np.random.default_rng(seed)
    for k in range(300):
        h = random_hints(rng, vattr, k)
        addr = T.Address(f"11.0.{k // 250}.{k % 250 + 1}")
        down, up = top.attach(addr, rnd, **h)
        want = attach_ref.find_attachment_vertex(vattr, g.n, ref_rng, **h)
        got = top.vertex_of_ip(addr.ip)
        assert got == want, (k, h)
        assert (down, up) == (10240, 10240)
    att = top.attached()
    assert len(set(att.tolist())) == len(att)
    top.free()


def test_failed_computation_is_not_retried(tmp_path):
    """a failed attached-pair computation is remembered: later queries return -1 at once
    instead of re-running the GPU work under the compute lock"""
    g, text, _ = attach_graph(n=20, seed=11)
    top = T.Topology.new(write(tmp_path, "f.xml", text))
    a, b = T.Address("11.1.1.1"), T.Address("11.1.1.2")
    r = T.Random(2)
    top.attach(a, r)
    top.attach(b, r)
    top.set_device(1000)  # no such device: engine creation fails
    assert top.getLatency(a, b) == -1.0
    assert top.info()["compute_failed"] == 1
    assert top.getReliability(a, b) == -1.0 and not top.isRoutable(a, b)
    assert top.info()["compute_failed"] == 1
    top.free()


def test_infinite_latency_rejected_at_load(tmp_path):
    g = synth.random_sparse(V=10, seed=12)
    g.latency[3] = np.inf
    assert T.Topology.new(write(tmp_path, "inf.xml", synth.to_graphml(g))) is None


def test_detach_keeps_attached_vertex(tmp_path):
    g, text, vattr = attach_graph(n=20, seed=5)
    top = T.Topology.new(write(tmp_path, "d.xml", text))
    a = T.Address("11.1.1.1")
    top.attach(a, T.Random(1))
    v = top.vertex_of_ip("11.1.1.1")
    assert v >= 0
    top.detach(a)
    assert top.vertex_of_ip("11.1.1.1") == -1
    assert v in top.attached().tolist()  # verticesWithAttachedHosts never shrinks (topology.c:2432-2439)
    top.free()


@pytest.mark.skipif(E.device_count() > 0, reason="CPU-only behaviour")
def test_queries_fail_loudly_without_gpu(tmp_path):
    g, text, _ = attach_graph(n=20, seed=6)
    top = T.Topology.new(write(tmp_path, "n.xml", text))
    a, b = T.Address("11.1.1.1"), T.Address("11.1.1.2")
    r = T.Random(2)
    top.attach(a, r)
    top.attach(b, r)
    assert top.getLatency(a, b) == -1.0
    assert top.getReliability(a, b) == -1.0
    assert not top.isRoutable(a, b)
    top.free()


def test_unattached_address_is_unroutable(tmp_path):
    g, text, _ = attach_graph(n=20, seed=7)
    top = T.Topology.new(write(tmp_path, "u.xml", text))
    a, b = T.Address("11.1.1.1"), T.Address("11.1.1.9")
    top.attach(a, T.Random(3))
    assert top.getLatency(a, b) == -1.0  # topology.c:1979-1984 -> -1 (topology.c:2073)
    top.free()


HARNESS = os.path.join(os.path.dirname(__file__), "c", "topo_harness.c")


def build_harness(tmp_path):
    """compile the C caller against the in-tree library, as Shadow links it"""
    import subprocess
    lib_dir = os.path.dirname(E.LIB_PATH)
    exe = str(tmp_path / "topo_harness")
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-pthread", "-I", INCLUDE, HARNESS, "-o", exe, "-L", lib_dir,
                    "-lshadowtopo_hip", f"-Wl,-rpath,{lib_dir}"], check=True)
    return exe


def run_harness(exe, *args):
    import json
    import subprocess
    out = subprocess.run([exe] + [str(a) for a in args], check=True, capture_output=True, text=True, timeout=300)
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_c_harness_ingest_and_attach(tmp_path, mode):
    """a C program linked against libshadowtopo_hip drives topology_new + topology_attach
    (no queries: no GPU needed)"""
    g, text, _ = attach_graph(n=300, seed=13)
    path = write(tmp_path, "h.xml", text)
    res = run_harness(build_harness(tmp_path), path, 500, 1, 0, mode)
    assert res["vertices"] == 300 and res["hosts"] == 500
    assert 0 < res["attached"] <= 300


def test_ip_table_lookups_through_attach_detach_churn(tmp_path):
    """The per-packet IP -> vertex table (topology_hip.c iptab, read with no lock): lookups of
    stable hosts from several threads stay right while another thread attaches and detaches
    other hosts (table growth and tombstone rehashes replace the table under the readers),
    and the memory the retired tables keep stays bounded by the churn (one full
    snapshot per detach before)."""
    import threading
    g, text, _ = attach_graph(n=200, seed=13)
    top = T.Topology.new(write(tmp_path, "ipt.xml", text))
    rnd = T.Random(9)
    stable = [T.Address(f"12.0.{k // 200}.{k % 200 + 1}") for k in range(300)]
    for a in stable:
        top.attach(a, rnd)
    want = {a.ip: top.vertex_of_ip(a.ip) for a in stable}
    assert all(v >= 0 for v in want.values())
    stop = threading.Event()
    bad = []

    def reader(seed):
        rng = np.random.default_rng(seed)
        n = 0
        while not stop.is_set() or n < 2000:
            a = stable[rng.integers(0, len(stable))]
            if top.vertex_of_ip(a.ip) != want[a.ip]:
                bad.append(a.ip)
            n += 1

    threads = [threading.Thread(target=reader, args=(s,)) for s in range(4)]
    for t in threads:
        t.start()
    churn = [T.Address(f"13.{k // 60000}.{(k // 250) % 240}.{k % 250 + 1}") for k in range(2500)]
    detaches = 0
    for rnd_i in range(2):
        for a in churn:
            top.attach(a, rnd)
        for a in churn[: 2000]:
            top.detach(a)
            detaches += 1
            assert top.vertex_of_ip(a.ip) == -1
    stop.set()
    for t in threads:
        t.join()
    assert not bad, f"{len(bad)} wrong lookups of stable hosts during churn"
    for a in churn[2000:]:
        assert top.vertex_of_ip(a.ip) >= 0
    inf = top.info()
    assert inf["ip_table_slots"] >= 2 * (len(stable) + 500) and inf["ip_tables_retired"] >= 2
    # growth retires tables half the size of their successor; tombstone rehashes need
    # cap / 4 detaches each: bounded by the live table plus 32 bytes per detach
    assert inf["ip_retired_bytes"] <= 8 * inf["ip_table_slots"] + 32 * detaches + 4096 * inf["ip_tables_retired"]
    top.free()


@pytest.mark.parametrize("n_edges", [1000, 3_000_000])  # the sequential and the threaded scan
def test_engine_edge_validation_reports_the_first_bad_edge(n_edges):
    """shadowtopo_create checks every edge (topology.c:1070, :1090 and the endpoint range)
    before it touches a device; past 2^20 edges the scan is split over host threads and
    must still name the FIRST failing edge in edge order, with that edge's own message."""
    rng = np.random.default_rng(5)
    V = 5000
    src = rng.integers(0, V, n_edges).astype(np.int32)
    dst = rng.integers(0, V, n_edges).astype(np.int32)
    lat = rng.uniform(1.0, 50.0, n_edges)
    loss = rng.uniform(0.0, 0.02, n_edges)
    cases = [  # (index, field, value, message) -- the later, different fault must not win
        (int(n_edges * 0.61), "lat", 0.0, "latency must be > 0"),
        (int(n_edges * 0.37), "loss", 1.5, "packetloss out of [0,1]"),
        (int(n_edges * 0.12), "dst", V, "endpoint out of range"),
        (n_edges - 1, "lat", np.inf, "latency must be > 0"),
    ]
    arrays = {"src": src, "dst": dst, "lat": lat, "loss": loss}
    for k in range(len(cases)):
        first = min(cases[: k + 1])  # faults 0..k present: the lowest index is reported
        a = {key: v.copy() for key, v in arrays.items()}
        for idx, field, val, _ in cases[: k + 1]:
            a[field][idx] = val
        with pytest.raises(E.ShadowTopoError) as ei:
            E.Engine(V, a["src"], a["dst"], a["lat"], a["loss"])
        msg = str(ei.value)
        assert f"edge {first[0]} " in msg and first[3] in msg, msg


def test_prepare_rejects_a_bad_device():
    """shadowtopo_prepare validates the ordinal before starting its thread (no device here:
    every ordinal is out of range; on a GPU box -1 still is)."""
    with pytest.raises(E.ShadowTopoError):
        E.prepare(-1)
    with pytest.raises(E.ShadowTopoError):
        E.prepare(E.device_count())


def test_host_paths_under_address_sanitizer(tmp_path):
    """The shim's host code -- GraphML reader, validation (accepted and rejected graphs,
    truncated and garbage files), the three attach hint paths, detach / re-attach churn of
    the lock-free IP table, teardown -- compiled with AddressSanitizer and UBSan
    (tests/c/shim_asan.c; host code only, the engine library uninstrumented): no memory
    error, no undefined behaviour, and the same accept / reject decisions as the library."""
    import subprocess
    csrc = os.path.join(os.path.dirname(os.path.dirname(__file__)), "shadow_amd", "csrc")
    lib_dir = os.path.dirname(E.LIB_PATH)
    exe = str(tmp_path / "shim_asan")
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-std=gnu11", "-pthread", "-ffp-contract=off", "-I", INCLUDE, "-I", csrc,
                    os.path.join(os.path.dirname(__file__), "c", "shim_asan.c")] +
                   [os.path.join(csrc, f) for f in ("topology_hip.c", "graphml.c", "shadow_hooks.c")] +
                   ["-o", exe, "-L", lib_dir, "-lshadowtopo_hip", f"-Wl,-rpath,{lib_dir}", "-lm"], check=True)
    files, want = [], []
    shipped = lzma.open(os.path.join(GOLD, "c1_topology.graphml.xml.xz"), "rt").read()
    files.append(write(tmp_path, "c1.xml", shipped))
    want.append(True)
    for i, (kw, ok) in enumerate([({}, True), ({"lat": "0"}, False), ({"loss": "1.5"}, False), ({"lt": "string"}, False),
                                  ({"ed": "directed"}, False)]):
        files.append(write(tmp_path, f"v{i}.xml", mk(**kw)))
        want.append(ok)
    for seed, dup in ((13, False), (14, True)):
        _, text, _ = attach_graph(n=300, seed=seed, dup_ips=dup)
        files.append(write(tmp_path, f"a{seed}.xml", text))
        want.append(True)
        files.append(write(tmp_path, f"t{seed}.xml", text[: len(text) // 2]))  # truncated mid-file
        want.append(False)
    files.append(write(tmp_path, "garbage.xml", "<graphml><graph><node id=\"a\"><data key=\"zz\">\x01\x02</data>"))
    want.append(False)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=66",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=67")
    res = subprocess.run([exe, "400"] + files, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0 and "Sanitizer" not in res.stderr and "runtime error" not in res.stderr, \
        res.stderr[-4000:]
    lines = res.stdout.strip().splitlines()
    assert len(lines) == len(files)
    for ln, f, ok in zip(lines, files, want):
        parts = ln.split()
        assert parts[0] == f and (parts[1] == "ok") == ok, ln
        if ok:
            assert int(parts[3]) > 0
