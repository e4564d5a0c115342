"""GPU parity tests: every hot-path kernel, through the C ABI, against the
CPU oracle (oracle/) and the reference's golden fixtures (tests/golden/).
Bit-exact for all integer work; the fp32 triad is bit-exact too (no FMA
contraction on either side), i.e. within the 1-ulp tolerance north_star
allows with 0 ulp observed."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import hclib_amd as H  # noqa: E402
from oracle import loader as L  # noqa: E402
from tests.conftest import GOLD  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def device():
    import torch

    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    H.init(0)
    yield


# ------------------------------------------------------------------ forasync
def _triad_expected(b, c, s):
    import torch

    return torch.add(b, torch.mul(c, s))  # two rounded ops, no contraction


@pytest.mark.parametrize("n", [1, 3, 4, 1000, 4097, 1 << 20, (1 << 20) + 7])
def test_triad_small_bit_exact(n):
    import torch

    g = torch.Generator(device="cpu").manual_seed(n)
    b = torch.rand(n, generator=g).cuda()
    c = torch.rand(n, generator=g).cuda()
    a = torch.full((n,), float("nan"), device="cuda")
    s = 3.0
    H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), s, n,
                torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = (b.cpu().numpy() + np.float32(s) * c.cpu().numpy()).astype(np.float32)
    assert np.array_equal(a.cpu().numpy(), exp)


def test_triad_full_size_2p28():
    """BASELINE config 1 size: 2^28 fp32, s=3.0; checked element-wise on
    device against two separately rounded torch ops."""
    import torch

    n = 1 << 28
    g = torch.Generator(device="cuda").manual_seed(1)
    b = torch.rand(n, device="cuda", generator=g)
    c = torch.rand(n, device="cuda", generator=g)
    a = torch.empty(n, device="cuda")
    H.triad_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), 3.0, n,
                torch.cuda.current_stream().cuda_stream)
    exp = _triad_expected(b, c, 3.0)
    assert torch.equal(a, exp)


def test_triad_through_forasync_api():
    import torch

    n = 123457
    b = torch.rand(n, device="cuda")
    c = torch.rand(n, device="cuda")
    a = torch.zeros(n, device="cuda")
    args = H.TriadArgs(a.data_ptr(), b.data_ptr(), c.data_ptr(), 2.5)
    for mode in (H.FORASYNC_MODE_FLAT, H.FORASYNC_MODE_RECURSIVE):
        a.zero_()
        dom = H.forasync(H.BODY_TRIAD_F32, args, [(0, n, 1, -1)], mode,
                         torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert dom[0][3] == (n + H.num_workers() - 1) // H.num_workers()  # tile write-back
        assert torch.equal(a, _triad_expected(b, c, 2.5))


def test_forasync1d_iota_check():
    """test/c/forasync1DCh.c: H1=1024, T1=33, FLAT; every ran[i]==-1 before."""
    import torch

    ran = torch.full((1024,), -1, dtype=torch.int32, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    H.forasync(H.BODY_IOTA_CHECK, H.IotaArgs(ran.data_ptr(), err.data_ptr()),
               [(0, 1024, 1, 33)], H.FORASYNC_MODE_FLAT)
    torch.cuda.synchronize()
    assert err.item() == 0
    assert torch.equal(ran.cpu(), torch.arange(1024, dtype=torch.int32))


CASES_1D = [
    ((10, 100, 1, 33), 0), ((10, 100, 1, 33), 1), ((0, 1000, 3, 7), 0), ((0, 1000, 3, 7), 1),
    ((5, 777, 4, -1), 0), ((5, 777, 4, -1), 1), ((0, 0, 1, 5), 0), ((3, 4, 1, 1), 1),
    ((0, 4096, 1, 1), 0),
]


@pytest.mark.parametrize("dom,mode", CASES_1D)
def test_forasync1d_iteration_set_matches_reference(dom, mode):
    import torch

    base, ext = -8, 1200 if dom[1] < 1100 else 4200
    counts = torch.zeros(ext, dtype=torch.int32, device="cuda")
    args = H.VisitArgs(counts.data_ptr(), (C.c_int * 3)(base, 0, 0), (C.c_int * 3)(ext, 1, 1))
    got_dom = H.forasync(H.BODY_VISIT_COUNT, args, [dom], mode)
    torch.cuda.synchronize()
    tiles, exp = L.forasync_nd_counts([dom], mode, H.num_workers(), [base], [ext])
    assert got_dom[0][3] == tiles[0]
    assert np.array_equal(counts.cpu().numpy(), exp)


CASES_ND = [
    ([(0, 30, 1, 7), (0, 20, 2, 3)], 0), ([(0, 30, 1, 7), (0, 20, 2, 3)], 1),
    ([(2, 17, 3, 4), (1, 9, 1, 2), (0, 5, 2, 2)], 0), ([(2, 17, 3, 4), (1, 9, 1, 2), (0, 5, 2, 2)], 1),
    ([(0, 64, 1, -1), (0, 64, 1, -1)], 0),
]


@pytest.mark.parametrize("doms,mode", CASES_ND)
def test_forasync_nd_iteration_set_matches_reference(doms, mode):
    import torch

    ext = [40, 24, 8][: len(doms)]
    full = ext + [1] * (3 - len(ext))
    counts = torch.zeros(int(np.prod(full)), dtype=torch.int32, device="cuda")
    args = H.VisitArgs(counts.data_ptr(), (C.c_int * 3)(0, 0, 0), (C.c_int * 3)(*full))
    got = H.forasync(H.BODY_VISIT_COUNT, args, doms, mode)
    torch.cuda.synchronize()
    tiles, exp = L.forasync_nd_counts(doms, mode, H.num_workers(), [0] * len(doms), ext)
    assert [d[3] for d in got] == tiles
    assert np.array_equal(counts.cpu().numpy().reshape(ext), exp)


# ----------------------------------------------------------------------- UTS
@pytest.mark.parametrize("name", ["T1", "T2", "T3", "T4", "T5"])
def test_uts_small_trees_bit_exact(golden, name):
    g = golden("uts_goldens.json")
    pub = g["published"][name]
    r = H.uts(pub["args"], max_levels=pub["depth"] + 1 if pub["depth"] < 1000 else 0)
    assert (r["nodes"], r["leaves"], r["max_depth"]) == (pub["nodes"], pub["leaves"], pub["depth"])
    if name in g["levels"]:
        assert r["levels"] == g["levels"][name]


@pytest.mark.parametrize("name,want", [
    # bench.py's T1 launch: the plain kernel (no per-level counts), fixed-shape
    # GEO, breadth-first seeded, 512-item rings, 8 waves per CU
    ("T1", {"mode": "geo_fixed", "feat": 0, "seeded": 1, "ring": 512, "waves_per_cu": 8,
            "workers_per_group": 1}),
    # BIN: four worker waves per workgroup (one per SIMD, LDS inboxes), the plain kernel
    ("T3", {"mode": "bin", "feat": 0, "seeded": 0, "ring": 1024, "workers_per_group": 4, "waves_per_cu": 4}),
])
def test_uts_bench_launch_shape_bit_exact(golden, name, want):
    """The exact launch the bench runs (no max_levels: FEAT = 0, the kernel
    test_uts_small_trees_bit_exact does not reach) against the published
    counts (test/uts/sample_trees.sh:17-18, 26-27), and the launch shape
    itself (hclib_hip_uts_last_launch)."""
    pub = golden("uts_goldens.json")["published"][name]
    r = H.uts(pub["args"])
    assert (r["nodes"], r["leaves"], r["max_depth"]) == (pub["nodes"], pub["leaves"], pub["depth"])
    shape = H.uts_last_launch()
    for k, v in want.items():
        assert shape[k] == v, (name, k, shape)


def test_uts_unseeded_fixed_shape(golden, monkeypatch):
    """T1 with the seeding off (HCLIB_HIP_UTS_SEED=0) takes the unseeded
    shape — 2 waves per CU on 256-item rings, as measured before seeding
    existed (round-4 advisor) — and is bit-exact."""
    monkeypatch.setenv("HCLIB_HIP_UTS_SEED", "0")
    pub = golden("uts_goldens.json")["published"]["T1"]
    r = H.uts(pub["args"])
    assert (r["nodes"], r["leaves"], r["max_depth"]) == (pub["nodes"], pub["leaves"], pub["depth"])
    shape = H.uts_last_launch()
    assert (shape["seeded"], shape["ring"], shape["waves_per_cu"]) == (0, 256, 2), shape


@pytest.mark.parametrize("name", ["T3L", "T1L"])
def test_uts_large_trees_bit_exact(golden, name):
    pub = golden("uts_goldens.json")["published"][name]
    r = H.uts(pub["args"])
    assert (r["nodes"], r["leaves"], r["max_depth"]) == (pub["nodes"], pub["leaves"], pub["depth"])


@pytest.mark.parametrize("nshards,split", [(2, 3), (3, 5), (8, 6), (4, 9)])
def test_uts_shards_sum_to_tree(golden, nshards, split):
    """T1's shards sum to the tree. Split 9 is deeper than the seeding's
    buffers reach (774 K depth-9 slots): that shard seeds only to its target
    and filters in the worker loop (FEAT = 1); the others filter inside the
    seeding and run the plain kernel (hclib_hip_uts_last_launch)."""
    pub = golden("uts_goldens.json")["published"]["T1"]
    parts = []
    for s in range(nshards):
        parts.append(H.uts(pub["args"], s, nshards, split))
        # every shard's own launch, not only the last one's (round-5 advisor)
        assert H.uts_last_launch()["feat"] == (1 if split == 9 else 0), (s, H.uts_last_launch())
    assert sum(p["nodes"] for p in parts) == pub["nodes"]
    assert sum(p["leaves"] for p in parts) == pub["leaves"]
    assert max(p["max_depth"] for p in parts) == pub["depth"]


def test_uts_t1xl_8_shards_split_10(golden, capsys):
    """The case that failed in round 5 (gpurun_out/r05/shard_split.log: T1XL,
    8 shards, split 10, "device error 2 (LDS ring overflow)" at b3f2efe):
    every shard once, bit-exact in sum (test/uts/sample_trees.sh:50-51), and
    which path each shard took. Depth 10 holds ~1 M slots, more than the
    seeding's level buffer, so each shard seeds to its target only and its
    worker loop filters (FEAT = 1)."""
    pub = golden("uts_goldens.json")["published"]["T1XL"]
    parts, feats = [], []
    for s in range(8):
        parts.append(H.uts(pub["args"], s, 8, 10))
        feats.append(H.uts_last_launch()["feat"])
    with capsys.disabled():
        print(f"\nT1XL split 10: feat per shard {feats}; shards (nodes, ms): " +
              ", ".join(f"({p['nodes']}, {p['kernel_ms']:.2f})" for p in parts))
    assert feats == [1] * 8
    assert sum(p["nodes"] for p in parts) == pub["nodes"]
    assert sum(p["leaves"] for p in parts) == pub["leaves"]
    assert max(p["max_depth"] for p in parts) == pub["depth"]


def test_uts_t3l_shards_sum_to_tree(golden):
    pub = golden("uts_goldens.json")["published"]["T3L"]
    parts = [H.uts(pub["args"], s, 4, 2000) for s in range(4)]
    assert sum(p["nodes"] for p in parts) == pub["nodes"]
    assert sum(p["leaves"] for p in parts) == pub["leaves"]
    assert max(p["max_depth"] for p in parts) == pub["depth"]


@pytest.mark.parametrize("name,split", [("T3L", 1), ("T1XL", 7)])
def test_uts_bench_partition_8_ranks(golden, name, split, capsys):
    """bench.py's exact N=8 partition (split depth 1 for T3L, 7 for T1XL;
    shard = node-state hash mod 8, bench.py:46-69), every shard through
    hclib_hip_uts_search as its rank runs it: the shards sum to the
    published tree (test/uts/sample_trees.sh:42-43, :50-51) and each
    shard's kernel time is printed. Every shard is seeded through its split
    and runs the plain kernel (FEAT = 0). T3L is span-bound: the shard
    holding the deepest chain takes about the whole-tree time on its own,
    and no more (round 5: +2.3 ms with the filter in the worker loop)."""
    pub = golden("uts_goldens.json")["published"][name]
    # one untimed launch first: whichever shard runs first in a process is
    # ~10% slower, in either order (profiles/r05/shard_order.log), so
    # without it the printed times blame shard 0 for the cold start
    H.uts(pub["args"], 7, 8, split)
    parts, shapes = [], []
    for s in range(8):
        parts.append(H.uts(pub["args"], s, 8, split))
        shapes.append(H.uts_last_launch())
    assert all(sh["feat"] == 0 and sh["seeded"] == 1 for sh in shapes), shapes
    assert sum(p["nodes"] for p in parts) == pub["nodes"]
    assert sum(p["leaves"] for p in parts) == pub["leaves"]
    assert max(p["max_depth"] for p in parts) == pub["depth"]
    whole = H.uts(pub["args"])
    with capsys.disabled():
        print(f"\n{name} split {split}: whole {whole['kernel_ms']:.2f} ms; shards (nodes, ms): " +
              ", ".join(f"({p['nodes']}, {p['kernel_ms']:.2f})" for p in parts))
    # the slowest shard is at most the whole search (+ its seeding, + noise)
    assert max(p["kernel_ms"] for p in parts) < 1.05 * whole["kernel_ms"] + 0.5


@pytest.mark.parametrize("chunk", ["16", "32"])
def test_uts_t1xl_non_default_chunk(chunk, monkeypatch):
    """HCLIB_HIP_CHUNK below the default 64 on the 1.6 G-node wide tree
    (test/uts/sample_trees.sh:50-51): the HBM deques are sized in items, not
    slots, so a smaller chunk does not shrink what the frontier can spill to,
    and a full ring fills the deques past their half mark before it waits
    (round 2 ended this launch with "LDS ring overflow")."""
    monkeypatch.setenv("HCLIB_HIP_CHUNK", chunk)
    r = H.uts("-t 1 -a 3 -d 15 -b 4 -r 29")
    assert (r["nodes"], r["leaves"], r["max_depth"]) == (1635119272, 1308100063, 15)


@pytest.mark.parametrize("wpg", ["2", "4"])
def test_uts_bin_sibling_inbox_narrow_trees(wpg, monkeypatch):
    """BIN trees near the critical branching factor (q*m = 0.9975 and
    0.99925: 30 K - 2.6 M nodes, depth 120-2,367, long narrow chains with one
    or two waves holding work most of the time) with 2 or 4 worker waves per
    workgroup handing chunks through LDS inboxes: every tree's node / leaf /
    depth counts equal the serial oracle's (test/uts/uts.c restated), i.e. no
    inbox chunk is lost at termination."""
    monkeypatch.setenv("HCLIB_HIP_WPG", wpg)
    for b, q, seed in [(2000, 0.1995, s) for s in range(8)] + [(500, 0.19985, s) for s in range(8)]:
        args = f"-t 0 -b {b} -q {q} -m 5 -r {seed}"
        (n, lv, d), _ = L.uts_serial(L.parse_uts_args(args))
        r = H.uts(args)
        assert (r["nodes"], r["leaves"], r["max_depth"]) == (n, lv, d), args


def test_uts_other_shapes_vs_oracle():
    for args in ["-t 1 -a 1 -d 8 -b 3 -r 5", "-t 3 -d 6 -b 5 -r 3", "-t 0 -b 200 -q 0.19 -m 5 -r 11",
                 "-t 1 -a 3 -d 7 -b 4 -r 19 -g 3"]:
        (n, lv, d), _ = L.uts_serial(L.parse_uts_args(args))
        r = H.uts(args)
        assert (r["nodes"], r["leaves"], r["max_depth"]) == (n, lv, d), args


# ----------------------------------------------------------------------- fib
def test_fib_table(golden):
    vals = golden("fib_goldens.json")["values"]
    for n in [0, 1, 2, 3, 10, 20, 25]:
        v, _ = H.fib(n)
        assert v == vals[str(n)]


def test_fib30_tasks_and_joins():
    v, st = H.fib(30)
    assert v == 832040
    assert st["tasks"] == 2 * 1346269 - 1  # every fib call is one task
    assert st["joins"] == 1346269 - 1      # one finish scope per internal call


def test_persistent_launch_that_cannot_be_resident_fails_fast(monkeypatch):
    """A megakernel grid the CUs cannot hold at once (here 64 fib waves per CU
    against ~5 that fit its LDS) is refused on the host before the launch,
    instead of spinning to the idle timeout on waves that never start."""
    monkeypatch.setenv("HCLIB_HIP_WAVES_PER_CU", "64")
    with pytest.raises(H.HclibError, match="cannot all be resident"):
        H.fib(20)
    monkeypatch.delenv("HCLIB_HIP_WAVES_PER_CU")
    assert H.fib(20)[0] == 6765


@pytest.mark.parametrize("mode", [{"HCLIB_HIP_FIB_LOCAL": "0"}, {},
                                  {"HCLIB_HIP_FIB_SEED": "0"}, {"HCLIB_HIP_FIB_SEED": "1"},
                                  {"HCLIB_HIP_FIB_SEED": "4", "HCLIB_HIP_WAVES_PER_CU": "2"},
                                  {"HCLIB_HIP_FIB_BLOCKS": "0"},
                                  {"HCLIB_HIP_FIB_BLOCKS": "0", "HCLIB_HIP_GRID": "300"}])
def test_fib_finish_scope_modes(mode, monkeypatch):
    """Every join mode gives the same value, tasks and joins: HBM scopes only;
    LDS scopes (hx_finish.h LocalScopes, the default) climbing inline with
    their HBM check-outs resolved a batch later (finish_issue /
    finish_resolve); breadth-first seeding of the call tree's top levels
    (HCLIB_HIP_FIB_SEED items per worker); scope ids taken one at a time
    (HCLIB_HIP_FIB_BLOCKS=0), also on a grid whose seeding reservation is
    not a power of two: the arena holds the seeding's whole reservation
    (round-4 advisor). fib(10) (a 90-id call tree, smaller than the
    reservation), fib(25) and fib(30)."""
    for k, v in mode.items():
        monkeypatch.setenv(k, v)
    for n, want, calls in [(10, 55, 177), (25, 75025, 242785), (30, 832040, 2692537)]:
        v, st = H.fib(n)
        assert v == want, (mode, n)
        assert st["tasks"] == calls and st["joins"] == (calls - 1) // 2, (mode, n, st)


# ------------------------------------------------------------------------ SW
def _sw_inputs(size):
    a = open(os.path.join(GOLD, "sw", f"string1-{size}.txt"), "rb").read()
    b = open(os.path.join(GOLD, "sw", f"string2-{size}.txt"), "rb").read()
    return H.sw_map(a), H.sw_map(b)


@pytest.mark.parametrize("size", ["tiny", "medium", "large", "huge"])
def test_sw_published_scores(golden, size):
    g = golden("sw_goldens.json")["published"][size]
    s1, s2 = _sw_inputs(size)
    score, st = H.sw(s1, s2, g["tile_w"], g["tile_h"])
    assert score == g["score"]
    assert st["tiles"] == (len(s1) // g["tile_w"]) * (len(s2) // g["tile_h"])


def test_sw_oracle_configs(golden):
    for cfg in golden("sw_goldens.json")["configs"]:
        s1, s2 = _sw_inputs(cfg["input"])
        s1, s2 = s1[: cfg["len1"]], s2[: cfg["len2"]]
        score, _ = H.sw(s1, s2, cfg["tile_w"], cfg["tile_h"])
        assert score == cfg["score"], cfg


def test_sw_64k_golden(golden):
    g = golden("sw_goldens.json")["sw64k"]
    s1, s2 = _sw_inputs("huge")
    score, st = H.sw(s1[:65536], s2[:65536], 256, 256)
    assert score == g["score"] == 128772
    assert st["tiles"] == 65536
    assert st["releases"] == 3 * 255 * 255 + 2 * 255


def test_sw_64k_golden_on_generic_promise_dag(golden, monkeypatch):
    """The 64K config as the reference writes it — 65,536 async_await tiles,
    196,608 promises — through device promises/futures: score 128772."""
    monkeypatch.setenv("HCLIB_HIP_SW_SCHED", "dag")
    g = golden("sw_goldens.json")["sw64k"]
    s1, s2 = _sw_inputs("huge")
    score, st = H.sw(s1[:65536], s2[:65536], 256, 256)
    assert score == g["score"] == 128772
    assert st["tiles"] == 65536


@pytest.mark.parametrize("pk", ["1", "0"])
def test_sw_64k_golden_on_packed_bodies(golden, pk, monkeypatch):
    """SW-64K on the promise DAG with the packed one-sweep-wave tile body (1)
    and the int32 band body (0): 128772."""
    monkeypatch.setenv("HCLIB_HIP_SW_SCHED", "dag")
    monkeypatch.setenv("HCLIB_HIP_SW_PK", pk)
    s1, s2 = _sw_inputs("huge")
    score, st = H.sw(s1[:65536], s2[:65536], 256, 256)
    assert score == golden("sw_goldens.json")["sw64k"]["score"] == 128772
    assert st["tiles"] == 65536


@pytest.mark.parametrize("tw", [1, 30, 63, 64, 65, 100, 256, 300, 511, 512])
def test_sw_dag_packed_half_tiles(tw, monkeypatch):
    """256-row tiles at most 512 wide run the promise DAG's packed-half body
    (one wave per tile, two cells per v_pk_maximum3_f16, values relative to
    each tile's corner): the oracle's score on ragged random inputs and on
    all-match inputs (+4 on every diagonal, so the relative values reach the
    f16-exact bound of 2048 at tw = 512), and the int32 band form's
    (HCLIB_HIP_SW_PK=0) on the same inputs."""
    monkeypatch.setenv("HCLIB_HIP_SW_SCHED", "dag")
    rng = np.random.default_rng(tw)
    n1 = tw * (3 if tw >= 64 else 17) + tw // 3
    n2 = 256 * 3 + 100
    cases = [(rng.integers(1, 5, n1), rng.integers(1, 5, n2)), (np.full(n1, 1), np.full(n2, 1)),
             (np.full(n1, 2), rng.integers(1, 5, n2))]
    for a, b in cases:
        a, b = a.astype(np.int8).tobytes(), b.astype(np.int8).tobytes()
        want = L.sw_score(a, b, tw, 256)
        score, st = H.sw(a, b, tw, 256)
        assert score == want and st["tiles"] == (n1 // tw) * 3, (tw, score, want)
        monkeypatch.setenv("HCLIB_HIP_SW_PK", "0")
        assert H.sw(a, b, tw, 256)[0] == want
        monkeypatch.delenv("HCLIB_HIP_SW_PK")


def test_sw_random_vs_oracle():
    rng = np.random.default_rng(5)
    for (n1, n2, tw, th) in [(300, 200, 17, 13), (1000, 777, 64, 300), (513, 1025, 256, 64)]:
        s1 = bytes(rng.integers(1, 5, n1, dtype=np.int8).tobytes())
        s2 = bytes(rng.integers(1, 5, n2, dtype=np.int8).tobytes())
        score, _ = H.sw(s1, s2, tw, th)
        assert score == L.sw_score(s1, s2, tw, th)


@pytest.mark.parametrize("sched", ["queue", "rows", "rows1", "dag", "dag-wave"])
def test_sw_both_schedules(golden, sched, monkeypatch):
    """The tile-counter schedule (device dependency counters + ready list),
    the row schedule (owner-computes tile rows, granule hand-offs; "rows" =
    th / 64 waves per tile row where th % 64 == 0, "rows1" = one wave) and the
    reference's own promise program on the generic device DAG (3 futures, 3
    puts per tile, include/hclib_hip/hx_dag.h) give the published scores and
    the oracle's on ragged tile grids. The DAG's tile tasks run on workgroups
    of th / 64 + 2 waves where th % 64 == 0 ("dag"), or one wave each
    ("dag-wave")."""
    if sched == "dag-wave":
        sched = "dag"
        monkeypatch.setenv("HCLIB_HIP_SW_DAG_WAVE", "1")
    monkeypatch.setenv("HCLIB_HIP_SW_SCHED", sched)
    g = golden("sw_goldens.json")["published"]["large"]
    s1, s2 = _sw_inputs("large")
    score, _ = H.sw(s1, s2, g["tile_w"], g["tile_h"])
    assert score == g["score"]
    rng = np.random.default_rng(11)
    for (n1, n2, tw, th) in [(700, 900, 64, 300), (2000, 513, 256, 256), (4096, 4096, 256, 512)]:
        a = bytes(rng.integers(1, 5, n1, dtype=np.int8).tobytes())
        b = bytes(rng.integers(1, 5, n2, dtype=np.int8).tobytes())
        score, _ = H.sw(a, b, tw, th)
        assert score == L.sw_score(a, b, tw, th), (n1, n2, tw, th)


@pytest.mark.parametrize("progressive", ["0", "1"])
def test_sw_row_schedule_hand_off_forms(golden, progressive, monkeypatch):
    """The row schedule's bottom-row hand-off — whole rows at the end of a
    tile (0) or 64-column chunks as the tile computes them (1, default) —
    gives the 64K golden and the oracle's scores on grids where the chunked
    form applies (th = 256, tw % 64 == 0) and where it does not."""
    monkeypatch.setenv("HCLIB_HIP_SW_SCHED", "rows")
    monkeypatch.setenv("HCLIB_HIP_SW_PROGRESSIVE", progressive)
    s1, s2 = _sw_inputs("huge")
    score, st = H.sw(s1[:65536], s2[:65536], 256, 256)
    assert score == 128772 and st["tiles"] == 65536
    rng = np.random.default_rng(23)
    for (n1, n2, tw, th) in [(4096, 2048, 64, 256), (8192, 1536, 512, 256), (3000, 1000, 192, 256),
                             (2048, 2048, 256, 128), (1000, 777, 100, 256)]:
        a = bytes(rng.integers(1, 5, n1, dtype=np.int8).tobytes())
        b = bytes(rng.integers(1, 5, n2, dtype=np.int8).tobytes())
        score, _ = H.sw(a, b, tw, th)
        assert score == L.sw_score(a, b, tw, th), (n1, n2, tw, th)
    # column bands use the same kernel
    score, tiles, _ = _sw_bands_in_order(s1[:16384], s2[:16384], 256, 256, 4, 8)
    assert score == L.sw_score(s1[:16384], s2[:16384], 256, 256)


@pytest.mark.parametrize("n1,n2,tw,th", [
    (50, 300, 50, 64), (1000, 640, 30, 128), (4100, 1024, 4100, 512), (5000, 1792, 100, 896),
    (2048, 2048, 64, 64), (3333, 768, 1111, 256), (640, 192, 64, 192)])
def test_sw_multiwave_tile_rows(n1, n2, tw, th, monkeypatch):
    """The multi-wave row kernel (one 64-row band per wave, th / 64 waves per
    tile row, inter-wave LDS rings): band widths below one 64-column chunk,
    ragged last chunks, widths past the 512-column ring (wrap slot), 1..14
    compute waves per workgroup — the oracle's score; the one-wave kernel agrees."""
    rng = np.random.default_rng(n1 * 7 + th)
    s1 = bytes(rng.integers(1, 5, n1, dtype=np.int8).tobytes())
    s2 = bytes(rng.integers(1, 5, n2, dtype=np.int8).tobytes())
    want = L.sw_score(s1, s2, tw, th)
    # every (rows per lane, skew, hand-off) form: 100 R + 10 S + K / 16
    for form in ("11", "12", "14", "21", "22", "211", "212", "214", "411", "412", "414"):
        monkeypatch.setenv("HCLIB_HIP_SW_FORM", form)
        score, st = H.sw(s1, s2, tw, th)
        assert score == want and st["tiles"] == (n1 // tw) * (n2 // th), form
        monkeypatch.setenv("HCLIB_HIP_SW_SCHED", "dag")
        assert H.sw(s1, s2, tw, th)[0] == want, ("dag", form)
        monkeypatch.delenv("HCLIB_HIP_SW_SCHED")
    monkeypatch.setenv("HCLIB_HIP_SW_SCHED", "rows1")
    assert H.sw(s1, s2, tw, th)[0] == want


def _sw_bands_in_order(s1, s2, tw, th, nbands, block_rows):
    """Every band of an nbands-way column split, run one after the other on
    cuda:0 through hclib_hip_sw_band_* in blocks of tile rows; band r's left
    column is band r-1's right column (what ShardedSw moves between ranks)."""
    import torch

    from hclib_amd import dist

    ntw, nth = len(s1) // tw, len(s2) // th
    stream = torch.cuda.current_stream().cuda_stream
    left, score, tiles, rights = None, None, 0, []
    for r, (j0, j1) in enumerate(dist.sw_bands(ntw, nbands)):
        band = H.SwBand(s1, s2, tw, th, j0, j1)
        right = None
        if r < nbands - 1:
            right = torch.full((nth * th,), -(1 << 30), dtype=torch.int32, device="cuda")
        for i0, i1 in dist.sw_blocks(nth, block_rows):
            band.rows(i0, i1, None if left is None else left.data_ptr(),
                      None if right is None else right.data_ptr(), stream)
        score, t = band.end(stream)
        tiles += t
        rights.append((j1, None if right is None else right.cpu().tolist()))
        left = right
    return score, tiles, rights


@pytest.mark.parametrize("n1,n2,tw,th,nbands,block_rows", [
    (1000, 777, 64, 64, 3, 2), (2048, 1024, 256, 256, 4, 1), (700, 900, 64, 300, 2, 2),
    (4096, 4096, 256, 512, 16, 3), (513, 1025, 17, 13, 5, 7)])
def test_sw_column_bands_vs_oracle(n1, n2, tw, th, nbands, block_rows):
    """Multi-GPU SW's band kernel: each band's right column is
    the oracle's last column of the matrix cut at the band's edge, and the
    last band's corner is the score; every tile runs once."""
    rng = np.random.default_rng(n1 + n2 + nbands)
    s1 = bytes(rng.integers(1, 5, n1, dtype=np.int8).tobytes())
    s2 = bytes(rng.integers(1, 5, n2, dtype=np.int8).tobytes())
    score, tiles, rights = _sw_bands_in_order(s1, s2, tw, th, nbands, block_rows)
    assert score == L.sw_score(s1, s2, tw, th)
    assert tiles == (n1 // tw) * (n2 // th)
    for j1, right in rights:
        if right is not None:
            _, _, col = L.sw_score(s1[:j1 * tw], s2, tw, th, want_edges=True)
            assert right == col[1:], j1


def test_sw_64k_golden_in_column_bands(golden):
    """The 64K config split into 8 column bands of 32 tile columns, 16 tile
    rows per exchanged block (bench.py's N=8 shape): score 128772."""
    s1, s2 = _sw_inputs("huge")
    score, tiles, _ = _sw_bands_in_order(s1[:65536], s2[:65536], 256, 256, 8, 16)
    assert score == golden("sw_goldens.json")["sw64k"]["score"] == 128772
    assert tiles == 65536


def _sw_rank(rank, world, port, s1, s2, tw, th, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from hclib_amd import dist

    r, w, _ = dist.init_from_env("gloo", share_device=True)
    job = dist.ShardedSw(s1, s2, tw, th, r, w, "gloo", block_rows=4)
    score, tiles = job.run()
    dist.barrier(w, "gloo")
    dist.shutdown(w)
    q.put((r, score, tiles))


def test_sharded_sw_two_ranks_sharing_the_gpu(golden):
    """ShardedSw end to end with two processes (gloo, both on cuda:0): the
    published 'large' score, every tile once over the ranks."""
    import socket

    import torch.multiprocessing as mp

    g = golden("sw_goldens.json")["published"]["large"]
    s1, s2 = _sw_inputs("large")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sw_rank, args=(r, 2, port, s1, s2, g["tile_w"], g["tile_h"], q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for _, score, tiles in res:
        assert score == g["score"]
        assert tiles == (len(s1) // g["tile_w"]) * (len(s2) // g["tile_h"])


def test_atomic_calibration_shapes():
    """The three L2 atomic shapes run and rank as the hardware must: a single
    hot word is far slower than atomics spread over many lines, and the
    coalesced streaming shape is the fastest."""
    scatter, _ = H.atomic_calibrate(H.ATOMIC_SCATTER_RET64, 64)
    hot, _ = H.atomic_calibrate(H.ATOMIC_HOT_WORD, 64)
    coal, _ = H.atomic_calibrate(H.ATOMIC_COALESCED32, 64)
    assert 0 < hot < scatter < coal


# ------------------------------------------------ cross-GPU work sharing
def test_cross_gpu_sharing_two_ranks_one_gpu():
    """dist.GlobalPool: two ranks, one process each,
    both on this GPU (gloo; the region in rank 0's HBM is mapped into rank
    1's process over IPC exactly as between two GPUs). T1L split at depth 1
    gives rank 0 two nodes and rank 1 the rest; sharing work must move
    subtrees to rank 0 and keep the counts bit-exact; T3L (span-bound, its
    busy rank always has hungry waves of its own) must stay exact too."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, REHEARSE_CASES="T1L:1,T3L:64", HCLIB_HIP_SPIN_LIMIT_MS="10000",
               HCLIB_HIP_WAVES_PER_CU="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29547", "scripts/rehearse_global.py"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 4 and all(x["bit_exact"] for x in lines)
    static, shared = lines[0], lines[1]
    assert static["nodes_per_rank"][0] == 2 and not static["shared"]
    assert shared["shared"] and shared["imported"][0] > 0 and shared["exported"][1] > 0
    assert shared["nodes_per_rank"][0] > 1000 * static["nodes_per_rank"][0]
    assert shared["active_after"] == 0 and shared["queued_after"] == 0
    assert sum(shared["exported"]) == sum(shared["imported"])
    assert shared["region_memory"] == os.environ.get("HCLIB_GLOBAL_MEM", "uncached")


# ------------------------------------------------ bench.py as its own launcher
def test_bench_self_launch_two_ranks_one_gpu():
    """`python bench.py --gpus 2` with no torchrun around it (the driver's
    command shape): bench.py starts two rank processes itself (gloo, both on
    this GPU) and re-prints rank 0's line: world size 2, the sharded T3L
    search bit-exact over the ranks (bench.py checks the combined counts
    against test/uts/sample_trees.sh:42-43 before it prints)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HCLIB_BENCH_LAUNCH_TIMEOUT_S"] = "100"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--share-device",
                        "--no-extras", "--steps", "1", "--warmup", "0"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    ln = lines[0]
    assert ln["collectives"]["world_size"] == 2 and ln["n_gpus"] == 2
    assert ln["config"]["bit_exact"] and sum(ln["nodes_per_rank"]) == 111345631
    assert "self-launch" in ln["launcher"]
