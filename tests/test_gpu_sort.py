"""GPU: the multi-level coherence sorts (rt_sort.hip) checked directly through rt_debug_sort, on synthetic sharded
queues, against a stable CPU argsort of the keys — the permutation AND its stability (equal keys keep queue order),
the sorted queue's sharded layout and the rewritten shard lengths.

The film tests reach the sort only through its effect on traversal coherence (the results are per ray), so a
tile-boundary slip that lost or duplicated a few rays could hide there.  The sizes here cover every code path of the
three kernels: empty and one-item queues, the sub-tile edges (512 items for the 9-bit ray digits, 256 for the 8-bit
NEE digits), very unbalanced shard lengths, heavy key duplication (stability), and the NEE sort in place.  A scatter
tile is kRsIpt x 2^RB items (4096 for the ray digits, 2048 for the NEE digits) and rs_chunk rounds ceil(n / 1024) up
to a whole tile, so a block walks more than one tile only above 1024 x 4096 = 4.19 M rays or 1024 x 2048 = 2.10 M
vertices: test_ray_sort_multi_tile / test_nee_sort_multi_tile cover that loop (the running per-digit count carried
across tiles and the LDS staging arrays reused behind the tile's trailing barrier) with unbalanced shards and
duplicated keys; 1080p bounces reach it (16 Mi-sample batches).
"""
import numpy as np
import pytest

from computational_ray_tracer_amd import capi, scene
from computational_ray_tracer_amd.renderer import Renderer

pytestmark = pytest.mark.gpu
NS = capi.QUEUE_SHARDS


@pytest.fixture(scope="module")
def ctx():
    return Renderer(scene.cfg_cornell(res=(16, 16), spp_side=1))


def _expect(which, S, lens, keys, slots, nbits):
    pos = np.concatenate([j * S + np.arange(lens[j]) for j in range(NS)]).astype(np.int64)
    k = keys[pos] & np.uint32((1 << nbits) - 1)
    order = np.argsort(k, kind="stable")
    vals = (pos if which == 0 else slots[pos])[order]
    n = len(pos)
    S2 = ((-(-n // NS)) + 63) // 64 * 64
    d = np.arange(n)
    dst = (d // S2) * S + d % S2 if n else d
    olen = np.array([min(max(n - j * S2, 0), S2) for j in range(NS)], np.int32) if n else np.zeros(NS, np.int32)
    return dst, vals, olen


def _run(ctx, which, S, lens, key_range, seed, bits_a=3, bits_b=3):
    rng = np.random.default_rng(seed)
    nbits = 3 + 2 * bits_a + 3 * bits_b if which == 0 else 3 * bits_a
    keys = rng.integers(0, min(key_range, 1 << nbits), NS * S, dtype=np.uint64).astype(np.uint32)
    slots = rng.permutation(NS * S).astype(np.int32) if which == 1 else None
    lens = np.asarray(lens, np.int32)
    out, olen = ctx.debug_sort(which, S, lens, keys, slots, bits_a, bits_b)
    dst, vals, elen = _expect(which, S, lens, keys, slots, nbits)
    assert np.array_equal(olen, elen), (olen, elen)
    assert np.array_equal(out[dst], vals)
    if which == 0:  # the ray sort writes only the sorted positions (the rest keeps the 0xff fill)
        rest = np.ones(NS * S, bool)
        rest[dst] = False
        assert np.all(out[rest] == -1)
    else:  # in place: positions the sorted queue does not cover keep their slots
        rest = np.ones(NS * S, bool)
        rest[dst] = False
        assert np.array_equal(out[rest], slots[rest])


@pytest.mark.parametrize("n_total", [0, 1, 63, 511, 512, 513, 4096, 524287, 524288, 524289])
def test_ray_sort_sizes(ctx, n_total):
    S = max(64, ((-(-n_total // NS)) + 63) // 64 * 64)
    lens = [min(S, max(0, n_total - j * S)) for j in range(NS)]  # front-loaded shards
    _run(ctx, 0, S, lens, 1 << 18, seed=n_total)


@pytest.mark.parametrize("n_total", [0, 1, 255, 256, 257, 262143, 262144, 262145])
def test_nee_sort_sizes(ctx, n_total):
    S = max(64, ((-(-n_total // NS)) + 63) // 64 * 64)
    lens = [min(S, max(0, n_total - j * S)) for j in range(NS)]
    _run(ctx, 1, S, lens, 1 << 24, seed=100 + n_total, bits_a=8)


@pytest.mark.parametrize("key_range", [1, 16, 1 << 18])
def test_ray_sort_unbalanced_shards_and_stability(ctx, key_range):
    S = 200064
    lens = [S, 0, S // 3, 1, S, 17, S - 1, 150000]  # 1.15 M rays: several tiles per block
    _run(ctx, 0, S, lens, key_range, seed=key_range)


@pytest.mark.parametrize("key_range", [3, 1 << 24])
def test_nee_sort_unbalanced_in_place(ctx, key_range):
    S = 131072
    lens = [5, S, 0, 70001, S, 1, 99999, 64]
    _run(ctx, 1, S, lens, key_range, seed=7 + key_range, bits_a=8)


def test_sort_key_widths(ctx):
    # 3 + 2 x 2 + 3 x 2 = 13-bit ray keys (1 pass), 3 + 2 x 4 + 3 x 4 = 23 bits (3 passes); 7-bit NEE axes (21 bits)
    S = 65536
    lens = [S, 3, S, 0, 12345, S, 64, 1]
    _run(ctx, 0, S, lens, 1 << 30, seed=1, bits_a=2, bits_b=2)
    _run(ctx, 0, S, lens, 1 << 30, seed=2, bits_a=4, bits_b=4)
    _run(ctx, 1, S, lens, 1 << 30, seed=3, bits_a=7)


@pytest.mark.parametrize("key_range", [1, 16, 1 << 18])
def test_ray_sort_multi_tile(ctx, key_range):
    S = 700032  # (a multiple of 64) 4.55 M rays: blocks walk two tiles of 4096
    lens = [S, S, S // 2, 1, S, S, S - 1, S]
    assert sum(lens) > 1024 * 4096
    _run(ctx, 0, S, lens, key_range, seed=7 + key_range)


@pytest.mark.parametrize("key_range", [1, 16, 1 << 24])
def test_nee_sort_multi_tile(ctx, key_range):
    S = 360000  # 2.28 M vertices: blocks walk two tiles of 2048
    lens = [S, S, S, 0, S, S // 3, S, S]
    assert sum(lens) > 1024 * 2048
    _run(ctx, 1, S, lens, key_range, seed=11 + key_range, bits_a=8)
