"""bench.py's per-rank HBM plan: at N = 1, 2, 4, 8 the configs[3] (16M, nb = 2048) and configs[4]
(4M, nb = 4096) legs -- double-buffered shard outputs, the all-gather receive buffers, the library's work, the decrypt
check -- fit beside the largest fixed-base tables an MI355X holds (W = 22 / W = 20 with the 4096-bit Shoup rows beside the
factored rows, W = 21 without), and a device too small for both
is refused up front instead of running with a silently smaller window. CPU only: the plan is arithmetic."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import pytest  # noqa: E402

import bench  # noqa: E402

MI355X = 287 * 10 ** 9          # free HBM of an idle MI355X as hipMemGetInfo reports it (288 GB less the runtime's share)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("cfg,window", [(1, 22), (3, 22), (4, 20)])
def test_plan_fits_an_mi355x_at_every_world_size(cfg, window, world):
    nb = bench.CONFIGS[cfg]["nb"]
    pf = bench.preflight_window(cfg, world, nb, 23, MI355X)
    assert pf["ok"] and pf["window"] == window == pf["window_tables_alone"]
    assert pf["tables_bytes"] + max(pf["legs_bytes"], pf["reserve_bytes"]) <= MI355X


def test_table_sizes_match_the_design():
    assert bench.fb_table_bytes(2048, 22) == 2 * 47 * (1 << 22) * 448        # 2 x 88.3 GB
    assert bench.fb_table_bytes(4096, 20) == 2 * 103 * (1 << 20) * (512 + 640)   # 2 x 124.4 GB: factored + Shoup rows
    assert bench.fb_table_bytes(4096, 21) > MI355X
    assert bench.fb_table_bytes(2048, 23) > MI355X                           # W = 23 Shoup rows do not fit


@pytest.mark.parametrize("world", [2, 8])
def test_gather_buffers_are_the_whole_array_on_every_rank(world):
    plan = bench.rank_memory_plan(3, world, 2048)
    leg = plan["config3"]
    assert leg["gathered_outputs"] == 2 * (-(-(16 << 20) // world)) * world * (128 * 4 + 4)   # two buffers of 16M rows
    assert leg["shard_outputs"] >= 2 * (-(-(16 << 20) // world)) * (128 * 4 + 4)


def test_a_device_too_small_for_tables_and_legs_is_refused():
    nb = 4096
    dev = bench.fb_table_bytes(nb, 20) + 23 * 10 ** 9    # the library's reserve (1/12: 22.7 GB) fits, one rank's legs not
    pf = bench.preflight_window(4, 1, nb, 23, dev)
    assert pf["legs_bytes"] > 23 * 10 ** 9 > pf["reserve_bytes"]
    assert pf["window_tables_alone"] == 20
    assert not pf["ok"] and pf["window"] < 20          # the legs would drop the window: bench.py exits


def test_factored_rows_alone_without_shoup_rows(monkeypatch):
    monkeypatch.setenv("FLEXPAI_SGS", "0")
    assert bench.fb_table_bytes(4096, 21) == 2 * 98 * (1 << 21) * 512        # 2 x 105.2 GB
    pf = bench.preflight_window(4, 1, 4096, 23, MI355X)
    assert pf["ok"] and pf["window"] == 21
