"""bench.py's per-kernel roofline arithmetic (CPU): algorithmic bytes per launch from the device counters, the
sort gather fused into the multi-level trace, the NEE record, the PMC traffic ratio and the stale-counter rule."""
import bench


def _stats(**kw):
    st = dict(ms_trace=10.0, launches_trace=10, ms_shade=20.0, launches_shade=10, ms_shadow=30.0,
              rays=1_000_000, samples=400_000, shadow_rays=800_000, nodes_tested=0, tris_tested=0,
              shadow_nodes_tested=0, shadow_tris_tested=0)
    st.update(kw)
    return st


def test_trace_bytes_with_and_without_the_sort_gather():
    st = _stats()
    plain = bench.kernel_rooflines(st, None, "k_path_shadow")
    srt = bench.kernel_rooflines(st, None, "k_path_shadow", sorted_bounces=True)
    assert plain["k_trace_closest"]["algorithmic_bytes_per_launch"] == 40 * 1_000_000 // 10
    # 36 B per bounce ray (rays - camera samples): the permutation index and the sorted side-queue write
    assert srt["k_trace_closest"]["algorithmic_bytes_per_launch"] == (40 * 1_000_000 + 36 * 600_000) // 10
    a = srt["k_trace_closest"]
    assert abs(a["achieved"] - a["algorithmic_bytes_per_launch"] / 1e-3 / 1e9) < 0.1  # 1 ms per launch
    assert a["frac"] <= 1.0


def test_nee_record_bytes_and_traffic_ratio():
    st = _stats(nee_vertices=250_000)
    counters = {"k_path_nee": {"dram_bytes_per_launch": 12_000_000, "valu_insts_per_launch": 1e6}}
    rl = bench.kernel_rooflines(st, counters, "k_path_nee", sorted_bounces=True, n_lights=4)
    nee = rl["k_path_nee"]
    # 32 B per shadow ray + per vertex the 64-B record (16 B point + material, 4 x 8 B light samples, 16 B
    # weights), the slot's λ, β, L read (96 B) and L, β written (64 B)
    assert nee["algorithmic_bytes_per_launch"] == (32 * 800_000 + (64 + 96 + 64) * 250_000) // 10
    assert nee["traffic"] == 12_000_000
    assert nee["traffic_over_algorithmic"] == round(12_000_000 / nee["algorithmic_bytes_per_launch"], 2)
    assert 0 < nee["valu"]["frac"] <= 1.0
    # the shade kernel keeps its own stream bytes, the shadow rays moved to k_path_nee
    assert rl["k_path_shade"]["algorithmic_bytes_per_launch"] == 312 * 1_000_000 // 10


def test_no_counters_means_no_traffic_fields():
    rl = bench.kernel_rooflines(_stats(), None, "k_path_shadow")
    for v in rl.values():
        assert v.get("traffic") is None and "valu" not in v and "traffic_over_algorithmic" not in v


def test_effective_cpus_reads_the_cgroup_quota(tmp_path):
    """The CPU baseline runs on the CPUs the process may use: the affinity mask capped by the cgroup quota."""
    (tmp_path / "cpu.max").write_text("1600000 100000\n")  # cgroup v2: 16 CPUs of quota
    eff, info = bench.effective_cpus(tmp_path, affinity=256)
    assert eff == 16 and info["cgroup_quota_cpus"] == 16.0 and info["affinity_cpus"] == 256
    (tmp_path / "cpu.max").write_text("max 100000\n")  # no quota: the affinity mask
    assert bench.effective_cpus(tmp_path, affinity=64)[0] == 64
    (tmp_path / "cpu.max").unlink()
    (tmp_path / "cpu").mkdir()
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("250000\n")  # cgroup v1: 2.5 CPUs -> 2
    (tmp_path / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert bench.effective_cpus(tmp_path, affinity=8)[0] == 2
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")  # v1 unlimited
    assert bench.effective_cpus(tmp_path, affinity=8)[0] == 8
