"""bench.py's bookkeeping against the committed profiles (CPU): the dominant kernel name it
reports is one rocprofv3 saw, the roofline's per-window MACs are the oracle's, and the HBM
traffic of the committed PMC summary is found for the default workload key."""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _latest_profile():
    """The newest profiles/<round> holding a headline kernel trace (a round's directory may hold
    probe summaries before its trace is taken)."""
    tags = sorted(t for t in glob.glob(os.path.join(ROOT, "profiles", "r*"))
                  if os.path.exists(os.path.join(t, "kernel_stats.csv")))
    assert tags, "no profiles/<round> directory with kernel_stats.csv"
    return tags[-1]


def test_layer_macs_are_the_oracle_count():
    import bench
    from oracle.beluga_np import macs_per_window
    assert bench.WINDOW_MACS == macs_per_window()


def test_reported_kernel_names_exist_in_the_committed_kernel_trace():
    import bench
    names = [r["Name"] for r in csv.DictReader(open(os.path.join(_latest_profile(), "kernel_stats.csv")))]
    for layer in ("conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "fc1", "fc2"):
        k = bench.kernel_name(layer, "f16x3")
        assert any(k in n for n in names), (layer, k)


def test_committed_traffic_matches_the_default_workload_key():
    import bench
    key = bench.profile_key()
    for layer in ("fc1", "conv2"):   # the MFMA roofline's kernel (FC1) and the k-mer gather
        traffic, src = bench.pmc_traffic(key, bench.kernel_name(layer, "f16x3"))
        assert traffic is not None and traffic > 0, "re-take profiles: STEPS=prof,pmc tools/gpu_session.sh + collect_profiles.py"
        assert src.startswith("profiles/")


def test_committed_sq_counters_give_the_held_clock():
    import bench
    key = bench.profile_key()
    held = bench.pmc_held_clock(key, bench.kernel_name("fc1", "f16x3"))   # the dominant MFMA kernel
    assert held is not None, "re-take profiles: STEPS=prof,pmc tools/gpu_session.sh + collect_profiles.py"
    assert 0.3 < held["mfma_busy"] <= 1.0 and 1.0 < held["held_clock_ghz"] < 2.6


def test_cpu_baseline_share_is_this_jobs_cpus():
    """cpu_baseline's P is the job's CPU share (affinity mask, cgroup quota), not os.cpu_count()
    of the whole machine."""
    import bench
    s = bench.host_cpu_share()
    assert 1 <= s["share"] <= s["affinity_cpus"] <= (os.cpu_count() or s["affinity_cpus"])
    if s["cgroup_cpus"] is not None:
        assert s["share"] <= max(1, int(-(-s["cgroup_cpus"] // 1)))
