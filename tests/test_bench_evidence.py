"""CPU checks of bench.py's host-side arithmetic against the committed evidence.

The roofline in a bench.py JSON line must follow from the files under
profiles/.  Round 4's lines (profiles/r04/): the contract's HBM roofline =
algorithmic bytes per launch / kernel_ms against 8 TB/s, traffic = the PMC
FETCH_SIZE bytes of the same config AND camera path, and every view
(device time against HBM and L2, measured HBM, vector-memory issue, lane
utilisation) recomputed from the line and the PMC CSVs it names.  Round 3's
lines (profiles/r03/evidence_r3fin2, vmem-issue bound): SQ_INSTS_VMEM_RD per
launch over the line's device time per launch against CUs / TA_NS_PER_VMEM.
The rocprofv3 kernel trace's union of the timed launches must agree with
ms_per_step.  No GPU: these read JSON and CSV files.
"""
import csv
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EVID = os.path.join(ROOT, "profiles", "r03", "evidence_r3fin2")
R04 = os.path.join(ROOT, "profiles", "r04")
R04_LINES = [("r4b", "bench.json"), ("r4b", "bench_orbit.json"), ("r4b", "prof3.json"),
             # the final layout (aligned leaf records, 32-slot windows for config 5), PMC of r4h
             ("r4i", "bench.json"), ("r4i", "bench_orbit.json"), ("r4i", "prof3.json"), ("r4i", "prof5.json"),
             ("r4h", "bench_cfg5.json"),
             # the final tree (packed records and the r4d walk for config 3; aligned + 32-slot windows for
             # config 5), PMC of the same session
             ("r4s", "bench.json"), ("r4s", "bench_orbit.json"), ("r4s", "prof3.json"), ("r4s", "prof5.json"),
             ("r4s", "bench_cfg5.json"),
             # + the walk's buffer loads (RT_CHAIN 2): the shipped build
             ("r4u", "bench.json"), ("r4u", "bench_orbit.json"), ("r4u", "prof3.json"), ("r4u", "prof5.json"),
             ("r4u", "bench_cfg5.json"),
             # + 16x4 tiles for scenes past 32 MB of records (config 5)
             ("r4ad", "prof5.json"), ("r4ad", "bench_cfg5.json")]
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (module level: argparse-free helpers, no torch)


def _line(name):
    with open(os.path.join(EVID, name)) as fh:
        return json.loads([x for x in fh if x.startswith("{")][-1])


def _pmc_mean(path, counter, kernel="trace_simple<false, false, 72, 2>"):
    # the bench's own launches: grids above 2/3 of the largest (tools/pmc_summary.py
    # bench_rows; drops the one-frame verification launches of a 2-frame-per-launch run)
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    g = max((int(r["Grid_Size"]) for r in rows), default=0)
    vals = [float(r["Counter_Value"]) for r in rows if 3 * int(r["Grid_Size"]) > 2 * g]
    assert vals, (path, counter)
    return sum(vals) / len(vals)


@pytest.mark.parametrize("name", ["bench.json", "bench200.json", "prof3.json"])
def test_roofline_reproduces_from_profiles(name):
    d = _line(name)
    r = d["roofline"]
    # the PMC record the line was computed from (profiles/pmc_latest.json at the time)
    src = os.path.join(ROOT, r["pmc_source"].split(" ")[0])
    vmem = _pmc_mean(os.path.join(src, "A_counter_collection.csv"), "SQ_INSTS_VMEM_RD")
    fetch = _pmc_mean(os.path.join(src, "C_counter_collection.csv"), "FETCH_SIZE")
    # the same kernel and config measured again in the final session's passes
    again = _pmc_mean(os.path.join(EVID, "pmc3", "A_counter_collection.csv"), "SQ_INSTS_VMEM_RD")
    assert again == pytest.approx(vmem, rel=0.01)
    assert r["vmem_rd_per_launch"] == pytest.approx(vmem, rel=1e-6)
    t = r["frame_ms_device"] * 1e-3
    peak = 256 / bench.TA_NS_PER_VMEM
    assert r["bound"] == "vmem_issue"
    assert r["peak"] == pytest.approx(peak, abs=1e-3)
    assert r["frac"] == pytest.approx(vmem / t / 1e9 / peak, rel=2e-3)   # frame_ms_device is rounded to 4 digits
    hbm = fetch * 1024 * 2                                          # gfx950: 64-B halves, KiB
    assert r["traffic"] == pytest.approx(hbm, rel=1e-6)
    assert r["hbm"]["frac"] == pytest.approx(hbm / t / 1e9 / bench.HBM_PEAK_GBS, rel=2e-3)
    assert 0.0 < r["frac"] < 1.0 and 0.0 < r["hbm"]["frac"] < 1.0


def test_value_is_segments_over_wall_time():
    for name in ("bench.json", "bench200.json"):
        d = _line(name)
        seg = d["config"]["segments_per_frame"] * d["steps"]
        assert d["value"] == pytest.approx(seg / (d["ms_per_step"] * d["steps"] * 1e-3) / 1e6, rel=2e-3)
        assert d["metric"] == bench.BASELINE["metric"] and d["n_gpus"] == 1 and d["unit"] == "Mrays/s"
        cpu = d["cpu_baseline"]
        assert cpu["kind"] == "port" and cpu["cores"] >= 1 and cpu["value"] > 0


@pytest.mark.parametrize("cfg", [3, 5])
def test_rocprof_union_agrees_with_ms_per_step(cfg):
    u = json.load(open(os.path.join(EVID, f"union_cfg{cfg}.json")))
    assert u["launches"] == u["frames"]
    assert u["union_ms_per_frame"] == pytest.approx(u["bench_ms_per_step"], rel=0.05)
    # the mean launch agrees with the rocprofv3 stats of the same run
    with open(os.path.join(EVID, f"kernel_stats_cfg{cfg}.csv")) as fh:
        rows = [r for r in csv.DictReader(fh) if "trace_simple<false, false" in r["Name"]]
    assert rows
    avg_ms = float(rows[0]["AverageNs"]) / 1e6
    assert avg_ms == pytest.approx(u["launch_ms_mean"], rel=0.05)


def test_default_schedule_helpers():
    assert bench.default_inflight(1) == 4
    assert bench.default_batch(1) == 4 and bench.default_batch(1, steps=20) == 4
    assert bench.default_batch(1, steps=6) == 2       # whole pairs, not quadruples
    assert bench.default_batch(1, steps=5) == 1       # an odd frame count: no 1-frame launch of a new key
    for n in (2, 4, 8):
        assert bench.default_batch(n, weak=True) == n
        assert 0.5 < bench.default_root_weight(n) < 1.0
    assert bench.default_root_weight(1) == 1.0


def _r04(session, name):
    with open(os.path.join(R04, session, name)) as fh:
        return json.loads([x for x in fh if x.startswith("{")][-1])


def _pmc_file(src, pas):
    d = os.path.join(src, pas)
    return os.path.join(d, next(f for f in os.listdir(d) if f.endswith("counter_collection.csv")))


@pytest.mark.parametrize("session,name", R04_LINES)
def test_r04_roofline_reproduces(session, name):
    d = _r04(session, name)
    r = d["roofline"]
    alg = r["alg_bytes_per_launch"]
    # the contract's roofline: algorithmic bytes per launch / the mean launch duration, against 8 TB/s
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert r["achieved"] == pytest.approx(alg / (r["kernel_ms"] * 1e-3) / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    # the algorithmic bytes are SURVEY §8d's sum over the line's own counts per launch
    c = d["config"]
    seg = c["segments_per_frame"]
    assert alg / seg == pytest.approx(r["alg_bytes_per_segment"], rel=1e-3)
    # 32 B per node visit + 36 B per triangle test, plus at most 16 B (one material read) + 4 B (one
    # pixel) per segment
    extra = alg / seg - (32 * c["node_visits_per_segment"] + 36 * c["tri_tests_per_segment"])
    assert 0.0 < extra <= 20.0 + 0.1
    # PMC: a record of this config AND camera path, from CSVs under profiles/
    src = os.path.join(ROOT, r["pmc_source"].split(" ")[0])
    assert ("--camera-path orbit" in r["pmc_source"]) == (c["camera_path"] == "orbit")
    fetch = _pmc_mean(_pmc_file(src, "C"), "FETCH_SIZE", kernel="trace_simple<false, false")
    vmem = _pmc_mean(_pmc_file(src, "A"), "SQ_INSTS_VMEM_RD", kernel="trace_simple<false, false")
    assert r["traffic"] == pytest.approx(fetch * 1024 * 2, rel=1e-6)
    assert r["traffic_over_alg"] == pytest.approx(r["traffic"] / alg, abs=5e-5)      # rounded to 4 digits
    v = r["views"]
    tf = r["frame_ms_device"] * 1e-3
    assert v["device_time"]["achieved"] == pytest.approx(alg / tf / 1e9, rel=2e-3)
    assert v["device_time"]["l2_frac"] == pytest.approx(alg / tf / 1e9 / bench.L2_PEAK_GBS, rel=2e-3)
    assert v["device_time"]["hbm_frac"] == pytest.approx(alg / tf / 1e9 / bench.HBM_PEAK_GBS, rel=2e-3)
    assert v["hbm_measured"]["frac"] == pytest.approx(r["traffic"] / tf / 1e9 / bench.HBM_PEAK_GBS, rel=2e-3)
    vi = v["vmem_issue"]
    assert vi["vmem_rd_per_launch"] == pytest.approx(vmem, rel=1e-6)
    assert vi["frac"] == pytest.approx(vmem / tf / 1e9 / (256 / bench.TA_NS_PER_VMEM), rel=2e-3)
    lu = v["lane_utilisation"]
    assert lu["lockstep_lane_utilisation"] == pytest.approx(lu["lane_steps"] / (64 * lu["wave_steps"]), rel=1e-3)
    assert 0.0 < lu["lockstep_lane_utilisation"] < 1.0
    assert 0.0 < r["frac"] < 1.0
    # timing fits the steps: value = segments x steps / wall time
    assert d["value"] == pytest.approx(seg * d["steps"] / (d["ms_per_step"] * d["steps"] * 1e-3) / 1e6, rel=2e-3)
    assert c["frames_verified"] is True


@pytest.mark.parametrize("session,cfg", [("r4b", 3), ("r4i", 3), ("r4i", 5), ("r4s", 3), ("r4s", 5),
                                         ("r4u", 3), ("r4u", 5), ("r4ad", 5)])
def test_r04_rocprof_union(session, cfg):
    u = json.load(open(os.path.join(R04, session, f"union_cfg{cfg}.json")))
    p = _r04(session, f"prof{cfg}.json")
    assert u["launches"] == u["frames"] == p["steps"]
    assert u["union_ms_per_frame"] == pytest.approx(p["ms_per_step"], rel=0.05)
    with open(os.path.join(R04, session, f"kernel_stats_cfg{cfg}.csv")) as fh:
        rows = [r for r in csv.DictReader(fh) if "trace_simple<false, false" in r["Name"]]
    # rocprofv3's mean launch duration agrees with bench.py's kernel_ms (HIP events on the launch streams)
    assert float(rows[0]["AverageNs"]) / 1e6 == pytest.approx(p["roofline"]["kernel_ms"], rel=0.05)
    assert u["launch_ms_mean"] == pytest.approx(p["roofline"]["kernel_ms"], rel=0.05)


@pytest.mark.parametrize("session", ["r4i", "r4s", "r4u"])
def test_r04_camera_stop_learning_frame(session):
    """The frames after the camera stops (the first: its learning launch, the
    order then learned on the device; the second: the launch behind those
    learning kernels) cost at most 2x the steady lone frame (round 3's host
    learning: 4.4 ms against ~0.65; r4b, an earlier build of this round:
    4.16 ms for the second)."""
    cs = _r04(session, "bench_orbit.json")["camera_stop"]["ms_per_frame"]
    steady = sorted(cs[2:])[len(cs[2:]) // 2]
    assert cs[0] <= 2.0 * steady and max(cs) <= 2.0 * steady, cs


# ---- round 5: the headline over the device time per frame
R05 = os.path.join(ROOT, "profiles", "r05")


# (session, file) of the round-5 lines this round's evidence rests on (r5c's
# lines predate the PMC records keyed by accel: their traffic came from the
# reference walk's round-4 record, so they are not listed)
R05_LINES = [("r5au", "bench.json"), ("r5au", "bench200.json"), ("r5au", "prof3.json"), ("r5au", "prof5.json"),
             ("r5au", "bench_cfg5.json"), ("r5au", "bench_cfg6.json"), ("r5au", "bench_if4.json"),
             ("r5au", "bench_if6.json"), ("r5au", "bench_if8.json"),
             ("r5ah", "bench.json"), ("r5ah", "prof3.json"), ("r5ah", "prof5.json"), ("r5ah", "bench_cfg5.json"),
             ("r5ah", "bench_cfg6.json"), ("r5ah", "bench_if4.json"), ("r5ah", "bench_if8.json"),
             ("r5aa", "bench.json"), ("r5aa", "prof3.json"), ("r5aa", "prof5.json"), ("r5aa", "bench_cfg5.json"),
             ("r5aa", "bench_cfg6.json"), ("r5aa", "bench_if4.json"), ("r5aa", "bench_if6.json"),
             ("r5aa", "bench_if8.json")]


def _r05_lines():
    return [x for x in R05_LINES if os.path.exists(os.path.join(R05, *x))]


@pytest.mark.parametrize("session,name", _r05_lines())
def test_r05_roofline_reproduces(session, name):
    with open(os.path.join(R05, session, name)) as fh:
        d = json.loads([x for x in fh if x.startswith("{")][-1])
    r = d["roofline"]
    alg = r["alg_bytes_per_launch"]
    tf = r["frame_ms_device"] * 1e-3
    tk = r["kernel_ms"] * 1e-3
    assert r["views"]["device_time"]["l2_frac"] == pytest.approx(alg / tf / 1e9 / bench.L2_PEAK_GBS, rel=2e-3)
    assert r["views"]["per_launch"]["frac"] == pytest.approx(alg / tk / 1e9 / bench.HBM_PEAK_GBS, rel=2e-3)
    if r["bound"] == "l2":
        assert r["peak"] == bench.L2_PEAK_GBS
        assert r["frac"] == pytest.approx(alg / tf / 1e9 / bench.L2_PEAK_GBS, rel=2e-3)
    else:
        assert r["bound"] == "hbm" and r["peak"] == bench.HBM_PEAK_GBS
        num = r["traffic"] if r["traffic"] else alg
        assert r["frac"] == pytest.approx(num / tf / 1e9 / bench.HBM_PEAK_GBS, rel=2e-3)
    if r["traffic"]:
        # the PMC record it names: FETCH_SIZE (KiB of 64-B halves) x 1024 x 2
        src = os.path.join(ROOT, r["pmc_source"].split(" ")[0])
        fetch = _pmc_mean(_pmc_file(src, "C"), "FETCH_SIZE", kernel="trace_simple<false, false")
        assert r["traffic"] == pytest.approx(fetch * 1024 * 2, rel=1e-6)
        assert r["bound"] == ("hbm" if r["traffic"] / tf / 1e9 / bench.HBM_PEAK_GBS >
                              alg / tf / 1e9 / bench.L2_PEAK_GBS else "l2")
    # throughput: segments of the timed frames over the wall time
    seg = d["config"]["segments_per_frame"] * d["steps"] * d["config"]["frames_per_step"]
    assert d["value"] == pytest.approx(seg / (d["ms_per_step"] * 1e-3 * d["steps"]) / 1e6, rel=2e-3)
    assert 0.0 < r["frac"] < 1.0


def test_r05_frac_does_not_move_with_launches_in_flight():
    """the headline frac is computed over frame_ms_device
    (the device time per frame of the running loop), so once the device is
    saturated it does not move with the launches in flight: 4, 6 and 8 in
    flight on one build give frac within 5% (r5aa).  Below saturation it
    measures idle device time: one launch in flight leaves the device idle
    through each frame's serial tail (r5z: 0.38 ms per frame, frac 0.064)."""
    fr = {}
    for k in (4, 6, 8):
        with open(os.path.join(R05, "r5aa", f"bench_if{k}.json")) as fh:
            d = json.loads([x for x in fh if x.startswith("{")][-1])
        assert d["config"]["launches_in_flight"] == k
        fr[k] = d["roofline"]["frac"]
    assert max(fr.values()) <= 1.05 * min(fr.values()), fr
    with open(os.path.join(R05, "r5z", "bench_if1.json")) as fh:
        one = json.loads([x for x in fh if x.startswith("{")][-1])
    assert one["roofline"]["frac"] < 0.5 * min(fr.values())


@pytest.mark.parametrize("session,cfg", [("r5z", 3), ("r5z", 5), ("r5aa", 3), ("r5aa", 5), ("r5ah", 3), ("r5ah", 5),
                                         ("r5au", 3), ("r5au", 5)])
def test_r05_rocprof_union(session, cfg):
    """The rocprofv3 kernel trace of the same command: the union of the timed
    launches per frame agrees with ms_per_step, and rocprofv3's mean launch
    duration with bench.py's kernel_ms (HIP events on the launch streams)."""
    u = json.load(open(os.path.join(R05, session, f"union_cfg{cfg}.json")))
    with open(os.path.join(R05, session, f"prof{cfg}.json")) as fh:
        p = json.loads([x for x in fh if x.startswith("{")][-1])
    assert u["launches"] * u.get("frames_per_launch", 1) == u["frames"] == p["steps"]
    assert u.get("frames_per_launch", 1) == p["config"]["frames_per_launch"]
    assert u["union_ms_per_frame"] == pytest.approx(p["ms_per_step"], rel=0.06)
    with open(os.path.join(R05, session, f"kernel_stats_cfg{cfg}.csv")) as fh:
        rows = [r for r in csv.DictReader(fh) if "trace_simple<false, false" in r["Name"]]
    if u.get("frames_per_launch", 1) == 1:
        assert float(rows[0]["AverageNs"]) / 1e6 == pytest.approx(p["roofline"]["kernel_ms"], rel=0.05)
    else:
        # 2 frames per launch: rocprofv3's mean also holds the one-frame
        # verification launches after the timed region; the union tool
        # restates it from the trace and averages the timed launches alone
        assert float(rows[0]["AverageNs"]) / 1e6 == pytest.approx(u["all_launch_ms_mean"], rel=1e-3)
        assert int(rows[0]["Calls"]) == u["all_launches"]
        assert u["launch_ms_mean"] == pytest.approx(p["roofline"]["kernel_ms"], rel=0.05)


def test_r05_frac_two_frames_per_launch():
    """The N = 1 default of 2 frames per launch (r5au): frac within 5% at 4,
    6 and 8 launches in flight; PMC records keyed "@f2" (one launch is two
    frames: config 5 fetches 1.99 GB per frame, 2.04 at 1 frame per launch)."""
    fr = {}
    for k in (4, 6, 8):
        with open(os.path.join(R05, "r5au", f"bench_if{k}.json")) as fh:
            d = json.loads([x for x in fh if x.startswith("{")][-1])
        assert d["config"]["launches_in_flight"] == k and d["config"]["frames_per_launch"] == 2
        assert d["roofline"]["pmc_source"].startswith("profiles/r05/r5au/pmc3 ")
        fr[k] = d["roofline"]["frac"]
    assert max(fr.values()) <= 1.05 * min(fr.values()), fr
    with open(os.path.join(R05, "r5au", "bench_cfg5.json")) as fh:
        d = json.loads([x for x in fh if x.startswith("{")][-1])
    per_frame = d["roofline"]["traffic"] / d["config"]["frames_per_launch"]
    assert per_frame < 20.1e9 / 4 and d["ms_per_step"] < 7.85 / 4
    assert d["config"]["frames_verified"] is True


def test_r05_config5_traffic():
    """VERDICT r04 item 2 (config 5 below 20.1 GB of fetch and 7.85 ms per
    frame): the accel tree's launch of config 5 fetches 2.05 GB from HBM
    (PMC FETCH_SIZE, r5aa pmc5) at 1.20 ms per frame."""
    with open(os.path.join(R05, "r5aa", "bench_cfg5.json")) as fh:
        d = json.loads([x for x in fh if x.startswith("{")][-1])
    assert d["roofline"]["traffic"] < 20.1e9 / 4 and d["ms_per_step"] < 7.85 / 4
    assert d["config"]["frames_verified"] is True


R06 = os.path.join(ROOT, "profiles", "r06")
# the final tree's lines (r6m: bench at 20 and 200 steps, the profiled runs,
# configs 4-6, launches in flight, orbit), every one on the PMC records of the
# same session
R06_LINES = [(ses, f) for ses in ("r6m", "r6t", "r6w", "r6ae", "r6ah")
             for f in ("bench.json", "bench200.json", "prof3.json", "prof5.json", "bench_cfg4.json",
                       "bench_cfg5.json", "bench_cfg6.json", "bench_if1.json", "bench_if2.json",
                       "bench_if4.json", "bench_orbit.json")]


def _line6(path):
    with open(path) as fh:
        return json.loads([x for x in fh if x.startswith("{")][-1])


@pytest.mark.parametrize("session,name", R06_LINES)
def test_r06_roofline_reproduces(session, name):
    """Every fraction of the round-6 lines recomputes from the line and the
    PMC CSVs it names, and value = segments / wall time."""
    global R05
    saved = R05
    try:
        R05 = R06
        test_r05_roofline_reproduces(session, name)
    finally:
        R05 = saved
    d = _line6(os.path.join(R06, session, name))
    src = d["roofline"]["pmc_source"]
    if d["config"]["workload"].startswith(("cfg3", "cfg5", "cfg6")) and "orbit" not in name:
        # this session's records, or a round-6 one of the same launch size
        # (a line at 2 frames per launch, config 5 at 10 steps, keys "@f2")
        assert src.startswith(f"profiles/r06/{session}/pmc" if d["config"]["frames_per_launch"] == 4 or
                              session != "r6ah" else "profiles/r06/"), src


@pytest.mark.parametrize("session", ["r6m", "r6t", "r6w", "r6ae", "r6ah"])
@pytest.mark.parametrize("cfg", [3, 5])
def test_r06_rocprof_union(session, cfg):
    global R05
    saved = R05
    try:
        R05 = R06
        test_r05_rocprof_union(session, cfg)
    finally:
        R05 = saved


@pytest.mark.parametrize("session", ["r6m", "r6t", "r6w", "r6ae", "r6ah"])
def test_r06_final_tree(session):
    """The final tree's sessions (r6ah; r6ae: at 2 frames per launch; r6w:
    before the walk's priority; r6t:
    before option accel_octants; r6m: before the walk started inside the root): every GPU test green, smoke, frames verified, frac
    within 5% at 2 and 4 launches in flight, and config 3 faster per frame
    than round 5's final build on its box (r5au: 0.1239 ms at 20 steps,
    0.1198 at 200; boxes differ by a few percent)."""
    with open(os.path.join(R06, session, "pytest_gpu.log")) as fh:
        tail = fh.read().strip().splitlines()[-1]
    assert " passed" in tail and "failed" not in tail and "error" not in tail, tail
    fr = {k: _line6(os.path.join(R06, session, f"bench_if{k}.json"))["roofline"]["frac"] for k in (2, 4)}
    assert max(fr.values()) <= 1.05 * min(fr.values()), fr
    b20, b200 = (_line6(os.path.join(R06, session, f)) for f in ("bench.json", "bench200.json"))
    assert b20["config"]["frames_verified"] and b200["config"]["frames_verified"]
    assert b20["cpu_baseline"]["gpu_rows_match"] is True
    assert b200["ms_per_step"] < 0.1198 * 1.02 and b20["ms_per_step"] < 0.1239 * 1.02
