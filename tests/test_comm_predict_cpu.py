"""The data-parallel exchange model bench.py's ``dp_rehearsal`` prints (comm.BucketTimeline.predict): buckets replayed
through one comm stream at a ring bus bandwidth, each started after its measured comm-kernel start latency.  Pure
arithmetic, checked on hand-computed timelines."""

import pytest

from spine_vision_amd.training.comm import BucketTimeline

MB = 2**20


def _xfer_ms(mb, world, bw):
    return 2.0 * (world - 1) / world * mb * MB / (bw * 1e9) * 1e3


def test_mid_backward_bucket_waits_the_mid_delay():
    r = BucketTimeline.predict([(64.0, 10.0)], 30.0, 31.0, 8, 200.0, 0.0, (2.9, 0.05))
    assert r["comm_end_ms"] == pytest.approx(10.0 + 2.9 + _xfer_ms(64.0, 8, 200.0), abs=1e-3)
    assert r["exposed_ms"] == 0.0 and r["predicted_scaling"] == pytest.approx(8.0)


def test_bucket_ready_at_the_backward_end_waits_only_for_the_rest_of_it():
    # ready 5 us before the end: the comm kernel cannot wait behind backward kernels that no longer exist
    r = BucketTimeline.predict([(10.0, 31.959)], 31.964, 32.592, 8, 200.0, 0.0, (2.9, 0.05))
    end = 31.959 + (31.964 - 31.959) + 0.05 + _xfer_ms(10.0, 8, 200.0)
    assert r["comm_end_ms"] == pytest.approx(end, abs=1e-3)
    assert r["exposed_ms"] == pytest.approx(end - 31.964, abs=1e-3)


def test_serialised_buckets_and_reserve_stretch():
    ready = [(64.0, 10.0), (64.0, 10.1), (8.0, None)]
    r = BucketTimeline.predict(ready, 20.0, 21.0, 4, 100.0, 0.1, 1.0)
    f = 1.1
    t = 10.0 * f + 1.0 + _xfer_ms(64.0, 4, 100.0)
    t = max(t, 10.1 * f + 1.0) + _xfer_ms(64.0, 4, 100.0)
    t = max(t, 20.0 * f + 1.0) + _xfer_ms(8.0, 4, 100.0)  # never ready in the backward: launched at its end
    assert r["comm_end_ms"] == pytest.approx(t, abs=1e-3)
    assert r["predicted_step_ms"] == pytest.approx(21.0 * f + (t - 20.0 * f), abs=1e-3)


def test_expected_max_over_ranks():
    xs = [1.0, 2.0, 3.0, 4.0]
    assert BucketTimeline.expected_max(xs, 1) == pytest.approx(2.5)  # one rank: the mean
    # n draws: P(max <= x_(i)) = (i/4)^n
    e2 = sum(x * ((i / 4) ** 2 - ((i - 1) / 4) ** 2) for i, x in enumerate(xs, 1))
    assert BucketTimeline.expected_max(xs, 2) == pytest.approx(e2)
    assert BucketTimeline.expected_max(xs, 8) > BucketTimeline.expected_max(xs, 2) > 2.5
    assert BucketTimeline.expected_max(xs, 64) == pytest.approx(4.0, abs=1e-6)


def test_sampled_latency_charges_the_slowest_rank():
    samples = [0.05] * 90 + [2.0] * 10  # 10 % of launches wait 2 ms
    r1 = BucketTimeline.predict([(64.0, 10.0)], 30.0, 31.0, 1, 200.0, latency_samples_ms=samples)
    r8 = BucketTimeline.predict([(64.0, 10.0)], 30.0, 31.0, 8, 200.0, latency_samples_ms=samples)
    d1, d8 = r1["launch_delay_ms"][0], r8["launch_delay_ms"][0]
    assert d1 == pytest.approx(0.05 * 0.9 + 2.0 * 0.1)
    assert d8 == pytest.approx(0.05 * 0.9 ** 8 + 2.0 * (1 - 0.9 ** 8))
    assert r8["comm_end_ms"] == pytest.approx(10.0 + d8 + _xfer_ms(64.0, 8, 200.0), abs=1e-3)


def test_rccl_hbm_traffic_stretches_the_backward():
    ready = [(300.0, 20.0), (51.0, None)]
    r = BucketTimeline.predict(ready, 30.0, 31.0, 8, 200.0, 0.0, (0.0, 0.0), hbm_gbs=5000.0)
    hbm = 6.0 * 7 / 8 * 351.0 * MB / 5000e9 * 1e3
    assert r["rccl_hbm_stretch_ms"] == pytest.approx(hbm, abs=1e-3)
    g = 1.0 + hbm / 30.0
    t = 20.0 * g + _xfer_ms(300.0, 8, 200.0)
    t = max(t, 30.0 * g) + _xfer_ms(51.0, 8, 200.0)
    assert r["comm_end_ms"] == pytest.approx(t, abs=1e-3)
    assert r["predicted_step_ms"] == pytest.approx(31.0 + hbm + max(0.0, t - 30.0 * g), abs=1e-3)
